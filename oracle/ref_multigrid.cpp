// ORACLE TEST INFRASTRUCTURE -- NOT PART OF THE PRODUCT.
//
// The host operator pipeline on general octrees (ddpca_multigrid_*: MULTIGRID::TRANSFER + PATCH +
// STIF_MATR + CONSTRAINT(1) restated in multigrid.cpp) against the reference's own pipeline on the
// same element trees.  The reference's CYLINDER example (examples/CYLINDER_1.h) generates its
// meshes (MESH: curved cylinders, inhomogeneous global refinement with the 4-way patterns,
// local refinement towards the contact lines -> hanging nodes); every subdomain's element tree,
// constraints and loads go through libddpca_amd, then the reference runs TRANSFER / STIF_MATR /
// CONSTRAINT(1) on its own MULTIGRID, and the outputs are compared: positions (posiNode) and the
// level counts exactly, node coordinates after PATCH, consFlag, consStif[l] entrywise (relative to
// the level's largest entry), realProl[l] and the hanging rows of prolOper[maxiLeve] exactly,
// consForc and dispForc.  "rot": nodal rotations (nodeRota) on every seventh node -- fine, coarse
// and hanging ones -- so every prolongation case (rotated child, rotated parent, both) occurs.
// "beam": the BEAM example's uniformly refined tree (every element 8-way) through the same general
// path -- the host generators' fast path must be this algorithm's special case.
// One JSON line per subdomain on stdout, a summary line last.  CPU only.
//   ref_multigrid cylinder [locaLeve globInho [rot]]
//   ref_multigrid beam [globLeve [rot]]
#include <unistd.h>

#include <cstdio>

#include "examples/BEAM.h"
#include "examples/CYLINDER_1.h"
#include "ref_bind.hpp"

namespace {

using SpMat = ddpca_bind::SpMat;

template <typename T>
std::vector<T> view(ddpca_multigrid_t g, const char* what, int64_t level) {
    const void* data = nullptr;
    int64_t n = 0;
    int dt = -1;
    ddpca_bind::check(ddpca_multigrid_view(g, what, level, &data, &n, &dt));
    return std::vector<T>((const T*)data, (const T*)data + n);
}

SpMat csr(ddpca_multigrid_t g, const std::string& base, int64_t level) {
    auto shape = view<int64_t>(g, (base + ":shape").c_str(), level);
    auto ptr = view<int64_t>(g, (base + ":ptr").c_str(), level);
    auto col = view<int32_t>(g, (base + ":col").c_str(), level);
    auto val = view<double>(g, (base + ":val").c_str(), level);
    std::vector<Eigen::Triplet<double>> t;
    for (int64_t r = 0; r < shape[0]; ++r)
        for (int64_t k = ptr[r]; k < ptr[r + 1]; ++k) t.emplace_back(r, col[k], val[k]);
    SpMat m(shape[0], shape[1]);
    m.setFromTriplets(t.begin(), t.end());
    return m;
}

double maxabs(const SpMat& a) {
    double m = 0.0;
    for (int k = 0; k < a.outerSize(); ++k)
        for (SpMat::InnerIterator it(a, k); it; ++it) m = std::max(m, std::abs(it.value()));
    return m;
}

Eigen::Matrix3d rotation(long node) {
    return Eigen::AngleAxisd(0.3 + 0.001 * (double)node, Eigen::Vector3d(1.0, 2.0, 3.0).normalized()).toRotationMatrix();
}

int saved_stdout = -1;

// our pipeline and the reference's on one MULTIGRID's tree; prints the comparison, true = match
bool compare(MULTIGRID& g, size_t tg, bool rot, long& total_hang) {
    const int saved = saved_stdout;
    {
        if (rot)
            for (const auto& nc : g.nodeCoor)
                if (nc.first % 7 == 3) g.nodeRota.emplace(nc.first, rotation(nc.first));
        // ---- the element tree as the reference's REFINE left it, through the binding
        ddpca_multigrid_t h = ddpca_bind::tree_build(g);

        // ---- the reference's pipeline on the same tree
        std::fflush(stdout);
        if (!std::freopen("/dev/null", "w", stdout)) return 2;
        g.TRANSFER();
        g.STIF_MATR();
        g.CONSTRAINT(1);
        std::fflush(stdout);
        dup2(saved, 1);
        const long L = g.mgpi.maxiLeve;
        const auto posi = view<int64_t>(h, "posiNode", 0);
        bool pos_eq = (int64_t)posi.size() == (int64_t)g.posiNode.size();
        for (size_t p = 0; pos_eq && p < posi.size(); ++p) pos_eq = posi[p] == g.posiNode[p];
        const auto lc = view<int64_t>(h, "leveCount", 0);
        bool lev_eq = (long)lc.size() == L + 2;
        for (long l = 0, acc = 0; lev_eq && l <= L + 1; ++l) lev_eq = lc[l] == (acc += (long)g.leveNode[l].size());
        const auto co = view<double>(h, "nodeCoor", 0);
        double dx = 0.0;
        for (const auto& nc : g.nodeCoor)
            for (int a = 0; a < 3; ++a) dx = std::max(dx, std::abs(co[3 * nc.first + a] - nc.second[a]));
        const auto cf = view<uint8_t>(h, "consFlag", 0);
        bool flag_eq = (int64_t)cf.size() == g.consFlag.size();
        for (int64_t d = 0; flag_eq && d < (int64_t)cf.size(); ++d) flag_eq = (int)cf[d] == g.consFlag(d);
        double dK = 0.0, dP = 0.0;
        for (long l = 0; l <= L; ++l) {
            const SpMat K = csr(h, "K", l);
            const SpMat& Kr = g.mgpi.consStif[l];
            if (K.rows() != Kr.rows()) { dK = 1e300; break; }
            dK = std::max(dK, maxabs(K - Kr) / maxabs(Kr));
        }
        for (long l = 0; l < L; ++l) {
            const SpMat P = csr(h, "P", l);
            if (P.rows() != g.mgpi.realProl[l].rows()) { dP = 1e300; break; }
            dP = std::max(dP, maxabs(P - g.mgpi.realProl[l]));
        }
        const int64_t NL = lc[L], N = lc[L + 1];
        const SpMat& Pm = g.prolOper[L];
        double dH = 0.0;
        if (N > NL) {
            const SpMat H = csr(h, "H", 0);
            const SpMat Hr = Pm.bottomRows(Pm.rows() - 3 * NL).leftCols(3 * NL);
            dH = H.rows() == Hr.rows() && H.cols() == Hr.cols() ? maxabs(H - Hr) : 1e300;
        }
        const auto f = view<double>(h, "consForc", 0);
        double df = 0.0, fm = 0.0;
        for (int64_t i = 0; i < g.consForc.size(); ++i) {
            fm = std::max(fm, std::abs(g.consForc(i)));
            df = std::max(df, std::abs((i < (int64_t)f.size() ? f[i] : 0.0) - g.consForc(i)));
        }
        if ((int64_t)f.size() != g.consForc.size()) df = 1e300;
        const auto dv = view<double>(h, "dispForc", 0);
        bool disp_eq = (int64_t)dv.size() == g.dispForc.size();
        for (int64_t i = 0; disp_eq && i < (int64_t)dv.size(); ++i) disp_eq = dv[i] == g.dispForc(i);
        const double drel = fm > 0 ? df / fm : df;
        const bool sub_ok = pos_eq && lev_eq && dx <= 1e-15 && flag_eq && dK <= 1e-13 && dP == 0.0 && dH == 0.0 &&
                            drel <= 1e-12 && disp_eq;
        total_hang += (long)(N - NL);
        std::printf("{\"subdomain\": %zu, \"ok\": %s, \"nodes\": %ld, \"levels\": %ld, \"hanging\": %ld, \"rotated\": %zu, "
                    "\"elements\": %ld, \"positions_equal\": %s, \"levels_equal\": %s, \"coords\": %.3g, \"consFlag_equal\": %s, "
                    "\"K_rel\": %.3g, \"realProl\": %.3g, \"hang\": %.3g, \"consForc_rel\": %.3g, \"dispForc_equal\": %s}\n",
                    tg, sub_ok ? "true" : "false", (long)N, L + 1, (long)(N - NL), g.nodeRota.size(), (long)g.elemVect.size(),
                    pos_eq ? "true" : "false", lev_eq ? "true" : "false", dx, flag_eq ? "true" : "false", dK, dP, dH, drel,
                    disp_eq ? "true" : "false");
        ddpca_multigrid_destroy(h);
        return sub_ok;
    }
}

}  // namespace

int main(int argc, char** argv) {
    const std::string mode = argc > 1 ? argv[1] : "cylinder";
    saved_stdout = dup(1);
    if (!std::freopen("/dev/null", "w", stdout)) return 2;  // the reference's progress output
    bool ok = true;
    long total_hang = 0;
    size_t nsub = 0;
    if (mode == "beam") {
        BEAM beam(0);
        beam.diviNumb = {8, 2, 2};
        beam.globLeve = argc > 2 ? std::atol(argv[2]) : 2;
        beam.MESH_NODD(0);
        std::fflush(stdout);
        dup2(saved_stdout, 1);
        nsub = 1;
        ok = compare(beam.multGrid[0], 0, argc > 3 && std::string(argv[3]) == "rot", total_hang);
    } else {
        CYLINDER_1 c;
        c.copyNumb = 1;
        c.locaLeve = argc > 2 ? std::atol(argv[2]) : 2;
        c.globInho = argc > 3 ? std::atol(argv[3]) : 1;
        c.MESH();
        std::fflush(stdout);
        dup2(saved_stdout, 1);
        nsub = c.multGrid.size();
        for (size_t tg = 0; tg < nsub; ++tg) ok = compare(c.multGrid[tg], tg, argc > 4 && std::string(argv[4]) == "rot", total_hang) && ok;
    }
    std::printf("{\"ok\": %s, \"subdomains\": %zu, \"hanging_nodes\": %ld}\n", ok ? "true" : "false", nsub, total_hang);
    return ok ? 0 : 1;
}
