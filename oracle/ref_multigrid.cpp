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
// "refine": MULTIGRID::REFINE itself (ddpca_multigrid_refine: GRLE_CHECK, the seven patterns,
// planSurf, spliFlag) against the reference's REFINE round by round on the same box, trees compared
// exactly (node ids and coordinates bitwise, corners, parents, levels, patterns, children, the next
// split); "refine_pipeline": CYLINDER_1's refinement schedule on that box through the library,
// then the pipeline comparison above on the library's own refined tree.
//   ref_multigrid cylinder [locaLeve globInho [rot]]
//   ref_multigrid beam [globLeve [rot]]
//   ref_multigrid refine [rounds]
//   ref_multigrid refine_pipeline [globInho globHomo locaLeve [rot]]
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
// pre: an unbuilt handle holding the same tree (made by ddpca_multigrid_refine), else made from g's tree
bool compare(MULTIGRID& g, size_t tg, bool rot, long& total_hang, ddpca_multigrid_t pre = nullptr) {
    const int saved = saved_stdout;
    {
        if (rot)
            for (const auto& nc : g.nodeCoor)
                if (nc.first % 7 == 3) g.nodeRota.emplace(nc.first, rotation(nc.first));
        // ---- the element tree as the reference's REFINE left it, through the binding
        ddpca_multigrid_t h = pre;
        std::string ours_error;
        try {
            if (h)
                ddpca_bind::tree_inputs(h, g);
            else
                h = ddpca_bind::tree_build(g);
        } catch (const std::exception& e) {
            ours_error = e.what();
        }

        // ---- the reference's pipeline on the same tree
        std::fflush(stdout);
        if (!std::freopen("/dev/null", "w", stdout)) return 2;
        g.TRANSFER();
        g.STIF_MATR();
        g.CONSTRAINT(1);
        std::fflush(stdout);
        dup2(saved, 1);
        const long L = g.mgpi.maxiLeve;
        if (!ours_error.empty()) {
            std::set<long> seen(g.posiNode.begin(), g.posiNode.end());
            std::printf("{\"subdomain\": %zu, \"ok\": false, \"ours_error\": \"%s\", \"reference_positions\": %zu, "
                        "\"reference_distinct_positions\": %zu, \"nodes\": %zu}\n",
                        tg, ours_error.c_str(), g.posiNode.size(), seen.size(), g.nodeCoor.size());
            if (h) ddpca_multigrid_destroy(h);
            return false;
        }
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
        double drel = fm > 0 ? df / fm : df;
        // dispForc: the prescribed values of the fine level's constrained rows in position order
        // (MULTIGRID.h:1187-1204).  The reference's last step there, dispForc = dispForc.block(0, 0,
        // n, 1), shrinks the vector onto a block of itself (an Eigen aliasing resize: it reads the
        // freed buffer) whenever consDofv also holds hanging nodes' dofs, so its own vector can be
        // garbage; the expected one is restated here from consDofv and posiNode, and the
        // reference's consForc (computed from that vector) is compared only when its dispForc is
        // intact.
        const auto dv = view<double>(h, "dispForc", 0);
        std::vector<double> want;
        for (int64_t ti = 0; ti < 3 * lc[L]; ++ti)
            if (g.consFlag(ti) == 0) {
                const auto it = g.consDofv.find(3 * g.posiNode[ti / 3] + ti % 3);
                want.push_back(it == g.consDofv.end() ? 0.0 : it->second);
            }
        const bool disp_eq = dv == want;
        bool ref_intact = (int64_t)want.size() == g.dispForc.size();
        for (size_t i = 0; ref_intact && i < want.size(); ++i) ref_intact = want[i] == g.dispForc(i);
        if (!ref_intact) drel = -1.0;  // not compared
        const bool sub_ok = pos_eq && lev_eq && dx <= 1e-15 && flag_eq && dK <= 1e-13 && dP == 0.0 && dH == 0.0 &&
                            drel <= 1e-12 && disp_eq;
        total_hang += (long)(N - NL);
        std::printf("{\"subdomain\": %zu, \"ok\": %s, \"nodes\": %ld, \"levels\": %ld, \"hanging\": %ld, \"rotated\": %zu, "
                    "\"elements\": %ld, \"positions_equal\": %s, \"levels_equal\": %s, \"coords\": %.3g, \"consFlag_equal\": %s, "
                    "\"K_rel\": %.3g, \"realProl\": %.3g, \"hang\": %.3g, \"consForc_rel\": %.3g, \"dispForc_equal\": %s, \"reference_dispForc_intact\": %s}\n",
                    tg, sub_ok ? "true" : "false", (long)N, L + 1, (long)(N - NL), g.nodeRota.size(), (long)g.elemVect.size(),
                    pos_eq ? "true" : "false", lev_eq ? "true" : "false", dx, flag_eq ? "true" : "false", dK, dP, dH, drel,
                    disp_eq ? "true" : "false", ref_intact ? "true" : "false");
        ddpca_multigrid_destroy(h);
        return sub_ok;
    }
}

// ---------------------------------------------------------------- local refinement (REFINE)
// A box of nx x ny x nz level-0 elements (the examples' corner order, CYLINDER_1.h:324-344); the
// face y = 0 is a "curved surface": a new node whose corner set lies on it moves to
// y = bump(x, z) through planSurf, as CURVEDS::REFINE does for the cylinders (CURVEDS.h:58-100).
struct Box {
    MULTIGRID g;
    int nx, ny, nz;
};

void box_make(Box& b, int nx, int ny, int nz) {
    b.nx = nx, b.ny = ny, b.nz = nz;
    std::vector<long> id((nx + 1) * (ny + 1) * (nz + 1));
    auto at = [&](int i, int j, int k) -> long& { return id[(k * (ny + 1) + j) * (nx + 1) + i]; };
    for (int k = 0; k <= nz; ++k)
        for (int j = 0; j <= ny; ++j)
            for (int i = 0; i <= nx; ++i) at(i, j, k) = b.g.TRY_ADD_NODE(COOR(0.5 * i, 0.5 * j, 0.5 * k));
    for (int k = 0; k < nz; ++k)
        for (int j = 0; j < ny; ++j)
            for (int i = 0; i < nx; ++i) {
                TREE_ELEM t;
                t.parent = -1;
                t.cornNode = {at(i, j, k), at(i + 1, j, k), at(i + 1, j + 1, k), at(i, j + 1, k),
                              at(i, j, k + 1), at(i + 1, j, k + 1), at(i + 1, j + 1, k + 1), at(i, j + 1, k + 1)};
                t.level = 0;
                t.refiPatt = 7;
                t.children.resize(0);
                b.g.ADD_ELEMENT(t);
            }
}

double bump(double x, double z) { return -0.04 * std::sin(1.3 * x + 0.2) * std::sin(2.1 * z + 0.5); }

std::map<std::vector<long>, COOR> plan_surface(const MULTIGRID& g, const std::set<long>& split) {
    static const int line[12][2] = {{0, 1}, {1, 2}, {2, 3}, {3, 0}, {4, 5}, {5, 6}, {6, 7}, {7, 4}, {0, 4}, {1, 5}, {2, 6}, {3, 7}};
    static const int face[6][4] = {{0, 3, 7, 4}, {1, 2, 6, 5}, {0, 4, 5, 1}, {3, 7, 6, 2}, {0, 1, 2, 3}, {4, 5, 6, 7}};
    std::map<std::vector<long>, COOR> plan;
    auto on = [&](long n) { return g.nodeCoor.at(n)[1] <= 1e-12; };
    auto add = [&](std::vector<long> key) {
        for (long n : key)
            if (!on(n)) return;
        COOR c(0.0, 0.0, 0.0);
        for (long n : key) c = c + g.nodeCoor.at(n);
        c = c / (double)key.size();
        c[1] = bump(c[0], c[2]);
        std::sort(key.begin(), key.end());
        plan.emplace(key, c);
    };
    for (long e : split) {
        const auto& cn = g.elemVect[e].cornNode;
        for (const auto& l : line) add({cn[l[0]], cn[l[1]]});
        for (const auto& f : face) add({cn[f[0]], cn[f[1]], cn[f[2]], cn[f[3]]});
    }
    return plan;
}

// one REFINE round on the reference's MULTIGRID and through ddpca_multigrid_refine on h, then the
// trees compared exactly; split (refiPatt set on g) returns the next round's elements
bool refine_round(MULTIGRID& g, ddpca_multigrid_t h, std::set<long>& split, const std::map<long, std::set<long>>& flag,
                  int round, bool curved) {
    const std::map<std::vector<long>, COOR> plan = curved ? plan_surface(g, split) : std::map<std::vector<long>, COOR>{};
    std::vector<int64_t> el, pa, pp{0}, pn, fe, fc;
    std::vector<double> px;
    for (long e : split) el.push_back(e), pa.push_back(g.elemVect[e].refiPatt);
    for (const auto& kv : plan) {
        pn.insert(pn.end(), kv.first.begin(), kv.first.end());
        pp.push_back((int64_t)pn.size());
        for (int a = 0; a < 3; ++a) px.push_back(kv.second[a]);
    }
    for (const auto& kv : flag)
        for (long c : kv.second) fe.push_back(kv.first), fc.push_back(c);
    const int rc = ddpca_multigrid_refine(h, (int64_t)el.size(), el.data(), pa.data(), (int64_t)plan.size(), pp.data(),
                                          pn.data(), px.data(), (int64_t)fe.size(), fe.data(), fc.data());
    const long ne0 = (long)g.elemVect.size();
    g.REFINE(split, flag, plan);
    if (rc != 0) {
        std::printf("{\"round\": %d, \"ok\": false, \"error\": \"%s\"}\n", round, ddpca_last_error());
        return false;
    }
    auto tree = [&](const char* what, auto tag) {
        const void* data = nullptr;
        int64_t n = 0;
        int dt = -1;
        ddpca_bind::check(ddpca_multigrid_tree(h, what, &data, &n, &dt));
        using T = decltype(tag);
        return std::vector<T>((const T*)data, (const T*)data + n);
    };
    const auto xyz = tree("nodeCoor", 0.0);
    const auto corner = tree("corner", int64_t{}), parent = tree("parent", int64_t{}), level = tree("level", int64_t{}),
               patt = tree("refiPatt", int64_t{}), cptr = tree("child_ptr", int64_t{}), child = tree("child", int64_t{}),
               next = tree("nextSplit", int64_t{});
    const long nn = (long)g.nodeCoor.size(), ne = (long)g.elemVect.size();
    bool nodes_eq = (long)xyz.size() == 3 * nn, elem_eq = (long)parent.size() == ne;
    for (const auto& nc : g.nodeCoor)
        for (int a = 0; nodes_eq && a < 3; ++a) nodes_eq = nc.first < nn && xyz[3 * nc.first + a] == nc.second[a];
    long hang_children = 0;
    for (long e = 0; elem_eq && e < ne; ++e) {
        const TREE_ELEM& t = g.elemVect[e];
        for (int k = 0; k < 8; ++k) elem_eq = elem_eq && corner[8 * e + k] == t.cornNode[k];
        elem_eq = elem_eq && parent[e] == t.parent && level[e] == t.level && patt[e] == t.refiPatt;
        const long nch = t.children.empty() ? 0 : t.refiPatt == 0 ? 8 : t.refiPatt <= 3 ? 4 : 2;
        elem_eq = elem_eq && cptr[e + 1] - cptr[e] == nch;
        for (long q = 0; elem_eq && q < nch; ++q) elem_eq = child[cptr[e] + q] == t.children[q];
        hang_children += nch;
        if (!elem_eq)
            std::fprintf(stderr, "element %ld differs: parent %ld/%ld level %ld/%ld patt %ld/%ld children %ld/%ld\n", e,
                         (long)parent[e], t.parent, (long)level[e], t.level, (long)patt[e], t.refiPatt,
                         (long)(cptr[e + 1] - cptr[e]), nch);
    }
    bool next_eq = next.size() == split.size() && std::equal(split.begin(), split.end(), next.begin());
    const bool ok = nodes_eq && elem_eq && next_eq;
    std::printf("{\"round\": %d, \"ok\": %s, \"split\": %zu, \"planSurf\": %zu, \"new_elements\": %ld, \"nodes\": %ld, "
                "\"nodes_equal\": %s, \"elements_equal\": %s, \"next_split_equal\": %s}\n",
                round, ok ? "true" : "false", el.size(), plan.size(), ne - ne0, nn, nodes_eq ? "true" : "false",
                elem_eq ? "true" : "false", next_eq ? "true" : "false");
    (void)hang_children;
    return ok;
}

std::vector<long> leaves(const MULTIGRID& g) {
    std::vector<long> out;
    for (long e = 0; e < (long)g.elemVect.size(); ++e)
        if (g.elemVect[e].children.empty()) out.push_back(e);
    return out;
}

// mixed anisotropic patterns, spliFlag chains and GRLE_CHECK balancing, tree comparison only
bool refine_patterns(int rounds) {
    Box b;
    box_make(b, 3, 2, 2);
    ddpca_multigrid_t h = ddpca_bind::tree_create(b.g);
    uint64_t s = 12345;
    auto rnd = [&](uint64_t m) { s = s * 6364136223846793005ull + 1442695040888963407ull; return (long)((s >> 33) % m); };
    bool ok = true;
    std::set<long> split;
    for (long e : leaves(b.g)) split.insert(e), b.g.elemVect[e].refiPatt = (int)(e % 7);
    for (int r = 0; r < rounds && ok; ++r) {
        std::map<long, std::set<long>> flag;
        for (long e : split)
            if (rnd(3) == 0) {
                const long nch = b.g.elemVect[e].refiPatt == 0 ? 8 : b.g.elemVect[e].refiPatt <= 3 ? 4 : 2;
                flag[e] = {rnd(nch), rnd(nch)};
            }
        ok = refine_round(b.g, h, split, flag, r, true);
        // the next round: spliFlag's children (pattern 0, the examples' contact-band choice) and a
        // few more leaves with any pattern
        for (long e : split) b.g.elemVect[e].refiPatt = 0;
        for (long e : leaves(b.g))
            if (!split.count(e) && rnd(9) == 0) split.insert(e), b.g.elemVect[e].refiPatt = (int)rnd(7);
    }
    ddpca_multigrid_destroy(h);
    return ok;
}

// CYLINDER_1's schedule on the box (MESH, CYLINDER_1.h:346-443): globInho rounds of pattern 1 and
// globHomo of pattern 0 over every leaf, then locaLeve rounds of pattern 0 on a band of the curved
// face (GRLE_CHECK balances the levels around it: hanging nodes), constraints and a load; then the
// operator pipeline on the library's refined tree against the reference's
bool refine_pipeline(int globInho, int globHomo, int locaLeve, bool rot, long& total_hang) {
    Box b;
    box_make(b, 3, 2, 2);
    ddpca_multigrid_t h = ddpca_bind::tree_create(b.g);
    bool ok = true;
    std::set<long> split;
    for (int r = 0; r < globInho + globHomo && ok; ++r) {
        split.clear();
        for (long e : leaves(b.g)) split.insert(e), b.g.elemVect[e].refiPatt = r < globInho ? 1 : 0;
        ok = refine_round(b.g, h, split, {}, r, true);
    }
    for (int r = 0; r < locaLeve && ok; ++r) {
        split.clear();
        for (long e : leaves(b.g)) {
            // a band along the curved face, off the constrained faces z = 0 and x = 0: no hanging
            // node carries a prescribed value (see dispForc in compare)
            bool near = false, off = true;
            for (long n : b.g.elemVect[e].cornNode) {
                const COOR& c = b.g.nodeCoor.at(n);
                near = near || (std::abs(c[0] - 0.75) <= 0.2 && c[1] <= 0.3);
                off = off && c[2] >= 0.2;
            }
            near = near && off;
            if (near) split.insert(e), b.g.elemVect[e].refiPatt = 0;
        }
        ok = refine_round(b.g, h, split, {}, globInho + globHomo + r, true);
    }
    if (!ok) {
        ddpca_multigrid_destroy(h);
        return false;
    }
    for (const auto& nc : b.g.nodeCoor) {
        if (nc.second[2] <= 1e-10)
            for (int a = 0; a < 3; ++a) b.g.consDofv.emplace(3 * nc.first + a, 0.0);
        else if (nc.second[0] <= 1e-10)
            b.g.consDofv.emplace(3 * nc.first + 0, 0.01 * nc.second[2]);
    }
    for (const auto& nc : b.g.nodeCoor)
        if (nc.second[2] >= 0.5 * b.nz - 1e-10) b.g.LOAD_ACCU(3 * nc.first + 1, -1.0 + 0.1 * nc.second[0]);
    return compare(b.g, 0, rot, total_hang, h);  // builds h (destroyed there)
}

}  // namespace

int main(int argc, char** argv) {
    const std::string mode = argc > 1 ? argv[1] : "cylinder";
    saved_stdout = dup(1);
    if (!std::freopen("/dev/null", "w", stdout)) return 2;  // the reference's progress output
    bool ok = true;
    long total_hang = 0;
    size_t nsub = 0;
    if (mode == "refine") {
        dup2(saved_stdout, 1);
        nsub = 1;
        ok = refine_patterns(argc > 2 ? std::atoi(argv[2]) : 3);
    } else if (mode == "refine_pipeline") {
        dup2(saved_stdout, 1);
        nsub = 1;
        ok = refine_pipeline(argc > 2 ? std::atoi(argv[2]) : 1, argc > 3 ? std::atoi(argv[3]) : 1,
                             argc > 4 ? std::atoi(argv[4]) : 2, argc > 5 && std::string(argv[5]) == "rot", total_hang);
    } else if (mode == "beam") {
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
