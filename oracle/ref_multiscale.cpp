// ORACLE TEST INFRASTRUCTURE -- NOT PART OF THE PRODUCT.
//
// The coarse spaces on general trees: the library's host MULTISCALE_1 (muscSett 2) and MULTISCALE
// (muscSett 1), built by its own ESTABLISH from element trees + integration points
// (ddpca_problem_set_subdomain_tree / set_contact / set_ips, multiscale.cpp), against the
// reference's own MCONTACT::MULTISCALE_1 / MULTISCALE (MCONTACT.h:898-1536, 1672-2301) on the same
// input: globCoup(_1), globForc_1, globTran_1 or globTran / globTran_pena / globTran_D per side,
// globTran_D_1 and accuProl per subdomain -- each relative to its own largest entry, shapes equal;
// also the mortar operators of ESTABLISH with CONT_ROTA (systTran, systTran_pena, pemaInpo_r).
//   ref_multiscale cylinder MUSC [locaLeve globInho bandWidt]   (globInho + globHomo must exceed 1,
//       CYLINDER_1.h:48-49)
//       the reference's CYLINDER example (CYLINDER_1.h: curved cylinders, local refinement towards the
//       contact lines -> hanging level, curved contact search) with muscSett = MUSC, doleMcsc = 2,
//       run by its own SOLVE (MESH, search, ESTABLISH, CONTACT_ANALYSIS); the library gets the same
//       element trees (a second MESH) and the reference's integration points
//   ref_multiscale dehw MUSC [gl rotstep]
//       the library's DEHW-synthetic general mesh (the contact band refined once more -> hanging
//       level; rotated support nodes), 2 worm/wheel groups: its trees, constraints, loads, rotations
//       and integration points go to a reference MCONTACT built here, whose ESTABLISH (TRANSFER,
//       STIF_MATR, CONSTRAINT(1), the coarse space) runs on them; rotstep k > 0 also rotates every
//       k-th node of every body (contact and hanging nodes included), on both sides
// One JSON line on stdout; exit 0 when every operator is within 1e-12 (1e-11 for globTran_D_1).
#include <unistd.h>

#include <cmath>
#include <cstdio>
#include <memory>
#include <string>

#include "examples/CYLINDER_1.h"
#include "ref_bind.hpp"

namespace {

using SpMat = ddpca_bind::SpMat;

double maxabs(const SpMat& a) {
    double m = 0.0;
    for (int k = 0; k < a.outerSize(); ++k)
        for (SpMat::InnerIterator it(a, k); it; ++it) m = std::max(m, std::abs(it.value()));
    return m;
}

template <typename T>
std::vector<T> pview(ddpca_problem_t p, const std::string& what, int64_t index, int64_t level = 0) {
    const void* data = nullptr;
    int64_t n = 0;
    int dt = -1;
    ddpca_bind::check(ddpca_problem_view(p, what.c_str(), index, level, &data, &n, &dt));
    return std::vector<T>((const T*)data, (const T*)data + n);
}

Eigen::Matrix3d rotation(long node) {
    return Eigen::AngleAxisd(0.3 + 0.001 * (double)node, Eigen::Vector3d(1.0, 2.0, 3.0).normalized()).toRotationMatrix();
}

struct Cmp {
    std::string out = "{";
    double worst = 0.0;
    bool shapes = true;
    void add(const std::string& name, const SpMat& lib, const SpMat& ref) {
        double d;
        if (lib.rows() != ref.rows() || lib.cols() != ref.cols()) {
            shapes = false;
            d = 1e300;
        } else {
            const double r = maxabs(ref);
            d = r > 0 ? maxabs(SpMat(lib - ref)) / r : maxabs(lib);
        }
        worst = std::max(worst, name.rfind("globTran_D_1", 0) == 0 ? d / 10.0 : d);
        char buf[160];
        std::snprintf(buf, sizeof(buf), "%s\"%s\": %.3g", out.size() > 1 ? ", " : "", name.c_str(), d);
        out += buf;
    }
    void vec(const std::string& name, const std::vector<double>& lib, const Eigen::VectorXd& ref) {
        SpMat a(lib.size(), 1), b(ref.size(), 1);
        for (size_t i = 0; i < lib.size(); ++i)
            if (lib[i] != 0.0) a.insert(i, 0) = lib[i];
        for (int i = 0; i < ref.size(); ++i)
            if (ref[i] != 0.0) b.insert(i, 0) = ref[i];
        add(name, a, b);
    }
};

// the library's problem from element trees (unbuilt multigrid handles) + the reference's ips
ddpca_problem_t library_problem(const std::vector<MULTIGRID>& trees, const MCONTACT& ref, long musc) {
    const int64_t nsub = (int64_t)trees.size(), nint = (int64_t)ref.searCont.size();
    ddpca_problem_t p = nullptr;
    ddpca_bind::check(ddpca_problem_empty(nsub, nint, &p));
    for (int64_t tv = 0; tv < nsub; ++tv) {
        ddpca_multigrid_t h = ddpca_bind::tree_create(trees[tv]);
        ddpca_bind::tree_inputs(h, trees[tv], nullptr, false);
        ddpca_bind::check(ddpca_problem_set_subdomain_tree(p, tv, h));
        ddpca_multigrid_destroy(h);
    }
    for (int64_t ts = 0; ts < nint; ++ts) {
        ddpca_bind::check(ddpca_problem_set_contact(p, ts, ref.contBody[ts][0], ref.contBody[ts][1]));
        const auto& ips = ref.searCont[ts].intePoin;
        const int64_t n = (int64_t)ips.size();
        std::vector<int64_t> node(8 * n);
        std::vector<double> shap(8 * n), basis(9 * n), gap(n), w(n);
        for (int64_t q = 0; q < n; ++q) {
            for (int s = 0; s < 2; ++s)
                for (int k = 0; k < 4; ++k) {
                    node[8 * q + 4 * s + k] = ips[q].node[s][k];
                    shap[8 * q + 4 * s + k] = ips[q].shapFunc[s][k];
                }
            for (int a = 0; a < 3; ++a)
                for (int b = 0; b < 3; ++b) basis[9 * q + 3 * a + b] = ips[q].basiVect[a](b);
            gap[q] = ips[q].initNgap;
            w[q] = ips[q].quadWeig;
        }
        ddpca_bind::check(ddpca_problem_set_ips(p, ts, n, node.data(), shap.data(), basis.data(), gap.data(), w.data(),
                                                ref.fricCoef[ts], ref.penaFact_n[ts], ref.penaFact_f[ts]));
    }
    std::vector<int64_t> dole(ref.doleMcsc.begin(), ref.doleMcsc.end());
    ddpca_bind::check(ddpca_problem_set_coarse(p, musc, dole.data()));
    ddpca_bind::check(ddpca_problem_establish(p));
    return p;
}

// the comparisons: coarse operators (positions on the nodal columns: X * earlTran) and the mortar
// operators that carry CONT_ROTA
Cmp compare(ddpca_problem_t p, MCONTACT& ref, long musc) {
    Cmp c;
    const int64_t nsub = (int64_t)ref.multGrid.size(), nint = (int64_t)ref.searCont.size();
    auto lib = [&](const std::string& b, int64_t i) { return ddpca_bind::problem_csr(p, b, i, 0); };
    for (int64_t ts = 0; ts < nint; ++ts)
        for (int s = 0; s < 2; ++s) {
            const SpMat& E = ref.multGrid[ref.contBody[ts][s]].earlTran;  // position -> node id
            const std::string sfx = "[" + std::to_string(ts) + "," + std::to_string(s) + "]";
            c.add("systTran" + sfx, lib("systTran", 2 * ts + s), SpMat(E.transpose() * ref.systTran[ts][s]));
            c.add("systTran_pena" + sfx, lib("systTran_pena", 2 * ts + s), SpMat(E.transpose() * ref.systTran_pena[ts][s]));
            c.add("pemaInpo_r" + sfx, lib("pemaInpo_r", 2 * ts + s), SpMat(ref.pemaInpo_r[ts][s] * E));
        }
    if (musc == 2) {
        c.add("globCoup_1", lib("globCoup_1", 0), ref.globCoup_1);
        c.vec("globForc_1", pview<double>(p, "globForc_1", 0), ref.globForc_1);
        for (int64_t ts = 0; ts < nint; ++ts)
            for (int s = 0; s < 2; ++s)
                c.add("globTran_1[" + std::to_string(ts) + "," + std::to_string(s) + "]", lib("globTran_1", 2 * ts + s),
                      ref.globTran_1[ts][s]);
        for (int64_t tv = 0; tv < nsub; ++tv)
            c.add("globTran_D_1[" + std::to_string(tv) + "]", lib("globTran_D_1", tv),
                  SpMat(ref.globTran_D_1[tv] * ref.multGrid[tv].earlTran));
    } else {
        c.add("globCoup", lib("globCoup_1", 0), ref.globCoup);
        for (int64_t ts = 0; ts < nint; ++ts)
            for (int s = 0; s < 2; ++s) {
                const std::string sfx = "[" + std::to_string(ts) + "," + std::to_string(s) + "]";
                c.add("globTran" + sfx, lib("globTran", 2 * ts + s), ref.globTran[ts][s]);
                c.add("globTran_pena" + sfx, lib("globTran_pena", 2 * ts + s), ref.globTran_pena[ts][s]);
                c.add("globTran_D" + sfx, lib("globTran_D", 2 * ts + s),
                      SpMat(ref.globTran_D[ts][s] * ref.multGrid[ref.contBody[ts][s]].earlTran));
            }
    }
    for (int64_t tv = 0; tv < nsub; ++tv) c.add("accuProl[" + std::to_string(tv) + "]", lib("accuProl", tv), ref.accuProl[tv]);
    return c;
}

int saved_stdout = -1;

template <typename F>
void quiet(F&& f) {
    std::fflush(stdout);
    if (!std::freopen("/dev/null", "w", stdout)) std::exit(2);
    f();
    std::fflush(stdout);
    dup2(saved_stdout, 1);
}

void rotate_every(std::vector<MULTIGRID>& grids, long step) {
    if (step <= 0) return;
    for (auto& g : grids)
        for (const auto& nc : g.nodeCoor)
            if (nc.first % step == 3 && !g.nodeRota.count(nc.first)) g.nodeRota.emplace(nc.first, rotation(nc.first));
}

// ---------------------------------------------------------------- the reference's CYLINDER example
int run_cylinder(long musc, long locaLeve, long globInho, double bandWidt) {
    std::unique_ptr<CYLINDER_1> c(new CYLINDER_1);
    std::unique_ptr<CYLINDER_1> t(new CYLINDER_1);
    quiet([&] {
        c->copyNumb = 1;
        c->locaLeve = locaLeve;
        c->globInho = globInho;
        c->bandWidt = bandWidt;
        c->muscSett = musc;
        std::fprintf(stderr, "[ref_multiscale] reference SOLVE\n");
        c->SOLVE(1);  // MESH, contact search, ESTABLISH (MULTISCALE / MULTISCALE_1), CONTACT_ANALYSIS
        t->copyNumb = 1;
        t->locaLeve = locaLeve;
        t->globInho = globInho;
        t->bandWidt = bandWidt;
        t->MESH();  // the same element trees, before TRANSFER
    });
    std::fprintf(stderr, "[ref_multiscale] library ESTABLISH\n");
    ddpca_problem_t p = library_problem(t->multGrid, *c, musc);
    std::fprintf(stderr, "[ref_multiscale] compare\n");
    Cmp cmp = compare(p, *c, musc);
    long nhang = 0;
    for (auto& g : c->multGrid) nhang += (long)g.leveNode[g.mgpi.maxiLeve + 1].size();
    const long n = musc == 2 ? (long)c->globCoup_1.rows() : (long)c->globCoup.rows();
    const bool ok = cmp.shapes && cmp.worst <= 1e-12;
    std::printf("{\"case\": \"cylinder\", \"muscSett\": %ld, \"ok\": %s, \"coarse_rows\": %ld, \"hanging_nodes\": %ld, "
                "\"reference_iterations\": %ld, \"worst\": %.3g, \"operators\": %s}}\n",
                musc, ok ? "true" : "false", n, nhang, (long)c->iterNumbReco, cmp.worst, cmp.out.c_str());
    ddpca_problem_destroy(p);
    return ok ? 0 : 1;
}

// ---------------------------------------------------------------- the library's DEHW-synthetic general mesh
int run_dehw(long musc, long gl, long rotstep) {
    // 2 groups, 3 x 2 x 2 coarse hexes, Coulomb mu 0.2, contact / glued faces over 2 x 2 / 1 x 1
    // polygons, the contact band refined once more (hanging level), rotated support nodes
    const double par[10] = {2, 3, 2, 2, (double)gl, 0.2, 1, 0, 1, 1};
    ddpca_problem_t gen = nullptr;
    ddpca_bind::check(ddpca_problem_create("dehw", par, 10, &gen));
    const int64_t nsub = pview<int64_t>(gen, "sizes", 0)[0], nint = pview<int64_t>(gen, "sizes", 0)[1];
    std::unique_ptr<MCONTACT> ref(new MCONTACT);
    ref->multGrid.resize(nsub);
    for (int64_t tv = 0; tv < nsub; ++tv) {
        MULTIGRID& g = ref->multGrid[tv];
        const auto xyz = pview<double>(gen, "coords", tv);
        for (size_t i = 0; i < xyz.size() / 3; ++i)
            if (g.TRY_ADD_NODE(COOR(xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2])) != (long)i) {
                std::fprintf(stderr, "node %zu: coordinates not distinct\n", i);
                return 2;
            }
        const auto corner = pview<int64_t>(gen, "tree:corner", tv), parent = pview<int64_t>(gen, "tree:parent", tv),
                   level = pview<int64_t>(gen, "tree:level", tv), patt = pview<int64_t>(gen, "tree:refiPatt", tv),
                   cptr = pview<int64_t>(gen, "tree:child_ptr", tv), child = pview<int64_t>(gen, "tree:child", tv);
        for (size_t e = 0; e < parent.size(); ++e) {
            TREE_ELEM el;
            el.parent = parent[e];
            el.cornNode.assign(corner.begin() + 8 * e, corner.begin() + 8 * e + 8);
            el.level = level[e];
            el.refiPatt = patt[e];
            el.children.resize(0);
            if (cptr[e + 1] > cptr[e]) {
                el.children.assign(8, 0);  // REFINE: children.resize(8), the pattern's first 8 / 4 / 2 set
                for (int64_t q = cptr[e]; q < cptr[e + 1]; ++q) el.children[q - cptr[e]] = child[q];
            }
            g.ADD_ELEMENT(el);
        }
        g.coupReps = -1;
        const auto mat = pview<double>(gen, "material", tv);
        g.mateElas = mat[0];
        g.matePois = mat[1];
        const auto cd = pview<int64_t>(gen, "consDofv", tv);
        const auto cv = pview<double>(gen, "consDofv_val", tv);
        for (size_t k = 0; k < cd.size(); ++k) g.consDofv.emplace(cd[k], cv[k]);
        const auto f = pview<double>(gen, "exteForc", tv);
        for (size_t d = 0; d < f.size(); ++d)
            if (f[d] != 0.0) g.exteForc.emplace((long)d, f[d]);
        const auto rn = pview<int64_t>(gen, "nodeRota", tv);
        const auto rv = pview<double>(gen, "nodeRota_val", tv);
        for (size_t k = 0; k < rn.size(); ++k) {
            Eigen::Matrix3d R;
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j) R(i, j) = rv[9 * k + 3 * i + j];
            g.nodeRota.emplace(rn[k], R);
        }
    }
    rotate_every(ref->multGrid, rotstep);
    const std::vector<MULTIGRID> trees = ref->multGrid;  // before the reference's TRANSFER
    ref->searCont.resize(nint);
    ref->contBody.resize(nint);
    ref->fricCoef.resize(nint);
    ref->penaFact_n.resize(nint);
    ref->penaFact_f.resize(nint);
    for (int64_t ts = 0; ts < nint; ++ts) {
        const auto body = pview<int64_t>(gen, "iface_body", ts);
        const auto prm = pview<double>(gen, "iface_param", ts);
        ref->contBody[ts] = {(long)body[0], (long)body[1]};
        ref->fricCoef[ts] = prm[0];
        ref->penaFact_n[ts] = prm[1];
        ref->penaFact_f[ts] = prm[2];
        ref->searCont[ts].mastGrid = &ref->multGrid[body[0]];
        ref->searCont[ts].slavGrid = &ref->multGrid[body[1]];
        const auto node = pview<int64_t>(gen, "ip_node", ts);
        const auto shap = pview<double>(gen, "ip_shap", ts), basis = pview<double>(gen, "ip_basis", ts),
                   gap = pview<double>(gen, "ip_gap", ts), w = pview<double>(gen, "ip_w", ts);
        for (size_t q = 0; q < w.size(); ++q) {
            INTEGRAL_POINT ip;
            for (int s = 0; s < 2; ++s)
                for (int k = 0; k < 4; ++k) {
                    ip.node[s][k] = node[8 * q + 4 * s + k];
                    ip.shapFunc[s][k] = shap[8 * q + 4 * s + k];
                }
            for (int a = 0; a < 3; ++a) ip.basiVect[a] = Eigen::Vector3d(basis[9 * q + 3 * a], basis[9 * q + 3 * a + 1], basis[9 * q + 3 * a + 2]);
            ip.initNgap = gap[q];
            ip.quadWeig = w[q];
            ref->searCont[ts].intePoin.push_back(ip);
        }
    }
    ref->muscSett = musc;
    ref->doleMcsc.assign(nsub, 1);
    ddpca_problem_destroy(gen);
    quiet([&] { ref->ESTABLISH(); });
    ddpca_problem_t p = library_problem(trees, *ref, musc);
    Cmp cmp = compare(p, *ref, musc);
    long nhang = 0, nrot = 0;
    for (auto& g : ref->multGrid) nhang += (long)g.leveNode[g.mgpi.maxiLeve + 1].size(), nrot += (long)g.nodeRota.size();
    const long n = musc == 2 ? (long)ref->globCoup_1.rows() : (long)ref->globCoup.rows();
    const bool ok = cmp.shapes && cmp.worst <= 1e-12;
    std::printf("{\"case\": \"dehw\", \"muscSett\": %ld, \"gl\": %ld, \"rotstep\": %ld, \"ok\": %s, \"coarse_rows\": %ld, "
                "\"hanging_nodes\": %ld, \"rotated_nodes\": %ld, \"worst\": %.3g, \"operators\": %s}}\n",
                musc, gl, rotstep, ok ? "true" : "false", n, nhang, nrot, cmp.worst, cmp.out.c_str());
    ddpca_problem_destroy(p);
    return ok ? 0 : 1;
}

}  // namespace

int main(int argc, char** argv) {
    saved_stdout = dup(1);
    const std::string mode = argc > 1 ? argv[1] : "cylinder";
    const long musc = argc > 2 ? std::atol(argv[2]) : 2;
    try {
        if (mode == "cylinder")
            return run_cylinder(musc, argc > 3 ? std::atol(argv[3]) : 2, argc > 4 ? std::atol(argv[4]) : 2,
                                argc > 5 ? std::atof(argv[5]) : 2.0e-4);
        if (mode == "dehw") return run_dehw(musc, argc > 3 ? std::atol(argv[3]) : 2, argc > 4 ? std::atol(argv[4]) : 0);
    } catch (const std::exception& e) {
        std::printf("{\"ok\": false, \"error\": \"%s\"}\n", e.what());
        return 1;
    }
    std::fprintf(stderr, "usage: ref_multiscale cylinder|dehw MUSC [...]\n");
    return 2;
}
