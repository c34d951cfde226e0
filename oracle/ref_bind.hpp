// Reference-side binding of the MI355X path -- the code a DDPCA-ADMM maintainer adds to call
// libddpca_amd.so from the reference's own classes (INTEGRATION.md quotes it).  Compiled here
// only as a check against the reference headers (oracle/ref_bind.cpp, TEST INFRASTRUCTURE);
// nothing in the product includes it.
//
//   ddpca_bind::from_reference(mc)     MCONTACT after ESTABLISH() -> established ddpca_problem_t
//   ddpca_bind::mgpis_create(g, ...)   one MULTIGRID's MGPIS hierarchy -> mgpis_t (CG_SOLV drop-in)
//
// Numbering: MULTIGRID keeps operators in the level-ordered position numbering (nodeLepo /
// posiNode, MULTIGRID.h:884-910) and maps to node ids with earlTran (OUTP_SUB1,
// MULTIGRID.h:1263-1281).  The device problem uses ONE nodal numbering per subdomain -- the
// position numbering -- so the interface operators that act on node-id vectors are moved to it:
// systTran(_pena) rows by earlTran^T, pemaInpo_r columns by earlTran.  Positions past the MGPIS
// fine level are the hanging level (hanging nodes of local refinement, coupled nodes; MULTIGRID.h:
// 836-848, 884-910): their rows of prolOper[maxiLeve] go along (ddpca_problem_set_hanging).  A
// subdomain with rotated nodes (nodeRota) hands its realProl over instead of scalProl: its
// transfers carry w R_off^T R_par blocks (MULTIGRID.h:1141-1181) a scalar stencil cannot hold.
#pragma once
#include <functional>
#include <stdexcept>
#include <string>
#include <vector>

#include "ddpca_amd.h"

namespace ddpca_bind {

using SpMat = Eigen::SparseMatrix<double, Eigen::RowMajor>;

inline void check(int rc) {
    if (rc < 0) throw std::runtime_error(std::string("libddpca_amd: ") + ddpca_last_error());
}

// A CSR view with the int64 row pointer the C ABI takes; owns that pointer copy.
struct Csr {
    SpMat m;
    std::vector<int64_t> ptr;
    explicit Csr(SpMat a) : m(std::move(a)) {
        m.makeCompressed();
        ptr.assign(m.outerIndexPtr(), m.outerIndexPtr() + m.rows() + 1);
    }
    ddpca_csr_t view() const { return {m.rows(), m.cols(), ptr.data(), m.innerIndexPtr(), m.valuePtr()}; }
};

// The MGPIS hierarchy of one MULTIGRID in mgpis_gpu_create's layout (+ what set_subdomain needs).
struct Hierarchy {
    int nlev = 0;
    std::vector<int64_t> nnodes, nfree;
    std::vector<std::vector<int32_t>> free_dof;
    std::vector<Csr> K, S;
    std::vector<const int32_t*> fd_p;
    std::vector<const int64_t*> Kp, Sp;
    std::vector<const int32_t*> Kc, Sc;
    std::vector<const double*> Kv, Sv;
    std::vector<double> presc, coords;

    explicit Hierarchy(MULTIGRID& g) {
        MGPIS& mg = g.mgpi;
        nlev = (int)mg.maxiLeve + 1;
        int64_t acc = 0;
        for (int l = 0; l < nlev; ++l) {
            acc += (int64_t)g.leveNode[l].size();
            nnodes.push_back(acc);
        }
        for (int l = 0; l < nlev; ++l) {
            SpMat C = g.consOper[l];  // one 1 per row: condensed row -> position dof
            C.makeCompressed();
            free_dof.emplace_back(C.innerIndexPtr(), C.innerIndexPtr() + C.rows());
            nfree.push_back(C.rows());
            K.emplace_back(mg.consStif[l]);
        }
        for (int l = 0; l + 1 < nlev; ++l) S.emplace_back(g.scalProl[l]);
        for (int l = 0; l < nlev; ++l) {
            fd_p.push_back(free_dof[l].data());
            Kp.push_back(K[l].ptr.data());
            Kc.push_back(K[l].m.innerIndexPtr());
            Kv.push_back(K[l].m.valuePtr());
        }
        for (auto& s : S) {
            Sp.push_back(s.ptr.data());
            Sc.push_back(s.m.innerIndexPtr());
            Sv.push_back(s.m.valuePtr());
        }
        // Dirichlet values (dispForc: constrained dofs in position order) and coordinates
        const int64_t N = nnodes.back();
        presc.assign(3 * N, 0.0);
        for (int64_t d = 0, k = 0; d < 3 * N; ++d)
            if (g.consFlag(d) == 0) presc[d] = g.dispForc(k++);
        coords.resize(3 * N);
        for (int64_t p = 0; p < N; ++p)
            for (int a = 0; a < 3; ++a) coords[3 * p + a] = g.nodeCoor.at(g.posiNode[p])[a];
    }
};

// MGPIS::CG_SOLV drop-in: a device solver for this MULTIGRID (solve with mgpis_gpu_solve on the
// condensed consForc-shaped vectors, exactly CG_SOLV's arguments).
inline mgpis_t mgpis_create(MULTIGRID& g, int device, const mgpis_options_t* opt) {
    Hierarchy h(g);
    mgpis_t out = nullptr;
    check(mgpis_gpu_create(device, h.nlev, h.nnodes.data(), h.nfree.data(), h.fd_p.data(), h.Kp.data(), h.Kc.data(),
                           h.Kv.data(), h.Sp.data(), h.Sc.data(), h.Sv.data(), opt, &out));
    return out;
}

// The same drop-in when the hierarchy has rotated nodes (MULTIGRID::nodeRota set before
// CONSTRAINT(1)): realProl carries w*R_off^T*R_par blocks a scalar stencil cannot hold
// (MULTIGRID.h:1141-1181), so it is handed over as the reference holds it.
inline mgpis_t mgpis_create_prol(MULTIGRID& g, int device, const mgpis_options_t* opt) {
    Hierarchy h(g);
    std::vector<Csr> P;
    std::vector<const int64_t*> Pp;
    std::vector<const int32_t*> Pc;
    std::vector<const double*> Pv;
    for (int l = 0; l + 1 < h.nlev; ++l) P.emplace_back(g.mgpi.realProl[l]);
    for (auto& q : P) {
        Pp.push_back(q.ptr.data());
        Pc.push_back(q.m.innerIndexPtr());
        Pv.push_back(q.m.valuePtr());
    }
    mgpis_t out = nullptr;
    check(mgpis_gpu_create_prol(device, h.nlev, h.nnodes.data(), h.nfree.data(), h.fd_p.data(), h.Kp.data(),
                                h.Kc.data(), h.Kv.data(), Pp.data(), Pc.data(), Pv.data(), opt, &out));
    return out;
}

// Read an operator back from a problem (ddpca_problem_view's CSR parts) as an Eigen matrix.
inline SpMat problem_csr(ddpca_problem_t p, const std::string& base, int64_t index, int64_t level) {
    auto get = [&](const std::string& part, const void** d, int64_t* n) {
        int dt = -1;
        check(ddpca_problem_view(p, (base + ":" + part).c_str(), index, level, d, n, &dt));
    };
    const void *sh, *pt, *cl, *vl;
    int64_t n0, n1, n2, n3;
    get("shape", &sh, &n0);
    const int64_t rows = ((const int64_t*)sh)[0], cols = ((const int64_t*)sh)[1];
    get("ptr", &pt, &n1);
    get("col", &cl, &n2);
    get("val", &vl, &n3);
    std::vector<Eigen::Triplet<double>> t;
    for (int64_t r = 0; r < rows; ++r)
        for (int64_t k = ((const int64_t*)pt)[r]; k < ((const int64_t*)pt)[r + 1]; ++k)
            t.emplace_back(r, ((const int32_t*)cl)[k], ((const double*)vl)[k]);
    SpMat m(rows, cols);
    m.setFromTriplets(t.begin(), t.end());
    return m;
}

// A MULTIGRID's element tree as REFINE left it (before TRANSFER) -> the library's operator
// pipeline (ddpca_multigrid_*), built with `extra` added to origStif (node ids; ESTABLISH adds the
// contact interfaces' systMass there, MCONTACT.h:816-822).  REFINE sizes children to 8 and fills
// the pattern's 8 / 4 / 2 (MULTIGRID.h:515-533): only those go over.
inline ddpca_multigrid_t tree_create(const MULTIGRID& g) {
    const int64_t nn = (int64_t)g.nodeCoor.size(), ne = (int64_t)g.elemVect.size();
    std::vector<double> xyz(3 * nn);
    for (const auto& nc : g.nodeCoor)
        for (int a = 0; a < 3; ++a) xyz[3 * nc.first + a] = nc.second[a];
    std::vector<int64_t> corner(8 * ne), parent(ne), level(ne), patt(ne), cptr{0}, child;
    for (int64_t e = 0; e < ne; ++e) {
        const TREE_ELEM& t = g.elemVect[e];
        for (int k = 0; k < 8; ++k) corner[8 * e + k] = t.cornNode[k];
        parent[e] = t.parent;
        level[e] = t.level;
        patt[e] = t.refiPatt;
        const size_t nch = t.children.empty() ? 0 : t.refiPatt == 0 ? 8 : t.refiPatt <= 3 ? 4 : 2;
        for (size_t q = 0; q < nch; ++q) child.push_back(t.children[q]);
        cptr.push_back((int64_t)child.size());
    }
    ddpca_multigrid_t h = nullptr;
    check(ddpca_multigrid_create(nn, xyz.data(), ne, corner.data(), parent.data(), level.data(), patt.data(), cptr.data(),
                                 child.data(), &h));
    return h;
}

// the MULTIGRID's constraints, loads, rotations, coupled nodes and material onto an unbuilt handle, then
// build (build = false: leave it unbuilt for ddpca_problem_set_subdomain_tree)
inline void tree_inputs(ddpca_multigrid_t h, const MULTIGRID& g, const SpMat* extra = nullptr, bool build = true) {
    std::vector<int64_t> idx;
    std::vector<double> val;
    auto put = [&](const char* what) {
        check(ddpca_multigrid_set(h, what, (int64_t)idx.size(), idx.data(), val.data()));
        idx.clear();
        val.clear();
    };
    for (const auto& kv : g.consDofv) idx.push_back(kv.first), val.push_back(kv.second);
    put("consDofv");  // before the loads, as the reference sets them
    for (const auto& kv : g.exteForc) idx.push_back(kv.first), val.push_back(kv.second);
    put("exteForc");
    for (const auto& kv : g.nodeRota) {
        idx.push_back(kv.first);
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) val.push_back(kv.second(i, j));
    }
    put("nodeRota");
    for (long c : g.coupNode) idx.push_back(c);
    check(ddpca_multigrid_set(h, "coupNode", (int64_t)idx.size(), idx.data(), nullptr));
    idx.clear();
    const int64_t reps = g.coupReps;
    check(ddpca_multigrid_set(h, "coupReps", 1, &reps, nullptr));
    const double mat[2] = {g.mateElas, g.matePois};
    check(ddpca_multigrid_set(h, "material", 2, nullptr, mat));
    if (!build) return;
    if (extra) {
        const Csr e(*extra);
        const ddpca_csr_t v = e.view();
        check(ddpca_multigrid_build(h, &v));
    } else {
        check(ddpca_multigrid_build(h, nullptr));
    }
}

inline ddpca_multigrid_t tree_build(const MULTIGRID& g, const SpMat* extra = nullptr) {
    ddpca_multigrid_t h = tree_create(g);
    tree_inputs(h, g, extra);
    return h;
}

// MCONTACT after ESTABLISH() -> an established device problem; with muscSett = 2 its
// MULTISCALE_1 coarse operators go along (globTran_D_1 columns moved to positions like the
// systTran rows; accuProl and globTran_1 are in free / contact numbering already).
// set_sub (optional): sets subdomain tv itself (e.g. from the element tree through
// ddpca_multigrid_* + ddpca_problem_set_subdomain_multigrid) and returns true, or false to let the
// reference's MULTIGRID operators go.
inline ddpca_problem_t from_reference(MCONTACT& mc,
                                      const std::function<bool(ddpca_problem_t, int64_t)>& set_sub = {}) {
    const int64_t nsub = (int64_t)mc.multGrid.size(), nint = (int64_t)mc.searCont.size();
    ddpca_problem_t p = nullptr;
    check(ddpca_problem_empty(nsub, nint, &p));
    for (int64_t tv = 0; tv < nsub; ++tv) {
        if (set_sub && set_sub(p, tv)) continue;
        MULTIGRID& g = mc.multGrid[tv];
        Hierarchy h(g);
        if (g.nodeRota.empty()) {
            check(ddpca_problem_set_subdomain(p, tv, h.nlev, h.nnodes.data(), h.nfree.data(), h.fd_p.data(), h.Kp.data(),
                                              h.Kc.data(), h.Kv.data(), h.Sp.data(), h.Sc.data(), h.Sv.data(),
                                              g.consForc.data(), h.presc.data(), h.coords.data()));
        } else {
            std::vector<Csr> P;
            std::vector<const int64_t*> Pp;
            std::vector<const int32_t*> Pc;
            std::vector<const double*> Pv;
            for (int l = 0; l + 1 < h.nlev; ++l) P.emplace_back(g.mgpi.realProl[l]);
            for (auto& q : P) {
                Pp.push_back(q.ptr.data());
                Pc.push_back(q.m.innerIndexPtr());
                Pv.push_back(q.m.valuePtr());
            }
            check(ddpca_problem_set_subdomain_prol(p, tv, h.nlev, h.nnodes.data(), h.nfree.data(), h.fd_p.data(),
                                                   h.Kp.data(), h.Kc.data(), h.Kv.data(), Pp.data(), Pc.data(), Pv.data(),
                                                   g.consForc.data(), h.presc.data(), h.coords.data()));
        }
        const int64_t NL = h.nnodes.back(), Nall = (int64_t)g.nodeCoor.size();
        if (Nall > NL) {  // hanging level: rows 3 NL.. of prolOper[maxiLeve] (positions x positions)
            const SpMat& Pm = g.prolOper[g.mgpi.maxiLeve];
            const Csr hang(SpMat(Pm.bottomRows(Pm.rows() - 3 * NL)));
            const ddpca_csr_t hv = hang.view();
            check(ddpca_problem_set_hanging(p, tv, Nall, &hv));
        }
    }
    for (int64_t ts = 0; ts < nint; ++ts) {
        std::vector<Csr> ops;
        for (int s = 0; s < 2; ++s) {
            const SpMat& E = mc.multGrid[mc.contBody[ts][s]].earlTran;  // position -> node id
            ops.emplace_back(mc.inpoLagr[ts][s]);
            ops.emplace_back(SpMat(mc.pemaInpo_r[ts][s] * E));
            ops.emplace_back(SpMat(E.transpose() * mc.systTran[ts][s]));
            ops.emplace_back(SpMat(E.transpose() * mc.systTran_pena[ts][s]));
            ops.emplace_back(mc.inteMass[ts][s]);
            ops.emplace_back(mc.inteMass_pena[ts][s]);
            ops.emplace_back(mc.inteInpo[ts][s]);
        }
        std::vector<ddpca_csr_t> v;
        for (const auto& o : ops) v.push_back(o.view());
        Eigen::VectorXd pema = mc.pemaInpo[ts].diagonal();
        check(ddpca_problem_set_interface(p, ts, mc.contBody[ts][0], mc.contBody[ts][1], mc.fricCoef[ts],
                                          (int64_t)mc.searCont[ts].intePoin.size(), (int64_t)mc.nodeCont[ts][0].size(),
                                          (int64_t)mc.nodeCont[ts][1].size(), pema.data(), mc.inpoNgap[ts].data(),
                                          v.data()));
    }
    if ((mc.muscSett >> 1) % 2 == 1) {
        std::vector<int64_t> dole(mc.doleMcsc.begin(), mc.doleMcsc.end());
        std::vector<int64_t> base(mc.baseReco.begin(), mc.baseReco.end());
        std::vector<Csr> gt, gd, ap;
        for (int64_t ts = 0; ts < nint; ++ts)
            for (int s = 0; s < 2; ++s) gt.emplace_back(mc.globTran_1[ts][s]);
        for (int64_t tv = 0; tv < nsub; ++tv) {
            gd.emplace_back(SpMat(mc.globTran_D_1[tv] * mc.multGrid[tv].earlTran));
            ap.emplace_back(mc.accuProl[tv]);
        }
        Csr gc(mc.globCoup_1);
        std::vector<ddpca_csr_t> vt, vd, va;
        for (const auto& o : gt) vt.push_back(o.view());
        for (const auto& o : gd) vd.push_back(o.view());
        for (const auto& o : ap) va.push_back(o.view());
        const ddpca_csr_t vc = gc.view();
        check(ddpca_problem_set_coarse_operators(p, 2, dole.data(), base.data(), &vc, mc.globForc_1.data(), vt.data(),
                                                 vd.data(), va.data()));
    }
    if ((mc.muscSett >> 0) % 2 == 1) {                         // MULTISCALE (LATIN-type) output
        std::vector<int64_t> dole(mc.doleMcsc.begin(), mc.doleMcsc.end());
        std::vector<int64_t> base(mc.baseReco.begin(), mc.baseReco.end());
        std::vector<Csr> gt, gp, gd, ap;
        for (int64_t ts = 0; ts < nint; ++ts)
            for (int s = 0; s < 2; ++s) {
                gt.emplace_back(mc.globTran[ts][s]);
                gp.emplace_back(mc.globTran_pena[ts][s]);
                gd.emplace_back(SpMat(mc.globTran_D[ts][s] * mc.multGrid[mc.contBody[ts][s]].earlTran));
            }
        for (int64_t tv = 0; tv < nsub; ++tv) ap.emplace_back(mc.accuProl[tv]);
        Csr gc(mc.globCoup);
        std::vector<ddpca_csr_t> vt, vp, vd, va;
        for (const auto& o : gt) vt.push_back(o.view());
        for (const auto& o : gp) vp.push_back(o.view());
        for (const auto& o : gd) vd.push_back(o.view());
        for (const auto& o : ap) va.push_back(o.view());
        const ddpca_csr_t vc = gc.view();
        check(ddpca_problem_set_coarse_latin(p, dole.data(), base.data(), &vc, vt.data(), vp.data(), vd.data(), va.data()));
        // MULTISCALE's coarNode (a local there, MCONTACT.h:903-957): the level-doleMcsc positions
        // of the slave body that scalEarl * scalProl[maxiLeve..doleMcsc] reaches from a contact node
        for (int64_t ts = 0; ts < nint; ++ts) {
            const MULTIGRID& g = mc.multGrid[mc.contBody[ts][0]];
            SpMat F = g.scalEarl;
            for (long l = g.mgpi.maxiLeve; l >= mc.doleMcsc[mc.contBody[ts][0]]; --l) F = SpMat(F * g.scalProl[l]);
            std::vector<char> used(F.cols(), 0);
            for (const auto& nc : mc.nodeCont[ts][0])
                for (SpMat::InnerIterator it(F, nc.first); it; ++it) used[it.col()] = 1;
            std::vector<int64_t> nodes;
            for (int64_t c = 0; c < (int64_t)used.size(); ++c)
                if (used[c]) nodes.push_back(c);
            check(ddpca_problem_set_coarse_nodes(p, ts, (int64_t)nodes.size(), nodes.data()));
        }
    }
    check(ddpca_problem_finalize(p));
    return p;
}

}  // namespace ddpca_bind
