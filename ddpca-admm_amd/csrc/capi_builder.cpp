// C ABI: operator-level problem builder.  A caller that already owns the reference's operators
// (its MULTIGRID/MGPIS hierarchy per subdomain and the interface operators MCONTACT::ESTABLISH
// produced, MCONTACT.h:181-896) hands them over in the reference's own layouts, and the result
// is an established ddpca_problem_t that mcontact_gpu_create / ddpca_problem_mgpis accept --
// the host restatement (multigrid.cpp, mcontact.cpp) is bypassed entirely.
#include <cstring>
#include <memory>
#include <string>

#include "../../include/ddpca_amd.h"
#include "common.hpp"
#include "problem.hpp"

using namespace ddpca;

namespace {

Csr to_csr(const ddpca_csr_t& m, const char* what) {
    if (m.nrow < 0 || m.ncol < 0 || (!m.ptr && m.nrow > 0)) throw ApiError(DDPCA_EINVAL, std::string(what) + ": bad CSR");
    Csr c;
    c.nrow = m.nrow;
    c.ncol = m.ncol;
    c.ptr.assign(m.ptr, m.ptr + m.nrow + 1);
    if (m.nrow == 0) c.ptr.assign(1, 0);
    const int64_t nnz = c.ptr.back();
    if (nnz < 0 || (nnz > 0 && (!m.col || !m.val))) throw ApiError(DDPCA_EINVAL, std::string(what) + ": bad CSR");
    c.col.assign(m.col, m.col + nnz);
    c.val.assign(m.val, m.val + nnz);
    for (int64_t r = 0; r < c.nrow; ++r)
        if (c.ptr[r + 1] < c.ptr[r]) throw ApiError(DDPCA_EINVAL, std::string(what) + ": row pointer not monotone");
    for (int32_t j : c.col)
        if (j < 0 || j >= c.ncol) throw ApiError(DDPCA_EINVAL, std::string(what) + ": column out of range");
    return c;
}

void expect_shape(const Csr& c, int64_t r, int64_t k, const char* what) {
    if (c.nrow != r || c.ncol != k)
        throw ApiError(DDPCA_EINVAL, std::string(what) + ": shape " + std::to_string(c.nrow) + "x" + std::to_string(c.ncol) +
                                         ", expected " + std::to_string(r) + "x" + std::to_string(k));
}

Problem& builder(ddpca_problem_t h) {
    Problem& P = *reinterpret_cast<Problem*>(h);
    if (P.established) throw ApiError(DDPCA_ESTATE, "problem already established");
    return P;
}

}  // namespace

extern "C" {

int ddpca_problem_empty(int64_t nsub, int64_t nint, ddpca_problem_t* out) {
    return guarded([&] {
        if (nsub < 1 || nint < 0 || !out) throw ApiError(DDPCA_EINVAL, "nsub >= 1, nint >= 0");
        auto P = std::make_unique<Problem>();
        P->mc.multGrid.resize(nsub);
        P->mc.searCont.resize(nint);
        P->owned.assign(nsub, 0);
        *out = reinterpret_cast<ddpca_problem_t>(P.release());
    });
}

}  // extern "C"

namespace {

// Shared body of set_subdomain / set_subdomain_prol: `transfers(g)` fills g.scalProl.
template <typename Tr>
void set_subdomain_common(ddpca_problem_t h, int64_t tv, int nlev, const int64_t* nnodes, const int64_t* nfree,
                          const int32_t* const* free_dof, const int64_t* const* K_ptr, const int32_t* const* K_col,
                          const double* const* K_val, bool have_transfers, Tr&& transfers, const double* consForc,
                          const double* presc, const double* coords) {
    Problem& P = builder(h);
    if (tv < 0 || tv >= (int64_t)P.mc.multGrid.size()) throw ApiError(DDPCA_EINVAL, "subdomain index");
    if (nlev < 1 || !nnodes || !nfree || !free_dof || !K_ptr || !K_col || !K_val || !consForc)
        throw ApiError(DDPCA_EINVAL, "null argument");
    if (nlev > 1 && !have_transfers) throw ApiError(DDPCA_EINVAL, "transfer operators missing");
    for (int l = 0; l < nlev; ++l) {
        if (nnodes[l] < 1 || (l > 0 && nnodes[l] < nnodes[l - 1])) throw ApiError(DDPCA_EINVAL, "nnodes must grow by level");
        if (nfree[l] < 0 || nfree[l] > 3 * nnodes[l]) throw ApiError(DDPCA_EINVAL, "nfree out of range");
    }
    MULTIGRID g;
    const int64_t N = nnodes[nlev - 1];
    g.maxiLeve = nlev - 1;
    g.leveCount.assign(nnodes, nnodes + nlev);
    g.freeCount.assign(nfree, nfree + nlev);
    g.levelStif.resize(nlev);
    for (int l = 0; l < nlev; ++l) {
        // the level-l free dofs must be the level-(l+1) free dofs of the first nnodes[l] nodes
        // (level-ordered numbering, MULTIGRID.h:884-910)
        for (int64_t r = 0; r < nfree[l]; ++r)
            if (free_dof[l][r] < 0 || free_dof[l][r] >= 3 * nnodes[l] || (r && free_dof[l][r] <= free_dof[l][r - 1]))
                throw ApiError(DDPCA_EINVAL, "free_dof[" + std::to_string(l) + "] must be increasing nodal dofs of the level");
        g.levelStif[l] = condensed_to_bsr3(nnodes[l], nfree[l], free_dof[l], K_ptr[l], K_col[l], K_val[l]);
    }
    transfers(g);
    g.consFlag.assign(3 * N, 0);
    g.freeIndex.assign(3 * N, -1);
    for (int64_t r = 0; r < nfree[nlev - 1]; ++r) {
        g.consFlag[free_dof[nlev - 1][r]] = 1;
        g.freeIndex[free_dof[nlev - 1][r]] = (int32_t)r;
    }
    for (int l = 0; l + 1 < nlev; ++l)
        for (int64_t r = 0; r < nfree[l]; ++r)
            if (!g.consFlag[free_dof[l][r]]) throw ApiError(DDPCA_EINVAL, "coarse free dof constrained on the fine level");
    g.consForc.assign(consForc, consForc + nfree[nlev - 1]);
    g.dispForc.clear();  // constrained dofs' values in dof order (MULTIGRID::CONSTRAINT layout)
    for (int64_t d = 0; d < 3 * N; ++d)
        if (!g.consFlag[d]) {
            const double v = presc ? presc[d] : 0.0;
            g.consDofv[d] = v;
            g.dispForc.push_back(v);
        }
    if (coords) {
        g.nodeCoor.resize(N);
        for (int64_t i = 0; i < N; ++i)
            for (int a = 0; a < 3; ++a) g.nodeCoor[i][a] = coords[3 * i + a];
    }
    P.mc.multGrid[tv] = std::move(g);
    P.owned[tv] = 1;
}

}  // namespace

extern "C" {

int ddpca_problem_set_subdomain(ddpca_problem_t h, int64_t tv, int nlev, const int64_t* nnodes, const int64_t* nfree,
                                const int32_t* const* free_dof, const int64_t* const* K_ptr,
                                const int32_t* const* K_col, const double* const* K_val,
                                const int64_t* const* S_ptr, const int32_t* const* S_col,
                                const double* const* S_w, const double* consForc, const double* presc,
                                const double* coords) {
    return guarded([&] {
        set_subdomain_common(
            h, tv, nlev, nnodes, nfree, free_dof, K_ptr, K_col, K_val, S_ptr && S_col && S_w,
            [&](MULTIGRID& g) {
                for (int l = 0; l + 1 < nlev; ++l)
                    g.scalProl.push_back(make_stencil(nnodes[l + 1], nnodes[l], S_ptr[l], S_col[l], S_w[l]));
            },
            consForc, presc, coords);
    });
}

int ddpca_problem_set_subdomain_prol(ddpca_problem_t h, int64_t tv, int nlev, const int64_t* nnodes,
                                     const int64_t* nfree, const int32_t* const* free_dof,
                                     const int64_t* const* K_ptr, const int32_t* const* K_col,
                                     const double* const* K_val, const int64_t* const* P_ptr,
                                     const int32_t* const* P_col, const double* const* P_val,
                                     const double* consForc, const double* presc, const double* coords) {
    return guarded([&] {
        set_subdomain_common(
            h, tv, nlev, nnodes, nfree, free_dof, K_ptr, K_col, K_val, P_ptr && P_col && P_val,
            [&](MULTIGRID& g) {
                for (int l = 0; l + 1 < nlev; ++l) {
                    const int64_t nnz = P_ptr[l][nfree[l + 1]];
                    for (int64_t k = 0; k < nnz; ++k)
                        if (P_col[l][k] < 0 || P_col[l][k] >= nfree[l]) throw ApiError(DDPCA_EINVAL, "realProl column out of range");
                    g.scalProl.push_back(prol_to_stencil(nnodes[l + 1], nnodes[l], nfree[l + 1], free_dof[l + 1], free_dof[l],
                                                         P_ptr[l], P_col[l], P_val[l]));
                }
            },
            consForc, presc, coords);
    });
}

int ddpca_problem_set_hanging(ddpca_problem_t h, int64_t tv, int64_t nnodes_all, const ddpca_csr_t* hang) {
    return guarded([&] {
        Problem& P = builder(h);
        if (tv < 0 || tv >= (int64_t)P.mc.multGrid.size() || !hang) throw ApiError(DDPCA_EINVAL, "subdomain index / null");
        MULTIGRID& g = P.mc.multGrid[tv];
        if (g.leveCount.empty()) throw ApiError(DDPCA_ESTATE, "set the subdomain before its hanging level");
        for (const Interface& itf : P.mc.searCont)
            if (!itf.inteMass[0].ptr.empty() && (itf.body[0] == tv || itf.body[1] == tv))
                throw ApiError(DDPCA_ESTATE, "set the hanging level before the subdomain's interfaces");
        const int64_t NL = g.leveCount.back();
        if (nnodes_all < NL) throw ApiError(DDPCA_EINVAL, "nnodes_all below the fine level's node count");
        Csr H = to_csr(*hang, "hanging prolongation");
        expect_shape(H, 3 * (nnodes_all - NL), 3 * NL, "hanging prolongation");
        g.nodeAll = nnodes_all == NL ? 0 : nnodes_all;
        g.hangProl = std::move(H);
    });
}

int ddpca_problem_set_interface(ddpca_problem_t h, int64_t ts, int64_t body0, int64_t body1, double fric,
                                int64_t nip, int64_t nnc0, int64_t nnc1, const double* pemaDiag,
                                const double* inpoNgap, const ddpca_csr_t* ops) {
    return guarded([&] {
        Problem& P = builder(h);
        const int64_t nsub = (int64_t)P.mc.multGrid.size();
        if (ts < 0 || ts >= (int64_t)P.mc.searCont.size()) throw ApiError(DDPCA_EINVAL, "interface index");
        if (body0 < 0 || body0 >= nsub || body1 < 0 || body1 >= nsub || body0 == body1)
            throw ApiError(DDPCA_EINVAL, "interface bodies");
        if (nip < 0 || nnc0 < 0 || nnc1 < 0 || !ops || (nip > 0 && (!pemaDiag || !inpoNgap)))
            throw ApiError(DDPCA_EINVAL, "null argument");
        Interface I;
        I.body[0] = body0;
        I.body[1] = body1;
        I.fric = fric;
        I.ip.resize(nip);  // the device path needs the count only; the geometry stays with the caller
        I.nodeCont[0].resize(nnc0);
        I.nodeCont[1].resize(nnc1);
        const int64_t mip = I.mip();
        I.pemaDiag.assign(pemaDiag, pemaDiag + mip);
        I.inpoNgap.assign(inpoNgap, inpoNgap + mip);
        static const char* kName[7] = {"inpoLagr", "pemaInpo_r", "systTran", "systTran_pena", "inteMass",
                                       "inteMass_pena", "inteInpo"};
        for (int s = 0; s < 2; ++s) {
            const ddpca_csr_t* o = ops + 7 * s;
            Csr* dst[7] = {&I.inpoLagr[s], &I.pemaInpo_r[s], &I.systTran[s], &I.systTran_pena[s], &I.inteMass[s],
                           &I.inteMass_pena[s], &I.inteInpo[s]};
            for (int k = 0; k < 7; ++k) *dst[k] = to_csr(o[k], kName[k]);
            const int64_t m = I.mside(s);
            if (P.mc.multGrid[I.body[s]].leveCount.empty())
                throw ApiError(DDPCA_ESTATE, "set the interface's subdomains before the interface");
            const int64_t n3 = 3 * P.mc.multGrid[I.body[s]].nodalCount();
            expect_shape(I.inpoLagr[s], mip, m, "inpoLagr");
            expect_shape(I.pemaInpo_r[s], mip, n3, "pemaInpo_r");
            expect_shape(I.systTran[s], n3, m, "systTran");
            expect_shape(I.systTran_pena[s], n3, m, "systTran_pena");
            expect_shape(I.inteMass[s], m, m, "inteMass");
            expect_shape(I.inteMass_pena[s], m, m, "inteMass_pena");
            expect_shape(I.inteInpo[s], m, mip, "inteInpo");
        }
        P.mc.searCont[ts] = std::move(I);
    });
}

int ddpca_problem_set_coarse_operators(ddpca_problem_t h, int64_t muscSett, const int64_t* doleMcsc,
                                       const int64_t* baseReco, const ddpca_csr_t* globCoup_1, const double* globForc_1,
                                       const ddpca_csr_t* globTran_1, const ddpca_csr_t* globTran_D_1,
                                       const ddpca_csr_t* accuProl) {
    return guarded([&] {
        Problem& P = builder(h);
        const int64_t nsub = (int64_t)P.mc.multGrid.size(), nint = (int64_t)P.mc.searCont.size();
        if (muscSett != 2) throw ApiError(DDPCA_EINVAL, "only muscSett = 2 (MULTISCALE_1) is supported");
        if (!doleMcsc || !baseReco || !globCoup_1 || !globForc_1 || (nint && !globTran_1) || !globTran_D_1 || !accuProl)
            throw ApiError(DDPCA_EINVAL, "null argument");
        CoarseSpace C;
        C.assembled = true;
        C.baseReco.assign(baseReco, baseReco + nsub + 1);
        C.n = C.baseReco[nsub];
        P.mc.doleMcsc.assign(doleMcsc, doleMcsc + nsub);
        for (int64_t tv = 0; tv < nsub; ++tv) {
            const MULTIGRID& g = P.mc.multGrid[tv];
            if (g.leveCount.empty()) throw ApiError(DDPCA_ESTATE, "set every subdomain before the coarse operators");
            const int64_t d = P.mc.doleMcsc[tv];
            if (d < 0 || d > g.maxiLeve) throw ApiError(DDPCA_EINVAL, "doleMcsc out of range");
            if (C.baseReco[tv + 1] - C.baseReco[tv] != g.freeCount[d]) throw ApiError(DDPCA_EINVAL, "baseReco does not match nfree[doleMcsc]");
        }
        C.globCoup_1 = to_csr(*globCoup_1, "globCoup_1");
        expect_shape(C.globCoup_1, C.n, C.n, "globCoup_1");
        C.globForc_1.assign(globForc_1, globForc_1 + C.n);
        C.globTran_1.assign(nint, {});
        for (int64_t ts = 0; ts < nint; ++ts)
            for (int s = 0; s < 2; ++s) {
                const Interface& itf = P.mc.searCont[ts];
                if (itf.inteMass[s].ptr.empty()) throw ApiError(DDPCA_ESTATE, "set every interface before the coarse operators");
                C.globTran_1[ts][s] = to_csr(globTran_1[2 * ts + s], "globTran_1");
                expect_shape(C.globTran_1[ts][s], C.n, itf.mside(s), "globTran_1");
            }
        for (int64_t tv = 0; tv < nsub; ++tv) {
            const MULTIGRID& g = P.mc.multGrid[tv];
            C.globTran_D_full.push_back(to_csr(globTran_D_1[tv], "globTran_D_1"));
            expect_shape(C.globTran_D_full.back(), C.n, 3 * g.nodalCount(), "globTran_D_1");
            C.accuProl_full.push_back(to_csr(accuProl[tv], "accuProl"));
            expect_shape(C.accuProl_full.back(), g.freeCount.back(), g.freeCount[P.mc.doleMcsc[tv]], "accuProl");
        }
        C.built.assign(nsub, 1);
        C.ready = true;
        P.mc.coarse = std::move(C);
        P.mc.muscSett = muscSett;
    });
}

int ddpca_problem_set_coarse_nodes(ddpca_problem_t h, int64_t ts, int64_t n, const int64_t* nodes) {
    return guarded([&] {
        Problem& P = builder(h);
        CoarseSpace& C = P.mc.coarse;
        if (!C.latin) throw ApiError(DDPCA_ESTATE, "set_coarse_nodes after set_coarse_latin");
        const int64_t nint = (int64_t)P.mc.searCont.size();
        if (ts < 0 || ts >= nint) throw ApiError(DDPCA_EINVAL, "interface index");
        if (n < 0 || (n > 0 && !nodes)) throw ApiError(DDPCA_EINVAL, "null argument");
        const int64_t b0 = P.mc.searCont[ts].body[0];
        const int64_t lim = P.mc.multGrid[b0].leveCount[P.mc.doleMcsc[b0]];
        for (int64_t k = 0; k < n; ++k)
            if (nodes[k] < 0 || nodes[k] >= lim || (k && nodes[k] <= nodes[k - 1]))
                throw ApiError(DDPCA_EINVAL, "coarse contact nodes: increasing level-doleMcsc positions of the slave body");
        if ((int64_t)C.coarNode.size() != nint) C.coarNode.assign(nint, {});
        C.coarNode[ts].assign(nodes, nodes + n);
    });
}

int ddpca_problem_set_coarse_latin(ddpca_problem_t h, const int64_t* doleMcsc, const int64_t* baseReco,
                                   const ddpca_csr_t* globCoup, const ddpca_csr_t* globTran,
                                   const ddpca_csr_t* globTran_pena, const ddpca_csr_t* globTran_D,
                                   const ddpca_csr_t* accuProl) {
    return guarded([&] {
        Problem& P = builder(h);
        const int64_t nsub = (int64_t)P.mc.multGrid.size(), nint = (int64_t)P.mc.searCont.size();
        if (!doleMcsc || !baseReco || !globCoup || (nint && (!globTran || !globTran_pena || !globTran_D)) || !accuProl)
            throw ApiError(DDPCA_EINVAL, "null argument");
        CoarseSpace C;
        C.assembled = true;
        C.latin = true;
        C.baseReco.assign(baseReco, baseReco + nsub + 1);
        P.mc.doleMcsc.assign(doleMcsc, doleMcsc + nsub);
        C.globCoup_1 = to_csr(*globCoup, "globCoup");
        C.n = C.globCoup_1.nrow;
        expect_shape(C.globCoup_1, C.n, C.n, "globCoup");
        if (C.n < C.baseReco[nsub]) throw ApiError(DDPCA_EINVAL, "globCoup smaller than baseReco[nsub]");
        for (int64_t tv = 0; tv < nsub; ++tv) {
            const MULTIGRID& g = P.mc.multGrid[tv];
            if (g.leveCount.empty()) throw ApiError(DDPCA_ESTATE, "set every subdomain before the coarse operators");
            const int64_t d = P.mc.doleMcsc[tv];
            if (d < 0 || d > g.maxiLeve) throw ApiError(DDPCA_EINVAL, "doleMcsc out of range");
            if (C.baseReco[tv + 1] - C.baseReco[tv] != g.freeCount[d]) throw ApiError(DDPCA_EINVAL, "baseReco does not match nfree[doleMcsc]");
            C.accuProl_full.push_back(to_csr(accuProl[tv], "accuProl"));
            expect_shape(C.accuProl_full.back(), g.freeCount.back(), g.freeCount[d], "accuProl");
        }
        C.globForc_1.assign(C.n, 0.0);
        C.globTran_L.assign(nint, {});
        C.globTran_pena_L.assign(nint, {});
        C.globTran_D_L.assign(nint, {});
        for (int64_t ts = 0; ts < nint; ++ts)
            for (int s = 0; s < 2; ++s) {
                const Interface& itf = P.mc.searCont[ts];
                if (itf.inteMass[s].ptr.empty()) throw ApiError(DDPCA_ESTATE, "set every interface before the coarse operators");
                const int64_t n3 = 3 * P.mc.multGrid[itf.body[s]].nodalCount();
                C.globTran_L[ts][s] = to_csr(globTran[2 * ts + s], "globTran");
                C.globTran_pena_L[ts][s] = to_csr(globTran_pena[2 * ts + s], "globTran_pena");
                C.globTran_D_L[ts][s] = to_csr(globTran_D[2 * ts + s], "globTran_D");
                expect_shape(C.globTran_L[ts][s], C.n, itf.mside(s), "globTran");
                expect_shape(C.globTran_pena_L[ts][s], C.n, itf.mside(s), "globTran_pena");
                expect_shape(C.globTran_D_L[ts][s], C.n, n3, "globTran_D");
            }
        C.built.assign(nsub, 1);
        C.ready = true;
        P.mc.coarse = std::move(C);
        P.mc.muscSett = 1;
    });
}

int ddpca_problem_finalize(ddpca_problem_t h) {
    return guarded([&] {
        Problem& P = builder(h);
        for (size_t tv = 0; tv < P.mc.multGrid.size(); ++tv)
            if (!P.owned[tv]) throw ApiError(DDPCA_ESTATE, "subdomain " + std::to_string(tv) + " was not set");
        for (size_t ts = 0; ts < P.mc.searCont.size(); ++ts)
            if (P.mc.searCont[ts].inteMass[0].ptr.empty())
                throw ApiError(DDPCA_ESTATE, "interface " + std::to_string(ts) + " was not set");
        P.established = true;
    });
}

}  // extern "C"
