// C ABI of the LAGRANGE path (MCONTACT::LAGRANGE, MCONTACT.h:2847-3701): the caller hands over
// what LAGRANGE reads from MCONTACT after TRANSFER / STIF_MATR / CONSTRAINT -- per subdomain the
// MGPIS hierarchy (consStif, realProl), consForc and the node-id -> condensed map, per interface
// the integration points -- and ddpca_lagrange_solve runs the semi-smooth Newton loop: host
// assembly in lagrange.cpp, every Newton step's condensed system solved on the device by
// BiCGSTAB (MGPIS.h:350-432) with the MGPIS V-cycle of the hierarchy the reference builds for it
// (precType 1) or the diagonal preconditioner (precType 2: the reference's Eigen::BiCGSTAB,
// whose default preconditioner is the diagonal).
//
// Device layout of a step's system: ONE MgpisDevice "subdomain" holding every subdomain's nodes in
// a level-ordered global numbering (all level-0 nodes of all subdomains, then the level-1-only
// nodes, ...), so each level is a prefix of the next as the transfers require; the condensed
// non-mortar dofs are masked like Dirichlet dofs, the condensation's extra transfer couplings
// (condProl, MCONTACT.h:3456-3509) run as 3x3 block entries, the coarse inverse is an LU inverse
// (the system is nonsymmetric under Coulomb friction).
#include <algorithm>
#include <memory>
#include <numeric>
#include <string>

#include "../../include/ddpca_amd.h"
#include "common.hpp"
#include "device_mgpis.hpp"
#include "lagrange.hpp"

using namespace ddpca;

struct ddpca_lagrange {
    std::vector<LagrangeSub> subs;
    std::vector<LagrangeItf> itfs;
    std::vector<uint8_t> have_sub, have_itf;
    LagrangeResult res;
    std::vector<double> solver_relres;   // per Newton step: BiCGSTAB's ||r|| / ||b|| at exit
    std::vector<double> solver_brk;      // per Newton step: 0, 1 (rho = 0), 2 (attainable-accuracy stop)
    std::vector<double> coarse_inv;      // per Newton step: coarse inverse kind (1 LU, 2 SVD), LU residual, dropped
    bool solved = false;
};

namespace {

// the largest BiCGSTAB ||r|| / ||b|| a Newton step may continue from (else DDPCA_ENUMERIC)
constexpr double kLagrangeMaxRelres = 1e-10;

Csr csr_in(const ddpca_csr_t& m, const char* what) {
    if (m.nrow < 0 || m.ncol < 0 || (m.nrow > 0 && !m.ptr)) throw ApiError(DDPCA_EINVAL, std::string(what) + ": bad CSR");
    Csr c;
    c.nrow = m.nrow;
    c.ncol = m.ncol;
    if (m.nrow == 0) c.ptr.assign(1, 0);
    else c.ptr.assign(m.ptr, m.ptr + m.nrow + 1);
    const int64_t nnz = c.ptr.back();
    if (c.ptr[0] != 0 || nnz < 0 || (nnz > 0 && (!m.col || !m.val))) throw ApiError(DDPCA_EINVAL, std::string(what) + ": bad CSR");
    for (int64_t r = 0; r < c.nrow; ++r)
        if (c.ptr[r + 1] < c.ptr[r]) throw ApiError(DDPCA_EINVAL, std::string(what) + ": row pointer not monotone");
    c.col.assign(m.col, m.col + nnz);
    c.val.assign(m.val, m.val + nnz);
    for (int64_t r = 0; r < c.nrow; ++r)
        for (int64_t k = c.ptr[r]; k < c.ptr[r + 1]; ++k) {
            if (c.col[k] < 0 || c.col[k] >= c.ncol) throw ApiError(DDPCA_EINVAL, std::string(what) + ": column out of range");
            if (k > c.ptr[r] && c.col[k] <= c.col[k - 1]) throw ApiError(DDPCA_EINVAL, std::string(what) + ": columns not increasing");
        }
    return c;
}

// BiCGSTAB on the device for one Newton step's system (levels lo..L of the hierarchy)
// relres / brk: the solve's ||r|| / ||b|| and breakdown code (1 rho = 0, 2 attainable-accuracy stop)
int64_t device_solve(int device, int prec_type, const mgpis_options_t& o, const std::vector<LagrangeSub>& subs,
                     const LagrangeSystem& sys, std::vector<double>& x, double& relres, int& brk,
                     std::vector<double>& coarse_inv) {
    const int L = (int)sys.K.size() - 1;
    const int lo = prec_type == 1 ? 0 : L;
    const int nl = L - lo + 1;
    const int64_t nsub = (int64_t)subs.size();
    // level-ordered global node numbering: gnode(tv, n) = first[k][tv] + n - nnodes_tv[k-1], k = level of n
    std::vector<std::vector<int64_t>> first(L + 1, std::vector<int64_t>(nsub, 0));
    std::vector<int64_t> NG(L + 1, 0);
    int64_t acc = 0;
    for (int k = 0; k <= L; ++k) {
        for (int64_t tv = 0; tv < nsub; ++tv) {
            first[k][tv] = acc;
            acc += subs[tv].nnodes[k] - (k ? subs[tv].nnodes[k - 1] : 0);
        }
        NG[k] = acc;
    }
    auto gnode = [&](int64_t tv, int64_t n) {
        const auto& nn = subs[tv].nnodes;
        const int k = (int)(std::upper_bound(nn.begin(), nn.end(), n) - nn.begin());
        return first[k][tv] + n - (k ? nn[k - 1] : 0);
    };
    std::vector<std::vector<int32_t>> fd(L + 1);
    for (int l = lo; l <= L; ++l)
        for (const auto& d : sys.dofs[l]) {
            const int32_t nd = subs[d.first].free_dof[l][d.second];
            fd[l].push_back((int32_t)(3 * gnode(d.first, nd / 3) + nd % 3));
        }
    std::vector<Bsr3> B(nl);
    std::vector<Stencil> S(nl - 1);
    try {
        for (int l = lo; l <= L; ++l)
            B[l - lo] = condensed_to_bsr3(NG[l], (int64_t)fd[l].size(), fd[l].data(), sys.K[l].ptr.data(), sys.K[l].col.data(),
                                          sys.K[l].val.data());
        for (int l = lo; l < L; ++l)
            S[l - lo] = prol_to_stencil(NG[l + 1], NG[l], (int64_t)fd[l + 1].size(), fd[l + 1].data(), fd[l].data(),
                                        sys.P[l].ptr.data(), sys.P[l].col.data(), sys.P[l].val.data());
    } catch (const std::invalid_argument& e) {
        throw ApiError(DDPCA_EINVAL, std::string("LAGRANGE hierarchy: ") + e.what());
    }
    std::vector<uint8_t> fr(3 * NG[L], 0);
    for (int32_t d : fd[L]) fr[d] = 1;
    SubdomainOps ops;
    for (int l = lo; l <= L; ++l) ops.nnodes.push_back(NG[l]);
    for (auto& b : B) ops.K.push_back(&b);
    for (auto& s : S) ops.S.push_back(&s);
    ops.dof_free = fr.data();
    mgpis_options_t oo = o;
    oo.precond_fp32 = 0;  // the symmetric fp32 / fp16 copies assume K = K^T
    oo.table_mode = 0;
    oo.warm_start = 0;
    // precType 2 runs the diagonal preconditioner only: no dense coarse pseudo-inverse
    MgpisDevice D(device, std::vector<SubdomainOps>{ops}, oo, true, prec_type != 1);
    for (const auto& c : D.coarse_inverse) coarse_inv.insert(coarse_inv.end(), {(double)c.kind, c.resid, (double)c.dropped});
    if (D.coarse_inverse.empty()) coarse_inv.insert(coarse_inv.end(), {-1.0, 0.0, 0.0});  // diagonal preconditioner
    // the device's condensed order is increasing nodal dof; the hierarchy's is subdomain-major
    const int64_t n = (int64_t)fd[L].size();
    if (D.nfree[0] != n) throw ApiError(DDPCA_ESTATE, "LAGRANGE: device dof count");
    std::vector<int64_t> ord(n), rank(n);
    std::iota(ord.begin(), ord.end(), 0);
    std::sort(ord.begin(), ord.end(), [&](int64_t a, int64_t b) { return fd[L][a] < fd[L][b]; });
    for (int64_t k = 0; k < n; ++k) rank[ord[k]] = k;
    std::vector<double> b(n), xd(n);
    for (int64_t r = 0; r < n; ++r) b[rank[r]] = sys.F[r];
    DevBuf<double> tmp;
    tmp.upload(b);
    D.bs.zero(D.stream);
    D.scatter_free(0, tmp.p, D.bs.p);
    relres = 0.0;
    brk = 0;
    // the singular frictionless systems can stall just above 1e-14: the
    // attainable-accuracy stop is on for LAGRANGE's steps only
    const int64_t it = krylov_bicgstab(D, prec_type == 1 ? 1 : 0, D.bs.p, D.xs.p, 1e-14, n, &relres, &brk, true);
    D.gather_free(0, D.xs.p, tmp.p);
    DDPCA_HIP(hipMemcpyAsync(xd.data(), tmp.p, n * sizeof(double), hipMemcpyDeviceToHost, D.stream));
    DDPCA_HIP(hipStreamSynchronize(D.stream));
    x.assign(n, 0.0);
    for (int64_t r = 0; r < n; ++r) x[r] = xd[rank[r]];
    return it;
}

template <typename T>
int64_t copy_out(const std::vector<T>& v, double* out, int64_t cap) {
    if (out)
        for (int64_t i = 0; i < std::min<int64_t>(cap, (int64_t)v.size()); ++i) out[i] = (double)v[i];
    return (int64_t)v.size();
}

}  // namespace

extern "C" {

int ddpca_lagrange_create(int64_t nsub, int64_t nint, ddpca_lagrange_t* out) {
    return guarded([&] {
        if (nsub < 1 || nint < 0 || !out) throw ApiError(DDPCA_EINVAL, "nsub >= 1, nint >= 0");
        auto h = std::make_unique<ddpca_lagrange>();
        h->subs.resize(nsub);
        h->itfs.resize(nint);
        h->have_sub.assign(nsub, 0);
        h->have_itf.assign(nint, 0);
        *out = h.release();
    });
}

int ddpca_lagrange_set_subdomain(ddpca_lagrange_t h, int64_t tv, int nlev, const int64_t* nnodes, const int64_t* nfree,
                                 const int32_t* const* free_dof, const ddpca_csr_t* K, const ddpca_csr_t* P,
                                 const double* consForc, int64_t nnodes_all, const ddpca_csr_t* G, const uint8_t* hanging) {
    return guarded([&] {
        if (!h || tv < 0 || tv >= (int64_t)h->subs.size()) throw ApiError(DDPCA_EINVAL, "subdomain index");
        if (nlev < 1 || !nnodes || !nfree || !free_dof || !K || (nlev > 1 && !P) || !consForc || !G)
            throw ApiError(DDPCA_EINVAL, "null argument");
        LagrangeSub s;
        s.nlev = nlev;
        s.nnodes.assign(nnodes, nnodes + nlev);
        s.nfree.assign(nfree, nfree + nlev);
        for (int l = 0; l < nlev; ++l) {
            if (nnodes[l] < 1 || (l && nnodes[l] < nnodes[l - 1])) throw ApiError(DDPCA_EINVAL, "nnodes must grow by level");
            if (nfree[l] < 0 || nfree[l] > 3 * nnodes[l]) throw ApiError(DDPCA_EINVAL, "nfree out of range");
            s.free_dof.emplace_back(free_dof[l], free_dof[l] + nfree[l]);
            for (int64_t r = 0; r < nfree[l]; ++r)
                if (free_dof[l][r] < 0 || free_dof[l][r] >= 3 * nnodes[l] || (r && free_dof[l][r] <= free_dof[l][r - 1]))
                    throw ApiError(DDPCA_EINVAL, "free_dof must be increasing nodal dofs of the level");
            if (l && nfree[l] < nfree[l - 1]) throw ApiError(DDPCA_EINVAL, "nfree must not shrink from one level to the next");
            if (l && nfree[l - 1] > 0 && !std::equal(free_dof[l - 1], free_dof[l - 1] + nfree[l - 1], free_dof[l]))
                throw ApiError(DDPCA_EINVAL, "the free dofs of a level must be a prefix of the next level's");
            s.K.push_back(csr_in(K[l], "consStif"));
            if (s.K[l].nrow != nfree[l] || s.K[l].ncol != nfree[l]) throw ApiError(DDPCA_EINVAL, "consStif shape");
        }
        for (int l = 0; l + 1 < nlev; ++l) {
            s.P.push_back(csr_in(P[l], "realProl"));
            if (s.P[l].nrow != nfree[l + 1] || s.P[l].ncol != nfree[l]) throw ApiError(DDPCA_EINVAL, "realProl shape");
        }
        s.consForc.assign(consForc, consForc + nfree[nlev - 1]);
        if (nnodes_all < 1) throw ApiError(DDPCA_EINVAL, "nnodes_all");
        s.nall = nnodes_all;
        s.G = csr_in(*G, "node-id map");
        if (s.G.nrow != 3 * nnodes_all || s.G.ncol != nfree[nlev - 1]) throw ApiError(DDPCA_EINVAL, "node-id map shape");
        if (hanging) s.hanging.assign(hanging, hanging + nnodes_all);
        h->subs[tv] = std::move(s);
        h->have_sub[tv] = 1;
        h->solved = false;
    });
}

int ddpca_lagrange_set_interface(ddpca_lagrange_t h, int64_t ts, int64_t body0, int64_t body1, double fric, int64_t n,
                                 const int64_t* node, const double* shap, const double* basis, const double* gap,
                                 const double* w) {
    return guarded([&] {
        if (!h || ts < 0 || ts >= (int64_t)h->itfs.size()) throw ApiError(DDPCA_EINVAL, "interface index");
        if (n < 0 || (n > 0 && (!node || !shap || !basis || !gap || !w))) throw ApiError(DDPCA_EINVAL, "null argument");
        const int64_t nsub = (int64_t)h->subs.size();
        if (body0 < 0 || body0 >= nsub || body1 < 0 || body1 >= nsub) throw ApiError(DDPCA_EINVAL, "contact body out of range");
        LagrangeItf f;
        f.body[0] = body0;
        f.body[1] = body1;
        f.fric = fric;
        f.ips.resize(n);
        for (int64_t i = 0; i < n; ++i) {
            LagrangeIp& q = f.ips[i];
            for (int s = 0; s < 2; ++s)
                for (int k = 0; k < 4; ++k) {
                    q.node[s][k] = node[8 * i + 4 * s + k];
                    q.shap[s][k] = shap[8 * i + 4 * s + k];
                }
            for (int a = 0; a < 3; ++a)
                for (int c = 0; c < 3; ++c) q.basis[a][c] = basis[9 * i + 3 * a + c];
            q.gap = gap[i];
            q.w = w[i];
        }
        h->itfs[ts] = std::move(f);
        h->have_itf[ts] = 1;
        h->solved = false;
    });
}

int64_t ddpca_lagrange_solve(ddpca_lagrange_t h, int device, int prec_type, const mgpis_options_t* opt, int64_t max_newton) {
    int64_t tc = 0;
    const int rc = guarded([&] {
        if (!h) throw ApiError(DDPCA_EINVAL, "null handle");
        if (prec_type != 1 && prec_type != 2) throw ApiError(DDPCA_EINVAL, "precType must be 1 (MGPIS) or 2 (diagonal)");
        if (max_newton < 1) throw ApiError(DDPCA_EINVAL, "max_newton >= 1");
        for (uint8_t v : h->have_sub)
            if (!v) throw ApiError(DDPCA_ESTATE, "every subdomain must be set");
        for (uint8_t v : h->have_itf)
            if (!v) throw ApiError(DDPCA_ESTATE, "every interface must be set");
        for (const auto& f : h->itfs)
            for (const auto& q : f.ips)
                for (int s = 0; s < 2; ++s)
                    for (int k = 0; k < 4; ++k)
                        if (q.node[s][k] < 0 || q.node[s][k] >= h->subs[f.body[s]].nall)
                            throw ApiError(DDPCA_EINVAL, "integration point node out of range");
        select_device(device);
        mgpis_options_t o;
        mgpis_default_options(&o);
        if (opt) o = *opt;
        // run_lagrange drops hanging non-mortar points and sets the dual basis in place: work on copies
        std::vector<LagrangeSub> subs = h->subs;
        std::vector<LagrangeItf> itfs = h->itfs;
        h->solver_relres.clear();
        h->solver_brk.clear();
        h->coarse_inv.clear();
        try {
            h->res = run_lagrange(subs, itfs, max_newton, [&](const LagrangeSystem& sys, std::vector<double>& x) {
                double relres = 0.0;
                int brk = 0;
                const int64_t it = device_solve(device, prec_type, o, subs, sys, x, relres, brk, h->coarse_inv);
                h->solver_relres.push_back(relres);
                h->solver_brk.push_back((double)brk);
                // a Newton step must not continue from a solve that did not converge: the
                // reference's own stop is 1e-14, the attainable-accuracy stop 1e-12
                if (!(relres <= kLagrangeMaxRelres))
                    throw std::runtime_error("BiCGSTAB of Newton step " + std::to_string(h->solver_relres.size()) +
                                             " ended at ||r||/||b|| = " + std::to_string(relres) + " after " +
                                             std::to_string(it) + " iterations (breakdown " + std::to_string(brk) + ")");
                return it;
            });
        } catch (const ApiError&) {
            throw;  // device errors keep their own code
        } catch (const std::invalid_argument& e) {
            throw ApiError(DDPCA_EINVAL, e.what());
        } catch (const std::runtime_error& e) {
            throw ApiError(DDPCA_ENUMERIC, e.what());
        }
        h->solved = true;
        tc = h->res.newton;
        if (!h->res.converged) throw ApiError(DDPCA_ENOCONV, "semi-smooth Newton not converged within max_newton steps");
    });
    return rc != 0 ? rc : tc;
}

int64_t ddpca_lagrange_get(ddpca_lagrange_t h, const char* what, int64_t index, double* out, int64_t cap) {
    int64_t n = 0;
    const int rc = guarded([&] {
        if (!h || !what) throw ApiError(DDPCA_EINVAL, "null argument");
        if (!h->solved) throw ApiError(DDPCA_ESTATE, "ddpca_lagrange_solve has not run");
        const std::string w(what);
        const LagrangeResult& r = h->res;
        auto sub = [&]() {
            if (index < 0 || index >= (int64_t)r.u.size()) throw ApiError(DDPCA_EINVAL, "subdomain index");
        };
        auto itf = [&]() {
            if (index < 0 || index >= (int64_t)r.node.size()) throw ApiError(DDPCA_EINVAL, "interface index");
        };
        if (w == "u") sub(), n = copy_out(r.u[index], out, cap);
        else if (w == "node") itf(), n = copy_out(r.node[index], out, cap);
        else if (w == "status") itf(), n = copy_out(r.status[index], out, cap);
        else if (w == "lambda") itf(), n = copy_out(r.lambda[index], out, cap);
        else if (w == "wedi") itf(), n = copy_out(r.wedi[index], out, cap);
        else if (w == "solver_iters") n = copy_out(r.solver_iters, out, cap);
        else if (w == "changes") n = copy_out(r.changes, out, cap);
        else if (w == "solver_relres") n = copy_out(h->solver_relres, out, cap);
        else if (w == "solver_breakdown") n = copy_out(h->solver_brk, out, cap);
        else if (w == "coarse_inverse") n = copy_out(h->coarse_inv, out, cap);
        else throw ApiError(DDPCA_EINVAL, "unknown quantity: " + w);
    });
    return rc != 0 ? rc : n;
}

int ddpca_lagrange_destroy(ddpca_lagrange_t h) {
    delete h;
    return 0;
}

}  // extern "C"
