// C ABI: MGPIS device solver entry points (mgpis_gpu_*), see include/ddpca_amd.h.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <memory>

#include "../../include/ddpca_amd.h"
#include "device_mgpis.hpp"
#include "problem.hpp"

using namespace ddpca;

struct ddpca_mgpis {
    std::unique_ptr<MgpisDevice> dev;
};

namespace {

mgpis_options_t resolve(const mgpis_options_t* opt) {
    mgpis_options_t o;
    mgpis_default_options(&o);
    if (opt) o = *opt;
    return o;
}

std::unique_ptr<MgpisDevice> single(int device, const std::vector<int64_t>& nn, const std::vector<const Bsr3*>& B,
                                    const std::vector<uint8_t>& fr, const std::vector<const Stencil*>& S,
                                    const mgpis_options_t* opt, const double* coords = nullptr) {
    SubdomainOps ops;
    ops.nnodes = nn;
    ops.K = B;
    ops.dof_free = fr.data();
    ops.S = S;
    ops.coords = coords;
    auto d = std::make_unique<MgpisDevice>(device, std::vector<SubdomainOps>{ops}, resolve(opt));
    // The reference calls CG_SOLV on different MGPIS objects from an omp parallel for
    // (MCONTACT.h:2511-2531): every graph a solve replays is captured here, on the creating
    // thread, so a solve only replays (no capture on a solving thread), and the
    // solve's condensed staging buffer is allocated here too (no hipMalloc / hipFree per solve).
    d->prepare_graphs(0);
    if (!d->no_coarse) d->prepare_graphs(1);
    d->stage.alloc((size_t)std::max<int64_t>(d->nfree[0], 1));
    return d;
}

}  // namespace

extern "C" {

void mgpis_default_options(mgpis_options_t* opt) {
    opt->smoother = 1;
    opt->nu = 1;
    opt->omega = -1.7;  // 1.7 / lambda_max: damping sweep, profiles/r01_sweep_omega.txt
    opt->coarse_level = -1;
    opt->iters_per_graph = 4;
    opt->warm_start = 0;
    opt->precond_fp32 = 0;
    opt->table_mode = 1;
}

int ddpca_gpu_available(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return 0;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, 0) != hipSuccess) return 0;
    return std::strncmp(prop.gcnArchName, "gfx950", 6) == 0 ? 1 : 0;
}

int mgpis_gpu_create(int device, int nlev, const int64_t* nnodes, const int64_t* nfree,
                     const int32_t* const* free_dof, const int64_t* const* K_ptr, const int32_t* const* K_col,
                     const double* const* K_val, const int64_t* const* S_ptr, const int32_t* const* S_col,
                     const double* const* S_w, const mgpis_options_t* opt, mgpis_t* out) {
    return guarded([&] {
        if (nlev < 1 || !nnodes || !nfree || !free_dof || !K_ptr || !K_col || !K_val || !out)
            throw ApiError(DDPCA_EINVAL, "null argument");
        std::vector<Bsr3> B(nlev);
        std::vector<Stencil> S(nlev - 1);
        for (int l = 0; l < nlev; ++l) B[l] = condensed_to_bsr3(nnodes[l], nfree[l], free_dof[l], K_ptr[l], K_col[l], K_val[l]);
        for (int l = 0; l + 1 < nlev; ++l) S[l] = make_stencil(nnodes[l + 1], nnodes[l], S_ptr[l], S_col[l], S_w[l]);
        const int64_t nn = nnodes[nlev - 1];
        std::vector<uint8_t> fr(3 * nn, 0);
        for (int64_t r = 0; r < nfree[nlev - 1]; ++r) fr[free_dof[nlev - 1][r]] = 1;
        std::vector<int64_t> nn_v(nnodes, nnodes + nlev);
        std::vector<const Bsr3*> Bp;
        std::vector<const Stencil*> Sp;
        for (auto& b : B) Bp.push_back(&b);
        for (auto& s : S) Sp.push_back(&s);
        auto h = std::make_unique<ddpca_mgpis>();
        h->dev = single(device, nn_v, Bp, fr, Sp, opt);
        *out = h.release();
    });
}

int mgpis_gpu_create_prol(int device, int nlev, const int64_t* nnodes, const int64_t* nfree,
                          const int32_t* const* free_dof, const int64_t* const* K_ptr, const int32_t* const* K_col,
                          const double* const* K_val, const int64_t* const* P_ptr, const int32_t* const* P_col,
                          const double* const* P_val, const mgpis_options_t* opt, mgpis_t* out) {
    return guarded([&] {
        if (nlev < 1 || !nnodes || !nfree || !free_dof || !K_ptr || !K_col || !K_val || !out)
            throw ApiError(DDPCA_EINVAL, "null argument");
        if (nlev > 1 && (!P_ptr || !P_col || !P_val)) throw ApiError(DDPCA_EINVAL, "null realProl");
        std::vector<Bsr3> B(nlev);
        std::vector<Stencil> S(nlev - 1);
        for (int l = 0; l < nlev; ++l) B[l] = condensed_to_bsr3(nnodes[l], nfree[l], free_dof[l], K_ptr[l], K_col[l], K_val[l]);
        for (int l = 0; l + 1 < nlev; ++l) {
            try {
                S[l] = prol_to_stencil(nnodes[l + 1], nnodes[l], nfree[l + 1], free_dof[l + 1], free_dof[l], P_ptr[l],
                                       P_col[l], P_val[l]);
            } catch (const std::invalid_argument& e) {
                throw ApiError(DDPCA_EINVAL, e.what());
            }
        }
        const int64_t nn = nnodes[nlev - 1];
        std::vector<uint8_t> fr(3 * nn, 0);
        for (int64_t r = 0; r < nfree[nlev - 1]; ++r) fr[free_dof[nlev - 1][r]] = 1;
        std::vector<int64_t> nn_v(nnodes, nnodes + nlev);
        std::vector<const Bsr3*> Bp;
        std::vector<const Stencil*> Sp;
        for (auto& b : B) Bp.push_back(&b);
        for (auto& s : S) Sp.push_back(&s);
        auto h = std::make_unique<ddpca_mgpis>();
        h->dev = single(device, nn_v, Bp, fr, Sp, opt);
        *out = h.release();
    });
}

int mgpis_gpu_create_bsr3(int device, int nlev, const int64_t* nnodes, const int64_t* const* B_ptr,
                          const int32_t* const* B_col, const double* const* B_val, const uint8_t* dof_free,
                          const int64_t* const* S_ptr, const int32_t* const* S_col, const double* const* S_w,
                          const mgpis_options_t* opt, mgpis_t* out) {
    return guarded([&] {
        if (nlev < 1 || !nnodes || !B_ptr || !B_col || !B_val || !dof_free || !out) throw ApiError(DDPCA_EINVAL, "null argument");
        std::vector<Bsr3> B(nlev);
        std::vector<Stencil> S(nlev - 1);
        for (int l = 0; l < nlev; ++l) {
            B[l].nb = B[l].mb = nnodes[l];
            B[l].ptr.assign(B_ptr[l], B_ptr[l] + nnodes[l] + 1);
            B[l].col.assign(B_col[l], B_col[l] + B_ptr[l][nnodes[l]]);
            B[l].val.assign(B_val[l], B_val[l] + 9 * B_ptr[l][nnodes[l]]);
        }
        for (int l = 0; l + 1 < nlev; ++l) S[l] = make_stencil(nnodes[l + 1], nnodes[l], S_ptr[l], S_col[l], S_w[l]);
        std::vector<uint8_t> fr(dof_free, dof_free + 3 * nnodes[nlev - 1]);
        std::vector<int64_t> nn_v(nnodes, nnodes + nlev);
        std::vector<const Bsr3*> Bp;
        std::vector<const Stencil*> Sp;
        for (auto& b : B) Bp.push_back(&b);
        for (auto& s : S) Sp.push_back(&s);
        auto h = std::make_unique<ddpca_mgpis>();
        h->dev = single(device, nn_v, Bp, fr, Sp, opt);
        *out = h.release();
    });
}

int ddpca_problem_mgpis(ddpca_problem_t p, int64_t tv, int device, const mgpis_options_t* opt, mgpis_t* out) {
    return guarded([&] {
        Problem& P = *reinterpret_cast<Problem*>(p);
        if (!P.established) throw ApiError(DDPCA_ESTATE, "problem not established");
        if (tv < 0 || tv >= (int64_t)P.mc.multGrid.size()) throw ApiError(DDPCA_EINVAL, "subdomain index");
        const MULTIGRID& g = P.mc.multGrid[tv];
        std::vector<int64_t> nn(g.leveCount.begin(), g.leveCount.end());
        std::vector<const Bsr3*> Bp;
        std::vector<const Stencil*> Sp;
        for (const auto& b : g.levelStif) Bp.push_back(&b);
        for (const auto& s : g.scalProl) Sp.push_back(&s);
        auto h = std::make_unique<ddpca_mgpis>();
        h->dev = single(device, nn, Bp, g.consFlag, Sp, opt, g.nodeCoor.empty() ? nullptr : g.nodeCoor[0].data());
        *out = h.release();
    });
}

int mgpis_gpu_solve(mgpis_t h, const double* b, double* x, int prec, double rtol, int64_t maxit, int64_t* iters,
                    double* relres) {
    int64_t it = 0;
    int rc = guarded([&] {
        if (!h || !b || !x) throw ApiError(DDPCA_EINVAL, "null argument");
        if (prec != 0 && prec != 1) throw ApiError(DDPCA_EINVAL, "prec must be 0 or 1");
        MgpisDevice& D = *h->dev;
        select_device(D.device);
        if (prec == 1 && D.no_coarse) throw ApiError(DDPCA_ESTATE, "one-level handle without a coarse inverse: diagonal preconditioner only");
        // stream-ordered only: the handle's own staging buffer and stream, graphs captured at create
        DDPCA_HIP(hipMemcpyAsync(D.stage.p, b, D.nfree[0] * sizeof(double), hipMemcpyHostToDevice, D.stream));
        D.scatter_free(0, D.stage.p, D.bs.p);
        D.pcg_solve(prec, rtol, {maxit});
        it = D.sc_host[0].iter;
        D.gather_free(0, D.xs.p, D.stage.p);
        DDPCA_HIP(hipMemcpyAsync(x, D.stage.p, D.nfree[0] * sizeof(double), hipMemcpyDeviceToHost, D.stream));
        DDPCA_HIP(hipStreamSynchronize(D.stream));
        if (iters) *iters = it;
        if (relres) *relres = D.sc_host[0].bb > 0 ? std::sqrt(D.sc_host[0].rr / D.sc_host[0].bb) : 0.0;
    });
    if (rc != 0) return rc;
    return (maxit > 0 && it >= maxit) ? (int)std::min<int64_t>(it, 1 << 30) : 0;
}

}  // extern "C"
namespace {
// Shared shell of the non-CG drivers: condensed host b -> device nodal layout, run, gather x.
template <typename F>
int run_driver(mgpis_t h, const double* b, double* x, int64_t maxit, int64_t* iters, F body) {
    int64_t it = 0;
    int rc = guarded([&] {
        if (!h || !b || !x) throw ApiError(DDPCA_EINVAL, "null argument");
        if (maxit < 0) throw ApiError(DDPCA_EINVAL, "maxit must be >= 0");
        MgpisDevice& D = *h->dev;
        if (D.nsub != 1) throw ApiError(DDPCA_EINVAL, "driver needs a one-subdomain handle");
        select_device(D.device);
        DevBuf<double> tmp;
        tmp.upload(b, D.nfree[0]);
        D.bs.zero(D.stream);
        D.scatter_free(0, tmp.p, D.bs.p);
        it = body(D, D.bs.p, D.xs.p);
        D.gather_free(0, D.xs.p, tmp.p);
        DDPCA_HIP(hipMemcpyAsync(x, tmp.p, D.nfree[0] * sizeof(double), hipMemcpyDeviceToHost, D.stream));
        DDPCA_HIP(hipStreamSynchronize(D.stream));
        if (iters) *iters = it;
    });
    if (rc != 0) return rc;
    return (maxit > 0 && it >= maxit) ? (int)std::min<int64_t>(it, 1 << 30) : 0;
}
}  // namespace
extern "C" {

int mgpis_gpu_mult_solve(mgpis_t h, const double* b, double* x, int64_t maxit, int64_t* iters, double* relres) {
    return run_driver(h, b, x, maxit, iters, [&](MgpisDevice& D, const double* bd, double* xd) {
        return krylov_mult_solv(D, bd, xd, maxit, relres);
    });
}

int mgpis_gpu_bicgstab(mgpis_t h, const double* b, double* x, int prec, double rtol, int64_t maxit, int64_t* iters,
                       double* relres, int* breakdown) {
    if (prec != 0 && prec != 1) return guarded([] { throw ApiError(DDPCA_EINVAL, "prec must be 0 or 1"); });
    return run_driver(h, b, x, maxit, iters, [&](MgpisDevice& D, const double* bd, double* xd) {
        return krylov_bicgstab(D, prec, bd, xd, rtol, maxit, relres, breakdown);
    });
}

int mgpis_gpu_gmres(mgpis_t h, const double* b, double* x, int prec, double rtol, int64_t maxit, int64_t restart,
                    int64_t* iters, double* relres) {
    if (prec != 0 && prec != 1) return guarded([] { throw ApiError(DDPCA_EINVAL, "prec must be 0 or 1"); });
    return run_driver(h, b, x, maxit, iters, [&](MgpisDevice& D, const double* bd, double* xd) {
        return krylov_gmres(D, prec, bd, xd, rtol, maxit, restart, relres);
    });
}

int mgpis_gpu_spmv(mgpis_t h, int level, const double* x, double* y) { return mgpis_gpu_spmv_copy(h, level, 0, x, y); }

int mgpis_gpu_spmv_copy(mgpis_t h, int level, int vcycle_copy, const double* x, double* y) {
    return guarded([&] {
        if (!h || !x || !y) throw ApiError(DDPCA_EINVAL, "null argument");
        MgpisDevice& D = *h->dev;
        select_device(D.device);
        if (level < 0 || level >= (int)D.lev.size()) throw ApiError(DDPCA_EINVAL, "level");
        if (level != (int)D.lev.size() - 1) throw ApiError(DDPCA_EINVAL, "condensed spmv is defined on the fine level");
        if (vcycle_copy && D.vc_type(level) == kVal64) throw ApiError(DDPCA_EINVAL, "no reduced-precision V-cycle copy (precond_fp32 = 0)");
        DevBuf<double> tmp, full_x, full_y;
        tmp.upload(x, D.nfree[0]);
        full_x.alloc(3 * D.lev.back().nn);
        full_y.alloc(3 * D.lev.back().nn);
        D.scatter_free(0, tmp.p, full_x.p);
        D.spmv(level, full_x.p, full_y.p, vcycle_copy != 0);
        D.gather_free(0, full_y.p, tmp.p);
        DDPCA_HIP(hipMemcpyAsync(y, tmp.p, D.nfree[0] * sizeof(double), hipMemcpyDeviceToHost, D.stream));
        DDPCA_HIP(hipStreamSynchronize(D.stream));
    });
}

int mgpis_gpu_vcycle(mgpis_t h, const double* r, double* z) {
    return guarded([&] {
        if (!h || !r || !z) throw ApiError(DDPCA_EINVAL, "null argument");
        MgpisDevice& D = *h->dev;
        select_device(D.device);
        DDPCA_HIP(hipMemcpyAsync(D.stage.p, r, D.nfree[0] * sizeof(double), hipMemcpyHostToDevice, D.stream));
        D.scatter_free(0, D.stage.p, D.rs.p);
        DDPCA_HIP(hipMemsetAsync(D.sc.p, 0, sizeof(PcgScal), D.stream));  // done = 0
        D.vcycle(D.rs.p, D.zs.p, false);
        D.gather_free(0, D.zs.p, D.stage.p);
        DDPCA_HIP(hipMemcpyAsync(z, D.stage.p, D.nfree[0] * sizeof(double), hipMemcpyDeviceToHost, D.stream));
        DDPCA_HIP(hipStreamSynchronize(D.stream));
    });
}

int mgpis_gpu_info(mgpis_t h, int64_t* out7) {
    return guarded([&] {
        MgpisDevice& D = *h->dev;
        out7[0] = (int64_t)D.lev.size();
        const double lmax = D.lev.size() > 1 ? D.lev.back().lmax[0] : 0.0;
        out7[1] = D.nfree[0];
        out7[2] = D.lev.back().nnzb;
        out7[3] = D.lev.back().nch;
        const double scale = D.opt.omega < 0.0 ? -D.opt.omega : 4.0 / 3.0;
        out7[4] = (int64_t)((D.opt.omega > 0.0 ? D.opt.omega : lmax > 0.0 ? scale / lmax : 1.0) * 1e6);
        out7[5] = (int64_t)(lmax * 1e6);
        out7[6] = D.device;
    });
}

int mgpis_gpu_bench_spmv(mgpis_t h, int variant, int reps, double* ms, double* bytes) {
    return guarded([&] {
        if (!h || !ms) throw ApiError(DDPCA_EINVAL, "null argument");
        MgpisDevice& D = *h->dev;
        select_device(D.device);
        *ms = D.bench_spmv(variant, reps);
        // 76 B per block + x gathered once (24 B/node) + per-node vector traffic of the mode:
        // y = Kx writes y; PCG reads/writes p, q; residual reads b, writes r; Chebyshev reads b,
        // x, d, the 9-entry block inverse and writes d, x_new
        const double per_node[4] = {24.0, 96.0, 48.0, 24.0 * 5.0 + 72.0};
        const int mode = (variant >> 2) & 3;
        const bool f32 = (variant & 16) != 0;
        if (bytes) *bytes = D.fine_matrix_bytes(0, !f32 ? kVal64 : D.vc_type((int)D.lev.size() - 1), false) + (24.0 + per_node[mode]) * (double)D.lev.back().nloc[0];
    });
}

int mgpis_gpu_destroy(mgpis_t h) {
    return guarded([&] { delete h; });
}

}  // extern "C"
