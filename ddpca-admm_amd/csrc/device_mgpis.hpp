// MGPIS on the GPU: multigrid-preconditioned CG (MGPIS.h:163-225) with a V-cycle
// (MGPIS.h:55-128) whose smoother is (block-)Jacobi or Chebyshev, built for gfx950.
//
// Layout in HBM (per level l, nodes in the reference's level order):
//   K  : SELL-64 over 3x3 blocks ("SELL-BSR3"): chunk = 64 consecutive node rows = one
//        wavefront, lane = node row; slot k of chunk c holds one block per lane:
//          col[(off[c]+k)*64 + lane]            int32 block column
//          val[((off[c]+k)*9 + ij)*64 + lane]   fp64, ij = 3*a + b of the 3x3 block
//        so every load of a slot is a contiguous 256 B (col) / 512 B (val) wave access.
//        Constrained dofs are kept in place with identity rows/cols (mask), which is the
//        reference's condensed operator consOper*K*consOper^T (MULTIGRID.h:1227) embedded
//        in the nodal space -- the 3x3 block structure survives Dirichlet condensation.
//   P  : scalar stencil (x) I3, fine-major (<= 8 parents, slot-major) for prolongation and
//        coarse-major children lists for restriction (gather, deterministic, no atomics).
//   A0^-1 : dense inverse of the coarsest level (exact coarse solve, one GEMV per cycle).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#include "../../include/ddpca_amd.h"
#include "device_common.hpp"
#include "sparse.hpp"

namespace ddpca {

// Device scalar block of one PCG solve (lives in device memory, read by every kernel).
struct PcgScal {
    double delta;     // r^T z
    double alpha, beta;
    double rr;        // ||r||^2
    double tol2;      // (rtol ||b||)^2
    double pq;        // p^T q
    double bb;        // ||b||^2
    int64_t iter;
    int64_t maxit;
    int done;         // set on convergence / cap / breakdown
    int fail;         // 1: NaN/Inf or non-positive curvature
};

struct LevelDev {
    int64_t nn = 0, nch = 0, nslots = 0, nnzb = 0;
    DevBuf<int32_t> slots, col;
    DevBuf<int64_t> off;
    DevBuf<double> val;
    DevBuf<double> minv;   // point: 3 per node; block: 9 per node
    DevBuf<double> dinv;   // point Jacobi inverse (diagonal preconditioner at the fine level)
    DevBuf<uint8_t> mask;  // bit a set = dof 3i+a free
    // transfer from level l-1
    int64_t nc = 0;
    DevBuf<int32_t> ppar;  // 8 x (nn - nc), slot-major, -1 = unused
    DevBuf<double> pw;
    DevBuf<int64_t> rptr;  // nc + 1
    DevBuf<int32_t> rch;
    DevBuf<double> rw;
    // vectors (3 nn)
    DevBuf<double> x, t, b, r, d;
    double omega = 0.0, lmax = 0.0;
};

class MgpisDevice {
public:
    MgpisDevice(int device, const std::vector<int64_t>& nnodes, const std::vector<const Bsr3*>& K,
                const std::vector<uint8_t>& dof_free, const std::vector<const Stencil*>& S,
                const mgpis_options_t& opt);
    ~MgpisDevice();

    int device = 0;
    hipStream_t stream = nullptr;
    mgpis_options_t opt{};
    std::vector<LevelDev> lev;
    int64_t n0 = 0;            // coarse dofs (3 nn_0)
    DevBuf<double> ainv;       // n0 x n0
    int64_t nfree = 0;         // condensed fine dofs
    DevBuf<int32_t> free_dof;  // condensed -> nodal dof (fine)
    std::vector<int32_t> free_dof_host;

    // PCG work vectors (fine level, 3 nn_L) + scalars
    DevBuf<double> xs, rs, zs, ps, qs, bs, partial;
    DevBuf<PcgScal> sc;
    PcgScal* sc_host = nullptr;  // pinned mirror
    int64_t nblk_fine = 0;

    // ---- operations (all asynchronous on `stream` unless stated)
    void spmv(int level, const double* x, double* y);      // full-layout device vectors
    void vcycle(const double* r, double* z, bool dot);     // z = M^-1 r (fine level, full layout)
    // PCG on full-layout device vectors; b in bs, result in xs.  begin() enqueues the setup,
    // step() enqueues one graph replay (iters_per_graph iterations), poll() reads done.
    void pcg_begin(int prec, double rtol, int64_t maxit);
    void pcg_step(int prec);    // one graph replay (iters_per_graph iterations)
    bool pcg_poll();           // synchronises the stream
    int64_t pcg_solve(int prec, double rtol, int64_t maxit, int64_t* iters, double* relres);
    void scatter_free(const double* cond, double* full);   // device pointers
    void gather_free(const double* full, double* cond);
    // timing of the fine-level SpMV (HIP events around it in the eager first iteration)
    hipEvent_t ev_k0 = nullptr, ev_k1 = nullptr;
    double timed_kernel_ms = 0.0;
    int64_t timed_kernel_samples = 0;
    bool time_kernel = false;
    double fine_kernel_bytes() const;  // algorithmic bytes of the timed kernel

private:
    hipGraphExec_t graph_[2] = {nullptr, nullptr};
    bool sample_pending_ = false;
    void build_graph(int prec);
    void enqueue_iteration(int prec, bool timed);
    void estimate_lmax(int level);
};

}  // namespace ddpca
