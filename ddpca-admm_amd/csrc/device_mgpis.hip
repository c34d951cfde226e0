// MGPIS device path: SELL-BSR3 kernels, V-cycle and PCG for gfx950 (see device_mgpis.hpp).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <numeric>
#include <omp.h>
#include <random>

#include "device_mgpis.hpp"

namespace ddpca {

// ============================================================================== kernels
namespace {

enum SellMode { kSpmv = 0, kResid = 1, kJac = 2, kPcg = 3, kCheb = 4 };
enum FinWhat { kFinInit = 0, kFinBeta0 = 1, kFinAlpha = 2, kFinRR = 3, kFinBeta = 4 };

struct SellArgs {
    const int32_t* slots;
    const int64_t* off;
    const int32_t* col;
    const double* val;
    int64_t nn, nch;
    const double* x;   // gathered operand
    double* y;         // SPMV / RESID output, PCG: q (in place)
    const double* b;   // RESID / JAC / CHEB right-hand side
    const double* minv;
    double omega;
    double* xo;        // JAC / CHEB new iterate
    double* p;         // PCG: p (in place), CHEB: direction d (in place)
    double c1, c2;     // CHEB coefficients
    const PcgScal* sc;
    double* partial;
    const int* done;
};

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// Deterministic per-workgroup partial sum (4 waves of 64 lanes).
__device__ __forceinline__ void block_partial(double v, double* partial) {
    __shared__ double red[kBlock / kWave];
    v = wave_sum(v);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    if (threadIdx.x == 0) partial[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

template <bool BJ>
__device__ __forceinline__ void apply_m(const double* minv, int64_t row, double r0, double r1, double r2,
                                        double& m0, double& m1, double& m2) {
    if (BJ) {
        const double* m = minv + 9 * row;
        m0 = m[0] * r0 + m[1] * r1 + m[2] * r2;
        m1 = m[3] * r0 + m[4] * r1 + m[5] * r2;
        m2 = m[6] * r0 + m[7] * r1 + m[8] * r2;
    } else {
        const double* m = minv + 3 * row;
        m0 = m[0] * r0;
        m1 = m[1] * r1;
        m2 = m[2] * r2;
    }
}

// One wavefront per 64-node chunk, one lane per node row, three accumulators per lane.
template <int MODE, bool BJ, bool DOT>
__global__ __launch_bounds__(kBlock) void k_sell(SellArgs a) {
    if (*a.done) return;
    const int lane = threadIdx.x & 63;
    const int64_t c = (int64_t)blockIdx.x * (kBlock / kWave) + (threadIdx.x >> 6);
    double dotv = 0.0;
    if (c < a.nch) {
        const int64_t row = c * kChunk + lane;
        const int ns = a.slots[c];
        const int64_t base = a.off[c];
        const int32_t* colp = a.col + base * kChunk + lane;
        const double* valp = a.val + base * 9 * kChunk + lane;
        double s0 = 0.0, s1 = 0.0, s2 = 0.0;
#pragma unroll 3
        for (int k = 0; k < ns; ++k) {
            const int64_t j = colp[(int64_t)k * kChunk];
            const double* xj = a.x + 3 * j;
            const double x0 = xj[0], x1 = xj[1], x2 = xj[2];
            const double* v = valp + (int64_t)k * 9 * kChunk;
            s0 += v[0 * kChunk] * x0 + v[1 * kChunk] * x1 + v[2 * kChunk] * x2;
            s1 += v[3 * kChunk] * x0 + v[4 * kChunk] * x1 + v[5 * kChunk] * x2;
            s2 += v[6 * kChunk] * x0 + v[7 * kChunk] * x1 + v[8 * kChunk] * x2;
        }
        if (row < a.nn) {
            const int64_t o = 3 * row;
            if (MODE == kSpmv) {
                a.y[o] = s0;
                a.y[o + 1] = s1;
                a.y[o + 2] = s2;
            } else if (MODE == kResid) {
                a.y[o] = a.b[o] - s0;
                a.y[o + 1] = a.b[o + 1] - s1;
                a.y[o + 2] = a.b[o + 2] - s2;
            } else if (MODE == kJac) {
                const double b0 = a.b[o], b1 = a.b[o + 1], b2 = a.b[o + 2];
                double m0, m1, m2;
                apply_m<BJ>(a.minv, row, b0 - s0, b1 - s1, b2 - s2, m0, m1, m2);
                const double n0 = a.x[o] + a.omega * m0, n1 = a.x[o + 1] + a.omega * m1, n2 = a.x[o + 2] + a.omega * m2;
                a.xo[o] = n0;
                a.xo[o + 1] = n1;
                a.xo[o + 2] = n2;
                if (DOT) dotv = b0 * n0 + b1 * n1 + b2 * n2;
            } else if (MODE == kPcg) {
                // q = K z + beta q_old, p = z + beta p_old  (K p = K z + beta K p_old)
                const double be = a.sc->beta;
                const double q0 = s0 + be * a.y[o], q1 = s1 + be * a.y[o + 1], q2 = s2 + be * a.y[o + 2];
                const double p0 = a.x[o] + be * a.p[o], p1 = a.x[o + 1] + be * a.p[o + 1], p2 = a.x[o + 2] + be * a.p[o + 2];
                a.y[o] = q0;
                a.y[o + 1] = q1;
                a.y[o + 2] = q2;
                a.p[o] = p0;
                a.p[o + 1] = p1;
                a.p[o + 2] = p2;
                if (DOT) dotv = p0 * q0 + p1 * q1 + p2 * q2;
            } else if (MODE == kCheb) {
                const double b0 = a.b[o], b1 = a.b[o + 1], b2 = a.b[o + 2];
                double m0, m1, m2;
                apply_m<BJ>(a.minv, row, b0 - s0, b1 - s1, b2 - s2, m0, m1, m2);
                const double d0 = a.c1 * a.p[o] + a.c2 * m0, d1 = a.c1 * a.p[o + 1] + a.c2 * m1,
                             d2 = a.c1 * a.p[o + 2] + a.c2 * m2;
                a.p[o] = d0;
                a.p[o + 1] = d1;
                a.p[o + 2] = d2;
                const double n0 = a.x[o] + d0, n1 = a.x[o + 1] + d1, n2 = a.x[o + 2] + d2;
                a.xo[o] = n0;
                a.xo[o + 1] = n1;
                a.xo[o + 2] = n2;
                if (DOT) dotv = b0 * n0 + b1 * n1 + b2 * n2;
            }
        }
    }
    if (DOT) block_partial(dotv, a.partial);
}

// x = omega M b  (first smoothing sweep from a zero guess); CHEB: also d = x
template <bool BJ, bool SETD>
__global__ __launch_bounds__(kBlock) void k_jac0(const double* b, const double* minv, double omega, double* x,
                                                 double* d, int64_t nn, const int* done) {
    if (*done) return;
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= nn) return;
    double m0, m1, m2;
    apply_m<BJ>(minv, i, b[3 * i], b[3 * i + 1], b[3 * i + 2], m0, m1, m2);
    x[3 * i] = omega * m0;
    x[3 * i + 1] = omega * m1;
    x[3 * i + 2] = omega * m2;
    if (SETD) {
        d[3 * i] = omega * m0;
        d[3 * i + 1] = omega * m1;
        d[3 * i + 2] = omega * m2;
    }
}

// b_c = mask_c (r_f[j] + sum_children w r_f[child]); optionally x_c = omega M b_c (CHEB: d_c too)
template <bool INIT, bool BJ, bool SETD>
__global__ __launch_bounds__(kBlock) void k_restrict(const double* rf, const int64_t* rptr, const int32_t* rch,
                                                     const double* rw, const uint8_t* cmask, double* bc, double* xc,
                                                     double* dc, const double* minv, double omega, int64_t nc,
                                                     const int* done) {
    if (*done) return;
    const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (j >= nc) return;
    double s0 = rf[3 * j], s1 = rf[3 * j + 1], s2 = rf[3 * j + 2];
    for (int64_t k = rptr[j]; k < rptr[j + 1]; ++k) {
        const int64_t i = rch[k];
        const double w = rw[k];
        s0 += w * rf[3 * i];
        s1 += w * rf[3 * i + 1];
        s2 += w * rf[3 * i + 2];
    }
    const uint8_t m = cmask[j];
    s0 = (m & 1) ? s0 : 0.0;
    s1 = (m & 2) ? s1 : 0.0;
    s2 = (m & 4) ? s2 : 0.0;
    bc[3 * j] = s0;
    bc[3 * j + 1] = s1;
    bc[3 * j + 2] = s2;
    if (INIT) {
        double m0, m1, m2;
        apply_m<BJ>(minv, j, s0, s1, s2, m0, m1, m2);
        xc[3 * j] = omega * m0;
        xc[3 * j + 1] = omega * m1;
        xc[3 * j + 2] = omega * m2;
        if (SETD) {
            dc[3 * j] = omega * m0;
            dc[3 * j + 1] = omega * m1;
            dc[3 * j + 2] = omega * m2;
        }
    }
}

// x_f += mask_f (P e_c)
__global__ __launch_bounds__(kBlock) void k_prolong(const double* ec, const int32_t* ppar, const double* pw,
                                                    const uint8_t* fmask, double* xf, int64_t nf, int64_t nc,
                                                    const int* done) {
    if (*done) return;
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= nf) return;
    double e0, e1, e2;
    if (i < nc) {
        e0 = ec[3 * i];
        e1 = ec[3 * i + 1];
        e2 = ec[3 * i + 2];
    } else {
        e0 = e1 = e2 = 0.0;
        const int64_t k = i - nc, stride = nf - nc;
#pragma unroll
        for (int p = 0; p < 8; ++p) {
            const int32_t c = ppar[p * stride + k];
            if (c < 0) break;
            const double w = pw[p * stride + k];
            e0 += w * ec[3 * (int64_t)c];
            e1 += w * ec[3 * (int64_t)c + 1];
            e2 += w * ec[3 * (int64_t)c + 2];
        }
    }
    const uint8_t m = fmask[i];
    if (m & 1) xf[3 * i] += e0;
    if (m & 2) xf[3 * i + 1] += e1;
    if (m & 4) xf[3 * i + 2] += e2;
}

// x0 = A0^-1 b0, one wavefront per row
__global__ __launch_bounds__(kBlock) void k_coarse(const double* ainv, const double* b, double* x, int64_t n,
                                                   const int* done) {
    if (*done) return;
    const int64_t row = (int64_t)blockIdx.x * (kBlock / kWave) + (threadIdx.x >> 6);
    if (row >= n) return;
    const int lane = threadIdx.x & 63;
    double s = 0.0;
    for (int64_t k = lane; k < n; k += kWave) s += ainv[row * n + k] * b[k];
    s = wave_sum(s);
    if (lane == 0) x[row] = s;
}

// r = b, x = p = q = 0, partial ||b||^2  (per node, 256 nodes per workgroup)
__global__ __launch_bounds__(kBlock) void k_pcg_init(const double* b, double* x, double* r, double* p, double* q,
                                                     double* partial, int64_t nn) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    double s = 0.0;
    if (i < nn)
        for (int a = 0; a < 3; ++a) {
            const double v = b[3 * i + a];
            r[3 * i + a] = v;
            x[3 * i + a] = 0.0;
            p[3 * i + a] = 0.0;
            q[3 * i + a] = 0.0;
            s += v * v;
        }
    block_partial(s, partial);
}

// x += alpha p, r -= alpha q, partial ||r||^2
__global__ __launch_bounds__(kBlock) void k_axpy(double* x, double* r, const double* p, const double* q,
                                                 const PcgScal* sc, double* partial, int64_t nn, const int* done) {
    if (*done) return;
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const double al = sc->alpha;
    double s = 0.0;
    if (i < nn)
        for (int a = 0; a < 3; ++a) {
            x[3 * i + a] += al * p[3 * i + a];
            const double v = r[3 * i + a] - al * q[3 * i + a];
            r[3 * i + a] = v;
            s += v * v;
        }
    block_partial(s, partial);
}

// z = D^-1 r (diagonal preconditioner, DIAG_PREC), partial r^T z
__global__ __launch_bounds__(kBlock) void k_diag(const double* r, const double* dinv, double* z, double* partial,
                                                 int64_t nn, const int* done) {
    if (*done) return;
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    double s = 0.0;
    if (i < nn)
        for (int a = 0; a < 3; ++a) {
            const double v = dinv[3 * i + a] * r[3 * i + a];
            z[3 * i + a] = v;
            s += r[3 * i + a] * v;
        }
    block_partial(s, partial);
}

// partial x^T y per node block (used after a coarse-only "V-cycle")
__global__ __launch_bounds__(kBlock) void k_dot(const double* x, const double* y, double* partial, int64_t nn,
                                                const int* done) {
    if (*done) return;
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    double s = 0.0;
    if (i < nn)
        for (int a = 0; a < 3; ++a) s += x[3 * i + a] * y[3 * i + a];
    block_partial(s, partial);
}

// Scalar updates of the PCG recurrence (one workgroup, fixed summation order).
__global__ __launch_bounds__(kBlock) void k_fin(int what, const double* partial, int64_t nblk, PcgScal* sc) {
    if (what != kFinInit && sc->done) return;
    double s = 0.0;
    for (int64_t k = threadIdx.x; k < nblk; k += kBlock) s += partial[k];
    __shared__ double red[kBlock / kWave];
    s = wave_sum(s);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x != 0) return;
    s = (red[0] + red[1]) + (red[2] + red[3]);
    if (what == kFinInit) {
        sc->rr = s;
        sc->bb = s;
        sc->tol2 = sc->tol2 * s;  // tol2 holds rtol^2 on entry
        sc->iter = 0;
        sc->fail = 0;
        sc->beta = 0.0;
        sc->done = (s <= sc->tol2 || sc->maxit <= 0) ? 1 : 0;
    } else if (what == kFinBeta0) {
        sc->delta = s;
        sc->beta = 0.0;
    } else if (what == kFinAlpha) {
        sc->pq = s;
        if (!(s > 0.0) || !isfinite(s)) {
            sc->fail = 1;
            sc->done = 1;
        }
        sc->alpha = sc->delta / s;
    } else if (what == kFinRR) {
        sc->rr = s;
        sc->iter += 1;
        if (!isfinite(s)) {
            sc->fail = 1;
            sc->done = 1;
        }
        if (s <= sc->tol2 || sc->iter >= sc->maxit) sc->done = 1;
    } else {
        if (!isfinite(s)) {
            sc->fail = 1;
            sc->done = 1;
        }
        sc->beta = s / sc->delta;
        sc->delta = s;
    }
}

// full[free_dof[i]] = cond[i] (full zero-filled first) / cond[i] = full[free_dof[i]]
__global__ void k_scatter(const double* cond, const int32_t* free_dof, double* full, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < n) full[free_dof[i]] = cond[i];
}
__global__ void k_gather(const double* full, const int32_t* free_dof, double* cond, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < n) cond[i] = full[free_dof[i]];
}

// y = M x, partial ||y||^2 (power iteration for lambda_max(M K) at setup)
template <bool BJ>
__global__ void k_apply_m(const double* x, const double* minv, double* y, double* partial, int64_t nn) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    double s = 0.0;
    if (i < nn) {
        double m0, m1, m2;
        apply_m<BJ>(minv, i, x[3 * i], x[3 * i + 1], x[3 * i + 2], m0, m1, m2);
        y[3 * i] = m0;
        y[3 * i + 1] = m1;
        y[3 * i + 2] = m2;
        s = m0 * m0 + m1 * m1 + m2 * m2;
    }
    block_partial(s, partial);
}

const int* zero_flag() {
    static int* z = nullptr;
    if (!z) {
        DDPCA_HIP(hipMalloc(&z, sizeof(int)));
        DDPCA_HIP(hipMemset(z, 0, sizeof(int)));
    }
    return z;
}

// ---- host helpers
void invert_spd_dense(std::vector<double>& A, int64_t n) {
    // Cholesky A = L L^T (lower, in place), then A^-1 = L^-T L^-1.
    for (int64_t j = 0; j < n; ++j) {
        double d = A[j * n + j];
        for (int64_t k = 0; k < j; ++k) d -= A[j * n + k] * A[j * n + k];
        if (!(d > 0.0)) throw ApiError(DDPCA_ENUMERIC, "coarse operator is not positive definite");
        const double ljj = std::sqrt(d);
        A[j * n + j] = ljj;
#pragma omp parallel for schedule(static) if (n - j > 256)
        for (int64_t i = j + 1; i < n; ++i) {
            double s = A[i * n + j];
            const double* ai = &A[i * n];
            const double* aj = &A[j * n];
            for (int64_t k = 0; k < j; ++k) s -= ai[k] * aj[k];
            A[i * n + j] = s / ljj;
        }
    }
    // Linv (lower) by columns
    std::vector<double> Li(n * n, 0.0);
#pragma omp parallel for schedule(dynamic, 16)
    for (int64_t c = 0; c < n; ++c) {
        Li[c * n + c] = 1.0 / A[c * n + c];
        for (int64_t i = c + 1; i < n; ++i) {
            double s = 0.0;
            for (int64_t k = c; k < i; ++k) s -= A[i * n + k] * Li[k * n + c];
            Li[i * n + c] = s / A[i * n + i];
        }
    }
    // A^-1 = Li^T Li
#pragma omp parallel for schedule(dynamic, 16)
    for (int64_t i = 0; i < n; ++i)
        for (int64_t j = 0; j <= i; ++j) {
            double s = 0.0;
            for (int64_t k = i; k < n; ++k) s += Li[k * n + i] * Li[k * n + j];
            A[i * n + j] = s;
            A[j * n + i] = s;
        }
}

bool invert3(const double m[9], double r[9]) {
    const double det = m[0] * (m[4] * m[8] - m[5] * m[7]) - m[1] * (m[3] * m[8] - m[5] * m[6]) +
                       m[2] * (m[3] * m[7] - m[4] * m[6]);
    if (!(std::abs(det) > 0.0)) return false;
    r[0] = (m[4] * m[8] - m[5] * m[7]) / det;
    r[1] = (m[2] * m[7] - m[1] * m[8]) / det;
    r[2] = (m[1] * m[5] - m[2] * m[4]) / det;
    r[3] = (m[5] * m[6] - m[3] * m[8]) / det;
    r[4] = (m[0] * m[8] - m[2] * m[6]) / det;
    r[5] = (m[2] * m[3] - m[0] * m[5]) / det;
    r[6] = (m[3] * m[7] - m[4] * m[6]) / det;
    r[7] = (m[1] * m[6] - m[0] * m[7]) / det;
    r[8] = (m[0] * m[4] - m[1] * m[3]) / det;
    return true;
}

}  // namespace

// ============================================================================== setup
void select_device(int device) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) throw ApiError(DDPCA_ENOGPU, "no HIP device visible");
    if (device < 0 || device >= n) throw ApiError(DDPCA_EINVAL, "device index out of range");
    DDPCA_HIP(hipSetDevice(device));
    hipDeviceProp_t prop;
    DDPCA_HIP(hipGetDeviceProperties(&prop, device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        throw ApiError(DDPCA_ENOGPU, std::string("device is ") + prop.gcnArchName + ", kernels are built for gfx950");
}

MgpisDevice::MgpisDevice(int dev, const std::vector<int64_t>& nnodes, const std::vector<const Bsr3*>& K,
                         const std::vector<uint8_t>& dof_free, const std::vector<const Stencil*>& S,
                         const mgpis_options_t& o)
    : device(dev), opt(o) {
    select_device(device);
    DDPCA_HIP(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    const int nlev = (int)nnodes.size();
    if (nlev < 1 || (int)K.size() != nlev || (int)S.size() != nlev - 1) throw ApiError(DDPCA_EINVAL, "level counts");
    if ((int64_t)dof_free.size() != 3 * nnodes.back()) throw ApiError(DDPCA_EINVAL, "dof_free length");
    if (opt.nu < 1) opt.nu = 1;
    if (opt.iters_per_graph < 1) opt.iters_per_graph = 1;
    const bool bj = opt.smoother >= 1;
    lev.resize(nlev);
    for (int l = 0; l < nlev; ++l) {
        LevelDev& L = lev[l];
        const Bsr3& A = *K[l];
        const int64_t nn = nnodes[l];
        if (A.nb != nn || A.mb != nn) throw ApiError(DDPCA_EINVAL, "operator size does not match nnodes");
        L.nn = nn;
        L.nch = (nn + kChunk - 1) / kChunk;
        L.nnzb = A.nnzb();
        auto fr = [&](int64_t dof) { return dof_free[dof] != 0; };
        std::vector<int32_t> slots(L.nch);
        std::vector<int64_t> off(L.nch + 1, 0);
        for (int64_t c = 0; c < L.nch; ++c) {
            int64_t mx = 0;
            for (int64_t r = c * kChunk; r < std::min(nn, (c + 1) * kChunk); ++r) mx = std::max(mx, A.ptr[r + 1] - A.ptr[r]);
            slots[c] = (int32_t)mx;
            off[c + 1] = off[c] + mx;
        }
        L.nslots = off[L.nch];
        std::vector<int32_t> col(L.nslots * kChunk, 0);
        std::vector<double> val(L.nslots * kChunk * 9, 0.0);
        std::vector<double> dinv(3 * nn, 0.0), minv(bj ? 9 * nn : 3 * nn, 0.0);
        std::vector<uint8_t> mask(nn, 0);
#pragma omp parallel for schedule(static)
        for (int64_t r = 0; r < nn; ++r) {
            const int64_t c = r / kChunk, lane = r % kChunk;
            uint8_t m = 0;
            for (int a = 0; a < 3; ++a) m |= fr(3 * r + a) ? (1 << a) : 0;
            mask[r] = m;
            double diag[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
            for (int64_t k = A.ptr[r]; k < A.ptr[r + 1]; ++k) {
                const int64_t s = off[c] + (k - A.ptr[r]);
                const int64_t j = A.col[k];
                col[s * kChunk + lane] = (int32_t)j;
                for (int a = 0; a < 3; ++a)
                    for (int b = 0; b < 3; ++b) {
                        double v = A.val[9 * k + 3 * a + b];
                        if (!fr(3 * r + a) || !fr(3 * j + b)) v = (j == r && a == b) ? 1.0 : 0.0;
                        val[(s * 9 + 3 * a + b) * kChunk + lane] = v;
                        if (j == r) diag[3 * a + b] = v;
                    }
            }
            for (int64_t s = off[c] + (A.ptr[r + 1] - A.ptr[r]); s < off[c + 1]; ++s) col[s * kChunk + lane] = (int32_t)r;
            for (int a = 0; a < 3; ++a) dinv[3 * r + a] = fr(3 * r + a) ? 1.0 / diag[4 * a] : 0.0;
            if (bj) {
                double inv[9];
                if (!invert3(diag, inv)) for (int q = 0; q < 9; ++q) inv[q] = 0.0;
                for (int a = 0; a < 3; ++a)
                    for (int b = 0; b < 3; ++b) minv[9 * r + 3 * a + b] = (fr(3 * r + a) && fr(3 * r + b)) ? inv[3 * a + b] : 0.0;
            } else {
                for (int a = 0; a < 3; ++a) minv[3 * r + a] = dinv[3 * r + a];
            }
        }
        // padding lanes of the last chunk point at node 0 with zero values
        L.slots.upload(slots);
        L.off.upload(off);
        L.col.upload(col);
        L.val.upload(val);
        L.dinv.upload(dinv);
        L.minv.upload(minv);
        L.mask.upload(mask);
        L.x.alloc(3 * nn);
        L.t.alloc(3 * nn);
        L.b.alloc(3 * nn);
        L.r.alloc(3 * nn);
        L.d.alloc(3 * nn);
        L.x.zero(stream);
        L.t.zero(stream);
        if (l > 0) {
            const Stencil& st = *S[l - 1];
            if (st.nf != nn || st.nc != nnodes[l - 1]) throw ApiError(DDPCA_EINVAL, "stencil shape");
            const int64_t nc = st.nc, nfn = nn - nc;
            L.nc = nc;
            std::vector<int32_t> ppar(8 * std::max<int64_t>(nfn, 1), -1);
            std::vector<double> pw(8 * std::max<int64_t>(nfn, 1), 0.0);
            std::vector<int64_t> cnt(nc + 1, 0);
            for (int64_t i = 0; i < nn; ++i) {
                const int64_t np = st.ptr[i + 1] - st.ptr[i];
                if (i < nc) {
                    if (np != 1 || st.col[st.ptr[i]] != i || st.w[st.ptr[i]] != 1.0)
                        throw ApiError(DDPCA_EINVAL, "stencil is not identity on coarse nodes");
                    continue;
                }
                if (np > 8) throw ApiError(DDPCA_EINVAL, "more than 8 parents");
                for (int64_t k = 0; k < np; ++k) {
                    ppar[k * nfn + (i - nc)] = st.col[st.ptr[i] + k];
                    pw[k * nfn + (i - nc)] = st.w[st.ptr[i] + k];
                    cnt[st.col[st.ptr[i] + k] + 1]++;
                }
            }
            for (int64_t c = 0; c < nc; ++c) cnt[c + 1] += cnt[c];
            std::vector<int32_t> rch(cnt[nc]);
            std::vector<double> rw(cnt[nc]);
            std::vector<int64_t> fill(cnt.begin(), cnt.end() - 1);
            for (int64_t i = nc; i < nn; ++i)
                for (int64_t k = st.ptr[i]; k < st.ptr[i + 1]; ++k) {
                    const int64_t p = fill[st.col[k]]++;
                    rch[p] = (int32_t)i;
                    rw[p] = st.w[k];
                }
            L.ppar.upload(ppar);
            L.pw.upload(pw);
            L.rptr.upload(cnt);
            L.rch.upload(rch);
            L.rw.upload(rw);
        }
    }
    // exact coarse solve: dense inverse of the masked level-0 operator
    {
        const Bsr3& A = *K[0];
        n0 = 3 * nnodes[0];
        std::vector<double> D(n0 * n0, 0.0);
        for (int64_t r = 0; r < nnodes[0]; ++r)
            for (int64_t k = A.ptr[r]; k < A.ptr[r + 1]; ++k) {
                const int64_t j = A.col[k];
                for (int a = 0; a < 3; ++a)
                    for (int b = 0; b < 3; ++b) {
                        double v = A.val[9 * k + 3 * a + b];
                        if (!dof_free[3 * r + a] || !dof_free[3 * j + b]) v = (j == r && a == b) ? 1.0 : 0.0;
                        D[(3 * r + a) * n0 + 3 * j + b] = v;
                    }
            }
        invert_spd_dense(D, n0);
        for (int64_t d = 0; d < n0; ++d)
            if (!dof_free[d])
                for (int64_t e = 0; e < n0; ++e) D[d * n0 + e] = D[e * n0 + d] = 0.0;
        ainv.upload(D);
    }
    // condensed <-> nodal map of the fine level
    for (int64_t d = 0; d < 3 * nnodes.back(); ++d)
        if (dof_free[d]) free_dof_host.push_back((int32_t)d);
    nfree = (int64_t)free_dof_host.size();
    free_dof.upload(free_dof_host);
    const int64_t nnL = nnodes.back();
    for (auto* v : {&xs, &rs, &zs, &ps, &qs, &bs}) {
        v->alloc(3 * nnL);
        v->zero(stream);
    }
    nblk_fine = ceil_div(nnL, kBlock);
    int64_t maxblk = nblk_fine;
    for (auto& L : lev) maxblk = std::max<int64_t>(maxblk, ceil_div(L.nn, kBlock));
    partial.alloc(maxblk);
    sc.alloc(1);
    DDPCA_HIP(hipHostMalloc(&sc_host, sizeof(PcgScal)));
    std::memset(sc_host, 0, sizeof(PcgScal));
    DDPCA_HIP(hipEventCreate(&ev_k0));
    DDPCA_HIP(hipEventCreate(&ev_k1));
    // smoother damping from the spectrum of M K on each smoothed level
    for (int l = 1; l < nlev; ++l) {
        estimate_lmax(l);
        lev[l].omega = opt.omega > 0.0 ? opt.omega : 4.0 / (3.0 * lev[l].lmax);
    }
    if (nlev == 1) lev[0].omega = 1.0;
    DDPCA_HIP(hipStreamSynchronize(stream));
}

MgpisDevice::~MgpisDevice() {
    (void)hipSetDevice(device);
    if (stream) (void)hipStreamSynchronize(stream);
    for (auto& g : graph_)
        if (g) (void)hipGraphExecDestroy(g);
    if (sc_host) (void)hipHostFree(sc_host);
    if (ev_k0) (void)hipEventDestroy(ev_k0);
    if (ev_k1) (void)hipEventDestroy(ev_k1);
    if (stream) (void)hipStreamDestroy(stream);
}

void MgpisDevice::estimate_lmax(int l) {
    LevelDev& L = lev[l];
    const bool bj = opt.smoother >= 1;
    const int64_t n = 3 * L.nn;
    std::vector<double> h(n);
    std::mt19937_64 rng(20251017 + l);
    std::uniform_real_distribution<double> U(-1.0, 1.0);
    std::vector<uint8_t> mask = L.mask.download();
    for (int64_t i = 0; i < n; ++i) h[i] = (mask[i / 3] >> (i % 3)) & 1 ? U(rng) : 0.0;
    DevBuf<double> v, w;
    v.upload(h);
    w.alloc(n);
    const int nb = ceil_div(L.nn, kBlock);
    double lam = 0.0;
    auto norm2 = [&]() {
        std::vector<double> p(nb);
        DDPCA_HIP(hipMemcpyAsync(p.data(), partial.p, nb * sizeof(double), hipMemcpyDeviceToHost, stream));
        DDPCA_HIP(hipStreamSynchronize(stream));
        return std::accumulate(p.begin(), p.end(), 0.0);
    };
    // normalise
    if (bj) hipLaunchKernelGGL((k_apply_m<true>), dim3(nb), dim3(kBlock), 0, stream, v.p, L.minv.p, w.p, partial.p, L.nn);
    else hipLaunchKernelGGL((k_apply_m<false>), dim3(nb), dim3(kBlock), 0, stream, v.p, L.minv.p, w.p, partial.p, L.nn);
    double nrm = std::sqrt(norm2());
    for (int it = 0; it < 24; ++it) {
        // v <- w / |w| ; w <- M K v
        std::vector<double> tmp(n);
        DDPCA_HIP(hipMemcpyAsync(tmp.data(), w.p, n * sizeof(double), hipMemcpyDeviceToHost, stream));
        DDPCA_HIP(hipStreamSynchronize(stream));
        for (auto& t : tmp) t /= nrm;
        DDPCA_HIP(hipMemcpyAsync(v.p, tmp.data(), n * sizeof(double), hipMemcpyHostToDevice, stream));
        spmv(l, v.p, L.r.p);
        if (bj) hipLaunchKernelGGL((k_apply_m<true>), dim3(nb), dim3(kBlock), 0, stream, L.r.p, L.minv.p, w.p, partial.p, L.nn);
        else hipLaunchKernelGGL((k_apply_m<false>), dim3(nb), dim3(kBlock), 0, stream, L.r.p, L.minv.p, w.p, partial.p, L.nn);
        nrm = std::sqrt(norm2());
        lam = nrm;
    }
    L.lmax = lam * 1.05;  // safety margin on the power-iteration estimate
}

// ============================================================================== operations
void MgpisDevice::spmv(int level, const double* x, double* y) {
    LevelDev& L = lev[level];
    SellArgs a{};
    a.slots = L.slots.p; a.off = L.off.p; a.col = L.col.p; a.val = L.val.p;
    a.nn = L.nn; a.nch = L.nch; a.x = x; a.y = y; a.done = zero_flag();
    hipLaunchKernelGGL((k_sell<kSpmv, false, false>), dim3(ceil_div(L.nch, 4)), dim3(kBlock), 0, stream, a);
}

void MgpisDevice::vcycle(const double* rin, double* zout, bool dot) {
    const int nlev = (int)lev.size();
    const int Lf = nlev - 1;
    const bool bj = opt.smoother >= 1;
    const bool cheb = opt.smoother == 2;
    const int nu = opt.nu;
    const int* done = reinterpret_cast<const int*>(&sc.p->done);
    if (Lf == 0) {
        hipLaunchKernelGGL(k_coarse, dim3(ceil_div(n0, 4)), dim3(kBlock), 0, stream, ainv.p, rin, zout, n0, done);
        if (dot) hipLaunchKernelGGL(k_dot, dim3(nblk_fine), dim3(kBlock), 0, stream, rin, zout, partial.p, lev[0].nn, done);
        return;
    }
    std::vector<double*> cur(nlev), oth(nlev);
    for (int l = 0; l < nlev; ++l) { cur[l] = lev[l].x.p; oth[l] = lev[l].t.p; }
    cur[Lf] = lev[Lf].t.p;
    oth[Lf] = zout;
    auto bvec = [&](int l) -> const double* { return l == Lf ? rin : lev[l].b.p; };
    auto sell_args = [&](int l) {
        LevelDev& L = lev[l];
        SellArgs a{};
        a.slots = L.slots.p; a.off = L.off.p; a.col = L.col.p; a.val = L.val.p;
        a.nn = L.nn; a.nch = L.nch; a.minv = L.minv.p; a.omega = L.omega; a.done = done; a.partial = partial.p;
        a.sc = sc.p;
        return a;
    };
    // Chebyshev coefficients on [lmax/30, lmax] of M K (sweep k uses coefficient pair k)
    auto cheb_coef = [&](int l, int k, double& c1, double& c2) {
        const double lmax = lev[l].lmax, lmin = lmax / 30.0;
        const double theta = 0.5 * (lmax + lmin), delta = 0.5 * (lmax - lmin), sigma = theta / delta;
        double rho_old = 1.0 / sigma, rho = rho_old;
        for (int i = 1; i <= k; ++i) {
            rho = 1.0 / (2.0 * sigma - rho_old);
            if (i < k) rho_old = rho;
        }
        c1 = rho * rho_old;
        c2 = 2.0 * rho / delta;
    };
    // smoothing sweeps on level l from the current iterate (first: jac0/restrict already did sweep 0)
    auto smooth = [&](int l, int first, int count, bool last_dot) {
        for (int s = first; s < first + count; ++s) {
            SellArgs a = sell_args(l);
            a.x = cur[l];
            a.b = bvec(l);
            a.xo = oth[l];
            const bool d = last_dot && s == first + count - 1;
            const int grid = ceil_div(lev[l].nch, 4);
            if (cheb) {
                a.p = lev[l].d.p;
                cheb_coef(l, s, a.c1, a.c2);
                if (s == 0) { a.c1 = 0.0; a.c2 = 1.0 / (0.5 * (lev[l].lmax + lev[l].lmax / 30.0)); }
                if (d) hipLaunchKernelGGL((k_sell<kCheb, true, true>), dim3(grid), dim3(kBlock), 0, stream, a);
                else hipLaunchKernelGGL((k_sell<kCheb, true, false>), dim3(grid), dim3(kBlock), 0, stream, a);
            } else if (bj) {
                if (d) hipLaunchKernelGGL((k_sell<kJac, true, true>), dim3(grid), dim3(kBlock), 0, stream, a);
                else hipLaunchKernelGGL((k_sell<kJac, true, false>), dim3(grid), dim3(kBlock), 0, stream, a);
            } else {
                if (d) hipLaunchKernelGGL((k_sell<kJac, false, true>), dim3(grid), dim3(kBlock), 0, stream, a);
                else hipLaunchKernelGGL((k_sell<kJac, false, false>), dim3(grid), dim3(kBlock), 0, stream, a);
            }
            std::swap(cur[l], oth[l]);
        }
    };
    // omega of the zero-guess first sweep (Chebyshev: 1/theta)
    auto first_omega = [&](int l) { return cheb ? 1.0 / (0.5 * (lev[l].lmax + lev[l].lmax / 30.0)) : lev[l].omega; };
    // ---- descend
    {
        const int grid = ceil_div(lev[Lf].nn, kBlock);
        const double om = first_omega(Lf);
        if (cheb) hipLaunchKernelGGL((k_jac0<true, true>), dim3(grid), dim3(kBlock), 0, stream, rin, lev[Lf].minv.p, om, cur[Lf], lev[Lf].d.p, lev[Lf].nn, done);
        else if (bj) hipLaunchKernelGGL((k_jac0<true, false>), dim3(grid), dim3(kBlock), 0, stream, rin, lev[Lf].minv.p, om, cur[Lf], nullptr, lev[Lf].nn, done);
        else hipLaunchKernelGGL((k_jac0<false, false>), dim3(grid), dim3(kBlock), 0, stream, rin, lev[Lf].minv.p, om, cur[Lf], nullptr, lev[Lf].nn, done);
    }
    for (int l = Lf; l >= 1; --l) {
        smooth(l, 1, nu - 1, false);
        {
            SellArgs a = sell_args(l);
            a.x = cur[l];
            a.b = bvec(l);
            a.y = lev[l].r.p;
            hipLaunchKernelGGL((k_sell<kResid, false, false>), dim3(ceil_div(lev[l].nch, 4)), dim3(kBlock), 0, stream, a);
        }
        const int c = l - 1;
        const int grid = ceil_div(lev[c].nn, kBlock);
        const LevelDev& F = lev[l];
        const double om = c > 0 ? first_omega(c) : 0.0;
        if (c == 0)
            hipLaunchKernelGGL((k_restrict<false, false, false>), dim3(grid), dim3(kBlock), 0, stream, F.r.p, F.rptr.p, F.rch.p, F.rw.p, lev[c].mask.p, lev[c].b.p, nullptr, nullptr, nullptr, 0.0, lev[c].nn, done);
        else if (cheb)
            hipLaunchKernelGGL((k_restrict<true, true, true>), dim3(grid), dim3(kBlock), 0, stream, F.r.p, F.rptr.p, F.rch.p, F.rw.p, lev[c].mask.p, lev[c].b.p, cur[c], lev[c].d.p, lev[c].minv.p, om, lev[c].nn, done);
        else if (bj)
            hipLaunchKernelGGL((k_restrict<true, true, false>), dim3(grid), dim3(kBlock), 0, stream, F.r.p, F.rptr.p, F.rch.p, F.rw.p, lev[c].mask.p, lev[c].b.p, cur[c], nullptr, lev[c].minv.p, om, lev[c].nn, done);
        else
            hipLaunchKernelGGL((k_restrict<true, false, false>), dim3(grid), dim3(kBlock), 0, stream, F.r.p, F.rptr.p, F.rch.p, F.rw.p, lev[c].mask.p, lev[c].b.p, cur[c], nullptr, lev[c].minv.p, om, lev[c].nn, done);
    }
    hipLaunchKernelGGL(k_coarse, dim3(ceil_div(n0, 4)), dim3(kBlock), 0, stream, ainv.p, lev[0].b.p, cur[0], n0, done);
    // ---- ascend
    for (int l = 1; l <= Lf; ++l) {
        const LevelDev& F = lev[l];
        hipLaunchKernelGGL(k_prolong, dim3(ceil_div(F.nn, kBlock)), dim3(kBlock), 0, stream, cur[l - 1], F.ppar.p, F.pw.p, F.mask.p, cur[l], F.nn, F.nc, done);
        // post-smoothing restarts the smoother (Chebyshev recurrence) from the prolongated iterate
        smooth(l, 0, nu, dot && l == Lf);
    }
    if (cur[Lf] != zout) throw ApiError(DDPCA_ESTATE, "V-cycle buffer parity");
}

double MgpisDevice::fine_kernel_bytes() const {
    // algorithmic bytes of one fine-level k_sell<kPcg>: 76 B per stored block (72 value + 4 index)
    // + z gathered once (24 B/node) + p, q read and written (4 x 24 B/node)
    const LevelDev& L = lev.back();
    return 76.0 * (double)L.nnzb + 24.0 * 5.0 * (double)L.nn;
}

void MgpisDevice::enqueue_iteration(int prec, bool timed) {
    LevelDev& L = lev.back();
    const int* done = reinterpret_cast<const int*>(&sc.p->done);
    SellArgs a{};
    a.slots = L.slots.p; a.off = L.off.p; a.col = L.col.p; a.val = L.val.p;
    a.nn = L.nn; a.nch = L.nch; a.x = zs.p; a.y = qs.p; a.p = ps.p; a.sc = sc.p; a.partial = partial.p; a.done = done;
    if (timed) DDPCA_HIP(hipEventRecord(ev_k0, stream));
    hipLaunchKernelGGL((k_sell<kPcg, false, true>), dim3(ceil_div(L.nch, 4)), dim3(kBlock), 0, stream, a);
    if (timed) DDPCA_HIP(hipEventRecord(ev_k1, stream));
    hipLaunchKernelGGL(k_fin, dim3(1), dim3(kBlock), 0, stream, (int)kFinAlpha, partial.p, nblk_fine, sc.p);
    hipLaunchKernelGGL(k_axpy, dim3(nblk_fine), dim3(kBlock), 0, stream, xs.p, rs.p, ps.p, qs.p, sc.p, partial.p, L.nn, done);
    hipLaunchKernelGGL(k_fin, dim3(1), dim3(kBlock), 0, stream, (int)kFinRR, partial.p, nblk_fine, sc.p);
    if (prec == 1) vcycle(rs.p, zs.p, true);
    else hipLaunchKernelGGL(k_diag, dim3(nblk_fine), dim3(kBlock), 0, stream, rs.p, L.dinv.p, zs.p, partial.p, L.nn, done);
    hipLaunchKernelGGL(k_fin, dim3(1), dim3(kBlock), 0, stream, (int)kFinBeta, partial.p, nblk_fine, sc.p);
}

// graph_[prec]: iters_per_graph PCG iterations captured once and replayed.
void MgpisDevice::build_graph(int prec) {
    if (graph_[prec]) return;
    hipGraph_t g;
    DDPCA_HIP(hipStreamBeginCapture(stream, hipStreamCaptureModeThreadLocal));
    for (int k = 0; k < opt.iters_per_graph; ++k) enqueue_iteration(prec, false);
    DDPCA_HIP(hipStreamEndCapture(stream, &g));
    DDPCA_HIP(hipGraphInstantiate(&graph_[prec], g, nullptr, nullptr, 0));
    DDPCA_HIP(hipGraphDestroy(g));
}

void MgpisDevice::pcg_begin(int prec, double rtol, int64_t maxit) {
    select_device(device);
    build_graph(prec);
    LevelDev& L = lev.back();
    PcgScal init{};
    init.tol2 = rtol * rtol;
    init.maxit = maxit;
    DDPCA_HIP(hipMemcpyAsync(sc.p, &init, sizeof(PcgScal), hipMemcpyHostToDevice, stream));
    hipLaunchKernelGGL(k_pcg_init, dim3(nblk_fine), dim3(kBlock), 0, stream, bs.p, xs.p, rs.p, ps.p, qs.p, partial.p, L.nn);
    hipLaunchKernelGGL(k_fin, dim3(1), dim3(kBlock), 0, stream, (int)kFinInit, partial.p, nblk_fine, sc.p);
    const int* done = reinterpret_cast<const int*>(&sc.p->done);
    if (prec == 1) vcycle(rs.p, zs.p, true);
    else hipLaunchKernelGGL(k_diag, dim3(nblk_fine), dim3(kBlock), 0, stream, rs.p, L.dinv.p, zs.p, partial.p, L.nn, done);
    hipLaunchKernelGGL(k_fin, dim3(1), dim3(kBlock), 0, stream, (int)kFinBeta0, partial.p, nblk_fine, sc.p);
    if (time_kernel) {
        // first iteration eagerly, with HIP events around its fine-level SpMV on this stream
        enqueue_iteration(prec, true);
        sample_pending_ = true;
    }
}

void MgpisDevice::pcg_step(int prec) { DDPCA_HIP(hipGraphLaunch(graph_[prec], stream)); }

bool MgpisDevice::pcg_poll() {
    DDPCA_HIP(hipMemcpyAsync(sc_host, sc.p, sizeof(PcgScal), hipMemcpyDeviceToHost, stream));
    DDPCA_HIP(hipStreamSynchronize(stream));
    if (sample_pending_) {
        // keep the sample only if the timed SpMV ran a real iteration (done was 0)
        float ms = 0.f;
        if (sc_host->iter >= 1 && hipEventElapsedTime(&ms, ev_k0, ev_k1) == hipSuccess && ms > 0.f) {
            timed_kernel_ms += ms;
            timed_kernel_samples += 1;
        }
        sample_pending_ = false;
    }
    return sc_host->done != 0;
}

int64_t MgpisDevice::pcg_solve(int prec, double rtol, int64_t maxit, int64_t* iters, double* relres) {
    pcg_begin(prec, rtol, maxit);
    while (!pcg_poll()) pcg_step(prec);
    if (sc_host->fail) throw ApiError(DDPCA_ENUMERIC, "PCG breakdown (non-finite or non-positive curvature)");
    if (iters) *iters = sc_host->iter;
    if (relres) *relres = sc_host->bb > 0 ? std::sqrt(sc_host->rr / sc_host->bb) : 0.0;
    return sc_host->iter;
}

void MgpisDevice::scatter_free(const double* cond, double* full) {
    DDPCA_HIP(hipMemsetAsync(full, 0, 3 * lev.back().nn * sizeof(double), stream));
    hipLaunchKernelGGL(k_scatter, dim3(ceil_div(nfree, kBlock)), dim3(kBlock), 0, stream, cond, free_dof.p, full, nfree);
}

void MgpisDevice::gather_free(const double* full, double* cond) {
    hipLaunchKernelGGL(k_gather, dim3(ceil_div(nfree, kBlock)), dim3(kBlock), 0, stream, full, free_dof.p, cond, nfree);
}

}  // namespace ddpca
