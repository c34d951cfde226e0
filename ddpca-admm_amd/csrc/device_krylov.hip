// The other solver drivers of the MGPIS class surface on the device: MULT_SOLV (MGPIS.h:130-160),
// BiCGSTAB_SOLV (MGPIS.h:350-432) and GMRES_SOLV (MGPIS.h:228-348).  They reuse the CG path's
// operators and kernels -- the fp64 SELL-BSR3 SpMV of the fine level and the V-cycle (or the
// point-Jacobi inverse for precSwit = 0) -- and add the vector kernels below: a multi-dot
// (up to kMaxDots pairs in one pass, fixed-order two-stage reduction, deterministic) and the
// fused update kernels of each recurrence.  The Krylov scalars are formed on the host exactly in
// the reference's order (the small dense GMRES least-squares problem included); every vector
// stays in HBM in the fine level's batch nodal layout.  These drivers serve one subdomain (the
// mgpis_gpu_create handles); the batched ADMM loop uses CG only, as the reference does
// (MCONTACT.h:2531).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "device_mgpis.hpp"

namespace ddpca {
namespace {

constexpr int kMaxDots = 12;
constexpr int kDotBlocks = 1024;
constexpr int kMaxBasis = 24;  // GMRES restart length bound (the reference uses 10)

struct DotArgs {
    const double* a[kMaxDots];
    const double* b[kMaxDots];
    int m;
};

__device__ __forceinline__ double wsum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// partial[k * gridDim.x + block] = sum over this block's grid-stride share of a_k . b_k
__global__ __launch_bounds__(kBlock) void k_mdot(DotArgs d, int64_t n, double* partial) {
    double s[kMaxDots];
#pragma unroll
    for (int k = 0; k < kMaxDots; ++k) s[k] = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
#pragma unroll
        for (int k = 0; k < kMaxDots; ++k)
            if (k < d.m) s[k] += d.a[k][i] * d.b[k][i];
    }
    __shared__ double red[kMaxDots][kBlock / kWave];
#pragma unroll
    for (int k = 0; k < kMaxDots; ++k) {
        if (k < d.m) {
            const double v = wsum(s[k]);
            if ((threadIdx.x & 63) == 0) red[k][threadIdx.x >> 6] = v;
        }
    }
    __syncthreads();
    if (threadIdx.x < d.m) {
        const int k = threadIdx.x;
        partial[(int64_t)k * gridDim.x + blockIdx.x] = (red[k][0] + red[k][1]) + (red[k][2] + red[k][3]);
    }
}

// out[k] = sum of the kDotBlocks partials of dot k, one workgroup per dot, fixed order
__global__ __launch_bounds__(kBlock) void k_mdot_fin(const double* partial, int nblk, double* out) {
    const int k = blockIdx.x;
    double s = 0.0;
    for (int j = threadIdx.x; j < nblk; j += kBlock) s += partial[(int64_t)k * nblk + j];
    s = wsum(s);
    __shared__ double red[kBlock / kWave];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) out[k] = (red[0] + red[1]) + (red[2] + red[3]);
}

#define GRID_STRIDE(n) for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < (n); i += (int64_t)gridDim.x * kBlock)

// out = x + a y (r = b - Kx with a = -1, s = r - alpha v, x += z with a = 1)
__global__ __launch_bounds__(kBlock) void k_xpay(int64_t n, const double* x, double a, const double* y, double* out) {
    GRID_STRIDE(n) out[i] = x[i] + a * y[i];
}

// z = D^-1 r (DIAG_PREC, PREP.h; the inverse is zero on constrained dofs and padding)
__global__ __launch_bounds__(kBlock) void k_hadamard(int64_t n, const double* d, const double* r, double* z) {
    GRID_STRIDE(n) z[i] = d[i] * r[i];
}

// out = x / s (basis normalisation: the reference divides, MGPIS.h:271, 303)
__global__ __launch_bounds__(kBlock) void k_div(int64_t n, const double* x, double s, double* out) {
    GRID_STRIDE(n) out[i] = x[i] / s;
}

// BiCGSTAB direction: p = r + beta (p - omega v) (MGPIS.h:395)
__global__ __launch_bounds__(kBlock) void k_bicg_p(int64_t n, const double* r, double beta, double omega,
                                                   const double* v, double* p) {
    GRID_STRIDE(n) p[i] = r[i] + beta * (p[i] - omega * v[i]);
}

// BiCGSTAB update: x += alpha ph + omega sh; r = s - omega t (MGPIS.h:420-421)
__global__ __launch_bounds__(kBlock) void k_bicg_x(int64_t n, double alpha, const double* ph, double omega,
                                                   const double* sh, const double* s, const double* t, double* x,
                                                   double* r) {
    GRID_STRIDE(n) {
        x[i] += alpha * ph[i] + omega * sh[i];
        r[i] = s[i] - omega * t[i];
    }
}

struct Coef {
    double c[kMaxBasis + 1];
};

// out = base + sign * sum_{k<m} V_k c_k, V column-major with leading dimension ld
// (Arnoldi: q = pv - V b, MGPIS.h:268; iterate: x = x0 + V y, MGPIS.h:327)
__global__ __launch_bounds__(kBlock) void k_vcomb(int64_t n, const double* base, double sign, const double* V, int64_t ld,
                                                  int m, Coef c, double* out) {
    GRID_STRIDE(n) {
        double s = 0.0;
        for (int k = 0; k < m; ++k) s += V[k * ld + i] * c.c[k];
        out[i] = base[i] + sign * s;
    }
}

int grid_for(int64_t n) { return (int)std::min<int64_t>(ceil_div(n, kBlock), 4096); }

// Vectors of the fine level plus the reduction scratch of one driver call.
struct Work {
    MgpisDevice& D;
    int64_t n;  // 3 * nodes of the fine level (batch nodal layout, padding included)
    hipStream_t st;
    DevBuf<double> partial, out, mem;
    double* host = nullptr;
    Work(MgpisDevice& d, int nvec) : D(d), n(3 * d.lev.back().nn), st(d.stream) {
        partial.alloc((size_t)kMaxDots * kDotBlocks);
        out.alloc(kMaxDots);
        mem.alloc((size_t)nvec * n);
        mem.zero(st);
        DDPCA_HIP(hipHostMalloc(&host, kMaxDots * sizeof(double), hipHostMallocDefault));
        // the V-cycle kernels skip members whose stop flag is set: clear it (one member)
        DDPCA_HIP(hipMemsetAsync(D.sc.p, 0, sizeof(PcgScal) * D.nsub, st));
    }
    ~Work() {
        if (host) (void)hipHostFree(host);
    }
    double* vec(int k) { return mem.p + (int64_t)k * n; }
    // a_k . b_k for every pair, one pass over the operands, synchronising
    std::vector<double> dots(std::initializer_list<std::pair<const double*, const double*>> pairs) {
        DotArgs d{};
        d.m = 0;
        for (const auto& pr : pairs) {
            d.a[d.m] = pr.first;
            d.b[d.m] = pr.second;
            ++d.m;
        }
        return run(d);
    }
    std::vector<double> run(const DotArgs& d) {
        hipLaunchKernelGGL(k_mdot, dim3(kDotBlocks), dim3(kBlock), 0, st, d, n, partial.p);
        hipLaunchKernelGGL(k_mdot_fin, dim3(d.m), dim3(kBlock), 0, st, partial.p, kDotBlocks, out.p);
        DDPCA_HIP(hipGetLastError());
        DDPCA_HIP(hipMemcpyAsync(host, out.p, d.m * sizeof(double), hipMemcpyDeviceToHost, st));
        DDPCA_HIP(hipStreamSynchronize(st));
        return std::vector<double>(host, host + d.m);
    }
    double norm(const double* x) { return std::sqrt(dots({{x, x}})[0]); }
    void xpay(const double* x, double a, const double* y, double* o) {
        hipLaunchKernelGGL(k_xpay, dim3(grid_for(n)), dim3(kBlock), 0, st, n, x, a, y, o);
    }
    // z = M^-1 r: V-cycle (prec 1) or point Jacobi (prec 0); r, z distinct from the V-cycle's
    // own level buffers
    void precond(int prec, const double* r, double* z) {
        if (prec == 0)
            hipLaunchKernelGGL(k_hadamard, dim3(grid_for(n)), dim3(kBlock), 0, st, n, D.lev.back().dinv.p, r, z);
        else
            D.vcycle(r, z, false);
    }
    void spmv(const double* x, double* y) { D.spmv((int)D.lev.size() - 1, x, y); }
};

void check_finite(double v, const char* what) {
    if (!std::isfinite(v)) throw ApiError(DDPCA_ENUMERIC, std::string("non-finite ") + what);
}

// VECT_MEDI_OSCI (PREP.h:147-153)
void medi_osci(const std::vector<double>& v, double& medi, double& osci) {
    const double mx = *std::max_element(v.begin(), v.end()), mn = *std::min_element(v.begin(), v.end());
    medi = (mx + mn) / 2.0;
    osci = mx - mn;
}

}  // namespace

// MGPIS::MULT_SOLV (MGPIS.h:130-160).  The reference applies MULT_VCYC(maxiLeve, b, x) to the
// running iterate; a V-cycle is affine in its initial guess, so that is x + B (b - K x) with B
// the V-cycle from zero: one V-cycle and one fp64 SpMV per iteration (the residual of iteration
// k is the V-cycle input of k + 1).  Stop when the last five residual norms oscillate by less
// than 0.1 of their median, or after maxit V-cycles.  Returns iterNumb at exit.
int64_t krylov_mult_solv(MgpisDevice& D, const double* b, double* x, int64_t maxit, double* relres) {
    Work w(D, 3);
    double *r = w.vec(0), *z = w.vec(1), *kx = w.vec(2);
    DDPCA_HIP(hipMemsetAsync(x, 0, w.n * sizeof(double), w.st));
    DDPCA_HIP(hipMemcpyAsync(r, b, w.n * sizeof(double), hipMemcpyDeviceToDevice, w.st));
    const double bn = w.norm(b);
    if (bn == 0.0) {  // x = 0 is exact (the reference would cycle to maxit on zero residuals)
        if (relres) *relres = 0.0;
        return 0;
    }
    std::vector<double> moni(5, 0.0);
    int64_t it = 0;
    double rn = 0.0;
    while (it < maxit) {
        w.precond(1, r, z);
        w.xpay(x, 1.0, z, x);
        w.spmv(x, kx);
        w.xpay(b, -1.0, kx, r);
        rn = w.norm(r);
        check_finite(rn, "residual (MULT_SOLV)");
        moni[it % 5] = rn;
        if (it >= 4) {
            double medi, osci;
            medi_osci(moni, medi, osci);
            if (osci < 0.1 * medi) break;
        }
        ++it;
    }
    if (relres) *relres = bn > 0 ? rn / bn : 0.0;
    return it;
}

// MGPIS::BiCGSTAB_SOLV (MGPIS.h:350-432): right-preconditioned BiCGSTAB from x0 = 0 with the
// shadow residual r^ = r0 = b; stop on the recursive residual ||r|| <= rtol ||b||, on
// rho = 0 (the reference's "ERROR 1" exit, reported through *breakdown = 1), after maxit, or --
// only when `attainable` is set (LAGRANGE's Newton steps; the public MGPIS entry point keeps the
// reference's rules) -- at the attainable accuracy: ||r|| <= 100 rtol ||b|| and flat over five
// iterations, reported through *breakdown = 2.
// The dot products that share operands are fused into one pass: (r^ v), (t s) + (t t),
// (r r) + (r^ r) for the next iteration.  Returns iterNumb at exit.
int64_t krylov_bicgstab(MgpisDevice& D, int prec, const double* b, double* x, double rtol, int64_t maxit,
                        double* relres, int* breakdown, bool attainable) {
    Work w(D, 8);
    double *r = w.vec(0), *rh = w.vec(1), *p = w.vec(2), *v = w.vec(3), *ph = w.vec(4), *s = w.vec(5),
           *sh = w.vec(6), *t = w.vec(7);
    DDPCA_HIP(hipMemsetAsync(x, 0, w.n * sizeof(double), w.st));
    DDPCA_HIP(hipMemcpyAsync(r, b, w.n * sizeof(double), hipMemcpyDeviceToDevice, w.st));
    DDPCA_HIP(hipMemcpyAsync(rh, b, w.n * sizeof(double), hipMemcpyDeviceToDevice, w.st));
    std::vector<double> d = w.dots({{r, r}, {rh, r}});
    const double bn = std::sqrt(d[0]);
    const double tol = rtol * bn;
    double rr = d[0], rhr = d[1];
    double rho[2] = {0.0, 0.0}, alph = 0.0, omeg = 0.0;
    int64_t it = 0;
    if (breakdown) *breakdown = 0;
    static const bool trace = std::getenv("DDPCA_KRYLOV_TRACE") != nullptr;  // per-iteration scalars on stderr
    std::vector<double> moni(5, 0.0);
    while (it < maxit && std::sqrt(rr) > tol) {
        double& rc = rho[(it + 1) % 2];
        rc = rhr;
        if (std::fabs(rc) == 0.0) {
            if (breakdown) *breakdown = 1;
            break;
        }
        if (it == 0)
            DDPCA_HIP(hipMemcpyAsync(p, r, w.n * sizeof(double), hipMemcpyDeviceToDevice, w.st));
        else {
            const double beta = (rc / rho[it % 2]) * (alph / omeg);
            hipLaunchKernelGGL(k_bicg_p, dim3(grid_for(w.n)), dim3(kBlock), 0, w.st, w.n, r, beta, omeg, v, p);
        }
        w.precond(prec, p, ph);
        w.spmv(ph, v);
        const double rhv = w.dots({{rh, v}})[0];
        alph = rc / rhv;
        if (trace)
            std::fprintf(stderr, "[ddpca bicgstab] it %lld  |r|/|b| %.3e  rho %.3e  rh.v %.3e  alpha %.3e  omega %.3e\n",
                         (long long)it, std::sqrt(rr) / bn, rc, rhv, alph, omeg);
        check_finite(alph, "alpha (BiCGSTAB)");
        w.xpay(r, -alph, v, s);
        w.precond(prec, s, sh);
        w.spmv(sh, t);
        d = w.dots({{t, s}, {t, t}, {s, s}});
        if (std::sqrt(d[2]) <= 0.0) {  // reference order: ||s|| test before the second half
            w.xpay(x, alph, ph, x);
            rr = 0.0;
            break;
        }
        omeg = d[0] / d[1];
        check_finite(omeg, "omega (BiCGSTAB)");
        hipLaunchKernelGGL(k_bicg_x, dim3(grid_for(w.n)), dim3(kBlock), 0, w.st, w.n, alph, ph, omeg, sh, s, t, x, r);
        d = w.dots({{r, r}, {rh, r}});
        rr = d[0];
        rhr = d[1];
        check_finite(rr, "residual (BiCGSTAB)");
        ++it;
        // attainable-accuracy stop (the reference's GMRES_SOLV rule, MGPIS.h:228-348): within
        // 100 tol and the last five residual norms flat to 10 % of their median.  On singular
        // systems (LAGRANGE, frictionless sliding modes) the recursive residual can stall just
        // above tol; BiCGSTAB then loses r^ . r to rounding and diverges (profiles/r02q_*)
        moni[(it - 1) % 5] = std::sqrt(rr);
        if (attainable && it >= 5 && std::sqrt(rr) > tol && std::sqrt(rr) <= 100.0 * tol) {
            double medi, osci;
            medi_osci(moni, medi, osci);
            if (osci < 0.1 * medi) {
                if (breakdown) *breakdown = 2;
                break;
            }
        }
    }
    DDPCA_HIP(hipStreamSynchronize(w.st));
    if (relres) *relres = bn > 0 ? std::sqrt(rr) / bn : 0.0;
    return it;
}

// MGPIS::GMRES_SOLV (MGPIS.h:228-348): GMRES(restart) on M^-1 K from x0 = 0 (see
// oracle/oracle.cpp orc_gmres for the recurrence): one classical Gram-Schmidt Arnoldi step per
// iteration (one multi-dot V^T pv, one fused q = pv - V b), the Hessenberg's Gram-Schmidt QR
// and the triangular solve on the host, x = x0 + V y and the true residual on the device.
// Stop: ||b - Kx|| <= tol, or <= 100 tol with the last `restart` values oscillating by less
// than 0.1 of their median (tol = rtol ||b||, reference rtol = 1e-12), or maxit.
int64_t krylov_gmres(MgpisDevice& D, int prec, const double* b, double* x, double rtol, int64_t maxit, int64_t restart,
                     double* relres) {
    const int64_t m = restart;
    if (m < 1 || m > kMaxBasis) throw ApiError(DDPCA_EINVAL, "GMRES restart length must be in [1, 24]");
    Work w(D, 5 + (int)m + 1);
    double *x0 = w.vec(0), *r = w.vec(1), *kv = w.vec(2), *pv = w.vec(3), *q = w.vec(4), *V = w.vec(5);
    const int64_t ld = w.n;
    const int64_t hd = m + 1;  // column-major small matrices, leading dimension m + 1
    std::vector<double> H(hd * m), Q(hd * m), R(hd * m), moni(m, 0.0);
    DDPCA_HIP(hipMemsetAsync(x, 0, w.n * sizeof(double), w.st));
    const double bn = w.norm(b);
    if (bn == 0.0) {  // x = 0 is exact (the reference's basis would divide by zero)
        if (relres) *relres = 0.0;
        return 0;
    }
    const double tol = rtol * bn;
    double nr0 = 0.0, rn = 0.0;
    int64_t it = 0;
    while (it < maxit) {
        const int64_t j = it % m;
        if (j == 0) {
            DDPCA_HIP(hipMemcpyAsync(x0, x, w.n * sizeof(double), hipMemcpyDeviceToDevice, w.st));
            w.spmv(x0, kv);
            w.xpay(b, -1.0, kv, r);
            w.precond(prec, r, pv);
            nr0 = w.norm(pv);
            check_finite(nr0, "preconditioned residual (GMRES)");
            hipLaunchKernelGGL(k_div, dim3(grid_for(w.n)), dim3(kBlock), 0, w.st, w.n, pv, nr0, V);
            std::fill(H.begin(), H.end(), 0.0);
            std::fill(Q.begin(), Q.end(), 0.0);
            std::fill(R.begin(), R.end(), 0.0);
        }
        w.spmv(V + j * ld, kv);
        w.precond(prec, kv, pv);
        // b_i = V^T pv (j + 1 dots, in passes of kMaxDots)
        std::vector<double> bi;
        for (int64_t k0 = 0; k0 <= j; k0 += kMaxDots) {
            DotArgs d{};
            d.m = (int)std::min<int64_t>(kMaxDots, j + 1 - k0);
            for (int k = 0; k < d.m; ++k) {
                d.a[k] = V + (k0 + k) * ld;
                d.b[k] = pv;
            }
            const std::vector<double> part = w.run(d);
            bi.insert(bi.end(), part.begin(), part.end());
        }
        Coef c{};
        for (int64_t k = 0; k <= j; ++k) c.c[k] = bi[k];
        hipLaunchKernelGGL(k_vcomb, dim3(grid_for(w.n)), dim3(kBlock), 0, w.st, w.n, pv, -1.0, V, ld, (int)(j + 1), c, q);
        const double nq = w.norm(q);
        check_finite(nq, "Arnoldi norm (GMRES)");
        for (int64_t k = 0; k <= j; ++k) H[j * hd + k] = bi[k];
        H[j * hd + j + 1] = nq;
        hipLaunchKernelGGL(k_div, dim3(grid_for(w.n)), dim3(kBlock), 0, w.st, w.n, q, nq, V + (j + 1) * ld);
        if (j == 0) {
            const double hn = std::sqrt(H[0] * H[0] + H[1] * H[1]);
            Q[0] = H[0] / hn;
            Q[1] = H[1] / hn;
            R[0] = hn;
        } else {
            for (int64_t cc = 0; cc < j; ++cc) {
                double s = 0.0;
                for (int64_t k = 0; k <= j + 1; ++k) s += Q[cc * hd + k] * H[j * hd + k];
                R[j * hd + cc] = s;
            }
            double qq = 0.0;
            for (int64_t k = 0; k <= j + 1; ++k) {
                double s = 0.0;
                for (int64_t cc = 0; cc < j; ++cc) s += Q[cc * hd + k] * R[j * hd + cc];
                Q[j * hd + k] = H[j * hd + k] - s;
                qq += Q[j * hd + k] * Q[j * hd + k];
            }
            const double rjj = std::sqrt(qq);
            R[j * hd + j] = rjj;
            for (int64_t k = 0; k <= j + 1; ++k) Q[j * hd + k] /= rjj;
        }
        Coef y{};
        for (int64_t t = j; t >= 0; --t) {
            double s = 0.0;
            for (int64_t cc = t + 1; cc <= j; ++cc) s += R[cc * hd + t] * y.c[cc];
            y.c[t] = (nr0 * Q[t * hd + 0] - s) / R[t * hd + t];
        }
        hipLaunchKernelGGL(k_vcomb, dim3(grid_for(w.n)), dim3(kBlock), 0, w.st, w.n, x0, 1.0, V, ld, (int)(j + 1), y, x);
        w.spmv(x, kv);
        w.xpay(b, -1.0, kv, r);
        rn = w.norm(r);
        check_finite(rn, "residual (GMRES)");
        moni[it % m] = rn;
        if (it >= m - 1) {
            double medi, osci;
            medi_osci(moni, medi, osci);
            if (rn <= tol || (rn <= 1e2 * tol && osci < 0.1 * medi)) break;
        }
        ++it;
    }
    DDPCA_HIP(hipStreamSynchronize(w.st));
    if (relres) *relres = bn > 0 ? rn / bn : 0.0;
    return it;
}

}  // namespace ddpca
