// MCONTACT device path: the ADMM loop of CONTACT_ANALYSIS (MCONTACT.h:2493-2723) for the
// subdomains and interface sides owned by one rank (one process per GPU).
//
// Per iteration (same data flow as the reference):
//   body balance   b_tv = consForc + consOper (systTran_pena aux - systTran lambda)   (2514-2524)
//                  u_tv = OUTP_SUB1(MGPIS PCG(b_tv))                                 (2531-2533)
//                  -- every owned subdomain in ONE batched PCG (device_mgpis.hpp)
//   interface      gamma = 1/2 (L0 l0 - L1 l1 + R0 u0 - R1 u1 - pema g)              (2632-2636)
//                  -- each side contributes its half; sides on different ranks swap their
//                     halves with one RCCL send/recv pair over xGMI (no global collective)
//                  normal / Coulomb projection                                        (2637-2668)
//                  aux = (M^rho)^-1 (T^T u + M l + I gamma)                           (2671-2684)
//   Lagrange       l += M^-1 (T^T u - M^rho aux)                                      (2689-2704)
//   MONITOR        squared norms reduced on device, one small RCCL all-reduce,
//                  reference stopping logic on the host                               (2725-2845)
//
// Layout: one device workspace W = [u | aux, lambda | gamma] per rank.  u: displacements of all
// owned subdomains in the batch's fine layout (reference node order inside each subdomain);
// aux / lambda: all owned sides, each padded to 64 rows; gamma: every interface.  The three
// interface products (gamma, the aux right-hand side, the lambda right-hand side) of ALL owned
// sides are each ONE SELL-64 operator whose columns index W, so each is one coalesced launch.
// The surface mass solves (LDLT in the reference, < 120000 rows) run as ONE batched Jacobi-PCG
// over every owned side (ELL-64 rows, per-side scalars) to a 1e-14 relative residual.
// Everything runs on the batch's single stream.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <rocblas/rocblas.h>
#include <rocsolver/rocsolver.h>

#include <algorithm>
#include <chrono>
#include <climits>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <numeric>
#include <thread>
#include <tuple>
#include <unordered_map>

#include "../../include/ddpca_amd.h"
#include "device_mgpis.hpp"
#include "problem.hpp"

using namespace ddpca;

namespace {

#define DDPCA_NCCL(call)                                                                                  \
    do {                                                                                                  \
        ncclResult_t r_ = (call);                                                                         \
        if (r_ != ncclSuccess) throw ApiError(DDPCA_ECOMM, std::string(#call) + ": " + ncclGetErrorString(r_)); \
    } while (0)

Csr transpose(const Csr& A) {
    Csr T;
    T.nrow = A.ncol;
    T.ncol = A.nrow;
    T.ptr.assign(T.nrow + 1, 0);
    for (int32_t c : A.col) T.ptr[c + 1]++;
    for (int64_t r = 0; r < T.nrow; ++r) T.ptr[r + 1] += T.ptr[r];
    T.col.resize(A.col.size());
    T.val.resize(A.val.size());
    std::vector<int64_t> fill(T.ptr.begin(), T.ptr.end() - 1);
    for (int64_t r = 0; r < A.nrow; ++r)
        for (int64_t k = A.ptr[r]; k < A.ptr[r + 1]; ++k) {
            const int64_t p = fill[A.col[k]]++;
            T.col[p] = (int32_t)r;
            T.val[p] = A.val[k];
        }
    return T;
}

// ------------------------------------------------------------------------------- kernels
__device__ __forceinline__ double wsum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ double csr_row(const int64_t* ptr, const int32_t* col, const double* val, const double* x,
                                          int64_t r) {
    double s = 0.0;
    for (int64_t k = ptr[r]; k < ptr[r + 1]; ++k) s += val[k] * x[col[k]];
    return s;
}

// y = x, 16 B per lane (n even: batch vectors are 3 * multiple-of-64 long, or 2R)
__global__ void k_copy2(double2* y, const double2* x, int64_t n2) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n2) y[i] = x[i];
}

// b[rows[i]] += sum_k val[k] W[col[k]]  (coupling of the body-balance RHS, surface rows only,
// ~50 entries each): 16 lanes per row, so a row's entries are read as one coalesced segment
__global__ __launch_bounds__(256) void k_cpl(const int32_t* rows, const int64_t* ptr, const int32_t* col,
                                             const double* val, const double* W, double* b, int64_t n) {
    const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 4;
    const int sl = threadIdx.x & 15;
    double s = 0.0;
    if (i < n)
        for (int64_t k = ptr[i] + sl; k < ptr[i + 1]; k += 16) s += val[k] * W[col[k]];
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) s += __shfl_xor(s, o, 16);
    if (i < n && sl == 0) b[rows[i]] += s;
}

// u = mask ? x : prescribed  (OUTP_SUB1 without rotations); x and mask in the solver's device
// node order, u and presc in the reference order (onode: device node -> reference node)
__global__ void k_outp(const double* x, const uint8_t* mask, const int32_t* onode, const double* presc, double* u,
                       int64_t nn) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nn) return;
    const uint8_t m = mask[i];
    const int64_t o = onode[i];
    for (int a = 0; a < 3; ++a) u[3 * o + a] = ((m >> a) & 1) ? x[3 * i + a] : presc[3 * o + a];
}

// y = a - b
__global__ void k_sub(const double* a, const double* b, double* y, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) y[i] = a[i] - b[i];
}

__global__ void k_add(double* y, const double* x, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) y[i] += x[i];
}

// y[row] = sum_k val * W[col] (+ add[row]): one wavefront per 64 rows, slot-major (SELL-64)
__global__ __launch_bounds__(256) void k_sell_w(const int32_t* slots, const int64_t* off, const int32_t* col,
                                                const double* val, int64_t nch, const double* W, double* y,
                                                const double* add) {
    const int64_t c = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (c >= nch) return;
    const int lane = threadIdx.x & 63;
    const int ns = slots[c];
    const int32_t* cp = col + off[c] * 64 + lane;
    const double* vp = val + off[c] * 64 + lane;
    double s = 0.0;
#pragma unroll 4
    for (int k = 0; k < ns; ++k)
        s += __builtin_nontemporal_load(vp + (int64_t)k * 64) * W[__builtin_nontemporal_load(cp + (int64_t)k * 64)];
    const int64_t row = c * 64 + lane;
    y[row] = add ? s + add[row] : s;
}

// normal / Coulomb projection at integration points (MCONTACT.h:2637-2668)
__global__ void k_project(double* g, int32_t* stat, int64_t nip, int comp, double fric) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nip) return;
    if (comp == 1) {
        g[q] = fmax(0.0, g[q]);
        stat[q] = 0;
        return;
    }
    double* v = g + 3 * q;
    if (fric < 0.0) {
        stat[q] = 0;
        return;
    }
    v[0] = fmax(0.0, v[0]);
    if (fric == 0.0) {
        stat[q] = 0;
        return;
    }
    if (v[0] > 0.0) {
        const double slid = fric * v[0];
        const double nt = sqrt(v[1] * v[1] + v[2] * v[2]);
        if (nt >= slid) {
            v[1] = slid / nt * v[1];
            v[2] = slid / nt * v[2];
            stat[q] = 1;
        } else {
            stat[q] = 2;
        }
    } else {
        v[1] = 0.0;
        v[2] = 0.0;
        stat[q] = 0;
    }
}

// ---- factored per-ip interface operators (host-built interfaces, Interface::factored).  Every
// row of inpoLagr, pemaInpo_r and inteInpo is an outer product of ONE integration point's shape
// values, basis and weight (mcontact.cpp BUILD, MCONTACT.h:570-714), so the gamma product and the
// inteInpo product are applied from the ip data -- 4 shape values, 4 + 4 node indices per side and
// the 3x3 basis per ip -- instead of streaming the 24 (frictional: 24 per row, 3 rows) stored
// entries of every gamma row.  Per-ip arrays are slot-major (x[slot * nip + q]).
struct IpSide {
    const double* M;     // 4 x nip shape values
    const int32_t* lam;  // 4 x nip: workspace index of the contact node's first lambda component
    const int32_t* u;    // 4 x nip: workspace index of the body node's first dof
};

// gamma[C q + m] = gcst + sum over owned sides s of h_s (inpoLagr_s lambda_s + pemaInpo_r_s u_s),
// h_0 = 1/2, h_1 = -1/2 (MCONTACT.h:2632-2636); one thread per ip
__global__ __launch_bounds__(256) void k_gamma_ip(const double* B, IpSide s0, IpSide s1, int own0, int own1, double p0,
                                                  double p1, double p2, int C, int64_t nip, const double* W,
                                                  double* gamma, const double* gcst) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nip) return;
    double b[3][3];
#pragma unroll
    for (int j = 0; j < 9; ++j) b[j / 3][j % 3] = B[(int64_t)j * nip + q];
    const double pen[3] = {p0, p1, p2};
    // gamma = (constant + side 0's half) + side 1's half, in that order whichever rank holds which
    // side (a cross-rank interface adds the received half to its own: the same two sums, and a + b
    // is b + a): the same bits on every rank layout
    double g[3] = {0.0, 0.0, 0.0};
    for (int m = 0; m < C; ++m) g[m] = gcst[C * q + m];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        if (!(s ? own1 : own0)) continue;
        const IpSide& S = s ? s1 : s0;
        const double h = s ? -0.5 : 0.5;
        double l[3] = {0.0, 0.0, 0.0}, u[3] = {0.0, 0.0, 0.0};
#pragma unroll
        for (int a = 0; a < 4; ++a) {
            const double m = S.M[(int64_t)a * nip + q];
            const double* lp = W + S.lam[(int64_t)a * nip + q];
            const double* up = W + S.u[(int64_t)a * nip + q];
            l[0] += m * lp[0];
            if (C == 3) {
                l[1] += m * lp[1];
                l[2] += m * lp[2];
            }
            u[0] += m * up[0];
            u[1] += m * up[1];
            u[2] += m * up[2];
        }
        if (C == 1) {
            g[0] += h * (l[0] + pen[0] * (b[0][0] * u[0] + b[0][1] * u[1] + b[0][2] * u[2]));
        } else {
#pragma unroll
            for (int m = 0; m < 3; ++m)
                g[m] += h * ((b[m][0] * l[0] + b[m][1] * l[1] + b[m][2] * l[2]) +
                             pen[m] * (b[m][0] * u[0] + b[m][1] * u[1] + b[m][2] * u[2]));
        }
    }
    for (int m = 0; m < C; ++m) gamma[C * q + m] = g[m];
}

// y[dst[i]] += x[i]: the side-1 halves of rank-local interfaces onto their side-0 halves
__global__ void k_add_idx(double* y, const double* x, const int32_t* dst, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) y[dst[i]] += x[i];
}

// the projected traction in global components, T[3 q + k] = sum_m basis[m][k] gamma[3 q + m]
// (C = 1: T[q] = gamma[q]) -- what inteInpo's rows contract gamma with
__global__ void k_traction_ip(const double* B, const double* gamma, double* T, int C, int64_t nip) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nip) return;
    if (C == 1) {
        T[q] = gamma[q];
        return;
    }
    const double g0 = gamma[3 * q], g1 = gamma[3 * q + 1], g2 = gamma[3 * q + 2];
#pragma unroll
    for (int k = 0; k < 3; ++k)
        T[3 * q + k] = B[(int64_t)k * nip + q] * g0 + B[(int64_t)(3 + k) * nip + q] * g1 + B[(int64_t)(6 + k) * nip + q] * g2;
}

// out[C a + k] = sum over the ips q touching contact node a of coef (= sgn w_q M_a(q)) T[C q + k]:
// inteInpo gamma (MCONTACT.h:2671-2684) node-major; a contact node collects up to ~1000 ips on
// refined contact faces, so one wavefront per node splits its list over the lanes
__global__ __launch_bounds__(256) void k_inpo_node(const int64_t* ptr, const int32_t* iq, const double* coef,
                                                   const double* T, int C, int64_t nnc, double* out) {
    const int64_t a = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (a >= nnc) return;
    const int lane = threadIdx.x & 63;
    double v0 = 0.0, v1 = 0.0, v2 = 0.0;
    for (int64_t e = ptr[a] + lane; e < ptr[a + 1]; e += 64) {
        const double c = coef[e];
        const double* t = T + (int64_t)C * iq[e];
        v0 += c * t[0];
        if (C == 3) {
            v1 += c * t[1];
            v2 += c * t[2];
        }
    }
    v0 = wsum(v0);
    if (C == 3) {
        v1 = wsum(v1);
        v2 = wsum(v2);
    }
    if (lane == 0) {
        out[C * a] = v0;
        if (C == 3) {
            out[C * a + 1] = v1;
            out[C * a + 2] = v2;
        }
    }
}

// ---- batched Jacobi-PCG over the owned sides' surface mass systems.  Rows of all systems
// are concatenated, each padded to a multiple of 64 (ELL-64: chunk = 64 rows = one wave,
// lane = row, slot k at (off[c]+k)*64 + lane); per-system scalars live in PcgScal.
struct EllArgs {
    const int32_t* slots;
    const int64_t* off;
    const int32_t* col;
    const double* val;
    const int32_t* csys;
    const double* dinv;
    int64_t nch;
};

// r = b, x = 0, z = D^-1 b, p = q = 0; partials (b.z, b.b) per chunk
__global__ __launch_bounds__(256) void k_mcg_init(const double* b, const double* dinv, double* x, double* r, double* z,
                                                  double* p, double* q, double* partial, int64_t nrow) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= nrow) return;
    const double bi = b[i], zi = dinv[i] * bi;
    x[i] = 0.0;
    r[i] = bi;
    z[i] = zi;
    p[i] = 0.0;
    q[i] = 0.0;
    const double a = wsum(bi * zi), c = wsum(bi * bi);
    if ((threadIdx.x & 63) == 0) {
        partial[2 * (i >> 6)] = a;
        partial[2 * (i >> 6) + 1] = c;
    }
}

// q = A z + beta q, p = z + beta p; partial p.q per chunk
__global__ __launch_bounds__(256) void k_mcg_spmv(EllArgs e, const PcgScal* sc, const double* z, double* q, double* p,
                                                  double* partial, int ostride = 2) {
    const int64_t c = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (c >= e.nch) return;
    const int sys = e.csys[c];
    if (sc[sys].done) return;
    const int lane = threadIdx.x & 63;
    const int64_t row = c * 64 + lane;
    const int ns = e.slots[c];
    const int32_t* cp = e.col + e.off[c] * 64 + lane;
    const double* vp = e.val + e.off[c] * 64 + lane;
    double s = 0.0;
#pragma unroll 4
    for (int k = 0; k < ns; ++k) s += vp[(int64_t)k * 64] * z[cp[(int64_t)k * 64]];
    const double be = sc[sys].beta;
    const double qi = s + be * q[row], pi = z[row] + be * p[row];
    q[row] = qi;
    p[row] = pi;
    const double d = wsum(pi * qi);
    if (lane == 0) partial[ostride * c] = d;
}

// k_mcg_spmv over a batch whose second half repeats the first half's matrices R rows further on
// (the fused w|v interface update: both sides' v systems carry the w systems' inteMass): a wave
// takes chunk c and its twin c + nch2, reads the stored entries once and gathers z at j and j + R.
// Each row's sum runs over the same slots in the same order as in k_mcg_spmv, so q, p and the
// partials are bit for bit those of the unpaired launch; the matrix stream is halved.
__global__ __launch_bounds__(256) void k_mcg_spmv2(EllArgs e, const PcgScal* sc, const double* z, double* q, double* p,
                                                   double* partial, int ostride, int64_t R, int64_t nch2) {
    const int64_t c = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (c >= nch2) return;
    const int sw = e.csys[c], sv = e.csys[c + nch2];
    const bool dw = sc[sw].done != 0, dv = sc[sv].done != 0;
    if (dw && dv) return;
    const int lane = threadIdx.x & 63;
    const int64_t row = c * 64 + lane;
    const int ns = e.slots[c];
    const int32_t* cp = e.col + e.off[c] * 64 + lane;
    const double* vp = e.val + e.off[c] * 64 + lane;
    const double* zv = z + R;
    double s0 = 0.0, s1 = 0.0;
#pragma unroll 4
    for (int k = 0; k < ns; ++k) {
        const double v = vp[(int64_t)k * 64];
        const int32_t j = cp[(int64_t)k * 64];
        s0 += v * z[j];
        s1 += v * zv[j];
    }
    if (!dw) {
        const double be = sc[sw].beta;
        const double qi = s0 + be * q[row], pi = z[row] + be * p[row];
        q[row] = qi;
        p[row] = pi;
        const double d = wsum(pi * qi);
        if (lane == 0) partial[ostride * c] = d;
    }
    if (!dv) {
        const double be = sc[sv].beta;
        const int64_t rv = row + R;
        const double qi = s1 + be * q[rv], pi = z[rv] + be * p[rv];
        q[rv] = qi;
        p[rv] = pi;
        const double d = wsum(pi * qi);
        if (lane == 0) partial[ostride * (c + nch2)] = d;
    }
}

// k_mcg_axpy with alpha computed in place of a k_mcg_fin(kMcgAlpha) launch: every wave sums its
// system's p.q chunk partials (ppq, written by k_mcg_spmv with stride 1 -- not the (r.r, r.z)
// pairs this kernel writes) in one fixed order, so all waves hold the same alpha; the system's
// first chunk stores alpha / p.q and the breakdown flag as k_mcg_fin did.  On a breakdown (p.q
// not positive or not finite) every wave sees the same p.q and leaves x, r, z untouched, so x
// keeps the last good iterate as with the separate k_mcg_fin launch.  Every wave re-reads its
// system's partials (chunks^2 L2 reads per system), so MassBatch takes this form only up to
// kMcgFuseMaxChunks chunks (65,536 rows) per system; the headline's sides have up to ~300.
constexpr int64_t kMcgFuseMaxChunks = 1024;
__global__ __launch_bounds__(256) void k_mcg_axpy_fa(EllArgs e, PcgScal* sc, double* x, double* r, double* z,
                                                     const double* p, const double* q, double* partial,
                                                     const double* ppq, const int64_t* cb, PcgMirror* mirror) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t c = i >> 6;
    if (c >= e.nch) return;
    const int sys = e.csys[c];
    if (sc[sys].done) return;
    const int lane = threadIdx.x & 63;
    double pq = 0.0;
    for (int64_t k = cb[sys] + lane; k < cb[sys + 1]; k += 64) pq += ppq[k];
    pq = wsum(pq);
    const double al = sc[sys].delta / pq;
    const bool bad = !(pq > 0.0) || !isfinite(pq);  // the same in every wave of the system
    if (c == cb[sys] && lane == 0) {
        sc[sys].pq = pq;
        sc[sys].alpha = al;
        if (bad) {
            sc[sys].fail = 1;
            sc[sys].done = 1;
            mirror_store(mirror + sys, sc[sys].iter, 1, 1);
        }
    }
    if (bad) return;
    x[i] += al * p[i];
    const double ri = r[i] - al * q[i], zi = e.dinv[i] * ri;
    r[i] = ri;
    z[i] = zi;
    const double a = wsum(ri * ri), b = wsum(ri * zi);
    if (lane == 0) {
        partial[2 * c] = a;
        partial[2 * c + 1] = b;
    }
}

// x += alpha p, r -= alpha q, z = D^-1 r; partials (r.r, r.z) per chunk
__global__ __launch_bounds__(256) void k_mcg_axpy(EllArgs e, const PcgScal* sc, double* x, double* r, double* z,
                                                  const double* p, const double* q, double* partial) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t c = i >> 6;
    if (c >= e.nch) return;
    const int sys = e.csys[c];
    if (sc[sys].done) return;
    const double al = sc[sys].alpha;
    x[i] += al * p[i];
    const double ri = r[i] - al * q[i], zi = e.dinv[i] * ri;
    r[i] = ri;
    z[i] = zi;
    const double a = wsum(ri * ri), b = wsum(ri * zi);
    if ((threadIdx.x & 63) == 0) {
        partial[2 * c] = a;
        partial[2 * c + 1] = b;
    }
}

// ---- Chebyshev iteration on D^-1 M (MassBatch::cheb_; Saad, Iterative Methods, Alg. 12.1): a fixed
// number of steps from setup bounds of each system's spectrum, one launch per step, no reductions;
// the CG below then restarts from its iterate (k_mcg_restart) and usually finds it converged.
// x = 0, r = b, d = D^-1 b / theta_sys
__global__ __launch_bounds__(256) void k_mcheb_init(const double* b, const double* dinv, const double* ith,
                                                    const int32_t* csys, double* x, double* r, double* d, int64_t nrow) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= nrow) return;
    const double bi = b[i];
    x[i] = 0.0;
    r[i] = bi;
    d[i] = ith[csys[i >> 6]] * dinv[i] * bi;
}

// step k: x += d, r -= M d, dn = c1 d + c2 D^-1 r (coef[(k nsys + sys) 2 + {0, 1}]); systems whose
// step count kmax is reached keep their x, r.  The paired form (MassBatch::paired_) reads the
// shared matrix once for chunk c and its twin c + nch2, as k_mcg_spmv2.
template <bool PAIR>
__global__ __launch_bounds__(256) void k_mcheb_step(EllArgs e, const double* coef, const int32_t* kmax, int nsys, int k,
                                                    const double* d, double* dn, double* x, double* r, int64_t R,
                                                    int64_t nch_launch) {
    const int64_t c = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (c >= nch_launch) return;
    const int sw = e.csys[c];
    const int sv = PAIR ? e.csys[c + nch_launch] : sw;
    const bool aw = k < kmax[sw], av = PAIR && k < kmax[sv];
    if (!aw && !av) return;
    const int lane = threadIdx.x & 63;
    const int64_t row = c * 64 + lane;
    const int ns = e.slots[c];
    const int32_t* cp = e.col + e.off[c] * 64 + lane;
    const double* vp = e.val + e.off[c] * 64 + lane;
    double s0 = 0.0, s1 = 0.0;
#pragma unroll 4
    for (int q = 0; q < ns; ++q) {
        const double v = vp[(int64_t)q * 64];
        const int32_t j = cp[(int64_t)q * 64];
        s0 += v * d[j];
        if (PAIR) s1 += v * d[j + R];
    }
    auto upd = [&](int sys, int64_t i, double sum) {
        const double di = d[i];
        x[i] += di;
        const double ri = r[i] - sum;
        r[i] = ri;
        const double* cc = coef + 2 * ((int64_t)k * nsys + sys);
        dn[i] = cc[0] * di + cc[1] * e.dinv[i] * ri;
    };
    if (aw) upd(sw, row, s0);
    if (av) upd(sv, row + R, s1);
}

// CG restart from the Chebyshev iterate: z = D^-1 r, p = q = 0; partials (r.z, r.r) per chunk and
// b.b per chunk at bb (the stop rule stays relative to ||b||)
__global__ __launch_bounds__(256) void k_mcg_restart(const double* b, const double* dinv, const double* r, double* z,
                                                     double* p, double* q, double* partial, double* bbp, int64_t nrow) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= nrow) return;
    const double ri = r[i], zi = dinv[i] * ri, bi = b[i];
    z[i] = zi;
    p[i] = 0.0;
    q[i] = 0.0;
    const double a = wsum(ri * zi), c = wsum(ri * ri), d = wsum(bi * bi);
    if ((threadIdx.x & 63) == 0) {
        partial[2 * (i >> 6)] = a;
        partial[2 * (i >> 6) + 1] = c;
        bbp[i >> 6] = d;
    }
}

enum McgWhat { kMcgInit = 0, kMcgAlpha = 1, kMcgBeta = 2 };

// per-system scalars: one workgroup per system, fixed order over its chunks
__global__ __launch_bounds__(256) void k_mcg_fin(int what, const double* partial, const int64_t* cb, PcgScal* scv,
                                                 PcgMirror* mirror) {
    const int sys = blockIdx.x;
    PcgScal* sc = scv + sys;
    if (what != kMcgInit && sc->done) return;
    __shared__ double r0[4], r1[4];
    // four independent accumulator pairs per thread (loads in flight together), fixed order
    double av[4] = {0.0, 0.0, 0.0, 0.0}, bv[4] = {0.0, 0.0, 0.0, 0.0};
    const int64_t k1 = cb[sys + 1];
    for (int64_t k = cb[sys] + threadIdx.x; k < k1; k += 4 * 256) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int64_t q = k + 256 * u;
            if (q < k1) {
                av[u] += partial[2 * q];
                bv[u] += partial[2 * q + 1];
            }
        }
    }
    double a = wsum((av[0] + av[1]) + (av[2] + av[3]));
    double b = wsum((bv[0] + bv[1]) + (bv[2] + bv[3]));
    if ((threadIdx.x & 63) == 0) {
        r0[threadIdx.x >> 6] = a;
        r1[threadIdx.x >> 6] = b;
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    a = (r0[0] + r0[1]) + (r0[2] + r0[3]);
    b = (r1[0] + r1[1]) + (r1[2] + r1[3]);
    if (what == kMcgInit) {
        // x0 = 0: ||r0||^2 = b.b
        sc->delta = a;
        sc->bb = b;
        sc->rr = b;
        sc->tol2 = sc->tol2 * b;
        sc->beta = 0.0;
        sc->iter = 0;
        sc->fail = 0;
        sc->done = (b <= sc->tol2 || sc->maxit <= 0) ? 1 : 0;
        mirror_store(mirror + sys, 0, sc->done, 0);
    } else if (what == kMcgAlpha) {
        sc->pq = a;
        if (!(a > 0.0) || !isfinite(a)) {
            sc->fail = 1;
            sc->done = 1;
            mirror_store(mirror + sys, sc->iter, 1, 1);
        }
        sc->alpha = sc->delta / a;
    } else {
        sc->rr = a;
        sc->iter += 1;
        if (!isfinite(a) || !isfinite(b)) sc->fail = 1;
        if (sc->fail || a <= sc->tol2 || sc->iter >= sc->maxit) sc->done = 1;
        sc->beta = b / sc->delta;
        sc->delta = b;
        mirror_store(mirror + sys, sc->iter, sc->done, sc->fail);
    }
}

// the CG's scalars after k_mcg_restart: delta = r.z, rr = r.r, bb = b.b (one workgroup per system,
// a fixed order), tol2 scaled by b.b as k_mcg_fin's init does
__global__ __launch_bounds__(256) void k_mcg_fin_restart(const double* partial, const double* bbp, const int64_t* cb,
                                                         PcgScal* scv, PcgMirror* mirror) {
    const int sys = blockIdx.x;
    PcgScal* sc = scv + sys;
    __shared__ double r0[4], r1[4], r2[4];
    double a = 0.0, b = 0.0, c = 0.0;
    for (int64_t k = cb[sys] + threadIdx.x; k < cb[sys + 1]; k += 256) {
        a += partial[2 * k];
        b += partial[2 * k + 1];
        c += bbp[k];
    }
    a = wsum(a);
    b = wsum(b);
    c = wsum(c);
    if ((threadIdx.x & 63) == 0) {
        r0[threadIdx.x >> 6] = a;
        r1[threadIdx.x >> 6] = b;
        r2[threadIdx.x >> 6] = c;
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    a = (r0[0] + r0[1]) + (r0[2] + r0[3]);
    b = (r1[0] + r1[1]) + (r1[2] + r1[3]);
    c = (r2[0] + r2[1]) + (r2[2] + r2[3]);
    sc->delta = a;
    sc->bb = c;
    sc->rr = b;
    sc->tol2 = sc->tol2 * c;
    sc->beta = 0.0;
    sc->iter = 0;
    sc->fail = 0;
    sc->done = (b <= sc->tol2 || sc->maxit <= 0 || !(c > 0.0)) ? 1 : 0;
    if (!isfinite(a) || !isfinite(b)) {
        sc->fail = 1;
        sc->done = 1;
    }
    mirror_store(mirror + sys, 0, sc->done, sc->fail);
}

// All MONITOR pair norms of an iteration in two launches (instead of two per vector pair, 3.63 ->
// 3.40 ms interface step at the headline, profiles/r03ab): block b of k_pair_norms_all is block
// b - blk0[g] of segment g = bseg[b] (256 elements, the pair's squared difference and square), and
// k_reduce_pairs_all reduces segment g's blocks in one workgroup, a fixed order
struct NormSeg {
    const double* a;
    const double* o;
    int64_t n;
    int64_t blk0;  // first block of the segment in the batched grid
    int64_t nb;    // its blocks
    int64_t slot;  // moni slot (2 doubles)
};

__global__ void k_pair_norms_all(const NormSeg* seg, const int32_t* bseg, double* partial) {
    __shared__ double r1[4], r2[4];
    const NormSeg& S = seg[bseg[blockIdx.x]];
    const int64_t i = (int64_t)(blockIdx.x - S.blk0) * blockDim.x + threadIdx.x;
    double d = 0.0, s = 0.0;
    if (i < S.n) {
        const double ai = S.a[i], di = ai - S.o[i];
        d = di * di;
        s = ai * ai;
    }
    d = wsum(d);
    s = wsum(s);
    if ((threadIdx.x & 63) == 0) {
        r1[threadIdx.x >> 6] = d;
        r2[threadIdx.x >> 6] = s;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        partial[2 * blockIdx.x] = (r1[0] + r1[1]) + (r1[2] + r1[3]);
        partial[2 * blockIdx.x + 1] = (r2[0] + r2[1]) + (r2[2] + r2[3]);
    }
}

__global__ void k_reduce_pairs_all(const NormSeg* seg, const double* partial, double* moni) {
    __shared__ double r1[4], r2[4];
    const NormSeg& S = seg[blockIdx.x];
    const double* pp = partial + 2 * S.blk0;
    double d = 0.0, s = 0.0;
    for (int64_t k = threadIdx.x; k < S.nb; k += blockDim.x) {
        d += pp[2 * k];
        s += pp[2 * k + 1];
    }
    d = wsum(d);
    s = wsum(s);
    if ((threadIdx.x & 63) == 0) {
        r1[threadIdx.x >> 6] = d;
        r2[threadIdx.x >> 6] = s;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        moni[S.slot] = (r1[0] + r1[1]) + (r1[2] + r1[3]);
        moni[S.slot + 1] = (r2[0] + r2[1]) + (r2[2] + r2[3]);
    }
}

// ---- interface-eliminated coarse-space correction (MCONTACT.h:2578-2612)
// y[r] = sum_k val[k] W[col[k]] + add[r]: one wavefront per row (coarse rows are long:
// thousands of surface entries each)
__global__ __launch_bounds__(256) void k_csr_wave(const int64_t* ptr, const int32_t* col, const double* val,
                                                  int64_t nrow, const double* W, double* y, const double* add) {
    const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= nrow) return;
    const int lane = threadIdx.x & 63;
    double s = 0.0;
    for (int64_t k = ptr[r] + lane; k < ptr[r + 1]; k += 64) s += val[k] * W[col[k]];
    s = wsum(s);
    if (lane == 0) y[r] = add[r] + s;
}

// g[r] = the row's per-source slots in ascending source order (build_coarse)
__global__ void k_slot_sum(const int64_t* sptr, const double* gs, double* g, int64_t n) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    double s = 0.0;
    for (int64_t k = sptr[r]; k < sptr[r + 1]; ++k) s += gs[k];
    g[r] = s;
}

// g[rows[i]] -= yd[src[i]]: the stiffness part of globTran_D_1 u, restricted on the device
__global__ void k_cs_kpart(const int32_t* rows, const int64_t* src, const double* yd, double* g, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) g[rows[i]] -= yd[src[i]];
}

// x[i] = sum_j A[i n + j] g[j]: one wavefront per row of the owned block of globCoup_1^-1
__global__ __launch_bounds__(256) void k_gemv_wave(const double* A, const double* g, double* x, int64_t m, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= m) return;
    const int lane = threadIdx.x & 63;
    const double* a = A + i * n;
    double s = 0.0;
    for (int64_t j = lane; j < n; j += 64) s += a[j] * g[j];
    s = wsum(s);
    if (lane == 0) x[i] = s;
}

// xn = C_d^T xc: nodal level-d values of the owned subdomains (constrained dofs 0)
__global__ void k_cs_scatter(const int32_t* src, const double* xc, double* xn, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) xn[i] = src[i] >= 0 ? xc[src[i]] : 0.0;
}

// u += OUTP_SUB1(accuProl xc): free dofs get (Q (x) I3) xn, constrained dofs their prescribed
// value again (MCONTACT.h:2606-2608 adds OUTP_SUB1's output, Dirichlet values included).
// One thread per batch fine node in the reference order; Q slot-major, <= 8 parents.
__global__ void k_cs_prolong(const int32_t* qcol, const double* qw, int64_t nn, const double* xn, const uint8_t* flag,
                             const double* presc, double* u) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nn) return;
    double e0 = 0.0, e1 = 0.0, e2 = 0.0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int32_t c = qcol[(int64_t)k * nn + i];
        if (c < 0) break;
        const double w = qw[(int64_t)k * nn + i];
        e0 += w * xn[c];
        e1 += w * xn[c + 1];
        e2 += w * xn[c + 2];
    }
    const double e[3] = {e0, e1, e2};
    for (int a = 0; a < 3; ++a) {
        const int64_t d = 3 * i + a;
        u[d] += flag[d] ? e[a] : presc[d];
    }
}

// assembled accuProl (operator-level builder): u[tgt[r]] += sum_k val[k] xc[col[k]] over the owned
// subdomains' fine free dofs (one row per thread), then u[cdof[i]] += presc[cdof[i]] on the
// constrained dofs (OUTP_SUB1 writes their prescribed values again, MCONTACT.h:2606-2608)
__global__ void k_cs_prolong_csr(const int64_t* ptr, const int32_t* col, const double* val, const int32_t* tgt,
                                 const double* xc, double* u, int64_t nrow) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nrow) return;
    double s = 0.0;
    for (int64_t k = ptr[r]; k < ptr[r + 1]; ++k) s += val[k] * xc[col[k]];
    u[tgt[r]] += s;
}

__global__ void k_cs_presc(const int32_t* cdof, const double* presc, double* u, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) u[cdof[i]] += presc[cdof[i]];
}

// coarse right-hand side into the coarse MGPIS's fine layout / its solution back to the own rows
__global__ void k_perm_scatter(const int32_t* perm, const double* g, double* b, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) b[perm[i]] = g[i];
}

__global__ void k_perm_gather(const int32_t* perm, const int32_t* rows, const double* x, double* xc, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) xc[i] = x[perm[rows[i]]];
}

// potri(lower) on the column-major view leaves the inverse in the row-major upper triangle;
// mirror it into the lower one
__global__ void k_fill_lower(double* A, int64_t n) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= n * n) return;
    const int64_t i = idx / n, j = idx % n;
    if (j < i) A[i * n + j] = A[j * n + i];
}

// Fused interface update (penalty mass operators proportional to the plain ones, rho = penN =
// penF): with w = M^-1 T^T u and v = M^-1 I gamma from one batched solve,
//   aux = (rho M)^-1 (rho T^T u + M lambda + I gamma) = w + (lambda + v) / rho   (MCONTACT.h:2671-2684)
//   lambda += M^-1 (rho T^T u - rho M aux)             = -v                      (2689-2704)
__global__ void k_fuse_aux_lambda(double* state, const double* wv, const double* rinv, int64_t R) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= R) return;
    const double w = wv[i], v = wv[R + i];
    state[i] = w + (state[R + i] + v) * rinv[i];
    state[R + i] = -v;
}

inline int nb256(int64_t n) { return (int)std::max<int64_t>(1, (n + 255) / 256); }

// Row lists -> SELL-64 (rows padded to a multiple of 64; padding slots: column 0, value 0).
using Rows = std::vector<std::vector<std::pair<int64_t, double>>>;

struct SellOp {
    int64_t nrow = 0, nch = 0;
    DevBuf<int32_t> slots, col;
    DevBuf<int64_t> off;
    DevBuf<double> val;
    // algorithmic bytes of one apply: the stored entries (8 B value + 4 B column), each distinct
    // gathered W entry once, every real row written once (an `add` operand adds 8 B per row)
    double bytes = 0.0;
    void build(const Rows& rows) {
        nrow = pad64((int64_t)rows.size());
        nch = nrow / 64;
        std::vector<int32_t> sl(std::max<int64_t>(nch, 1), 0);
        std::vector<int64_t> of(nch + 1, 0);
        for (int64_t c = 0; c < nch; ++c) {
            size_t mx = 0;
            for (int64_t r = c * 64; r < std::min<int64_t>((int64_t)rows.size(), (c + 1) * 64); ++r) mx = std::max(mx, rows[r].size());
            sl[c] = (int32_t)mx;
            of[c + 1] = of[c] + (int64_t)mx;
        }
        std::vector<int32_t> co(std::max<int64_t>(of[nch] * 64, 1), 0);
        std::vector<double> va(std::max<int64_t>(of[nch] * 64, 1), 0.0);
        for (int64_t r = 0; r < (int64_t)rows.size(); ++r) {
            const int64_t c = r / 64, lane = r % 64;
            for (size_t k = 0; k < rows[r].size(); ++k) {
                if (rows[r][k].first > INT32_MAX) throw ApiError(DDPCA_EINVAL, "workspace index exceeds int32");
                co[(of[c] + (int64_t)k) * 64 + lane] = (int32_t)rows[r][k].first;
                va[(of[c] + (int64_t)k) * 64 + lane] = rows[r][k].second;
            }
        }
        slots.upload(sl);
        off.upload(of);
        col.upload(co);
        val.upload(va);
        int64_t ent = 0;
        std::vector<int64_t> cols;
        for (const auto& r : rows) {
            ent += (int64_t)r.size();
            for (const auto& e : r) cols.push_back(e.first);
        }
        std::sort(cols.begin(), cols.end());
        const int64_t uniq = (int64_t)(std::unique(cols.begin(), cols.end()) - cols.begin());
        bytes = 12.0 * (double)ent + 8.0 * (double)uniq + 8.0 * (double)rows.size();
    }
    void apply(hipStream_t s, const double* W, double* y, const double* add) const {
        if (nch) hipLaunchKernelGGL(k_sell_w, dim3(ceil_div(nch, 4)), dim3(256), 0, s, slots.p, off.p, col.p, val.p, nch, W, y, add);
    }
};

// DDPCA_STREAMS=1: the batched PCG and the mass CG on one stream each (A/B runs); default two
bool two_streams() {
    const char* v = std::getenv("DDPCA_STREAMS");
    return !(v && v[0] == '1');
}

// scs[h][i] = sc[i] with done forced on the other half's systems / sc[i] = its half's copy
__global__ void k_scal_split(const PcgScal* sc, PcgScal* scs, const int32_t* half, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    for (int h = 0; h < 2; ++h) {
        PcgScal v = sc[i];
        if (half[i] != h) v.done = 1;
        scs[h * n + i] = v;
    }
}
__global__ void k_scal_merge(PcgScal* sc, const PcgScal* scs, const int32_t* half, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) sc[i] = scs[half[i] * n + i];
}

// Extreme eigenvalues of D^-1 M for an SPD CSR M (MassBatch's Chebyshev steps): Lanczos on the
// symmetric D^-1/2 M D^-1/2 (m steps from a fixed start vector), Ritz extremes by bisection on
// the tridiagonal (Sturm counts); *gersh = max_i sum_j |M_ij| / M_ii, an upper bound
void mass_spectrum(const Csr& M, int m, double* lmin, double* lmax, double* gersh) {
    const int64_t n = M.nrow;
    std::vector<double> dis(n, 0.0);
    double g = 0.0;
    for (int64_t r = 0; r < n; ++r) {
        double dg = 0.0, sa = 0.0;
        for (int64_t k = M.ptr[r]; k < M.ptr[r + 1]; ++k) {
            sa += std::abs(M.val[k]);
            if (M.col[k] == r) dg = M.val[k];
        }
        dis[r] = dg > 0.0 ? 1.0 / std::sqrt(dg) : 0.0;
        if (dg > 0.0) g = std::max(g, sa / dg);
    }
    *gersh = g;
    m = (int)std::min<int64_t>(m, n);
    std::vector<double> v(n), vp(n, 0.0), w(n), alpha, beta;
    double nv = 0.0;
    for (int64_t i = 0; i < n; ++i) v[i] = 1.0 + 0.5 * std::sin(0.7 * (double)i + 0.3), nv += v[i] * v[i];
    nv = std::sqrt(nv);
    for (double& x : v) x /= nv;
    double bprev = 0.0;
    for (int j = 0; j < m; ++j) {
        for (int64_t r = 0; r < n; ++r) {
            double acc = 0.0;
            for (int64_t k = M.ptr[r]; k < M.ptr[r + 1]; ++k) acc += M.val[k] * dis[M.col[k]] * v[M.col[k]];
            w[r] = dis[r] * acc - bprev * vp[r];
        }
        double a = 0.0;
        for (int64_t r = 0; r < n; ++r) a += w[r] * v[r];
        double b = 0.0;
        for (int64_t r = 0; r < n; ++r) {
            w[r] -= a * v[r];
            b += w[r] * w[r];
        }
        b = std::sqrt(b);
        alpha.push_back(a);
        if (j + 1 == m || !(b > 1e-14)) break;
        beta.push_back(b);
        for (int64_t r = 0; r < n; ++r) {
            vp[r] = v[r];
            v[r] = w[r] / b;
        }
        bprev = b;
    }
    const int t = (int)alpha.size();
    auto count_below = [&](double x) {  // eigenvalues of T below x (Sturm sequence)
        int c = 0;
        double q = alpha[0] - x;
        if (q < 0) ++c;
        for (int i = 1; i < t; ++i) {
            const double qq = std::abs(q) < 1e-300 ? 1e-300 : q;
            q = alpha[i] - x - beta[i - 1] * beta[i - 1] / qq;
            if (q < 0) ++c;
        }
        return c;
    };
    double lo = 0.0, hi = 0.0;
    for (int i = 0; i < t; ++i) {
        const double rad = (i > 0 ? std::abs(beta[i - 1]) : 0.0) + (i + 1 < t ? std::abs(beta[i]) : 0.0);
        lo = std::min(lo, alpha[i] - rad);
        hi = std::max(hi, alpha[i] + rad);
    }
    auto kth = [&](int k) {  // the k-th smallest eigenvalue (0-based)
        double a = lo, b = hi;
        for (int it = 0; it < 200; ++it) {
            const double mid = 0.5 * (a + b);
            if (count_below(mid) > k) b = mid;
            else a = mid;
        }
        return 0.5 * (a + b);
    };
    *lmin = kth(0);
    *lmax = kth(t - 1);
}

// Batched surface-mass solver: one graph of `k` CG iterations over every system, replayed
// until every system reports done through the host-mapped mirror.  Chebyshev mode (cheb_, the
// default where every system's steps fit kChebMax): a fixed-length Chebyshev iteration first, one
// launch per step, then the CG from its iterate -- usually converged at its first check.
constexpr int64_t kChebMax = 120;
class MassBatch {
public:
    int nsys = 0;
    int64_t nrow = 0, nch = 0;
    DevBuf<int32_t> slots, col, csys;
    DevBuf<int64_t> off, cb;
    DevBuf<double> val, dinv, b, x, r, z, p, q, partial;
    DevBuf<PcgScal> sc;
    PcgScal* sc_host = nullptr;
    MirrorBuf mirror;
    int64_t k = 8;
    int64_t last_iters = 0;
    double alg_bytes = 0.0;  // accumulated by check(): init + iterations of every system
    // Chebyshev mode: spectral bounds per system from build(), steps from the first solve's rtol
    bool cheb_ = false;
    int64_t cheb_k_ = 0;                       // steps of the captured Chebyshev graph (max over systems)
    std::vector<double> lam_lo_, lam_hi_;      // D^-1 M spectrum bounds used, per system
    std::vector<int32_t> cheb_ks_;             // steps per system

    // A[i] = system i (rows m_i), placed at rows roff[i] (multiples of 64) of nrow_total.
    void build(const std::vector<const Csr*>& A, const std::vector<int64_t>& roff, int64_t nrow_total) {
        nsys = (int)A.size();
        nrow = nrow_total;
        nch = nrow / 64;
        std::vector<int32_t> sl(std::max<int64_t>(nch, 1), 0), cs(std::max<int64_t>(nch, 1), 0);
        std::vector<int64_t> of(nch + 1, 0), c0(nsys + 1, nch);
        std::vector<double> di(std::max<int64_t>(nrow, 1), 0.0);
        for (int s = 0; s < nsys; ++s) {
            const Csr& M = *A[s];
            c0[s] = roff[s] / 64;
            for (int64_t c = roff[s] / 64; c < (roff[s] + pad64(M.nrow)) / 64; ++c) {
                cs[c] = s;
                int64_t mx = 0;
                for (int64_t r = (c * 64 - roff[s]); r < std::min(M.nrow, c * 64 - roff[s] + 64); ++r)
                    mx = std::max(mx, M.ptr[r + 1] - M.ptr[r]);
                sl[c] = (int32_t)mx;
            }
        }
        for (int64_t c = 0; c < nch; ++c) of[c + 1] = of[c] + sl[c];
        std::vector<int32_t> co(std::max<int64_t>(of[nch] * 64, 1), 0);
        std::vector<double> va(std::max<int64_t>(of[nch] * 64, 1), 0.0);
        for (int64_t c = 0; c < nch; ++c)
            for (int64_t q2 = of[c]; q2 < of[c + 1]; ++q2)
                for (int lane = 0; lane < 64; ++lane) co[q2 * 64 + lane] = (int32_t)(c * 64 + lane);  // pad: self, 0
        for (int s = 0; s < nsys; ++s) {
            const Csr& M = *A[s];
            for (int64_t r0 = 0; r0 < M.nrow; ++r0) {
                const int64_t g = roff[s] + r0, c = g / 64, lane = g % 64;
                for (int64_t k2 = M.ptr[r0]; k2 < M.ptr[r0 + 1]; ++k2) {
                    const int64_t q2 = of[c] + (k2 - M.ptr[r0]);
                    co[q2 * 64 + lane] = (int32_t)(roff[s] + M.col[k2]);
                    va[q2 * 64 + lane] = M.val[k2];
                    if (M.col[k2] == r0) di[g] = 1.0 / M.val[k2];
                }
            }
        }
        // paired batch: systems i and i + nsys/2 share one matrix, R = nrow/2 rows apart
        paired_ = nsys >= 2 && nsys % 2 == 0 && nrow % 128 == 0;
        for (int s = 0; paired_ && s < nsys / 2; ++s)
            paired_ = A[s] == A[s + nsys / 2] && roff[s + nsys / 2] == roff[s] + nrow / 2;
        slots.upload(sl);
        csys.upload(cs);
        off.upload(of);
        col.upload(co);
        val.upload(va);
        dinv.upload(di);
        cb.upload(c0);
        cb_host_ = c0;
        // algorithmic bytes per system: init (b, D^-1 read; x r z p q written: 56 B per row) and
        // per CG iteration -- k_mcg_spmv: stored entries (12 B), z gathered once, z, q, p read
        // and q, p written; k_mcg_axpy: x, r read + written, z written, p, q, D^-1 read (112 B per row)
        init_bytes_.assign(nsys, 0.0);
        it_bytes_.assign(nsys, 0.0);
        mat_bytes_.assign(nsys, 0.0);
        for (int s = 0; s < nsys; ++s) {
            const double rows = (double)A[s]->nrow, ent = (double)A[s]->nnz();
            init_bytes_[s] = 56.0 * rows;
            // (+ the p.q and (r.r, r.z) chunk partials written once and read once: 24 B each way per chunk)
            it_bytes_[s] = 8.0 * rows + 40.0 * rows + 64.0 * rows + 48.0 * (double)(pad64(A[s]->nrow) / 64);
            mat_bytes_[s] = 12.0 * ent;  // (k_mcg_spmv2: once per pair, for the pair's longer solve)
        }
        for (auto* v : {&b, &x, &r, &z, &p, &q}) {
            v->alloc(std::max<int64_t>(nrow, 2));
            v->zero();
        }
        partial.alloc(3 * std::max<int64_t>(nch, 1));  // (a, b) pairs + the fused form's p.q
        sc.alloc(std::max(nsys, 1));
        // Chebyshev bounds: [0.9 Ritz min, min(Gershgorin, 1.05 Ritz max)] of D^-1 M after 60 Lanczos
        // steps (the CG that follows the fixed step count repairs an estimate that was off);
        // DDPCA_MASS_CHEB=0 keeps the plain CG
        const char* ce = std::getenv("DDPCA_MASS_CHEB");
        cheb_ = !(ce && ce[0] == '0') && nsys > 0;
        lam_lo_.assign(nsys, 0.0);
        lam_hi_.assign(nsys, 0.0);
        if (cheb_) {
            std::vector<double> lo(nsys), hi(nsys), gh(nsys);
#pragma omp parallel for schedule(dynamic, 1)
            for (int s2 = 0; s2 < nsys; ++s2) mass_spectrum(*A[s2], 60, &lo[s2], &hi[s2], &gh[s2]);
            for (int s2 = 0; s2 < nsys; ++s2) {
                lam_lo_[s2] = 0.9 * lo[s2];
                lam_hi_[s2] = std::min(gh[s2], 1.05 * hi[s2]);
                if (!(lam_lo_[s2] > 0.0) || !(lam_hi_[s2] > lam_lo_[s2])) cheb_ = false;
            }
        }
        // the ADMM loop's tolerance planned here, at setup: solve() uploads nothing while other
        // in-process ranks may be capturing graphs
        if (cheb_) cheb_plan(1.0e-14);
        DDPCA_HIP(hipHostMalloc(reinterpret_cast<void**>(&sc_host), std::max(nsys, 1) * sizeof(PcgScal)));
        mirror.alloc(nsys);
    }
    ~MassBatch() {
        if (s2_) (void)hipStreamSynchronize(s2_);
        drop_graphs();
        if (ev_fork_) (void)hipEventDestroy(ev_fork_);
        if (ev_join_) (void)hipEventDestroy(ev_join_);
        if (s2_) (void)hipStreamDestroy(s2_);
        if (sc_host) (void)hipHostFree(sc_host);
    }

    // x_out (nrow) = A^-1 b.  Asynchronous on `s` except for the host pacing of replays.
    void solve(hipStream_t s, double* x_out, double rtol, int64_t maxit) {
        if (nsys == 0) return;
        solved_ = true;
        if (x_out != x_target_) {
            drop_graphs();
            x_target_ = x_out;
        }
        if (cheb_ && rtol != cheb_rtol_) {
            // a tolerance other than the setup plan's (1e-14, the ADMM loop's): re-plan and
            // re-capture here -- the capture holds the library's capture lock (device_common.hpp)
            drop_graphs();
            cheb_plan(rtol);
        }
        if (!graph_) capture(s);
        mirror.reset();  // the previous solve on `s` was paced to completion before this point
        for (int i = 0; i < nsys; ++i) {
            sc_host[i] = PcgScal{};
            sc_host[i].tol2 = rtol * rtol;
            sc_host[i].maxit = maxit;
        }
        DDPCA_HIP(hipMemcpyAsync(sc.p, sc_host, nsys * sizeof(PcgScal), hipMemcpyHostToDevice, s));
        // Chebyshev mode: the fixed-length Chebyshev graph, then the CG restarted from its iterate
        // (the host launches CG replays only once the mirror says a system is not done, or the
        // stream drained); else x0 = 0 (warm starts from the previous ADMM iteration's solution:
        // 39.3 -> 37.1 mass-CG iterations at the headline, no measurable gain, profiles/r03v)
        int64_t launched0 = 0;
        cheb_used_ = cheb_ && cgraph_;
        if (cheb_used_) {
            DDPCA_HIP(hipGraphLaunch(cgraph_, s));
            launched0 = k + 1;
        } else {
            hipLaunchKernelGGL(k_mcg_init, dim3(nb256(nrow)), dim3(256), 0, s, b.p, dinv.p, x_out, r.p, z.p, p.p, q.p,
                               partial.p, nrow);
            hipLaunchKernelGGL(k_mcg_fin, dim3(nsys), dim3(256), 0, s, (int)kMcgInit, partial.p, cb.p, sc.p, mirror.dev);
        }
        if (split_) {
            // fork into the two halves' streams, pace both, join and merge the scalars back
            hipLaunchKernelGGL(k_scal_split, dim3(ceil_div(nsys, 64)), dim3(64), 0, s, sc.p, sc_half_.p, half_.p, nsys);
            DDPCA_HIP(hipEventRecord(ev_fork_, s));
            DDPCA_HIP(hipStreamWaitEvent(s2_, ev_fork_, 0));
            hipStream_t st[2] = {s, s2_};
            const int64_t hz[2] = {horizon(0), horizon(1)};
            pace_halves(st, graph_h_, mirror, half_host_, k, launched0, graph1_h_, hz);
            DDPCA_HIP(hipEventRecord(ev_join_, s2_));
            DDPCA_HIP(hipStreamWaitEvent(s, ev_join_, 0));
            hipLaunchKernelGGL(k_scal_merge, dim3(ceil_div(nsys, 64)), dim3(64), 0, s, sc.p, sc_half_.p, half_.p, nsys);
            return;
        }
        pace_until_done(s, graph_, mirror, k, launched0, graph1_, horizon(-1));
    }

    // capture the solve's graphs now (create time, one thread) for solves into x_out: the first
    // solve of an in-process rank then captures nothing while the other rank threads run
    void prepare(hipStream_t s, double* x_out) {
        if (nsys == 0) return;
        if (x_out != x_target_) {
            drop_graphs();
            x_target_ = x_out;
        }
        if (!graph_) capture(s);
    }

    // Two-stream split of the systems (as MgpisDevice::set_split): two halves of equal rows, each
    // half's CG iterations a graph of its own on its own stream, on a copy of the scalars where
    // the other half's systems are done -- the latency-bound launches of the two halves overlap.
    void set_split(bool on) {
        on = on && nsys >= 2;
        if (on && !s2_) {
            DDPCA_HIP(hipStreamCreateWithFlags(&s2_, hipStreamNonBlocking));
            DDPCA_HIP(hipEventCreateWithFlags(&ev_fork_, hipEventDisableTiming));
            DDPCA_HIP(hipEventCreateWithFlags(&ev_join_, hipEventDisableTiming));
            sc_half_.alloc(2 * nsys);
            // a paired batch splits by pairs, so that a pair's shared matrix is read by one half
            const int nu = paired_ ? nsys / 2 : nsys;
            std::vector<int64_t> rows(nu, 0);
            std::vector<int> ord(nu);
            for (int i = 0; i < nsys; ++i) rows[i % nu] += cb_host_[i + 1] - cb_host_[i];
            for (int i = 0; i < nu; ++i) ord[i] = i;
            std::stable_sort(ord.begin(), ord.end(), [&](int a, int c) { return rows[a] > rows[c]; });
            half_host_.assign(nsys, 0);
            int64_t w[2] = {0, 0};
            for (int i : ord) {
                const int h = w[1] < w[0] ? 1 : 0;
                for (int j = i; j < nsys; j += nu) half_host_[j] = h;
                w[h] += rows[i];
            }
            half_.upload(half_host_);
        }
        if (on != split_) drop_graphs();
        split_ = on;
    }

    // alpha inside k_mcg_axpy_fa: default while every system has at most kMcgFuseMaxChunks chunks
    // (each wave re-reads its system's p.q partials); DDPCA_MCG_FUSE_ALPHA=0 forces the separate
    // k_mcg_fin launch, =1 the fused form at any size (read at graph capture)
    int fuse_override = -1;  // ddpca_mass_solve: 0 / 1 forces the form (tests), -1 the rule below
    bool fuse_alpha() const {
        if (fuse_override >= 0) return fuse_override != 0;
        const char* ef = std::getenv("DDPCA_MCG_FUSE_ALPHA");
        if (ef && std::atoi(ef) == 0) return false;
        if (ef && std::atoi(ef) == 1) return true;
        for (int s = 0; s < nsys; ++s)
            if (cb_host_[s + 1] - cb_host_[s] > kMcgFuseMaxChunks) return false;
        return true;
    }

    // after the stream synchronised: iterations of the last solve, breakdown check
    void check() {
        last_iters = 0;
        expect_.resize(nsys);
        for (int i = 0; i < nsys; ++i) {
            if (mirror.host[i].fail) {
                solved_ = false;
                throw ApiError(DDPCA_ENUMERIC, "surface mass CG breakdown in system " + std::to_string(i));
            }
            expect_[i] = mirror.host[i].iter;  // paces the next solve's tail
            const int64_t ck = cheb_used_ ? (int64_t)cheb_ks_[i] : 0;
            last_iters = std::max<int64_t>(last_iters, mirror.host[i].iter + ck);
            if (solved_) {
                int64_t mit = mirror.host[i].iter;
                if (pair_used_) mit = i < nsys / 2 ? std::max(mit, mirror.host[i + nsys / 2].iter) : 0;
                alg_bytes += init_bytes_[i] + (double)mirror.host[i].iter * it_bytes_[i] + (double)mit * mat_bytes_[i];
                // Chebyshev: init (b, D^-1 read; x, r, d written) + per step (d gathered once, read;
                // x, r read + written; D^-1 read; d' written: 56 B per row) + the matrix once per
                // pair + the restart (b, r, D^-1 read; z, p, q written)
                if (cheb_used_)
                    alg_bytes += init_bytes_[i] * (40.0 / 56.0) + (double)ck * (it_bytes_[i] * (56.0 / 112.0)) +
                                 (pair_used_ ? (i < nsys / 2 ? (double)ck * mat_bytes_[i] : 0.0) : (double)ck * mat_bytes_[i]) +
                                 init_bytes_[i] * (48.0 / 56.0);
            }
        }
        solved_ = false;
    }

private:
    hipGraphExec_t graph_ = nullptr;
    hipGraphExec_t graph_h_[2] = {nullptr, nullptr};
    // one-iteration graphs for the tail (MgpisDevice::graph1_): past the systems' previous
    // iteration counts the host queues single iterations two ahead of the slowest system
    hipGraphExec_t graph1_ = nullptr;
    hipGraphExec_t graph1_h_[2] = {nullptr, nullptr};
    std::vector<int64_t> expect_;
    int64_t horizon(int half) const {
        const char* e = std::getenv("DDPCA_TAIL_PACING");
        if ((e && std::atoi(e) == 0) || (int)expect_.size() != nsys) return INT64_MAX;
        int64_t h = 0;
        for (int i = 0; i < nsys; ++i) {
            if (half >= 0 && half_host_[i] != half) continue;
            if (expect_[i] <= 0) return INT64_MAX;
            h = std::max(h, expect_[i]);
        }
        return h;
    }
    void drop_graphs() {
        for (hipGraphExec_t* g : {&graph_h_[0], &graph_h_[1], &graph1_h_[0], &graph1_h_[1], &graph1_, &cgraph_}) {
            if (*g) (void)hipGraphExecDestroy(*g);
            *g = nullptr;
        }
        if (graph_ && !split_) (void)hipGraphExecDestroy(graph_);  // (split: graph_ aliases graph_h_[0])
        graph_ = nullptr;
    }
    double* x_target_ = nullptr;
    hipGraphExec_t cgraph_ = nullptr;  // Chebyshev: init, steps, CG restart
    double cheb_rtol_ = -1.0;
    bool cheb_used_ = false;
    DevBuf<double> ccoef_, cith_;
    DevBuf<int32_t> ckmax_;
    // the step counts and coefficients for a relative residual rtol: per system kappa = hi / lo,
    // K = ceil(ln(4 sqrt(kappa) / rtol) / ln sigma), sigma = (sqrt(kappa) + 1) / (sqrt(kappa) - 1)
    // (the residual bound 2 sqrt(kappa) sigma^-K at half of rtol); none past kChebMax
    void cheb_plan(double rtol) {
        cheb_rtol_ = rtol;
        cheb_ks_.assign(nsys, 0);
        int64_t K = 0;
        for (int s2 = 0; s2 < nsys; ++s2) {
            const double kap = lam_hi_[s2] / lam_lo_[s2], sk = std::sqrt(kap);
            const double sig = (sk + 1.0) / (sk - 1.0);
            const int64_t ks = (int64_t)std::ceil(std::log(4.0 * sk / rtol) / std::log(sig));
            cheb_ks_[s2] = (int32_t)std::max<int64_t>(1, ks);
            K = std::max<int64_t>(K, cheb_ks_[s2]);
        }
        cheb_k_ = K;
        // past kChebMax steps this tolerance runs the plain CG (capture() skips the Chebyshev
        // graph); cheb_ stays set, so a later solve at a looser tolerance plans it again
        if (K > kChebMax) return;
        std::vector<double> coef((size_t)2 * K * nsys, 0.0), ith(nsys);
        for (int s2 = 0; s2 < nsys; ++s2) {
            const double th = 0.5 * (lam_hi_[s2] + lam_lo_[s2]), de = 0.5 * (lam_hi_[s2] - lam_lo_[s2]);
            const double s1 = th / de;
            ith[s2] = 1.0 / th;
            double rho = 1.0 / s1;
            for (int64_t kk = 0; kk < K; ++kk) {
                const double rn = 1.0 / (2.0 * s1 - rho);
                coef[2 * (kk * nsys + s2)] = rn * rho;
                coef[2 * (kk * nsys + s2) + 1] = 2.0 * rn / de;
                rho = rn;
            }
        }
        ccoef_.upload(coef);
        cith_.upload(ith);
        ckmax_.upload(cheb_ks_);
    }
    bool split_ = false;
    hipStream_t s2_ = nullptr;
    hipEvent_t ev_fork_ = nullptr, ev_join_ = nullptr;
    DevBuf<PcgScal> sc_half_;
    DevBuf<int32_t> half_;
    std::vector<int> half_host_;
    std::vector<int64_t> cb_host_;
    std::vector<double> init_bytes_, it_bytes_, mat_bytes_;
    bool solved_ = false;
    bool paired_ = false, pair_used_ = false;
    void capture(hipStream_t s) {
        if (cheb_ && cheb_k_ > 0 && cheb_k_ <= kChebMax) capture_cheb(s);
        if (split_) {
            capture_one(s, sc_half_.p, &graph_h_[0], k);
            capture_one(s, sc_half_.p + nsys, &graph_h_[1], k);
            if (k > 1) {
                capture_one(s, sc_half_.p, &graph1_h_[0], 1);
                capture_one(s, sc_half_.p + nsys, &graph1_h_[1], 1);
            }
            graph_ = graph_h_[0];  // marks the capture done (destroyed through graph_h_)
            return;
        }
        capture_one(s, sc.p, &graph_, k);
        if (k > 1) capture_one(s, sc.p, &graph1_, 1);
    }
    void capture_cheb(hipStream_t s) {
        EllArgs e{slots.p, off.p, col.p, val.p, csys.p, dinv.p, nch};
        const char* ep = std::getenv("DDPCA_MCG_PAIR");
        const bool pair = paired_ && !(ep && std::atoi(ep) == 0);
        hipGraph_t g;
        CaptureSection capture_section;  // device_common.hpp CaptureLock
        DDPCA_HIP(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        hipLaunchKernelGGL(k_mcheb_init, dim3(nb256(nrow)), dim3(256), 0, s, b.p, dinv.p, cith_.p, csys.p, x_target_, r.p,
                           z.p, nrow);
        double* d[2] = {z.p, p.p};
        for (int64_t kk = 0; kk < cheb_k_; ++kk) {
            const double* din = d[kk & 1];
            double* dout = d[(kk + 1) & 1];
            if (pair)
                hipLaunchKernelGGL(k_mcheb_step<true>, dim3(ceil_div(nch / 2, 4)), dim3(256), 0, s, e, ccoef_.p, ckmax_.p,
                                   nsys, (int)kk, din, dout, x_target_, r.p, nrow / 2, nch / 2);
            else
                hipLaunchKernelGGL(k_mcheb_step<false>, dim3(ceil_div(nch, 4)), dim3(256), 0, s, e, ccoef_.p, ckmax_.p,
                                   nsys, (int)kk, din, dout, x_target_, r.p, (int64_t)0, nch);
        }
        hipLaunchKernelGGL(k_mcg_restart, dim3(nb256(nrow)), dim3(256), 0, s, b.p, dinv.p, r.p, z.p, p.p, q.p, partial.p,
                           partial.p + 2 * nch, nrow);
        hipLaunchKernelGGL(k_mcg_fin_restart, dim3(nsys), dim3(256), 0, s, partial.p, partial.p + 2 * nch, cb.p, sc.p,
                           mirror.dev);
        DDPCA_HIP(hipStreamEndCapture(s, &g));
        DDPCA_HIP(hipGraphInstantiate(&cgraph_, g, nullptr, nullptr, 0));
        DDPCA_HIP(hipGraphDestroy(g));
    }
    void capture_one(hipStream_t s, PcgScal* scp, hipGraphExec_t* out, int64_t iters) {
        EllArgs e{slots.p, off.p, col.p, val.p, csys.p, dinv.p, nch};
        hipGraph_t g;
        CaptureSection capture_section;  // device_common.hpp CaptureLock
        DDPCA_HIP(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        const bool fa = fuse_alpha();
        // DDPCA_MCG_PAIR=0: the unpaired k_mcg_spmv on a paired batch (bit-identical, A/B and tests)
        const char* ep = std::getenv("DDPCA_MCG_PAIR");
        const bool pair = paired_ && !(ep && std::atoi(ep) == 0);
        pair_used_ = pair;
        double* ppq = partial.p + 2 * nch;  // p.q per chunk
        auto spmv = [&](double* part, int stride) {
            if (pair)
                hipLaunchKernelGGL(k_mcg_spmv2, dim3(ceil_div(nch / 2, 4)), dim3(256), 0, s, e, scp, z.p, q.p, p.p, part,
                                   stride, nrow / 2, nch / 2);
            else
                hipLaunchKernelGGL(k_mcg_spmv, dim3(ceil_div(nch, 4)), dim3(256), 0, s, e, scp, z.p, q.p, p.p, part, stride);
        };
        for (int64_t it = 0; it < iters; ++it) {
            if (fa) {
                spmv(ppq, 1);
                hipLaunchKernelGGL(k_mcg_axpy_fa, dim3(nb256(nrow)), dim3(256), 0, s, e, scp, x_target_, r.p, z.p, p.p,
                                   q.p, partial.p, (const double*)ppq, cb.p, mirror.dev);
            } else {
                spmv(partial.p, 2);
                hipLaunchKernelGGL(k_mcg_fin, dim3(nsys), dim3(256), 0, s, (int)kMcgAlpha, partial.p, cb.p, scp, mirror.dev);
                hipLaunchKernelGGL(k_mcg_axpy, dim3(nb256(nrow)), dim3(256), 0, s, e, scp, x_target_, r.p, z.p, p.p, q.p,
                                   partial.p);
            }
            hipLaunchKernelGGL(k_mcg_fin, dim3(nsys), dim3(256), 0, s, (int)kMcgBeta, partial.p, cb.p, scp, mirror.dev);
        }
        DDPCA_HIP(hipStreamEndCapture(s, &g));
        DDPCA_HIP(hipGraphInstantiate(out, g, nullptr, nullptr, 0));
        DDPCA_HIP(hipGraphDestroy(g));
    }
};

}  // namespace

// Interface-eliminated coarse space on the device (MCONTACT.h:2578-2612, operators from
// MULTISCALE_1).  Per ADMM iteration, after the subdomain solves:
//   g  = globForc_1 + sum globTran_1 lambda - sum globTran_D_1 u          (2580-2587)
//        globTran_D_1 u = Rc (consStif[L] x) + interface part; the stiffness part is one fp64
//        SpMV of the batch's fine operator followed by the restriction chain to level doleMcsc
//        (factored: Rc consStif[L] would have ~30 entries per fine dof), the rest is one CSR
//        product over the workspace W (columns: owned u and lambda)
//   g summed over ranks (each rank holds the columns it owns), one RCCL all-reduce
//   xc = globCoup_1^-1 g, rows of the owned subdomains (dense inverse from rocSOLVER potrf/potri
//        at setup; the reference factorises with SimplicialLDLT, 2589-2591)
//   u += OUTP_SUB1(accuProl xc)                                             (2600-2610)
struct CoarseDev {
    bool on = false, inverted = false;
    int64_t n = 0, nown = 0, nxn = 0, qnn = 0;
    double dense_bytes = 0.0;  // n^2 8 B: what the dense inverse would hold per rank
    bool mg_fallback = false;  // (kept for the "coarse_solve" getter: DOUBLE_M is always buildable now)
    DevBuf<double> g, f0, xc, xn, ainv;
    // the right-hand side's per-source slots (build_coarse): rptr/rcol/rval and f0 are per slot,
    // gs the slot values (all-reduced), sptr the slots of each coarse row
    int64_t nslot = 0;
    DevBuf<double> gs;
    DevBuf<int64_t> sptr;
    DevBuf<int64_t> rptr;
    DevBuf<int32_t> rcol;
    DevBuf<double> rval;
    struct KGroup {
        int level = 0;
        DevBuf<int32_t> rows;
        DevBuf<int64_t> src;
    };
    std::vector<KGroup> kg;
    int dmin = 0;
    DevBuf<int32_t> xsrc, qcol;
    DevBuf<double> qw;
    DevBuf<uint8_t> flag;
    // assembled variant (cs.assembled): the caller's globTran_D_1 in the right-hand side CSR and
    // accuProl as CSR rows over the owned fine free dofs; factored: the scalar stencil (<= 8
    // parents) for every node it can hold, CSR rows (same arrays) for the rest -- nodes whose chain
    // meets a nodal rotation's 3x3 block (general trees)
    bool assembled = false, latin = false;
    int64_t npr = 0, ncd = 0;
    DevBuf<int64_t> pptr;
    DevBuf<int32_t> pcol, ptgt, cdof;
    DevBuf<double> pval;
    std::vector<int64_t> own_rows;  // global coarse rows of this rank, in xc order
    double bytes_iter = 0.0;        // algorithmic bytes of one correction (without DOUBLE_M's PCG)
    std::vector<double> dense;      // host, until inverted: this rank's rows of globCoup_1 (n x n, zeros elsewhere)
    // DOUBLE_M_1 (MCONTACT.h:2303-2341; the reference's choice once globCoup_1 has DIRE_MAXI rows,
    // 1857-1865): the coarse problem solved by its own MGPIS-PCG, redundantly on every rank, on a
    // hierarchy whose transfers are every subdomain's realProl below doleMcsc, block-diagonal
    bool mg = false;
    bool mg_gather = false;  // a rank-local build: the whole operator is gathered at coarse_invert
    // the coarse MGPIS's structure (plan_coarse_mg, at setup): nodes per level, transfers, the
    // coarse rows' dofs, per-level dof flags; kept until the operator is there (finish_coarse_mg)
    struct MgPlan {
        std::vector<int64_t> nglob;
        std::vector<Stencil> S;
        std::vector<int32_t> fdg;
        std::vector<std::vector<uint8_t>> flev;
        bool latin = false;
        void swap_into(MgPlan& o) { std::swap(*this, o); }
    } plan;
    Csr gathered_rows;  // this rank's rows of a rank-local operator (sent once at coarse_invert)
    std::unique_ptr<MgpisDevice> cmg;
    DevBuf<int32_t> cperm;  // coarse row -> dof of cmg's fine level (device layout)
    DevBuf<int32_t> cown;   // xc index -> coarse row
    hipEvent_t ev_in = nullptr, ev_out = nullptr;
    ~CoarseDev() {
        if (ev_in) (void)hipEventDestroy(ev_in);
        if (ev_out) (void)hipEventDestroy(ev_out);
    }
};

// ============================================================================= transport
// The exchanges of a multi-rank run, all stream-ordered on the rank's stream:
//   exchange()      the gamma halves of cross-rank interfaces (one grouped send/recv per peer)
//   allreduce_sum() the MONITOR norms and the coarse right-hand side every iteration, the dense
//                   coarse matrix once at setup
// RcclTransport is the production path (RCCL over xGMI); LocalTransport connects the handles of
// ONE process through host-staged copies (mcontact_gpu_comm_local) so the multi-rank bookkeeping
// (owner maps, gamma offsets, rank-local coarse rows) runs on a single GPU in the tests.
struct Transport {
    struct Msg {
        int peer;
        int64_t tag;  // interface index
        const double* send;
        double* recv;
        int64_t n;
    };
    virtual ~Transport() = default;
    virtual void allreduce_sum(double* buf, int64_t n, hipStream_t st) = 0;
    virtual void exchange(const std::vector<Msg>& msgs, hipStream_t st) = 0;
};

struct RcclTransport : Transport {
    ncclComm_t comm = nullptr;
    ~RcclTransport() override {
        if (comm) (void)ncclCommDestroy(comm);
    }
    void allreduce_sum(double* buf, int64_t n, hipStream_t st) override {
        DDPCA_NCCL(ncclAllReduce(buf, buf, (size_t)n, ncclDouble, ncclSum, comm, st));
    }
    void exchange(const std::vector<Msg>& msgs, hipStream_t st) override {
        DDPCA_NCCL(ncclGroupStart());
        for (const Msg& m : msgs) {
            DDPCA_NCCL(ncclSend(m.send, (size_t)m.n, ncclDouble, m.peer, comm, st));
            DDPCA_NCCL(ncclRecv(m.recv, (size_t)m.n, ncclDouble, m.peer, comm, st));
        }
        DDPCA_NCCL(ncclGroupEnd());
    }
};

// Timing-only transport (mcontact_gpu_comm_loopback): every receive from peer p gets what this
// rank sent p, as an on-device copy on the solve stream; all-reduces keep this rank's own values.
// One rank of an N-rank layout then runs its own share of the work on a single GPU.
struct LoopbackTransport : Transport {
    void allreduce_sum(double*, int64_t, hipStream_t) override {}
    void exchange(const std::vector<Msg>& msgs, hipStream_t st) override {
        for (const Msg& m : msgs)
            if (m.n) DDPCA_HIP(hipMemcpyAsync(m.recv, m.send, (size_t)m.n * sizeof(double), hipMemcpyDeviceToDevice, st));
    }
};

// Rendezvous of the ranks of one process (each rank's calls come from its own host thread).
struct LocalHub {
    int n = 0;
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    int64_t generation = 0;
    bool broken = false;
    std::vector<std::vector<double>> slot;  // allreduce staging per rank
    // posted sends per (src, dst) in issue order -- matched against the receiver's receives from
    // src in ITS issue order, as RCCL matches grouped ncclSend / ncclRecv pairs per peer (tags and
    // sizes are only checked, never used for matching: an ordering bug fails here as on the wire)
    struct Posted {
        int64_t tag;
        const double* buf;
        int64_t n;
    };
    std::map<std::pair<int, int>, std::deque<Posted>> post;
    void barrier() {
        std::unique_lock<std::mutex> lk(mu);
        if (broken) throw ApiError(DDPCA_ECOMM, "local transport: a peer failed");
        const int64_t g = generation;
        if (++arrived == n) {
            arrived = 0;
            ++generation;
            cv.notify_all();
        } else if (!cv.wait_for(lk, std::chrono::seconds(120), [&] { return generation != g || broken; }) || broken) {
            broken = true;
            cv.notify_all();
            throw ApiError(DDPCA_ECOMM, "local transport: peers did not arrive");
        }
    }
};

struct LocalTransport : Transport {
    std::shared_ptr<LocalHub> hub;
    int rank = 0;
    void allreduce_sum(double* buf, int64_t n, hipStream_t st) override {
        auto& mine = hub->slot[rank];
        mine.resize(n);
        DDPCA_HIP(hipMemcpyAsync(mine.data(), buf, n * sizeof(double), hipMemcpyDeviceToHost, st));
        DDPCA_HIP(hipStreamSynchronize(st));
        hub->barrier();
        std::vector<double> sum(n, 0.0);
        for (int q = 0; q < hub->n; ++q)  // rank order: every rank gets the same bits
            for (int64_t i = 0; i < n; ++i) sum[i] += hub->slot[q][i];
        DDPCA_HIP(hipMemcpyAsync(buf, sum.data(), n * sizeof(double), hipMemcpyHostToDevice, st));
        DDPCA_HIP(hipStreamSynchronize(st));
        hub->barrier();  // nobody restages before every rank has read the slots
    }
    void exchange(const std::vector<Msg>& msgs, hipStream_t st) override {
        DDPCA_HIP(hipStreamSynchronize(st));
        {
            std::lock_guard<std::mutex> lk(hub->mu);
            for (const Msg& m : msgs) hub->post[{rank, m.peer}].push_back({m.tag, m.send, m.n});
        }
        hub->barrier();
        std::string err;
        for (const Msg& m : msgs) {
            LocalHub::Posted p{};
            {
                std::lock_guard<std::mutex> lk(hub->mu);
                auto& q = hub->post[{m.peer, rank}];
                if (q.empty()) {
                    err = "local transport: receive from rank " + std::to_string(m.peer) + " has no matching send";
                    break;
                }
                p = q.front();
                q.pop_front();
            }
            if (p.tag != m.tag || p.n != m.n) {
                err = "local transport: message order differs between ranks " + std::to_string(m.peer) + " and " +
                      std::to_string(rank) + " (tag " + std::to_string(p.tag) + " sent, " + std::to_string(m.tag) +
                      " expected)";
                break;
            }
            DDPCA_HIP(hipMemcpyAsync(m.recv, p.buf, m.n * sizeof(double), hipMemcpyDeviceToDevice, st));
        }
        DDPCA_HIP(hipStreamSynchronize(st));
        if (!err.empty()) {
            std::lock_guard<std::mutex> lk(hub->mu);
            hub->broken = true;
            hub->cv.notify_all();
            throw ApiError(DDPCA_ECOMM, err);
        }
        hub->barrier();  // the peers' send buffers stay untouched until every copy has landed
        std::lock_guard<std::mutex> lk(hub->mu);
        for (const Msg& m : msgs)
            if (!hub->post[{rank, m.peer}].empty()) {
                hub->broken = true;
                throw ApiError(DDPCA_ECOMM, "local transport: a send to rank " + std::to_string(m.peer) + " was not received");
            }
    }
};

// ================================================================================ handle
struct ddpca_mcontact {
    struct Sub {
        int64_t tv = 0, nn = 0;
        int64_t dof0 = 0;  // first dof in the batch's fine layout
        int64_t nh = 0;    // hanging-level dofs (MULTIGRID::hangProl rows), at W[oH + hoff]
        int64_t hoff = 0;
        // workspace index of the subdomain's nodal dof c (position numbering, hanging level last)
        int64_t wcol(int64_t c, int64_t oH) const { return c < 3 * nn ? dof0 + c : oH + hoff + (c - 3 * nn); }
    };
    struct Side {
        int64_t ts = 0, s = 0, tv = 0, m = 0, mip = 0;
        int64_t roff = 0;  // rows of aux at W[oS + roff], lambda at W[oS + R + roff]
        int sub = 0;       // index into subs
    };
    struct Itf {
        int64_t ts = 0, mip = 0, goff = 0;
        int comp = 1;
        double fric = -1.0;
        int owner[2] = {0, 0};
        bool mine = false, cross = false;
        DevBuf<int32_t> stat;
        DevBuf<double> recv;
    };
    int device = 0, rank = 0, nranks = 1;
    int64_t nsub = 0, nint = 0;
    std::vector<int32_t> owner;
    std::vector<Sub> subs;
    std::vector<Side> sides;
    std::vector<Itf> itfs;
    std::unique_ptr<MgpisDevice> mg;
    std::vector<int64_t> maxit;          // per owned subdomain: n_free (reference maxit = rows)
    DevBuf<double> cf;                   // consForc, solver (device) node order
    DevBuf<double> presc;                // Dirichlet values, reference node order (3 nn_L)
    DevBuf<int32_t> onode;               // device node -> reference-order node of the batch
    DevBuf<int32_t> crow;                // coupling rows (solver dofs, surface rows only)
    DevBuf<int64_t> cptr;
    DevBuf<int32_t> ccol;                // columns index W
    DevBuf<double> cval;
    int64_t ncrow = 0;
    int64_t R = 0;                       // padded rows of all owned sides
    // workspace W = [u (NU) | u on hanging levels (NH) | aux, lambda (2R) | gamma (G)] and its regions
    DevBuf<double> W;
    int64_t NU = 0, NH = 0, G = 0, oH = 0, oS = 0, oG = 0;
    SellOp op_hang;                      // hanging-level values: rows of prolOper[maxiLeve] over u
    double* u = nullptr;
    double* state = nullptr;
    double* gamma = nullptr;
    DevBuf<double> uo, state_old, gcst, moni;
    // the MONITOR pair norms as one batch (k_pair_norms_all): segments, block -> segment
    std::vector<NormSeg> norm_seg_host;
    DevBuf<NormSeg> norm_seg;
    DevBuf<int32_t> norm_bseg;
    DevBuf<double> norm_partial;
    SellOp op_gamma, op_aux, op_lam;     // gamma (my halves), aux RHS, lambda RHS
    // rank-local interfaces' side-1 halves (SELL rows; the factored ones in k_gamma_ip), added onto
    // the side-0 halves by k_add_idx: gamma = (constant + half 0) + half 1 on every rank layout
    SellOp op_gamma1;
    DevBuf<double> gam1;
    DevBuf<int32_t> gam1_dst;
    // interfaces whose per-ip operators are applied in factored form (Interface::factored)
    struct FactItf {
        int64_t ts = 0, nip = 0, goff = 0;
        int C = 1, own[2] = {0, 0};
        double pen[3] = {0.0, 0.0, 0.0};
        DevBuf<double> B, M[2], T;
        DevBuf<int32_t> lam[2], u[2];
        int64_t nnc[2] = {0, 0}, roff[2] = {0, 0};  // node-major inteInpo (fused update)
        DevBuf<int64_t> nptr[2];
        DevBuf<int32_t> niq[2];
        DevBuf<double> ncoef[2];
        double bytes_gamma = 0.0, bytes_inpo = 0.0;  // algorithmic bytes of k_gamma_ip / k_traction_ip + k_inpo_node
    };
    std::vector<FactItf> fitfs;
    MassBatch mb_aux, mb_lam;
    // fused interface update (every owned side has inteMass_pena = rho inteMass and
    // systTran_pena = rho systTran): one batched solve of M [w | v] = [T^T u | I gamma]
    bool fused = false;
    SellOp op_wv;
    MassBatch mb_wv;
    DevBuf<double> rinv;
    CoarseDev cs;
    std::vector<double> moni_host;
    hipStream_t main = nullptr;          // == mg->stream
    std::unique_ptr<Transport> comm;     // RCCL (any rank count, 1 included), or the in-process test transport
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
    // reference MONITOR state (MCONTACT.h:2494-2498, 2725-2845)
    int64_t tc = 0;
    int64_t mult_maxi = 1000;  // PREP.h:75 (global in the reference)
    std::vector<std::vector<double>> moniReco;
    std::vector<std::vector<double>> rows;
    double timing[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    double mass_iters = 0.0;
    // algorithmic HBM bytes since the last mcontact_gpu_iterate started (include/ddpca_amd.h,
    // mcontact_gpu_bytes): [0] fine-level PCG kernels, [1] PCG kernels below the fine level + the
    // scalar kernels, [2] coarse-space correction, [3] body-balance RHS + OUTP_SUB1, [4] interface
    // products and projection, [5] batched surface-mass CG, [6] MONITOR snapshot + norms,
    // [7] body-balance PCG launches
    double bytes[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    double bytes_rhs = 0.0, bytes_iface = 0.0, bytes_moni = 0.0;  // per ADMM iteration (model, build)
    mgpis_options_t opt{};
};

namespace {

void build(ddpca_mcontact& H, Problem& P) {
    MCONTACT& mc = P.mc;
    H.nsub = (int64_t)mc.multGrid.size();
    H.nint = (int64_t)mc.searCont.size();
    // ---- owned subdomains: one batched MGPIS
    std::vector<SubdomainOps> ops;
    for (int64_t tv = 0; tv < H.nsub; ++tv) {
        if (H.owner[tv] != H.rank) continue;
        if (P.owned.size() != (size_t)H.nsub || !P.owned[tv])
            throw ApiError(DDPCA_ESTATE, "subdomain " + std::to_string(tv) + " is owned by this rank but was not established");
        const MULTIGRID& g = mc.multGrid[tv];
        SubdomainOps o;
        o.nnodes.assign(g.leveCount.begin(), g.leveCount.end());
        for (const auto& b : g.levelStif) o.K.push_back(&b);
        // prolOper: scalProl with the nodal rotations' 3x3 blocks as block entries (MULTIGRID.h:
        // 1141-1181; == scalProl without nodeRota); an operator-level subdomain has scalProl only
        // (its block entries already in it)
        for (const auto& s : g.prolOper.empty() ? g.scalProl : g.prolOper) o.S.push_back(&s);
        o.dof_free = g.consFlag.data();
        o.coords = g.nodeCoor.empty() ? nullptr : g.nodeCoor[0].data();
        ops.push_back(o);
        ddpca_mcontact::Sub S;
        S.tv = tv;
        S.nn = g.leveCount.back();
        S.nh = 3 * (g.nodalCount() - S.nn);
        H.subs.push_back(S);
    }
    if (!ops.empty()) {
        H.mg = std::make_unique<MgpisDevice>(H.device, ops, H.opt);
        H.main = H.mg->stream;
        // the body balance's batch on two streams (MgpisDevice::set_split); DDPCA_STREAMS=1 keeps
        // the single-stream graph, DDPCA_PCG_STREAMS=3 / 4 splits it three / four ways (A/B runs)
        const char* ps = std::getenv("DDPCA_PCG_STREAMS");
        H.mg->set_split(two_streams(), ps ? std::max(2, std::min(kMaxParts, std::atoi(ps))) : 2);
    } else {
        DDPCA_HIP(hipStreamCreateWithFlags(&H.main, hipStreamNonBlocking));
    }
    auto sub_index = [&](int64_t tv) {
        for (size_t i = 0; i < H.subs.size(); ++i)
            if (H.subs[i].tv == tv) return (int)i;
        return -1;
    };
    const int64_t NN = H.mg ? H.mg->lev.back().nn : 0;
    H.NU = std::max<int64_t>(3 * NN, 64);
    for (auto& S : H.subs) {
        S.hoff = H.NH;
        H.NH += S.nh;
    }
    H.NH = pad64(H.NH);
    {
        std::vector<double> cf(H.NU, 0.0), pr(H.NU, 0.0);
        std::vector<int32_t> on(std::max<int64_t>(NN, 1));
        std::iota(on.begin(), on.end(), 0);  // padding nodes map to themselves
        for (size_t i = 0; i < H.subs.size(); ++i) {
            auto& S = H.subs[i];
            S.dof0 = H.mg->fine_dof_offset((int)i);
            // DDPCA_PCG_MAXIT (diagnostics only): cap the body solves below the reference's maxit = rows
            static const int64_t cap = std::getenv("DDPCA_PCG_MAXIT") ? std::atoll(std::getenv("DDPCA_PCG_MAXIT")) : 0;
            H.maxit.push_back(cap > 0 ? std::min<int64_t>(cap, H.mg->nfree[i]) : H.mg->nfree[i]);
            const MULTIGRID& g = mc.multGrid[S.tv];
            for (int64_t d = 0; d < 3 * S.nn; ++d)
                if (g.consFlag[d]) cf[H.mg->fine_dof((int)i, d)] = g.consForc[g.freeIndex[d]];
            for (const auto& kv : g.consDofv) pr[S.dof0 + kv.first] = kv.second;
            for (int64_t r = 0; r < S.nn; ++r) on[S.dof0 / 3 + H.mg->fine_perm[i][r]] = (int32_t)(S.dof0 / 3 + r);
        }
        H.cf.upload(cf);
        H.presc.upload(pr);
        H.onode.upload(on);
    }
    // ---- owned interface sides: aux rows [roff, roff + m), lambda rows R + the same
    int64_t roff = 0;
    std::map<std::pair<int64_t, int64_t>, size_t> side_of;
    for (int64_t ts = 0; ts < H.nint; ++ts) {
        const Interface& itf = mc.searCont[ts];
        for (int s = 0; s < 2; ++s) {
            if (H.owner[itf.body[s]] != H.rank) continue;
            ddpca_mcontact::Side sd;
            sd.ts = ts;
            sd.s = s;
            sd.tv = itf.body[s];
            sd.sub = sub_index(sd.tv);
            sd.m = itf.mside(s);
            sd.mip = itf.mip();
            sd.roff = roff;
            roff += pad64(sd.m);
            side_of[{ts, s}] = H.sides.size();
            H.sides.push_back(sd);
        }
    }
    H.R = roff;
    // ---- interfaces: gamma layout (cross-rank interfaces first, then rank-local)
    int64_t goff = 0;
    for (int pass = 0; pass < 2; ++pass)
        for (int64_t ts = 0; ts < H.nint; ++ts) {
            const Interface& itf = mc.searCont[ts];
            const int o0 = H.owner[itf.body[0]], o1 = H.owner[itf.body[1]];
            const bool cross = o0 != o1;
            if ((pass == 0) != cross) continue;
            ddpca_mcontact::Itf I;
            I.ts = ts;
            I.mip = itf.mip();
            I.comp = itf.comp();
            I.fric = itf.fric;
            I.owner[0] = o0;
            I.owner[1] = o1;
            I.cross = cross;
            I.mine = (o0 == H.rank || o1 == H.rank);
            I.goff = goff;
            goff += I.mip;
            if (I.mine) {
                I.stat.alloc(std::max<int64_t>(I.mip / I.comp, 1));
                if (cross) I.recv.alloc(I.mip);
            }
            H.itfs.push_back(std::move(I));
        }
    std::sort(H.itfs.begin(), H.itfs.end(), [](const auto& a, const auto& b) { return a.ts < b.ts; });
    H.G = pad64(std::max<int64_t>(goff, 1));
    // ---- workspace
    H.oH = H.NU;
    H.oS = H.NU + H.NH;
    H.oG = H.oS + 2 * H.R;
    H.W.alloc(H.oG + H.G);
    H.W.zero(H.main);
    H.u = H.W.p;
    H.state = H.W.p + H.oS;
    H.gamma = H.W.p + H.oG;
    H.uo.alloc(H.NU + H.NH);
    H.uo.zero(H.main);
    H.state_old.alloc(std::max<int64_t>(2 * H.R, 2));
    H.state_old.zero(H.main);
    auto itf_of = [&](int64_t ts) -> const ddpca_mcontact::Itf& {
        return *std::find_if(H.itfs.begin(), H.itfs.end(), [&](const auto& x) { return x.ts == ts; });
    };
    // ---- factored per-ip operators of host-built interfaces this rank handles
    for (const auto& I : H.itfs) {
        const Interface& itf = mc.searCont[I.ts];
        if (!I.mine || !itf.factored) continue;
        ddpca_mcontact::FactItf F;
        F.ts = I.ts;
        F.nip = (int64_t)itf.ip.size();
        F.goff = I.goff;
        F.C = itf.comp();
        for (int m = 0; m < F.C; ++m) F.pen[m] = itf.pemaDiag[m];  // pemaDiag[C q + m] = pen[m] for every q
        const int64_t nip = F.nip;
        std::vector<double> B(9 * std::max<int64_t>(nip, 1));
        for (int64_t q = 0; q < nip; ++q)
            for (int j = 0; j < 9; ++j) B[j * nip + q] = itf.ip[q].basis[j / 3][j % 3];
        F.B.upload(B);
        F.T.alloc(std::max<int64_t>(F.C * nip, 1));
        for (int s = 0; s < 2; ++s) {
            if (H.owner[itf.body[s]] != H.rank) continue;
            F.own[s] = 1;
            const auto& sd = H.sides[side_of.at({I.ts, s})];
            const auto& Su = H.subs[sd.sub];
            const int64_t lam0 = H.oS + H.R + sd.roff;
            std::unordered_map<int64_t, int32_t> cidx;
            for (size_t a = 0; a < itf.nodeCont[s].size(); ++a) cidx.emplace(itf.nodeCont[s][a], (int32_t)a);
            std::vector<double> M(4 * std::max<int64_t>(nip, 1));
            std::vector<int32_t> lam(4 * std::max<int64_t>(nip, 1)), u(4 * std::max<int64_t>(nip, 1));
            std::vector<std::vector<std::pair<int32_t, double>>> bynode(itf.nodeCont[s].size());
            const double sgn = s == 0 ? -1.0 : 1.0;  // inteInpo's sign (mcontact.cpp BUILD)
            for (int64_t q = 0; q < nip; ++q)
                for (int a = 0; a < 4; ++a) {
                    const int64_t node = itf.ip[q].node[s][a];
                    const int32_t c = cidx.at(node);
                    M[a * nip + q] = itf.ip[q].shap[s][a];
                    lam[a * nip + q] = (int32_t)(lam0 + F.C * c);
                    u[a * nip + q] = (int32_t)Su.wcol(3 * node, H.oH);
                    bynode[c].push_back({(int32_t)q, sgn * (itf.ip[q].w * itf.ip[q].shap[s][a])});
                }
            F.M[s].upload(M);
            F.lam[s].upload(lam);
            F.u[s].upload(u);
            std::vector<int64_t> ptr{0};
            std::vector<int32_t> iq;
            std::vector<double> coef;
            for (const auto& v : bynode) {
                for (const auto& e : v) {
                    iq.push_back(e.first);
                    coef.push_back(e.second);
                }
                ptr.push_back((int64_t)iq.size());
            }
            F.nnc[s] = (int64_t)bynode.size();
            F.roff[s] = sd.roff;
            // k_gamma_ip's share of this side: shape values, lambda and u indices per ip, the
            // side's contact-node lambda (C per node) and body-node u (3 per node) once;
            // k_inpo_node: index + coefficient per (node, ip) entry, the node's C outputs
            F.bytes_gamma += 48.0 * (double)nip + (double)F.nnc[s] * 8.0 * (F.C + 3);
            F.bytes_inpo += 12.0 * (double)iq.size() + 8.0 * F.C * (double)nip + 8.0 * F.C * (double)F.nnc[s];
            F.nptr[s].upload(ptr);
            F.niq[s].upload(iq.empty() ? std::vector<int32_t>{0} : iq);
            F.ncoef[s].upload(coef.empty() ? std::vector<double>{0.0} : coef);
        }
        // per ip: the 3x3 basis, gamma written and the constant part read (k_gamma_ip); basis,
        // gamma read and the traction written (k_traction_ip)
        F.bytes_gamma += (double)nip * (72.0 + 16.0 * F.C);
        F.bytes_inpo += (double)nip * ((F.C == 3 ? 72.0 : 0.0) + 16.0 * F.C);
        H.fitfs.push_back(std::move(F));
    }
    // ---- interface operators over W (MCONTACT.h:2632-2636, 2671-2704)
    {
        Rows rg(H.G), ra(H.R), rl(H.R), rg1;
        std::vector<int32_t> g1dst;
        std::map<int64_t, int64_t> g1off;  // rank-local SELL interface -> its first row in rg1
        std::vector<double> gc(H.G, 0.0);
        for (const auto& sd : H.sides) {
            const Interface& itf = mc.searCont[sd.ts];
            const auto& I = itf_of(sd.ts);
            const int s = (int)sd.s;
            const double half = s == 0 ? 0.5 : -0.5;
            const auto& Su = H.subs[sd.sub];
            const int64_t lam0 = H.oS + H.R + sd.roff, aux0 = H.oS + sd.roff;
            // gamma half: +-1/2 (inpoLagr lambda + pemaInpo_r u); side 0 adds -1/2 pema g
            const Csr& Lg = itf.inpoLagr[s];
            const Csr& Rg = itf.pemaInpo_r[s];
            // a rank-local interface's side 1 sums its half in rows of its own (op_gamma1)
            const bool own_rows1 = !itf.factored && s == 1 && !I.cross;
            if (own_rows1 && !g1off.count(sd.ts)) {
                g1off[sd.ts] = (int64_t)rg1.size();
                for (int64_t i = 0; i < sd.mip; ++i) g1dst.push_back((int32_t)(I.goff + i));
                rg1.resize(rg1.size() + sd.mip);
            }
            for (int64_t i = 0; i < sd.mip; ++i) {
                if (!itf.factored) {  // factored interfaces: k_gamma_ip
                    auto& row = own_rows1 ? rg1[g1off[sd.ts] + i] : rg[I.goff + i];
                    for (int64_t k = Lg.ptr[i]; k < Lg.ptr[i + 1]; ++k) row.push_back({lam0 + Lg.col[k], half * Lg.val[k]});
                    for (int64_t k = Rg.ptr[i]; k < Rg.ptr[i + 1]; ++k) row.push_back({Su.wcol(Rg.col[k], H.oH), half * Rg.val[k]});
                }
                if (s == 0) gc[I.goff + i] = -0.5 * (itf.pemaDiag[i] * itf.inpoNgap[i]);
            }
            // aux RHS: systTran_pena^T u + inteMass lambda + inteInpo gamma
            const Csr tTp = transpose(itf.systTran_pena[s]);
            const Csr& M = itf.inteMass[s];
            const Csr& Mp = itf.inteMass_pena[s];
            const Csr& Ii = itf.inteInpo[s];
            for (int64_t r = 0; r < sd.m; ++r) {
                auto& a = ra[sd.roff + r];
                auto& l = rl[sd.roff + r];
                for (int64_t k = tTp.ptr[r]; k < tTp.ptr[r + 1]; ++k) {
                    a.push_back({Su.wcol(tTp.col[k], H.oH), tTp.val[k]});
                    l.push_back({Su.wcol(tTp.col[k], H.oH), tTp.val[k]});
                }
                for (int64_t k = M.ptr[r]; k < M.ptr[r + 1]; ++k) a.push_back({lam0 + M.col[k], M.val[k]});
                for (int64_t k = Ii.ptr[r]; k < Ii.ptr[r + 1]; ++k) a.push_back({H.oG + I.goff + Ii.col[k], Ii.val[k]});
                // lambda RHS: systTran_pena^T u - inteMass_pena aux
                for (int64_t k = Mp.ptr[r]; k < Mp.ptr[r + 1]; ++k) l.push_back({aux0 + Mp.col[k], -Mp.val[k]});
            }
        }
        H.op_gamma.build(rg);
        if (!rg1.empty()) {
            H.op_gamma1.build(rg1);
            H.gam1.alloc(H.op_gamma1.nrow);
            H.gam1_dst.upload(g1dst);
        }
        H.op_aux.build(ra);
        H.op_lam.build(rl);
        H.gcst.upload(gc);
        std::vector<const Csr*> Ma, Ml;
        std::vector<int64_t> ro;
        for (auto& sd : H.sides) {
            const Interface& itf = mc.searCont[sd.ts];
            Ma.push_back(&itf.inteMass_pena[sd.s]);
            Ml.push_back(&itf.inteMass[sd.s]);
            ro.push_back(sd.roff);
        }
        H.mb_aux.build(Ma, ro, H.R);
        H.mb_lam.build(Ml, ro, H.R);
        H.mb_aux.set_split(two_streams());
        H.mb_lam.set_split(two_streams());
        // fused update when the penalty operators are exact multiples of the plain ones
        // (entries agree to rounding: the penalty operators are accumulated with pen inside the
        // basis products, e.g. off-diagonal T^T P T entries are rounding noise around 0)
        auto proportional = [](const Csr& A, const Csr& B, double rho) {
            if (A.nrow != B.nrow || A.ptr != B.ptr || A.col != B.col) return false;
            double amax = 0.0;
            for (double v : A.val) amax = std::max(amax, std::abs(v));
            for (int64_t k = 0; k < A.nnz(); ++k)
                if (std::abs(A.val[k] - rho * B.val[k]) > 1e-13 * amax) return false;
            return true;
        };
        const char* env = std::getenv("DDPCA_MASS_FUSED");
        bool fuse = !H.sides.empty() && (!env || std::atoi(env) != 0);
        for (const auto& sd : H.sides) {
            const Interface& itf = mc.searCont[sd.ts];
            const double rho = itf.penN;
            fuse = fuse && itf.penN == itf.penF && rho > 0.0 && proportional(itf.inteMass_pena[sd.s], itf.inteMass[sd.s], rho) &&
                   proportional(itf.systTran_pena[sd.s], itf.systTran[sd.s], rho);
        }
        if (fuse) {
            H.fused = true;
            Rows rwv(2 * H.R);
            std::vector<double> ri(std::max<int64_t>(H.R, 1), 0.0);
            std::vector<const Csr*> M2;
            std::vector<int64_t> ro2;
            for (const auto& sd : H.sides) {
                const Interface& itf = mc.searCont[sd.ts];
                const auto& I = itf_of(sd.ts);
                const auto& Su = H.subs[sd.sub];
                const Csr tT = transpose(itf.systTran[sd.s]);
                const Csr& Ii = itf.inteInpo[sd.s];
                for (int64_t r = 0; r < sd.m; ++r) {
                    for (int64_t k = tT.ptr[r]; k < tT.ptr[r + 1]; ++k) rwv[sd.roff + r].push_back({Su.wcol(tT.col[k], H.oH), tT.val[k]});
                    if (!itf.factored)  // factored interfaces: k_traction_ip + k_inpo_node
                        for (int64_t k = Ii.ptr[r]; k < Ii.ptr[r + 1]; ++k)
                            rwv[H.R + sd.roff + r].push_back({H.oG + I.goff + Ii.col[k], Ii.val[k]});
                    ri[sd.roff + r] = 1.0 / itf.penN;
                }
                M2.push_back(&itf.inteMass[sd.s]);
                ro2.push_back(sd.roff);
            }
            for (const auto& sd : H.sides) {
                M2.push_back(&mc.searCont[sd.ts].inteMass[sd.s]);
                ro2.push_back(H.R + sd.roff);
            }
            H.op_wv.build(rwv);
            H.mb_wv.build(M2, ro2, 2 * H.R);
            H.mb_wv.set_split(two_streams());
            H.rinv.upload(ri);
        }
        if (std::getenv("DDPCA_VERBOSE"))
            std::fprintf(stderr, "[ddpca] interface update: %s\n", H.fused ? "fused (one batched mass solve)" : "sequential");
    }
    // ---- coupling rows of the body-balance RHS: sum over incident sides of
    //      [systTran_pena | -systTran] on free dofs, solver dofs x W columns
    {
        std::map<int64_t, std::vector<std::pair<int32_t, double>>> rowmap;
        for (size_t si = 0; si < H.subs.size(); ++si) {
            const auto& S = H.subs[si];
            const MULTIGRID& g = mc.multGrid[S.tv];
            for (int64_t ts = 0; ts < H.nint; ++ts) {
                const Interface& itf = mc.searCont[ts];
                for (int s = 0; s < 2; ++s) {
                    if (itf.body[s] != S.tv) continue;
                    const auto& sd = H.sides[side_of.at({ts, s})];
                    const Csr& Tp = itf.systTran_pena[s];
                    const Csr& T = itf.systTran[s];
                    const int64_t n3 = 3 * S.nn;
                    for (int64_t r = 0; r < Tp.nrow; ++r) {
                        // only the rows the interface actually couples (surface rows)
                        if (Tp.ptr[r] == Tp.ptr[r + 1] && T.ptr[r] == T.ptr[r + 1]) continue;
                        // a hanging-level row reaches the free dofs through prolOper[maxiLeve]^T
                        // (ADDITIONAL_FORCE, MULTIGRID.h:1257-1261)
                        std::vector<std::pair<int64_t, double>> tgt;
                        if (r < n3) {
                            tgt.push_back({r, 1.0});
                        } else {
                            const Csr& Hp = g.hangProl;
                            for (int64_t k = Hp.ptr[r - n3]; k < Hp.ptr[r - n3 + 1]; ++k) tgt.push_back({Hp.col[k], Hp.val[k]});
                        }
                        for (const auto& [d, w] : tgt) {
                            if (!g.consFlag[d] || w == 0.0) continue;
                            auto& row = rowmap[H.mg->fine_dof((int)si, d)];  // added into the solver RHS
                            for (int64_t k = Tp.ptr[r]; k < Tp.ptr[r + 1]; ++k)
                                row.push_back({(int32_t)(H.oS + sd.roff + Tp.col[k]), w * Tp.val[k]});
                            for (int64_t k = T.ptr[r]; k < T.ptr[r + 1]; ++k)
                                row.push_back({(int32_t)(H.oS + H.R + sd.roff + T.col[k]), -w * T.val[k]});
                        }
                    }
                }
            }
        }
        std::vector<int32_t> crow;
        std::vector<int64_t> cptr{0};
        std::vector<int32_t> ccol;
        std::vector<double> cval;
        for (auto& kv : rowmap) {
            crow.push_back((int32_t)kv.first);
            // merge duplicate columns (hanging rows folded onto the same free dof)
            std::stable_sort(kv.second.begin(), kv.second.end(),
                             [](const auto& a, const auto& b) { return a.first < b.first; });
            for (size_t e = 0; e < kv.second.size();) {
                size_t f = e;
                double v = 0.0;
                for (; f < kv.second.size() && kv.second[f].first == kv.second[e].first; ++f) v += kv.second[f].second;
                ccol.push_back(kv.second[e].first);
                cval.push_back(v);
                e = f;
            }
            cptr.push_back((int64_t)ccol.size());
        }
        H.ncrow = (int64_t)crow.size();
        {
            // k_cpl: entries, the row's target index and pointer, b read + written, W's aux and
            // lambda entries once
            std::vector<int32_t> uc(ccol);
            std::sort(uc.begin(), uc.end());
            const double uniq = (double)(std::unique(uc.begin(), uc.end()) - uc.begin());
            H.bytes_rhs += 12.0 * (double)ccol.size() + 28.0 * (double)H.ncrow + 8.0 * uniq;
        }
        H.crow.upload(crow);
        H.cptr.upload(cptr);
        H.ccol.upload(ccol);
        H.cval.upload(cval);
    }
    // ---- hanging-level values over u: one SELL-64 product (rows of prolOper[maxiLeve])
    if (H.NH) {
        Rows rh(H.NH);
        for (const auto& S : H.subs) {
            const Csr& Hp = mc.multGrid[S.tv].hangProl;
            for (int64_t r = 0; r < S.nh; ++r)
                for (int64_t k = Hp.ptr[r]; k < Hp.ptr[r + 1]; ++k) rh[S.hoff + r].push_back({S.wcol(Hp.col[k], H.oH), Hp.val[k]});
        }
        H.op_hang.build(rh);
    }
    // per-ADMM-iteration byte model of the launches outside the PCG, mass CG and coarse space
    {
        double nu = 0.0, rows = 0.0;
        for (auto& S : H.subs) nu += 3.0 * (double)S.nn + (double)S.nh;
        for (auto& sd : H.sides) rows += (double)sd.m;
        double fine_nodes = 0.0;
        for (auto& S : H.subs) fine_nodes += (double)S.nn;
        // consForc copied into b (16 B per dof), k_outp (x, presc read, u written, mask, node map:
        // 77 B per node), the hanging rows
        H.bytes_rhs += 16.0 * 3.0 * fine_nodes + 77.0 * fine_nodes + (H.NH ? H.op_hang.bytes : 0.0);
        // interface: gamma (stored rows + the constant), factored per-ip kernels, projection,
        // the aux / lambda right-hand sides, the fused update (or the lambda add)
        H.bytes_iface += H.op_gamma.nch ? H.op_gamma.bytes + 8.0 * (double)H.op_gamma.nrow : 0.0;
        // side-1 halves of rank-local interfaces: their rows, then gamma read + written and the half read
        H.bytes_iface += H.op_gamma1.nch ? H.op_gamma1.bytes + 28.0 * (double)H.gam1_dst.n : 0.0;
        for (auto& F : H.fitfs) H.bytes_iface += F.bytes_gamma + (H.fused ? F.bytes_inpo : 0.0);
        for (auto& I : H.itfs)
            if (I.mine) H.bytes_iface += (double)(I.mip / I.comp) * (16.0 * I.comp + 4.0) + (I.cross ? 24.0 * I.mip : 0.0);
        if (H.fused) H.bytes_iface += H.op_wv.bytes + 56.0 * rows;
        else if (!H.sides.empty()) H.bytes_iface += H.op_aux.bytes + H.op_lam.bytes + 24.0 * rows;
        // MONITOR: snapshots of u and [aux, lambda] (read + written), the pair norms (16 B per entry)
        H.bytes_moni = 16.0 * (nu + 2.0 * rows) + 16.0 * (nu + 2.0 * rows);
    }
    // monitor norms [2 nsub u | 8 nint aux, lambda | 2 nsub hanging-level parts of u]
    const int64_t nmon = 4 * H.nsub + 8 * H.nint;
    H.moni.alloc(nmon);
    H.moni_host.assign(nmon, 0.0);
    H.moniReco.assign(H.nsub + 4 * H.nint, std::vector<double>(10, 0.0));
    DDPCA_HIP(hipStreamSynchronize(H.main));
}

// ---- DOUBLE_M_1 (MCONTACT.h:2303-2341): level l of the coarse hierarchy (l = Lc = max doleMcsc is
// globCoup_1 itself) holds level max(0, doleMcsc[tv] - (Lc - l)) of every subdomain; the transfer
// below it is each subdomain's realProl at that level (identity where a subdomain has reached its
// level 0), and the level operators are Galerkin products.  Nodes are numbered so that every level
// is a prefix of the next (the layout MgpisDevice takes): level l = level l-1's nodes, then the new
// nodes of every subdomain in order.  Needs every subdomain's coarse rows on this rank.
void plan_coarse_mg(const MCONTACT& mc, CoarseDev& C) {
    const CoarseSpace& cs = mc.coarse;
    const int64_t nsub = (int64_t)mc.multGrid.size(), n = C.n;
    CoarseDev::MgPlan& PL = C.plan;
    const int64_t Lc = *std::max_element(mc.doleMcsc.begin(), mc.doleMcsc.end());
    auto lev = [&](int64_t tv, int64_t l) { return std::max<int64_t>(0, mc.doleMcsc[tv] - (Lc - l)); };
    std::vector<std::vector<std::vector<int64_t>>> gid(Lc + 1, std::vector<std::vector<int64_t>>(nsub));
    // LATIN (DOUBLE_M, MCONTACT.h:1538-1670): the coarse contact unknowns of every interface are a
    // group of their own -- at level Lc the level-doleMcsc nodes coarNode[ts] of contBody[ts][0],
    // one level down the columns its scalProl rows touch (ficoCotr), comp unknowns per node
    // (the node's first dof for frictionless contact).  The sets need not be nested: a node of
    // level l - 1 that level l does not carry (stacked bodies: BLOCK) keeps the prefix layout as a
    // masked copy on level l and above (per-level dof flags, SubdomainOps::dof_free_lev) -- the
    // masked transfer C_l P C_{l-1}^T then is the reference's ficoCotr
    const int64_t nint = cs.latin ? (int64_t)mc.searCont.size() : 0;
    if (cs.latin && (int64_t)cs.coarNode.size() != nint)
        throw ApiError(DDPCA_EINVAL, "DOUBLE_M for the LATIN coarse space needs the coarse contact nodes (coarNode)");
    std::vector<std::vector<std::vector<int64_t>>> cset(Lc + 1, std::vector<std::vector<int64_t>>(nint));
    for (int64_t ts = 0; ts < nint; ++ts) {
        const int64_t b0 = mc.searCont[ts].body[0];
        const MULTIGRID& g = mc.multGrid[b0];
        cset[Lc][ts] = cs.coarNode[ts];
        for (int64_t l = Lc; l >= 1; --l) {
            const int64_t fl = mc.doleMcsc[b0] - (Lc - l);  // the group's node level at l
            if (fl - 1 < 0) {
                cset[l - 1][ts] = cset[l][ts];
                continue;
            }
            const Stencil& Sp = g.scalProl[fl - 1];  // scalar, no rotations (MCONTACT.h:1553)
            if (!Sp.bent.empty())
                throw ApiError(DDPCA_EINVAL, "LATIN DOUBLE_M: ficoCotr needs the scalar scalProl (a caller's rotated realProl has none)");
            std::vector<int64_t> cols;
            for (int64_t f : cset[l][ts])
                for (int64_t k = Sp.ptr[f]; k < Sp.ptr[f + 1]; ++k) cols.push_back(Sp.col[k]);
            std::sort(cols.begin(), cols.end());
            cols.erase(std::unique(cols.begin(), cols.end()), cols.end());
            cset[l - 1][ts] = cols;
        }
    }
    std::vector<std::unordered_map<int64_t, int64_t>> cg(nint);  // (interface, node) -> global node
    std::vector<int64_t> nglob(Lc + 1, 0);
    for (int64_t l = 0; l <= Lc; ++l) {
        int64_t cnt = l ? nglob[l - 1] : 0;
        for (int64_t tv = 0; tv < nsub; ++tv) {
            auto& v = gid[l][tv];
            v.resize(mc.multGrid[tv].leveCount[lev(tv, l)]);
            int64_t keep = 0;
            if (l) {
                keep = (int64_t)gid[l - 1][tv].size();
                std::copy(gid[l - 1][tv].begin(), gid[l - 1][tv].end(), v.begin());
            }
            for (int64_t j = keep; j < (int64_t)v.size(); ++j) v[j] = cnt++;
        }
        for (int64_t ts = 0; ts < nint; ++ts)
            for (int64_t node : cset[l][ts])
                if (cg[ts].emplace(node, cnt).second) ++cnt;
        nglob[l] = cnt;
    }
    std::vector<Stencil> S(Lc);
    for (int64_t l = 1; l <= Lc; ++l) {
        std::vector<std::vector<std::pair<int32_t, double>>> rows(nglob[l]);
        for (int64_t i = 0; i < nglob[l - 1]; ++i) rows[i].push_back({(int32_t)i, 1.0});
        std::vector<std::vector<std::array<double, 9>>> rblk(nglob[l]);  // block entries, parallel to rows (NaN-free marker below)
        for (int64_t tv = 0; tv < nsub; ++tv) {
            if (lev(tv, l) == lev(tv, l - 1)) continue;  // identity (MCONTACT.h:2325-2331)
            // the subdomain's realProl at that level (MCONTACT.h:1632, 2316): prolOper's rotation
            // blocks as block entries (a caller's operator-level stencil carries them in scalProl)
            const MULTIGRID& g = mc.multGrid[tv];
            const Stencil& Sp = g.prolOper.empty() ? g.scalProl[lev(tv, l - 1)] : g.prolOper[lev(tv, l - 1)];
            std::vector<int64_t> bo(Sp.col.size(), -1);
            for (size_t q = 0; q < Sp.bent.size(); ++q) bo[Sp.bent[q]] = (int64_t)q;
            for (int64_t j = (int64_t)gid[l - 1][tv].size(); j < (int64_t)gid[l][tv].size(); ++j)
                for (int64_t k = Sp.ptr[j]; k < Sp.ptr[j + 1]; ++k) {
                    const int64_t r = gid[l][tv][j];
                    rows[r].push_back({(int32_t)gid[l - 1][tv][Sp.col[k]], Sp.w[k]});
                    std::array<double, 9> b;
                    if (bo[k] >= 0) std::copy(&Sp.bval[9 * bo[k]], &Sp.bval[9 * bo[k]] + 9, b.begin());
                    else b[0] = std::numeric_limits<double>::quiet_NaN();  // scalar entry
                    rblk[r].resize(rows[r].size());
                    rblk[r].back() = b;
                }
        }
        for (int64_t ts = 0; ts < nint; ++ts) {  // ficoCotr rows of the nodes new on level l
            const int64_t b0 = mc.searCont[ts].body[0];
            const int64_t fl = mc.doleMcsc[b0] - (Lc - l);
            if (fl - 1 < 0) continue;
            const Stencil& Sp = mc.multGrid[b0].scalProl[fl - 1];
            for (int64_t f : cset[l][ts]) {
                if (std::binary_search(cset[l - 1][ts].begin(), cset[l - 1][ts].end(), f)) continue;  // coarse copy
                auto& row = rows[cg[ts].at(f)];
                for (int64_t k = Sp.ptr[f]; k < Sp.ptr[f + 1]; ++k) row.push_back({(int32_t)cg[ts].at(Sp.col[k]), Sp.w[k]});
            }
        }
        Stencil& T = S[l - 1];
        T.nf = nglob[l];
        T.nc = nglob[l - 1];
        T.ptr.assign(1, 0);
        for (int64_t r = 0; r < nglob[l]; ++r) {
            for (size_t q = 0; q < rows[r].size(); ++q) {
                const bool blk = q < rblk[r].size() && !std::isnan(rblk[r][q][0]);
                if (blk) {
                    T.bent.push_back((int64_t)T.col.size());
                    T.bval.insert(T.bval.end(), rblk[r][q].begin(), rblk[r][q].end());
                }
                T.col.push_back(rows[r][q].first);
                T.w.push_back(blk ? 0.0 : rows[r][q].second);
            }
            T.ptr.push_back((int64_t)T.col.size());
        }
    }
    // globCoup(_1) rows: subdomain tv's level-doleMcsc free dofs in increasing order (consOper),
    // then (LATIN) every interface's coarse contact unknowns, comp per node
    std::vector<int32_t> fdg(n);
    for (int64_t tv = 0; tv < nsub; ++tv) {
        const MULTIGRID& g = mc.multGrid[tv];
        int64_t r = cs.baseReco[tv];
        for (int64_t dof = 0; dof < 3 * g.leveCount[mc.doleMcsc[tv]]; ++dof)
            if (g.consFlag[dof]) fdg[r++] = (int32_t)(3 * gid[Lc][tv][dof / 3] + dof % 3);
        if (r != cs.baseReco[tv + 1]) throw ApiError(DDPCA_EINVAL, "DOUBLE_M: baseReco does not match the free dofs");
    }
    {
        int64_t r = cs.baseReco[nsub];
        for (int64_t ts = 0; ts < nint; ++ts) {
            const int comp = mc.searCont[ts].comp();
            for (int64_t node : cset[Lc][ts])
                for (int j = 0; j < comp; ++j) fdg[r++] = (int32_t)(3 * cg[ts].at(node) + j);
        }
        if (r != n) throw ApiError(DDPCA_EINVAL, "DOUBLE_M: coarse contact unknowns do not match the coarse rows");
    }
    // per-level dof flags: a subdomain node's dofs as its consOper (the prefix of its flags), a
    // contact unknown's comp dofs free on the levels that carry it, its masked copies none
    std::vector<std::vector<uint8_t>> flev(Lc + 1);
    for (int64_t l = 0; l <= Lc; ++l) {
        auto& f = flev[l];
        f.assign(3 * nglob[l], 0);
        for (int64_t tv = 0; tv < nsub; ++tv) {
            const MULTIGRID& g = mc.multGrid[tv];
            for (size_t j = 0; j < gid[l][tv].size(); ++j)
                for (int a = 0; a < 3; ++a) f[3 * gid[l][tv][j] + a] = g.consFlag[3 * j + a];
        }
        for (int64_t ts = 0; ts < nint; ++ts) {
            const int comp = mc.searCont[ts].comp();
            for (int64_t node : cset[l][ts])
                for (int j = 0; j < comp; ++j) f[3 * cg[ts].at(node) + j] = 1;
        }
    }
    for (int32_t d : fdg)
        if (!flev[Lc][d]) throw ApiError(DDPCA_EINVAL, "DOUBLE_M: a coarse row on a constrained dof");
    PL.nglob = std::move(nglob);
    PL.S = std::move(S);
    PL.fdg = std::move(fdg);
    PL.flev = std::move(flev);
    PL.latin = cs.latin;
}

// The coarse MGPIS from the plan and the whole coarse operator A (globCoup_1 / globCoup):
// K[Lc] = A on the hierarchy's fine level, the levels below Galerkin products (MCONTACT.h:
// 1664-1665, 2337-2338)
void finish_coarse_mg(ddpca_mcontact& H, CoarseDev& C, const Csr& A) {
    CoarseDev::MgPlan& PL = C.plan;
    const int64_t n = C.n, Lc = (int64_t)PL.nglob.size() - 1;
    if (A.nrow != n || A.ncol != n) throw ApiError(DDPCA_EINVAL, "DOUBLE_M coarse solve: the whole coarse operator is needed");
    std::vector<Bsr3> K(Lc + 1);
    K[Lc] = condensed_to_bsr3(PL.nglob[Lc], n, PL.fdg.data(), A.ptr.data(), A.col.data(), A.val.data());
    for (int64_t l = Lc - 1; l >= 0; --l) K[l] = galerkin_rap(K[l + 1], PL.S[l]);
    SubdomainOps o;
    o.nnodes = PL.nglob;
    for (const auto& k : K) o.K.push_back(&k);
    for (const auto& s : PL.S) o.S.push_back(&s);
    o.dof_free = PL.flev[Lc].data();
    for (const auto& f : PL.flev) o.dof_free_lev.push_back(f.data());
    C.cmg = std::make_unique<MgpisDevice>(H.device, std::vector<SubdomainOps>{o}, H.opt);
    std::vector<int32_t> perm(n), own(C.own_rows.begin(), C.own_rows.end());
    for (int64_t r = 0; r < n; ++r) perm[r] = (int32_t)C.cmg->fine_dof(0, PL.fdg[r]);
    C.cperm.upload(perm);
    C.cown.upload(own.empty() ? std::vector<int32_t>{0} : own);
    DDPCA_HIP(hipEventCreateWithFlags(&C.ev_in, hipEventDisableTiming));
    DDPCA_HIP(hipEventCreateWithFlags(&C.ev_out, hipEventDisableTiming));
    if (std::getenv("DDPCA_VERBOSE"))
        std::fprintf(stderr, "[ddpca] DOUBLE_M%s coarse solve: %ld rows, %ld levels%s\n", PL.latin ? "" : "_1", (long)n,
                     (long)(Lc + 1), C.mg_gather ? " (operator gathered from every rank)" : "");
    CoarseDev::MgPlan().swap_into(PL);
}

// ---- coarse space: device operands from the host MULTISCALE_1 output
void build_coarse(ddpca_mcontact& H, Problem& P) {
    MCONTACT& mc = P.mc;
    const CoarseSpace& cs = mc.coarse;
    CoarseDev& C = H.cs;
    if (!(mc.muscSett & 3)) return;
    if (!cs.ready) throw ApiError(DDPCA_ESTATE, "muscSett set but the coarse space was not built");
    C.on = true;
    C.n = cs.n;
    const int64_t n = C.n;
    std::vector<int64_t> xoff(H.subs.size());
    for (size_t i = 0; i < H.subs.size(); ++i) {
        const int64_t tv = H.subs[i].tv;
        if (!cs.built[tv]) throw ApiError(DDPCA_ESTATE, "coarse rows of an owned subdomain were not built");
        xoff[i] = (int64_t)C.own_rows.size();
        for (int64_t r = cs.baseReco[tv]; r < cs.baseReco[tv + 1]; ++r) C.own_rows.push_back(r);
    }
    C.nown = (int64_t)C.own_rows.size();
    // ---- the right-hand side in per-source slots.  Row r of the coarse right-hand side sums
    // contributions of several subdomains (its own u and lambda, its interface mates' through
    // globTran_1 / globTran_S; LATIN's contact rows both bodies of the interface), and every source
    // subdomain lives on exactly one rank.  Summing the row over this rank's W columns and then
    // all-reducing across ranks would round differently for every rank layout; instead every row
    // has one slot per structurally possible source (the same layout on every rank: itself and its
    // interface mates, for LATIN's contact rows both bodies), each slot is summed in a fixed,
    // layout-independent order by its source's owner (the other ranks contribute exact zeros to
    // it), the slots are all-reduced, and k_slot_sum adds a row's slots in ascending source order.
    // The coarse right-hand side -- and so the whole trajectory -- is then the same bits on any
    // number of ranks (tests/test_mcontact_gpu.py: resuMoni rows of the multi-rank runs).
    const int64_t nsg = (int64_t)cs.baseReco.size() - 1, nbase = cs.baseReco.back();
    std::vector<std::vector<int64_t>> srcs(n);
    {
        std::vector<std::vector<int64_t>> nbr(nsg);
        std::vector<int64_t> bodies;
        for (int64_t tv = 0; tv < nsg; ++tv) nbr[tv].push_back(tv);
        for (const auto& itf : mc.searCont) {
            nbr[itf.body[0]].push_back(itf.body[1]);
            nbr[itf.body[1]].push_back(itf.body[0]);
            bodies.push_back(itf.body[0]);
            bodies.push_back(itf.body[1]);
        }
        auto uniq = [](std::vector<int64_t>& v) {
            std::sort(v.begin(), v.end());
            v.erase(std::unique(v.begin(), v.end()), v.end());
        };
        for (auto& v : nbr) uniq(v);
        uniq(bodies);
        for (int64_t tv = 0; tv < nsg; ++tv)
            for (int64_t r = cs.baseReco[tv]; r < cs.baseReco[tv + 1]; ++r) srcs[r] = nbr[tv];
        // LATIN's coarse contact unknowns: rows of interface ts take its two bodies when the
        // unknowns are known per interface (coarNode), else every body of an interface
        int64_t known = 0;
        for (int64_t ts = 0; ts < (int64_t)cs.coarNode.size(); ++ts)
            known += mc.searCont[ts].comp() * (int64_t)cs.coarNode[ts].size();
        if (cs.coarNode.size() == mc.searCont.size() && nbase + known == n) {
            int64_t r = nbase;
            for (int64_t ts = 0; ts < (int64_t)cs.coarNode.size(); ++ts) {
                std::vector<int64_t> b{mc.searCont[ts].body[0], mc.searCont[ts].body[1]};
                uniq(b);
                for (int64_t q = 0; q < mc.searCont[ts].comp() * (int64_t)cs.coarNode[ts].size(); ++q) srcs[r++] = b;
            }
        } else {
            for (int64_t r = nbase; r < n; ++r) srcs[r] = bodies;
        }
    }
    std::vector<int64_t> sptr(n + 1, 0);
    for (int64_t r = 0; r < n; ++r) sptr[r + 1] = sptr[r] + (int64_t)srcs[r].size();
    C.nslot = sptr[n];
    auto slot_of = [&](int64_t r, int64_t tv) {
        const auto& v = srcs[r];
        const auto it = std::lower_bound(v.begin(), v.end(), tv);
        if (it == v.end() || *it != tv)
            throw ApiError(DDPCA_EINVAL, "coarse right-hand side: row " + std::to_string(r) + " has an entry of subdomain " +
                                             std::to_string(tv) + ", which is not on the row's interface graph");
        return sptr[r] + (int64_t)(it - v.begin());
    };
    // RHS entries over W: + globTran_1 (owned sides, lambda columns), - interface part of
    // globTran_D_1 (owned subdomains, u columns); LATIN + globTran lambda - globTran_pena aux +
    // globTran_D u.  Sort key inside a slot: (segment, global side, column in the source's own
    // numbering) -- none of it depends on where the source's columns sit in this rank's W
    struct Ent {
        int64_t seg, side, lcol;
        int32_t wc;
        double v;
        bool operator<(const Ent& o) const {
            return seg != o.seg ? seg < o.seg : side != o.side ? side < o.side : lcol < o.lcol;
        }
    };
    std::vector<std::vector<Ent>> ents(C.nslot);
    auto put = [&](int64_t r, int64_t tv, Ent e) { ents[slot_of(r, tv)].push_back(e); };
    for (const auto& sd : H.sides) {
        const int64_t lam0 = H.oS + H.R + sd.roff, aux0 = H.oS + sd.roff, sg = 2 * sd.ts + sd.s;
        const auto& Su = H.subs[sd.sub];
        auto add_rows = [&](const Csr& T, int64_t seg, int64_t c0, double sgn, bool ucol) {
            for (int64_t r = 0; r < T.nrow; ++r)
                for (int64_t k = T.ptr[r]; k < T.ptr[r + 1]; ++k)
                    put(r, sd.tv, Ent{seg, sg, T.col[k], (int32_t)(ucol ? Su.wcol(T.col[k], H.oH) : c0 + T.col[k]), sgn * T.val[k]});
        };
        if (cs.latin) {  // (MCONTACT.h:2540-2548)
            add_rows(cs.globTran_D_L[sd.ts][sd.s], 1, 0, 1.0, true);
            add_rows(cs.globTran_pena_L[sd.ts][sd.s], 2, aux0, -1.0, false);
            add_rows(cs.globTran_L[sd.ts][sd.s], 3, lam0, 1.0, false);
        } else {
            add_rows(cs.globTran_1[sd.ts][sd.s], 3, lam0, 1.0, false);
        }
    }
    for (size_t i = 0; i < H.subs.size() && !cs.latin; ++i) {
        // factored: the interface part (the stiffness part is the SpMV + restriction chain);
        // assembled: the caller's whole globTran_D_1
        const Csr& T = cs.assembled ? cs.globTran_D_full[H.subs[i].tv] : cs.globTran_S[H.subs[i].tv];
        const auto& Su = H.subs[i];
        for (int64_t r = 0; r < T.nrow; ++r)
            for (int64_t k = T.ptr[r]; k < T.ptr[r + 1]; ++k)
                put(r, Su.tv, Ent{0, 0, T.col[k], (int32_t)Su.wcol(T.col[k], H.oH), -T.val[k]});
    }
    {
        std::vector<int64_t> ptr(C.nslot + 1, 0);
        std::vector<int32_t> col;
        std::vector<double> val;
        for (int64_t q = 0; q < C.nslot; ++q) {
            auto& e = ents[q];
            std::stable_sort(e.begin(), e.end());
            for (const auto& x : e) {
                col.push_back(x.wc);
                val.push_back(x.v);
            }
            ptr[q + 1] = (int64_t)col.size();
            std::vector<Ent>().swap(e);
        }
        C.rptr.upload(ptr);
        C.rcol.upload(col.empty() ? std::vector<int32_t>{0} : col);
        C.rval.upload(val.empty() ? std::vector<double>{0.0} : val);
        C.sptr.upload(sptr);
        // right-hand side CSR over W: entries, each distinct W entry once, f0 read and the slot
        // written; the slot sum reads the slots and row pointers and writes g
        std::vector<int32_t> uc(col);
        std::sort(uc.begin(), uc.end());
        const double uniq = (double)(std::unique(uc.begin(), uc.end()) - uc.begin());
        C.bytes_iter = 12.0 * (double)col.size() + 8.0 * uniq + 16.0 * (double)C.nslot +
                       8.0 * (double)C.nslot + 16.0 * (double)n;
    }
    // globForc_1 enters the slot of the row's own subdomain (the rank that owns the row)
    std::vector<double> f0(std::max<int64_t>(C.nslot, 1), 0.0);
    for (size_t i = 0; i < H.subs.size(); ++i)
        for (int64_t r = cs.baseReco[H.subs[i].tv]; r < cs.baseReco[H.subs[i].tv + 1]; ++r)
            f0[slot_of(r, H.subs[i].tv)] = cs.globForc_1[r];
    C.f0.upload(f0);
    C.gs.alloc(std::max<int64_t>(C.nslot, 1));
    C.g.alloc(std::max<int64_t>(n, 1));
    C.xc.alloc(std::max<int64_t>(C.nown, 1));
    // the reference solves globCoup_1 directly below DIRE_MAXI = 120000 rows and with its DOUBLE_M_1
    // MGPIS above (PREP.h:69, MCONTACT.h:1857-1865); DDPCA_COARSE_MG_MIN moves the switch (tests).
    // The direct solve here is a dense explicit inverse, n^2 8 B on every rank and streamed by the
    // GEMV every ADMM iteration, so it is also bounded by memory: above DDPCA_COARSE_DENSE_MB
    // (default 1024 MiB, n ~ 11,600 rows) the multigrid solve takes over below DIRE_MAXI too --
    // where the inverse would cost ~0.2 ms of HBM streaming per iteration and grow as n^2
    const char* mg_env = std::getenv("DDPCA_COARSE_MG_MIN");
    const char* dense_env = std::getenv("DDPCA_COARSE_DENSE_MB");
    const double dense_max = (dense_env ? std::atof(dense_env) : 1024.0) * 1048576.0;
    C.dense_bytes = 8.0 * (double)n * (double)n;
    // LATIN: DOUBLE_M (MCONTACT.h:1236) on the coarse contact nodes (the host MULTISCALE's, or the
    // caller's through ddpca_problem_set_coarse_nodes)
    if (cs.latin && cs.coarNode.empty() && (n >= (mg_env ? std::atoll(mg_env) : 120000) || C.dense_bytes > dense_max))
        throw ApiError(DDPCA_EINVAL, "LATIN coarse space past the dense solve's limits needs its coarse contact nodes "
                                     "(ddpca_problem_set_coarse_nodes) for DOUBLE_M");
    const bool by_rows = n >= (mg_env ? std::atoll(mg_env) : 120000);
    const bool by_budget = C.dense_bytes > dense_max;  // the same decision on every rank: n is global
    C.mg = by_rows || by_budget;
    C.latin = cs.latin;
    // the multigrid hierarchy needs the whole coarse operator: a caller's full operator or a
    // single-rank build has it; a rank-local build gathers it from every rank once the transport
    // exists (coarse_invert)
    bool full = !cs.rank_local;
    for (int64_t tv = 0; tv < (int64_t)cs.built.size(); ++tv) full = full && cs.built[tv];
    if (C.mg && !full && H.nranks == 1)
        throw ApiError(DDPCA_ESTATE, "DOUBLE_M coarse solve: a single rank without every subdomain's coarse rows");
    C.mg_gather = C.mg && !full;
    if (C.mg && H.mg) {
        plan_coarse_mg(mc, C);
        if (!C.mg_gather) finish_coarse_mg(H, C, cs.globCoup_1);
        else C.gathered_rows = cs.globCoup_1;  // this rank's rows (its share of the contact rows)
    }
    // coarse solve: the owned rows of the dense inverse against g, or (DOUBLE_M) g scattered into
    // the coarse MGPIS and its owned rows gathered back (its PCG is counted by its own model)
    C.bytes_iter += C.mg ? 20.0 * (double)n + 24.0 * (double)C.nown
                         : 8.0 * (double)C.nown * (double)n + 8.0 * (double)n + 8.0 * (double)C.nown;
    if (!C.mg) {
        // dense rows of globCoup_1 (inverted once every rank holds all rows)
        C.dense.assign((size_t)n * n, 0.0);
        std::vector<int64_t> fill_rows = C.own_rows;
        // the coarse contact unknowns' rows: a caller's full operator is filled by rank 0 only; a
        // rank-local host build holds each rank's share (the all-reduce sums them)
        if (cs.latin && (cs.rank_local || H.rank == 0))
            for (int64_t r = cs.baseReco.back(); r < n; ++r) fill_rows.push_back(r);
        for (int64_t r : fill_rows)
            for (int64_t k = cs.globCoup_1.ptr[r]; k < cs.globCoup_1.ptr[r + 1]; ++k)
                C.dense[(size_t)r * n + cs.globCoup_1.col[k]] = cs.globCoup_1.val[k];
    }
    if (!H.mg) return;
    C.assembled = cs.assembled;
    if (cs.assembled) {
        std::vector<int64_t> ptr{0};
        std::vector<int32_t> col, tgt, cd;
        std::vector<double> val;
        for (size_t i = 0; i < H.subs.size(); ++i) {
            const int64_t tv = H.subs[i].tv;
            const MULTIGRID& g = mc.multGrid[tv];
            const Csr& A = cs.accuProl_full[tv];
            std::vector<int64_t> f2d(g.freeCount.back(), -1);
            for (int64_t d = 0; d < 3 * g.leveCount.back(); ++d)  // the fine level (not the hanging one)
                if (g.freeIndex[d] >= 0) f2d[g.freeIndex[d]] = d;
                else cd.push_back((int32_t)(H.subs[i].dof0 + d));
            for (int64_t r = 0; r < A.nrow; ++r) {
                for (int64_t k = A.ptr[r]; k < A.ptr[r + 1]; ++k) {
                    col.push_back((int32_t)(xoff[i] + A.col[k]));
                    val.push_back(A.val[k]);
                }
                ptr.push_back((int64_t)col.size());
                tgt.push_back((int32_t)(H.subs[i].dof0 + f2d[r]));
            }
        }
        C.npr = (int64_t)tgt.size();
        C.ncd = (int64_t)cd.size();
        // u += accuProl x_c on the free rows (entries, target index, u read + written), the
        // constrained rows' prescribed values again
        C.bytes_iter += 12.0 * (double)col.size() + 20.0 * (double)C.npr + 28.0 * (double)C.ncd;
        C.pptr.upload(ptr);
        C.pcol.upload(col.empty() ? std::vector<int32_t>{0} : col);
        C.pval.upload(val.empty() ? std::vector<double>{0.0} : val);
        C.ptgt.upload(tgt.empty() ? std::vector<int32_t>{0} : tgt);
        C.cdof.upload(cd.empty() ? std::vector<int32_t>{0} : cd);
        return;
    }
    MgpisDevice& D = *H.mg;
    const int L = (int)D.lev.size() - 1;
    // stiffness part: gather level-d device values into the owned coarse rows
    C.dmin = L;
    std::map<int, std::pair<std::vector<int32_t>, std::vector<int64_t>>> groups;
    std::vector<int64_t> xnoff(H.subs.size(), 0);
    int64_t nxn = 0;
    for (size_t i = 0; i < H.subs.size(); ++i) {
        const int64_t tv = H.subs[i].tv;
        const MULTIGRID& g = mc.multGrid[tv];
        const int d = (int)mc.doleMcsc[tv];
        if (g.maxiLeve != L) throw ApiError(DDPCA_EINVAL, "batched subdomains need equal level counts");
        C.dmin = std::min(C.dmin, d);
        auto& grp = groups[d];
        const auto& perm = D.level_perm[d][i];
        for (int64_t dof = 0; dof < 3 * g.leveCount[d]; ++dof) {
            const int32_t fi = g.freeIndex[dof];
            if (fi < 0) continue;
            grp.first.push_back((int32_t)slot_of(cs.baseReco[tv] + fi, tv));  // the row's own slot
            grp.second.push_back(3 * (D.lev[d].noff[i] + perm[dof / 3]) + dof % 3);
        }
        xnoff[i] = nxn;
        nxn += 3 * g.leveCount[d];
    }
    for (auto& kv : groups) {
        CoarseDev::KGroup G;
        G.level = kv.first;
        G.rows.upload(kv.second.first);
        G.src.upload(kv.second.second);
        C.kg.push_back(std::move(G));
    }
    // xn <- xc, and the accumulated prolongation (fine node -> level-d node) per batch node
    C.nxn = nxn;
    std::vector<int32_t> xsrc(std::max<int64_t>(nxn, 1), -1);
    C.qnn = D.lev.back().nn;
    std::vector<int32_t> qcol(8 * C.qnn, -1);
    std::vector<double> qw(8 * C.qnn, 0.0);
    std::vector<uint8_t> flag(H.NU, 0);
    std::vector<int64_t> hptr{0};
    std::vector<int32_t> hcol, htgt;
    std::vector<double> hval;
    for (size_t i = 0; i < H.subs.size(); ++i) {
        const int64_t tv = H.subs[i].tv;
        const MULTIGRID& g = mc.multGrid[tv];
        const int d = (int)mc.doleMcsc[tv];
        for (int64_t dof = 0; dof < 3 * g.leveCount[d]; ++dof) {
            const int32_t fi = g.freeIndex[dof];
            xsrc[xnoff[i] + dof] = fi < 0 ? -1 : (int32_t)(xoff[i] + fi);
        }
        const Stencil& Q = cs.accuQ[tv];
        const int64_t b0 = H.subs[i].dof0 / 3;
        std::vector<int64_t> bo(Q.col.size(), -1);
        for (size_t q = 0; q < Q.bent.size(); ++q) bo[Q.bent[q]] = (int64_t)q;
        for (int64_t nd = 0; nd < Q.nf; ++nd) {
            const int64_t len = Q.ptr[nd + 1] - Q.ptr[nd];
            bool scalar = len <= 8;
            for (int64_t k = Q.ptr[nd]; k < Q.ptr[nd + 1] && scalar; ++k) scalar = bo[k] < 0;
            if (scalar) {
                for (int64_t k = 0; k < len; ++k) {
                    qcol[k * C.qnn + b0 + nd] = (int32_t)(xnoff[i] + 3 * Q.col[Q.ptr[nd] + k]);
                    qw[k * C.qnn + b0 + nd] = Q.w[Q.ptr[nd] + k];
                }
                continue;
            }
            // a CSR row per free dof over x_c (the scalar kernel adds 0 there and the prescribed
            // values of the node's constrained dofs)
            for (int a = 0; a < 3; ++a) {
                const int64_t dof = 3 * nd + a;
                if (!g.consFlag[dof]) continue;
                for (int64_t k = Q.ptr[nd]; k < Q.ptr[nd + 1]; ++k) {
                    const int64_t c = Q.col[k];
                    for (int b = 0; b < 3; ++b) {
                        if (bo[k] < 0 && b != a) continue;
                        const int32_t f = g.freeIndex[3 * c + b];
                        const double w = bo[k] < 0 ? Q.w[k] : Q.bval[9 * bo[k] + 3 * a + b];
                        if (f < 0 || w == 0.0) continue;
                        hcol.push_back((int32_t)(xoff[i] + f));
                        hval.push_back(w);
                    }
                }
                hptr.push_back((int64_t)hcol.size());
                htgt.push_back((int32_t)(H.subs[i].dof0 + dof));
            }
        }
        for (int64_t dof = 0; dof < 3 * g.leveCount.back(); ++dof) flag[H.subs[i].dof0 + dof] = g.consFlag[dof];
    }
    C.npr = (int64_t)htgt.size();
    C.ncd = 0;
    if (C.npr) {
        C.pptr.upload(hptr);
        C.pcol.upload(hcol.empty() ? std::vector<int32_t>{0} : hcol);
        C.pval.upload(hval.empty() ? std::vector<double>{0.0} : hval);
        C.ptgt.upload(htgt);
        C.bytes_iter += 12.0 * (double)hcol.size() + 20.0 * (double)C.npr;
    }
    C.xsrc.upload(xsrc);
    C.xn.alloc(std::max<int64_t>(nxn, 1));
    C.qcol.upload(qcol);
    C.qw.upload(qw);
    C.flag.upload(flag);
    // factored stiffness part and prolongation: K x = b - r (b, r read, the difference written:
    // 72 B per fine node), the plain restriction chain down to dmin (r_f once, mask + b_c per
    // coarse node, the lattice's child mask + fine copy or the stencil's index + weight), the
    // gather of level-d values into g, x_c scattered to nodal xn, and u += (Q (x) I3) xn: Q's
    // entries, flags, u read + written, xn once
    double nf = 0.0, qent = 0.0, kp = 0.0;
    for (size_t i = 0; i < H.subs.size(); ++i) {
        nf += (double)H.subs[i].nn;
        qent += (double)cs.accuQ[H.subs[i].tv].col.size();
        for (int l = L; l > C.dmin; --l) {
            const LevelDev& F = D.lev[l];
            kp += 24.0 * (double)F.nloc[i] + (25.0 + (F.lat ? 8.0 : 0.0)) * (double)D.lev[l - 1].nloc[i] +
                  (F.lat ? 0.0 : 12.0 * (double)F.tent_sub[i]);
        }
    }
    double krows = 0.0;
    for (auto& kv : groups) krows += (double)kv.second.first.size();
    C.bytes_iter += 72.0 * nf + kp + 36.0 * krows + 20.0 * (double)nxn + 12.0 * qent + 51.0 * nf + 8.0 * (double)nxn;
}

// globCoup_1^-1 rows of the owned subdomains: every rank's rows are summed into a full dense
// copy (one RCCL all-reduce at setup), factorised by rocSOLVER (potrf + potri) on the device
void coarse_invert(ddpca_mcontact& H) {
    CoarseDev& C = H.cs;
    if (!C.on || C.inverted) return;
    if (C.mg) {  // DOUBLE_M: nothing to factorise (the same decision on every rank: n is global)
        if (C.mg_gather) {
            // a rank-local build: every rank's rows (the LATIN contact rows as per-rank shares) as
            // (row, col, value) triplets, all-gathered by two all-reduces (the counts, then each
            // rank's triplets in its own slot); duplicates summed
            if (!H.comm) throw ApiError(DDPCA_ESTATE, "the DOUBLE_M coarse solve of a multi-rank run needs mcontact_gpu_comm_init");
            const Csr& M = C.gathered_rows;
            std::vector<double> cnt(H.nranks, 0.0);
            cnt[H.rank] = (double)M.nnz();
            DevBuf<double> dc;
            dc.upload(cnt);
            H.comm->allreduce_sum(dc.p, H.nranks, H.main);
            DDPCA_HIP(hipStreamSynchronize(H.main));
            cnt = dc.download();
            std::vector<int64_t> off(H.nranks + 1, 0);
            for (int r = 0; r < H.nranks; ++r) off[r + 1] = off[r] + (int64_t)cnt[r];
            std::vector<double> trip(3 * off[H.nranks], 0.0);
            for (int64_t r = 0, q = off[H.rank]; r < M.nrow; ++r)
                for (int64_t k = M.ptr[r]; k < M.ptr[r + 1]; ++k, ++q) {
                    trip[3 * q] = (double)r;
                    trip[3 * q + 1] = (double)M.col[k];
                    trip[3 * q + 2] = M.val[k];
                }
            DevBuf<double> dt;
            dt.upload(trip);
            H.comm->allreduce_sum(dt.p, (int64_t)trip.size(), H.main);
            DDPCA_HIP(hipStreamSynchronize(H.main));
            trip = dt.download();
            std::vector<std::vector<std::pair<int32_t, double>>> rows(C.n);
            for (int64_t q = 0; q < off[H.nranks]; ++q) rows[(int64_t)trip[3 * q]].push_back({(int32_t)trip[3 * q + 1], trip[3 * q + 2]});
            Csr A;
            A.nrow = A.ncol = C.n;
            A.ptr.assign(1, 0);
            for (auto& row : rows) {
                std::stable_sort(row.begin(), row.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
                for (size_t k = 0; k < row.size();) {
                    size_t e = k;
                    double v = 0.0;
                    for (; e < row.size() && row[e].first == row[k].first; ++e) v += row[e].second;
                    A.col.push_back(row[k].first);
                    A.val.push_back(v);
                    k = e;
                }
                A.ptr.push_back((int64_t)A.col.size());
            }
            C.gathered_rows = Csr();
            if (!C.plan.nglob.empty()) finish_coarse_mg(H, C, A);
        }
        C.inverted = true;
        return;
    }
    const int64_t n = C.n;
    if (n > 46000) throw ApiError(DDPCA_EINVAL, "coarse space too large for the dense inverse (n > 46000)");
    DevBuf<double> A;
    A.upload(C.dense);
    std::vector<double>().swap(C.dense);
    hipStream_t st = H.main;
    if (H.nranks > 1 && !H.comm) throw ApiError(DDPCA_ESTATE, "the coarse space of a multi-rank run needs mcontact_gpu_comm_init");
    const bool verbose = std::getenv("DDPCA_VERBOSE") != nullptr;
    auto checksum = [n](const std::vector<double>& v) {
        double a = 0.0, b = 0.0;
        for (int64_t i = 0; i < n * n; ++i) a += std::abs(v[i]), b += v[i] * (double)(i % 9973);
        return std::make_pair(a, b);
    };
    if (verbose) {
        const auto c = checksum(A.download());
        std::fprintf(stderr, "[ddpca] rank %d coarse rows %ld owned %ld: own part |.| %.17g w %.17g\n", H.rank, (long)n,
                     (long)C.nown, c.first, c.second);
    }
    if (H.comm) H.comm->allreduce_sum(A.p, n * n, st);
    if (verbose) {
        DDPCA_HIP(hipStreamSynchronize(st));
        const auto c = checksum(A.download());
        std::fprintf(stderr, "[ddpca] rank %d coarse matrix |.| %.17g w %.17g\n", H.rank, c.first, c.second);
    }
    auto solver_guard = solver_lock();
    rocblas_handle rh = nullptr;
    if (rocblas_create_handle(&rh) != rocblas_status_success) throw ApiError(DDPCA_EHIP, "rocblas_create_handle");
    DevBuf<rocblas_int> info(2);
    info.zero(st);
    rocblas_set_stream(rh, st);
    rocblas_status s1, s2;
    if (C.latin) {
        // globCoup (displacements + coarse contact unknowns) is symmetric but indefinite: pivoted
        // LU, then the inverse (symmetric again, so the row-major copy reads it as it is)
        DevBuf<rocblas_int> ipiv(std::max<int64_t>(n, 1));
        s1 = rocsolver_dgetrf(rh, (rocblas_int)n, (rocblas_int)n, A.p, (rocblas_int)n, ipiv.p, info.p);
        s2 = rocsolver_dgetri(rh, (rocblas_int)n, A.p, (rocblas_int)n, ipiv.p, info.p + 1);
        DDPCA_HIP(hipStreamSynchronize(st));
    } else {
        s1 = rocsolver_dpotrf(rh, rocblas_fill_lower, (rocblas_int)n, A.p, (rocblas_int)n, info.p);
        s2 = rocsolver_dpotri(rh, rocblas_fill_lower, (rocblas_int)n, A.p, (rocblas_int)n, info.p + 1);
        hipLaunchKernelGGL(k_fill_lower, dim3(std::max<int64_t>(1, ((int64_t)n * n + 255) / 256)), dim3(256), 0, st, A.p, n);
    }
    C.ainv.alloc(std::max<int64_t>(C.nown, 1) * n);
    // owned rows are contiguous per subdomain (baseReco blocks)
    for (size_t k = 0; k < C.own_rows.size();) {
        size_t e = k;
        while (e + 1 < C.own_rows.size() && C.own_rows[e + 1] == C.own_rows[e] + 1) ++e;
        DDPCA_HIP(hipMemcpyAsync(C.ainv.p + k * n, A.p + C.own_rows[k] * n, (e - k + 1) * n * sizeof(double),
                                 hipMemcpyDeviceToDevice, st));
        k = e + 1;
    }
    DDPCA_HIP(hipStreamSynchronize(st));
    rocblas_destroy_handle(rh);
    const auto inf = info.download();
    if (s1 != rocblas_status_success || s2 != rocblas_status_success)
        throw ApiError(DDPCA_EHIP, "rocsolver potrf/potri failed on globCoup_1");
    if (inf[0] != 0 || inf[1] != 0)
        throw ApiError(DDPCA_ENUMERIC, std::string(C.latin ? "globCoup is singular (getrf" : "globCoup_1 is not positive definite (potrf") +
                                           " info " + std::to_string(inf[0]) + ")");
    C.inverted = true;
}

// One coarse-space correction (MCONTACT.h:2578-2612) on the stream, after k_outp wrote u.
void coarse_correct(ddpca_mcontact& H) {
    CoarseDev& C = H.cs;
    if (!C.inverted) throw ApiError(DDPCA_ESTATE, "coarse space not factorised (multi-rank runs: comm_init first)");
    hipStream_t st = H.main;
    const int64_t n = C.n;
    if (H.mg && !C.assembled) {
        MgpisDevice& D = *H.mg;
        const int L = (int)D.lev.size() - 1;
        // consStif[L] x on every owned subdomain, then realProl^T down to level doleMcsc.  K x is
        // b - r with PCG's recursive residual r: it meets the true one to the PCG accuracy (the
        // reference's own CG_SOLV leaves a true residual of 1e-10 |b| behind its 1e-14 recursive
        // one), and it saves a full fine-level fp64 SpMV per ADMM iteration.  DDPCA_CS_SPMV=1 takes
        // the reference's explicit product instead (consStif * resuSolu, MCONTACT.h:2585-2587);
        // tests/test_headline_gpu.py bounds the difference on the headline option set
        const bool explicit_kx = std::getenv("DDPCA_CS_SPMV") && std::getenv("DDPCA_CS_SPMV")[0] == '1';
        if (explicit_kx) D.spmv(L, D.xs.p, D.lev[L].r.p);
        else
            hipLaunchKernelGGL(k_sub, dim3(nb256(3 * D.lev[L].nn)), dim3(256), 0, st, D.bs.p, D.rs.p, D.lev[L].r.p,
                               3 * D.lev[L].nn);
        for (int l = L; l > C.dmin; --l) D.restrict_level(l, l == L ? D.lev[L].r.p : D.lev[l].b.p, D.lev[l - 1].b.p);
    }
    hipLaunchKernelGGL(k_csr_wave, dim3(std::max(1, ceil_div(C.nslot, 4))), dim3(256), 0, st, C.rptr.p, C.rcol.p,
                       C.rval.p, C.nslot, H.W.p, C.gs.p, C.f0.p);
    if (H.mg && !C.assembled) {
        MgpisDevice& D = *H.mg;
        const int L = (int)D.lev.size() - 1;
        for (auto& G : C.kg) {
            const double* yd = G.level == L ? D.lev[L].r.p : D.lev[G.level].b.p;
            hipLaunchKernelGGL(k_cs_kpart, dim3(nb256(G.rows.n)), dim3(256), 0, st, G.rows.p, G.src.p, yd, C.gs.p,
                               (int64_t)G.rows.n);
        }
    }
    // every slot has one source subdomain, so one rank: the others add exact zeros
    if (H.comm) H.comm->allreduce_sum(C.gs.p, C.nslot, st);
    hipLaunchKernelGGL(k_slot_sum, dim3(nb256(n)), dim3(256), 0, st, C.sptr.p, C.gs.p, C.g.p, n);
    if (!C.nown) return;
    if (C.mg) {  // mgpi_1.CG_SOLV(1, globForc, globSolu) (MCONTACT.h:2594), on the coarse solver's stream
        MgpisDevice& M = *C.cmg;
        DDPCA_HIP(hipEventRecord(C.ev_in, st));
        DDPCA_HIP(hipStreamWaitEvent(M.stream, C.ev_in, 0));
        DDPCA_HIP(hipMemsetAsync(M.bs.p, 0, M.bs.n * sizeof(double), M.stream));
        hipLaunchKernelGGL(k_perm_scatter, dim3(nb256(n)), dim3(256), 0, M.stream, C.cperm.p, C.g.p, M.bs.p, n);
        M.pcg_solve(1, 1.0e-14, std::vector<int64_t>{n});
        hipLaunchKernelGGL(k_perm_gather, dim3(nb256(C.nown)), dim3(256), 0, M.stream, C.cperm.p, C.cown.p, M.xs.p, C.xc.p,
                           C.nown);
        DDPCA_HIP(hipEventRecord(C.ev_out, M.stream));
        DDPCA_HIP(hipStreamWaitEvent(st, C.ev_out, 0));
    } else {
        hipLaunchKernelGGL(k_gemv_wave, dim3(ceil_div(C.nown, 4)), dim3(256), 0, st, C.ainv.p, C.g.p, C.xc.p, C.nown, n);
    }
    if (C.assembled) {
        if (C.npr)
            hipLaunchKernelGGL(k_cs_prolong_csr, dim3(nb256(C.npr)), dim3(256), 0, st, C.pptr.p, C.pcol.p, C.pval.p, C.ptgt.p,
                               C.xc.p, H.u, C.npr);
        if (C.ncd) hipLaunchKernelGGL(k_cs_presc, dim3(nb256(C.ncd)), dim3(256), 0, st, C.cdof.p, H.presc.p, H.u, C.ncd);
        return;
    }
    hipLaunchKernelGGL(k_cs_scatter, dim3(nb256(C.nxn)), dim3(256), 0, st, C.xsrc.p, C.xc.p, C.xn.p, C.nxn);
    hipLaunchKernelGGL(k_cs_prolong, dim3(nb256(C.qnn)), dim3(256), 0, st, C.qcol.p, C.qw.p, C.qnn, C.xn.p, C.flag.p,
                       H.presc.p, H.u);
    if (C.npr)  // the nodes the scalar stencil cannot hold (rotation blocks)
        hipLaunchKernelGGL(k_cs_prolong_csr, dim3(nb256(C.npr)), dim3(256), 0, st, C.pptr.p, C.pcol.p, C.pval.p, C.ptgt.p,
                           C.xc.p, H.u, C.npr);
}

// Reference MONITOR (MCONTACT.h:2725-2845) on the reduced norms; true = converged.
bool monitor(ddpca_mcontact& H) {
    const int64_t cyc = 10;
    const int64_t tc = H.tc;
    const int64_t hb = 2 * H.nsub + 8 * H.nint;  // hanging-level parts of the subdomain norms
    for (int64_t k = 0; k < 2 * H.nsub; ++k) H.moni_host[k] += H.moni_host[hb + k];
    bool flag0 = tc >= cyc, flag1 = true;
    const double c0 = 0.1, c1 = 1.0e-12;
    double convValu = 0.0, convCrit = 0.0;
    std::vector<double> row;
    auto medi_osci = [](const std::vector<double>& v, double& medi, double& osci) {
        const double mx = *std::max_element(v.begin(), v.end()), mn = *std::min_element(v.begin(), v.end());
        medi = (mx + mn) / 2.0;
        osci = mx - mn;
    };
    for (int64_t tv = 0; tv < H.nsub; ++tv) {
        const double d = H.moni_host[2 * tv], a = H.moni_host[2 * tv + 1];
        H.moniReco[tv][tc % cyc] = d;
        convValu += d;
        convCrit += a;
        row.push_back(d);
        row.push_back(a);
        if (tc >= cyc) {
            double me, os;
            medi_osci(H.moniReco[tv], me, os);
            if (os > c0 * me) flag0 = false;
        }
        if (d > c1 * a) flag1 = false;
    }
    for (int64_t ts = 0; ts < H.nint; ++ts)
        for (int s = 0; s < 2; ++s) {
            const double* m = &H.moni_host[2 * H.nsub + 8 * ts + 4 * s];
            const int64_t idx = H.nsub + 4 * ts + 2 * s;
            H.moniReco[idx][tc % cyc] = m[0];
            convValu += m[0];
            convCrit += m[1];
            row.insert(row.end(), {m[0], m[1], m[2], m[3]});
            if (tc >= cyc) {
                double me, os;
                medi_osci(H.moniReco[idx], me, os);
                if (os > c0 * me) flag0 = false;
            }
            if (m[0] > c1 * m[1]) flag1 = false;
            H.moniReco[idx + 1][tc % cyc] = m[2];  // lambda criteria disabled in the reference
        }
    row.push_back(convValu);
    row.push_back(convCrit);
    H.rows.push_back(row);
    if (flag0) H.mult_maxi = tc;
    return flag1;
}

double ms_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

void copy_dev(hipStream_t s, double* y, const double* x, int64_t n) {
    // every copied vector has an even length (3 x multiple of 64, or 2R)
    hipLaunchKernelGGL(k_copy2, dim3(nb256(n / 2)), dim3(256), 0, s, reinterpret_cast<double2*>(y),
                       reinterpret_cast<const double2*>(x), n / 2);
}

// One ADMM iteration; returns true when MONITOR reports convergence.
bool iterate_once(ddpca_mcontact& H, bool check) {
    const auto t0 = std::chrono::steady_clock::now();
    hipStream_t st = H.main;
    // snapshot for MONITOR (resuDisp_0 / inteAuxi_0 / inteLagr_0, MCONTACT.h:2507-2509)
    if (H.R) copy_dev(st, H.state_old.p, H.state, 2 * H.R);
    copy_dev(st, H.uo.p, H.u, H.NU + H.NH);
    // ---- body balance: every owned subdomain in one batched PCG
    if (H.mg) {
        MgpisDevice& D = *H.mg;
        copy_dev(st, D.bs.p, H.cf.p, 3 * D.lev.back().nn);
        if (H.ncrow)
            hipLaunchKernelGGL(k_cpl, dim3(nb256(16 * H.ncrow)), dim3(256), 0, st, H.crow.p, H.cptr.p, H.ccol.p, H.cval.p,
                               H.W.p, D.bs.p, H.ncrow);
        D.pcg_begin(1, 1.0e-14, H.maxit, H.opt.warm_start != 0 && H.tc > 0);
        D.pcg_wait(1, 0);
        hipLaunchKernelGGL(k_outp, dim3(nb256(D.lev.back().nn)), dim3(256), 0, st, D.xs.p, D.lev.back().mask.p,
                           H.onode.p, H.presc.p, H.u, D.lev.back().nn);
        if (H.NH) H.op_hang.apply(st, H.W.p, H.W.p + H.oH, nullptr);  // OUTP_SUB1's prolOper[maxiLeve] rows
    }
    // ---- coarse-space correction (MCONTACT.h:2540-2612); OUTP_SUB1 of the correction reaches the
    //      hanging level through the same rows, so they are recomputed from the corrected u
    const bool cs_ran = H.cs.on && H.tc <= H.mult_maxi;
    if (cs_ran) {
        coarse_correct(H);
        if (H.NH) H.op_hang.apply(st, H.W.p, H.W.p + H.oH, nullptr);
    }
    DDPCA_HIP(hipEventRecord(H.ev[1], st));
    const double t_solve = ms_since(t0);
    // ---- interface balance: this rank's gamma halves, one launch for every owned side
    H.op_gamma.apply(st, H.W.p, H.gamma, H.gcst.p);
    if (H.op_gamma1.nch) {
        H.op_gamma1.apply(st, H.W.p, H.gam1.p, nullptr);
        hipLaunchKernelGGL(k_add_idx, dim3(nb256((int64_t)H.gam1_dst.n)), dim3(256), 0, st, H.gamma, H.gam1.p, H.gam1_dst.p,
                           (int64_t)H.gam1_dst.n);
    }
    for (auto& F : H.fitfs) {
        const IpSide s0{F.M[0].p, F.lam[0].p, F.u[0].p}, s1{F.M[1].p, F.lam[1].p, F.u[1].p};
        if (F.nip)
            hipLaunchKernelGGL(k_gamma_ip, dim3(nb256(F.nip)), dim3(256), 0, st, F.B.p, s0, s1, F.own[0], F.own[1], F.pen[0],
                               F.pen[1], F.pen[2], F.C, F.nip, H.W.p, H.gamma + F.goff, H.gcst.p + F.goff);
    }
    bool any_cross = false;
    for (auto& I : H.itfs) any_cross |= (I.cross && I.mine);
    DDPCA_HIP(hipEventRecord(H.ev[0], st));
    if (any_cross) {
        if (!H.comm) throw ApiError(DDPCA_ESTATE, "cross-rank interfaces need mcontact_gpu_comm_init");
        std::vector<Transport::Msg> msgs;
        for (auto& I : H.itfs) {
            if (!(I.cross && I.mine)) continue;
            const int peer = I.owner[0] == H.rank ? I.owner[1] : I.owner[0];
            msgs.push_back({peer, I.ts, H.gamma + I.goff, I.recv.p, I.mip});
        }
        H.comm->exchange(msgs, st);
        for (auto& I : H.itfs)
            if (I.cross && I.mine)
                hipLaunchKernelGGL(k_add, dim3(nb256(I.mip)), dim3(256), 0, st, H.gamma + I.goff, I.recv.p, I.mip);
    }
    DDPCA_HIP(hipEventRecord(H.ev[2], st));
    for (auto& I : H.itfs)
        if (I.mine)
            hipLaunchKernelGGL(k_project, dim3(nb256(I.mip / I.comp)), dim3(256), 0, st, H.gamma + I.goff, I.stat.p,
                               I.mip / I.comp, I.comp, I.fric);
    // ---- aux = (M^rho)^-1 (T^T u + M lambda + I gamma), lambda += M^-1 (T^T u - M^rho aux)
    if (H.fused) {
        H.op_wv.apply(st, H.W.p, H.mb_wv.b.p, nullptr);
        for (auto& F : H.fitfs) {  // the inteInpo gamma half of the factored interfaces
            if (!F.nip) continue;
            hipLaunchKernelGGL(k_traction_ip, dim3(nb256(F.nip)), dim3(256), 0, st, F.B.p, H.gamma + F.goff, F.T.p, F.C,
                               F.nip);
            for (int s = 0; s < 2; ++s)
                if (F.own[s] && F.nnc[s])
                    hipLaunchKernelGGL(k_inpo_node, dim3(ceil_div(F.nnc[s], 4)), dim3(256), 0, st, F.nptr[s].p, F.niq[s].p,
                                       F.ncoef[s].p, F.T.p, F.C, F.nnc[s], H.mb_wv.b.p + H.R + F.roff[s]);
        }
        H.mb_wv.solve(st, H.mb_wv.x.p, 1.0e-14, 2000);
        hipLaunchKernelGGL(k_fuse_aux_lambda, dim3(nb256(H.R)), dim3(256), 0, st, H.state, H.mb_wv.x.p, H.rinv.p, H.R);
    } else if (!H.sides.empty()) {
        H.op_aux.apply(st, H.W.p, H.mb_aux.b.p, nullptr);
        H.mb_aux.solve(st, H.state, 1.0e-14, 2000);
        // ---- lambda += M^-1 (T^T u - M^rho aux)
        H.op_lam.apply(st, H.W.p, H.mb_lam.b.p, nullptr);
        H.mb_lam.solve(st, H.mb_lam.x.p, 1.0e-14, 2000);
        hipLaunchKernelGGL(k_add, dim3(nb256(H.R)), dim3(256), 0, st, H.state + H.R, H.mb_lam.x.p, H.R);
    }
    // ---- MONITOR norms (owned entries; others zero) and their reduction across ranks
    DDPCA_HIP(hipMemsetAsync(H.moni.p, 0, H.moni.n * sizeof(double), st));
    {
        std::vector<NormSeg> seg;
        int64_t nblk = 0;
        auto add = [&](const double* a, const double* o, int64_t n, int64_t slot) {
            const int64_t nb = nb256(n);
            seg.push_back({a, o, n, nblk, nb, slot});
            nblk += nb;
        };
        for (auto& S : H.subs) {
            add(H.u + S.dof0, H.uo.p + S.dof0, 3 * S.nn, 2 * S.tv);
            if (S.nh) add(H.u + H.oH + S.hoff, H.uo.p + H.oH + S.hoff, S.nh, 2 * H.nsub + 8 * H.nint + 2 * S.tv);
        }
        for (auto& sd : H.sides) {
            const int64_t base = 2 * H.nsub + 8 * sd.ts + 4 * sd.s;
            add(H.state + sd.roff, H.state_old.p + sd.roff, sd.m, base);
            add(H.state + H.R + sd.roff, H.state_old.p + H.R + sd.roff, sd.m, base + 2);
        }
        if (!seg.empty()) {
            // the segments are the same every iteration: upload once (and again if they change)
            const bool same = seg.size() == H.norm_seg_host.size() &&
                              std::memcmp(seg.data(), H.norm_seg_host.data(), seg.size() * sizeof(NormSeg)) == 0;
            if (!same) {
                std::vector<int32_t> bseg(nblk);
                for (size_t g = 0; g < seg.size(); ++g)
                    for (int64_t k = 0; k < seg[g].nb; ++k) bseg[seg[g].blk0 + k] = (int32_t)g;
                DDPCA_HIP(hipStreamSynchronize(st));  // the previous iteration's launches read the old table
                H.norm_seg.upload(seg);
                H.norm_bseg.upload(bseg);
                H.norm_partial.alloc(2 * nblk);
                H.norm_seg_host = seg;
            }
            hipLaunchKernelGGL(k_pair_norms_all, dim3((unsigned)nblk), dim3(256), 0, st, H.norm_seg.p, H.norm_bseg.p,
                               H.norm_partial.p);
            hipLaunchKernelGGL(k_reduce_pairs_all, dim3((unsigned)seg.size()), dim3(256), 0, st, H.norm_seg.p,
                               H.norm_partial.p, H.moni.p);
        }
    }
    if (H.comm) H.comm->allreduce_sum(H.moni.p, H.moni.n, st);
    DDPCA_HIP(hipEventRecord(H.ev[3], st));
    DDPCA_HIP(hipMemcpyAsync(H.moni_host.data(), H.moni.p, H.moni.n * sizeof(double), hipMemcpyDeviceToHost, st));
    if (H.mg) H.mg->pcg_fetch();
    DDPCA_HIP(hipStreamSynchronize(st));
    if (H.mg) H.mg->pcg_check();
    H.mb_aux.check();
    H.mb_lam.check();
    H.mb_wv.check();
    float a = 0, b = 0;
    (void)hipEventElapsedTime(&a, H.ev[1], H.ev[3]);
    (void)hipEventElapsedTime(&b, H.ev[0], H.ev[2]);
    H.timing[0] += ms_since(t0);
    H.timing[1] += t_solve;
    H.timing[2] += a;
    H.timing[3] += any_cross ? b : 0.0;
    H.mass_iters += (double)(H.fused ? H.mb_wv.last_iters : H.mb_aux.last_iters + H.mb_lam.last_iters);
    if (H.mg) {
        MgpisDevice& D = *H.mg;
        for (int s = 0; s < D.nsub; ++s) {
            H.timing[6] += (double)D.sc_host[s].iter;
            H.timing[8] += (double)D.sc_host[s].iter * (double)D.nfree[s];
        }
        if (D.timed_kernel_samples) {
            H.timing[7] += D.timed_kernel_bytes;
            H.timing[4] += D.timed_kernel_ms;
            H.timing[5] += (double)D.timed_kernel_samples;
            D.timed_kernel_ms = 0.0;
            D.timed_kernel_bytes = 0.0;
            D.timed_kernel_samples = 0;
        }
    }
    if (H.mg) {
        MgpisDevice& D = *H.mg;
        H.bytes[0] += D.alg_bytes[0];
        H.bytes[1] += D.alg_bytes[1];
        H.bytes[7] += D.alg_bytes[2];
        D.alg_bytes[0] = D.alg_bytes[1] = D.alg_bytes[2] = 0.0;
    }
    if (cs_ran) {
        H.bytes[2] += H.cs.bytes_iter;
        if (H.cs.cmg) {
            H.bytes[2] += H.cs.cmg->alg_bytes[0] + H.cs.cmg->alg_bytes[1];
            H.cs.cmg->alg_bytes[0] = H.cs.cmg->alg_bytes[1] = H.cs.cmg->alg_bytes[2] = 0.0;
        }
    }
    H.bytes[3] += H.bytes_rhs;
    H.bytes[4] += H.bytes_iface;
    for (MassBatch* mb : {&H.mb_aux, &H.mb_lam, &H.mb_wv}) {
        H.bytes[5] += mb->alg_bytes;
        mb->alg_bytes = 0.0;
    }
    H.bytes[6] += H.bytes_moni;
    const bool conv = monitor(H);
    H.tc += 1;
    return check && conv;
}

}  // namespace

extern "C" {

// Every graph the ADMM iteration replays, captured on the calling thread (create, or after the
// in-process ranks' setup threads joined): a capture running on one rank thread was invalidated
// by another rank thread's synchronous HIP calls in the in-process multi-rank runs.
// Idempotent: what exists is kept.
void prepare_graphs(ddpca_mcontact& H) {
    if (H.mg) H.mg->prepare_graphs(1);
    if (H.fused) H.mb_wv.prepare(H.main, H.mb_wv.x.p);
    else if (!H.sides.empty()) {
        H.mb_aux.prepare(H.main, H.state);
        H.mb_lam.prepare(H.main, H.mb_lam.x.p);
    }
    if (H.cs.cmg) H.cs.cmg->prepare_graphs(1);
    DDPCA_HIP(hipStreamSynchronize(H.main));
}

int mcontact_gpu_create(ddpca_problem_t p, int device, int rank, int nranks, const int32_t* owner,
                        const mgpis_options_t* opt, mcontact_t* out) {
    return guarded([&] {
        Problem& P = *reinterpret_cast<Problem*>(p);
        if (!P.established) throw ApiError(DDPCA_ESTATE, "problem not established");
        if (nranks < 1 || rank < 0 || rank >= nranks || !owner || !out) throw ApiError(DDPCA_EINVAL, "rank/owner");
        select_device(device);
        auto H = std::make_unique<ddpca_mcontact>();
        H->device = device;
        H->rank = rank;
        H->nranks = nranks;
        H->owner.assign(owner, owner + P.mc.multGrid.size());
        for (int32_t o : H->owner)
            if (o < 0 || o >= nranks) throw ApiError(DDPCA_EINVAL, "owner out of range");
        if (opt) H->opt = *opt;
        else mgpis_default_options(&H->opt);
        for (auto& e : H->ev) DDPCA_HIP(hipEventCreate(&e));
        build(*H, P);
        build_coarse(*H, P);
        if (nranks == 1) coarse_invert(*H);
        prepare_graphs(*H);
        *out = H.release();
    });
}

int mcontact_gpu_unique_id(void* out128) {
    return guarded([&] {
        ncclUniqueId id;
        DDPCA_NCCL(ncclGetUniqueId(&id));
        std::memcpy(out128, &id, sizeof(id));
    });
}

int mcontact_gpu_comm_init(mcontact_t h, const void* uid) {
    return guarded([&] {
        if (!h || !uid) throw ApiError(DDPCA_EINVAL, "handle / unique id");
        select_device(h->device);
        if (h->comm) throw ApiError(DDPCA_ESTATE, "handle already has a communicator");
        // nranks == 1 builds a one-rank communicator too: the MONITOR and coarse-RHS all-reduces then
        // run through RCCL on the solve stream (bit-identical to the run without one)
        ncclUniqueId id;
        std::memcpy(&id, uid, sizeof(id));
        auto t = std::make_unique<RcclTransport>();
        DDPCA_NCCL(ncclCommInitRank(&t->comm, h->nranks, id, h->rank));
        h->comm = std::move(t);
        coarse_invert(*h);
        prepare_graphs(*h);
    });
}

int mcontact_gpu_comm_local(mcontact_t* handles, int n) {
    return guarded([&] {
        if (!handles || n < 1) throw ApiError(DDPCA_EINVAL, "handles");
        for (int r = 0; r < n; ++r) {
            if (!handles[r] || handles[r]->nranks != n || handles[r]->rank != r)
                throw ApiError(DDPCA_EINVAL, "handles[r] must be rank r of n");
            if (handles[r]->comm) throw ApiError(DDPCA_ESTATE, "handle already has a communicator");
        }
        auto hub = std::make_shared<LocalHub>();
        hub->n = n;
        hub->slot.resize(n);
        for (int r = 0; r < n; ++r) {
            auto t = std::make_unique<LocalTransport>();
            t->hub = hub;
            t->rank = r;
            handles[r]->comm = std::move(t);
        }
        // the setup all-reduce of the coarse matrix is collective: one host thread per rank
        std::vector<std::thread> th;
        std::vector<int> rc(n, 0);
        std::vector<std::string> msg(n);
        for (int r = 0; r < n; ++r)
            th.emplace_back([&, r] {
                rc[r] = guarded([&] {
                    select_device(handles[r]->device);
                    coarse_invert(*handles[r]);
                });
                if (rc[r] < 0) msg[r] = ddpca_last_error();
            });
        for (auto& t : th) t.join();
        for (int r = 0; r < n; ++r)
            if (rc[r] < 0) throw ApiError(rc[r], "rank " + std::to_string(r) + ": " + msg[r]);
        for (int r = 0; r < n; ++r) {  // the gathered DOUBLE_M solvers' graphs, one rank at a time
            select_device(handles[r]->device);
            prepare_graphs(*handles[r]);
        }
    });
}

int mcontact_gpu_comm_loopback(mcontact_t h, ddpca_problem_t p) {
    return guarded([&] {
        if (!h || !p) throw ApiError(DDPCA_EINVAL, "handle / problem");
        select_device(h->device);
        if (h->comm) throw ApiError(DDPCA_ESTATE, "handle already has a communicator");
        CoarseDev& C = h->cs;
        // a rank-local DOUBLE_M operator would be "gathered" through the identity all-reduce: this
        // rank's rows only, a singular coarse hierarchy
        if (C.on && !C.inverted && C.mg_gather)
            throw ApiError(DDPCA_ESTATE, "loopback: the problem must be the handle's, established in full "
                                         "(a rank-local DOUBLE_M coarse operator cannot be gathered)");
        h->comm = std::make_unique<LoopbackTransport>();
        if (C.on && !C.inverted && !C.mg) {
            // the other ranks' rows of the dense coarse operator come from the problem itself (the
            // setup all-reduce that would sum them is the identity here)
            const CoarseSpace& cs = reinterpret_cast<Problem*>(p)->mc.coarse;
            if (cs.rank_local || cs.n != C.n)
                throw ApiError(DDPCA_ESTATE, "loopback: the problem must be the handle's, established in full");
            const int64_t n = C.n;
            C.dense.assign((size_t)n * n, 0.0);
            for (int64_t r = 0; r < n; ++r)
                for (int64_t k = cs.globCoup_1.ptr[r]; k < cs.globCoup_1.ptr[r + 1]; ++k)
                    C.dense[(size_t)r * n + cs.globCoup_1.col[k]] = cs.globCoup_1.val[k];
        }
        coarse_invert(*h);
        prepare_graphs(*h);
    });
}

int mcontact_gpu_comm_check(mcontact_t h, int64_t n) {
    return guarded([&] {
        if (!h || n < 1) throw ApiError(DDPCA_EINVAL, "handle / n");
        select_device(h->device);
        if (!h->comm) throw ApiError(DDPCA_ESTATE, "no communicator (mcontact_gpu_comm_init / _comm_local)");
        const int R = h->nranks, me = h->rank;
        hipStream_t st = h->main;
        // exchange: to every rank q (me included) two messages, tagged by the unordered pair {me, q}
        // and k as the interfaces' gamma halves are (both ends name the same tag);
        // message (me -> q, k) carries v = 1e6 me + 1e3 q + k + i 2^-20 (exact in fp64)
        auto val = [](int src, int dst, int k, int64_t i) { return 1.0e6 * src + 1.0e3 * dst + k + std::ldexp((double)i, -20); };
        std::vector<double> hs((size_t)R * 2 * n);
        for (int q = 0; q < R; ++q)
            for (int k = 0; k < 2; ++k)
                for (int64_t i = 0; i < n; ++i) hs[((size_t)q * 2 + k) * n + i] = val(me, q, k, i);
        DevBuf<double> sbuf, rbuf((size_t)R * 2 * n), ar(n);
        sbuf.upload(hs);
        std::vector<Transport::Msg> msgs;
        for (int q = 0; q < R; ++q)
            for (int k = 0; k < 2; ++k)
                msgs.push_back({q, 2 * ((int64_t)std::min(me, q) * R + std::max(me, q)) + k, sbuf.p + ((size_t)q * 2 + k) * n, rbuf.p + ((size_t)q * 2 + k) * n, n});
        h->comm->exchange(msgs, st);
        // all-reduce: rank r contributes (r + 1) (i + 1); the sum is R (R + 1) / 2 (i + 1)
        std::vector<double> ha(n);
        for (int64_t i = 0; i < n; ++i) ha[i] = (double)(me + 1) * (double)(i + 1);
        DDPCA_HIP(hipMemcpyAsync(ar.p, ha.data(), n * sizeof(double), hipMemcpyHostToDevice, st));
        h->comm->allreduce_sum(ar.p, n, st);
        DDPCA_HIP(hipStreamSynchronize(st));
        const auto hr = rbuf.download();
        const auto hsum = ar.download();
        for (int q = 0; q < R; ++q)
            for (int k = 0; k < 2; ++k)
                for (int64_t i = 0; i < n; ++i)
                    if (hr[((size_t)q * 2 + k) * n + i] != val(q, me, k, i))
                        throw ApiError(DDPCA_ECOMM, "comm check: message " + std::to_string(k) + " from rank " + std::to_string(q) +
                                                        " arrived wrong at element " + std::to_string(i));
        for (int64_t i = 0; i < n; ++i)
            if (hsum[i] != 0.5 * R * (R + 1) * (double)(i + 1))
                throw ApiError(DDPCA_ECOMM, "comm check: all-reduce element " + std::to_string(i) + " wrong");
    });
}

int64_t mcontact_gpu_iterate(mcontact_t h, int64_t maxit, int check) {
    int64_t n = 0;
    const int rc = guarded([&] {
        select_device(h->device);
        for (double& t : h->timing) t = 0.0;
        for (double& b : h->bytes) b = 0.0;
        h->mass_iters = 0.0;
        if (h->mg) h->mg->time_kernel = true;
        if (h->nranks > 1 && !h->comm) throw ApiError(DDPCA_ESTATE, "a multi-rank run needs mcontact_gpu_comm_init");
        for (; n < maxit;) {
            const bool conv = iterate_once(*h, check != 0);
            ++n;
            if (conv) break;
        }
    });
    return rc < 0 ? rc : n;
}

int64_t mcontact_gpu_monitor(mcontact_t h, double* out, int64_t cap_rows) {
    const int64_t rows = (int64_t)h->rows.size();
    if (!out) return rows;
    const int64_t ncol = 2 * h->nsub + 8 * h->nint + 2;
    for (int64_t r = 0; r < std::min(rows, cap_rows); ++r) std::memcpy(out + r * ncol, h->rows[r].data(), ncol * sizeof(double));
    return std::min(rows, cap_rows);
}

int64_t mcontact_gpu_get(mcontact_t h, const char* what, int64_t index, void* out, int64_t cap) {
    int64_t n = 0;
    const int rc = guarded([&] {
        select_device(h->device);
        const std::string w(what);
        DDPCA_HIP(hipStreamSynchronize(h->main));
        if (w == "resuDisp") {
            for (auto& S : h->subs)
                if (S.tv == index) {  // position numbering: level-maxiLeve nodes, then the hanging level
                    n = 3 * S.nn + S.nh;
                    if (out) {
                        DDPCA_HIP(hipMemcpy(out, h->u + S.dof0, std::min(3 * S.nn, cap) * sizeof(double), hipMemcpyDeviceToHost));
                        if (cap > 3 * S.nn && S.nh)
                            DDPCA_HIP(hipMemcpy(static_cast<double*>(out) + 3 * S.nn, h->u + h->oH + S.hoff,
                                                std::min(S.nh, cap - 3 * S.nn) * sizeof(double), hipMemcpyDeviceToHost));
                    }
                    return;
                }
            throw ApiError(DDPCA_EINVAL, "subdomain not owned by this rank");
        }
        if (w == "inteAuxi" || w == "inteLagr") {
            for (auto& sd : h->sides)
                if (2 * sd.ts + sd.s == index) {
                    n = sd.m;
                    const double* src = h->state + sd.roff + (w == "inteAuxi" ? 0 : h->R);
                    if (out) DDPCA_HIP(hipMemcpy(out, src, std::min(n, cap) * sizeof(double), hipMemcpyDeviceToHost));
                    return;
                }
            throw ApiError(DDPCA_EINVAL, "interface side not owned by this rank");
        }
        if (w == "inpoGamm") {
            for (auto& I : h->itfs)
                if (I.ts == index && I.mine) {
                    n = I.mip;
                    if (out) DDPCA_HIP(hipMemcpy(out, h->gamma + I.goff, std::min(n, cap) * sizeof(double), hipMemcpyDeviceToHost));
                    return;
                }
            throw ApiError(DDPCA_EINVAL, "interface not handled by this rank");
        }
        if (w == "fricStat") {
            for (auto& I : h->itfs)
                if (I.ts == index && I.mine) {
                    n = I.mip / I.comp;
                    if (out) DDPCA_HIP(hipMemcpy(out, I.stat.p, std::min(n, cap) * sizeof(int32_t), hipMemcpyDeviceToHost));
                    return;
                }
            throw ApiError(DDPCA_EINVAL, "interface not handled by this rank");
        }
        if (w == "pcg_iters") {
            n = (int64_t)h->subs.size();
            if (out)
                for (int64_t i = 0; i < std::min(n, cap); ++i) static_cast<int64_t*>(out)[i] = h->mg->sc_host[i].iter;
            return;
        }
        if (w == "owned") {
            n = (int64_t)h->subs.size();
            if (out)
                for (int64_t i = 0; i < std::min(n, cap); ++i) static_cast<int64_t*>(out)[i] = h->subs[i].tv;
            return;
        }
        if (w == "coarse_solve") {
            // [rows, 1 = multigrid (DOUBLE_M / DOUBLE_M_1) else 0, dense inverse bytes,
            //  1 = the budget asked for DOUBLE_M but its hierarchy was not buildable (dense kept)]
            n = 4;
            if (out && cap >= 4) {
                auto* o = static_cast<int64_t*>(out);
                o[0] = h->cs.on ? h->cs.n : 0;
                o[1] = h->cs.on && h->cs.mg ? 1 : 0;
                o[2] = h->cs.on && !h->cs.mg ? (int64_t)h->cs.dense_bytes : 0;
                o[3] = h->cs.mg_fallback ? 1 : 0;
            }
            return;
        }
        if (w == "mass_iters") {
            n = 1;
            if (out && cap >= 1) static_cast<int64_t*>(out)[0] = (int64_t)h->mass_iters;
            return;
        }
        if (w == "gs_rows") {  // int64 [rows the colour sweeps cover, ring rows, far rows] (GsFine::band)
            int64_t v[3] = {0, 0, 0};
            if (h->mg && h->mg->gs_fine()) {
                const GsFine& G = h->mg->gs;
                for (int s = 0; s < h->mg->nsub; ++s) {
                    v[0] += G.band ? G.band_rows_sub[s] : h->mg->lev.back().nloc[s];
                    v[1] += G.band ? G.ring_rows_sub[s] : 0;
                    v[2] += G.band ? G.far_rows_sub[s] : 0;
                }
            }
            n = 3;
            if (out)
                for (int64_t i = 0; i < std::min<int64_t>(3, cap); ++i) static_cast<int64_t*>(out)[i] = v[i];
            return;
        }
        if (w == "gs_launch_bytes") {  // the colour sweeps' per-launch byte model (GsFine::launch_bytes), doubles
            if (!h->mg) throw ApiError(DDPCA_ESTATE, "no owned subdomain");
            const auto& v = h->mg->gs.launch_bytes;
            n = (int64_t)v.size();
            if (out)
                for (int64_t i = 0; i < std::min(n, cap); ++i) static_cast<double*>(out)[i] = v[i];
            return;
        }
        throw ApiError(DDPCA_EINVAL, "unknown quantity " + w);
    });
    return rc < 0 ? rc : n;
}

int mcontact_gpu_timing(mcontact_t h, double* out10) {
    std::memcpy(out10, h->timing, sizeof(h->timing));
    if (h->timing[5] > 0) out10[7] = h->timing[7] / h->timing[5];  // bytes per timed launch
    double dofs = 0.0;
    if (h->mg)
        for (int64_t nf : h->mg->nfree) dofs += (double)nf;
    out10[9] = dofs;
    return DDPCA_OK;
}

int64_t mcontact_gpu_bytes(mcontact_t h, double* out, int64_t cap) {
    const int64_t n = (int64_t)(sizeof(h->bytes) / sizeof(double));
    if (out)
        for (int64_t i = 0; i < std::min(n, cap); ++i) out[i] = h->bytes[i];
    return n;
}

int ddpca_mass_solve(int device, int64_t nsys, const ddpca_csr_t* A, const double* b, double* x, double rtol,
                     int64_t maxit, int fuse_alpha, int64_t* iters) {
    int64_t nrow = 0;
    std::vector<int64_t> roff;
    std::vector<Csr> sys;
    DevBuf<double> xd;
    MassBatch mb;
    hipStream_t st = nullptr;
    auto copy_out = [&]() {  // the systems' rows of the padded batch vector, in order
        std::vector<double> h(std::max<int64_t>(nrow, 1));
        DDPCA_HIP(hipMemcpy(h.data(), xd.p, nrow * sizeof(double), hipMemcpyDeviceToHost));
        int64_t o = 0;
        for (int64_t s = 0; s < nsys; ++s) {
            std::memcpy(x + o, h.data() + roff[s], sys[s].nrow * sizeof(double));
            o += sys[s].nrow;
        }
    };
    const int rc = guarded([&] {
        if (nsys < 1 || !A || !b || !x || !(rtol > 0.0) || maxit < 1) throw ApiError(DDPCA_EINVAL, "ddpca_mass_solve: arguments");
        select_device(device);
        for (int64_t s = 0; s < nsys; ++s) {
            const ddpca_csr_t& a = A[s];
            if (a.nrow < 1 || a.ncol != a.nrow || !a.ptr || (a.ptr[a.nrow] > 0 && (!a.col || !a.val)))
                throw ApiError(DDPCA_EINVAL, "ddpca_mass_solve: system " + std::to_string(s) + " is not a square CSR");
            Csr c;
            c.nrow = c.ncol = a.nrow;
            c.ptr.assign(a.ptr, a.ptr + a.nrow + 1);
            if (c.ptr[0] != 0) throw ApiError(DDPCA_EINVAL, "ddpca_mass_solve: ptr[0] != 0");
            for (int64_t r = 0; r < a.nrow; ++r)
                if (c.ptr[r + 1] < c.ptr[r]) throw ApiError(DDPCA_EINVAL, "ddpca_mass_solve: row pointer decreases");
            c.col.assign(a.col, a.col + c.ptr[a.nrow]);
            c.val.assign(a.val, a.val + c.ptr[a.nrow]);
            bool diag = false;
            for (int64_t r = 0; r < a.nrow; ++r)
                for (int64_t k = c.ptr[r]; k < c.ptr[r + 1]; ++k) {
                    if (c.col[k] < 0 || c.col[k] >= a.nrow) throw ApiError(DDPCA_EINVAL, "ddpca_mass_solve: column out of range");
                    diag |= c.col[k] == r;
                }
            if (!diag) throw ApiError(DDPCA_EINVAL, "ddpca_mass_solve: a system without diagonal entries");
            roff.push_back(nrow);
            nrow += pad64(a.nrow);
            sys.push_back(std::move(c));
        }
        std::vector<const Csr*> ptrs;
        for (const Csr& c : sys) ptrs.push_back(&c);
        mb.build(ptrs, roff, nrow);
        mb.fuse_override = fuse_alpha;
        std::vector<double> hb(nrow, 0.0);
        int64_t o = 0;
        for (int64_t s = 0; s < nsys; ++s) {
            std::memcpy(hb.data() + roff[s], b + o, sys[s].nrow * sizeof(double));
            o += sys[s].nrow;
        }
        DDPCA_HIP(hipMemcpy(mb.b.p, hb.data(), nrow * sizeof(double), hipMemcpyHostToDevice));
        xd.alloc(nrow);
        DDPCA_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
        mb.solve(st, xd.p, rtol, maxit);
        DDPCA_HIP(hipStreamSynchronize(st));
        if (iters)
            for (int64_t s = 0; s < nsys; ++s) iters[s] = mb.mirror.host[s].iter;
        copy_out();
        mb.check();  // DDPCA_ENUMERIC on a breakdown (x already copied: the last good iterate)
    });
    if (st) {
        (void)hipStreamSynchronize(st);
        (void)hipStreamDestroy(st);
    }
    return rc;
}

int mcontact_gpu_destroy(mcontact_t h) {
    return guarded([&] {
        if (!h) return;
        (void)hipSetDevice(h->device);
        if (h->main) (void)hipStreamSynchronize(h->main);
        h->comm.reset();
        for (auto& e : h->ev)
            if (e) (void)hipEventDestroy(e);
        const bool own_stream = !h->mg && h->main;
        hipStream_t st = h->main;
        delete h;
        if (own_stream) (void)hipStreamDestroy(st);
    });
}

}  // extern "C"
