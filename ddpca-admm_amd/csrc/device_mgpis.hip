// MGPIS device path: SELL-BSR3 kernels, V-cycle and PCG for gfx950 over a batch of
// subdomains (see device_mgpis.hpp for the layout).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <deque>
#include <array>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <tuple>
#include <type_traits>
#include <omp.h>
#include <random>
#include <thread>
#include <unordered_map>

#include <rocblas/rocblas.h>
#include <rocsolver/rocsolver.h>

#include "device_mgpis.hpp"

namespace ddpca {

// ============================================================================== kernels
namespace {

enum SellMode { kSpmv = 0, kResid = 1, kJac = 2, kPcg = 3, kCheb = 4 };
enum FinWhat { kFinInit = 0, kFinBeta0 = 1, kFinAlpha = 2, kFinRR = 3, kFinBeta = 4, kFinInitWarm = 5 };

struct SellArgs {
    const int32_t* slots;
    const int64_t* off;
    const int32_t* col;
    const int16_t* col16;  // column offsets from the row node (levels whose offsets fit), or null
    const void* val;       // double (Krylov operator) or float (fp32-stored V-cycle operator)
    const int32_t* csub;   // chunk -> subdomain
    int64_t nch;
    const double* x;       // gathered operand
    double* y;             // SPMV / RESID output, PCG: q (in place)
    const double* b;       // RESID / JAC / CHEB right-hand side
    const void* minv;      // smoother inverse: double, or float on reduced-precision levels
    const double* coef;    // per subdomain (c1, c2) of this sweep; JAC uses c2 = omega
    double* xo;            // JAC / CHEB new iterate
    double* p;             // PCG: p (in place), CHEB: direction d (in place)
    const PcgScal* sc;     // per-subdomain stop flags / beta; nullptr = never stopped
    double* partial;       // per chunk
    const int32_t* rtype;  // table mode: row -> table row
    const double* tab;     // table mode: tstride doubles per table row, slot-major 3x3 blocks
    int64_t tstride;
    const int32_t* ctype;  // table mode: chunk -> its rows' common table row, -1 = mixed
    // fp32 iterate copies of a block-Jacobi level (LevelDev::x4a / x4b, precond_fp32 = 4): the
    // sweep / residual gathers x (and the sweep its own row's x) from x4; the sweep writes its new
    // iterate to xo4 and / or, when xo is set (the level's last sweep), to xo in fp64
    const float4* x4;
    float4* xo4;
};

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// Chunk partial of a dot product: one wavefront = one 64-node chunk, fixed shuffle order.
__device__ __forceinline__ void chunk_partial(double v, double* partial, int64_t chunk) {
    v = wave_sum(v);
    if ((threadIdx.x & 63) == 0) partial[chunk] = v;
}

__device__ __forceinline__ bool stopped(const PcgScal* sc, int sub) { return sc && sc[sub].done; }

template <bool BJ, typename MT = double>
__device__ __forceinline__ void apply_m(const MT* minv, int64_t row, double r0, double r1, double r2,
                                        double& m0, double& m1, double& m2) {
    if (BJ) {
        const MT* m = minv + 9 * row;
        m0 = __builtin_fma((double)m[2], r2, __builtin_fma((double)m[1], r1, (double)m[0] * r0));
        m1 = __builtin_fma((double)m[5], r2, __builtin_fma((double)m[4], r1, (double)m[3] * r0));
        m2 = __builtin_fma((double)m[8], r2, __builtin_fma((double)m[7], r1, (double)m[6] * r0));
    } else {
        const MT* m = minv + 3 * row;
        m0 = m[0] * r0;
        m1 = m[1] * r1;
        m2 = m[2] * r2;
    }
}

// Value layout of one slot (64 lanes x one 3x3 block) of a streamed SELL-BSR3 operator.
// fp64, paired (DDPCA_PAIRED_VALUES = 1, default): 16-B lane loads -- four 1-KiB wave runs of
// (v[2p], v[2p+1]), then a 512-B run of v[8]: 5 load instructions per block instead of 9, the
// fine PCG SpMV 5-8 % faster (profiles/r01_spmv_ab.json).  fp32 keeps nine 256-B runs, one per
// entry: its paired forms -- two 16-B quads + v[8], or four 8-B pairs + v[8] -- measured 4-13 %
// SLOWER in the smoothing and residual kernels (profiles/r01_spmv_ab.json, _f32pairs.json).  Element (ij, lane) of slot base sb:
//   paired fp64: sb[(ij < 8 ? 128 * (ij / 2) + 2 * lane + ij % 2 : 512 + lane)]
//   otherwise:   sb[ij * 64 + lane]
#ifndef DDPCA_PAIRED_VALUES
#define DDPCA_PAIRED_VALUES 1
#endif
template <typename T>
constexpr bool paired_values() { return DDPCA_PAIRED_VALUES != 0 && sizeof(T) == 8; }
typedef double dbl2_t __attribute__((ext_vector_type(2)));

// Block-exponent fp16 storage (T = uint16_t; precond_fp32 = 2, the fine level's V-cycle copy):
// each 3x3 block is 2^e times nine fp16 values, e = the binary exponent of the block's largest
// |entry| (so |values| < 1 and every entry within 2^14 of the block maximum keeps fp16's 11
// significant bits); the record is ten halves, (v0,v1) (v2,v3) (v4,v5) (v6,v7) (v8,e), one
// 256-B dword run per pair: a slot is 1280 B, 20 B per block against 36 B for fp32.  A block
// and its transpose share e and round alike, so the operator stays exactly symmetric.
//
// Block-scaled int8 storage (T = uint8_t; precond_fp32 = 3): nine int8 values times a per-block
// scale max|entry| / 127 kept to 16 mantissa bits (the fp32 scale's top 24 bits, the low byte of
// its word holds q8), so the largest entry maps to 127 and every entry is within half a scale of
// its value; the record is three 256-B dword runs per slot, (q0..q3) (q4..q7) (q8 | scale bits
// 8..31): 12 B per block against 20 for fp16.  Symmetric as the fp16 copy (a block and its
// transpose share the scale).  With the Krylov operator and the stop rule in fp64 only the
// preconditioner moves: 18-19 PCG iterations per solve against 18 with the fp16 copy, the
// headline +5.7 % (a power-of-two scale, 10 B per block, took 19-20 and +4.0 %).
template <typename T>
constexpr int slot_vals() { return sizeof(T) == 1 ? 12 : sizeof(T) == 2 ? 10 : 9; }

// storage type of the smoother inverse on a level whose operator values are stored as T: fp64
// with fp64 operators, fp32 on the reduced-precision levels (precond_fp32 >= 1)
template <typename T>
using SmoothInv = typename std::conditional<sizeof(T) == 8, double, float>::type;

__device__ __forceinline__ double h16_lo(uint32_t w) {
    return (double)__builtin_bit_cast(_Float16, (uint16_t)(w & 0xFFFFu));
}
__device__ __forceinline__ double h16_hi(uint32_t w) { return (double)__builtin_bit_cast(_Float16, (uint16_t)(w >> 16)); }

// host: one block (9 fp64 entries, row-major) -> the ten-half record
inline void to_h16_block(const double* v, uint16_t* rec) {
    double m = 0.0;
    for (int k = 0; k < 9; ++k) m = std::max(m, std::fabs(v[k]));
    int e = 0;
    if (m > 0.0) std::frexp(m, &e);
    for (int k = 0; k < 9; ++k) rec[k] = __builtin_bit_cast(uint16_t, (_Float16)std::ldexp(v[k], -e));
    rec[9] = (uint16_t)(int16_t)e;
}

// host: one block -> the twelve-byte int8 record (nine values, then the scale's bits 8..31)
inline bool to_q8_block(const double* v, uint8_t* rec) {
    double m = 0.0;
    for (int k = 0; k < 9; ++k) m = std::max(m, std::fabs(v[k]));
    const float s32 = (float)(m / 127.0);
    if (m > 0.0 && !(s32 > 0.0f && std::isfinite(s32) && std::isnormal(s32))) return false;
    const uint32_t bits = __builtin_bit_cast(uint32_t, s32) & 0xFFFFFF00u;
    const double sc = (double)__builtin_bit_cast(float, bits);
    for (int k = 0; k < 9; ++k)
        rec[k] = (uint8_t)(int8_t)(sc > 0.0 ? std::max(-127.0, std::min(127.0, std::nearbyint(v[k] / sc))) : 0.0);
    rec[9] = (uint8_t)(bits >> 8);
    rec[10] = (uint8_t)(bits >> 16);
    rec[11] = (uint8_t)(bits >> 24);
    return true;
}

// position of record byte k (0..11) of `lane` in a 768-B int8 slot
inline int64_t q8_pos(int k, int64_t lane) { return 256 * (k / 4) + 4 * lane + k % 4; }

// stored bytes of one 3x3 block's values in storage type vt (ValType)
inline double vbytes(int vt) {
    return vt == kValQ8 ? 12.0 : vt == kValH16 ? 20.0 : vt == kVal32 ? 36.0 : 72.0;
}

template <typename T>
__host__ __device__ inline int64_t slot_elem(int ij, int64_t lane) {
    if (!paired_values<T>()) return (int64_t)ij * kChunk + lane;
    return ij == 8 ? 512 + lane : 128 * (ij / 2) + 2 * lane + ij % 2;
}

// x_j gathered for a block product: three fp64 values at stride 3 (three 8-B loads), or -- the
// multicolour sweeps' fp32 iterate copy (GsFine::x4, precond_fp32 = 4) -- one 16-B load of the
// node's (x0, x1, x2, 0) in fp32, widened to fp64
struct X3 {
    double a, b, c;
};
__device__ __forceinline__ X3 ldx(const double* x, int64_t j) { return X3{x[3 * j], x[3 * j + 1], x[3 * j + 2]}; }
__device__ __forceinline__ X3 ldx(const float4* x, int64_t j) {
    const float4 v = x[j];
    return X3{(double)v.x, (double)v.y, (double)v.z};
}

// 3x3 block times x_j, accumulated in fp64; v = slot base + lane.  The matrix is streamed once
// per launch (NT: non-temporal loads, leaving the caches to the x gathers).
template <bool NT, typename T>
__device__ __forceinline__ void block_fma_any(const T* v, X3 xj, double& s0, double& s1, double& s2, int lane) {
    const double x0 = xj.a, x1 = xj.b, x2 = xj.c;
    auto ldv = [](const auto* p) { if constexpr (NT) return __builtin_nontemporal_load(p); else return *p; };
    // row . x as fma(v2, x2, fma(v1, x1, v0 x0)), added to the accumulator: the contraction is
    // spelled out so every kernel instantiating this rounds alike (left to fp-contract, the
    // compiler fused different products in different kernels, e.g. the colour sweeps over
    // column-indexed and stencil-coded slots)
    auto dot3 = [x0, x1, x2](double v0, double v1, double v2) { return __builtin_fma(v2, x2, __builtin_fma(v1, x1, v0 * x0)); };
    if constexpr (sizeof(T) == 1) {
        // v = slot base + lane in bytes; the lane's dwords at 4 lane, 256 + 4 lane, 512 + 4 lane
        const uint32_t* p = reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(v) - lane) + lane;
        const uint32_t a = ldv(p), b = ldv(p + 64), c = ldv(p + 128);
        auto q = [](uint32_t w, int k) { return (double)((int32_t)(w << (24 - 8 * k)) >> 24); };  // signed byte k
        const double sc = (double)__builtin_bit_cast(float, c & 0xFFFFFF00u);
        s0 = __builtin_fma(sc, dot3(q(a, 0), q(a, 1), q(a, 2)), s0);
        s1 = __builtin_fma(sc, dot3(q(a, 3), q(b, 0), q(b, 1)), s1);
        s2 = __builtin_fma(sc, dot3(q(b, 2), q(b, 3), q(c, 0)), s2);
    } else if constexpr (sizeof(T) == 2) {
        // v = slot base + lane in halves; the lane's dword of pair p is at dword 64 p + lane
        const uint32_t* p = reinterpret_cast<const uint32_t*>(v - lane) + lane;
        const uint32_t a = ldv(p), b = ldv(p + 64), c = ldv(p + 128), d = ldv(p + 192), e = ldv(p + 256);
        const double sc = __builtin_amdgcn_ldexp(1.0, (int)(int16_t)(e >> 16));
        s0 = __builtin_fma(sc, dot3(h16_lo(a), h16_hi(a), h16_lo(b)), s0);
        s1 = __builtin_fma(sc, dot3(h16_hi(b), h16_lo(c), h16_hi(c)), s1);
        s2 = __builtin_fma(sc, dot3(h16_lo(d), h16_hi(d), h16_lo(e)), s2);
    } else if constexpr (paired_values<T>() && sizeof(T) == 8) {
        const dbl2_t* p = reinterpret_cast<const dbl2_t*>(v - lane) + lane;
        const dbl2_t a = ldv(p), b = ldv(p + 64), c = ldv(p + 128), d = ldv(p + 192);
        const double v8 = ldv(v + 512);
        s0 = s0 + dot3(a.x, a.y, b.x);
        s1 = s1 + dot3(b.y, c.x, c.y);
        s2 = s2 + dot3(d.x, d.y, v8);
    } else {
        auto ld = [&](int i) { return (double)ldv(v + i * kChunk); };
        s0 = s0 + dot3(ld(0), ld(1), ld(2));
        s1 = s1 + dot3(ld(3), ld(4), ld(5));
        s2 = s2 + dot3(ld(6), ld(7), ld(8));
    }
}

template <typename T>
__device__ __forceinline__ void block_fma(const T* v, X3 xj, double& s0, double& s1, double& s2) {
    block_fma_any<true>(v, xj, s0, s1, s2, threadIdx.x & 63);
}

template <typename T>
__device__ __forceinline__ void block_fma_plain(const T* v, X3 xj, double& s0, double& s1, double& s2) {
    block_fma_any<false>(v, xj, s0, s1, s2, threadIdx.x & 63);
}

// Row sums of one chunk, loop variant V (the production kernels use default_variant; the others
// are kept for mgpis_gpu_bench_spmv, which times them on a live operator):
//   0  slot loop unrolled x3, cached loads
//   1  as 0 with non-temporal matrix loads
//   2  groups of 3 slots with the next group's columns prefetched, non-temporal matrix loads
// Column of slot k for this lane: CT = int32_t holds the block column, CT = int16_t its offset
// from the row's own node (col16: every |column - row| of the level < 2^15, which the
// lexicographic device numbering gives for subdomains up to ~180 x 180 nodes per plane) --
// 2 B instead of 4 per block.
template <typename CT>
__device__ __forceinline__ int64_t col_of(CT c, int64_t row) {
    if constexpr (sizeof(CT) == 2) return row + (int64_t)c;
    else return (int64_t)c;
}

// slot-loop unroll of the sweeps gathering an fp32 iterate copy (colour sweeps, block-Jacobi
// levels; A/B builds: -DDDPCA_GS_UNROLL=n)
#ifndef DDPCA_GS_UNROLL
#define DDPCA_GS_UNROLL 3
#endif
constexpr int kGsUnroll = DDPCA_GS_UNROLL;

template <int V, typename T, typename CT = int32_t, typename XT = double, int U = 3>
__device__ __forceinline__ void sell_rows(const CT* colp, const T* valp, const XT* x, int ns, int64_t row,
                                          double& s0, double& s1, double& s2) {
    constexpr int64_t SV = slot_vals<T>() * kChunk;
    if constexpr (V == 0) {
#pragma unroll 3
        for (int k = 0; k < ns; ++k)
            block_fma_plain(valp + (int64_t)k * SV, ldx(x, col_of(colp[(int64_t)k * kChunk], row)), s0, s1, s2);
    } else if constexpr (V == 1) {
#pragma unroll U
        for (int k = 0; k < ns; ++k)
            block_fma(valp + (int64_t)k * SV, ldx(x, col_of(__builtin_nontemporal_load(colp + (int64_t)k * kChunk), row)),
                      s0, s1, s2);
    } else if constexpr (V == 3) {
        // diagnostic bound only (wrong product): as 1 but x gathered at the row's own node, i.e.
        // perfectly coalesced gathers -- what a locality-optimal node numbering could approach
#pragma unroll 3
        for (int k = 0; k < ns; ++k) {
            const int64_t j = col_of(__builtin_nontemporal_load(colp + (int64_t)k * kChunk), row);
            block_fma(valp + (int64_t)k * SV, ldx(x, row + (j & 0)), s0, s1, s2);
        }
    } else {
        int k = 0;
        CT c0 = 0, c1 = 0, c2 = 0;
        if (ns >= 3) {
            c0 = __builtin_nontemporal_load(colp);
            c1 = __builtin_nontemporal_load(colp + kChunk);
            c2 = __builtin_nontemporal_load(colp + 2 * kChunk);
        }
        for (; k + 3 <= ns; k += 3) {
            const int64_t j0 = col_of(c0, row), j1 = col_of(c1, row), j2 = col_of(c2, row);
            if (k + 6 <= ns) {
                c0 = __builtin_nontemporal_load(colp + (int64_t)(k + 3) * kChunk);
                c1 = __builtin_nontemporal_load(colp + (int64_t)(k + 4) * kChunk);
                c2 = __builtin_nontemporal_load(colp + (int64_t)(k + 5) * kChunk);
            }
            const T* v = valp + (int64_t)k * SV;
            block_fma(v, ldx(x, j0), s0, s1, s2);
            block_fma(v + SV, ldx(x, j1), s0, s1, s2);
            block_fma(v + 2 * SV, ldx(x, j2), s0, s1, s2);
        }
        for (; k < ns; ++k) block_fma(valp + (int64_t)k * SV, ldx(x, col_of(colp[(int64_t)k * kChunk], row)), s0, s1, s2);
    }
}

// Table mode: the row's blocks are the 9-double records tv[9k .. 9k+8] of its table row (shared
// with every row of the same type, so they come from L1/L2), columns prefetched one group ahead.
__device__ __forceinline__ void sell_rows_tbl(const int32_t* colp, const double* tv, const double* x, int ns,
                                              double& s0, double& s1, double& s2) {
    int k = 0;
    int32_t c0 = 0, c1 = 0, c2 = 0;
    if (ns >= 3) {
        c0 = __builtin_nontemporal_load(colp);
        c1 = __builtin_nontemporal_load(colp + kChunk);
        c2 = __builtin_nontemporal_load(colp + 2 * kChunk);
    }
    auto blk = [&](const double* v, const double* xj) {  // block_fma_any's contraction (bit-identical sums)
        const double x0 = xj[0], x1 = xj[1], x2 = xj[2];
        s0 = s0 + __builtin_fma(v[2], x2, __builtin_fma(v[1], x1, v[0] * x0));
        s1 = s1 + __builtin_fma(v[5], x2, __builtin_fma(v[4], x1, v[3] * x0));
        s2 = s2 + __builtin_fma(v[8], x2, __builtin_fma(v[7], x1, v[6] * x0));
    };
    for (; k + 3 <= ns; k += 3) {
        const int64_t j0 = c0, j1 = c1, j2 = c2;
        if (k + 6 <= ns) {
            c0 = __builtin_nontemporal_load(colp + (int64_t)(k + 3) * kChunk);
            c1 = __builtin_nontemporal_load(colp + (int64_t)(k + 4) * kChunk);
            c2 = __builtin_nontemporal_load(colp + (int64_t)(k + 5) * kChunk);
        }
        blk(tv + 9 * k, x + 3 * j0);
        blk(tv + 9 * (k + 1), x + 3 * j1);
        blk(tv + 9 * (k + 2), x + 3 * j2);
    }
    for (; k < ns; ++k) blk(tv + 9 * k, x + 3 * (int64_t)colp[(int64_t)k * kChunk]);
}

// Table mode, type-homogeneous chunk: the table row is wave-uniform, so its values are read with
// scalar loads into SGPRs (the FMAs take them as scalar operands): no per-lane value traffic.
// XV selects how x_j is read: 0 production (x stride 3, three 8-B loads); diagnostics for
// mgpis_gpu_bench_spmv: 3 x at the row's own node (coalesced bound, wrong product), 4 x stride 4
// as one 16-B + one 8-B load, 5 x stride 4 as two 16-B loads.
template <int XV = 0>
__device__ __forceinline__ void sell_rows_uniform(const int32_t* colp, const double* __restrict__ tv, const double* x,
                                                  int ns, int64_t row, double& s0, double& s1, double& s2) {
#pragma unroll 3
    for (int k = 0; k < ns; ++k) {
        const int64_t j = __builtin_nontemporal_load(colp + (int64_t)k * kChunk);
        double x0, x1, x2;
        if constexpr (XV == 3) {
            x0 = x[3 * row + (j & 0)];
            x1 = x[3 * row + 1];
            x2 = x[3 * row + 2];
        } else if constexpr (XV == 4) {
            const double2 a = reinterpret_cast<const double2*>(x)[2 * j];
            x0 = a.x;
            x1 = a.y;
            x2 = x[4 * j + 2];
        } else if constexpr (XV == 5) {
            const double2 a = reinterpret_cast<const double2*>(x)[2 * j];
            const double2 b = reinterpret_cast<const double2*>(x)[2 * j + 1];
            x0 = a.x;
            x1 = a.y;
            x2 = b.x;
        } else {
            x0 = x[3 * j];
            x1 = x[3 * j + 1];
            x2 = x[3 * j + 2];
        }
        const double* v = tv + 9 * k;
        s0 = s0 + __builtin_fma(v[2], x2, __builtin_fma(v[1], x1, v[0] * x0));
        s1 = s1 + __builtin_fma(v[5], x2, __builtin_fma(v[4], x1, v[3] * x0));
        s2 = s2 + __builtin_fma(v[8], x2, __builtin_fma(v[7], x1, v[6] * x0));
    }
}

// Production loop variant per mode.  Measured on a 1.22M-dof fine level (mgpis_gpu_bench_spmv):
// the column prefetch pays for the light-epilogue modes (y = Kx, residual), plain non-temporal
// streaming for the PCG and Chebyshev epilogues; an XCD-contiguous chunk mapping (each XCD one
// range of chunks) was 17 % slower than the dispatcher's round-robin and is gone.
constexpr int default_variant(int mode) { return (mode == 0 || mode == 1) ? 2 : 1; }

// One wavefront per 64-node chunk, one lane per node row, three accumulators per lane; T is the
// storage type of streamed operator values (all arithmetic fp64); TBL: values from the table.
template <int MODE, bool BJ, bool DOT, typename T = double, int V = default_variant(MODE), bool TBL = false,
          typename CT = int32_t, bool X4 = false>
__global__ __launch_bounds__(kBlock) void k_sell(SellArgs a, const double* __restrict__ tab) {
    const int lane = threadIdx.x & 63;
    const int64_t c = (int64_t)blockIdx.x * (kBlock / kWave) + (threadIdx.x >> 6);
    if (c >= a.nch) return;
    const int sub = a.csub[c];
    if (stopped(a.sc, sub)) return;
    const int64_t row = c * kChunk + lane;
    const int ns = a.slots[c];
    const int64_t base = a.off[c];
    double s0 = 0.0, s1 = 0.0, s2 = 0.0;
    if (TBL) {
        // table loop variants (mgpis_gpu_bench_spmv): 0 per-lane table rows only, 3/4/5 the
        // sell_rows_uniform diagnostics, others production
        const int ct = V == 0 ? -1 : __builtin_amdgcn_readfirstlane(a.ctype[c]);
        if (ct >= 0)
            sell_rows_uniform<(V >= 3 ? V : 0)>(a.col + base * kChunk + lane, tab + (int64_t)ct * a.tstride, a.x, ns, row,
                                                s0, s1, s2);
        else
            sell_rows_tbl(a.col + base * kChunk + lane, tab + (int64_t)a.rtype[row] * a.tstride, a.x, ns, s0, s1, s2);
    } else if constexpr (X4 && sizeof(CT) == 2)
        sell_rows<V, T, CT, float4, kGsUnroll>(a.col16 + base * kChunk + lane,
                                               static_cast<const T*>(a.val) + base * slot_vals<T>() * kChunk + lane, a.x4, ns,
                                               row, s0, s1, s2);
    else if constexpr (sizeof(CT) == 2)
        sell_rows<V, T, CT>(a.col16 + base * kChunk + lane, static_cast<const T*>(a.val) + base * slot_vals<T>() * kChunk + lane,
                            a.x, ns, row, s0, s1, s2);
    else
        sell_rows<V, T, CT>(a.col + base * kChunk + lane, static_cast<const T*>(a.val) + base * slot_vals<T>() * kChunk + lane,
                            a.x, ns, row, s0, s1, s2);
    double dotv = 0.0;
    const int64_t o = 3 * row;
    if (MODE == kSpmv) {
        a.y[o] = s0;
        a.y[o + 1] = s1;
        a.y[o + 2] = s2;
    } else if (MODE == kResid) {
        const double r0 = a.b[o] - s0, r1 = a.b[o + 1] - s1, r2 = a.b[o + 2] - s2;
        a.y[o] = r0;
        a.y[o + 1] = r1;
        a.y[o + 2] = r2;
        if (DOT) dotv = __builtin_fma(r2, r2, __builtin_fma(r1, r1, r0 * r0));
    } else if (MODE == kJac) {
        const double om = a.coef[2 * sub + 1];
        const double b0 = a.b[o], b1 = a.b[o + 1], b2 = a.b[o + 2];
        double m0, m1, m2;
        apply_m<BJ>(static_cast<const SmoothInv<T>*>(a.minv), row, b0 - s0, b1 - s1, b2 - s2, m0, m1, m2);
        // (explicit contraction throughout the epilogues: every instantiation rounds alike)
        double x0, x1, x2;
        if constexpr (X4) {
            const float4 xv = a.x4[row];
            x0 = xv.x, x1 = xv.y, x2 = xv.z;
        } else {
            x0 = a.x[o], x1 = a.x[o + 1], x2 = a.x[o + 2];
        }
        const double n0 = __builtin_fma(om, m0, x0), n1 = __builtin_fma(om, m1, x1), n2 = __builtin_fma(om, m2, x2);
        if (!X4 || a.xo) {
            a.xo[o] = n0;
            a.xo[o + 1] = n1;
            a.xo[o + 2] = n2;
        }
        if (X4 && a.xo4) a.xo4[row] = make_float4((float)n0, (float)n1, (float)n2, 0.0f);
        if (DOT) dotv = __builtin_fma(b2, n2, __builtin_fma(b1, n1, b0 * n0));
    } else if (MODE == kPcg) {
        // q = K z + beta q_old, p = z + beta p_old  (K p = K z + beta K p_old)
        const double be = a.sc[sub].beta;
        const double q0 = __builtin_fma(be, a.y[o], s0), q1 = __builtin_fma(be, a.y[o + 1], s1),
                     q2 = __builtin_fma(be, a.y[o + 2], s2);
        const double p0 = __builtin_fma(be, a.p[o], a.x[o]), p1 = __builtin_fma(be, a.p[o + 1], a.x[o + 1]),
                     p2 = __builtin_fma(be, a.p[o + 2], a.x[o + 2]);
        a.y[o] = q0;
        a.y[o + 1] = q1;
        a.y[o + 2] = q2;
        a.p[o] = p0;
        a.p[o + 1] = p1;
        a.p[o + 2] = p2;
        if (DOT) dotv = __builtin_fma(p2, q2, __builtin_fma(p1, q1, p0 * q0));
    } else if (MODE == kCheb) {
        const double c1 = a.coef[2 * sub], c2 = a.coef[2 * sub + 1];
        const double b0 = a.b[o], b1 = a.b[o + 1], b2 = a.b[o + 2];
        double m0, m1, m2;
        apply_m<BJ>(static_cast<const SmoothInv<T>*>(a.minv), row, b0 - s0, b1 - s1, b2 - s2, m0, m1, m2);
        const double d0 = __builtin_fma(c2, m0, c1 * a.p[o]), d1 = __builtin_fma(c2, m1, c1 * a.p[o + 1]),
                     d2 = __builtin_fma(c2, m2, c1 * a.p[o + 2]);
        a.p[o] = d0;
        a.p[o + 1] = d1;
        a.p[o + 2] = d2;
        const double n0 = a.x[o] + d0, n1 = a.x[o + 1] + d1, n2 = a.x[o + 2] + d2;
        a.xo[o] = n0;
        a.xo[o + 1] = n1;
        a.xo[o + 2] = n2;
        if (DOT) dotv = __builtin_fma(b2, n2, __builtin_fma(b1, n1, b0 * n0));
    }
    if (DOT) chunk_partial(dotv, a.partial, c);
}

// Small levels (fewer chunks than the chip has SIMDs): one workgroup per chunk, each of its four
// waves 16 of the chunk's rows, each lane a quarter of its row's slots (k = g, g + 4, ...), the
// quarters summed by lane shuffles -- four times the waves and a quarter of the dependent
// column -> x chain per lane.  Same operator bytes; y = Kx, residual and Jacobi-sweep epilogues
// (the V-cycle's small-level launches carry no dot product).
template <int MODE, bool BJ, typename T, typename CT, bool X4 = false>
__global__ __launch_bounds__(kBlock) void k_sell_split(SellArgs a) {
    const int64_t c = blockIdx.x;
    const int sub = a.csub[c];
    if (stopped(a.sc, sub)) return;
    const int lane = threadIdx.x & 63;
    const int rin = (threadIdx.x >> 6) * 16 + (lane & 15), g = lane >> 4;
    const int64_t row = c * kChunk + rin;
    const int ns = a.slots[c];
    const int64_t base = a.off[c];
    constexpr int64_t SV = slot_vals<T>() * kChunk;
    double s0 = 0.0, s1 = 0.0, s2 = 0.0;
    {
        const T* valp = static_cast<const T*>(a.val) + base * SV + rin;
        const CT* colp;
        if constexpr (sizeof(CT) == 2) colp = a.col16 + base * kChunk + rin;
        else colp = a.col + base * kChunk + rin;
#pragma unroll 2
        for (int k = g; k < ns; k += 4) {
            const int64_t j = col_of(colp[(int64_t)k * kChunk], row);
            if constexpr (X4) block_fma_any<true>(valp + (int64_t)k * SV, ldx(a.x4, j), s0, s1, s2, rin);
            else block_fma_any<true>(valp + (int64_t)k * SV, ldx(a.x, j), s0, s1, s2, rin);
        }
    }
    s0 += __shfl_xor(s0, 16, 64);
    s1 += __shfl_xor(s1, 16, 64);
    s2 += __shfl_xor(s2, 16, 64);
    s0 += __shfl_xor(s0, 32, 64);
    s1 += __shfl_xor(s1, 32, 64);
    s2 += __shfl_xor(s2, 32, 64);
    if (g != 0) return;
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
        const double om = a.coef[2 * sub + 1];
        double m0, m1, m2;
        apply_m<BJ>(static_cast<const SmoothInv<T>*>(a.minv), row, a.b[o] - s0, a.b[o + 1] - s1, a.b[o + 2] - s2, m0, m1, m2);
        if constexpr (X4) {
            const float4 xv = a.x4[row];
            const double n0 = (double)xv.x + om * m0, n1 = (double)xv.y + om * m1, n2 = (double)xv.z + om * m2;
            if (a.xo) {
                a.xo[o] = n0;
                a.xo[o + 1] = n1;
                a.xo[o + 2] = n2;
            }
            if (a.xo4) a.xo4[row] = make_float4((float)n0, (float)n1, (float)n2, 0.0f);
        } else {
            a.xo[o] = a.x[o] + om * m0;
            a.xo[o + 1] = a.x[o + 1] + om * m1;
            a.xo[o + 2] = a.x[o + 2] + om * m2;
        }
    }
}

// Multicolour block Gauss-Seidel on the fine level (GsFine): one wavefront per colour chunk,
// lane = one row of that colour.  PH 0: forward sweep from zero over the L part, x_i = M_i (b_i -
// L_i x); PH 1: the residual after the forward sweep, r_i = -U_i x (every chunk, one launch);
// PH 2: backward sweep, x_i = M_i (b_i - L_i x - U_i x), DOT: partial = b . x_new per chunk.
// In place: rows of one colour are never each other's neighbours.
struct GsArgs {
    const int32_t* list;  // chunk ids of this launch (nullptr: chunks 0 .. n-1)
    int64_t n;
    const int32_t* rowidx;
    const int32_t* csub;
    const int32_t* nsl;
    const int32_t* nsu;
    const int64_t* offl;
    const int64_t* offu;
    const int32_t* col;
    const int16_t* col16;
    const void* val;
    const void* minv;
    double* x;
    const double* b;
    double* r;
    const PcgScal* sc;
    double* partial;
    const float* minvc;  // chunk-ordered fp32 inverses (GsFine::minvc), or null (fp64 copy): minv by row
    float4* x4;          // the fp32 iterate copy the sweeps gather (GsFine::x4), or null
    float4* r4;          // X4 residual (PH 1) in fp32 for the restriction (GsFine::r4), or null: r in fp64
    double* w;           // SSOR (k_gs_ssor): the partial sums a sweep hands to the next one, 3 per row
};

// the colour sweep's per-row tail: PH 1 stores r = -s; PH 0 / 2 store x = M (b - s) and return
// its share of b.x (DOT); ln = the row's position in its colour chunk.  X4 (GsFine::x4): the new
// x goes to the fp32 iterate copy the sweeps gather; only the backward sweep (PH 2), whose x is
// the V-cycle's output, also writes it in fp64
template <int PH, bool DOT, typename T, bool X4 = false>
__device__ __forceinline__ double gs_epilogue(const GsArgs& a, int64_t c, int ln, int64_t row, bool real, double s0,
                                              double s1, double s2) {
    const int64_t o = 3 * row;
    double dotv = 0.0;
    if (PH == 1) {
        if (real) {
            if (X4 && a.r4) {
                a.r4[row] = make_float4((float)-s0, (float)-s1, (float)-s2, 0.0f);
            } else {
                a.r[o] = -s0;
                a.r[o + 1] = -s1;
                a.r[o + 2] = -s2;
            }
        }
    } else {
        const double b0 = a.b[o], b1 = a.b[o + 1], b2 = a.b[o + 2];
        double m0, m1, m2;
        if (a.minvc) {
            const float* m = a.minvc + c * 9 * kChunk + ln;
            const double r0 = b0 - s0, r1 = b1 - s1, r2 = b2 - s2;
            // explicit contraction, as in block_fma_any (bit-identical across instantiations)
            m0 = __builtin_fma((double)m[2 * kChunk], r2, __builtin_fma((double)m[kChunk], r1, (double)m[0] * r0));
            m1 = __builtin_fma((double)m[5 * kChunk], r2, __builtin_fma((double)m[4 * kChunk], r1, (double)m[3 * kChunk] * r0));
            m2 = __builtin_fma((double)m[8 * kChunk], r2, __builtin_fma((double)m[7 * kChunk], r1, (double)m[6 * kChunk] * r0));
        } else {
            apply_m<true>(static_cast<const SmoothInv<T>*>(a.minv), row, b0 - s0, b1 - s1, b2 - s2, m0, m1, m2);
        }
        if (real) {
            if (X4) a.x4[row] = make_float4((float)m0, (float)m1, (float)m2, 0.0f);
            if (!X4 || PH == 2) {
                a.x[o] = m0;
                a.x[o + 1] = m1;
                a.x[o + 2] = m2;
            }
            if (DOT) dotv = __builtin_fma(b2, m2, __builtin_fma(b1, m1, b0 * m0));
        }
    }
    return dotv;
}

// One wave per workgroup: a colour's chunks spread over more CUs than four-wave groups (+1 % at 8
// subdomains per GPU, profiles/r03j)
template <int PH, bool DOT, typename T, typename CT, bool X4 = false>
__global__ __launch_bounds__(kWave) void k_gs(GsArgs a) {
    const int lane = threadIdx.x;
    const int64_t li = blockIdx.x;
    if (li >= a.n) return;
    const int64_t c = a.list ? (int64_t)a.list[li] : li;
    const int sub = a.csub[c];
    if (stopped(a.sc, sub)) return;
    const int32_t rr = a.rowidx[c * kChunk + lane];
    const bool real = rr >= 0;
    const int64_t row = real ? rr : ~rr;  // pad lanes gather at a real row with zero blocks
    constexpr int64_t SV = slot_vals<T>() * kChunk;
    const T* val = static_cast<const T*>(a.val);
    double s0 = 0.0, s1 = 0.0, s2 = 0.0;
    const CT* colp;
    if constexpr (sizeof(CT) == 2) colp = a.col16;
    else colp = a.col;
    if (PH != 1) {
        const int64_t o = a.offl[c];
        if constexpr (X4) sell_rows<1, T, CT, float4, kGsUnroll>(colp + o * kChunk + lane, val + o * SV + lane, (const float4*)a.x4, a.nsl[c], row, s0, s1, s2);
        else sell_rows<1, T, CT>(colp + o * kChunk + lane, val + o * SV + lane, (const double*)a.x, a.nsl[c], row, s0, s1, s2);
    }
    if (PH != 0) {
        const int64_t o = a.offu[c];
        if constexpr (X4) sell_rows<1, T, CT, float4, kGsUnroll>(colp + o * kChunk + lane, val + o * SV + lane, (const float4*)a.x4, a.nsu[c], row, s0, s1, s2);
        else sell_rows<1, T, CT>(colp + o * kChunk + lane, val + o * SV + lane, (const double*)a.x, a.nsu[c], row, s0, s1, s2);
    }
    const double dotv = gs_epilogue<PH, DOT, T, X4>(a, c, lane, row, real, s0, s1, s2);
    if (DOT) chunk_partial(dotv, a.partial, c);
}

// Multicolour block SSOR on the fine level (opt.smoother = 4, the reference's MULT_VCYC smoothing
// order, MGPIS.h:64-76, 101-114: a forward AND a backward sweep before and after the coarse
// correction), with the reference's reuse of the previous sweep's partial sums (its p0 / p1) so
// that each sweep reads only the blocks it must: per row the sums L x, U x of the colour split
// (L = earlier colours), w = 3 doubles per row handed from one phase to the next.
//   PH 6  forward from zero:      x = M (b - L x),          w = L x                 (L)
//   PH 7  backward:               x = M (b - w - U x)                               (U)
//   PH 8  residual:               r = w - L x   (= b - M^-1 x - L x - U x)          (L)
//   PH 9  forward from P e:       x = M (b - L x - U x),    w = b - L x             (L + U)
//   PH 10 backward:               x = M (w - U x), DOT: b . x                       (U)
// Three operator passes per V-cycle against the Gauss-Seidel pair's two.
template <int PH, bool DOT, typename T, typename CT, bool X4 = false>
__global__ __launch_bounds__(kWave) void k_gs_ssor(GsArgs a) {
    const int lane = threadIdx.x;
    const int64_t li = blockIdx.x;
    if (li >= a.n) return;
    const int64_t c = a.list ? (int64_t)a.list[li] : li;
    const int sub = a.csub[c];
    if (stopped(a.sc, sub)) return;
    const int32_t rr = a.rowidx[c * kChunk + lane];
    const bool real = rr >= 0;
    const int64_t row = real ? rr : ~rr;
    constexpr int64_t SV = slot_vals<T>() * kChunk;
    const T* val = static_cast<const T*>(a.val);
    const CT* colp;
    if constexpr (sizeof(CT) == 2) colp = a.col16;
    else colp = a.col;
    double l0 = 0.0, l1 = 0.0, l2 = 0.0, u0 = 0.0, u1 = 0.0, u2 = 0.0;
    if constexpr (PH == 6 || PH == 8 || PH == 9) {
        const int64_t o = a.offl[c];
        if constexpr (X4) sell_rows<1, T, CT>(colp + o * kChunk + lane, val + o * SV + lane, (const float4*)a.x4, a.nsl[c], row, l0, l1, l2);
        else sell_rows<1, T, CT>(colp + o * kChunk + lane, val + o * SV + lane, (const double*)a.x, a.nsl[c], row, l0, l1, l2);
    }
    if constexpr (PH == 7 || PH == 9 || PH == 10) {
        const int64_t o = a.offu[c];
        if constexpr (X4) sell_rows<1, T, CT>(colp + o * kChunk + lane, val + o * SV + lane, (const float4*)a.x4, a.nsu[c], row, u0, u1, u2);
        else sell_rows<1, T, CT>(colp + o * kChunk + lane, val + o * SV + lane, (const double*)a.x, a.nsu[c], row, u0, u1, u2);
    }
    const int64_t o = 3 * row;
    if constexpr (PH == 8) {
        if (!real) return;
        const double r0 = a.w[o] - l0, r1 = a.w[o + 1] - l1, r2 = a.w[o + 2] - l2;
        if (X4 && a.r4) {
            a.r4[row] = make_float4((float)r0, (float)r1, (float)r2, 0.0f);
        } else {
            a.r[o] = r0;
            a.r[o + 1] = r1;
            a.r[o + 2] = r2;
        }
        return;
    } else {
        const double b0 = a.b[o], b1 = a.b[o + 1], b2 = a.b[o + 2];
        double c0, c1, c2;
        if constexpr (PH == 6) {
            c0 = b0 - l0, c1 = b1 - l1, c2 = b2 - l2;
        } else if constexpr (PH == 7) {
            c0 = (b0 - a.w[o]) - u0, c1 = (b1 - a.w[o + 1]) - u1, c2 = (b2 - a.w[o + 2]) - u2;
        } else if constexpr (PH == 9) {
            c0 = (b0 - l0) - u0, c1 = (b1 - l1) - u1, c2 = (b2 - l2) - u2;
        } else {
            c0 = a.w[o] - u0, c1 = a.w[o + 1] - u1, c2 = a.w[o + 2] - u2;
        }
        const float* m = a.minvc + c * 9 * kChunk + lane;
        const double m0 = __builtin_fma((double)m[2 * kChunk], c2, __builtin_fma((double)m[kChunk], c1, (double)m[0] * c0));
        const double m1 = __builtin_fma((double)m[5 * kChunk], c2, __builtin_fma((double)m[4 * kChunk], c1, (double)m[3 * kChunk] * c0));
        const double m2 = __builtin_fma((double)m[8 * kChunk], c2, __builtin_fma((double)m[7 * kChunk], c1, (double)m[6 * kChunk] * c0));
        double dotv = 0.0;
        if (real) {
            if constexpr (PH == 6) {
                a.w[o] = l0;
                a.w[o + 1] = l1;
                a.w[o + 2] = l2;
            } else if constexpr (PH == 9) {
                a.w[o] = b0 - l0;
                a.w[o + 1] = b1 - l1;
                a.w[o + 2] = b2 - l2;
            }
            // x4 mode: every sweep writes the fp32 copy the later colours gather; the last backward
            // sweep (PH 10) also the fp64 output z
            if (X4) a.x4[row] = make_float4((float)m0, (float)m1, (float)m2, 0.0f);
            if (!X4 || PH == 10) {
                a.x[o] = m0;
                a.x[o + 1] = m1;
                a.x[o + 2] = m2;
            }
            if (DOT) dotv = __builtin_fma(b2, m2, __builtin_fma(b1, m1, b0 * m0));
        }
        if (DOT) chunk_partial(dotv, a.partial, c);
    }
}

// Band mode's rows outside the colours (GsFine::band; one wave per chunk of the ring / far groups):
// PH 5: x = 0, r = b before the forward sweep (the ring's r is recomputed by PH 3); PH 3: the
// ring's residual r = b - K x over its stored band columns (x is zero elsewhere after the forward
// sweep from zero); PH 4: the dot product's chunk partial b . x of rows the backward sweep leaves
// as the prolongation wrote them
template <int PH, typename T, typename CT>
__global__ __launch_bounds__(kWave) void k_gs_aux(GsArgs a) {
    const int lane = threadIdx.x;
    const int64_t li = blockIdx.x;
    if (li >= a.n) return;
    const int64_t c = a.list[li];
    const int sub = a.csub[c];
    if (stopped(a.sc, sub)) return;
    const int32_t rr = a.rowidx[c * kChunk + lane];
    const bool real = rr >= 0;
    const int64_t row = real ? rr : ~rr;
    const int64_t o = 3 * row;
    if (PH == 5) {
        if (real)
            for (int e = 0; e < 3; ++e) {
                a.x[o + e] = 0.0;
                a.r[o + e] = a.b[o + e];
            }
        return;
    }
    if (PH == 4) {
        const double d = real ? __builtin_fma(a.b[o + 2], a.x[o + 2], __builtin_fma(a.b[o + 1], a.x[o + 1], a.b[o] * a.x[o])) : 0.0;
        chunk_partial(d, a.partial, c);
        return;
    }
    double s0 = 0.0, s1 = 0.0, s2 = 0.0;
    const CT* colp;
    if constexpr (sizeof(CT) == 2) colp = a.col16;
    else colp = a.col;
    constexpr int64_t SV = slot_vals<T>() * kChunk;
    const int64_t q = a.offl[c];
    sell_rows<1, T, CT>(colp + q * kChunk + lane, static_cast<const T*>(a.val) + q * SV + lane, (const double*)a.x, a.nsl[c], row, s0, s1, s2);
    if (real) {
        a.r[o] = a.b[o] - s0;
        a.r[o + 1] = a.b[o + 1] - s1;
        a.r[o + 2] = a.b[o + 2] - s2;
    }
}

// Node-parallel kernels: thread = node, 256 nodes per workgroup; a wavefront is one chunk, so
// the subdomain (and its stop flag) is uniform per wavefront.  nn is a multiple of 64.
#define NODE_PROLOGUE(nn, csub, sc)                         \
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; \
    if (i >= (nn)) return;                                  \
    const int sub = (csub)[i >> 6];                         \
    if (stopped((sc), sub)) return;

// x = omega M b  (first smoothing sweep from a zero guess); CHEB: also d = x
// (x4: the level's fp32 iterate copy takes x instead, LevelDev::x4a)
template <bool BJ, bool SETD, typename MT = double>
__global__ __launch_bounds__(kBlock) void k_jac0(const double* b, const MT* minv, const double* coef, double* x,
                                                 double* d, int64_t nn, const int32_t* csub, const PcgScal* sc,
                                                 float4* x4 = nullptr) {
    NODE_PROLOGUE(nn, csub, sc)
    const double om = coef[2 * sub + 1];
    double m0, m1, m2;
    apply_m<BJ>(minv, i, b[3 * i], b[3 * i + 1], b[3 * i + 2], m0, m1, m2);
    if (x4) {
        x4[i] = make_float4((float)(om * m0), (float)(om * m1), (float)(om * m2), 0.0f);
    } else {
        x[3 * i] = om * m0;
        x[3 * i + 1] = om * m1;
        x[3 * i + 2] = om * m2;
    }
    if (SETD) {
        d[3 * i] = om * m0;
        d[3 * i + 1] = om * m1;
        d[3 * i + 2] = om * m2;
    }
}

// b_c = mask_c (sum_children w r_f[child]), the coarse node's own fine copy first with w = 1;
// optionally x_c = omega M b_c (CHEB: d_c too).  Children in SELL-64 layout: slot k of chunk c
// at (roff[c] + k) * 64 + lane, so index and weight loads are contiguous wave accesses.
// 1/k for the uniform-averaging stencils (weight = 1 / number of parents; k_prolong<true>)
__constant__ double kInvCount[9] = {0.0, 1.0, 0.5, 1.0 / 3.0, 0.25, 0.2, 1.0 / 6.0, 1.0 / 7.0, 0.125};

// restriction epilogue: b_c = mask s; INIT: x_c = omega M b_c (SETD: d_c = x_c)
template <bool INIT, bool BJ, bool SETD, typename MT>
__device__ __forceinline__ void restrict_store(const uint8_t* cmask, double* bc, double* xc, double* dc, const MT* minv,
                                               const double* coef, int64_t j, int sub, double s0, double s1,
                                               double s2, float4* xc4) {
    const uint8_t m = cmask[j];
    s0 = (m & 1) ? s0 : 0.0;
    s1 = (m & 2) ? s1 : 0.0;
    s2 = (m & 4) ? s2 : 0.0;
    bc[3 * j] = s0;
    bc[3 * j + 1] = s1;
    bc[3 * j + 2] = s2;
    if (INIT) {
        const double om = coef[2 * sub + 1];
        double m0, m1, m2;
        apply_m<BJ>(minv, j, s0, s1, s2, m0, m1, m2);
        if (xc4) {  // the coarse level's fp32 iterate copy (LevelDev::x4a) instead of x_c
            xc4[j] = make_float4((float)(om * m0), (float)(om * m1), (float)(om * m2), 0.0f);
        } else {
            xc[3 * j] = om * m0;
            xc[3 * j + 1] = om * m1;
            xc[3 * j + 2] = om * m2;
        }
        if (SETD) {
            dc[3 * j] = om * m0;
            dc[3 * j + 1] = om * m1;
            dc[3 * j + 2] = om * m2;
        }
    }
}

template <bool INIT, bool BJ, bool SETD, typename MT = double>
__global__ __launch_bounds__(kBlock) void k_restrict(const double* rf, const int32_t* rslots, const int64_t* roff,
                                                     const int32_t* rcol, const double* rwt, const uint8_t* cmask,
                                                     double* bc, double* xc, double* dc, const MT* minv,
                                                     const double* coef, int64_t nc, const int32_t* csub,
                                                     const PcgScal* sc, float4* xc4) {
    NODE_PROLOGUE(nc, csub, sc)
    const int64_t j = i, c = j >> 6;
    const int ns = rslots[c];
    const int32_t* cp = rcol + roff[c] * kChunk + (j & 63);
    const double* wp = rwt + roff[c] * kChunk + (j & 63);
    double s0 = 0.0, s1 = 0.0, s2 = 0.0;
#pragma unroll 4
    for (int k = 0; k < ns; ++k) {
        const int64_t f = __builtin_nontemporal_load(cp + (int64_t)k * kChunk);
        const double w = __builtin_nontemporal_load(wp + (int64_t)k * kChunk);
        s0 += w * rf[3 * f];
        s1 += w * rf[3 * f + 1];
        s2 += w * rf[3 * f + 2];
    }
    restrict_store<INIT, BJ, SETD>(cmask, bc, xc, dc, minv, coef, j, sub, s0, s1, s2, xc4);
}

// Lattice restriction (LevelDev::lat): children f0 + d0 t0 + d1 t1 + d2 t2 for the bits of the
// coarse node's 27-bit mask, weight 2^-(|d0|+|d1|+|d2|); every index is computed, the 27 gathers
// are independent (no index / weight stream)
template <bool INIT, bool BJ, bool SETD, typename MT = double, typename RT = double>
__global__ __launch_bounds__(kBlock) void k_restrict_lat(const RT* rf, const uint32_t* rmsk, const int32_t* rf0,
                                                         const int32_t* rstr, const uint8_t* cmask, double* bc,
                                                         double* xc, double* dc, const MT* minv, const double* coef,
                                                         int64_t nc, const int32_t* csub, const PcgScal* sc,
                                                         float4* xc4) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= nc) return;
    const int sub = csub[i >> 6];
    if (stopped(sc, sub)) return;
    const int64_t j = i;
    const uint32_t msk = rmsk[j];
    const int64_t f0 = rf0[j];
    const int64_t t0 = rstr[3 * sub], t1 = rstr[3 * sub + 1], t2 = rstr[3 * sub + 2];
    double s0 = 0.0, s1 = 0.0, s2 = 0.0;
#pragma unroll
    for (int q = 0; q < 27; ++q) {
        const int d0 = q % 3 - 1, d1 = (q / 3) % 3 - 1, d2 = q / 9 - 1;
        const double w = 1.0 / (double)(1 << ((d0 != 0) + (d1 != 0) + (d2 != 0)));
        const int64_t f = f0 + d0 * t0 + d1 * t1 + d2 * t2;
        if ((msk >> q) & 1u) {
            const X3 v = ldx(rf, f);  // RT = float4: the fine residual's fp32 copy (GsFine::r4), one 16-B load
            s0 += w * v.a;
            s1 += w * v.b;
            s2 += w * v.c;
        }
    }
    restrict_store<INIT, BJ, SETD>(cmask, bc, xc, dc, minv, coef, j, sub, s0, s1, s2, xc4);
}

// x_f += mask_f (P e_c)
template <bool UW = false>  // UW: weights 1 / parent count (see k_restrict), pw unread
__global__ __launch_bounds__(kBlock) void k_prolong(const double* ec, const int32_t* ppar, const double* pw,
                                                    const uint8_t* fmask, double* xf, int64_t nf, const int32_t* csub,
                                                    const PcgScal* sc) {
    NODE_PROLOGUE(nf, csub, sc)
    double e0 = 0.0, e1 = 0.0, e2 = 0.0;
    int np = 0;
#pragma unroll
    for (int p = 0; p < 8; ++p) {
        const int32_t c = ppar[p * nf + i];
        if (c < 0) break;
        const double w = UW ? 1.0 : pw[p * nf + i];
        e0 += w * ec[3 * (int64_t)c];
        e1 += w * ec[3 * (int64_t)c + 1];
        e2 += w * ec[3 * (int64_t)c + 2];
        ++np;
    }
    if (UW) {
        const double w = kInvCount[np];
        e0 *= w;
        e1 *= w;
        e2 *= w;
    }
    const uint8_t m = fmask[i];
    if (m & 1) xf[3 * i] += e0;
    if (m & 2) xf[3 * i + 1] += e1;
    if (m & 4) xf[3 * i + 2] += e2;
}

// the same into a block-Jacobi level's fp32 iterate copy (LevelDev::x4a): the sum and the add in fp64
template <bool UW = false>
__global__ __launch_bounds__(kBlock) void k_prolong_x4(const double* ec, const int32_t* ppar, const double* pw,
                                                       const uint8_t* fmask, float4* x4, int64_t nf, const int32_t* csub,
                                                       const PcgScal* sc) {
    NODE_PROLOGUE(nf, csub, sc)
    double e0 = 0.0, e1 = 0.0, e2 = 0.0;
    int np = 0;
#pragma unroll
    for (int p = 0; p < 8; ++p) {
        const int32_t c = ppar[p * nf + i];
        if (c < 0) break;
        const double w = UW ? 1.0 : pw[p * nf + i];
        e0 += w * ec[3 * (int64_t)c];
        e1 += w * ec[3 * (int64_t)c + 1];
        e2 += w * ec[3 * (int64_t)c + 2];
        ++np;
    }
    if (UW) {
        const double w = kInvCount[np];
        e0 *= w;
        e1 *= w;
        e2 *= w;
    }
    const uint8_t m = fmask[i];
    float4 v = x4[i];
    if (m & 1) v.x = (float)((double)v.x + e0);
    if (m & 2) v.y = (float)((double)v.y + e1);
    if (m & 4) v.z = (float)((double)v.z + e2);
    x4[i] = v;
}

// Lattice prolongation (LevelDev::lat): parents p0 + the subset sums of the coarse strides the
// node's code selects, weight 1 / 2^popcount(code); one 4-B word per fine node, the (up to 8)
// parent gathers independent of each other
__global__ __launch_bounds__(kBlock) void k_prolong_lat(const double* ec, const uint32_t* ppk, const int32_t* pstr,
                                                        const uint8_t* fmask, double* xf, int64_t nf,
                                                        const int32_t* csub, const PcgScal* sc) {
    NODE_PROLOGUE(nf, csub, sc)
    const uint32_t w = ppk[i];
    const int64_t p0 = w & 0x1fffffffu;
    const uint32_t code = w >> 29;
    const int64_t s0 = pstr[3 * sub], s1 = pstr[3 * sub + 1], s2 = pstr[3 * sub + 2];
    double e0 = 0.0, e1 = 0.0, e2 = 0.0;
    // every lane issues all eight parent loads (a parent outside the node's subset reads p0 and
    // weighs 0): no divergent branches, the loads issue back to back (47.8 -> 46.0 us per fine
    // launch against the branching form, profiles/r02m_prolong_ab.txt)
#pragma unroll
    for (uint32_t q = 0; q < 8; ++q) {
        const bool in = (q & ~code) == 0;
        const int64_t c = in ? p0 + ((q & 1) ? s0 : 0) + ((q & 2) ? s1 : 0) + ((q & 4) ? s2 : 0) : p0;
        const double w = in ? 1.0 : 0.0;
        e0 += w * ec[3 * c];
        e1 += w * ec[3 * c + 1];
        e2 += w * ec[3 * c + 2];
    }
    const double wt = 1.0 / (double)(1 << __popc(code));
    const uint8_t m = fmask[i];
    if (m & 1) xf[3 * i] += wt * e0;
    if (m & 2) xf[3 * i + 1] += wt * e1;
    if (m & 4) xf[3 * i + 2] += wt * e2;
}

// The same into the multicolour sweeps' fp32 iterate copy (GsFine::x4): x4_f = fp32(x4_f + mask_f
// 2^-k sum e_c), the sum and the add in fp64 -- what the backward sweep then gathers
__global__ __launch_bounds__(kBlock) void k_prolong_lat_x4(const double* ec, const uint32_t* ppk, const int32_t* pstr,
                                                           const uint8_t* fmask, float4* x4, int64_t nf,
                                                           const int32_t* csub, const PcgScal* sc) {
    NODE_PROLOGUE(nf, csub, sc)
    const uint32_t w = ppk[i];
    const int64_t p0 = w & 0x1fffffffu;
    const uint32_t code = w >> 29;
    const int64_t s0 = pstr[3 * sub], s1 = pstr[3 * sub + 1], s2 = pstr[3 * sub + 2];
    double e0 = 0.0, e1 = 0.0, e2 = 0.0;
#pragma unroll
    for (uint32_t q = 0; q < 8; ++q) {
        const bool in = (q & ~code) == 0;
        const int64_t c = in ? p0 + ((q & 1) ? s0 : 0) + ((q & 2) ? s1 : 0) + ((q & 4) ? s2 : 0) : p0;
        const double w = in ? 1.0 : 0.0;
        e0 += w * ec[3 * c];
        e1 += w * ec[3 * c + 1];
        e2 += w * ec[3 * c + 2];
    }
    const double wt = 1.0 / (double)(1 << __popc(code));
    const uint8_t m = fmask[i];
    float4 v = x4[i];
    if (m & 1) v.x = (float)((double)v.x + wt * e0);
    if (m & 2) v.y = (float)((double)v.y + wt * e1);
    if (m & 4) v.z = (float)((double)v.z + wt * e2);
    x4[i] = v;
}

// Block transfer entries (rotated nodes): x_f += mask_f (B e_c) per fine node that owns one
// (after k_prolong, whose weight for those entries is 0); thread = fine node.
__global__ __launch_bounds__(kBlock) void k_prolong_rot(const double* ec, const int32_t* row, const int64_t* ptr,
                                                        const int32_t* par, const double* blk, const uint8_t* fmask,
                                                        double* xf, int64_t nr, const int32_t* csub,
                                                        const PcgScal* sc) {
    const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (t >= nr) return;
    const int64_t i = row[t];
    if (stopped(sc, csub[i >> 6])) return;
    double e0 = 0.0, e1 = 0.0, e2 = 0.0;
    for (int64_t k = ptr[t]; k < ptr[t + 1]; ++k) {
        const double* B = blk + 9 * k;
        const int64_t c = par[k];
        const double c0 = ec[3 * c], c1 = ec[3 * c + 1], c2 = ec[3 * c + 2];
        e0 += B[0] * c0 + B[1] * c1 + B[2] * c2;
        e1 += B[3] * c0 + B[4] * c1 + B[5] * c2;
        e2 += B[6] * c0 + B[7] * c1 + B[8] * c2;
    }
    const uint8_t m = fmask[i];
    if (m & 1) xf[3 * i] += e0;
    if (m & 2) xf[3 * i + 1] += e1;
    if (m & 4) xf[3 * i + 2] += e2;
}

// the same into a block-Jacobi level's fp32 iterate copy (LevelDev::x4a), after k_prolong_x4
__global__ __launch_bounds__(kBlock) void k_prolong_rot_x4(const double* ec, const int32_t* row, const int64_t* ptr,
                                                           const int32_t* par, const double* blk, const uint8_t* fmask,
                                                           float4* x4, int64_t nr, const int32_t* csub,
                                                           const PcgScal* sc) {
    const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (t >= nr) return;
    const int64_t i = row[t];
    if (stopped(sc, csub[i >> 6])) return;
    double e0 = 0.0, e1 = 0.0, e2 = 0.0;
    for (int64_t k = ptr[t]; k < ptr[t + 1]; ++k) {
        const double* B = blk + 9 * k;
        const int64_t c = par[k];
        const double c0 = ec[3 * c], c1 = ec[3 * c + 1], c2 = ec[3 * c + 2];
        e0 += B[0] * c0 + B[1] * c1 + B[2] * c2;
        e1 += B[3] * c0 + B[4] * c1 + B[5] * c2;
        e2 += B[6] * c0 + B[7] * c1 + B[8] * c2;
    }
    const uint8_t m = fmask[i];
    float4 v = x4[i];
    if (m & 1) v.x = (float)((double)v.x + e0);
    if (m & 2) v.y = (float)((double)v.y + e1);
    if (m & 4) v.z = (float)((double)v.z + e2);
    x4[i] = v;
}

// ... and b_c += mask_c (B^T r_f) per coarse node that receives one (after k_restrict).
__global__ __launch_bounds__(kBlock) void k_restrict_rot(const double* rf, const int32_t* row, const int64_t* ptr,
                                                         const int32_t* kid, const double* blk, const uint8_t* cmask,
                                                         double* bc, int64_t nr, const int32_t* csub,
                                                         const PcgScal* sc) {
    const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (t >= nr) return;
    const int64_t j = row[t];
    if (stopped(sc, csub[j >> 6])) return;
    double s0 = 0.0, s1 = 0.0, s2 = 0.0;
    for (int64_t k = ptr[t]; k < ptr[t + 1]; ++k) {
        const double* B = blk + 9 * k;
        const int64_t f = kid[k];
        const double r0 = rf[3 * f], r1 = rf[3 * f + 1], r2 = rf[3 * f + 2];
        s0 += B[0] * r0 + B[3] * r1 + B[6] * r2;
        s1 += B[1] * r0 + B[4] * r1 + B[7] * r2;
        s2 += B[2] * r0 + B[5] * r1 + B[8] * r2;
    }
    const uint8_t m = cmask[j];
    if (m & 1) bc[3 * j] += s0;
    if (m & 2) bc[3 * j + 1] += s1;
    if (m & 4) bc[3 * j + 2] += s2;
}

// x0 = A0^-1 b0 per subdomain, one wavefront per coarse dof row.  Rows are padded to a multiple of
// 4 entries (ld, zero-filled), so every lane loads 16 B of the inverse per instruction (four fp32
// or two fp64 entries) and the matching b entries as fp64 pairs; two such loads in flight per lane.
// The padding reads b of the member's padding nodes, which the masked restriction keeps at zero.
template <typename AT = double>
__global__ __launch_bounds__(kBlock) void k_coarse(const AT* ainv, const int64_t* aoff, const int64_t* noff,
                                                   const int64_t* n0, const int64_t* ldv, const double* b, double* x,
                                                   int64_t nrow, const int32_t* csub, const PcgScal* sc) {
    const int64_t r = (int64_t)blockIdx.x * (kBlock / kWave) + (threadIdx.x >> 6);
    if (r >= nrow) return;
    const int sub = csub[(r / 3) >> 6];
    if (stopped(sc, sub)) return;
    const int lane = threadIdx.x & 63;
    const int64_t lr = r - 3 * noff[sub], n = n0[sub], ld = ldv[sub];
    if (lr >= n) {
        if (lane == 0) x[r] = 0.0;
        return;
    }
    const AT* arow = ainv + aoff[sub] + lr * ld;
    const double* bs = b + 3 * noff[sub];
    constexpr int V = 16 / sizeof(AT);  // entries per 16-B load
    double s0 = 0.0, s1 = 0.0;
    auto chunk = [&](int64_t k) {
        double acc = 0.0;
        if constexpr (V == 4) {
            const float4 a = *reinterpret_cast<const float4*>(arow + k);
            const double2 b0 = *reinterpret_cast<const double2*>(bs + k), b1 = *reinterpret_cast<const double2*>(bs + k + 2);
            acc = (double)a.x * b0.x + (double)a.y * b0.y + (double)a.z * b1.x + (double)a.w * b1.y;
        } else {
            const double2 a = *reinterpret_cast<const double2*>(arow + k);
            const double2 b0 = *reinterpret_cast<const double2*>(bs + k);
            acc = a.x * b0.x + a.y * b0.y;
        }
        return acc;
    };
    int64_t k = (int64_t)V * lane;
    for (; k + V * kWave < ld; k += 2 * V * kWave) {
        s0 += chunk(k);
        s1 += chunk(k + V * kWave);
    }
    if (k < ld) s0 += chunk(k);
    const double s = wave_sum(s0 + s1);
    if (lane == 0) x[r] = s;
}

// r = b, x = p = q = 0, partial ||b||^2 per chunk
__global__ __launch_bounds__(kBlock) void k_pcg_init(const double* b, double* x, double* r, double* p, double* q,
                                                     double* partial, int64_t nn) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= nn) return;
    double s = 0.0;
    for (int a = 0; a < 3; ++a) {
        const double v = b[3 * i + a];
        r[3 * i + a] = v;
        x[3 * i + a] = 0.0;
        p[3 * i + a] = 0.0;
        q[3 * i + a] = 0.0;
        s += v * v;
    }
    chunk_partial(s, partial, i >> 6);
}

// warm start: p = q = 0, partial ||b||^2 per chunk (r = b - K x0 by k_sell<kResid>)
__global__ __launch_bounds__(kBlock) void k_pcg_init_warm(const double* b, double* p, double* q, double* partial,
                                                          int64_t nn) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= nn) return;
    double s = 0.0;
    for (int a = 0; a < 3; ++a) {
        const double v = b[3 * i + a];
        p[3 * i + a] = 0.0;
        q[3 * i + a] = 0.0;
        s += v * v;
    }
    chunk_partial(s, partial, i >> 6);
}

// x += alpha p, r -= alpha q, partial ||r||^2
// x += alpha p, r -= alpha q, partial ||r||^2.  One wavefront per 64-node chunk walks the chunk's
// 192 doubles flat (lane, lane + 64, lane + 128): every load is a contiguous 512-B wave access
// instead of three 24-B-strided ones.
__global__ __launch_bounds__(kBlock) void k_axpy(double* x, double* r, const double* p, const double* q,
                                                 const PcgScal* sc, double* partial, int64_t nn, const int32_t* csub) {
    const int64_t c = (int64_t)blockIdx.x * (kBlock / kWave) + (threadIdx.x >> 6);
    if (c * kChunk >= nn) return;
    const int sub = csub[c];
    if (stopped(sc, sub)) return;
    const double al = sc[sub].alpha;
    const int64_t base = c * 3 * kChunk + (threadIdx.x & 63);
    double s = 0.0;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const int64_t k = base + j * kChunk;
        x[k] += al * p[k];
        const double v = r[k] - al * q[k];
        r[k] = v;
        s += v * v;
    }
    chunk_partial(s, partial, c);
}

// z = D^-1 r (diagonal preconditioner, DIAG_PREC), partial r^T z
__global__ __launch_bounds__(kBlock) void k_diag(const double* r, const double* dinv, double* z, double* partial,
                                                 int64_t nn, const int32_t* csub, const PcgScal* sc) {
    NODE_PROLOGUE(nn, csub, sc)
    double s = 0.0;
    for (int a = 0; a < 3; ++a) {
        const double v = dinv[3 * i + a] * r[3 * i + a];
        z[3 * i + a] = v;
        s += r[3 * i + a] * v;
    }
    chunk_partial(s, partial, i >> 6);
}

// partial x^T y per chunk (used after a coarse-only "V-cycle")
__global__ __launch_bounds__(kBlock) void k_dot(const double* x, const double* y, double* partial, int64_t nn,
                                                const int32_t* csub, const PcgScal* sc) {
    NODE_PROLOGUE(nn, csub, sc)
    double s = 0.0;
    for (int a = 0; a < 3; ++a) s += x[3 * i + a] * y[3 * i + a];
    chunk_partial(s, partial, i >> 6);
}

// Scalar updates of the PCG recurrence: one workgroup per subdomain, fixed summation order
// over that subdomain's chunk partials.  Stop-state changes are mirrored to host memory.
// kFinT = 1024 threads read a subdomain's ~6400 fine chunk partials in ~2 loads each (256: 0.2-0.6 %
// slower overall, profiles/r02u_ab.json)
constexpr int kFinT = 1024;
__global__ __launch_bounds__(kFinT) void k_fin(int what, const double* partial, const double* partial2,
                                               const int64_t* cb, PcgScal* scv, PcgMirror* mirror) {
    const int sub = blockIdx.x;
    PcgScal* sc = scv + sub;
    if (what != kFinInit && what != kFinInitWarm && sc->done) return;
    __shared__ double red[kFinT / kWave], red2[kFinT / kWave];
    // four independent accumulators per thread (loads in flight together), fixed combine order
    double a[4] = {0.0, 0.0, 0.0, 0.0}, b[4] = {0.0, 0.0, 0.0, 0.0};
    const int64_t k0 = cb[sub], k1 = cb[sub + 1];
    for (int64_t k = k0 + threadIdx.x; k < k1; k += 4 * kFinT) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int64_t q = k + (int64_t)u * kFinT;
            if (q < k1) {
                a[u] += partial[q];
                if (what == kFinInitWarm) b[u] += partial2[q];
            }
        }
    }
    double s = wave_sum((a[0] + a[1]) + (a[2] + a[3]));
    double s2 = wave_sum((b[0] + b[1]) + (b[2] + b[3]));
    if ((threadIdx.x & 63) == 0) {
        red[threadIdx.x >> 6] = s;
        red2[threadIdx.x >> 6] = s2;
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    s = 0.0;
    s2 = 0.0;
    for (int w = 0; w < kFinT / kWave; w += 4) {
        s += (red[w] + red[w + 1]) + (red[w + 2] + red[w + 3]);
        s2 += (red2[w] + red2[w + 1]) + (red2[w + 2] + red2[w + 3]);
    }
    const int was_done = sc->done;
    if (what == kFinInit || what == kFinInitWarm) {
        const double bb = what == kFinInit ? s : s2;
        sc->rr = s;
        sc->bb = bb;
        sc->tol2 = sc->tol2 * bb;  // tol2 holds rtol^2 on entry
        sc->iter = 0;
        sc->fail = 0;
        sc->beta = 0.0;
        sc->done = (s <= sc->tol2 || sc->maxit <= 0) ? 1 : 0;
        mirror_store(mirror + sub, 0, sc->done, 0);
        return;
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
        mirror_store(mirror + sub, sc->iter, sc->done, sc->fail);
        return;
    } else {
        if (!isfinite(s)) {
            sc->fail = 1;
            sc->done = 1;
        }
        sc->beta = s / sc->delta;
        sc->delta = s;
    }
    if (sc->done != was_done) mirror_store(mirror + sub, sc->iter, sc->done, sc->fail);
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

// y = M x, partial ||y||^2 per chunk (power iteration for lambda_max(M K) at setup)
template <bool BJ, typename MT = double>
__global__ void k_apply_m(const double* x, const MT* minv, double* y, double* partial, int64_t nn) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= nn) return;
    double m0, m1, m2;
    apply_m<BJ>(minv, i, x[3 * i], x[3 * i + 1], x[3 * i + 2], m0, m1, m2);
    y[3 * i] = m0;
    y[3 * i + 1] = m1;
    y[3 * i + 2] = m2;
    chunk_partial(m0 * m0 + m1 * m1 + m2 * m2, partial, i >> 6);
}

// v = w * scale[subdomain]
__global__ void k_scale_sub(const double* w, const double* scale, double* v, int64_t nn, const int32_t* csub) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= nn) return;
    const double s = scale[csub[i >> 6]];
    for (int a = 0; a < 3; ++a) v[3 * i + a] = w[3 * i + a] * s;
}

// ---- host helpers
__global__ void k_mirror_upper(double* A, int64_t n) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= n * n) return;
    const int64_t i = idx / n, j = idx % n;
    if (j < i) A[i * n + j] = A[j * n + i];
}

// In-place inverse of a dense SPD matrix (row-major = column-major, it is symmetric) with
// rocSOLVER potrf + potri on the device (setup only).
void invert_spd_device(std::vector<double>& A, int64_t n, hipStream_t st) {
    DevBuf<double> d;
    d.upload(A);
    DevBuf<rocblas_int> info(2);
    info.zero(st);
    auto solver_guard = solver_lock();
    rocblas_handle h = nullptr;
    if (rocblas_create_handle(&h) != rocblas_status_success) throw ApiError(DDPCA_EHIP, "rocblas_create_handle");
    rocblas_set_stream(h, st);
    const rocblas_status s1 = rocsolver_dpotrf(h, rocblas_fill_lower, (rocblas_int)n, d.p, (rocblas_int)n, info.p);
    const rocblas_status s2 = rocsolver_dpotri(h, rocblas_fill_lower, (rocblas_int)n, d.p, (rocblas_int)n, info.p + 1);
    hipLaunchKernelGGL(k_mirror_upper, dim3(std::max<int64_t>(1, (n * n + 255) / 256)), dim3(256), 0, st, d.p, n);
    DDPCA_HIP(hipStreamSynchronize(st));
    rocblas_destroy_handle(h);
    const auto inf = info.download();
    if (s1 != rocblas_status_success || s2 != rocblas_status_success) throw ApiError(DDPCA_EHIP, "rocsolver potrf/potri failed");
    if (inf[0] != 0 || inf[1] != 0) throw ApiError(DDPCA_ENUMERIC, "coarse operator is not positive definite");
    DDPCA_HIP(hipMemcpy(A.data(), d.p, A.size() * sizeof(double), hipMemcpyDeviceToHost));
}

// Scale row i of the column-major n x n matrix Vt by 1 / s_i, or 0 when s_i <= tol (pseudo-inverse)
__global__ void k_pinv_rows(double* Vt, const double* S, int64_t n, double tol) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= n * n) return;
    const double sv = S[idx % n];
    Vt[idx] *= sv > tol ? 1.0 / sv : 0.0;
}

__global__ void k_diag(const double* A, int64_t n, double* d) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) d[i] = A[i * n + i];
}

// row sums of |M - I| (M column-major n x n): the residual of an inverse read as M = A^-1 A
__global__ void k_resid_rows(const double* M, int64_t n, double* r) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    double s = 0.0;
    for (int64_t i = 0; i < n; ++i) s += std::abs(M[i * n + j] - (i == j ? 1.0 : 0.0));
    r[j] = s;
}

// In-place inverse of a dense general matrix by rocSOLVER getrf + getri when its LU is clearly
// regular (every |U_ii| above 1e-10 of the largest) and the inverse checks out (||A^-1 A - I||_inf
// <= kLuMaxResid by a rocBLAS gemm against the kept copy of A); returns false, A untouched,
// otherwise, and *resid the residual it measured (INFINITY when the pivot test failed).  The
// column-major view of the row-major buffer is A^T, whose inverse read back row-major is A^-1.
// (LAGRANGE's condensed coarse operators, 4851 rows at BLOCK: ~20 s per Newton step by gesvd.)
constexpr double kLuMaxResid = 1e-6;
bool inv_general_lu_device(std::vector<double>& A, int64_t n, hipStream_t st, double* resid) {
    *resid = INFINITY;
    DevBuf<double> d, a0, diag(std::max<int64_t>(n, 1));
    d.upload(A);
    a0.upload(A);
    DevBuf<rocblas_int> ipiv(std::max<int64_t>(n, 1)), info(2);
    info.zero(st);
    auto solver_guard = solver_lock();
    rocblas_handle h = nullptr;
    if (rocblas_create_handle(&h) != rocblas_status_success) throw ApiError(DDPCA_EHIP, "rocblas_create_handle");
    rocblas_set_stream(h, st);
    const rocblas_status s1 = rocsolver_dgetrf(h, (rocblas_int)n, (rocblas_int)n, d.p, (rocblas_int)n, ipiv.p, info.p);
    hipLaunchKernelGGL(k_diag, dim3(std::max<int64_t>(1, (n + 255) / 256)), dim3(256), 0, st, d.p, n, diag.p);
    DDPCA_HIP(hipStreamSynchronize(st));
    const auto u = diag.download();
    double umax = 0.0, umin = INFINITY;
    for (double x : u) {
        umax = std::max(umax, std::abs(x));
        umin = std::min(umin, std::abs(x));
    }
    if (s1 != rocblas_status_success || info.download()[0] != 0 || !(umin > 1e-10 * umax)) {
        rocblas_destroy_handle(h);
        return false;
    }
    const rocblas_status s2 = rocsolver_dgetri(h, (rocblas_int)n, d.p, (rocblas_int)n, ipiv.p, info.p + 1);
    // column-major: d = (A^T)^-1 and a0 = A^T, so M = d a0 = (A A^-1)^T; ||M - I|| by column sums
    // of M (= row sums of A A^-1 - I)
    DevBuf<double> M(std::max<int64_t>(n * n, 1)), rs(std::max<int64_t>(n, 1));
    const double one = 1.0, zero = 0.0;
    const rocblas_status s3 = rocblas_dgemm(h, rocblas_operation_none, rocblas_operation_none, (rocblas_int)n, (rocblas_int)n,
                                            (rocblas_int)n, &one, d.p, (rocblas_int)n, a0.p, (rocblas_int)n, &zero, M.p,
                                            (rocblas_int)n);
    hipLaunchKernelGGL(k_resid_rows, dim3(std::max<int64_t>(1, (n + 255) / 256)), dim3(256), 0, st, M.p, n, rs.p);
    DDPCA_HIP(hipStreamSynchronize(st));
    rocblas_destroy_handle(h);
    if (s2 != rocblas_status_success || s3 != rocblas_status_success || info.download()[1] != 0) return false;
    double r = 0.0;
    for (double x : rs.download()) r = std::max(r, x);
    *resid = r;
    if (!(r <= kLuMaxResid)) return false;
    DDPCA_HIP(hipMemcpy(A.data(), d.p, A.size() * sizeof(double), hipMemcpyDeviceToHost));
    return true;
}

// In-place pseudo-inverse of a dense general matrix (setup only): rocSOLVER gesvd of the buffer
// read column-major (M = A^T = U S Vt), then C = Vt^T S+ U^T (rocBLAS gemm) = (A^+)^T column-major,
// i.e. A^+ row-major.  Singular values below 1e-11 of the largest are dropped: the coarse operator
// of LAGRANGE's condensed system is singular when a frictionless contact leaves a body free to
// slide (the reference's LDLT meets the same zero pivots); the V-cycle then solves on the range.
void pinv_general_device(std::vector<double>& A, int64_t n, hipStream_t st, int64_t* dropped) {
    DevBuf<double> d, S(std::max<int64_t>(n, 1)), U(std::max<int64_t>(n * n, 1)), Vt(std::max<int64_t>(n * n, 1)),
        E(std::max<int64_t>(n, 1)), C(std::max<int64_t>(n * n, 1));
    d.upload(A);
    DevBuf<rocblas_int> info(1);
    info.zero(st);
    auto solver_guard = solver_lock();
    rocblas_handle h = nullptr;
    if (rocblas_create_handle(&h) != rocblas_status_success) throw ApiError(DDPCA_EHIP, "rocblas_create_handle");
    rocblas_set_stream(h, st);
    const rocblas_status s1 = rocsolver_dgesvd(h, rocblas_svect_all, rocblas_svect_all, (rocblas_int)n, (rocblas_int)n, d.p,
                                               (rocblas_int)n, S.p, U.p, (rocblas_int)n, Vt.p, (rocblas_int)n, E.p,
                                               rocblas_outofplace, info.p);
    std::vector<double> sv(n);
    DDPCA_HIP(hipMemcpyAsync(sv.data(), S.p, n * sizeof(double), hipMemcpyDeviceToHost, st));
    DDPCA_HIP(hipStreamSynchronize(st));
    const auto inf = info.download();
    if (s1 != rocblas_status_success || inf[0] != 0) {
        rocblas_destroy_handle(h);
        throw ApiError(DDPCA_EHIP, "rocsolver gesvd failed on the coarse operator");
    }
    const double tol = 1e-11 * (n ? sv[0] : 0.0);
    *dropped = 0;
    for (double x : sv) *dropped += !(x > tol);
    hipLaunchKernelGGL(k_pinv_rows, dim3(std::max<int64_t>(1, (n * n + 255) / 256)), dim3(256), 0, st, Vt.p, S.p, n, tol);
    const double one = 1.0, zero = 0.0;
    const rocblas_status s2 = rocblas_dgemm(h, rocblas_operation_transpose, rocblas_operation_transpose, (rocblas_int)n,
                                            (rocblas_int)n, (rocblas_int)n, &one, Vt.p, (rocblas_int)n, U.p, (rocblas_int)n,
                                            &zero, C.p, (rocblas_int)n);
    DDPCA_HIP(hipStreamSynchronize(st));
    rocblas_destroy_handle(h);
    if (s2 != rocblas_status_success) throw ApiError(DDPCA_EHIP, "rocblas gemm failed");
    DDPCA_HIP(hipMemcpy(A.data(), C.p, A.size() * sizeof(double), hipMemcpyDeviceToHost));
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

constexpr int64_t kMaxRowBlocks = 128;  // longest node-block row the table mode types (longer: streamed)

// Quantised (z, y, x) keys of a level's nodes: coordinates quantised to 1e-9 of the bounding
// box, so nodes of one mesh plane share a key despite rounding in their coordinates.
using Key3 = std::array<int64_t, 3>;
std::vector<Key3> quantised_keys(const double* xyz, int64_t n) {
    double lo[3] = {0, 0, 0}, hi[3] = {0, 0, 0};
    for (int64_t i = 0; i < n; ++i)
        for (int a = 0; a < 3; ++a) {
            lo[a] = i ? std::min(lo[a], xyz[3 * i + a]) : xyz[3 * i + a];
            hi[a] = i ? std::max(hi[a], xyz[3 * i + a]) : xyz[3 * i + a];
        }
    const double ext = std::max({hi[0] - lo[0], hi[1] - lo[1], hi[2] - lo[2]});
    const double q = ext > 0.0 ? 1e-9 * ext : 1.0;
    std::vector<Key3> key(n);
    for (int64_t i = 0; i < n; ++i)
        key[i] = {std::llround((xyz[3 * i + 2] - lo[2]) / q), std::llround((xyz[3 * i + 1] - lo[1]) / q),
                  std::llround((xyz[3 * i] - lo[0]) / q)};
    return key;
}

// Device node order of one level, p[reference node] = device node: lexicographic in (z, y, x);
// with row types, grouped by type first (lexicographic inside a type), so 64-row chunks are
// type-homogeneous wherever a type has enough rows.
std::vector<int32_t> device_order(const std::vector<Key3>& key, const std::vector<int32_t>* type) {
    const int64_t n = (int64_t)key.size();
    std::vector<int32_t> idx(n), p(n);
    std::iota(idx.begin(), idx.end(), 0);
    std::stable_sort(idx.begin(), idx.end(), [&](int32_t a, int32_t b) {
        if (type && (*type)[a] != (*type)[b]) return (*type)[a] < (*type)[b];
        return key[a] < key[b];
    });
    for (int64_t k = 0; k < n; ++k) p[idx[k]] = (int32_t)k;
    return p;
}

// Canonical slot order of row r: its blocks sorted by the neighbour's quantised offset from the
// row node -- independent of any numbering, so equal rows stay equal after renumbering.
void canonical_slots(const Bsr3& A, int64_t r, const std::vector<Key3>& key, int64_t* ord) {
    const int64_t len = A.ptr[r + 1] - A.ptr[r];
    for (int64_t t = 0; t < len; ++t) ord[t] = A.ptr[r] + t;
    const Key3& kr = key[r];
    std::sort(ord, ord + len, [&](int64_t u, int64_t v) {
        const Key3& a = key[A.col[u]];
        const Key3& b = key[A.col[v]];
        for (int d = 0; d < 3; ++d)
            if (a[d] - kr[d] != b[d] - kr[d]) return a[d] - kr[d] < b[d] - kr[d];
        return false;
    });
}

// Bit-exact row types of one level of one subdomain: masked block values in canonical slot order.
std::vector<int32_t> row_types(const Bsr3& A, const uint8_t* fr, const std::vector<Key3>& key, int64_t& ntypes) {
    const int64_t n = A.nb;
    std::vector<int32_t> t(n);
    std::unordered_map<uint64_t, std::vector<int32_t>> bucket;
    std::vector<std::vector<double>> reps;
    std::vector<double> v;
    int64_t ord[128];
    for (int64_t r = 0; r < n; ++r) {
        const int64_t len = A.ptr[r + 1] - A.ptr[r];
        canonical_slots(A, r, key, ord);
        v.assign(9 * len, 0.0);
        for (int64_t s = 0; s < len; ++s) {
            const int64_t k = ord[s], j = A.col[k];
            for (int a = 0; a < 3; ++a)
                for (int b = 0; b < 3; ++b) {
                    double x = A.val[9 * k + 3 * a + b];
                    if (!fr[3 * r + a] || !fr[3 * j + b]) x = (j == r && a == b) ? 1.0 : 0.0;
                    v[9 * s + 3 * a + b] = x;
                }
        }
        uint64_t h = 1469598103934665603ull ^ (uint64_t)len;
        for (double x : v) {
            uint64_t b;
            std::memcpy(&b, &x, 8);
            h = (h ^ b) * 1099511628211ull;
            h ^= h >> 29;
        }
        auto& cand = bucket[h];
        int32_t id = -1;
        for (int32_t c : cand)
            if (reps[c].size() == v.size() && std::memcmp(reps[c].data(), v.data(), v.size() * sizeof(double)) == 0) {
                id = c;
                break;
            }
        if (id < 0) {
            id = (int32_t)reps.size();
            cand.push_back(id);
            reps.push_back(v);
        }
        t[r] = id;
    }
    ntypes = (int64_t)reps.size();
    return t;
}

// Table mode of one level: every row's values (device slot order, masks applied, zero beyond the
// row) are deduplicated bit-exactly, per subdomain in parallel, then merged into one table.  Used
// when the table is at most a fifth of the streamed values (or when forced, for tests).
void build_table(LevelDev& L, const std::vector<int32_t>& slots, const std::vector<int64_t>& off,
                 const std::vector<double>& val, bool force) {
    int64_t tmax = 0;
    for (int32_t s : slots) tmax = std::max<int64_t>(tmax, s);
    const int64_t ts9 = std::max<int64_t>(tmax * 9, 1);
    const int nsub = (int)L.noff.size();
    std::vector<std::vector<double>> subtab(nsub);
    std::vector<int32_t> rt(L.nn, 0);
#pragma omp parallel for schedule(dynamic, 1)
    for (int s = 0; s < nsub; ++s) {
        std::unordered_map<uint64_t, std::vector<int32_t>> bucket;
        std::vector<double>& T = subtab[s];
        std::vector<double> rowv(ts9);
        int32_t nt = 0;
        for (int64_t g = L.noff[s]; g < L.noff[s] + pad64(L.nloc[s]); ++g) {
            const int64_t c = g / kChunk, lane = g % kChunk;
            std::fill(rowv.begin(), rowv.end(), 0.0);
            for (int64_t t = 0; t < slots[c]; ++t)
                for (int ij = 0; ij < 9; ++ij) rowv[t * 9 + ij] = val[((off[c] + t) * 9 + ij) * kChunk + lane];
            uint64_t h = 1469598103934665603ull;
            for (double v : rowv) {
                uint64_t b;
                std::memcpy(&b, &v, 8);
                h = (h ^ b) * 1099511628211ull;
                h ^= h >> 29;
            }
            int32_t id = -1;
            auto& cand = bucket[h];
            for (int32_t t : cand)
                if (std::memcmp(&T[(size_t)t * ts9], rowv.data(), ts9 * sizeof(double)) == 0) {
                    id = t;
                    break;
                }
            if (id < 0) {
                id = nt++;
                cand.push_back(id);
                T.insert(T.end(), rowv.begin(), rowv.end());
            }
            rt[g] = id;
        }
    }
    int64_t ntypes = 0;
    std::vector<int64_t> base(nsub);
    for (int s = 0; s < nsub; ++s) {
        base[s] = ntypes;
        ntypes += (int64_t)subtab[s].size() / ts9;
    }
    const double tab_bytes = (double)ntypes * ts9 * 8.0, val_bytes = (double)val.size() * 8.0;
    if (!force && tab_bytes > 0.2 * val_bytes) return;
    std::vector<double> tab;
    tab.reserve((size_t)ntypes * ts9);
    for (int s = 0; s < nsub; ++s) {
        tab.insert(tab.end(), subtab[s].begin(), subtab[s].end());
        for (int64_t g = L.noff[s]; g < L.noff[s] + pad64(L.nloc[s]); ++g) rt[g] += (int32_t)base[s];
    }
    // chunks whose 64 rows share one type read their table row through scalar loads
    std::vector<int32_t> ct(L.nch);
    int64_t uniform = 0;
    for (int64_t c = 0; c < L.nch; ++c) {
        ct[c] = rt[c * kChunk];
        for (int64_t lane = 1; lane < kChunk && ct[c] >= 0; ++lane)
            if (rt[c * kChunk + lane] != ct[c]) ct[c] = -1;
        uniform += ct[c] >= 0;
    }
    L.tbl = true;
    L.tstride = ts9;
    L.ntypes = ntypes;
    L.nuniform = uniform;
    L.rtype.upload(rt);
    L.ctype.upload(ct);
    L.tab.upload(tab);
}

std::vector<int32_t> identity_order(int64_t n) {
    std::vector<int32_t> p(n);
    std::iota(p.begin(), p.end(), 0);
    return p;
}

// Chebyshev coefficients of sweep k on [lmax/30, lmax] of M K (k = 0: the 1/theta start)
void cheb_coef(double lmax, int k, double& c1, double& c2) {
    const double lmin = lmax / 30.0;
    const double theta = 0.5 * (lmax + lmin), delta = 0.5 * (lmax - lmin), sigma = theta / delta;
    if (k == 0) {
        c1 = 0.0;
        c2 = 1.0 / theta;
        return;
    }
    double rho_old = 1.0 / sigma, rho = rho_old;
    for (int i = 1; i <= k; ++i) {
        rho = 1.0 / (2.0 * sigma - rho_old);
        if (i < k) rho_old = rho;
    }
    c1 = rho * rho_old;
    c2 = 2.0 * rho / delta;
}

}  // namespace

// ============================================================================== host plumbing
void select_device(int device) {
    static thread_local int checked = -1;  // last device verified to be a gfx950 part
    if (device == checked) {
        DDPCA_HIP(hipSetDevice(device));
        return;
    }
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) throw ApiError(DDPCA_ENOGPU, "no HIP device visible");
    if (device < 0 || device >= n) throw ApiError(DDPCA_EINVAL, "device index out of range");
    DDPCA_HIP(hipSetDevice(device));
    hipDeviceProp_t prop;
    DDPCA_HIP(hipGetDeviceProperties(&prop, device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        throw ApiError(DDPCA_ENOGPU, std::string("device is ") + prop.gcnArchName + ", kernels are built for gfx950");
    checked = device;
}

void MirrorBuf::alloc(int count) {
    n = count;
    DDPCA_HIP(hipHostMalloc(reinterpret_cast<void**>(&host), std::max(1, count) * sizeof(PcgMirror),
                            hipHostMallocMapped | hipHostMallocCoherent));
    DDPCA_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&dev), host, 0));
    reset();
}

void MirrorBuf::reset() { std::memset(host, 0, std::max(1, n) * sizeof(PcgMirror)); }

MirrorBuf::~MirrorBuf() {
    if (host) (void)hipHostFree(host);
}

int64_t pace_until_done(hipStream_t stream, hipGraphExec_t graph, const MirrorBuf& m, int64_t k, int64_t launched,
                        hipGraphExec_t graph1, int64_t horizon) {
    constexpr int64_t kRunway = 2;  // tail: single iterations kept this far ahead of the slowest member
    int64_t replays = 0;
    for (int64_t spin = 0;; ++spin) {
        bool all = true;
        int64_t slowest = INT64_MAX;
        for (int s = 0; s < m.n; ++s) {
            if (__atomic_load_n(&m.host[s].done, __ATOMIC_ACQUIRE)) continue;
            all = false;
            slowest = std::min<int64_t>(slowest, __atomic_load_n(&m.host[s].iter, __ATOMIC_RELAXED));
        }
        if (all) return replays;
        // keep one replay of runway: launch when the slowest solve has entered the last one;
        // past the expected iteration count, single iterations kRunway ahead
        const bool tail = graph1 && launched + k > horizon;
        if (tail ? launched - slowest <= kRunway : launched - slowest <= k) {
            DDPCA_HIP(hipGraphLaunch(tail ? graph1 : graph, stream));
            launched += tail ? 1 : k;
            ++replays;
            continue;
        }
        if ((spin & 255) == 255) {
            const hipError_t q = hipStreamQuery(stream);
            if (q == hipSuccess) {
                // stream drained: the mirror is final for everything enqueued so far
                bool done_now = true;
                for (int s = 0; s < m.n; ++s) done_now &= __atomic_load_n(&m.host[s].done, __ATOMIC_ACQUIRE) != 0;
                if (done_now) return replays;
                DDPCA_HIP(hipGraphLaunch(tail ? graph1 : graph, stream));
                launched += tail ? 1 : k;
                ++replays;
            } else if (q != hipErrorNotReady) {
                DDPCA_HIP(q);
            }
        }
        std::this_thread::yield();
    }
}

// ============================================================================== setup
namespace {
using KidList = std::vector<std::vector<std::pair<int32_t, double>>>;

// Lattice form of a uniformly averaging transfer l-1 -> l (LevelDev::lat): accepted only when it
// reproduces the explicit lists exactly, per subdomain: every fine node's parent set is p0 plus
// the subset sums of three coarse strides (the differences of the two-parent nodes), every coarse
// node's child set is its fine copy plus d . t for d in {-1,0,1}^3 (t from the half-weight
// children) with weight 2^-|d|, the 27 offsets distinct.  Box lattices numbered lexicographically
// (the device renumbering of levels >= 1) pass; anything else keeps the explicit lists.
bool lattice_reject(int why) {
    if (std::getenv("DDPCA_VERBOSE")) std::fprintf(stderr, "[ddpca] lattice transfer rejected (check %d)\n", why);
    return false;
}

bool lattice_transfer(LevelDev& L, const LevelDev& C, const std::vector<int32_t>& ppar, const KidList& kids) {
    const size_t ns = L.noff.size();
    std::vector<uint32_t> ppk(L.nn, 0u), rmsk(C.nn, 0u);
    std::vector<int32_t> pstr(3 * ns, 0), rstr(3 * ns, 0), rf0(C.nn, 0);
    if (C.nn >= (int64_t)1 << 29 || L.nn >= (int64_t)1 << 31) return lattice_reject(0);
    auto three = [](std::vector<int64_t>& d, int32_t* out, int64_t fill) {
        std::sort(d.begin(), d.end());
        d.erase(std::unique(d.begin(), d.end()), d.end());
        if (d.size() > 3 || (!d.empty() && d[0] <= 0)) return lattice_reject(1);
        for (int k = 0; k < 3; ++k) out[k] = (int32_t)(k < (int)d.size() ? d[k] : fill + k);
        return true;
    };
    for (size_t s = 0; s < ns; ++s) {
        // prolongation
        std::vector<int64_t> d;
        int32_t P[8];
        auto parents = [&](int64_t gf) {
            int np = 0;
            while (np < 8 && ppar[np * L.nn + gf] >= 0) {
                P[np] = ppar[np * L.nn + gf];
                ++np;
            }
            std::sort(P, P + np);
            return np;
        };
        const int64_t f_lo = L.noff[s], f_hi = f_lo + L.nloc[s];
        for (int64_t gf = f_lo; gf < f_hi; ++gf)
            if (parents(gf) == 2) d.push_back((int64_t)P[1] - P[0]);
        int32_t* st = &pstr[3 * s];
        if (!three(d, st, (int64_t)1 << 28)) return lattice_reject(2);
        for (int64_t gf = f_lo; gf < f_hi; ++gf) {
            const int np = parents(gf);
            if (np != 1 && np != 2 && np != 4 && np != 8) return lattice_reject(3);
            bool found = false;
            for (uint32_t code = 0; code < 8 && !found; ++code) {
                if ((1 << __builtin_popcount(code)) != np) continue;
                int64_t set[8];
                int m = 0;
                for (uint32_t q = 0; q < 8; ++q)
                    if ((q & ~code) == 0)
                        set[m++] = P[0] + ((q & 1) ? st[0] : 0) + ((q & 2) ? st[1] : 0) + ((q & 4) ? (int64_t)st[2] : 0);
                std::sort(set, set + m);
                bool eq = true;
                for (int k = 0; k < m; ++k) eq &= set[k] == P[k];
                if (eq) {
                    ppk[gf] = (uint32_t)P[0] | (code << 29);
                    found = true;
                }
            }
            if (!found) return lattice_reject(4);
        }
        // restriction
        const int64_t c_lo = C.noff[s], c_hi = c_lo + C.nloc[s];
        d.clear();
        for (int64_t j = c_lo; j < c_hi; ++j) {
            if (kids[j].empty() || kids[j][0].second != 1.0) return lattice_reject(5);
            for (const auto& k : kids[j])
                if (k.second == 0.5) d.push_back(std::abs((int64_t)k.first - kids[j][0].first));
        }
        int32_t* t = &rstr[3 * s];
        if (!three(d, t, (int64_t)1 << 29)) return lattice_reject(6);
        std::vector<std::pair<int64_t, int>> offs;  // offset -> bit
        for (int q = 0; q < 27; ++q)
            offs.push_back({(int64_t)(q % 3 - 1) * t[0] + (int64_t)((q / 3) % 3 - 1) * t[1] + (int64_t)(q / 9 - 1) * t[2], q});
        std::sort(offs.begin(), offs.end());
        for (int q = 1; q < 27; ++q)
            if (offs[q].first == offs[q - 1].first) return lattice_reject(7);
        for (int64_t j = c_lo; j < c_hi; ++j) {
            const int64_t f0 = kids[j][0].first;
            uint32_t msk = 0;
            for (const auto& k : kids[j]) {
                const int64_t o = (int64_t)k.first - f0;
                auto it = std::lower_bound(offs.begin(), offs.end(), std::make_pair(o, -1));
                if (it == offs.end() || it->first != o) return lattice_reject(8);
                const int q = it->second;
                const int nz = (q % 3 != 1) + ((q / 3) % 3 != 1) + (q / 9 != 1);
                if (k.second != 1.0 / (double)(1 << nz) || ((msk >> q) & 1u)) return lattice_reject(9);
                msk |= 1u << q;
            }
            rmsk[j] = msk;
            rf0[j] = (int32_t)f0;
        }
    }
    L.lat = true;
    L.uw = true;
    L.ppk.upload(ppk);
    L.pstr.upload(pstr);
    L.rmsk.upload(rmsk);
    L.rf0.upload(rf0);
    L.rstr.upload(rstr);
    return true;
}

// The fine level's colour structure (GsFine) from its host SELL arrays (col: batch device
// columns, val: masked fp64 blocks val[(q * 9 + ij) * 64 + lane]); vt: the V-cycle copy's type.
// A colour's rows go to chunks in device order, i.e. along the x lines of a box (16 x 16-node
// tiles of one plane measured 1.8 % slower at the headline, profiles/r03i).
// band (optional, per device node of the level): colour and sweep only the flagged rows; the others
// go to the ring group (a flagged neighbour) or the far group (none) -- GsFine::band
void build_gs(GsFine& G, const LevelDev& L, int nsub, const std::vector<int64_t>& off, const std::vector<int32_t>& col,
              const std::vector<double>& val, int vt, const std::vector<uint8_t>* band = nullptr) {
    // greedy colouring in device order, per member
    std::vector<int8_t> colour(L.nn, -1);
    std::vector<int> ncol_sub(nsub, 0);
    int too_many = 0;
#pragma omp parallel for schedule(dynamic, 1) reduction(max : too_many)
    for (int s = 0; s < nsub; ++s) {
        for (int64_t g = L.noff[s]; g < L.noff[s] + L.nloc[s]; ++g) {
            if (band && !(*band)[g]) continue;
            const int64_t c = g / kChunk, lane = g % kChunk;
            uint64_t used = 0;
            for (int64_t q = off[c]; q < off[c + 1]; ++q) {
                const int64_t j = col[q * kChunk + lane];
                if (j != g && colour[j] >= 0) used |= 1ull << colour[j];
            }
            if (used == ~0ull) {
                too_many = 1;
                break;
            }
            const int k = __builtin_ctzll(~used);
            colour[g] = (int8_t)k;
            ncol_sub[s] = std::max(ncol_sub[s], k + 1);
        }
    }
    if (too_many) throw ApiError(DDPCA_EINVAL, "multicolour smoother: a node graph needing more than 64 colours");
    const int K = *std::max_element(ncol_sub.begin(), ncol_sub.end());
    // chunk groups per member: the colours, then (band mode) the ring and the far rows
    const int KG = band ? K + 2 : K;
    auto is_band = [&](int64_t j) { return colour[j] >= 0; };
    // colour chunks, member-major and colour-minor
    std::vector<std::vector<int64_t>> rows((size_t)nsub * KG);
    for (int s = 0; s < nsub; ++s)
        for (int64_t g = L.noff[s]; g < L.noff[s] + L.nloc[s]; ++g) {
            int grp = colour[g];
            if (grp < 0) {
                grp = K + 1;  // far unless a neighbour is in the band
                const int64_t nc = g / kChunk, lane = g % kChunk;
                for (int64_t q = off[nc]; q < off[nc + 1] && grp == K + 1; ++q) {
                    const int64_t j = col[q * kChunk + lane];
                    if (j != g && is_band(j)) grp = K;
                }
            }
            rows[(size_t)s * KG + grp].push_back(g);
        }
    // which neighbours a row of group k stores: colours L = earlier colours and every non-band
    // column (x = 0 there in the forward sweep), U = the rest; ring rows: their band columns as L
    auto store = [&](int k, int64_t j) -> int {  // 0 L, 1 U, -1 not stored
        if (k < K) return colour[j] < k ? 0 : 1;
        if (k == K) return is_band(j) ? 0 : -1;
        return -1;
    };
    std::vector<int32_t> rowidx, csub, nsl, nsu;
    std::vector<int64_t> offl, offu, cb(nsub + 1, 0);
    std::vector<std::vector<int32_t>> bycol(KG);
    std::vector<int64_t> base;  // first row of each chunk in its (s, k) list
    std::vector<size_t> lists;
    G.nnzb_sub.assign(nsub, 0);
    G.slots_sub.assign(nsub, 0);
    G.band = band != nullptr;
    G.band_rows_sub.assign(nsub, 0);
    G.ring_rows_sub.assign(nsub, 0);
    G.far_rows_sub.assign(nsub, 0);
    G.ring_nnzb_sub.assign(nsub, 0);
    for (int s = 0; s < nsub; ++s) {
        cb[s] = (int64_t)csub.size();
        for (int k = 0; k < KG; ++k) {
            const auto& R = rows[(size_t)s * KG + k];
            (k < K ? G.band_rows_sub : k == K ? G.ring_rows_sub : G.far_rows_sub)[s] += (int64_t)R.size();
            for (size_t r0 = 0; r0 < R.size(); r0 += kChunk) {
                const int64_t c = (int64_t)csub.size();
                bycol[k].push_back((int32_t)c);
                csub.push_back(s);
                base.push_back((int64_t)r0);
                lists.push_back((size_t)s * KG + k);
                int32_t ml = 0, mu = 0;
                for (size_t i = r0; i < std::min(R.size(), r0 + kChunk); ++i) {
                    const int64_t g = R[i], nc = g / kChunk, lane = g % kChunk;
                    int32_t nl = 0, nu = 0;
                    for (int64_t q = off[nc]; q < off[nc + 1]; ++q) {
                        const int64_t j = col[q * kChunk + lane];
                        if (j == g) continue;
                        const int t = store(k, j);
                        if (t == 0) ++nl;
                        else if (t == 1) ++nu;
                    }
                    ml = std::max(ml, nl);
                    mu = std::max(mu, nu);
                    (k < K ? G.nnzb_sub : G.ring_nnzb_sub)[s] += nl + nu;
                }
                nsl.push_back(ml);
                nsu.push_back(mu);
            }
        }
    }
    const int64_t nch = (int64_t)csub.size();
    cb[nsub] = nch;
    // slots per chunk: the longest row's L and U counts
    int64_t nslot = 0;
    for (int64_t c = 0; c < nch; ++c) {
        offl.push_back(nslot);
        offu.push_back(nslot + nsl[c]);
        nslot += nsl[c] + nsu[c];
        G.slots_sub[csub[c]] += nsl[c] + nsu[c];
    }
    rowidx.assign(nch * kChunk, 0);
    const bool c16 = L.col16.p != nullptr;
    std::vector<int32_t> gcol(c16 ? 0 : std::max<int64_t>(nslot * kChunk, 1), 0);
    std::vector<int16_t> gcol16(c16 ? std::max<int64_t>(nslot * kChunk, 1) : 0, 0);
    const int nv = vt == kValQ8 ? 12 : vt == kValH16 ? 10 : 9;
    std::vector<uint16_t> v16(vt == kValH16 ? std::max<int64_t>(nslot * nv * kChunk, 1) : 0, 0);
    std::vector<uint8_t> v8(vt == kValQ8 ? std::max<int64_t>(nslot * nv * kChunk, 1) : 0, 0);
    std::atomic<bool> q8_ok{true};  // written from the omp loop below
    std::vector<float> v32(vt == kVal32 ? std::max<int64_t>(nslot * nv * kChunk, 1) : 0, 0.0f);
    std::vector<double> v64(vt == kVal64 ? std::max<int64_t>(nslot * nv * kChunk, 1) : 0, 0.0);
#pragma omp parallel for schedule(dynamic, 64)
    for (int64_t c = 0; c < nch; ++c) {
        const auto& R = rows[lists[c]];
        const int k = (int)(lists[c] % KG);
        const int64_t r0 = base[c], nr = std::min<int64_t>(kChunk, (int64_t)R.size() - r0);
        for (int64_t lane = 0; lane < kChunk; ++lane) {
            const bool real = lane < nr;
            const int64_t g = real ? R[r0 + lane] : R[r0];
            rowidx[c * kChunk + lane] = real ? (int32_t)g : ~(int32_t)g;
            // pad slots: the row itself (offset 0), zero blocks
            for (int64_t q = offl[c]; q < offl[c] + nsl[c] + nsu[c]; ++q) {
                if (c16) gcol16[q * kChunk + lane] = 0;
                else gcol[q * kChunk + lane] = (int32_t)g;
            }
            if (!real) continue;
            const int64_t nc = g / kChunk, nl = g % kChunk;
            int64_t ql = offl[c], qu = offu[c];
            for (int64_t q = off[nc]; q < off[nc + 1]; ++q) {
                const int64_t j = col[q * kChunk + nl];
                if (j == g) continue;
                const int st = store(k, j);
                if (st < 0) continue;
                const int64_t t = st == 0 ? ql++ : qu++;
                if (c16) gcol16[t * kChunk + lane] = (int16_t)(j - g);
                else gcol[t * kChunk + lane] = (int32_t)j;
                double blk[9];
                for (int ij = 0; ij < 9; ++ij) blk[ij] = val[(q * 9 + ij) * kChunk + nl];
                if (vt == kValH16) {
                    uint16_t rec[10];
                    to_h16_block(blk, rec);
                    for (int e = 0; e < 10; ++e) v16[t * 10 * kChunk + 128 * (e / 2) + 2 * lane + e % 2] = rec[e];
                } else if (vt == kValQ8) {
                    uint8_t rec[12];
                    if (!to_q8_block(blk, rec)) q8_ok.store(false, std::memory_order_relaxed);
                    for (int e = 0; e < 12; ++e) v8[t * 12 * kChunk + q8_pos(e, lane)] = rec[e];
                } else if (vt == kVal32) {
                    for (int ij = 0; ij < 9; ++ij) v32[t * 9 * kChunk + slot_elem<float>(ij, lane)] = (float)blk[ij];
                } else {
                    for (int ij = 0; ij < 9; ++ij) v64[t * 9 * kChunk + slot_elem<double>(ij, lane)] = blk[ij];
                }
            }
        }
    }
    // per-launch byte model: a block's stored value record + its column entry, per real row b, the
    // fp32 inverse, x or r written and the row index, and every distinct x entry the launch
    // gathers (forward colour k: rows of earlier colours; residual: later ones; backward: all
    // other colours) once
    {
        if (!q8_ok) throw ApiError(DDPCA_EINVAL, "block-scaled int8 copy: a block's scale is out of fp32's normal range");
        const double vb = vbytes(vt) + (c16 ? 2.0 : 4.0);
        const double rowf = 24.0 + (vt == kVal64 ? 72.0 : 36.0) + 24.0 + 4.0;
        std::vector<double> nl_k(K, 0.0), nu_k(K, 0.0), rows_k(K, 0.0), gx_f(K, 0.0), gx_b(K, 0.0);
        double gx_r = 0.0;
        std::vector<int32_t> seen_f(L.nn, -1), seen_b(L.nn, -1), seen_r(L.nn, 0), seen_u(L.nn, -1), seen_l(L.nn, 0);
        std::vector<double> gx_u(K, 0.0);
        double gx_l = 0.0;
        for (int k = 0; k < K; ++k)
            for (int s = 0; s < nsub; ++s)
                for (int64_t g : rows[(size_t)s * KG + k]) {
                    rows_k[k] += 1.0;
                    const int64_t nc = g / kChunk, lane = g % kChunk;
                    for (int64_t q = off[nc]; q < off[nc + 1]; ++q) {
                        const int64_t j = col[q * kChunk + lane];
                        if (j == g) continue;
                        if (colour[j] < k) {
                            nl_k[k] += 1.0;
                            if (seen_f[j] != k) seen_f[j] = k, gx_f[k] += 1.0;
                            if (!seen_l[j]) seen_l[j] = 1, gx_l += 1.0;
                        } else {
                            nu_k[k] += 1.0;
                            if (!seen_r[j]) seen_r[j] = 1, gx_r += 1.0;
                            if (seen_u[j] != k) seen_u[j] = k, gx_u[k] += 1.0;
                        }
                        if (seen_b[j] != k) seen_b[j] = k, gx_b[k] += 1.0;
                    }
                }
        G.launch_bytes.clear();
        double res = 0.0;
        for (int k = 0; k < K; ++k) {
            G.launch_bytes.push_back(vb * nl_k[k] + rowf * rows_k[k] + 24.0 * gx_f[k]);
            res += vb * nu_k[k] + 28.0 * rows_k[k];
        }
        G.launch_bytes.push_back(res + 24.0 * gx_r);
        for (int k = K - 1; k >= 0; --k) G.launch_bytes.push_back(vb * (nl_k[k] + nu_k[k]) + rowf * rows_k[k] + 24.0 * gx_b[k]);
        G.gx_f = gx_f;
        G.gx_b = gx_b;
        G.rows_k = rows_k;
        G.gx_r = gx_r;
        G.gx_u = gx_u;
        G.gx_l = gx_l;
        G.nl_k = nl_k;
        G.nu_k = nu_k;
        G.vb = vb;
    }
    G.ncol = K;
    G.nchunk = nch;
    G.first.assign(KG, 0);
    G.count.assign(KG, 0);
    std::vector<int32_t> list;
    for (int k = 0; k < KG; ++k) {
        G.first[k] = (int64_t)list.size();
        G.count[k] = (int64_t)bycol[k].size();
        list.insert(list.end(), bycol[k].begin(), bycol[k].end());
    }
    if (vt != kVal64 && L.minv32.p) {
        const std::vector<float> m32 = L.minv32.download();
        std::vector<float> mc((size_t)nch * 9 * kChunk, 0.0f);
#pragma omp parallel for schedule(static)
        for (int64_t c = 0; c < nch; ++c)
            for (int64_t lane = 0; lane < kChunk; ++lane) {
                const int32_t rr = rowidx[c * kChunk + lane];
                const int64_t g = rr >= 0 ? rr : ~rr;  // pad lanes: the chunk's first row (their x is not stored)
                for (int ij = 0; ij < 9; ++ij) mc[(c * 9 + ij) * kChunk + lane] = m32[9 * g + ij];
            }
        G.minvc.upload(mc);
    }
    G.list.upload(list);
    G.rowidx.upload(rowidx);
    G.csub.upload(csub);
    G.nsl.upload(nsl);
    G.nsu.upload(nsu);
    G.offl.upload(offl);
    G.offu.upload(offu);
    G.cb.upload(cb);
    if (c16) G.col16.upload(gcol16);
    else G.col.upload(gcol);
    if (vt == kValH16) G.val16.upload(v16);
    else if (vt == kValQ8) G.val8.upload(v8);
    else if (vt == kVal32) G.val32.upload(v32);
    else G.val64.upload(v64);
    if (std::getenv("DDPCA_VERBOSE")) {
        int64_t nb = 0, nr = 0, nf = 0;
        for (int s = 0; s < nsub; ++s) nb += G.band_rows_sub[s], nr += G.ring_rows_sub[s], nf += G.far_rows_sub[s];
        std::fprintf(stderr, "[ddpca] fine level: multicolour Gauss-Seidel, %d colours, %lld chunks, %lld slots%s\n", K,
                     (long long)nch, (long long)nslot,
                     band ? (", band " + std::to_string(nb) + " / ring " + std::to_string(nr) + " / far " + std::to_string(nf) + " rows").c_str() : "");
    }
}
}  // namespace

MgpisDevice::MgpisDevice(int dev, const std::vector<SubdomainOps>& subs, const mgpis_options_t& o, bool gen,
                         bool diag_only)
    : general(gen), device(dev), opt(o) {
    select_device(device);
    nsub = (int)subs.size();
    if (nsub < 1) throw ApiError(DDPCA_EINVAL, "empty subdomain batch");
    const int nlev = (int)subs[0].nnodes.size();
    for (const auto& S : subs) {
        if ((int)S.nnodes.size() != nlev || nlev < 1 || (int)S.K.size() != nlev || (int)S.S.size() != nlev - 1)
            throw ApiError(DDPCA_EINVAL, "level counts differ within the batch");
        if (!S.dof_free) throw ApiError(DDPCA_EINVAL, "dof_free missing");
        for (int l = 0; l < nlev; ++l)
            if (S.K[l]->nb != S.nnodes[l] || S.K[l]->mb != S.nnodes[l]) throw ApiError(DDPCA_EINVAL, "operator size does not match nnodes");
    }
    DDPCA_HIP(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    if (opt.nu < 1) opt.nu = 1;
    if (opt.iters_per_graph < 1) opt.iters_per_graph = 1;
    if (opt.smoother < 0 || opt.smoother > 4) throw ApiError(DDPCA_EINVAL, "smoother must be 0..4");
    // the multicolour sweeps' symmetric pairing needs K = K^T: nonsymmetric handles smooth with block Jacobi
    if (opt.smoother >= 3 && general) opt.smoother = 1;
    const bool bj = opt.smoother >= 1;
    // device numbering: perm[l][s][reference local node] = device local node.  Levels >= 1 with
    // coordinates: lexicographic, or -- table mode, when the level's distinct rows compress --
    // grouped by row type so chunks are type-homogeneous; their slots go in canonical order.
    std::vector<std::vector<std::vector<int32_t>>> perm(nlev, std::vector<std::vector<int32_t>>(nsub));
    std::vector<std::vector<std::vector<Key3>>> keys(nlev, std::vector<std::vector<Key3>>(nsub));
    std::vector<char> grouped(nlev, 0);
    for (int l = 0; l < nlev; ++l) {
        bool geo = l > 0;
        for (int s = 0; s < nsub; ++s) geo = geo && subs[s].coords != nullptr;
        if (!geo) {
            for (int s = 0; s < nsub; ++s) perm[l][s] = identity_order(subs[s].nnodes[l]);
            continue;
        }
        std::vector<std::vector<int32_t>> types(nsub);
        double tab_blocks = 0.0, blocks = 0.0;
#pragma omp parallel for schedule(dynamic, 1) reduction(+ : tab_blocks, blocks)
        for (int s = 0; s < nsub; ++s) {
            const Bsr3& A = *subs[s].K[l];
            keys[l][s] = quantised_keys(subs[s].coords, subs[s].nnodes[l]);
            if (opt.table_mode == 0) continue;
            int64_t nt = 0, tmax = 0;
            for (int64_t r = 0; r < A.nb; ++r) tmax = std::max<int64_t>(tmax, A.ptr[r + 1] - A.ptr[r]);
            if (tmax > kMaxRowBlocks) continue;  // long rows: no table for this subdomain
            types[s] = row_types(A, subs[s].free_flags(l), keys[l][s], nt);
            tab_blocks += (double)nt * (double)tmax;
            blocks += (double)A.nnzb();
        }
        grouped[l] = opt.table_mode == 2 || (opt.table_mode == 1 && tab_blocks <= 0.2 * blocks);
        for (int s = 0; s < nsub; ++s)
            perm[l][s] = device_order(keys[l][s], grouped[l] && !types[s].empty() ? &types[s] : nullptr);
    }
    lev.resize(nlev);
    for (int l = 0; l < nlev; ++l) {
        LevelDev& L = lev[l];
        L.noff.resize(nsub);
        L.nloc.resize(nsub);
        int64_t tot = 0;
        for (int s = 0; s < nsub; ++s) {
            L.noff[s] = tot;
            L.nloc[s] = subs[s].nnodes[l];
            tot += pad64(L.nloc[s]);
        }
        L.nn = tot;
        L.nch = tot / kChunk;
        std::vector<int32_t> slots(L.nch, 0), csub(L.nch, 0);
        std::vector<int64_t> off(L.nch + 1, 0);
        for (int s = 0; s < nsub; ++s) {
            const Bsr3& A = *subs[s].K[l];
            const auto& p = perm[l][s];
            const int64_t c0 = L.noff[s] / kChunk;
            for (int64_t c = c0; c < c0 + pad64(L.nloc[s]) / kChunk; ++c) csub[c] = s;
            for (int64_t r = 0; r < L.nloc[s]; ++r) {
                int32_t& sl = slots[c0 + p[r] / kChunk];
                sl = std::max<int32_t>(sl, (int32_t)(A.ptr[r + 1] - A.ptr[r]));
            }
            L.nnzb += A.nnzb();
            L.nnzb_sub.push_back(A.nnzb());
        }
        for (int64_t c = 0; c < L.nch; ++c) off[c + 1] = off[c] + slots[c];
        L.nslots = off[L.nch];
        std::vector<int32_t> col(L.nslots * kChunk, 0);
        std::vector<double> val(L.nslots * kChunk * 9, 0.0);
        std::vector<double> dinv(3 * L.nn, 0.0), minv(bj ? 9 * L.nn : 3 * L.nn, 0.0);
        std::vector<uint8_t> mask(L.nn, 0);
        for (int s = 0; s < nsub; ++s) {
            const Bsr3& A = *subs[s].K[l];
            const uint8_t* fr = subs[s].free_flags(l);  // reference order: level-l nodes are a prefix
            const auto& p = perm[l][s];
            const int64_t base = L.noff[s];
            // padded rows of the subdomain: self column, zero values
            for (int64_t r = L.nloc[s]; r < pad64(L.nloc[s]); ++r) {
                const int64_t g = base + r, c = g / kChunk, lane = g % kChunk;
                for (int64_t q = off[c]; q < off[c + 1]; ++q) col[q * kChunk + lane] = (int32_t)g;
            }
#pragma omp parallel for schedule(static)
            for (int64_t r = 0; r < L.nloc[s]; ++r) {
                const int64_t g = base + p[r], c = g / kChunk, lane = g % kChunk;
                uint8_t m = 0;
                for (int a = 0; a < 3; ++a) m |= fr[3 * r + a] ? (1 << a) : 0;
                mask[g] = m;
                // this row's blocks in canonical order (= increasing device column under the
                // lexicographic numbering), else in increasing device column
                const int64_t len = A.ptr[r + 1] - A.ptr[r];
                thread_local std::vector<int64_t> ordv;  // rows of any length (LAGRANGE's condensed systems)
                ordv.resize(len);
                int64_t* ord = ordv.data();
                if (!keys[l][s].empty()) {
                    canonical_slots(A, r, keys[l][s], ord);
                } else {
                    for (int64_t t = 0; t < len; ++t) ord[t] = A.ptr[r] + t;
                    std::sort(ord, ord + len, [&](int64_t u, int64_t v) { return p[A.col[u]] < p[A.col[v]]; });
                }
                double diag[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
                for (int64_t t = 0; t < len; ++t) {
                    const int64_t k = ord[t], q = off[c] + t;
                    const int64_t j = A.col[k];
                    col[q * kChunk + lane] = (int32_t)(base + p[j]);
                    for (int a = 0; a < 3; ++a)
                        for (int b = 0; b < 3; ++b) {
                            double v = A.val[9 * k + 3 * a + b];
                            if (!fr[3 * r + a] || !fr[3 * j + b]) v = (j == r && a == b) ? 1.0 : 0.0;
                            val[(q * 9 + 3 * a + b) * kChunk + lane] = v;
                            if (j == r) diag[3 * a + b] = v;
                        }
                }
                for (int64_t q = off[c] + len; q < off[c + 1]; ++q) col[q * kChunk + lane] = (int32_t)g;
                for (int a = 0; a < 3; ++a) dinv[3 * g + a] = fr[3 * r + a] ? 1.0 / diag[4 * a] : 0.0;
                if (bj) {
                    double inv[9];
                    if (!invert3(diag, inv)) for (int q = 0; q < 9; ++q) inv[q] = 0.0;
                    for (int a = 0; a < 3; ++a)
                        for (int b = 0; b < 3; ++b)
                            minv[9 * g + 3 * a + b] = (fr[3 * r + a] && fr[3 * r + b]) ? inv[3 * a + b] : 0.0;
                } else {
                    for (int a = 0; a < 3; ++a) minv[3 * g + a] = dinv[3 * g + a];
                }
            }
        }
        L.slots.upload(slots);
        L.csub.upload(csub);
        L.off.upload(off);
        L.col.upload(col);
        {
            // relative 16-bit columns when every offset of the level fits (DDPCA_COL16=0: off)
            static const bool want16 = !std::getenv("DDPCA_COL16") || std::atoi(std::getenv("DDPCA_COL16")) != 0;
            bool fits = want16;
            std::vector<int16_t> col16(want16 ? col.size() : 0);
            for (int64_t c = 0; c < L.nch && fits; ++c)
                for (int64_t q = off[c]; q < off[c + 1] && fits; ++q)
                    for (int64_t lane = 0; lane < kChunk; ++lane) {
                        const int64_t d = (int64_t)col[q * kChunk + lane] - (c * kChunk + lane);
                        if (d < INT16_MIN || d > INT16_MAX) { fits = false; break; }
                        col16[q * kChunk + lane] = (int16_t)d;
                    }
            if (fits) L.col16.upload(col16);
        }
        if (opt.table_mode != 0 && l >= 1) build_table(L, slots, off, val, opt.table_mode == 2 || grouped[l]);
        if (std::getenv("DDPCA_VERBOSE"))
            std::fprintf(stderr, "[ddpca] level %d: %lld nodes, %lld chunks, %lld slots, table %d (%lld types, %lld uniform chunks)\n",
                         l, (long long)L.nn, (long long)L.nch, (long long)L.nslots, (int)L.tbl, (long long)L.ntypes,
                         (long long)L.nuniform);
        // fp64 values: the fine level (Krylov operator) and, without the fp32 preconditioner
        // copy, every level; the fp32 copy serves the V-cycle on levels >= 1 (level 0 is the
        // dense inverse).  Table-mode levels need neither.
        const bool vc32 = opt.precond_fp32 != 0 && nlev > 1;
        const int64_t nslot = L.nslots;
        // every (slot, lane) of the V-cycle copy, in the Krylov operator's slot order
        auto for_vc_slots = [&](auto&& put) {
#pragma omp parallel for schedule(static)
            for (int64_t q = 0; q < nslot; ++q)
                for (int64_t lane = 0; lane < kChunk; ++lane) put(q, q, lane);
        };
        const int64_t vc_nslot = nslot;
        if (!L.tbl && (l == nlev - 1 || !vc32)) {
            std::vector<double> v64(val.size());
#pragma omp parallel for schedule(static)
            for (int64_t q = 0; q < nslot; ++q)
                for (int ij = 0; ij < 9; ++ij)
                    for (int64_t lane = 0; lane < kChunk; ++lane)
                        v64[q * 9 * kChunk + slot_elem<double>(ij, lane)] = val[(q * 9 + ij) * kChunk + lane];
            L.val.upload(v64);
        }
        // levels in block-exponent fp16: the finest h16_levels (DDPCA_H16_LEVELS, default 3: +2 % over 1 under block
        // Jacobi, profiles/r01_sweep_h16.txt; with the multicolour fine level 3 over 2 +1.1 % at 8 subdomains,
        // +0.4 % at 2, 1 over 2 -4 %, the same 18.0 PCG iterations, profiles/r04j/ab_h16.txt)
        static const int h16_levels = std::getenv("DDPCA_H16_LEVELS") ? std::atoi(std::getenv("DDPCA_H16_LEVELS")) : 3;
        // precond_fp32 = 3: the same levels in block-scaled int8 (the finest DDPCA_Q8_LEVELS of them, default all)
        static const int q8_levels = std::getenv("DDPCA_Q8_LEVELS") ? std::atoi(std::getenv("DDPCA_Q8_LEVELS")) : 64;
        const bool lowp = !L.tbl && vc32 && l >= 1 && l >= nlev - h16_levels && opt.precond_fp32 >= 2;
        // (a level with a block whose scale leaves fp32's normal range -- entries beyond ~1e38 or
        // below ~1e-36 -- keeps the block-exponent fp16 copy, whose exponent has no such limit)
        bool q8_done = false;
        if (lowp && opt.precond_fp32 >= 3 && l >= nlev - q8_levels) {
            std::vector<uint8_t> v8((size_t)vc_nslot * 12 * kChunk, 0);
            std::atomic<bool> ok{true};
            for_vc_slots([&](int64_t q, int64_t dst, int64_t lane) {
                double blk[9];
                uint8_t rec[12];
                for (int ij = 0; ij < 9; ++ij) blk[ij] = val[(q * 9 + ij) * kChunk + lane];
                if (!to_q8_block(blk, rec)) ok = false;
                for (int k = 0; k < 12; ++k) v8[dst * 12 * kChunk + q8_pos(k, lane)] = rec[k];
            });
            if (ok) {
                L.val8.upload(v8);
                q8_done = true;
            } else if (std::getenv("DDPCA_VERBOSE")) {
                std::fprintf(stderr, "[ddpca] level %d: int8 scale out of range, block-exponent fp16 copy instead\n", l);
            }
        }
        if (!q8_done && lowp) {
            // block-exponent fp16 copy of the fine level for the smoother and the V-cycle
            // residual (symmetric: a block and its transpose round alike); coarser levels fp32
            std::vector<uint16_t> v16((size_t)vc_nslot * 10 * kChunk, 0);  // zero blocks: e = 0, values 0
            for_vc_slots([&](int64_t q, int64_t dst, int64_t lane) {
                double blk[9];
                uint16_t rec[10];
                for (int ij = 0; ij < 9; ++ij) blk[ij] = val[(q * 9 + ij) * kChunk + lane];
                to_h16_block(blk, rec);
                for (int k = 0; k < 10; ++k) v16[dst * 10 * kChunk + 128 * (k / 2) + 2 * lane + k % 2] = rec[k];
            });
            L.val16.upload(v16);
        } else if (!q8_done && !L.tbl && vc32 && l >= 1) {
            std::vector<float> v32((size_t)vc_nslot * 9 * kChunk, 0.0f);
            for_vc_slots([&](int64_t q, int64_t dst, int64_t lane) {
                for (int ij = 0; ij < 9; ++ij)
                    v32[dst * 9 * kChunk + slot_elem<float>(ij, lane)] = (float)val[(q * 9 + ij) * kChunk + lane];
            });
            L.val32.upload(v32);
        }
        L.dinv.upload(dinv);
        L.minv.upload(minv);
        if (!L.tbl && vc32 && l >= 1) {
            // reduced-precision levels smooth with an fp32 inverse, symmetrised before rounding
            // so the V-cycle stays exactly symmetric (block Jacobi: M_ab = M_ba)
            std::vector<float> m32(minv.size());
            const int w = bj ? 9 : 3;
#pragma omp parallel for schedule(static)
            for (int64_t g = 0; g < L.nn; ++g) {
                const double* m = minv.data() + w * g;
                for (int k = 0; k < w; ++k)
                    m32[w * g + k] = bj && !general ? (float)(0.5 * (m[k] + m[3 * (k % 3) + k / 3])) : (float)m[k];
            }
            L.minv32.upload(m32);
        }
        if (l == nlev - 1 && nlev > 1 && opt.smoother >= 3) {
            // the V-cycle copy's storage type of this level (vc_type once the level is up)
            const int vt = (!vc32 || L.tbl) ? kVal64 : L.val8.p ? kValQ8 : L.val16.p ? kValH16 : kVal32;
            // band mode (locally refined fine level): sweep only the nodes this level
            // adds to level l - 1 (reference positions past nnodes[l - 1]) and their neighbours --
            // elsewhere the stencils are level l - 1's, which the V-cycle smooths next -- when that
            // is at most 60 % of the rows; DDPCA_GS_BAND=0 sweeps every row
            std::vector<uint8_t> bandv;
            const char* be = std::getenv("DDPCA_GS_BAND");
            if (!(be && be[0] == '0') && opt.smoother == 3) {  // (colour SSOR sweeps every row)
                bandv.assign(L.nn, 0);
                int64_t nreal = 0, nband = 0;
                for (int s = 0; s < nsub; ++s) {
                    nreal += L.nloc[s];
                    for (int64_t ref = subs[s].nnodes[l - 1]; ref < subs[s].nnodes[l]; ++ref)
                        bandv[L.noff[s] + perm[l][s][ref]] = 2;  // new node
                }
                for (int64_t g = 0; g < L.nn; ++g) {
                    if (bandv[g] != 2) continue;
                    const int64_t c = g / kChunk, lane = g % kChunk;
                    for (int64_t q = off[c]; q < off[c + 1]; ++q) {
                        bool nz = false;
                        for (int ij = 0; ij < 9 && !nz; ++ij) nz = val[(q * 9 + ij) * kChunk + lane] != 0.0;
                        const int64_t j = col[q * kChunk + lane];
                        if (nz && bandv[j] == 0) bandv[j] = 1;
                    }
                }
                for (uint8_t f : bandv) nband += f != 0;
                if (nband == 0 || nband > (nreal * 3) / 5) bandv.clear();
            }
            build_gs(gs, L, nsub, off, col, val, vt, bandv.empty() ? nullptr : &bandv);
        }
        L.mask.upload(mask);
        for (auto* v : {&L.x, &L.t, &L.b, &L.r, &L.d}) {
            v->alloc(3 * L.nn);
            v->zero(stream);
        }
        if (l > 0) {
            const LevelDev& C = lev[l - 1];
            std::vector<int32_t> ppar(8 * L.nn, -1);
            std::vector<double> pw(8 * L.nn, 0.0);
            bool uw = true;  // every weight == 1 / the node's parent count
            std::vector<std::vector<std::pair<int32_t, double>>> kids(C.nn);
            struct ExtraEnt {
                int32_t f, c;
                double b[9];
            };
            std::deque<ExtraEnt> extra;  // scalar parents past the eighth, as blocks
            L.tent_sub.assign(nsub, 0);
            L.tblk_sub.assign(nsub, 0);
            for (int s = 0; s < nsub; ++s) {
                const Stencil& st = *subs[s].S[l - 1];
                const auto& pf = perm[l][s];
                const auto& pc = perm[l - 1][s];
                const int64_t nc = C.nloc[s];
                if (st.nf != L.nloc[s] || st.nc != nc) throw ApiError(DDPCA_EINVAL, "stencil shape");
                L.tblk_sub[s] = (int64_t)st.bent.size();
                L.tent_sub[s] = (int64_t)st.col.size() - L.tblk_sub[s];
                // block entries (weight 0 in the scalar stencil) run in k_prolong_rot / k_restrict_rot
                // only: they take no parent slot (a node may have any number of them)
                std::vector<uint8_t> isblk(st.col.size(), 0);
                for (int64_t e : st.bent) isblk[e] = 1;
                if (!st.bent.empty()) uw = false;
                for (int64_t i = 0; i < L.nloc[s]; ++i) {
                    int64_t np = 0;
                    for (int64_t e = st.ptr[i]; e < st.ptr[i + 1]; ++e) np += !isblk[e];
                    const int64_t gf = L.noff[s] + pf[i];
                    if (i < nc) {
                        if (np != 1 || st.col[st.ptr[i]] != i || st.w[st.ptr[i]] != 1.0)
                            throw ApiError(DDPCA_EINVAL, "stencil is not identity on coarse nodes");
                        const int64_t gc = C.noff[s] + pc[i];
                        ppar[gf] = (int32_t)gc;
                        pw[gf] = 1.0;
                        kids[gc].insert(kids[gc].begin(), {(int32_t)gf, 1.0});
                        continue;
                    }
                    // parents past the eighth (LAGRANGE's condensed transfers) run as w*I blocks
                    if (np > 8) uw = false;
                    int64_t k = 0;
                    for (int64_t e = st.ptr[i]; e < st.ptr[i + 1]; ++e) {
                        if (isblk[e]) continue;
                        if (k == 8) {
                            extra.push_back({(int32_t)gf, (int32_t)(C.noff[s] + pc[st.col[e]]), {}});
                            for (int q = 0; q < 9; ++q) extra.back().b[q] = q % 4 == 0 ? st.w[e] : 0.0;
                            continue;
                        }
                        if (st.w[e] != 1.0 / (double)np) uw = false;
                        const int64_t gc = C.noff[s] + pc[st.col[e]];
                        ppar[k * L.nn + gf] = (int32_t)gc;
                        pw[k * L.nn + gf] = st.w[e];
                        kids[gc].push_back({(int32_t)gf, st.w[e]});
                        ++k;
                    }
                }
            }
            // restriction children in SELL-64 over the coarse chunks; padding slots carry weight 0
            // on the node's own first child (or fine node 0 for padding nodes)
            std::vector<int32_t> rsl(C.nch, 0);
            std::vector<int64_t> rof(C.nch + 1, 0);
            for (int64_t c = 0; c < C.nch; ++c) {
                size_t mx = 0;
                for (int64_t j = c * kChunk; j < (c + 1) * kChunk; ++j) mx = std::max(mx, kids[j].size());
                rsl[c] = (int32_t)mx;
                rof[c + 1] = rof[c] + (int64_t)mx;
            }
            std::vector<int32_t> rcol(std::max<int64_t>(rof[C.nch] * kChunk, 1), 0);
            std::vector<double> rwt(std::max<int64_t>(rof[C.nch] * kChunk, 1), 0.0);
            for (int64_t j = 0; j < C.nn; ++j) {
                const int64_t c = j / kChunk, lane = j % kChunk;
                for (int64_t k = 0; k < rsl[c]; ++k) {
                    const int64_t q = (rof[c] + k) * kChunk + lane;
                    const bool real = k < (int64_t)kids[j].size();
                    rcol[q] = real ? kids[j][k].first : (kids[j].empty() ? 0 : kids[j][0].first);
                    rwt[q] = real ? kids[j][k].second : 0.0;
                }
            }
            // block entries: (fine node, coarse node, 3x3) in batch-global indices, as CSR by
            // fine node (prolongation) and by coarse node (restriction)
            struct RotEnt {
                int32_t f, c;
                const double* b;
            };
            std::vector<RotEnt> ents;
            for (int s = 0; s < nsub; ++s) {
                const Stencil& st = *subs[s].S[l - 1];
                if (st.bent.empty()) continue;
                const auto& pf = perm[l][s];
                const auto& pc = perm[l - 1][s];
                int64_t i = 0;
                for (size_t q = 0; q < st.bent.size(); ++q) {
                    const int64_t e = st.bent[q];
                    while (st.ptr[i + 1] <= e) ++i;
                    if (st.w[e] != 0.0) throw ApiError(DDPCA_EINVAL, "block transfer entry with a scalar weight");
                    ents.push_back({(int32_t)(L.noff[s] + pf[i]), (int32_t)(C.noff[s] + pc[st.col[e]]), &st.bval[9 * q]});
                }
            }
            for (const ExtraEnt& x : extra) ents.push_back({x.f, x.c, x.b});
            if (!ents.empty()) {
                auto upload_csr = [&](bool by_fine, int64_t& nr, DevBuf<int32_t>& row, DevBuf<int64_t>& ptr_,
                                      DevBuf<int32_t>& other, DevBuf<double>& blk) {
                    std::stable_sort(ents.begin(), ents.end(), [by_fine](const RotEnt& a, const RotEnt& b) {
                        return by_fine ? a.f < b.f : a.c < b.c;
                    });
                    std::vector<int32_t> r, o;
                    std::vector<int64_t> pt{0};
                    std::vector<double> bv;
                    for (size_t q = 0; q < ents.size(); ++q) {
                        const int32_t key = by_fine ? ents[q].f : ents[q].c;
                        if (r.empty() || r.back() != key) {
                            if (!r.empty()) pt.push_back((int64_t)q);
                            r.push_back(key);
                        }
                        o.push_back(by_fine ? ents[q].c : ents[q].f);
                        bv.insert(bv.end(), ents[q].b, ents[q].b + 9);
                    }
                    pt.push_back((int64_t)ents.size());
                    nr = (int64_t)r.size();
                    row.upload(r);
                    ptr_.upload(pt);
                    other.upload(o);
                    blk.upload(bv);
                };
                upload_csr(true, L.nrot, L.rot_row, L.rot_ptr, L.rot_par, L.rot_blk);
                upload_csr(false, L.nrotc, L.rotc_row, L.rotc_ptr, L.rotc_kid, L.rotc_blk);
            }
            // (read per handle: the general-mesh tests and bench line switch it off in-process)
            const bool want_lat = !std::getenv("DDPCA_LATTICE") || std::atoi(std::getenv("DDPCA_LATTICE")) != 0;
            if (want_lat && uw && ents.empty() && lattice_transfer(L, C, ppar, kids)) {
                if (std::getenv("DDPCA_VERBOSE")) std::fprintf(stderr, "[ddpca] level %d: lattice transfers\n", l);
                continue;
            }
            if (std::getenv("DDPCA_VERBOSE"))
                std::fprintf(stderr, "[ddpca] level %d: explicit transfer lists (uniform averaging %d, block entries %zu)\n", l,
                             (int)uw, ents.size());
            L.ppar.upload(ppar);
            L.uw = uw;  // prolongation weights from the parent count (restriction keeps rwt)
            if (!uw) L.pw.upload(pw);
            L.rslots.upload(rsl);
            L.roff.upload(rof);
            L.rcol.upload(rcol);
            L.rwt.upload(rwt);
        }
    }
    fine_perm = perm[nlev - 1];
    level_perm = perm;
    // exact coarse solve: dense inverse of each subdomain's masked operator on level clev, in
    // that level's device order.  clev: the option, or the highest level below the fine one
    // whose inverses of all members fit in 256 MB (a few-subdomain batch trades the coarse
    // levels' latency-bound launches for one GEMV over a larger dense inverse)
    {
        clev = 0;
        if (opt.coarse_level >= 0) clev = std::min(opt.coarse_level, nlev - 1);
        else
            for (int l = nlev - 2; l >= 1; --l) {
                double bytes = 0.0;
                int64_t nmax = 0;
                for (int s = 0; s < nsub; ++s) {
                    const double n = 3.0 * (double)subs[s].nnodes[l];
                    bytes += 8.0 * n * n;
                    nmax = std::max<int64_t>(nmax, 3 * subs[s].nnodes[l]);
                }
                if (bytes <= 256.0 * 1024 * 1024 && nmax <= 12288) { clev = l; break; }
            }
        if (nlev > 1 && clev == nlev - 1) clev = nlev - 2;
        int64_t n0max = 0;
        for (int s = 0; s < nsub; ++s) n0max = std::max<int64_t>(n0max, 3 * subs[s].nnodes[clev]);
        // a one-level handle too large for a dense inverse serves the diagonal-preconditioned
        // drivers only (precSwit 0; the V-cycle then reports DDPCA_ESTATE)
        no_coarse = diag_only || (nlev == 1 && n0max > 12288);
    }
    if (!no_coarse) {
        std::vector<double> packed;
        std::vector<int64_t> ao(nsub), no(nsub), nz(nsub), ldv(nsub);
        for (int s = 0; s < nsub; ++s) {
            const Bsr3& A = *subs[s].K[clev];
            const uint8_t* fr = subs[s].free_flags(clev);
            const auto& p = perm[clev][s];
            const int64_t nc = subs[s].nnodes[clev], n0 = 3 * nc;
            std::vector<double> D(n0 * n0, 0.0);
            // a constrained dof's decoupled row and column (zeroed again after the inverse) carry 1,
            // or in the general path the largest free diagonal entry, so that its pivot does not
            // read as near-singular against stiffness-scaled ones (inv_general_lu_device's test)
            double cdiag = 1.0;
            if (general) {
                cdiag = 0.0;
                for (int64_t r = 0; r < nc; ++r)
                    for (int64_t k = A.ptr[r]; k < A.ptr[r + 1]; ++k)
                        if (A.col[k] == r)
                            for (int a = 0; a < 3; ++a)
                                if (fr[3 * r + a]) cdiag = std::max(cdiag, std::abs(A.val[9 * k + 4 * a]));
                if (!(cdiag > 0.0)) cdiag = 1.0;
            }
            for (int64_t r = 0; r < nc; ++r)
                for (int64_t k = A.ptr[r]; k < A.ptr[r + 1]; ++k) {
                    const int64_t j = A.col[k];
                    for (int a = 0; a < 3; ++a)
                        for (int b = 0; b < 3; ++b) {
                            double v = A.val[9 * k + 3 * a + b];
                            if (!fr[3 * r + a] || !fr[3 * j + b]) v = (j == r && a == b) ? cdiag : 0.0;
                            D[(3 * p[r] + a) * n0 + 3 * p[j] + b] = v;
                        }
                }
            if (general) {
                // LU inverse when the LU is clearly regular, else the SVD pseudo-inverse
                double resid = INFINITY;
                const bool lu = inv_general_lu_device(D, n0, stream, &resid);
                int64_t dropped = 0;
                if (!lu) pinv_general_device(D, n0, stream, &dropped);
                coarse_inverse.push_back({lu ? 1 : 2, resid, dropped});
                if (std::getenv("DDPCA_VERBOSE"))
                    std::fprintf(stderr, "[ddpca] coarse inverse: %s, %ld rows, LU residual %.3g, %ld singular values dropped\n",
                                 lu ? "LU" : "SVD pseudo-inverse", (long)n0, resid, (long)dropped);
            } else {
                invert_spd_device(D, n0, stream);
                coarse_inverse.push_back({0, 0.0, 0});
            }
            for (int64_t r = 0; r < nc; ++r)
                for (int a = 0; a < 3; ++a) {
                    if (fr[3 * r + a]) continue;
                    const int64_t d = 3 * p[r] + a;
                    for (int64_t e = 0; e < n0; ++e) D[d * n0 + e] = D[e * n0 + d] = 0.0;
                }
            ao[s] = (int64_t)packed.size();
            no[s] = lev[clev].noff[s];
            nz[s] = n0;
            const int64_t ld = (n0 + 3) / 4 * 4;  // rows padded for 16-B loads (k_coarse)
            if (ld > 3 * pad64(lev[clev].nloc[s])) throw ApiError(DDPCA_ESTATE, "coarse row padding beyond the member");
            ldv[s] = ld;
            for (int64_t r = 0; r < n0; ++r) {
                packed.insert(packed.end(), D.begin() + r * n0, D.begin() + (r + 1) * n0);
                packed.insert(packed.end(), ld - n0, 0.0);
            }
        }
        if (vc32()) {
            // reduced-precision preconditioner storage: the (exactly symmetric) dense inverses in
            // fp32 -- half the bytes of the coarse GEMV, which dominates small batches' coarse time
            std::vector<float> p32(packed.begin(), packed.end());
            ainv32.upload(p32);
        } else
            ainv.upload(packed);
        aoff.upload(ao);
        c_noff.upload(no);
        c_n.upload(nz);
        c_ld.upload(ldv);
        if (std::getenv("DDPCA_VERBOSE"))
            std::fprintf(stderr, "[ddpca] exact coarse solve on level %d (%zu doubles of dense inverses)\n", clev, packed.size());
    }
    // condensed <-> nodal map of the fine level
    const LevelDev& F = lev.back();
    nfree.resize(nsub);
    free_dof_host.resize(nsub);
    free_dof.resize(nsub);
    std::vector<int64_t> cb(nsub + 1, 0);
    for (int s = 0; s < nsub; ++s) {
        for (int64_t d = 0; d < 3 * F.nloc[s]; ++d)
            if (subs[s].dof_free[d]) free_dof_host[s].push_back((int32_t)fine_dof(s, d));
        nfree[s] = (int64_t)free_dof_host[s].size();
        free_dof[s].upload(free_dof_host[s]);
        cb[s] = F.noff[s] / kChunk;
    }
    cb[nsub] = F.nch;
    fin_cb.upload(cb);
    {
        // the six PCG vectors in one allocation; DDPCA_STAGGER (doubles) shifts each vector's
        // start so equal indices of z, p, q do not share address bits
#ifdef DDPCA_STAGGER
        const int64_t stag = DDPCA_STAGGER;
#else
        const int64_t stag = 0;
#endif
        const int64_t seg = (3 * F.nn + 511) / 512 * 512 + stag;
        pcg_mem.alloc(6 * seg);
        pcg_mem.zero(stream);
        int i = 0;
        for (auto* v : {&xs, &rs, &zs, &ps, &qs, &bs}) {
            v->p = pcg_mem.p + (i++) * seg;
            v->n = 3 * F.nn;
        }
    }
    int64_t maxch = 0;
    for (auto& L : lev) maxch = std::max<int64_t>(maxch, L.nch);
    partial.alloc(2 * maxch);
    if (gs_fine()) gs.partial.alloc(gs.nchunk);
    if (gs_fine() && opt.precond_fp32 == 4 && !gs.band && lev.back().lat && lev.back().nrot == 0) {
        gs.x4.alloc(4 * lev.back().nn);
        gs.x4.zero(stream);
        // the residual the restriction reads, in fp32 too (DDPCA_GS_R32=0: fp64, A/B)
        const char* er = std::getenv("DDPCA_GS_R32");
        if (!(er && er[0] == '0')) {
            gs.r4.alloc(4 * lev.back().nn);
            gs.r4.zero(stream);
        }
        // the per-launch byte model on the 16-B iterate: gathers 16 instead of 24 B per distinct
        // node, the forward sweep writes 16 B per row, the backward sweep 16 + 24 (colour SSOR
        // builds its own model below)
        const int K = opt.smoother == 3 ? gs.ncol : 0;
        for (int k = 0; k < K; ++k) {
            gs.launch_bytes[k] -= 8.0 * gs.gx_f[k] + 8.0 * gs.rows_k[k];
            gs.launch_bytes[2 * K - k] += -8.0 * gs.gx_b[k] + 16.0 * gs.rows_k[k];
        }
        if (K) gs.launch_bytes[K] -= 8.0 * gs.gx_r;
        if (gs.r4.p)
            for (int k = 0; k < K; ++k) gs.launch_bytes[K] -= 8.0 * gs.rows_k[k];  // r written in 16 B
    }
    // fp32 iterate copies of the block-Jacobi levels (precond_fp32 = 4, block-Jacobi smoothing;
    // DDPCA_BJ_X4=0 keeps them fp64, A/B): every level the V-cycle smooths by block Jacobi whose
    // copy has 16-bit columns and streamed values (rotation block entries into it included) -- its
    // sweeps and residual gather one 16-B load per neighbour, only the level's last sweep writes
    // fp64.  Alternating in one call (profiles/r06n): the N = 8 rank 9.52 / 9.55 -> 9.00 / 9.00 ms
    // per ADMM iteration, the headline 19.73 / 19.74 -> 20.05 / 20.06 ADMM it/s, PCG iterations equal
    {
        const char* eb = std::getenv("DDPCA_BJ_X4");
        const bool on = !(eb && eb[0] == '0');
        if (on && opt.precond_fp32 == 4 && (opt.smoother == 1 || opt.smoother >= 3))
            for (int l = clev + 1; l < (int)lev.size(); ++l) {
                LevelDev& L = lev[l];
                if ((gs_fine() && l == (int)lev.size() - 1) || !L.col16.p || L.tbl) continue;
                L.x4a.alloc(4 * L.nn);
                L.x4b.alloc(4 * L.nn);
                L.x4a.zero(stream);
                L.x4b.zero(stream);
            }
    }
    if (gs_fine() && opt.smoother == 4) {
        if (gs.band) throw ApiError(DDPCA_EINVAL, "colour SSOR (smoother 4) on a band-mode fine level");
        gs.w.alloc(3 * lev.back().nn);
        gs.w.zero(stream);
        // the per-launch byte model in k_gs_ssor's launch order: forward colours 0..K-1 (L), backward
        // K-1..0 (U), the residual (L, every chunk), forward 0..K-1 (L + U), backward K-1..0 (U); per
        // row b, the fp32 inverse, w and x as each phase moves them, x gathered once per distinct node
        const int K = gs.ncol;
        const double xb = gs.x4.p ? 16.0 : 24.0, rb = gs.r4.p ? 16.0 : 24.0, m = 36.0, ix = 4.0;
        std::vector<double> lb;
        for (int k = 0; k < K; ++k) lb.push_back(gs.vb * gs.nl_k[k] + gs.rows_k[k] * (24 + m + xb + 24 + ix) + xb * gs.gx_f[k]);
        for (int k = K - 1; k >= 0; --k) lb.push_back(gs.vb * gs.nu_k[k] + gs.rows_k[k] * (48 + m + xb + ix) + xb * gs.gx_u[k]);
        double res = xb * gs.gx_l;
        for (int k = 0; k < K; ++k) res += gs.vb * gs.nl_k[k] + gs.rows_k[k] * (24 + rb + ix);
        lb.push_back(res);
        for (int k = 0; k < K; ++k)
            lb.push_back(gs.vb * (gs.nl_k[k] + gs.nu_k[k]) + gs.rows_k[k] * (24 + m + xb + 24 + ix) + xb * gs.gx_b[k]);
        for (int k = K - 1; k >= 0; --k)
            lb.push_back(gs.vb * gs.nu_k[k] + gs.rows_k[k] * (48 + m + 24 + (gs.x4.p ? xb : 0.0) + ix) + xb * gs.gx_u[k]);
        gs.launch_bytes = lb;
    }
    sc.alloc(nsub);
    DDPCA_HIP(hipHostMalloc(reinterpret_cast<void**>(&sc_host), nsub * sizeof(PcgScal)));
    std::memset(sc_host, 0, nsub * sizeof(PcgScal));
    mirror.alloc(nsub);
    DDPCA_HIP(hipEventCreate(&ev_k0));
    DDPCA_HIP(hipEventCreate(&ev_k1));
    // smoother coefficients from the spectrum of M K on each smoothed level and subdomain
    for (int l = 1; l < nlev; ++l) {
        estimate_lmax(l);
        std::vector<double> coef(2 * (opt.nu + 1) * nsub, 0.0);
        for (int k = 0; k <= opt.nu; ++k)
            for (int s = 0; s < nsub; ++s) {
                double c1 = 0.0, c2;
                if (opt.smoother == 2) cheb_coef(lev[l].lmax[s], k, c1, c2);
                else c2 = opt.omega > 0.0 ? opt.omega
                          : (opt.omega < 0.0 ? -opt.omega : 4.0 / 3.0) / lev[l].lmax[s];
                coef[2 * (k * nsub + s)] = c1;
                coef[2 * (k * nsub + s) + 1] = c2;
            }
        lev[l].coef.upload(coef);
    }
    DDPCA_HIP(hipStreamSynchronize(stream));
}

MgpisDevice::~MgpisDevice() {
    (void)hipSetDevice(device);
    if (stream) (void)hipStreamSynchronize(stream);
    for (hipStream_t xs : xstream_)
        if (xs) (void)hipStreamSynchronize(xs);
    for (auto* ga : {graph_, graph1_})
        for (int p = 0; p < 2; ++p)
            if (ga[p]) (void)hipGraphExecDestroy(ga[p]);
    for (auto* gh : {graph_h_, graph1_h_})
        for (int p = 0; p < 2; ++p)
            for (int h = 0; h < kMaxParts; ++h)
                if (gh[p][h]) (void)hipGraphExecDestroy(gh[p][h]);
    if (ev_fork_) (void)hipEventDestroy(ev_fork_);
    for (hipEvent_t e : ev_join_)
        if (e) (void)hipEventDestroy(e);
    for (hipStream_t xs : xstream_)
        if (xs) (void)hipStreamDestroy(xs);
    if (sc_host) (void)hipHostFree(sc_host);
    if (ev_k0) (void)hipEventDestroy(ev_k0);
    if (ev_k1) (void)hipEventDestroy(ev_k1);
    if (stream) (void)hipStreamDestroy(stream);
}

// lambda_max(M K) per subdomain by 24 power iterations (all subdomains of the batch at once).
void MgpisDevice::estimate_lmax(int l) {
    LevelDev& L = lev[l];
    const bool bj = opt.smoother >= 1;
    const int64_t n = 3 * L.nn;
    std::vector<double> h(n, 0.0);
    std::vector<uint8_t> mask = L.mask.download();
    for (int s = 0; s < nsub; ++s) {
        std::mt19937_64 rng(20251017 + l);
        std::uniform_real_distribution<double> U(-1.0, 1.0);
        for (int64_t i = 3 * L.noff[s]; i < 3 * (L.noff[s] + L.nloc[s]); ++i) h[i] = (mask[i / 3] >> (i % 3)) & 1 ? U(rng) : 0.0;
    }
    DevBuf<double> v, w, scale(nsub);
    v.upload(h);
    w.alloc(n);
    const int nb = ceil_div(L.nn, kBlock);
    std::vector<double> part(L.nch), nrm(nsub), inv(nsub);
    auto norms = [&]() {
        DDPCA_HIP(hipMemcpyAsync(part.data(), partial.p, L.nch * sizeof(double), hipMemcpyDeviceToHost, stream));
        DDPCA_HIP(hipStreamSynchronize(stream));
        for (int s = 0; s < nsub; ++s) {
            double t = 0.0;
            for (int64_t c = L.noff[s] / kChunk; c < (L.noff[s] + pad64(L.nloc[s])) / kChunk; ++c) t += part[c];
            nrm[s] = std::sqrt(t);
            inv[s] = nrm[s] > 0.0 ? 1.0 / nrm[s] : 0.0;
        }
    };
    auto apply_m = [&](const double* x) {
        if (vc_type(l) != kVal64) {  // the smoother's own (fp32) inverse
            if (bj) hipLaunchKernelGGL((k_apply_m<true, float>), dim3(nb), dim3(kBlock), 0, stream, x, L.minv32.p, w.p, partial.p, L.nn);
            else hipLaunchKernelGGL((k_apply_m<false, float>), dim3(nb), dim3(kBlock), 0, stream, x, L.minv32.p, w.p, partial.p, L.nn);
        } else if (bj) hipLaunchKernelGGL((k_apply_m<true>), dim3(nb), dim3(kBlock), 0, stream, x, L.minv.p, w.p, partial.p, L.nn);
        else hipLaunchKernelGGL((k_apply_m<false>), dim3(nb), dim3(kBlock), 0, stream, x, L.minv.p, w.p, partial.p, L.nn);
    };
    apply_m(v.p);
    norms();
    for (int it = 0; it < 24; ++it) {
        // v <- w / |w| ; w <- M K v
        DDPCA_HIP(hipMemcpyAsync(scale.p, inv.data(), nsub * sizeof(double), hipMemcpyHostToDevice, stream));
        hipLaunchKernelGGL(k_scale_sub, dim3(nb), dim3(kBlock), 0, stream, w.p, scale.p, v.p, L.nn, L.csub.p);
        spmv(l, v.p, L.r.p, true);  // the smoother's operator
        apply_m(L.r.p);
        norms();
    }
    L.lmax.resize(nsub);
    for (int s = 0; s < nsub; ++s) L.lmax[s] = nrm[s] * 1.05;  // safety margin on the estimate
}

// ============================================================================== operations
namespace {
// Krylov-operator arguments (fp64 values) of a level
SellArgs level_args(const LevelDev& L) {
    SellArgs a{};
    a.slots = L.slots.p;
    a.off = L.off.p;
    a.col = L.col.p;
    a.col16 = L.col16.p;
    a.val = L.val.p;
    a.csub = L.csub.p;
    a.nch = L.nch;
    a.minv = L.minv.p;

    if (L.tbl) {
        a.val = nullptr;
        a.rtype = L.rtype.p;
        a.ctype = L.ctype.p;
        a.tab = L.tab.p;
        a.tstride = L.tstride;
    }
    return a;
}

// one SELL launch over a level: table mode when the arguments carry a table, else values
// streamed in storage type vt (kVal64 / kVal32 / kValH16 / kValQ8)
template <int MODE, bool BJ, bool DOT>
void launch_sell(int vt, const SellArgs& a, hipStream_t s) {
    const int grid = ceil_div(a.nch, 4);
    constexpr int V = default_variant(MODE);
    using I16 = int16_t;
    // small levels: the row-split kernel (DDPCA_SPLIT_CHUNKS = the largest level it takes, in chunks)
    // (read per launch: launches are captured into graphs once per handle, and tests switch it)
    const char* esp = std::getenv("DDPCA_SPLIT_CHUNKS");
    const int64_t split_max = esp ? std::atoll(esp) : 2048;
    if constexpr (MODE == kResid || MODE == kJac) {
        if (a.x4) {
            // a block-Jacobi level's fp32 iterate copy (LevelDev::x4a): the constructor enables it
            // on levels with 16-bit columns and streamed values only
            if (a.tab || !a.col16) throw ApiError(DDPCA_ESTATE, "fp32 iterate copy needs 16-bit columns and streamed values");
            if (!DOT && a.nch <= split_max) {
                const dim3 gs((unsigned)a.nch);
                if (vt == kValQ8) hipLaunchKernelGGL((k_sell_split<MODE, BJ, uint8_t, I16, true>), gs, dim3(kBlock), 0, s, a);
                else if (vt == kValH16) hipLaunchKernelGGL((k_sell_split<MODE, BJ, uint16_t, I16, true>), gs, dim3(kBlock), 0, s, a);
                else if (vt == kVal32) hipLaunchKernelGGL((k_sell_split<MODE, BJ, float, I16, true>), gs, dim3(kBlock), 0, s, a);
                else hipLaunchKernelGGL((k_sell_split<MODE, BJ, double, I16, true>), gs, dim3(kBlock), 0, s, a);
                return;
            }
            if (vt == kValQ8) hipLaunchKernelGGL((k_sell<MODE, BJ, DOT, uint8_t, V, false, I16, true>), dim3(grid), dim3(kBlock), 0, s, a, a.tab);
            else if (vt == kValH16) hipLaunchKernelGGL((k_sell<MODE, BJ, DOT, uint16_t, V, false, I16, true>), dim3(grid), dim3(kBlock), 0, s, a, a.tab);
            else if (vt == kVal32) hipLaunchKernelGGL((k_sell<MODE, BJ, DOT, float, V, false, I16, true>), dim3(grid), dim3(kBlock), 0, s, a, a.tab);
            else hipLaunchKernelGGL((k_sell<MODE, BJ, DOT, double, V, false, I16, true>), dim3(grid), dim3(kBlock), 0, s, a, a.tab);
            return;
        }
    }
    // (V-cycle modes only: y = Kx keeps the slot order the table mode reproduces bit for bit)
    if constexpr (!DOT && (MODE == kResid || MODE == kJac)) {
        if (!a.tab && a.nch <= split_max) {
            const dim3 gs((unsigned)a.nch);
            if (a.col16) {
                if (vt == kValQ8) hipLaunchKernelGGL((k_sell_split<MODE, BJ, uint8_t, I16>), gs, dim3(kBlock), 0, s, a);
                else if (vt == kValH16) hipLaunchKernelGGL((k_sell_split<MODE, BJ, uint16_t, I16>), gs, dim3(kBlock), 0, s, a);
                else if (vt == kVal32) hipLaunchKernelGGL((k_sell_split<MODE, BJ, float, I16>), gs, dim3(kBlock), 0, s, a);
                else hipLaunchKernelGGL((k_sell_split<MODE, BJ, double, I16>), gs, dim3(kBlock), 0, s, a);
            } else if (vt == kValQ8) hipLaunchKernelGGL((k_sell_split<MODE, BJ, uint8_t, int32_t>), gs, dim3(kBlock), 0, s, a);
            else if (vt == kValH16) hipLaunchKernelGGL((k_sell_split<MODE, BJ, uint16_t, int32_t>), gs, dim3(kBlock), 0, s, a);
            else if (vt == kVal32) hipLaunchKernelGGL((k_sell_split<MODE, BJ, float, int32_t>), gs, dim3(kBlock), 0, s, a);
            else hipLaunchKernelGGL((k_sell_split<MODE, BJ, double, int32_t>), gs, dim3(kBlock), 0, s, a);
            return;
        }
    }
    if (a.tab) hipLaunchKernelGGL((k_sell<MODE, BJ, DOT, double, V, true>), dim3(grid), dim3(kBlock), 0, s, a, a.tab);
    else if (a.col16) {
        if (vt == kValQ8) hipLaunchKernelGGL((k_sell<MODE, BJ, DOT, uint8_t, V, false, I16>), dim3(grid), dim3(kBlock), 0, s, a, a.tab);
        else if (vt == kValH16) hipLaunchKernelGGL((k_sell<MODE, BJ, DOT, uint16_t, V, false, I16>), dim3(grid), dim3(kBlock), 0, s, a, a.tab);
        else if (vt == kVal32) hipLaunchKernelGGL((k_sell<MODE, BJ, DOT, float, V, false, I16>), dim3(grid), dim3(kBlock), 0, s, a, a.tab);
        else hipLaunchKernelGGL((k_sell<MODE, BJ, DOT, double, V, false, I16>), dim3(grid), dim3(kBlock), 0, s, a, a.tab);
    } else if (vt == kValQ8) hipLaunchKernelGGL((k_sell<MODE, BJ, DOT, uint8_t>), dim3(grid), dim3(kBlock), 0, s, a, a.tab);
    else if (vt == kValH16) hipLaunchKernelGGL((k_sell<MODE, BJ, DOT, uint16_t>), dim3(grid), dim3(kBlock), 0, s, a, a.tab);
    else if (vt == kVal32) hipLaunchKernelGGL((k_sell<MODE, BJ, DOT, float>), dim3(grid), dim3(kBlock), 0, s, a, a.tab);
    else hipLaunchKernelGGL((k_sell<MODE, BJ, DOT, double>), dim3(grid), dim3(kBlock), 0, s, a, a.tab);
}

template <int MODE, bool BJ, bool DOT>
void launch_loop(int loop, int vt, const SellArgs& a, int grid, hipStream_t s) {
    if (vt == kValQ8) {
        switch (loop) {
            case 0: hipLaunchKernelGGL((k_sell<MODE, BJ, DOT, uint8_t, 0>), dim3(grid), dim3(kBlock), 0, s, a, a.tab); break;
            case 1: hipLaunchKernelGGL((k_sell<MODE, BJ, DOT, uint8_t, 1>), dim3(grid), dim3(kBlock), 0, s, a, a.tab); break;
            case 2: hipLaunchKernelGGL((k_sell<MODE, BJ, DOT, uint8_t, 2>), dim3(grid), dim3(kBlock), 0, s, a, a.tab); break;
            default: hipLaunchKernelGGL((k_sell<MODE, BJ, DOT, uint8_t, 3>), dim3(grid), dim3(kBlock), 0, s, a, a.tab); break;
        }
        return;
    }
    if (vt == kValH16) {
        switch (loop) {
            case 0: hipLaunchKernelGGL((k_sell<MODE, BJ, DOT, uint16_t, 0>), dim3(grid), dim3(kBlock), 0, s, a, a.tab); break;
            case 1: hipLaunchKernelGGL((k_sell<MODE, BJ, DOT, uint16_t, 1>), dim3(grid), dim3(kBlock), 0, s, a, a.tab); break;
            case 2: hipLaunchKernelGGL((k_sell<MODE, BJ, DOT, uint16_t, 2>), dim3(grid), dim3(kBlock), 0, s, a, a.tab); break;
            default: hipLaunchKernelGGL((k_sell<MODE, BJ, DOT, uint16_t, 3>), dim3(grid), dim3(kBlock), 0, s, a, a.tab); break;
        }
        return;
    }
    if (vt == kVal32) {
        switch (loop) {
            case 0: hipLaunchKernelGGL((k_sell<MODE, BJ, DOT, float, 0>), dim3(grid), dim3(kBlock), 0, s, a, a.tab); break;
            case 1: hipLaunchKernelGGL((k_sell<MODE, BJ, DOT, float, 1>), dim3(grid), dim3(kBlock), 0, s, a, a.tab); break;
            case 2: hipLaunchKernelGGL((k_sell<MODE, BJ, DOT, float, 2>), dim3(grid), dim3(kBlock), 0, s, a, a.tab); break;
            default: hipLaunchKernelGGL((k_sell<MODE, BJ, DOT, float, 3>), dim3(grid), dim3(kBlock), 0, s, a, a.tab); break;
        }
        return;
    }
    switch (loop) {
        case 0: hipLaunchKernelGGL((k_sell<MODE, BJ, DOT, double, 0>), dim3(grid), dim3(kBlock), 0, s, a, a.tab); break;
        case 1: hipLaunchKernelGGL((k_sell<MODE, BJ, DOT, double, 1>), dim3(grid), dim3(kBlock), 0, s, a, a.tab); break;
        case 2: hipLaunchKernelGGL((k_sell<MODE, BJ, DOT, double, 2>), dim3(grid), dim3(kBlock), 0, s, a, a.tab); break;
        default: hipLaunchKernelGGL((k_sell<MODE, BJ, DOT, double, 3>), dim3(grid), dim3(kBlock), 0, s, a, a.tab); break;
    }
}
}  // namespace

namespace {
// V-cycle-operator arguments of a level: the fp32 copy when the preconditioner stores it
SellArgs vc_level_args(const MgpisDevice& D, int level) {
    SellArgs a = level_args(D.lev[level]);
    const int vt = D.vc_type(level);
    const LevelDev& L = D.lev[level];
    if (vt == kValQ8) a.val = L.val8.p;
    else if (vt == kValH16) a.val = L.val16.p;
    else if (vt == kVal32) a.val = L.val32.p;
    if (vt != kVal64) a.minv = L.minv32.p;
    return a;
}
}  // namespace

namespace {
// k_restrict over level l -> l-1 with the transfer's weight form (stored or uniform)
template <bool INIT, bool BJ, bool SETD, typename MT>
void launch_restrict(const LevelDev& F, int grid, hipStream_t st, const double* rf, const uint8_t* cmask, double* bc,
                     double* xc, double* dc, const MT* minv, const double* coef, int64_t nc, const int32_t* csub,
                     const PcgScal* sc, const float4* rf4 = nullptr, float4* xc4 = nullptr) {
    // rf4: the fine residual in the colour sweeps' fp32 copy (lattice transfers only, GsFine::r4);
    // xc4: the fused first coarse sweep writes the coarse level's fp32 iterate copy (LevelDev::x4a)
    if (rf4) {
        if (!F.lat) throw ApiError(DDPCA_ESTATE, "fp32 residual copy without lattice transfers");
        hipLaunchKernelGGL((k_restrict_lat<INIT, BJ, SETD, MT, float4>), dim3(grid), dim3(kBlock), 0, st, rf4, F.rmsk.p,
                           F.rf0.p, F.rstr.p, cmask, bc, xc, dc, minv, coef, nc, csub, sc, xc4);
        return;
    }
    // stored weights: deriving them from a gathered parent count (as k_prolong<true> does)
    // measured 58 -> 102 us on the fine level (profiles/r01_transfer_weights.txt)
    if (F.lat) {
        hipLaunchKernelGGL((k_restrict_lat<INIT, BJ, SETD, MT>), dim3(grid), dim3(kBlock), 0, st, rf, F.rmsk.p, F.rf0.p,
                           F.rstr.p, cmask, bc, xc, dc, minv, coef, nc, csub, sc, xc4);
        return;
    }
    hipLaunchKernelGGL((k_restrict<INIT, BJ, SETD, MT>), dim3(grid), dim3(kBlock), 0, st, rf, F.rslots.p, F.roff.p,
                       F.rcol.p, F.rwt.p, cmask, bc, xc, dc, minv, coef, nc, csub, sc, xc4);
}
}  // namespace

void MgpisDevice::restrict_level(int l, const double* rf, double* bc) {
    if (l < 1 || l >= (int)lev.size()) throw ApiError(DDPCA_EINVAL, "restrict_level: level");
    const LevelDev& F = lev[l];
    const LevelDev& C = lev[l - 1];
    launch_restrict<false, false, false, double>(F, ceil_div(C.nn, kBlock), stream, rf, C.mask.p, bc, nullptr, nullptr,
                                                 nullptr, nullptr, C.nn, C.csub.p, nullptr);
    rot_restrict(l, rf, bc, nullptr);
}

void MgpisDevice::rot_restrict(int l, const double* rf, double* bc, const PcgScal* scp) {
    const LevelDev& F = lev[l];
    if (!F.nrotc) return;
    hipLaunchKernelGGL(k_restrict_rot, dim3(ceil_div(F.nrotc, kBlock)), dim3(kBlock), 0, stream, rf, F.rotc_row.p,
                       F.rotc_ptr.p, F.rotc_kid.p, F.rotc_blk.p, lev[l - 1].mask.p, bc, F.nrotc, lev[l - 1].csub.p, scp);
}

void MgpisDevice::rot_prolong(int l, const double* ec, double* xf, const PcgScal* scp, float4* xf4) {
    const LevelDev& F = lev[l];
    if (!F.nrot) return;
    if (xf4)  // the level's fp32 iterate copy (LevelDev::x4a)
        hipLaunchKernelGGL(k_prolong_rot_x4, dim3(ceil_div(F.nrot, kBlock)), dim3(kBlock), 0, stream, ec, F.rot_row.p,
                           F.rot_ptr.p, F.rot_par.p, F.rot_blk.p, F.mask.p, xf4, F.nrot, F.csub.p, scp);
    else
        hipLaunchKernelGGL(k_prolong_rot, dim3(ceil_div(F.nrot, kBlock)), dim3(kBlock), 0, stream, ec, F.rot_row.p,
                           F.rot_ptr.p, F.rot_par.p, F.rot_blk.p, F.mask.p, xf, F.nrot, F.csub.p, scp);
}

void MgpisDevice::spmv(int level, const double* x, double* y, bool vc_op) {
    SellArgs a = vc_op ? vc_level_args(*this, level) : level_args(lev[level]);
    if (!a.val && !a.tab) throw ApiError(DDPCA_ESTATE, "operator of this level is not stored in the requested precision");
    a.x = x;
    a.y = y;
    launch_sell<kSpmv, false, false>(vc_op ? vc_type(level) : kVal64, a, stream);
}

double MgpisDevice::bench_spmv(int variant, int reps) {
    // variant = loop (0..3) + 4 * mode (0 y = Kx, 1 PCG, 2 residual, 3 Chebyshev sweep) + 16 *
    // fp32 values (the V-cycle copy); fine level, whole batch, operands in the PCG work vectors
    // (values are irrelevant to the timing)
    // table-mode levels (y = Kx only): + 32 selects the table diagnostics, loop 0 per-lane
    // table rows, 1 production, 3 coalesced-x bound, 32 + 0/1 x stride 4 (16+8 B / 2x16 B loads)
    const LevelDev& L = lev.back();
    const int loop = variant & 3, mode = (variant >> 2) & 3;
    const bool f32 = (variant & 16) != 0;
    const int vt = !f32 ? kVal64 : vc_type((int)lev.size() - 1);  // the V-cycle's copy
    const int tloop = (variant & 32) ? 4 + (loop & 1) : loop;
    if (variant >= 64 || ((variant & 32) && (!L.tbl || mode != 0 || f32))) throw ApiError(DDPCA_EINVAL, "unknown SpMV variant");
    if (mode == 3 && (lev.size() < 2 || opt.smoother < 1)) throw ApiError(DDPCA_EINVAL, "Chebyshev mode needs block smoothing");
    if (f32 && !L.val32.p && !L.val16.p && !L.val8.p) throw ApiError(DDPCA_EINVAL, "no reduced-precision operator (precond_fp32 = 0)");
    DDPCA_HIP(hipMemsetAsync(sc.p, 0, nsub * sizeof(PcgScal), stream));  // done = 0, beta = 0
    SellArgs a = level_args(L);
    if (f32) {
        a.val = vc_level_args(*this, (int)lev.size() - 1).val;
        a.tab = nullptr;
    }
    a.x = xs.p;
    a.y = qs.p;
    a.p = ps.p;
    a.b = bs.p;
    a.xo = rs.p;
    a.partial = partial.p;
    a.sc = sc.p;
    if (lev.size() > 1) a.coef = L.coef.p;
    const int grid = ceil_div(a.nch, 4);
    DevBuf<double> x4;
    if (tloop >= 4) {  // x in a 4-double-per-node copy
        x4.alloc(4 * L.nn);
        DDPCA_HIP(hipMemcpy2DAsync(x4.p, 32, xs.p, 24, 24, L.nn, hipMemcpyDeviceToDevice, stream));
        a.x = x4.p;
    }
    auto launch = [&]() {
        if (a.tab && mode == 0 && tloop != 1) {
#define TBL_V(v) hipLaunchKernelGGL((k_sell<kSpmv, false, false, double, v, true>), dim3(grid), dim3(kBlock), 0, stream, a, a.tab)
            switch (tloop) {
                case 0: TBL_V(0); break;
                case 3: TBL_V(3); break;
                case 4: TBL_V(4); break;
                case 5: TBL_V(5); break;
                default: TBL_V(2); break;
            }
#undef TBL_V
            return;
        }
        if (a.tab) {  // table mode: one loop variant
            if (mode == 0) launch_sell<kSpmv, false, false>(kVal64, a, stream);
            else if (mode == 1) launch_sell<kPcg, false, true>(kVal64, a, stream);
            else if (mode == 2) launch_sell<kResid, false, false>(kVal64, a, stream);
            else launch_sell<kCheb, true, false>(kVal64, a, stream);
            return;
        }
        if (mode == 0) launch_loop<kSpmv, false, false>(loop, vt, a, grid, stream);
        else if (mode == 1) launch_loop<kPcg, false, true>(loop, vt, a, grid, stream);
        else if (mode == 2) launch_loop<kResid, false, false>(loop, vt, a, grid, stream);
        else launch_loop<kCheb, true, false>(loop, vt, a, grid, stream);
    };
    launch();
    DDPCA_HIP(hipEventRecord(ev_k0, stream));
    for (int r = 0; r < reps; ++r) launch();
    DDPCA_HIP(hipEventRecord(ev_k1, stream));
    DDPCA_HIP(hipEventSynchronize(ev_k1));
    float ms = 0.f;
    DDPCA_HIP(hipEventElapsedTime(&ms, ev_k0, ev_k1));
    return (double)ms / std::max(reps, 1);
}

namespace {
// one k_gs launch: phase ph over colour k's chunks (k < 0: every chunk)
template <int PH, bool DOT, typename T>
void launch_gs_t(const GsArgs& a, bool c16, hipStream_t st) {  // c16: 16-bit column offsets, else int32 columns
    if (a.x4) {
        if (c16) hipLaunchKernelGGL((k_gs<PH, DOT, T, int16_t, true>), dim3((unsigned)a.n), dim3(kWave), 0, st, a);
        else hipLaunchKernelGGL((k_gs<PH, DOT, T, int32_t, true>), dim3((unsigned)a.n), dim3(kWave), 0, st, a);
        return;
    }
    if (c16) hipLaunchKernelGGL((k_gs<PH, DOT, T, int16_t>), dim3((unsigned)a.n), dim3(kWave), 0, st, a);
    else hipLaunchKernelGGL((k_gs<PH, DOT, T, int32_t>), dim3((unsigned)a.n), dim3(kWave), 0, st, a);
}

template <int PH, bool DOT, typename T>
void launch_gs_ssor_t(const GsArgs& a, bool c16, hipStream_t st) {
    if (a.x4) {
        if (c16) hipLaunchKernelGGL((k_gs_ssor<PH, DOT, T, int16_t, true>), dim3((unsigned)a.n), dim3(kWave), 0, st, a);
        else hipLaunchKernelGGL((k_gs_ssor<PH, DOT, T, int32_t, true>), dim3((unsigned)a.n), dim3(kWave), 0, st, a);
        return;
    }
    if (c16) hipLaunchKernelGGL((k_gs_ssor<PH, DOT, T, int16_t>), dim3((unsigned)a.n), dim3(kWave), 0, st, a);
    else hipLaunchKernelGGL((k_gs_ssor<PH, DOT, T, int32_t>), dim3((unsigned)a.n), dim3(kWave), 0, st, a);
}

template <int PH, typename T>
void launch_gs_aux_t(const GsArgs& a, bool c16, hipStream_t st) {
    if (c16) hipLaunchKernelGGL((k_gs_aux<PH, T, int16_t>), dim3((unsigned)a.n), dim3(kWave), 0, st, a);
    else hipLaunchKernelGGL((k_gs_aux<PH, T, int32_t>), dim3((unsigned)a.n), dim3(kWave), 0, st, a);
}

// k >= 0: colour k; k = -1: every colour chunk (the residual); band mode: k = -2 the ring group,
// k = -3 the ring and far groups (PH 3..5 run k_gs_aux)
template <int PH, bool DOT>
void launch_gs(const MgpisDevice& D, int k, double* x, const double* b, double* r, const PcgScal* scp, double* partial) {
    const GsFine& G = D.gs;
    const LevelDev& F = D.lev.back();
    const int K = G.ncol;
    GsArgs a{};
    if (k >= 0) {
        a.list = G.list.p + G.first[k];
        a.n = G.count[k];
    } else if (k == -1) {
        a.list = G.band ? G.list.p : nullptr;
        a.n = G.band ? G.first[K] : G.nchunk;
    } else {
        if (!G.band) throw ApiError(DDPCA_ESTATE, "ring / far chunk groups without band mode");
        a.list = G.list.p + G.first[K];
        a.n = G.count[K] + (k == -3 ? G.count[K + 1] : 0);
    }
    if (a.n == 0) return;
    a.rowidx = G.rowidx.p;
    a.csub = G.csub.p;
    a.nsl = G.nsl.p;
    a.nsu = G.nsu.p;
    a.offl = G.offl.p;
    a.offu = G.offu.p;
    a.col = G.col.p;
    a.col16 = G.col16.p;
    a.x = x;
    a.b = b;
    a.r = r;
    a.sc = scp;
    a.partial = partial;
    // the rows' fp32 inverses in chunk order (coalesced: read by row at stride 2 nodes they pulled
    // whole lines for half the data, +1.1 %, profiles/r03o); the fp64 copy reads minv by row
    a.minvc = G.minvc.p;
    a.x4 = reinterpret_cast<float4*>(G.x4.p);
    a.r4 = reinterpret_cast<float4*>(G.r4.p);
    a.w = G.w.p;
    const bool c16 = G.col16.p != nullptr;
    if constexpr (PH >= 6) {  // SSOR phases: the reduced-precision copies' chunk-ordered inverses
        if (!G.minvc.p) throw ApiError(DDPCA_ESTATE, "colour SSOR needs a reduced-precision V-cycle copy (precond_fp32 >= 1)");
        a.minv = F.minv32.p;
        if (G.val8.p) a.val = G.val8.p, launch_gs_ssor_t<PH, DOT, uint8_t>(a, c16, D.stream);
        else if (G.val16.p) a.val = G.val16.p, launch_gs_ssor_t<PH, DOT, uint16_t>(a, c16, D.stream);
        else a.val = G.val32.p, launch_gs_ssor_t<PH, DOT, float>(a, c16, D.stream);
        return;
    }
    if (G.val8.p) {
        a.val = G.val8.p;
        a.minv = F.minv32.p;
        if constexpr (PH >= 3) launch_gs_aux_t<PH, uint8_t>(a, c16, D.stream);
        else launch_gs_t<PH, DOT, uint8_t>(a, c16, D.stream);
    } else if (G.val16.p) {
        a.val = G.val16.p;
        a.minv = F.minv32.p;
        if constexpr (PH >= 3) launch_gs_aux_t<PH, uint16_t>(a, c16, D.stream);
        else launch_gs_t<PH, DOT, uint16_t>(a, c16, D.stream);
    } else if (G.val32.p) {
        a.val = G.val32.p;
        a.minv = F.minv32.p;
        if constexpr (PH >= 3) launch_gs_aux_t<PH, float>(a, c16, D.stream);
        else launch_gs_t<PH, DOT, float>(a, c16, D.stream);
    } else {
        a.val = G.val64.p;
        a.minv = F.minv.p;
        if constexpr (PH >= 3) launch_gs_aux_t<PH, double>(a, c16, D.stream);
        else launch_gs_t<PH, DOT, double>(a, c16, D.stream);
    }
}
}  // namespace

void MgpisDevice::vcycle(const double* rin, double* zout, bool dot) {
    if (no_coarse) throw ApiError(DDPCA_ESTATE, "one-level handle without a coarse inverse: diagonal preconditioner only");
    const int nlev = (int)lev.size();
    const int Lf = nlev - 1;
    const bool bj = opt.smoother >= 1;
    const bool cheb = opt.smoother == 2;
    const int nu = opt.nu;
    const PcgScal* scp = sc_cur_ ? sc_cur_ : sc.p;
    const int cl = clev;  // the exact dense solve; levels below it are not visited
    if (Lf == cl) {
        if (ainv32.p) hipLaunchKernelGGL(k_coarse<float>, dim3(ceil_div(3 * lev[cl].nn, 4)), dim3(kBlock), 0, stream, ainv32.p, aoff.p, c_noff.p,
                           c_n.p, c_ld.p, rin, zout, 3 * lev[cl].nn, lev[cl].csub.p, scp);
        else hipLaunchKernelGGL(k_coarse<double>, dim3(ceil_div(3 * lev[cl].nn, 4)), dim3(kBlock), 0, stream, ainv.p, aoff.p, c_noff.p,
                           c_n.p, c_ld.p, rin, zout, 3 * lev[cl].nn, lev[cl].csub.p, scp);
        if (dot)
            hipLaunchKernelGGL(k_dot, dim3(ceil_div(lev[cl].nn, kBlock)), dim3(kBlock), 0, stream, rin, zout, partial.p,
                               lev[cl].nn, lev[cl].csub.p, scp);
        return;
    }
    std::vector<double*> cur(nlev), oth(nlev);
    for (int l = 0; l < nlev; ++l) { cur[l] = lev[l].x.p; oth[l] = lev[l].t.p; }
    cur[Lf] = lev[Lf].t.p;
    oth[Lf] = zout;
    // block-Jacobi levels with fp32 iterate copies (LevelDev::x4a / x4b, precond_fp32 = 4): their
    // first sweep, the sweeps and the prolongation into them write the copy, the sweeps and the
    // residual gather it, and only the level's last sweep writes its fp64 iterate
    std::vector<float4*> cur4(nlev, nullptr), oth4(nlev, nullptr);
    for (int l = 0; l < nlev; ++l)
        if (lev[l].x4a.p) {
            cur4[l] = reinterpret_cast<float4*>(lev[l].x4a.p);
            oth4[l] = reinterpret_cast<float4*>(lev[l].x4b.p);
        }
    auto bvec = [&](int l) -> const double* { return l == Lf ? rin : lev[l].b.p; };
    auto coef = [&](int l, int sweep) { return lev[l].coef.p + 2 * (int64_t)sweep * nsub; };
    // smoothing sweeps on level l from the current iterate (first: jac0/restrict already did sweep 0);
    // out64: the last of them is the level's output (fp64 also on an fp32-copy level)
    auto smooth = [&](int l, int first, int count, bool last_dot, bool out64) {
        const int f32 = vc_type(l);
        for (int s = first; s < first + count; ++s) {
            SellArgs a = vc_level_args(*this, l);
            a.sc = scp;
            a.partial = partial.p;
            a.x = cur[l];
            a.b = bvec(l);
            a.xo = oth[l];
            a.coef = coef(l, s);
            if (cur4[l]) {
                const bool fin = out64 && s == first + count - 1;
                a.x4 = cur4[l];
                a.xo4 = fin ? nullptr : oth4[l];
                a.xo = fin ? oth[l] : nullptr;
            }
            const bool d = last_dot && s == first + count - 1;
            if (cheb) {
                a.p = lev[l].d.p;
                if (d) launch_sell<kCheb, true, true>(f32, a, stream);
                else launch_sell<kCheb, true, false>(f32, a, stream);
            } else if (bj) {
                if (d) launch_sell<kJac, true, true>(f32, a, stream);
                else launch_sell<kJac, true, false>(f32, a, stream);
            } else {
                if (d) launch_sell<kJac, false, true>(f32, a, stream);
                else launch_sell<kJac, false, false>(f32, a, stream);
            }
            std::swap(cur[l], oth[l]);
            std::swap(cur4[l], oth4[l]);
        }
    };
    const bool gsf = gs_fine();
    if (gsf) cur[Lf] = zout;  // the Gauss-Seidel sweeps run in place
    // ---- descend
    const bool ssor = gsf && opt.smoother == 4;
    if (ssor) {
        // colour SSOR: forward sweep from zero, backward sweep, residual r = w - L x
        for (int k = 0; k < gs.ncol; ++k) launch_gs<6, false>(*this, k, zout, rin, nullptr, scp, nullptr);
        for (int k = gs.ncol - 1; k >= 0; --k) launch_gs<7, false>(*this, k, zout, rin, nullptr, scp, nullptr);
        launch_gs<8, false>(*this, -1, zout, rin, lev[Lf].r.p, scp, nullptr);
    } else if (gsf) {
        // forward sweep from zero, colour by colour, then r = -U x in one launch; band mode: the
        // rows outside the colours start at x = 0, r = b, the ring's r = b - K x after the sweep
        if (gs.band) launch_gs<5, false>(*this, -3, zout, rin, lev[Lf].r.p, scp, nullptr);
        for (int k = 0; k < gs.ncol; ++k) launch_gs<0, false>(*this, k, zout, rin, nullptr, scp, nullptr);
        launch_gs<1, false>(*this, -1, zout, nullptr, lev[Lf].r.p, scp, nullptr);
        if (gs.band) launch_gs<3, false>(*this, -2, zout, rin, lev[Lf].r.p, scp, nullptr);
    } else {
        const LevelDev& F = lev[Lf];
        const int grid = ceil_div(F.nn, kBlock);
        if (vc_type(Lf) != kVal64) {
            const float* m = F.minv32.p;
            if (cheb) hipLaunchKernelGGL((k_jac0<true, true, float>), dim3(grid), dim3(kBlock), 0, stream, rin, m, coef(Lf, 0), cur[Lf], F.d.p, F.nn, F.csub.p, scp, cur4[Lf]);
            else if (bj) hipLaunchKernelGGL((k_jac0<true, false, float>), dim3(grid), dim3(kBlock), 0, stream, rin, m, coef(Lf, 0), cur[Lf], nullptr, F.nn, F.csub.p, scp, cur4[Lf]);
            else hipLaunchKernelGGL((k_jac0<false, false, float>), dim3(grid), dim3(kBlock), 0, stream, rin, m, coef(Lf, 0), cur[Lf], nullptr, F.nn, F.csub.p, scp, cur4[Lf]);
        } else if (cheb) hipLaunchKernelGGL((k_jac0<true, true>), dim3(grid), dim3(kBlock), 0, stream, rin, F.minv.p, coef(Lf, 0), cur[Lf], F.d.p, F.nn, F.csub.p, scp, cur4[Lf]);
        else if (bj) hipLaunchKernelGGL((k_jac0<true, false>), dim3(grid), dim3(kBlock), 0, stream, rin, F.minv.p, coef(Lf, 0), cur[Lf], nullptr, F.nn, F.csub.p, scp, cur4[Lf]);
        else hipLaunchKernelGGL((k_jac0<false, false>), dim3(grid), dim3(kBlock), 0, stream, rin, F.minv.p, coef(Lf, 0), cur[Lf], nullptr, F.nn, F.csub.p, scp, cur4[Lf]);
    }
    for (int l = Lf; l >= cl + 1; --l) {
        if (!(gsf && l == Lf)) {
            smooth(l, 1, nu - 1, false, false);
            SellArgs a = vc_level_args(*this, l);
            a.sc = scp;
            a.x = cur[l];
            a.x4 = cur4[l];
            a.b = bvec(l);
            a.y = lev[l].r.p;
            launch_sell<kResid, false, false>(vc_type(l), a, stream);
        }
        const int c = l - 1;
        const LevelDev& F = lev[l];
        const LevelDev& C = lev[c];
        const int grid = ceil_div(C.nn, kBlock);
        const double* cf = c > 0 ? coef(c, 0) : nullptr;
        if (F.nrot) {
            // block transfer entries: plain restriction, the blocks' B^T part, then the first
            // coarse sweep x_c = omega M b_c that k_restrict otherwise fuses
            launch_restrict<false, false, false, double>(F, grid, stream, F.r.p, C.mask.p, C.b.p, nullptr, nullptr, nullptr, nullptr, C.nn, C.csub.p, scp);
            rot_restrict(l, F.r.p, C.b.p, scp);
            if (c != cl) {
                const bool f32c = vc_type(c) != kVal64;
                const float* m32 = C.minv32.p;
                if (cheb && f32c) hipLaunchKernelGGL((k_jac0<true, true, float>), dim3(grid), dim3(kBlock), 0, stream, C.b.p, m32, cf, cur[c], C.d.p, C.nn, C.csub.p, scp, cur4[c]);
                else if (bj && f32c) hipLaunchKernelGGL((k_jac0<true, false, float>), dim3(grid), dim3(kBlock), 0, stream, C.b.p, m32, cf, cur[c], nullptr, C.nn, C.csub.p, scp, cur4[c]);
                else if (f32c) hipLaunchKernelGGL((k_jac0<false, false, float>), dim3(grid), dim3(kBlock), 0, stream, C.b.p, m32, cf, cur[c], nullptr, C.nn, C.csub.p, scp, cur4[c]);
                else if (cheb) hipLaunchKernelGGL((k_jac0<true, true>), dim3(grid), dim3(kBlock), 0, stream, C.b.p, C.minv.p, cf, cur[c], C.d.p, C.nn, C.csub.p, scp, cur4[c]);
                else if (bj) hipLaunchKernelGGL((k_jac0<true, false>), dim3(grid), dim3(kBlock), 0, stream, C.b.p, C.minv.p, cf, cur[c], nullptr, C.nn, C.csub.p, scp, cur4[c]);
                else hipLaunchKernelGGL((k_jac0<false, false>), dim3(grid), dim3(kBlock), 0, stream, C.b.p, C.minv.p, cf, cur[c], nullptr, C.nn, C.csub.p, scp, cur4[c]);
            }
        } else {
            // x4 mode: the colour sweeps' residual is the fp32 copy (GsFine::r4)
            const float4* rf4 = gsf && l == Lf && gs.r4.p ? reinterpret_cast<const float4*>(gs.r4.p) : nullptr;
            if (c == cl)
                launch_restrict<false, false, false, double>(F, grid, stream, F.r.p, C.mask.p, C.b.p, nullptr, nullptr, nullptr, nullptr, C.nn, C.csub.p, scp, rf4);
            else if (vc_type(c) != kVal64) {
                const float* m = C.minv32.p;
                if (cheb)
                    launch_restrict<true, true, true, float>(F, grid, stream, F.r.p, C.mask.p, C.b.p, cur[c], C.d.p, m, cf, C.nn, C.csub.p, scp, rf4, cur4[c]);
                else if (bj)
                    launch_restrict<true, true, false, float>(F, grid, stream, F.r.p, C.mask.p, C.b.p, cur[c], nullptr, m, cf, C.nn, C.csub.p, scp, rf4, cur4[c]);
                else
                    launch_restrict<true, false, false, float>(F, grid, stream, F.r.p, C.mask.p, C.b.p, cur[c], nullptr, m, cf, C.nn, C.csub.p, scp, rf4, cur4[c]);
            } else if (cheb)
                launch_restrict<true, true, true, double>(F, grid, stream, F.r.p, C.mask.p, C.b.p, cur[c], C.d.p, C.minv.p, cf, C.nn, C.csub.p, scp, rf4, cur4[c]);
            else if (bj)
                launch_restrict<true, true, false, double>(F, grid, stream, F.r.p, C.mask.p, C.b.p, cur[c], nullptr, C.minv.p, cf, C.nn, C.csub.p, scp, rf4, cur4[c]);
            else
                launch_restrict<true, false, false, double>(F, grid, stream, F.r.p, C.mask.p, C.b.p, cur[c], nullptr, C.minv.p, cf, C.nn, C.csub.p, scp, rf4, cur4[c]);
        }
    }
    if (ainv32.p) hipLaunchKernelGGL(k_coarse<float>, dim3(ceil_div(3 * lev[cl].nn, 4)), dim3(kBlock), 0, stream, ainv32.p, aoff.p, c_noff.p,
                           c_n.p, c_ld.p, lev[cl].b.p, cur[cl], 3 * lev[cl].nn, lev[cl].csub.p, scp);
        else hipLaunchKernelGGL(k_coarse<double>, dim3(ceil_div(3 * lev[cl].nn, 4)), dim3(kBlock), 0, stream, ainv.p, aoff.p, c_noff.p,
                       c_n.p, c_ld.p, lev[cl].b.p, cur[cl], 3 * lev[cl].nn, lev[cl].csub.p, scp);
    // ---- ascend
    for (int l = cl + 1; l <= Lf; ++l) {
        const LevelDev& F = lev[l];
        if (gsf && l == Lf && gs.x4.p)  // (x4 mode: lattice fine transfer, no block entries, GsFine::x4)
            hipLaunchKernelGGL(k_prolong_lat_x4, dim3(ceil_div(F.nn, kBlock)), dim3(kBlock), 0, stream, cur[l - 1], F.ppk.p,
                               F.pstr.p, F.mask.p, reinterpret_cast<float4*>(gs.x4.p), F.nn, F.csub.p, scp);
        else if (cur4[l] && F.lat)  // a block-Jacobi level's fp32 copy (no block entries into it)
            hipLaunchKernelGGL(k_prolong_lat_x4, dim3(ceil_div(F.nn, kBlock)), dim3(kBlock), 0, stream, cur[l - 1], F.ppk.p,
                               F.pstr.p, F.mask.p, cur4[l], F.nn, F.csub.p, scp);
        else if (cur4[l] && F.uw) hipLaunchKernelGGL(k_prolong_x4<true>, dim3(ceil_div(F.nn, kBlock)), dim3(kBlock), 0, stream, cur[l - 1],
                                                F.ppar.p, F.pw.p, F.mask.p, cur4[l], F.nn, F.csub.p, scp);
        else if (cur4[l]) hipLaunchKernelGGL(k_prolong_x4<false>, dim3(ceil_div(F.nn, kBlock)), dim3(kBlock), 0, stream, cur[l - 1],
                                        F.ppar.p, F.pw.p, F.mask.p, cur4[l], F.nn, F.csub.p, scp);
        else if (F.lat) hipLaunchKernelGGL(k_prolong_lat, dim3(ceil_div(F.nn, kBlock)), dim3(kBlock), 0, stream, cur[l - 1], F.ppk.p,
                                      F.pstr.p, F.mask.p, cur[l], F.nn, F.csub.p, scp);
        else if (F.uw) hipLaunchKernelGGL(k_prolong<true>, dim3(ceil_div(F.nn, kBlock)), dim3(kBlock), 0, stream, cur[l - 1], F.ppar.p, F.pw.p,
                           F.mask.p, cur[l], F.nn, F.csub.p, scp);
        else hipLaunchKernelGGL(k_prolong<false>, dim3(ceil_div(F.nn, kBlock)), dim3(kBlock), 0, stream, cur[l - 1], F.ppar.p, F.pw.p,
                           F.mask.p, cur[l], F.nn, F.csub.p, scp);
        rot_prolong(l, cur[l - 1], cur[l], scp, cur4[l]);
        if (ssor && l == Lf) {
            // colour SSOR after the coarse correction: forward, then backward with the dot partials
            for (int k = 0; k < gs.ncol; ++k) launch_gs<9, false>(*this, k, zout, rin, nullptr, scp, nullptr);
            for (int k = gs.ncol - 1; k >= 0; --k) {
                if (dot) launch_gs<10, true>(*this, k, zout, rin, nullptr, scp, gs.partial.p);
                else launch_gs<10, false>(*this, k, zout, rin, nullptr, scp, nullptr);
            }
            continue;
        }
        if (gsf && l == Lf) {
            // backward sweep; the dot product's partials per colour chunk (vc_cb)
            for (int k = gs.ncol - 1; k >= 0; --k) {
                if (dot) launch_gs<2, true>(*this, k, zout, rin, nullptr, scp, gs.partial.p);
                else launch_gs<2, false>(*this, k, zout, rin, nullptr, scp, nullptr);
            }
            // band mode: the dot product's partials of the rows outside the colours
            if (dot && gs.band) launch_gs<4, false>(*this, -3, zout, rin, nullptr, scp, gs.partial.p);
            continue;
        }
        // post-smoothing restarts the smoother (Chebyshev recurrence) from the prolongated iterate
        smooth(l, 0, nu, dot && l == Lf, true);
    }
    if (cur[Lf] != zout) throw ApiError(DDPCA_ESTATE, "V-cycle buffer parity");
}

double MgpisDevice::fine_matrix_bytes(int s, int vt, bool prod_cols) const {
    // operator bytes one fine-level pass reads for member s: streamed values = 4 B index + 72 B
    // (fp64), 36 B (fp32), 20 B (block-exponent fp16) or 10 B (block-scaled int8) per stored block; table mode = 4 B index per block +
    // 4 B row type per node + the member's share of the table (read once per launch)
    const LevelDev& L = lev.back();
    // (the production kernels read 2-B column offsets where the level has them, prod_cols)
    const double cb = (prod_cols && L.col16.p) ? 2.0 : 4.0;
    if (!L.tbl) return (cb + vbytes(vt)) * (double)L.nnzb_sub[s];
    double nodes = 0.0;
    for (int64_t n : L.nloc) nodes += (double)n;
    return 4.0 * (double)L.nnzb_sub[s] + 4.0 * (double)L.nloc[s] +
           (double)L.ntypes * (double)L.tstride * 8.0 * (double)L.nloc[s] / nodes;
}

double MgpisDevice::fine_kernel_bytes(int s) const {
    // algorithmic bytes of one fine-level k_sell<kPcg> for member s: the operator + z gathered
    // once (24 B/node) + p, q read and written (4 x 24 B/node)
    return fine_matrix_bytes(s, kVal64) + 24.0 * 5.0 * (double)lev.back().nloc[s];
}

// ---- algorithmic byte model of the solve path (per member s; bytes every kernel must move at
// least once: streamed operator values + column indices, each vector read / written once, a
// gathered vector counted once per element).  The launch sequence is the one vcycle() and
// enqueue_iteration() issue; the sizes are the member's real (unpadded) nodes.

void MgpisDevice::vcycle_bytes(int s, double out[2]) const {
    out[0] = out[1] = 0.0;
    const int nlev = (int)lev.size(), Lf = nlev - 1, cl = clev;
    const bool bj = opt.smoother >= 1, cheb = opt.smoother == 2;
    auto n = [&](int l) { return (double)lev[l].nloc[s]; };
    auto mat = [&](int l) {  // one pass over the V-cycle's copy of level l
        const LevelDev& L = lev[l];
        if (L.tbl) return 4.0 * (double)L.nnzb_sub[s] + 4.0 * n(l);
        const double cb = L.col16.p ? 2.0 : 4.0;
        return (vbytes(vc_type(l)) + cb) * (double)L.nnzb_sub[s];
    };
    auto minv = [&](int l) { return (bj ? 9.0 : 3.0) * (vc_type(l) != kVal64 ? 4.0 : 8.0); };
    auto put = [&](int l, double b) { out[l == Lf ? 0 : 1] += b; };
    // x' = x + w M (b - K x): operator, x gathered, b, M^-1, x' (Chebyshev: d read + written); on a
    // level with fp32 iterate copies x is gathered in 16 B and x' written in 16 B, in fp64 by the
    // level's last sweep (fin)
    auto x4 = [&](int l) { return lev[l].x4a.p != nullptr; };
    auto sweep = [&](int l, bool fin = true) {
        if (x4(l)) return mat(l) + n(l) * (16.0 + 24.0 + (fin ? 24.0 : 16.0) + minv(l));
        return mat(l) + n(l) * (24.0 * 3 + minv(l) + (cheb ? 48.0 : 0.0));
    };
    const double n0 = 3.0 * (double)lev[cl].nloc[s];
    const double coarse = (ainv32.p ? 4.0 : 8.0) * n0 * n0 + 16.0 * n0;  // dense inverse + b in, x out
    if (Lf == cl) {
        out[0] += coarse + 16.0 * n0;  // + the dot product's second read
        return;
    }
    const bool gsf = gs_fine();
    // multicolour sweeps on the fine level: L + U = the off-diagonal blocks, read once by the
    // forward sweep + residual pair and once by the backward sweep; per launch the x entries of
    // the colours it reads (forward colour k: the k earlier ones, residual: the later ones,
    // backward: all others), and per row b, M^-1, the row index and x (or r) written
    const double K = gsf ? (double)gs.ncol : 0.0;
    const double gsvb = gsf ? vbytes(vc_type(Lf)) + (gs.col16.p ? 2.0 : 4.0) : 0.0;
    const double gsmat = gsvb * (gsf ? (double)gs.nnzb_sub[s] : 0.0);
    // rows the colours sweep (all of them unless band mode), and band mode's ring and far rows
    const double nsw = gsf && gs.band ? (double)gs.band_rows_sub[s] : n(Lf);
    const double nring = gsf && gs.band ? (double)gs.ring_rows_sub[s] : 0.0;
    const double nout = gsf && gs.band ? nring + (double)gs.far_rows_sub[s] : 0.0;
    // x4 mode (GsFine::x4): the iterate the sweeps gather and the forward sweep / prolongation
    // write is the 16-B fp32 copy; the backward sweep writes it and the fp64 output
    const double xb = gsf && gs.x4.p ? 16.0 : 24.0;
    const double rb = gsf && gs.r4.p ? 16.0 : 24.0;  // the residual written by the sweeps, read by the restriction
    const bool ssor = gsf && opt.smoother == 4;
    if (ssor) {
        // colour SSOR: forward from zero (L; b, M^-1, x, w written), backward (U; b, w, M^-1 read, x
        // written), residual (L; w read, r written); x entries gathered as the Gauss-Seidel pair's
        const double lpass = gsmat * 0.5, upass = gsmat * 0.5, row = 4.0;
        put(Lf, lpass + nsw * (24.0 + minv(Lf) + xb + 24.0 + row + xb * (K - 1.0) / 2.0));
        put(Lf, upass + nsw * (48.0 + minv(Lf) + xb + row + xb * (K - 1.0) / 2.0));
        put(Lf, lpass + nsw * (24.0 + rb + row + xb * (K - 1.0) / 2.0));
    } else if (gsf) {
        put(Lf, 76.0 * nout);  // band mode: x = 0, r = b outside the colours (b read, x, r written, row index)
        put(Lf, gsmat + nsw * (24.0 + minv(Lf) + xb + 4.0 + xb * (K - 1.0) / 2.0));  // forward
        put(Lf, nsw * (rb + 4.0 + xb * (K - 1.0) / 2.0));                            // residual
        // band mode: the ring's residual over its band columns (blocks, b read, r written, x gathered)
        put(Lf, gsvb * (double)(gs.band ? gs.ring_nnzb_sub[s] : 0) + nring * (24.0 + 24.0 + 4.0 + 24.0));
    } else {
        put(Lf, n(Lf) * ((x4(Lf) ? 40.0 : 48.0) + minv(Lf) + (cheb ? 24.0 : 0.0)));  // k_jac0: b in, x out
    }
    for (int l = Lf; l >= cl + 1; --l) {
        if (!(gsf && l == Lf)) {
            for (int k = 1; k < opt.nu; ++k) put(l, sweep(l, false));
            put(l, mat(l) + (x4(l) ? 64.0 : 72.0) * n(l));  // residual: x gathered, b, r
        }
        const LevelDev& F = lev[l];
        const int c = l - 1;
        const bool init = c != cl;
        // coarse node: mask + b_c written (+ x_c = w M b_c: M^-1 read, x_c written; Chebyshev d_c)
        double cn = 1.0 + 24.0 + (init ? minv(c) + (x4(c) ? 16.0 : 24.0) + (cheb ? 24.0 : 0.0) : 0.0);
        double tr = (gsf && l == Lf ? rb : 24.0) * n(l);  // r_f read once
        if (F.lat) cn += 8.0;     // 27-bit child mask + fine copy
        else tr += 12.0 * (double)F.tent_sub[s];  // child index + weight per stencil entry
        tr += 4.0 * 8.0 * (double)F.tblk_sub[s] + (F.tblk_sub[s] ? 24.0 * n(c) : 0.0);  // block entries (B^T r_f)
        put(l, tr + cn * n(c));
    }
    put(cl, coarse);
    for (int l = cl + 1; l <= Lf; ++l) {
        const LevelDev& F = lev[l];
        // x_f += mask P e_c: e_c read once, mask, x_f read + written, the parent encoding
        double pb = 24.0 * n(l - 1) + n(l) * (1.0 + (gsf && l == Lf ? 2.0 * xb : x4(l) ? 32.0 : 48.0));
        if (F.lat) pb += 4.0 * n(l);
        else pb += (F.uw ? 4.0 : 12.0) * (double)F.tent_sub[s];
        pb += 4.0 * 8.0 * (double)F.tblk_sub[s];
        put(l, pb);
        if (ssor && l == Lf) {
            // forward from the prolongated x (L + U; b, M^-1 read, x, w written), backward (U; b, w,
            // M^-1 read, z written)
            put(l, gsmat + nsw * (24.0 + minv(l) + xb + 24.0 + 4.0 + xb * (K - 1.0)));
            put(l, gsmat * 0.5 + nsw * (48.0 + minv(l) + 24.0 + 4.0 + xb * (K - 1.0) / 2.0));
            continue;
        }
        if (gsf && l == Lf) {
            put(l, gsmat + nsw * (24.0 + minv(l) + 24.0 + (xb < 24.0 ? xb : 0.0) + 4.0 + xb * (K - 1.0)));  // backward
            put(l, 52.0 * nout);  // band mode: b . x of the rows outside the colours (b, x read, row index)
            continue;
        }
        for (int k = 0; k < opt.nu; ++k) put(l, sweep(l, k == opt.nu - 1));
    }
}

void MgpisDevice::iteration_bytes(int s, double out[2]) const {
    vcycle_bytes(s, out);
    const LevelDev& F = lev.back();
    const double n = (double)F.nloc[s], nch = (double)pad64(F.nloc[s]) / kChunk;
    out[0] += fine_kernel_bytes(s) + 144.0 * n;  // k_sell<kPcg> + k_axpy (x, r read + written, p, q read)
    out[1] += 3.0 * 8.0 * nch;                   // three k_fin passes over the chunk partials
}

void MgpisDevice::setup_bytes(int s, double out[2]) const {
    vcycle_bytes(s, out);
    const LevelDev& F = lev.back();
    const double n = (double)F.nloc[s], nch = (double)pad64(F.nloc[s]) / kChunk;
    out[0] += 120.0 * n;  // k_pcg_init: b read, x r p q written
    out[1] += 2.0 * 8.0 * nch;
}

int64_t MgpisDevice::iteration_launches() const {
    // k_sell<kPcg>, k_axpy, 3 x k_fin, and the V-cycle: jac0 + per descended level (nu - 1 sweeps,
    // residual, restriction) + coarse + per ascended level (prolongation, nu sweeps); the
    // multicolour fine level: one forward and one backward launch per colour + the residual in
    // place of jac0, nu - 1 + 1 + nu sweep launches
    const int64_t nd = (int64_t)lev.size() - 1 - clev;
    const int64_t base = 5 + (nd == 0 ? 2 : 1 + nd * (opt.nu + 1) + 1 + nd * (1 + opt.nu));
    // (band mode: + the x = 0 / r = b launch, the ring's residual and the dot of the other rows)
    if (gs_fine() && nd > 0 && opt.smoother == 4) return base - 1 - 2 * opt.nu + 4 * gs.ncol + 1;  // colour SSOR
    return gs_fine() && nd > 0 ? base - 1 - 2 * opt.nu + 2 * gs.ncol + 1 + (gs.band ? 3 : 0) : base;
}

// k_fin over every member
void MgpisDevice::launch_fin(hipStream_t st, int what, const double* part, const double* part2, const int64_t* cb,
                             PcgScal* scp, PcgMirror* mir) {
    hipLaunchKernelGGL(k_fin, dim3(nsub), dim3(kFinT), 0, st, what, part, part2, cb, scp, mir);
}

void MgpisDevice::enqueue_iteration(int prec, bool timed) {
    LevelDev& L = lev.back();
    PcgScal* scp = sc_cur_ ? sc_cur_ : sc.p;
    SellArgs a = level_args(L);
    a.x = zs.p;
    a.y = qs.p;
    a.p = ps.p;
    a.sc = scp;
    a.partial = partial.p;
    const int nblk = ceil_div(L.nn, kBlock);
    if (timed) DDPCA_HIP(hipEventRecord(ev_k0, stream));
    launch_sell<kPcg, false, true>(kVal64, a, stream);
    if (timed) DDPCA_HIP(hipEventRecord(ev_k1, stream));
    launch_fin(stream, (int)kFinAlpha, partial.p, nullptr, fin_cb.p, scp, mirror.dev);
    hipLaunchKernelGGL(k_axpy, dim3(nblk), dim3(kBlock), 0, stream, xs.p, rs.p, ps.p, qs.p, scp, partial.p, L.nn, L.csub.p);
    launch_fin(stream, (int)kFinRR, partial.p, nullptr, fin_cb.p, scp, mirror.dev);
    if (prec == 1) vcycle(rs.p, zs.p, true);
    else hipLaunchKernelGGL(k_diag, dim3(nblk), dim3(kBlock), 0, stream, rs.p, L.dinv.p, zs.p, partial.p, L.nn, L.csub.p, scp);
    launch_fin(stream, (int)kFinBeta, prec == 1 ? vc_partial() : partial.p, nullptr, prec == 1 ? vc_cb() : fin_cb.p, scp,
               mirror.dev);
}

// graph_[prec]: iters_per_graph PCG iterations captured once and replayed; graph1_[prec]: one.
hipGraphExec_t MgpisDevice::capture_iterations(int prec, int count, PcgScal* scp) {
    sc_cur_ = scp;
    hipGraph_t g;
    hipGraphExec_t ge = nullptr;
    CaptureSection capture_section;  // device_common.hpp CaptureLock
    DDPCA_HIP(hipStreamBeginCapture(stream, hipStreamCaptureModeThreadLocal));
    for (int k = 0; k < count; ++k) enqueue_iteration(prec, false);
    DDPCA_HIP(hipStreamEndCapture(stream, &g));
    sc_cur_ = nullptr;
    DDPCA_HIP(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    DDPCA_HIP(hipGraphDestroy(g));
    return ge;
}

void MgpisDevice::build_graph(int prec) {
    if (split_) {
        for (int h = 0; h < nparts_; ++h) build_half_graph(prec, h);
        return;
    }
    if (graph_[prec]) return;
    graph_[prec] = capture_iterations(prec, opt.iters_per_graph, nullptr);
    if (opt.iters_per_graph > 1) graph1_[prec] = capture_iterations(prec, 1, nullptr);
}

// the same iterations bound to half h's copy of the scalars (captured on `stream`, replayed on
// the half's own stream)
void MgpisDevice::build_half_graph(int prec, int h) {
    if (graph_h_[prec][h]) return;
    graph_h_[prec][h] = capture_iterations(prec, opt.iters_per_graph, sc_half_.p + (int64_t)h * nsub);
    if (opt.iters_per_graph > 1) graph1_h_[prec][h] = capture_iterations(prec, 1, sc_half_.p + (int64_t)h * nsub);
}

int64_t MgpisDevice::horizon(int prec, int half) const {
    // DDPCA_TAIL_PACING=0: whole replays to the end (A/B)
    const char* e = std::getenv("DDPCA_TAIL_PACING");
    if ((e && std::atoi(e) == 0) || (int)expect_[prec].size() != nsub) return INT64_MAX;
    int64_t h = 0;
    for (int s = 0; s < nsub; ++s) {
        if (half >= 0 && half_host_[s] != half) continue;
        if (expect_[prec][s] <= 0) return INT64_MAX;
        h = std::max(h, expect_[prec][s]);
    }
    return h;
}

// scs[h][s] = sc[s], with done forced on the members of the other parts
__global__ void k_split_sc(const PcgScal* sc, PcgScal* scs, const int32_t* half, int nsub, int np) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= nsub) return;
    for (int h = 0; h < np; ++h) {
        PcgScal v = sc[s];
        if (half[s] != h) v.done = 1;
        scs[h * nsub + s] = v;
    }
}

// sc[s] = the copy of the half that ran member s
__global__ void k_merge_sc(PcgScal* sc, const PcgScal* scs, const int32_t* half, int nsub) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s < nsub) sc[s] = scs[half[s] * nsub + s];
}

void MgpisDevice::set_split(bool on, int parts) {
    select_device(device);
    if (on && (parts < 2 || parts > kMaxParts)) throw ApiError(DDPCA_EINVAL, "set_split: 2 .. 4 parts");
    parts = std::min<int>(parts, (int)nsub);
    on = on && nsub >= 2 && !no_coarse;
    if (on == split_ && (!on || parts == nparts_)) return;
    if (split_ && on) throw ApiError(DDPCA_ESTATE, "set_split: the part count is fixed once split");
    DDPCA_HIP(hipStreamSynchronize(stream));
    if (on && !xstream_[0]) {
        nparts_ = parts;
        for (int h = 0; h + 1 < parts; ++h) {
            DDPCA_HIP(hipStreamCreateWithFlags(&xstream_[h], hipStreamNonBlocking));
            DDPCA_HIP(hipEventCreateWithFlags(&ev_join_[h], hipEventDisableTiming));
        }
        DDPCA_HIP(hipEventCreateWithFlags(&ev_fork_, hipEventDisableTiming));
        sc_half_.alloc((size_t)parts * nsub);
        // deal the members into parts of equal fine-level work (largest first, to the lightest
        // part; the lower part index on ties)
        std::vector<int> ord(nsub);
        for (int s = 0; s < nsub; ++s) ord[s] = s;
        std::stable_sort(ord.begin(), ord.end(), [&](int x, int y) { return lev.back().nnzb_sub[x] > lev.back().nnzb_sub[y]; });
        half_host_.assign(nsub, 0);
        double w[kMaxParts] = {0.0, 0.0, 0.0, 0.0};
        for (int s : ord) {
            int h = 0;
            for (int q = 1; q < parts; ++q)
                if (w[q] < w[h]) h = q;
            half_host_[s] = h;
            w[h] += (double)lev.back().nnzb_sub[s];
        }
        half_.upload(half_host_);
    }
    split_ = on;
}

// Host pacing of the parts' replays (pace_until_done per part, one loop): a part gets its next
// replay when its slowest member has entered the last one enqueued for it.
int64_t pace_parts(int np, hipStream_t* st, hipGraphExec_t* g, const MirrorBuf& m, const std::vector<int>& part, int64_t k,
                   int64_t launched0, hipGraphExec_t* g1, const int64_t* horizon) {
    constexpr int64_t kRunway = 2;
    if (np < 1 || np > kMaxParts) throw ApiError(DDPCA_EINVAL, "pace_parts: part count");
    int64_t launched[kMaxParts], replays = 0;
    for (int h = 0; h < np; ++h) launched[h] = launched0;
    for (int64_t spin = 0;; ++spin) {
        bool all = true;
        int64_t slowest[kMaxParts];
        bool busy[kMaxParts], tail[kMaxParts];
        for (int h = 0; h < np; ++h) slowest[h] = INT64_MAX, busy[h] = false;
        for (int s = 0; s < m.n; ++s) {
            if (__atomic_load_n(&m.host[s].done, __ATOMIC_ACQUIRE)) continue;
            all = false;
            busy[part[s]] = true;
            slowest[part[s]] = std::min<int64_t>(slowest[part[s]], __atomic_load_n(&m.host[s].iter, __ATOMIC_RELAXED));
        }
        if (all) return replays;
        bool launched_now = false;
        for (int h = 0; h < np; ++h) {
            tail[h] = g1 && horizon && g1[h] && launched[h] + k > horizon[h];
            if (busy[h] && (tail[h] ? launched[h] - slowest[h] <= kRunway : launched[h] - slowest[h] <= k)) {
                DDPCA_HIP(hipGraphLaunch(tail[h] ? g1[h] : g[h], st[h]));
                launched[h] += tail[h] ? 1 : k;
                ++replays;
                launched_now = true;
            }
        }
        if (launched_now) continue;
        if ((spin & 255) == 255) {
            for (int h = 0; h < np; ++h) {
                if (!busy[h]) continue;
                const hipError_t q = hipStreamQuery(st[h]);
                if (q == hipSuccess) {
                    // this part's stream drained: its mirror entries are final for what it ran
                    bool done_now = true;
                    for (int s = 0; s < m.n; ++s)
                        if (part[s] == h) done_now &= __atomic_load_n(&m.host[s].done, __ATOMIC_ACQUIRE) != 0;
                    if (!done_now) {
                        DDPCA_HIP(hipGraphLaunch(tail[h] ? g1[h] : g[h], st[h]));
                        launched[h] += tail[h] ? 1 : k;
                        ++replays;
                    }
                } else if (q != hipErrorNotReady) {
                    DDPCA_HIP(q);
                }
            }
        }
        std::this_thread::yield();
    }
}

void MgpisDevice::pcg_begin(int prec, double rtol, const std::vector<int64_t>& maxit, bool warm) {
    select_device(device);
    last_prec_ = prec;
    solve_accounted_ = prec != 1 || warm;  // the byte model covers the V-cycle PCG from x0 = 0
    if ((int)maxit.size() != nsub) throw ApiError(DDPCA_EINVAL, "maxit per subdomain");
    build_graph(prec);
    LevelDev& L = lev.back();
    // the previous solve on this stream has finished (pcg_finish synchronised), so the
    // host-side reset of the mirror and the staging buffer cannot race a kernel
    mirror.reset();
    for (int s = 0; s < nsub; ++s) {
        sc_host[s] = PcgScal{};
        sc_host[s].tol2 = rtol * rtol;
        sc_host[s].maxit = maxit[s];
    }
    DDPCA_HIP(hipMemcpyAsync(sc.p, sc_host, nsub * sizeof(PcgScal), hipMemcpyHostToDevice, stream));
    const int nblk = ceil_div(L.nn, kBlock);
    if (!warm) {
        hipLaunchKernelGGL(k_pcg_init, dim3(nblk), dim3(kBlock), 0, stream, bs.p, xs.p, rs.p, ps.p, qs.p, partial.p, L.nn);
        launch_fin(stream, (int)kFinInit, partial.p, nullptr, fin_cb.p, sc.p, mirror.dev);
    } else {
        double* partial2 = partial.p + L.nch;
        hipLaunchKernelGGL(k_pcg_init_warm, dim3(nblk), dim3(kBlock), 0, stream, bs.p, ps.p, qs.p, partial2, L.nn);
        SellArgs a = level_args(L);
        a.x = xs.p;
        a.b = bs.p;
        a.y = rs.p;
        a.partial = partial.p;
        launch_sell<kResid, false, true>(kVal64, a, stream);
        launch_fin(stream, (int)kFinInitWarm, partial.p, partial2, fin_cb.p, sc.p, mirror.dev);
    }
    if (prec == 1) vcycle(rs.p, zs.p, true);
    else hipLaunchKernelGGL(k_diag, dim3(nblk), dim3(kBlock), 0, stream, rs.p, L.dinv.p, zs.p, partial.p, L.nn, L.csub.p, sc.p);
    launch_fin(stream, (int)kFinBeta0, prec == 1 ? vc_partial() : partial.p, nullptr, prec == 1 ? vc_cb() : fin_cb.p, sc.p,
               mirror.dev);
    sample_pending_ = false;
    if (time_kernel) {
        // first iteration eagerly, with HIP events around its fine-level SpMV on this stream
        enqueue_iteration(prec, true);
        sample_pending_ = true;
    }
    if (split_) {
        // fork: each half continues on its own stream from its own copy of the scalars
        hipLaunchKernelGGL(k_split_sc, dim3(ceil_div(nsub, 64)), dim3(64), 0, stream, sc.p, sc_half_.p, half_.p, nsub,
                           nparts_);
        DDPCA_HIP(hipEventRecord(ev_fork_, stream));
        for (int h = 1; h < nparts_; ++h) DDPCA_HIP(hipStreamWaitEvent(part_stream(h), ev_fork_, 0));
    }
}

void MgpisDevice::pcg_step(int prec) {
    if (split_) {
        for (int h = 0; h < nparts_; ++h) DDPCA_HIP(hipGraphLaunch(graph_h_[prec][h], part_stream(h)));
        graphs_launched += nparts_;
        return;
    }
    DDPCA_HIP(hipGraphLaunch(graph_[prec], stream));
    ++graphs_launched;
}

void MgpisDevice::pcg_wait(int prec, int64_t pre_enqueued) {
    const int64_t k = opt.iters_per_graph;
    const int64_t launched = (sample_pending_ ? 1 : 0) + pre_enqueued * k;
    if (split_) {
        hipStream_t st[kMaxParts];
        int64_t hz[kMaxParts];
        for (int h = 0; h < nparts_; ++h) st[h] = part_stream(h), hz[h] = horizon(prec, h);
        graphs_launched += pace_parts(nparts_, st, graph_h_[prec], mirror, half_host_, k, launched, graph1_h_[prec], hz);
        // join: `stream` continues after the other parts' replays; the scalars merge back
        for (int h = 1; h < nparts_; ++h) {
            DDPCA_HIP(hipEventRecord(ev_join_[h - 1], part_stream(h)));
            DDPCA_HIP(hipStreamWaitEvent(stream, ev_join_[h - 1], 0));
        }
        hipLaunchKernelGGL(k_merge_sc, dim3(ceil_div(nsub, 64)), dim3(64), 0, stream, sc.p, sc_half_.p, half_.p, nsub);
        return;
    }
    graphs_launched += pace_until_done(stream, graph_[prec], mirror, k, launched, graph1_[prec], horizon(prec, -1));
}

void MgpisDevice::pcg_fetch() {
    DDPCA_HIP(hipMemcpyAsync(sc_host, sc.p, nsub * sizeof(PcgScal), hipMemcpyDeviceToHost, stream));
}

void MgpisDevice::pcg_finish() {
    pcg_fetch();
    DDPCA_HIP(hipStreamSynchronize(stream));
    pcg_check();
}

void MgpisDevice::pcg_check() {
    if (sample_pending_) {
        // the sampled launch did work only for members that ran an iteration (the others were
        // done at init, e.g. zero right-hand side, and their chunks exited at once)
        double bytes = 0.0;
        for (int s = 0; s < nsub; ++s)
            if (sc_host[s].iter >= 1) bytes += fine_kernel_bytes(s);
        float ms = 0.f;
        if (bytes > 0.0 && hipEventElapsedTime(&ms, ev_k0, ev_k1) == hipSuccess && ms > 0.f) {
            timed_kernel_ms += ms;
            timed_kernel_bytes += bytes;
            timed_kernel_samples += 1;
        }
        sample_pending_ = false;
    }
    for (int s = 0; s < nsub; ++s)
        if (sc_host[s].fail) throw ApiError(DDPCA_ENUMERIC, "PCG breakdown (non-finite or non-positive curvature) in batch member " + std::to_string(s));
    // this solve's iteration counts pace the next one's tail (pcg_wait)
    if (last_prec_ >= 0) {
        expect_[last_prec_].resize(nsub);
        for (int s = 0; s < nsub; ++s) expect_[last_prec_][s] = sc_host[s].iter;
        last_prec_ = -1;
    }
    if (!no_coarse && !solve_accounted_) {
        // algorithmic bytes of the solve that just finished: members done at initialisation moved
        // only k_pcg_init's share; the others ran iter SpMVs and iter V-cycles (the setup's
        // first one and iter - 1 more: the converging iteration skips its V-cycle)
        for (int s = 0; s < nsub; ++s) {
            const double n = (double)lev.back().nloc[s];
            if (sc_host[s].iter == 0) {
                alg_bytes[0] += 120.0 * n;
                continue;
            }
            double a[2], b[2];
            setup_bytes(s, a);
            iteration_bytes(s, b);
            double v[2];
            vcycle_bytes(s, v);
            const double it = (double)sc_host[s].iter;
            alg_bytes[0] += a[0] + it * b[0] - v[0];
            alg_bytes[1] += a[1] + it * b[1] - v[1];
        }
        int64_t itmax = 0;
        for (int s = 0; s < nsub; ++s) itmax = std::max<int64_t>(itmax, sc_host[s].iter);
        alg_bytes[2] += (double)(itmax * iteration_launches());
        solve_accounted_ = true;
    }
}

void MgpisDevice::pcg_solve(int prec, double rtol, const std::vector<int64_t>& maxit, bool warm) {
    pcg_begin(prec, rtol, maxit, warm);
    pcg_wait(prec, 0);
    pcg_finish();
}

void MgpisDevice::scatter_free(int s, const double* cond, double* full) {
    DDPCA_HIP(hipMemsetAsync(full + 3 * lev.back().noff[s], 0, 3 * pad64(lev.back().nloc[s]) * sizeof(double), stream));
    hipLaunchKernelGGL(k_scatter, dim3(ceil_div(nfree[s], kBlock)), dim3(kBlock), 0, stream, cond, free_dof[s].p, full, nfree[s]);
}

void MgpisDevice::gather_free(int s, const double* full, double* cond) {
    hipLaunchKernelGGL(k_gather, dim3(ceil_div(nfree[s], kBlock)), dim3(kBlock), 0, stream, full, free_dof[s].p, cond, nfree[s]);
}

}  // namespace ddpca
