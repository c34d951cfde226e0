// Same-process HBM ceiling for the roofline line ("also report a measured
// STREAM-copy ceiling"): a STREAM copy and a STREAM read over buffers far larger than the 256 MiB
// Infinity Cache, timed with HIP events on a stream of their own.  bench.py divides the roofline
// kernel's achieved GB/s by these to report the fraction of what THIS box streams, next to the
// fraction of the 8 TB/s spec peak.  No reference counterpart (measurement only).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <vector>

#include "../../include/ddpca_amd.h"
#include "../../include/ddpca_probe.h"
#include "../csrc/device_common.hpp"

using namespace ddpca;

namespace {

typedef double dbl2_t __attribute__((ext_vector_type(2)));

// y = x, 16 B per lane, grid-stride, four loads in flight per lane; non-temporal both ways
__global__ __launch_bounds__(256) void k_stream_copy(const dbl2_t* __restrict__ x, dbl2_t* __restrict__ y, int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + 3 * stride < n; i += 4 * stride) {
        const dbl2_t a = __builtin_nontemporal_load(x + i), b = __builtin_nontemporal_load(x + i + stride),
                     c = __builtin_nontemporal_load(x + i + 2 * stride), d = __builtin_nontemporal_load(x + i + 3 * stride);
        __builtin_nontemporal_store(a, y + i);
        __builtin_nontemporal_store(b, y + i + stride);
        __builtin_nontemporal_store(c, y + i + 2 * stride);
        __builtin_nontemporal_store(d, y + i + 3 * stride);
    }
    for (; i < n; i += stride) __builtin_nontemporal_store(__builtin_nontemporal_load(x + i), y + i);
}

// partial[block] = sum of x over the block's share: 16 B per lane, four loads in flight per lane
__global__ __launch_bounds__(256) void k_stream_read(const dbl2_t* __restrict__ x, int64_t n, double* partial) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    double s0 = 0.0, s1 = 0.0;
    for (; i + 3 * stride < n; i += 4 * stride) {
        const dbl2_t a = __builtin_nontemporal_load(x + i), b = __builtin_nontemporal_load(x + i + stride),
                     c = __builtin_nontemporal_load(x + i + 2 * stride), d = __builtin_nontemporal_load(x + i + 3 * stride);
        s0 += (a.x + a.y) + (b.x + b.y);
        s1 += (c.x + c.y) + (d.x + d.y);
    }
    for (; i < n; i += stride) {
        const dbl2_t a = __builtin_nontemporal_load(x + i);
        s0 += a.x + a.y;
    }
    double s = s0 + s1;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    __shared__ double w[4];
    if ((threadIdx.x & 63) == 0) w[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) partial[blockIdx.x] = (w[0] + w[1]) + (w[2] + w[3]);
}

__global__ void k_fill(dbl2_t* x, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) x[i] = dbl2_t{1.0, 2.0};
}

// ---- grid barrier against a graph kernel boundary (the persistent below-fine V-cycle question,
// DESIGN §8): `phases` dependent passes y = (x[i] + x[i + n/2 + 977]) / 2 over n doubles (every
// pass reads what other workgroups, on other XCDs, wrote in the previous one), either as one
// graph of `phases` launches or as one persistent launch with a grid barrier between passes.
__device__ __forceinline__ double phase_value(const double* x, int64_t i, int64_t n) {
    int64_t j = i + n / 2 + 977;
    if (j >= n) j -= n;
    if (j >= n) j -= n;
    return 0.5 * (x[i] + x[j]);
}

__global__ __launch_bounds__(256) void k_phase(const double* x, double* y, int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) y[i] = phase_value(x, i, n);
}

// Every working workgroup of the launch is resident (the caller launches at most one per CU, or
// with pin one per CU of one XCD); the wait is bounded, so a grid that is not all resident ends with
// err = 1 instead of hanging.  pin: only the workgroups with id % 8 == 0 work (the round-robin
// dispatch puts them on one XCD), the others exit at once.  Barrier: one monotonic counter (zeroed
// by the caller) -- every storing wave drains its stores, the workgroup's lane 0 releases at agent
// scope and adds, polls relaxed with s_sleep, then acquires at agent scope (the XCD's L2 is shared
// by co-located workgroups, their L1s are not: the acquire is needed either way).
__global__ __launch_bounds__(256) void k_phase_persistent(double* x, double* y, int64_t n, int phases, int active, int pin,
                                                          unsigned* count, int* err) {
    if (pin && (blockIdx.x & 7)) return;
    const int64_t wid = pin ? blockIdx.x >> 3 : blockIdx.x;
    const int64_t stride = (int64_t)active * blockDim.x;
    __shared__ int bad;
    if (threadIdx.x == 0) bad = 0;
    for (int p = 0; p < phases; ++p) {
        const double* src = (p & 1) ? y : x;
        double* dst = (p & 1) ? x : y;
        for (int64_t i = wid * blockDim.x + threadIdx.x; i < n; i += stride) dst[i] = phase_value(src, i, n);
        if (p + 1 == phases) break;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_fetch_add(count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned target = (unsigned)(p + 1) * (unsigned)active;
            int64_t spin = 0;
            while (__hip_atomic_load(count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
                if (++spin > (int64_t)1 << 24) {
                    bad = 1;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __syncthreads();
        if (bad) {
            if (threadIdx.x == 0) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return;
        }
    }
}

}  // namespace

extern "C" int ddpca_probe_grid_barrier(int device, int64_t n, int phases, int blocks, int pin, double* out4) {
    return guarded([&] {
        if (!out4 || n < 1024 || n > ((int64_t)1 << 28) || phases < 2 || phases > 4096 || blocks < 1 || (pin != 0 && pin != 1))
            throw ApiError(DDPCA_EINVAL, "ddpca_probe_grid_barrier: arguments");
        select_device(device);
        int cus = 256;
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0) cus = prop.multiProcessorCount;
        if (blocks > (pin ? cus / 8 : cus)) throw ApiError(DDPCA_EINVAL, "ddpca_probe_grid_barrier: at most one workgroup per CU (of one XCD with pin)");
        const int grid = pin ? 8 * blocks : blocks;
        std::vector<double> h(n);
        for (int64_t i = 0; i < n; ++i) h[i] = (double)((i * 2654435761ll) % 1000003);
        DevBuf<double> xg, yg, xp, yp;
        DevBuf<unsigned> sync(1);
        DevBuf<int> err(1);
        sync.zero();
        err.zero();
        hipStream_t st;
        DDPCA_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
        hipEvent_t e0, e1;
        DDPCA_HIP(hipEventCreate(&e0));
        DDPCA_HIP(hipEventCreate(&e1));
        auto elapsed = [&] {
            DDPCA_HIP(hipEventSynchronize(e1));
            float ms = 0.f;
            DDPCA_HIP(hipEventElapsedTime(&ms, e0, e1));
            return (double)ms;
        };
        // graph of `phases` launches (blocks workgroups each, as the persistent form)
        hipGraph_t g;
        hipGraphExec_t ge;
        xg.upload(h);
        yg.alloc(n);
        DDPCA_HIP(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
        for (int p = 0; p < phases; ++p)
            hipLaunchKernelGGL(k_phase, dim3(blocks), dim3(256), 0, st, (p & 1) ? yg.p : xg.p, (p & 1) ? xg.p : yg.p, n);
        DDPCA_HIP(hipStreamEndCapture(st, &g));
        DDPCA_HIP(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        DDPCA_HIP(hipGraphLaunch(ge, st));  // warm-up
        DDPCA_HIP(hipMemcpyAsync(xg.p, h.data(), n * sizeof(double), hipMemcpyHostToDevice, st));
        DDPCA_HIP(hipEventRecord(e0, st));
        DDPCA_HIP(hipGraphLaunch(ge, st));
        DDPCA_HIP(hipEventRecord(e1, st));
        const double ms_graph = elapsed();
        // persistent launch
        xp.upload(h);
        yp.alloc(n);
        hipLaunchKernelGGL(k_phase_persistent, dim3(grid), dim3(256), 0, st, xp.p, yp.p, n, 2, blocks, pin, sync.p, err.p);
        DDPCA_HIP(hipMemcpyAsync(xp.p, h.data(), n * sizeof(double), hipMemcpyHostToDevice, st));
        DDPCA_HIP(hipMemsetAsync(sync.p, 0, sizeof(unsigned), st));
        DDPCA_HIP(hipEventRecord(e0, st));
        hipLaunchKernelGGL(k_phase_persistent, dim3(grid), dim3(256), 0, st, xp.p, yp.p, n, phases, blocks, pin, sync.p, err.p);
        DDPCA_HIP(hipEventRecord(e1, st));
        const double ms_pers = elapsed();
        DDPCA_HIP(hipStreamSynchronize(st));
        const std::vector<double> rg = ((phases & 1) ? yg : xg).download(), rp = ((phases & 1) ? yp : xp).download();
        double diff = 0.0;
        for (int64_t i = 0; i < n; ++i) diff = std::max(diff, std::abs(rg[i] - rp[i]));
        const int bad = err.download()[0];
        (void)hipGraphExecDestroy(ge);
        (void)hipGraphDestroy(g);
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
        (void)hipStreamDestroy(st);
        out4[0] = 1e3 * ms_graph / phases;  // us per pass
        out4[1] = 1e3 * ms_pers / phases;
        out4[2] = diff;                     // 0: the barrier made every pass's writes visible
        out4[3] = bad;                      // 1: a workgroup timed out waiting (not all resident)
    });
}

extern "C" int ddpca_stream_ceiling(int device, int64_t bytes, int reps, double* out4) {
    return guarded([&] {
        if (!out4 || bytes < (int64_t)(64 << 20) || reps < 1) throw ApiError(DDPCA_EINVAL, "ddpca_stream_ceiling: arguments");
        select_device(device);
        const int64_t n = bytes / 16;  // 16-B elements per buffer
        int cus = 256;
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0) cus = prop.multiProcessorCount;
        const int grid = cus * 8;  // 8 workgroups (32 waves) per CU
        DevBuf<double> a((size_t)2 * n), b((size_t)2 * n), part(grid);
        hipStream_t st;
        DDPCA_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
        hipEvent_t e0, e1;
        DDPCA_HIP(hipEventCreate(&e0));
        DDPCA_HIP(hipEventCreate(&e1));
        auto* x = reinterpret_cast<dbl2_t*>(a.p);
        auto* y = reinterpret_cast<dbl2_t*>(b.p);
        hipLaunchKernelGGL(k_fill, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, x, n);
        hipLaunchKernelGGL(k_fill, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, y, n);
        // best of three timed batches of `reps` back-to-back launches, after one warm-up launch
        auto timed = [&](auto launch) {
            launch();
            double best = 1e300;
            for (int t = 0; t < 3; ++t) {
                DDPCA_HIP(hipEventRecord(e0, st));
                for (int r = 0; r < reps; ++r) launch();
                DDPCA_HIP(hipEventRecord(e1, st));
                DDPCA_HIP(hipEventSynchronize(e1));
                float ms = 0.f;
                DDPCA_HIP(hipEventElapsedTime(&ms, e0, e1));
                best = std::min(best, (double)ms / reps);
            }
            return best;
        };
        const double ms_copy = timed([&] { hipLaunchKernelGGL(k_stream_copy, dim3(grid), dim3(256), 0, st, x, y, n); });
        const double ms_read = timed([&] { hipLaunchKernelGGL(k_stream_read, dim3(grid), dim3(256), 0, st, x, n, part.p); });
        DDPCA_HIP(hipStreamSynchronize(st));
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
        (void)hipStreamDestroy(st);
        const double B = 16.0 * (double)n;
        out4[0] = 2.0 * B / (ms_copy * 1e-3) / 1e9;  // copy: bytes read + bytes written
        out4[1] = B / (ms_read * 1e-3) / 1e9;
        out4[2] = ms_copy;
        out4[3] = ms_read;
    });
}
