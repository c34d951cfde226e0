// PMC calibration: streaming reads of a known byte count with the SELL kernels' access widths.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void rd8(const double* __restrict__ a, int64_t n, double* out) {
    double s = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) s += a[i];
    if (s == 123.456) out[0] = s;
}
__global__ void rd8nt(const double* __restrict__ a, int64_t n, double* out) {
    double s = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        s += __builtin_nontemporal_load(a + i);
    if (s == 123.456) out[0] = s;
}
__global__ void rd16(const double2* __restrict__ a, int64_t n2, double* out) {
    double s = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += (int64_t)gridDim.x * blockDim.x) {
        const double2 v = a[i];
        s += v.x + v.y;
    }
    if (s == 123.456) out[0] = s;
}
// 9 independent 8-B/lane streams per iteration, like one SELL-BSR3 block slot
__global__ void rd8x9(const double* __restrict__ a, int64_t nslot, double* out) {
    const int lane = threadIdx.x & 63;
    const int64_t w = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6, nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
    double s = 0.0;
    for (int64_t k = w; k < nslot; k += nw) {
        const double* v = a + k * 9 * 64 + lane;
#pragma unroll
        for (int j = 0; j < 9; ++j) s += __builtin_nontemporal_load(v + j * 64);
    }
    if (s == 123.456) out[0] = s;
}

int main() {
    const int64_t bytes = 1ll << 30;
    const int64_t n = bytes / 8;
    double *a, *o;
    hipMalloc(&a, bytes);
    hipMalloc(&o, 64);
    hipMemset(a, 0, bytes);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto run = [&](const char* name, auto launch) {
        for (int r = 0; r < 4; ++r) {
            hipEventRecord(e0);
            launch();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            printf("%s run %d: %.3f ms  %.2f TB/s\n", name, r, ms, bytes / (ms * 1e-3) / 1e12);
        }
    };
    const int grid = 256 * 32;
    run("rd8", [&] { hipLaunchKernelGGL(rd8, dim3(grid), dim3(256), 0, 0, a, n, o); });
    run("rd8nt", [&] { hipLaunchKernelGGL(rd8nt, dim3(grid), dim3(256), 0, 0, a, n, o); });
    run("rd16", [&] { hipLaunchKernelGGL(rd16, dim3(grid), dim3(256), 0, 0, (const double2*)a, n / 2, o); });
    run("rd8x9", [&] { hipLaunchKernelGGL(rd8x9, dim3(grid), dim3(256), 0, 0, a, n / (9 * 64), o); });
    hipDeviceSynchronize();
    printf("bytes per launch %lld (rd8x9 reads %lld)\n", (long long)bytes, (long long)(n / (9 * 64) * 9 * 64 * 8));
    return 0;
}
