// Device-side plumbing shared by the MGPIS and MCONTACT device code (gfx950, wave64).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

#include "common.hpp"

namespace ddpca {

#define DDPCA_HIP(call)                                                                          \
    do {                                                                                         \
        hipError_t e_ = (call);                                                                  \
        if (e_ != hipSuccess)                                                                    \
            throw ::ddpca::ApiError(-2, std::string(#call) + ": " + hipGetErrorString(e_) + " at " + \
                                            __FILE__ + ":" + std::to_string(__LINE__));          \
    } while (0)

constexpr int kWave = 64;      // CDNA wavefront
constexpr int kChunk = 64;     // SELL chunk = one node row per lane of a wave
constexpr int kBlock = 256;    // 4 waves per workgroup

// Owning device allocation.
template <typename T>
struct DevBuf {
    T* p = nullptr;
    size_t n = 0;
    DevBuf() = default;
    explicit DevBuf(size_t count) { alloc(count); }
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    DevBuf(DevBuf&& o) noexcept : p(o.p), n(o.n) { o.p = nullptr; o.n = 0; }
    DevBuf& operator=(DevBuf&& o) noexcept {
        if (this != &o) { release(); p = o.p; n = o.n; o.p = nullptr; o.n = 0; }
        return *this;
    }
    ~DevBuf() { release(); }
    void alloc(size_t count) {
        release();
        n = count;
        if (count) DDPCA_HIP(hipMalloc(&p, count * sizeof(T)));
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
    void upload(const T* h, size_t count) {
        alloc(count);
        if (count) DDPCA_HIP(hipMemcpy(p, h, count * sizeof(T), hipMemcpyHostToDevice));
    }
    void upload(const std::vector<T>& v) { upload(v.data(), v.size()); }
    void zero(hipStream_t s = 0) {
        if (n) DDPCA_HIP(hipMemsetAsync(p, 0, n * sizeof(T), s));
    }
    std::vector<T> download() const {
        std::vector<T> v(n);
        if (n) DDPCA_HIP(hipMemcpy(v.data(), p, n * sizeof(T), hipMemcpyDeviceToHost));
        return v;
    }
};

inline int ceil_div(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

// Make `device` current and check it is a gfx950 part (no silent fallback anywhere).
void select_device(int device);

}  // namespace ddpca
