// Device-side plumbing shared by the MGPIS and MCONTACT device code (gfx950, wave64).
#pragma once
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdlib>
#include <mutex>
#include <shared_mutex>
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

// Stream capture vs. synchronous HIP calls on other host threads.  ROCm 7.2 invalidated a
// hipStreamCaptureModeThreadLocal capture on one thread while another thread of the process made
// synchronous calls (its first solve's hipMalloc / hipMemcpy / hipFree: "hipStreamEndCapture:
// operation failed due to a previous error during capture", profiles/r05p/gputest_first.log).  So
// every capture of the library holds this lock exclusively (CaptureSection), and every device
// allocation, free and synchronous copy (DevBuf) holds it shared for the length of that one call:
// no synchronous call of the library overlaps a capture on another thread.  Neither side ever waits
// on another thread while holding it (no deadlock with the in-process ranks' barriers).  A thread
// inside its own capture skips the shared side (it makes no such call there).
struct CaptureLock {
    static std::shared_mutex& mutex() {
        static std::shared_mutex m;
        return m;
    }
    static bool& capturing() {
        static thread_local bool c = false;
        return c;
    }
};
struct CaptureSection {
    std::unique_lock<std::shared_mutex> g{CaptureLock::mutex()};
    CaptureSection() { CaptureLock::capturing() = true; }
    ~CaptureSection() { CaptureLock::capturing() = false; }
    CaptureSection(const CaptureSection&) = delete;
    CaptureSection& operator=(const CaptureSection&) = delete;
};
struct SyncCallGuard {
    std::shared_lock<std::shared_mutex> g;
    SyncCallGuard() {
        if (!CaptureLock::capturing()) g = std::shared_lock<std::shared_mutex>(CaptureLock::mutex());
    }
};

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
        if (count) {
            SyncCallGuard g;
            DDPCA_HIP(hipMalloc(&p, count * sizeof(T)));
        }
    }
    void release() {
        if (p) {
            SyncCallGuard g;
            (void)hipFree(p);
        }
        p = nullptr;
        n = 0;
    }
    void upload(const T* h, size_t count) {
        alloc(count);
        if (count) {
            SyncCallGuard g;
            DDPCA_HIP(hipMemcpy(p, h, count * sizeof(T), hipMemcpyHostToDevice));
        }
    }
    void upload(const std::vector<T>& v) { upload(v.data(), v.size()); }
    void zero(hipStream_t s = 0) {
        if (n) DDPCA_HIP(hipMemsetAsync(p, 0, n * sizeof(T), s));
    }
    std::vector<T> download() const {
        std::vector<T> v(n);
        if (n) {
            SyncCallGuard g;
            DDPCA_HIP(hipMemcpy(v.data(), p, n * sizeof(T), hipMemcpyDeviceToHost));
        }
        return v;
    }
};

// Non-owning device range carved out of a DevBuf.
template <typename T>
struct DevSpan {
    T* p = nullptr;
    size_t n = 0;
    void zero(hipStream_t s = 0) {
        if (n) DDPCA_HIP(hipMemsetAsync(p, 0, n * sizeof(T), s));
    }
};

inline int ceil_div(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }
inline int64_t pad64(int64_t n) { return (n + 63) / 64 * 64; }

// Make `device` current and check it is a gfx950 part (no silent fallback anywhere).
void select_device(int device);

// Host-visible stop state of one iterative solve, written by the device with system-scope
// stores into pinned, device-mapped host memory: the host paces graph replays by reading it,
// with no copy and no stream synchronisation per poll.
struct PcgMirror {
    int64_t iter;
    int32_t done;
    int32_t fail;
};

__device__ __forceinline__ void mirror_store(PcgMirror* m, int64_t iter, int done, int fail) {
    __hip_atomic_store(&m->iter, iter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&m->fail, fail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&m->done, done, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Pinned host array of n mirrors plus its device alias.
struct MirrorBuf {
    PcgMirror* host = nullptr;
    PcgMirror* dev = nullptr;
    int n = 0;
    void alloc(int count);
    void reset();  // host-side zeroing; only while no kernel can write it
    ~MirrorBuf();
};

// Replay `graph` (k iterations each) on `stream` until every mirror reports done, keeping
// about one replay queued ahead of the slowest unfinished solve.  `launched` = iterations
// already enqueued (eager + pre-enqueued replays).  Returns the number of replays launched.
// graph1 (one iteration) and horizon: once the queued iterations would pass `horizon` (the
// solves' expected count), single iterations are queued two ahead of the slowest solve instead.
int64_t pace_until_done(hipStream_t stream, hipGraphExec_t graph, const MirrorBuf& m, int64_t k, int64_t launched,
                        hipGraphExec_t graph1 = nullptr, int64_t horizon = INT64_MAX);
// the same for a batch split into np parts (part[s] in 0 .. np-1, np <= kMaxParts), each part's
// graph on its stream (g1 / horizon: per part, or null); pace_halves: np = 2
constexpr int kMaxParts = 4;
int64_t pace_parts(int np, hipStream_t* st, hipGraphExec_t* g, const MirrorBuf& m, const std::vector<int>& part, int64_t k,
                   int64_t launched0, hipGraphExec_t* g1 = nullptr, const int64_t* horizon = nullptr);
inline int64_t pace_halves(hipStream_t st[2], hipGraphExec_t g[2], const MirrorBuf& m, const std::vector<int>& half, int64_t k,
                           int64_t launched0, hipGraphExec_t* g1 = nullptr, const int64_t* horizon = nullptr) {
    return pace_parts(2, st, g, m, half, k, launched0, g1, horizon);
}

// rocSOLVER / rocBLAS from several host threads of one process (the in-process ranks of the
// multi-rank tests) gave non-deterministic potrf failures on the very same matrix (TORSION on 4
// ranks, n = 3468: info 2229, then 1479, while every rank held the 1-rank matrix bit for bit,
// profiles/r04b): the dense factorisations of one process take this lock (DESIGN.md §7 has the
// audit of our side of those setup paths).  A production rank is one process with one factorisation
// at a time, so it serialises nothing there.  DDPCA_SOLVER_LOCK=0 turns it off: the concurrency test
// (tests/test_mgpis_gpu.py::test_concurrent_dense_factorisations_bit_identical) runs that way.
inline std::mutex& solver_mutex() {
    static std::mutex m;
    return m;
}
inline std::unique_lock<std::mutex> solver_lock() {
    static const bool on = [] {
        const char* e = std::getenv("DDPCA_SOLVER_LOCK");
        return !(e && e[0] == '0');
    }();
    return on ? std::unique_lock<std::mutex>(solver_mutex()) : std::unique_lock<std::mutex>();
}

}  // namespace ddpca
