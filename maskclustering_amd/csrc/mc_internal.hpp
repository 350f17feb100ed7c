// mc_internal.hpp — shared definitions of libmcgraph (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <map>
#include <utility>
#include <string>
#include <vector>

#include "../../include/mcgraph.h"

namespace mc {

constexpr int kWave = 64;                 // CDNA wavefront
constexpr int kLocalBits = 12;            // point-list entry = (frame << 12) | mask-in-frame
constexpr int kMaxMasksPerFrame = 1 << kLocalBits;
constexpr int kMaxFrames = 1 << (32 - kLocalBits - 1);
constexpr int kMaxThresholds = 20;        // percentiles 95..0 step 5 (construction.py:88)

struct McError {
    int code;
    std::string msg;
};

#define MC_HIP(call)                                                                      \
    do {                                                                                  \
        hipError_t e_ = (call);                                                           \
        if (e_ != hipSuccess)                                                             \
            throw ::mc::McError{MC_ERR_HIP, std::string(#call) + ": " + hipGetErrorString(e_)}; \
    } while (0)

#define MC_REQUIRE(cond, code, msg)                                                       \
    do {                                                                                  \
        if (!(cond)) throw ::mc::McError{(code), (msg)};                                  \
    } while (0)

// Growable device buffer; only (re)allocated outside the timed path when the
// requested capacity exceeds the current one.
struct DevBuf {
    void *ptr = nullptr;
    size_t bytes = 0;
    DevBuf() = default;
    DevBuf(const DevBuf &) = delete;
    DevBuf &operator=(const DevBuf &) = delete;
    ~DevBuf() { release(); }  // temporaries of a call free themselves (after the call's sync)
    void swap(DevBuf &o) {
        std::swap(ptr, o.ptr);
        std::swap(bytes, o.bytes);
    }
    void reserve(size_t n) {
        if (n <= bytes) return;
        if (ptr) MC_HIP(hipFree(ptr));
        ptr = nullptr;
        size_t cap = n < 256 ? 256 : n;
        MC_HIP(hipMalloc(&ptr, cap));
        bytes = cap;
    }
    void release() {
        if (ptr) (void)hipFree(ptr);
        ptr = nullptr;
        bytes = 0;
    }
    template <typename T> T *as() const { return static_cast<T *>(ptr); }
};

inline int ceil_div(int64_t a, int64_t b) { return static_cast<int>((a + b - 1) / b); }

// Kernel timing with events (enabled only by bench/profiling runs).
struct KernelTimer {
    bool enabled = false;
    std::string filter;  // empty = every scope
    struct Rec {
        hipEvent_t a, b;
        std::string name;
    };
    std::vector<Rec> pending;
    std::vector<hipEvent_t> pool;
    std::map<std::string, std::pair<double, int64_t>> totals;
    hipEvent_t get() {
        if (!pool.empty()) {
            hipEvent_t e = pool.back();
            pool.pop_back();
            return e;
        }
        hipEvent_t e;
        MC_HIP(hipEventCreate(&e));
        return e;
    }
    void collect() {
        for (auto &r : pending) {
            float ms = 0.f;
            MC_HIP(hipEventSynchronize(r.b));
            MC_HIP(hipEventElapsedTime(&ms, r.a, r.b));
            auto &t = totals[r.name];
            t.first += ms;
            t.second += 1;
            pool.push_back(r.a);
            pool.push_back(r.b);
        }
        pending.clear();
    }
    ~KernelTimer() {
        for (auto &r : pending) {
            (void)hipEventDestroy(r.a);
            (void)hipEventDestroy(r.b);
        }
        for (auto e : pool) (void)hipEventDestroy(e);
    }
};

// Scoped launch timing: records an event pair around the launches in scope.
struct TimedScope {
    KernelTimer &t;
    hipStream_t s;
    hipEvent_t a{}, b{};
    const char *name;
    bool on;
    TimedScope(KernelTimer &t_, hipStream_t s_, const char *n)
        : t(t_), s(s_), name(n), on(t_.enabled && (t_.filter.empty() || t_.filter == n)) {
        if (on) {
            a = t.get();
            b = t.get();
            MC_HIP(hipEventRecord(a, s));
        }
    }
    ~TimedScope() {
        if (on) {
            (void)hipEventRecord(b, s);
            t.pending.push_back({a, b, name});
        }
    }
};

}  // namespace mc
