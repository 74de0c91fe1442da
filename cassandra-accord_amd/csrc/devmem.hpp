// devmem.hpp — device memory of libaccord_deps: one allocator and one buffer type for every
// translation unit (ABI, ingest, derivation/update, levels, exchange).
//
// Release ordering. Every ctx works on non-blocking streams, so a buffer freed (or grown) in the
// middle of a call may still be read or written by work queued on that call's streams. dev_free
// therefore first synchronizes the streams of the innermost StreamScope on this thread (the ctx
// stream, its copy stream, a caller's stream) -- not the whole device, so other ctxs, the caller's
// other streams and RCCL are not stalled -- and falls back to a device synchronization only when no
// scope is open (ctx destruction, calls spanning several ctxs).
//
// Debug (environment, read once): AD_GUARD=1 puts a 64 KB guard band of a known pattern after every
// allocation and checks it when the allocation is freed and on dev_guard_check() (the ABI exports it
// as ad_debug_guard_check): a kernel or copy writing past the end of a buffer is reported with the
// buffer's size instead of silently corrupting its neighbour. AD_GUARD=2 also poisons new allocations
// (0xA5 bytes), so a read of memory nothing wrote gives the same wrong value on every run instead of
// whatever the previous owner left there.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstddef>
#include <functional>
#include <string>

namespace adx {

void* dev_alloc(size_t bytes);                 // nullptr on failure
void dev_free(void* p);                        // stream-ordered (see above); null is a no-op
void dev_quiesce();                            // the current scope's streams, or the device
hipStream_t dev_scope_stream();                // the scope's first stream (null: none open)
// zero `bytes` at p, ordered on the scope's first stream and complete on return
hipError_t dev_zero_sync(void* p, size_t bytes);
int dev_guard_mode();                          // 0 off, 1 guards, 2 guards + poison

// Transfers between the device and host memory. The library never hands pageable host memory to a
// HIP copy: a host pointer that is not pinned (hipHostMalloc'd or hipHostRegister'ed by the caller)
// is bounced through this thread's pinned staging chunks with a host memcpy. (Pageable HIP copies were
// the common factor of the intermittent device faults and host corruption of rounds 3-4 -- DESIGN.md
// §7.) h2d: `src` may be reused on return, the copy is ordered on `st`. d2h: pinned `dst` -- queued on
// `st`, like hipMemcpyAsync; pageable `dst` -- complete on return.
bool host_pinned(const void* p);
hipError_t h2d(void* dst, const void* src, size_t bytes, hipStream_t st);
hipError_t d2h(void* dst, const void* src, size_t bytes, hipStream_t st);
// A persistent pool of host worker threads (process-wide, started on first use; OMP_NUM_THREADS or the
// hardware threads, at most 16 in all): host_parallel(n, f) runs f(0) .. f(n-1) over the workers and
// the calling thread and returns when every call has returned. One job runs at a time; a call made
// while the pool is busy (another thread's job, or from inside a job) runs its tasks on the calling
// thread. Spawning threads per call cost ~0.1 ms per copy of the host API's staging.
void host_parallel(size_t n, const std::function<void(size_t)>& f);
unsigned host_threads();
// damaged guard bands among the live allocations (and the ones freed since the last call); a
// description of each is appended to *report
int dev_guard_check(std::string* report);
// AD_HOST_TRACE=1 (read once): host_trace(what) prints, to stderr, the host time since the previous
// host_trace on this thread -- where a call's host-side work goes between its kernels
void host_trace(const char* what);

// the streams whose queued work may touch the buffers a call frees (innermost scope wins)
struct StreamScope {
    explicit StreamScope(hipStream_t a, hipStream_t b = nullptr, hipStream_t c = nullptr);
    ~StreamScope();
    StreamScope(const StreamScope&) = delete;
    StreamScope& operator=(const StreamScope&) = delete;
    void add(hipStream_t s);
    hipStream_t s[4] = {nullptr, nullptr, nullptr, nullptr};
    StreamScope* prev = nullptr;
};

// An event that only times stream work (stage times, ad_stats): recorded without the system-scope
// fence (cache write-back + invalidate) a default event performs -- measured ~6 us of idle GPU per
// record between two kernels on config 2, and the invalidate also costs the next kernel its warm L2.
// Never for events other work waits on.
inline hipError_t timing_event(hipEvent_t* e) { return hipEventCreateWithFlags(e, hipEventDisableSystemFence); }

// A growable device buffer. ensure() keeps the buffer when it is large enough, else frees it (stream-
// ordered) and allocates `bytes` (at least 64); grow() does the same with 1/4 slack and optional zeroing
// (buffers that grow every batch). Contents are not kept across a reallocation.
struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    ~DevBuf() { release(); }
    void release()
    {
        if (p) dev_free(p);
        p = nullptr;
        cap = 0;
    }
    bool ensure(size_t bytes)
    {
        if (p && bytes <= cap) return true;
        release();
        const size_t b = std::max<size_t>(bytes, 64);
        p = dev_alloc(b);
        if (!p) return false;
        cap = b;
        return true;
    }
    bool grow(size_t bytes, bool zero = false)
    {
        if (p && bytes <= cap) return true;
        release();
        const size_t b = std::max<size_t>(bytes + bytes / 4, 64);
        p = dev_alloc(b);
        if (!p) return false;
        cap = b;
        if (zero && dev_zero_sync(p, b) != hipSuccess) return false;
        return true;
    }
    template <class T> T* as() const { return reinterpret_cast<T*>(p); }
};

inline void swap_bufs(DevBuf& a, DevBuf& b)
{
    std::swap(a.p, b.p);
    std::swap(a.cap, b.cap);
}

}  // namespace adx
