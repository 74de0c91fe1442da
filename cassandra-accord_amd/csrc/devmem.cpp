// devmem.cpp — the library's device allocator (devmem.hpp): stream-ordered release and the
// AD_GUARD guard bands.
#include "devmem.hpp"

#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cstdint>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <vector>

namespace adx {

namespace {

constexpr size_t GUARD = 64 << 10;
constexpr unsigned char PATTERN = 0xA5;

thread_local StreamScope* tl_scope = nullptr;

int read_mode()
{
    const char* e = getenv("AD_GUARD");
    if (!e || !*e) return 0;
    const int m = atoi(e);
    return m >= 2 ? 2 : (m == 1 ? 1 : 0);
}

struct Registry {
    std::mutex mu;
    std::unordered_map<void*, size_t> live;        // allocation -> user bytes (guard follows)
    std::vector<std::string> damaged;              // found at free time, reported by the next check
};

Registry& reg()
{
    static Registry* r = new Registry();           // never destroyed: frees may run at exit
    return *r;
}

// this thread's pinned staging: two chunks, each with the event of its last device use
constexpr size_t STAGE = 8 << 20;

// ---- host worker pool (devmem.hpp): jobs queue up; a worker takes the next task of the oldest job
// that has any left, the calling thread works on its own job until every task of it is claimed, then
// waits for the ones still running. Jobs of several threads run side by side (the host API's staging of
// slice j + 1 beside the output expansion of slice j - 1); a task may start a job of its own.
struct PoolJob {
    const std::function<void(size_t)>* f;
    size_t n;
    std::atomic<size_t> next{0};
    size_t done = 0;                       // under HostPool::mu: tasks finished
    unsigned users = 0;                    // under HostPool::mu: workers holding the job
    std::condition_variable cv;
};

struct HostPool {
    std::mutex mu;
    std::condition_variable cv;
    std::vector<PoolJob*> jobs;            // jobs with tasks left to claim
    unsigned workers = 0;
    // claim a task of j (false: none left); called under no lock
    static bool run_one(PoolJob* j)
    {
        const size_t i = j->next.fetch_add(1);
        if (i >= j->n) return false;
        (*j->f)(i);
        return true;
    }
    void finish(PoolJob* j, size_t k)
    {
        std::lock_guard<std::mutex> g(mu);
        j->done += k;
        --j->users;
        if (j->done == j->n && j->users == 0) j->cv.notify_all();
    }
    void start(unsigned w)
    {
        workers = w;
        for (unsigned i = 0; i < w; ++i)
            std::thread([this] {
                while (true)
                {
                    PoolJob* j = nullptr;
                    {
                        std::unique_lock<std::mutex> g(mu);
                        cv.wait(g, [&] {
                            while (!jobs.empty() && jobs.front()->next.load() >= jobs.front()->n) jobs.erase(jobs.begin());
                            return !jobs.empty();
                        });
                        j = jobs.front();
                        ++j->users;
                    }
                    size_t k = 0;
                    while (run_one(j)) ++k;
                    finish(j, k);
                }
            }).detach();
    }
};

HostPool& host_pool()
{
    static HostPool* p = [] {
        auto* hp = new HostPool();          // never destroyed: workers may outlive static destruction
        unsigned n = std::max(1u, std::thread::hardware_concurrency());
        if (const char* e = getenv("OMP_NUM_THREADS")) n = (unsigned)std::max(1, atoi(e));
        hp->start(std::min(n, 16u) - 1);
        return hp;
    }();
    return *p;
}

// host copy between a staging chunk and pageable memory, split over the worker pool for a full chunk
// (one thread copies ~10 GB/s: the host side, not PCIe, bounds a staged transfer)
void stage_copy(void* dst, const void* src, size_t n)
{
    constexpr size_t PART = 1 << 20;
    const size_t parts = std::min<size_t>(n / PART, 16);
    if (parts < 2)
    {
        memcpy(dst, src, n);
        return;
    }
    const size_t per = (n / parts + 63) & ~size_t(63);
    host_parallel(parts, [&](size_t i) {
        const size_t a = i * per, b = std::min(n, a + per);
        if (a < b) memcpy((char*)dst + a, (const char*)src + a, b - a);
    });
}
struct Staging {
    void* buf[2] = {nullptr, nullptr};
    hipEvent_t ev[2] = {nullptr, nullptr};
    bool busy[2] = {false, false};
    bool ok = false;
    bool init()
    {
        if (ok) return true;
        for (int k = 0; k < 2; ++k)
        {
            if (!buf[k] && hipHostMalloc(&buf[k], STAGE, hipHostMallocPortable) != hipSuccess) return false;
            if (!ev[k] && hipEventCreateWithFlags(&ev[k], hipEventDisableTiming) != hipSuccess) return false;
        }
        ok = true;
        return true;
    }
    // chunk k free for the host to write / read
    hipError_t wait(int k)
    {
        if (!busy[k]) return hipSuccess;
        busy[k] = false;
        return hipEventSynchronize(ev[k]);
    }
};
// A process-wide pool per device (a chunk's event belongs to the device of the streams it is recorded
// on): a transfer checks a staging pair out and returns it, so the pairs number the most transfers ever in
// flight at once -- not one per thread that ever called in (pooled or short-lived host threads, a Java
// binding's, would otherwise each keep 2 x 8 MB of pinned memory). A pair returned with chunks still in
// flight is waited for (its events) by the next user. The pool lives as long as the process.
constexpr int MAX_DEV = 16;
struct StagingPool {
    std::mutex mu;
    std::vector<Staging*> free;
};
StagingPool g_stage_pool[MAX_DEV];
struct StagingLease {
    int d = -1;
    Staging* s = nullptr;
    StagingLease()
    {
        if (hipGetDevice(&d) != hipSuccess || d < 0 || d >= MAX_DEV) return;
        {
            std::lock_guard<std::mutex> g(g_stage_pool[d].mu);
            if (!g_stage_pool[d].free.empty())
            {
                s = g_stage_pool[d].free.back();
                g_stage_pool[d].free.pop_back();
            }
        }
        if (!s) s = new Staging();
        if (!s->init())
        {
            std::lock_guard<std::mutex> g(g_stage_pool[d].mu);
            g_stage_pool[d].free.push_back(s);        // whatever it holds is kept for a later init
            s = nullptr;
        }
    }
    // The pair goes back to the pool with nothing in flight, on every exit of a transfer, errors included: its
    // events were recorded on the caller's stream, which a context may destroy before the pair's next user would
    // wait on them (round 5 saw one "stream is capturing" error from a staged upload on a fresh context, DESIGN
    // §7). A transfer that failed between queuing a copy and recording its event (st_dirty) leaves a copy the
    // events do not cover: its stream is synchronised instead.
    hipStream_t st = nullptr;
    bool st_dirty = false;
    ~StagingLease()
    {
        if (!s) return;
        (void)s->wait(0);
        (void)s->wait(1);
        if (st_dirty) (void)hipStreamSynchronize(st);
        std::lock_guard<std::mutex> g(g_stage_pool[d].mu);
        g_stage_pool[d].free.push_back(s);
    }
    StagingLease(const StagingLease&) = delete;
    StagingLease& operator=(const StagingLease&) = delete;
};

// the guard band of an allocation of `bytes` at p, compared on the host (after the device is idle).
// *first_bad = SIZE_MAX when the band could not be read (a device already faulted)
bool guard_intact(void* p, size_t bytes, size_t* first_bad)
{
    std::vector<unsigned char> h(GUARD);
    if (d2h(h.data(), (char*)p + bytes, GUARD, nullptr) != hipSuccess)
    {
        *first_bad = SIZE_MAX;
        return false;
    }
    for (size_t i = 0; i < GUARD; ++i)
        if (h[i] != PATTERN)
        {
            *first_bad = i;
            return false;
        }
    return true;
}

void sync_scope(StreamScope* s)
{
    bool any = false;
    for (hipStream_t x : s->s)
        if (x)
        {
            (void)hipStreamSynchronize(x);
            any = true;
        }
    if (!any) (void)hipDeviceSynchronize();
}

}  // namespace

int dev_guard_mode()
{
    static const int m = read_mode();
    return m;
}

StreamScope::StreamScope(hipStream_t a, hipStream_t b, hipStream_t c)
{
    s[0] = a;
    s[1] = b;
    s[2] = c;
    prev = tl_scope;
    tl_scope = this;
}

StreamScope::~StreamScope() { tl_scope = prev; }

void StreamScope::add(hipStream_t x)
{
    if (!x) return;
    for (hipStream_t& y : s)
    {
        if (y == x) return;
        if (!y)
        {
            y = x;
            return;
        }
    }
}

hipStream_t dev_scope_stream() { return tl_scope ? tl_scope->s[0] : nullptr; }

void dev_quiesce()
{
    if (tl_scope) sync_scope(tl_scope);
    else (void)hipDeviceSynchronize();
}

hipError_t dev_zero_sync(void* p, size_t bytes)
{
    const hipStream_t st = dev_scope_stream();
    hipError_t e = hipMemsetAsync(p, 0, bytes, st);
    if (e != hipSuccess) return e;
    return st ? hipStreamSynchronize(st) : hipDeviceSynchronize();
}

void* dev_alloc(size_t bytes)
{
    const int mode = dev_guard_mode();
    void* p = nullptr;
    if (hipMalloc(&p, bytes + (mode ? GUARD : 0)) != hipSuccess) return nullptr;
    if (mode)
    {
        // filled before anything can use the buffer: complete on return
        if (hipMemset((char*)p + bytes, PATTERN, GUARD) != hipSuccess ||
            (mode == 2 && bytes && hipMemset(p, PATTERN, bytes) != hipSuccess) || hipDeviceSynchronize() != hipSuccess)
        {
            (void)hipFree(p);
            return nullptr;
        }
        std::lock_guard<std::mutex> g(reg().mu);
        reg().live[p] = bytes;
    }
    return p;
}

void dev_free(void* p)
{
    if (!p) return;
    dev_quiesce();
    if (dev_guard_mode())
    {
        size_t bytes = 0;
        {
            std::lock_guard<std::mutex> g(reg().mu);
            auto it = reg().live.find(p);
            if (it != reg().live.end())
            {
                bytes = it->second;
                reg().live.erase(it);
            }
        }
        (void)hipDeviceSynchronize();
        size_t at = 0;
        if (!guard_intact(p, bytes, &at))
        {
            char b[160];
            if (at == SIZE_MAX) snprintf(b, sizeof(b), "freed buffer %p of %zu bytes: guard unreadable (device error)", p, bytes);
            else snprintf(b, sizeof(b), "freed buffer %p of %zu bytes: guard overwritten at +%zu", p, bytes, at);
            fprintf(stderr, "AD_GUARD: %s\n", b);
            std::lock_guard<std::mutex> g(reg().mu);
            reg().damaged.push_back(b);
        }
    }
    (void)hipFree(p);
}

int dev_guard_check(std::string* report)
{
    if (!dev_guard_mode()) return 0;
    (void)hipDeviceSynchronize();
    std::vector<std::pair<void*, size_t>> snap;
    std::vector<std::string> found;
    {
        std::lock_guard<std::mutex> g(reg().mu);
        snap.assign(reg().live.begin(), reg().live.end());
        found.swap(reg().damaged);
    }
    for (auto& [p, bytes] : snap)
    {
        size_t at = 0;
        if (!guard_intact(p, bytes, &at))
        {
            char b[160];
            if (at == SIZE_MAX) snprintf(b, sizeof(b), "live buffer %p of %zu bytes: guard unreadable (device error)", p, bytes);
            else snprintf(b, sizeof(b), "live buffer %p of %zu bytes: guard overwritten at +%zu", p, bytes, at);
            found.push_back(b);
        }
    }
    if (report)
        for (auto& s : found) *report += s + "\n";
    return (int)found.size();
}

bool host_pinned(const void* p)
{
    if (!p) return false;
    hipPointerAttribute_t a{};
    if (hipPointerGetAttributes(&a, p) != hipSuccess)
    {
        (void)hipGetLastError();       // pageable memory: not an error of anything else
        return false;
    }
    return a.type == hipMemoryTypeHost;
}

hipError_t h2d(void* dst, const void* src, size_t bytes, hipStream_t st)
{
    if (!bytes) return hipSuccess;
    if (host_pinned(src)) return hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, st);
    StagingLease lease;
    if (!lease.s) return hipErrorOutOfMemory;
    lease.st = st;
    Staging& S = *lease.s;
    int k = 0;
    for (size_t off = 0; off < bytes; off += STAGE, k ^= 1)
    {
        const size_t n = std::min(STAGE, bytes - off);
        hipError_t e = S.wait(k);
        if (e != hipSuccess) return e;
        stage_copy(S.buf[k], (const char*)src + off, n);
        lease.st_dirty = true;          // until the chunk's event covers its copy
        if ((e = hipMemcpyAsync((char*)dst + off, S.buf[k], n, hipMemcpyHostToDevice, st)) != hipSuccess) return e;
        if ((e = hipEventRecord(S.ev[k], st)) != hipSuccess) return e;
        S.busy[k] = true;
        lease.st_dirty = false;
    }
    // drained here (not only by the lease) so that a failed copy is reported by this call
    hipError_t e = S.wait(0);
    const hipError_t e1 = S.wait(1);
    return e != hipSuccess ? e : e1;
}

hipError_t d2h(void* dst, const void* src, size_t bytes, hipStream_t st)
{
    if (!bytes) return hipSuccess;
    if (host_pinned(dst)) return hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, st);
    StagingLease lease;
    if (!lease.s) return hipErrorOutOfMemory;
    lease.st = st;
    Staging& S = *lease.s;
    // chunk i is copied to the host while chunk i + 1 is in flight
    size_t prev_off = 0, prev_n = 0;
    int k = 0;
    hipError_t e = hipSuccess;
    for (size_t off = 0; off < bytes; off += STAGE, k ^= 1)
    {
        const size_t n = std::min(STAGE, bytes - off);
        if ((e = S.wait(k)) != hipSuccess) return e;
        lease.st_dirty = true;          // until the chunk's event covers its copy
        if ((e = hipMemcpyAsync(S.buf[k], (const char*)src + off, n, hipMemcpyDeviceToHost, st)) != hipSuccess) return e;
        if ((e = hipEventRecord(S.ev[k], st)) != hipSuccess) return e;
        S.busy[k] = true;
        lease.st_dirty = false;
        if (prev_n)
        {
            if ((e = S.wait(k ^ 1)) != hipSuccess) return e;
            stage_copy((char*)dst + prev_off, S.buf[k ^ 1], prev_n);
        }
        prev_off = off;
        prev_n = n;
    }
    k ^= 1;            // the last chunk issued
    if ((e = S.wait(k)) != hipSuccess) return e;
    stage_copy((char*)dst + prev_off, S.buf[k], prev_n);
    return hipSuccess;
}

void host_parallel(size_t n, const std::function<void(size_t)>& f)
{
    if (n == 0) return;
    HostPool& P = host_pool();
    if (n == 1 || P.workers == 0)
    {
        for (size_t i = 0; i < n; ++i) f(i);
        return;
    }
    PoolJob j;
    j.f = &f;
    j.n = n;
    {
        std::lock_guard<std::mutex> g(P.mu);
        P.jobs.push_back(&j);
    }
    P.cv.notify_all();
    size_t k = 0;
    while (HostPool::run_one(&j)) ++k;
    std::unique_lock<std::mutex> g(P.mu);
    j.done += k;
    // every task is claimed: the job leaves the queue (a worker may have dropped it already)
    for (size_t i = 0; i < P.jobs.size(); ++i)
        if (P.jobs[i] == &j)
        {
            P.jobs.erase(P.jobs.begin() + i);
            break;
        }
    j.cv.wait(g, [&] { return j.done == j.n && j.users == 0; });
}

unsigned host_threads() { return host_pool().workers + 1; }

void host_trace(const char* what)
{
    static const bool on = getenv("AD_HOST_TRACE") != nullptr;
    if (!on) return;
    static thread_local std::chrono::steady_clock::time_point last = std::chrono::steady_clock::now();
    const auto now = std::chrono::steady_clock::now();
    fprintf(stderr, "[ht] %9.3f ms  %s\n", std::chrono::duration<double, std::milli>(now - last).count(), what);
    last = now;
}

}  // namespace adx
