// devmem.cpp — the library's device allocator (devmem.hpp): stream-ordered release and the
// AD_GUARD guard bands.
#include "devmem.hpp"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
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

// the guard band of an allocation of `bytes` at p, compared on the host (after the device is idle)
bool guard_intact(void* p, size_t bytes, size_t* first_bad)
{
    std::vector<unsigned char> h(GUARD);
    if (hipMemcpy(h.data(), (char*)p + bytes, GUARD, hipMemcpyDeviceToHost) != hipSuccess) return false;
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
            snprintf(b, sizeof(b), "freed buffer %p of %zu bytes: guard overwritten at +%zu", p, bytes, at);
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
            snprintf(b, sizeof(b), "live buffer %p of %zu bytes: guard overwritten at +%zu", p, bytes, at);
            found.push_back(b);
        }
    }
    if (report)
        for (auto& s : found) *report += s + "\n";
    return (int)found.size();
}

}  // namespace adx
