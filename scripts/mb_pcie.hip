// PCIe link peaks on the box: pinned H2D, D2H, both at once; pageable H2D/D2H (hipMemcpy)
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
int main()
{
    const size_t B = 256ull << 20;
    void *d0, *d1, *h0, *h1;
    hipMalloc(&d0, B); hipMalloc(&d1, B);
    hipHostMalloc(&h0, B, hipHostMallocDefault); hipHostMalloc(&h1, B, hipHostMallocDefault);
    memset(h0, 1, B); memset(h1, 2, B);
    hipStream_t s0, s1;
    hipStreamCreateWithFlags(&s0, hipStreamNonBlocking); hipStreamCreateWithFlags(&s1, hipStreamNonBlocking);
    for (int rep = 0; rep < 3; ++rep)
    {
        double t = now();
        hipMemcpyAsync(d0, h0, B, hipMemcpyHostToDevice, s0); hipStreamSynchronize(s0);
        const double h2d = B / (now() - t) / 1e9;
        t = now();
        hipMemcpyAsync(h1, d1, B, hipMemcpyDeviceToHost, s0); hipStreamSynchronize(s0);
        const double d2h = B / (now() - t) / 1e9;
        t = now();
        hipMemcpyAsync(d0, h0, B, hipMemcpyHostToDevice, s0);
        hipMemcpyAsync(h1, d1, B, hipMemcpyDeviceToHost, s1);
        hipStreamSynchronize(s0); hipStreamSynchronize(s1);
        const double both = 2.0 * B / (now() - t) / 1e9;
        // 4 MB chunks D2H (the copy-out's granularity)
        t = now();
        for (size_t o = 0; o < B; o += 4 << 20) hipMemcpyAsync((char*)h1 + o, (char*)d1 + o, 4 << 20, hipMemcpyDeviceToHost, s0);
        hipStreamSynchronize(s0);
        const double d2h_4m = B / (now() - t) / 1e9;
        printf("pinned 256 MB: H2D %.1f GB/s, D2H %.1f GB/s, both directions %.1f GB/s total, D2H in 4 MB copies %.1f GB/s\n",
               h2d, d2h, both, d2h_4m);
    }
    char* pg = (char*)malloc(B);
    memset(pg, 3, B);
    for (int rep = 0; rep < 2; ++rep)
    {
        double t = now();
        hipMemcpy(d0, pg, B, hipMemcpyHostToDevice);
        const double h2d = B / (now() - t) / 1e9;
        t = now();
        hipMemcpy(pg, d1, B, hipMemcpyDeviceToHost);
        const double d2h = B / (now() - t) / 1e9;
        t = now();
        memcpy(h0, pg, B);
        const double mc = B / (now() - t) / 1e9;
        printf("pageable 256 MB (hipMemcpy): H2D %.1f GB/s, D2H %.1f GB/s; host memcpy into pinned %.1f GB/s\n", h2d, d2h, mc);
    }
    return 0;
}
