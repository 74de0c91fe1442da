// PCIe duplex: SDMA copies vs kernels reading / writing mapped pinned host memory, alone and together
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstring>
static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
__global__ void k_copy(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n)
{
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}
__global__ void k_copy_plain(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n)
{
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) dst[i] = src[i];
}
int main()
{
    const size_t B = 256ull << 20, N = B / 16;
    void *d0, *d1, *h0, *h1, *h2, *h3;
    hipMalloc(&d0, B); hipMalloc(&d1, B);
    hipHostMalloc(&h0, B, hipHostMallocDefault); hipHostMalloc(&h1, B, hipHostMallocDefault);
    hipHostMalloc(&h2, B, hipHostMallocDefault); hipHostMalloc(&h3, B, hipHostMallocDefault);
    memset(h0, 1, B); memset(h1, 2, B); memset(h2, 3, B); memset(h3, 4, B);
    void *m1, *m2;
    hipHostGetDevicePointer(&m1, h1, 0); hipHostGetDevicePointer(&m2, h2, 0);
    hipStream_t s0, s1;
    hipStreamCreateWithFlags(&s0, hipStreamNonBlocking); hipStreamCreateWithFlags(&s1, hipStreamNonBlocking);
    for (int rep = 0; rep < 3; ++rep)
    {
        double t = now();
        k_copy<<<1024, 256, 0, s0>>>((const uint4*)d1, (uint4*)m1, N); hipStreamSynchronize(s0);
        const double kd2h = B / (now() - t) / 1e9;
        t = now();
        k_copy_plain<<<1024, 256, 0, s0>>>((const uint4*)m2, (uint4*)d0, N); hipStreamSynchronize(s0);
        const double kh2d = B / (now() - t) / 1e9;
        t = now();
        hipMemcpyAsync(d0, h0, B, hipMemcpyHostToDevice, s1);
        k_copy<<<1024, 256, 0, s0>>>((const uint4*)d1, (uint4*)m1, N);
        hipStreamSynchronize(s0); hipStreamSynchronize(s1);
        const double mix1 = 2.0 * B / (now() - t) / 1e9;
        t = now();
        hipMemcpyAsync(h3, d1, B, hipMemcpyDeviceToHost, s1);
        k_copy_plain<<<1024, 256, 0, s0>>>((const uint4*)m2, (uint4*)d0, N);
        hipStreamSynchronize(s0); hipStreamSynchronize(s1);
        const double mix2 = 2.0 * B / (now() - t) / 1e9;
        t = now();
        k_copy<<<512, 256, 0, s0>>>((const uint4*)d1, (uint4*)m1, N);
        k_copy_plain<<<512, 256, 0, s1>>>((const uint4*)m2, (uint4*)d0, N);
        hipStreamSynchronize(s0); hipStreamSynchronize(s1);
        const double mix3 = 2.0 * B / (now() - t) / 1e9;
        printf("kernel D2H %.1f GB/s, kernel H2D %.1f GB/s | SDMA H2D + kernel D2H %.1f GB/s total | SDMA D2H + kernel H2D "
               "%.1f | kernel both %.1f\n", kd2h, kh2d, mix1, mix2, mix3);
    }
    return 0;
}
