// ping-pong hand-off latency between two blocks: flag word round trips
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
template <int MODE>   // 0: sc1 store / sc1 load; 1: sc0 store / sc1 load
__global__ void k_pp(uint32_t* flag, int iters, uint32_t* xcc_out, uint64_t* t_out, int peer)
{
    uint32_t xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    if (threadIdx.x == 0) xcc_out[blockIdx.x] = xcc;
    const int me = blockIdx.x == 0 ? 0 : (blockIdx.x == (unsigned)peer ? 1 : -1);
    if (me < 0 || threadIdx.x != 0) return;
    uint64_t t0 = wall_clock64();
    for (int i = 0; i < iters; ++i)
    {
        const uint32_t want = 2 * i + me;       // block 0 waits for even values, writes odd
        uint64_t guard = 0;
        while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != want)
            if (++guard > (1ull << 26)) { t_out[2] = 1; return; }
        if (MODE == 0) __hip_atomic_store(flag, want + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else __hip_atomic_store(flag, want + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    if (me == 0) t_out[0] = wall_clock64() - t0;
}
// dependent sc1 load chain over a small array (L2 resident after the first pass)
__global__ void k_chase(const uint32_t* next, int steps, uint64_t* t_out, int sc1)
{
    uint32_t p = 0;
    uint64_t t0 = wall_clock64();
    for (int i = 0; i < steps; ++i)
        p = sc1 ? __hip_atomic_load(next + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : next[p];
    t_out[0] = wall_clock64() - t0;
    t_out[1] = p;
}
int main()
{
    int khz = 0; hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0);
    uint32_t *flag, *xcc; uint64_t* t; uint32_t* next;
    hipMalloc(&flag, 4096); hipMalloc(&xcc, 4096); hipMalloc(&t, 64); hipMalloc(&next, 4 << 20);
    const int N = 1 << 18;   // 1 MB chase ring, stride 64 B lines
    uint32_t* h = (uint32_t*)malloc(4 * N);
    for (int i = 0; i < N; ++i) h[i] = 0;
    int L = N / 16; for (int i = 0; i < L; ++i) h[i * 16] = ((i * 7919 + 1) % L) * 16;
    hipMemcpy(next, h, 4 * N, hipMemcpyHostToDevice);
    for (int sc = 0; sc < 2; ++sc) for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(k_chase, 1, 1, 0, 0, next, 20000, t, sc); hipDeviceSynchronize();
        uint64_t ht[2]; hipMemcpy(ht, t, 16, hipMemcpyDeviceToHost);
        printf("chase sc1=%d rep %d: %.1f ns/load\n", sc, rep, ht[0] * 1e6 / khz / 20000.0);
    }
    for (int peer : {8, 1, 16, 9}) for (int mode = 0; mode < 2; ++mode) {
        hipMemset(flag, 0, 4); hipMemset(t, 0, 64);
        const int iters = 20000;
        if (mode == 0) hipLaunchKernelGGL(k_pp<0>, 32, 64, 0, 0, flag, iters, xcc, t, peer);
        else hipLaunchKernelGGL(k_pp<1>, 32, 64, 0, 0, flag, iters, xcc, t, peer);
        hipDeviceSynchronize();
        uint64_t ht[3]; uint32_t hx[32]; hipMemcpy(ht, t, 24, hipMemcpyDeviceToHost); hipMemcpy(hx, xcc, 128, hipMemcpyDeviceToHost);
        printf("pp peer=%d (xcc %u vs %u) mode=%d: %.1f ns per one-way hand-off%s\n", peer, hx[0], hx[peer], mode,
               ht[0] * 1e6 / khz / (2.0 * iters), ht[2] ? " TIMEOUT" : "");
    }
    return 0;
}
