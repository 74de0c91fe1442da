// mb_lean.hip — the memory pattern of lean pass 1 (k_resolve_lean, config 2) without its compute, to measure
// what one MI355X sustains for it ("measure the ceiling, then change the layout").
//
// Per item (two requests of 8 keys, as pass 1 takes them two per wave):
//   * the two 16-byte request records (consecutive requests: coalesced across items);
//   * the 16 probes' line indices (k_prepare's output: 4 bytes each, consecutive);
//   * 16 random 128-byte KeyLine lines, one 16-byte quarter per lane (4 lanes per probe), the line index
//     dependent on the probe load (the kernel's chain: record -> probe -> line);
//   * optionally a second random line per probe for the list elements that are not inline;
//   * 12 SoA size / offset words per request (the size and region-offset arrays, indexed by request);
//   * the request's CSR regions: `region_words` u32 at a per-request offset (bump-allocated).
// Keys follow Zipf(s) over n_keys (config 2: 0.99 over 1M) or are uniform. The kernel software-pipelines one
// item ahead, as pass 1 does, and runs at a chosen occupancy (LDS padding forces waves per SIMD).
//
//   hipcc --offload-arch=gfx950 -O3 -o mb_lean scripts/mb_lean.hip && ./mb_lean [items] [zipf_s]
// Prints one JSON line per variant.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <random>
#include <vector>

#define CHK(x)                                                                                      \
    do {                                                                                            \
        hipError_t e_ = (x);                                                                        \
        if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); }  \
    } while (0)

struct Cfg {
    int n_items;            // items (2 requests each)
    int extra_line;         // 1: a second random line per probe (non-inline list elements)
    int size_stores;        // 12 size / offset words per request
    int region_words;       // u32 words of CSR regions per request
    int records;            // request records + probe loads (else the line indices are computed)
};

__device__ inline uint32_t lane_id() { return __lane_id(); }

__global__ __launch_bounds__(256) void k_pattern(Cfg cfg, const uint4* __restrict__ rec, const uint32_t* __restrict__ probe,
                                                 const uint4* __restrict__ lines, uint64_t n_lines, uint32_t* __restrict__ sizes,
                                                 uint32_t* __restrict__ regions, unsigned long long* __restrict__ sink)
{
    extern __shared__ uint32_t pad[];
    const uint32_t lane = lane_id();
    const int wv = threadIdx.x >> 6;
    const int nw = (int)(gridDim.x * (blockDim.x >> 6));
    const int w0 = (int)(blockIdx.x * (blockDim.x >> 6)) + wv;
    const uint32_t p = lane >> 2, q = lane & 3;          // probe of this lane (16 per item), quarter of its line
    uint4 acc = make_uint4(0, 0, 0, 0);
    const size_t n_req = 2ull * cfg.n_items;
    // one item ahead: record + probe index
    auto load_front = [&](int it, uint4* r, uint32_t* li) {
        const int c = it < cfg.n_items ? it : cfg.n_items - 1;
        *r = lane < 2 ? rec[2 * (size_t)c + lane] : make_uint4(0, 0, 0, 0);
        if (cfg.records) *li = probe[16 * (size_t)c + p];
        else *li = (uint32_t)(((uint64_t)(16 * (size_t)c + p) * 2654435761ull) % n_lines);
    };
    int it = w0;
    uint4 r;
    uint32_t li;
    load_front(it, &r, &li);
    for (; it < cfg.n_items; it += nw)
    {
        uint4 rn;
        uint32_t lin;
        load_front(it + nw, &rn, &lin);
        // the probe's line, one quarter per lane
        const uint4 v = lines[(size_t)li * 8 + q];
        acc.x ^= v.x; acc.y += v.y; acc.z ^= v.z; acc.w += v.w;
        if (cfg.extra_line)
        {
            const uint64_t l2 = (v.x * 0x9E3779B1u + li) % n_lines;
            const uint4 u = lines[(size_t)l2 * 8 + q];
            acc.x ^= u.x; acc.w += u.w;
        }
        acc.x ^= r.x + r.y;
        // per request: 12 size / offset words (arrays indexed by request), then its regions
        const uint32_t h = (uint32_t)__popcll(__ballot(acc.x & 1));
        if (cfg.size_stores && lane < 24)
        {
            const uint32_t m = lane >> 1, rq = lane & 1;
            sizes[(size_t)m * n_req + 2 * (size_t)it + rq] = h + m;
        }
        if (cfg.region_words)
        {
            // the two requests' regions back to back (the kernel's bump allocation, one per wave-chunk)
            const size_t base = (size_t)it * 2 * cfg.region_words;
            for (int w = (int)lane; w < 2 * cfg.region_words; w += 64) regions[base + w] = h ^ (uint32_t)w;
        }
        r = rn;
        li = lin;
    }
    if (cfg.n_items < 0) pad[threadIdx.x] = 0;
    const unsigned long long s = acc.x ^ acc.y ^ acc.z ^ acc.w;
    if (s == 0x1234567ull) sink[0] = s;          // keep the loads
}

int main(int argc, char** argv)
{
    const int n_items = argc > 1 ? atoi(argv[1]) : 500000;
    const double zipf_s = argc > 2 ? atof(argv[2]) : 0.99;
    const uint64_t n_keys = 1u << 20;                 // ~config 2's 894k keys with CommandsForKeys
    const uint64_t n_lines = n_keys * 5 / 4;          // the perfect hash's table (80 % full)
    // Zipf(s) probes: inverse CDF on the host
    std::vector<double> cdf(n_keys);
    double acc = 0;
    for (uint64_t k = 0; k < n_keys; ++k) { acc += 1.0 / std::pow((double)(k + 1), zipf_s); cdf[k] = acc; }
    std::mt19937_64 g(42);
    std::uniform_real_distribution<double> U(0, acc);
    std::vector<uint32_t> perm(n_keys);
    for (uint64_t k = 0; k < n_keys; ++k) perm[k] = (uint32_t)((k * 0x9E3779B97F4A7C15ull) % n_lines);   // rank -> line
    std::vector<uint32_t> probe(16ull * n_items);
    for (auto& x : probe)
    {
        const double u = zipf_s > 0 ? U(g) : 0;
        const uint64_t k = zipf_s > 0 ? (uint64_t)(std::lower_bound(cdf.begin(), cdf.end(), u) - cdf.begin())
                                      : (uint64_t)(g() % n_keys);
        x = perm[std::min<uint64_t>(k, n_keys - 1)];
    }
    uint4 *d_rec, *d_lines;
    uint32_t *d_probe, *d_sizes, *d_regions;
    unsigned long long* d_sink;
    const int region_words_max = 48;
    CHK(hipMalloc(&d_rec, sizeof(uint4) * 2 * n_items));
    CHK(hipMalloc(&d_lines, 128 * n_lines));
    CHK(hipMalloc(&d_probe, 4ull * probe.size()));
    CHK(hipMalloc(&d_sizes, 4ull * 12 * 2 * n_items));
    CHK(hipMalloc(&d_regions, 4ull * 2 * n_items * region_words_max));
    CHK(hipMalloc(&d_sink, 8));
    CHK(hipMemset(d_rec, 1, sizeof(uint4) * 2 * n_items));
    CHK(hipMemset(d_lines, 3, 128 * n_lines));
    CHK(hipMemcpy(d_probe, probe.data(), 4ull * probe.size(), hipMemcpyHostToDevice));
    hipDeviceProp_t prop;
    CHK(hipGetDeviceProperties(&prop, 0));
    const int n_cu = prop.multiProcessorCount;
    struct V { const char* name; Cfg c; int waves_per_simd; };
    const V vs[] = {
        {"lines_only", {n_items, 0, 0, 0, 0}, 4},
        {"records_probes_lines", {n_items, 0, 0, 0, 1}, 4},
        {"+size_stores", {n_items, 0, 1, 0, 1}, 4},
        {"+regions_22w", {n_items, 0, 1, 22, 1}, 4},
        {"+regions_22w_extra_line", {n_items, 1, 1, 22, 1}, 4},
        {"+regions_22w@8wps", {n_items, 0, 1, 22, 1}, 8},
        {"+regions_22w@2wps", {n_items, 0, 1, 22, 1}, 2},
    };
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    for (const V& v : vs)
    {
        // waves per SIMD through LDS padding: 160 KB per CU shared by 4 * wps waves = wps blocks of 4 waves
        const size_t lds = std::min<size_t>((size_t)(160 * 1024) / (size_t)v.waves_per_simd, 65536) - 256;
        const int blocks = n_cu * v.waves_per_simd;
        CHK(hipFuncSetAttribute((const void*)k_pattern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        float best = 1e9f;
        for (int rep = 0; rep < 12; ++rep)
        {
            CHK(hipEventRecord(a, 0));
            k_pattern<<<blocks, 256, lds, 0>>>(v.c, d_rec, d_probe, d_lines, n_lines, d_sizes, d_regions, d_sink);
            CHK(hipEventRecord(b, 0));
            CHK(hipEventSynchronize(b));
            float ms = 0;
            CHK(hipEventElapsedTime(&ms, a, b));
            if (rep >= 2 && ms < best) best = ms;
        }
        const double lines = 16.0 * n_items * (1 + v.c.extra_line);
        const double bytes_read = lines * 128 + (v.c.records ? n_items * (32.0 + 64.0) : 0);
        const double bytes_written = (v.c.size_stores ? 2.0 * n_items * 48 : 0) + 2.0 * n_items * 4 * v.c.region_words;
        printf("{\"variant\": \"%s\", \"items\": %d, \"zipf_s\": %.2f, \"waves_per_simd\": %d, \"ms\": %.4f, "
               "\"lines_per_s\": %.4g, \"gb_s_lines\": %.1f, \"gb_s_moved\": %.1f}\n",
               v.name, n_items, zipf_s, v.waves_per_simd, best, lines / (best * 1e-3), lines * 128 / (best * 1e6),
               (bytes_read + bytes_written) / (best * 1e6));
        fflush(stdout);
    }
    return 0;
}
