// region_probe.hip — random 8-byte reads of a 4 GB table (the join probe's pattern,
// k_random_read) when the reads in flight are confined to regions of the table:
// what a probe side partitioned by table region could gain from L2 / MALL locality.
// Each block reads `per_block` random slots inside one region; blocks map to
// regions either consecutively (a region's blocks spread over the 8 XCDs) or
// XCD-aware (a region's blocks on one XCD, so its lines meet in one L2).
//   hipcc --offload-arch=gfx950 -O3 tools/region_probe.hip -o tools/region_probe && tools/region_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e = (x);                                                     \
        if (e != hipSuccess) {                                                  \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));              \
            exit(1);                                                            \
        }                                                                       \
    } while (0)

__device__ __forceinline__ unsigned long long mix(unsigned long long x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

__device__ __forceinline__ unsigned xcd_tile(unsigned b, unsigned g) {
    const unsigned q = g >> 3, r = g & 7u, x = b & 7u;
    return x * q + (x < r ? x : r) + (b >> 3);
}

template <bool XCD>
__global__ __launch_bounds__(256) void k_region(const unsigned long long* __restrict__ t, int region_log2,
                                                unsigned blocks_per_region, unsigned per_thread,
                                                unsigned long long* __restrict__ sink) {
    const unsigned b = XCD ? xcd_tile(blockIdx.x, gridDim.x) : blockIdx.x;
    const unsigned long long region = b / blocks_per_region;
    const unsigned long long base = region << region_log2, mask = (1ull << region_log2) - 1;
    unsigned long long acc = 0, seed = ((unsigned long long)blockIdx.x << 32) ^ (threadIdx.x * 0x9E37ull);
    for (unsigned i = 0; i < per_thread; i += 8) {
        unsigned long long v[8];
#pragma unroll
        for (int u = 0; u < 8; u++) v[u] = t[base + (mix(seed + i + u) & mask)];
#pragma unroll
        for (int u = 0; u < 8; u++) acc += v[u];
    }
    if (acc == 0x12345) sink[0] = acc;
}

int main() {
    const int slots_log2 = 29;  // 2^29 x 8 B = 4 GB, the 2^28-row join table
    const unsigned long long slots = 1ull << slots_log2, reads = 1ull << 28;
    unsigned long long *t, *sink;
    CK(hipMalloc(&t, slots * 8));
    CK(hipMalloc(&sink, 8));
    CK(hipMemset(t, 1, slots * 8));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const unsigned G = 8192, per_thread = (unsigned)(reads / G / 256);
    for (int xcd = 0; xcd < 2; xcd++) {
        for (int rl = slots_log2; rl >= 16; rl -= (rl > 22 ? 2 : 1)) {  // region of 2^rl slots
            const unsigned regions = 1u << (slots_log2 - rl);
            const unsigned bpr = G / regions ? G / regions : 1;
            float best = 1e9f;
            for (int rep = 0; rep < 4; rep++) {
                CK(hipEventRecord(a));
                if (xcd)
                    hipLaunchKernelGGL(k_region<true>, dim3(G), dim3(256), 0, 0, t, rl, bpr, per_thread, sink);
                else
                    hipLaunchKernelGGL(k_region<false>, dim3(G), dim3(256), 0, 0, t, rl, bpr, per_thread, sink);
                CK(hipEventRecord(b));
                CK(hipEventSynchronize(b));
                float ms;
                CK(hipEventElapsedTime(&ms, a, b));
                if (ms < best) best = ms;
            }
            printf("%s region %8.1f MB (%5u regions): %7.3f ms for 2^28 reads = %6.1f G reads/s\n",
                   xcd ? "xcd-aware  " : "consecutive", (double)(8ull << rl) / 1048576.0, regions, best,
                   (double)reads / best / 1e6);
        }
    }
    return 0;
}
