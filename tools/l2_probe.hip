// l2_probe.hip — what an L2-partitioned join probe could gain (not product code;
// VERDICT r03 next-4). The 2^28 unique probe reads one random 32-byte bucket of a
// 4 GB table per probe row (k_ht_probe_unique: 7.2-7.5 ms, 5.2-5.6 ms of which is the
// random-request ceiling). Partitioning the probe rows by table slice would make each
// slice's reads L2 hits, at the price of a partition pass before and a pass restoring
// probe order after. Timed here, each with HIP events (median of 5 after 2 warm-ups):
//   random     2^28 random 32-byte bucket reads over the whole 2^29-slot table
//   part<MB>   the same reads grouped by slice: the 8 XCDs each take slices in turn
//              (slice = round * 8 + xcd) and the 256 blocks of an XCD read only their
//              current slice, so a slice's lines stay in that XCD's 4 MB L2;
//   scatter    2^28 random 4-byte stores into a 1 GB array (putting the probe's
//              results back in probe order by row index);
//   stream     2^28 x 8 bytes read and written in order (one partition pass's floor).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/l2_probe.hip -o tools/l2_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                    \
    do {                                                                         \
        hipError_t e = (x);                                                      \
        if (e != hipSuccess) {                                                   \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));               \
            exit(1);                                                             \
        }                                                                        \
    } while (0)

typedef unsigned long long u64;

__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

// n random bucket reads (two 16-byte loads) at slot (mix(i) & mask) & ~3, 2 in flight per lane
__global__ __launch_bounds__(256) void k_random(const u64* __restrict__ t, uint64_t mask, uint64_t n,
                                                u64* __restrict__ out) {
    u64 acc = 0;
    const uint64_t stride = (uint64_t)gridDim.x * 512;
    for (uint64_t i0 = (uint64_t)blockIdx.x * 512 + threadIdx.x; i0 < n; i0 += stride) {
        ulonglong2 a[2], b[2];
#pragma unroll
        for (int u = 0; u < 2; u++) {
            const uint64_t i = i0 + (uint64_t)u * 256;
            const uint64_t h = (uint64_t)mix((uint32_t)i) & mask & ~3ull;
            const ulonglong2* q = reinterpret_cast<const ulonglong2*>(t + h);
            a[u] = q[0];
            b[u] = q[1];
        }
#pragma unroll
        for (int u = 0; u < 2; u++) acc ^= a[u].x ^ a[u].y ^ b[u].x ^ b[u].y;
    }
    if (acc == 0x123456789ull) out[0] = acc;
}

// The same number of reads, slice by slice: nslice slices of 2^slog slots; XCD x (block
// b runs on XCD b % 8) takes slices x, x + 8, ...; its blocks split each slice's reads.
__global__ __launch_bounds__(256) void k_part(const u64* __restrict__ t, int slog, uint32_t nslice, uint64_t n,
                                              u64* __restrict__ out) {
    const uint32_t xcd = blockIdx.x & 7u, lb = blockIdx.x >> 3, nb = gridDim.x >> 3;
    const uint64_t per = n / nslice;  // reads per slice
    const uint64_t smask = (1ull << slog) - 1;
    u64 acc = 0;
    for (uint32_t s = xcd; s < nslice; s += 8) {
        const u64* base = t + ((uint64_t)s << slog);
        for (uint64_t i0 = (uint64_t)lb * 512 + threadIdx.x; i0 < per; i0 += (uint64_t)nb * 512) {
            ulonglong2 a[2], b[2];
#pragma unroll
            for (int u = 0; u < 2; u++) {
                const uint64_t i = i0 + (uint64_t)u * 256 + (uint64_t)s * per;
                const uint64_t h = (uint64_t)mix((uint32_t)i) & smask & ~3ull;
                const ulonglong2* q = reinterpret_cast<const ulonglong2*>(base + h);
                a[u] = q[0];
                b[u] = q[1];
            }
#pragma unroll
            for (int u = 0; u < 2; u++) acc ^= a[u].x ^ a[u].y ^ b[u].x ^ b[u].y;
        }
    }
    if (acc == 0x123456789ull) out[0] = acc;
}

// n random 4-byte stores: out[mix(i) & mask] = i
__global__ __launch_bounds__(256) void k_scatter(uint32_t* __restrict__ a, uint64_t mask, uint64_t n) {
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride)
        a[(uint64_t)mix((uint32_t)i * 2654435761u) & mask] = (uint32_t)i;
}

// n 8-byte words read and written in order (16-byte accesses)
__global__ __launch_bounds__(256) void k_stream(const ulonglong2* __restrict__ in, ulonglong2* __restrict__ out,
                                                uint64_t n2) {
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n2; i += stride) out[i] = in[i];
}

template <typename F>
float timed(F f) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    std::vector<float> ms;
    for (int r = 0; r < 7; r++) {
        CK(hipEventRecord(a));
        f();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float x;
        CK(hipEventElapsedTime(&x, a, b));
        if (r >= 2) ms.push_back(x);
    }
    std::sort(ms.begin(), ms.end());
    return ms[ms.size() / 2];
}

int main() {
    const int lslots = 29;  // the 2^28 join's table: 2^29 8-byte slots, 4 GB
    const uint64_t S = 1ull << lslots, N = 1ull << 28;
    u64 *t, *o;
    uint32_t* sc;
    CK(hipMalloc(&t, S * 8));
    CK(hipMalloc(&o, 64));
    CK(hipMalloc(&sc, N * 4));
    CK(hipMemset(t, 1, S * 8));
    CK(hipMemset(sc, 0, N * 4));
    hipDeviceProp_t pr;
    CK(hipGetDeviceProperties(&pr, 0));
    const int grid = pr.multiProcessorCount * 8;
    printf("{\"what\":\"random\",\"reads\":%llu,\"table_mb\":%llu,\"ms\":%.3f}\n", (unsigned long long)N,
           (unsigned long long)(S * 8 >> 20),
           timed([&] { hipLaunchKernelGGL(k_random, dim3(grid), dim3(256), 0, 0, t, S - 1, N, o); }));
    for (int slog : {15, 16, 17, 18, 19, 20}) {  // slices of 256 KB .. 8 MB
        const uint32_t ns = (uint32_t)(S >> slog);
        printf("{\"what\":\"part\",\"slice_mb\":%.2f,\"slices\":%u,\"ms\":%.3f}\n", (double)(8ull << slog) / (1 << 20),
               ns, timed([&] { hipLaunchKernelGGL(k_part, dim3(grid), dim3(256), 0, 0, t, slog, ns, N, o); }));
    }
    printf("{\"what\":\"scatter\",\"stores\":%llu,\"array_mb\":%llu,\"ms\":%.3f}\n", (unsigned long long)N,
           (unsigned long long)(N * 4 >> 20),
           timed([&] { hipLaunchKernelGGL(k_scatter, dim3(grid), dim3(256), 0, 0, sc, N - 1, N); }));
    ulonglong2* w = reinterpret_cast<ulonglong2*>(t);
    printf("{\"what\":\"stream\",\"words\":%llu,\"ms\":%.3f}\n", (unsigned long long)N,
           timed([&] { hipLaunchKernelGGL(k_stream, dim3(grid), dim3(256), 0, 0, w, w + N / 2, N / 2); }));
    return 0;
}
