// mix_probe.hip — the memory floor of shared_select's single-pass count (not product
// code). k_ssk_count streams the 4 GB column and, per 1024-row group, appends the
// group's (query, row) pairs to its wave's slice of the workspace: 1.6 % of the rows
// at Q = 16, 15 % at Q = 150 (0.1 % ranges), 4 bytes a pair. This kernel does only
// that memory traffic, in the same geometry (1024 blocks of 4 waves, a contiguous
// chunk of rows per wave, 16 nontemporal dword loads a lane per group, the group's
// pairs as full-wave u32 stores to the wave's slice), so the count pass's time can be
// read against what its bytes alone cost. HIP events, median of 5 after 2 warm-ups.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mix_probe.hip -o tools/mix_probe
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

// rows per wave = rpw (a multiple of 1024); npg pairs written per 1024-row group.
// B: the pairs of B groups go out together (4 B buffer stores, after the loads of the
// group that closes the batch); AUX: the stores' cache policy bits (2 = nontemporal)
template <int B, int AUX>
__global__ __launch_bounds__(256) void k_mix(const int* __restrict__ col, uint64_t rpw, uint32_t npg,
                                             uint32_t* __restrict__ pairs, uint64_t cap, int* __restrict__ sink,
                                             uint32_t wmask) {
    const int lane = threadIdx.x & 63;
    const uint64_t w = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int* c = col + w * rpw;
    uint32_t* list = pairs + w * cap;
    // as k_ssk_count: pairs go out after a group's loads, as buffer stores whose range
    // drops the unused lanes (a fixed count)
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(list, 0, (int)(cap * 4), 0x00020000);
    uint32_t run = 0, pend = 0;
    int acc = 0;
    uint64_t g = 0;
    for (uint64_t t = 0; t < rpw; t += 1024, g++) {
        int v[16];
#pragma unroll
        for (int i = 0; i < 16; i++) v[i] = __builtin_nontemporal_load(c + t + (uint64_t)i * 64 + lane);
        if (g % B == 0) {
#pragma unroll
            for (int k = 0; k < 4 * B; k++) {
                const uint32_t i = (uint32_t)(k * 64 + lane);
                __builtin_amdgcn_raw_buffer_store_b32((uint32_t)acc + i, rs,
                                                      i < pend ? (int)(((run - pend + i) & wmask) * 4u) : (int)0x80000000u, 0, AUX);
            }
            pend = 0;
        }
#pragma unroll
        for (int i = 0; i < 16; i++) acc ^= v[i];
        pend += npg;
        run += npg;
    }
    if (acc == 0x7fffffff) sink[0] = acc;
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
    const uint64_t waves = 4096, rpw = 244736;  // 1024 blocks x 4 waves, 239 groups a wave
    const uint64_t n = waves * rpw;             // 1.0024e9 rows, 4.0 GB
    int *col, *sink;
    uint32_t* pairs;
    const uint64_t cap = rpw / 4;  // up to 256 pairs a group
    CK(hipMalloc(&col, n * 4));
    CK(hipMalloc(&sink, 64));
    CK(hipMalloc(&pairs, waves * cap * 4));
    CK(hipMemset(col, 1, n * 4));
    // wmask: a wave's pairs wrap within its first wmask + 1 entries (MIX_WRAP runs 1 K
    // entries a wave = 16 MB in all, L2-sized, and 8 K = 128 MB, MALL-sized): whether the
    // cost of a write stream inside the read stream is in HBM or before it
    auto go = [&](const char* form, auto kern, uint32_t npg, uint32_t wmask = 0xffffffffu) {
        const float ms = timed([&] { hipLaunchKernelGGL(kern, dim3(1024), dim3(256), 0, 0, col, rpw, npg, pairs, cap, sink, wmask); });
        const double rb = 4.0 * n, wb = 4.0 * npg * (double)(n / 1024);
        printf("{\"what\":\"mix\",\"form\":\"%s\",\"rows\":%llu,\"pairs_per_1024\":%u,\"read_gb\":%.3f,"
               "\"write_gb\":%.3f,\"ms\":%.3f,\"tbs\":%.2f}\n",
               form, (unsigned long long)n, npg, rb / 1e9, wb / 1e9, ms, (rb + wb) / ms / 1e9);
    };
    const bool all = getenv("MIX_ALL") != nullptr;
    for (uint32_t npg : {0u, 16u, 64u, 154u, 256u}) go("per_group", k_mix<1, 0>, npg);
    if (getenv("MIX_WRAP")) {
        for (uint32_t npg : {16u, 154u}) {
            go("wrap_1k", k_mix<1, 0>, npg, 1023u);
            go("wrap_8k", k_mix<1, 0>, npg, 8191u);
            go("wrap_1k_nt", k_mix<1, 2>, npg, 1023u);
        }
    }
    if (all) {
        for (uint32_t npg : {16u, 154u}) {
            go("per_group_nt", k_mix<1, 2>, npg);
            go("batch4", k_mix<4, 0>, npg);
            go("batch16", k_mix<16, 0>, npg);
        }
    }
    return 0;
}
