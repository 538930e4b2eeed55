// mq_kernels.hip — gfx950 (MI355X, CDNA4) kernels behind the libmq device C-ABI
// (include/mq_device.h).
//
// The hot path of siyaoL1/Analytical-Database's src/query.c — range select,
// position-list fetch, sum/avg/min/max, add/sub — rebuilt as HBM-streaming
// filter/reduce kernels. Nothing here is a contraction, so nothing here uses
// MFMA; the limits are HBM bandwidth and, for ordered compaction, the number
// of passes over the column.
//
// Layout and decomposition:
//   * a column is a contiguous int32 array in HBM; a scan launches one block of
//     256 threads (4 wave64) per resident slot (CUs x occupancy), and block b
//     owns the contiguous row chunk [b*R, (b+1)*R), R a multiple of 1024;
//   * a tile is 1024 rows: each lane reads one dwordx4 (4 consecutive rows), so a
//     wave covers 256 consecutive rows and one load instruction moves 1 KiB;
//   * kUnroll tiles are loaded before any is consumed, so every lane keeps
//     kUnroll x 16 B in flight;
//   * per-block partial aggregates go to a workspace slab and a one-block kernel
//     combines them (no atomics, bitwise deterministic).
// Ordered compaction (select_column_scan's ascending position list,
// query.c:92-137) is two kernels: k_scan<MASK> writes one predicate bit per row
// (wave ballots, N/8 bytes) plus per-block counts; k_compact turns the bits into
// positions at offsets from an in-block prefix over the block counts. HBM
// traffic is 4N + N/8 + N/8 + 4K bytes for N rows and K matches.

#include <hip/hip_runtime.h>

#include <climits>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstring>

#include "mq_common.h"
#include "mq_device.h"

namespace {

constexpr int kTPB = 256;                 // scan block: 4 wave64
constexpr int kWaves = kTPB / 64;
constexpr int kTileRows = kTPB * 4;       // 1024 rows per tile (one dwordx4 per lane)
constexpr int kUnroll = 4;                // tiles in flight per thread
constexpr int kCompactTPB = 1024;         // compaction block: 16 wave64
constexpr int kCompactWaves = kCompactTPB / 64;
constexpr int kGroupsPerBatch = 16;       // 16 groups (256 rows each) per wave load
constexpr int kBatchesPerWave = 8;        // 128 groups per wave per round
constexpr int kMaxBlocks = 8192;

struct Partial {                          // 32 B, layout-identical to mq_agg
    unsigned long long count;
    long long sum;
    int mn;
    int mx;
    unsigned long long pad;
};
static_assert(sizeof(Partial) == sizeof(mq_agg), "Partial must mirror mq_agg");

// v matches when (uint32)(v - lo) <= wm1: one compare for low <= v < high
// (the host folds NULL bounds and empty ranges; see make_pred).
struct Pred {
    uint32_t lo;
    uint32_t wm1;
};

__device__ __forceinline__ bool match(int v, Pred p) { return ((uint32_t)v - p.lo) <= p.wm1; }

template <bool VEC>
__device__ __forceinline__ int4 load4(const int* __restrict__ p) {
    if constexpr (VEC) {
        return *reinterpret_cast<const int4*>(p);
    } else {
        return make_int4(p[0], p[1], p[2], p[3]);
    }
}

__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}
__device__ __forceinline__ long long wave_sum_i64(long long v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}
__device__ __forceinline__ int wave_min(int v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = min(v, __shfl_xor(v, off, 64));
    return v;
}
__device__ __forceinline__ int wave_max(int v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = max(v, __shfl_xor(v, off, 64));
    return v;
}

// Block-wide combine of per-thread aggregates into part[blockIdx.x].
__device__ __forceinline__ void block_store_partial(unsigned long long cnt, long long sum, int mn,
                                                    int mx, Partial* __restrict__ part) {
    __shared__ Partial sp[kWaves];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    cnt = wave_sum_u64(cnt);
    sum = wave_sum_i64(sum);
    mn = wave_min(mn);
    mx = wave_max(mx);
    if (lane == 0) sp[wave] = Partial{cnt, sum, mn, mx, 0ull};
    __syncthreads();
    if (threadIdx.x == 0) {
        Partial r = sp[0];
#pragma unroll
        for (int w = 1; w < kWaves; w++) {
            r.count += sp[w].count;
            r.sum += sp[w].sum;
            r.mn = min(r.mn, sp[w].mn);
            r.mx = max(r.mx, sp[w].mx);
        }
        part[blockIdx.x] = r;
    }
}

// ---------------------------------------------------------------------------
// k_scan: one streaming pass over a contiguous chunk of the column.
//   MASK = false: count / int64 sum / min / max of the matching values — or, with
//                 AUX, of aux[row] for the matching rows (select -> fetch -> agg
//                 fused, config 3). Implements query.c:92-137 + 223-243 + 306-354.
//   MASK = true : count per block + one predicate bit per row (first half of the
//                 ordered compaction).
// Mask word layout: masks[(tile*4 + wave)*4 + e] bit l = row tile*1024 + wave*256
// + 4*l + e, so a chunk's 256-row groups are contiguous 32-byte records.
// ---------------------------------------------------------------------------
template <bool MASK, bool AUX, bool VEC>
__global__ __launch_bounds__(kTPB) void k_scan(const int* __restrict__ col,
                                               const int* __restrict__ aux, uint64_t n,
                                               uint64_t rows_per_block, Pred pred,
                                               Partial* __restrict__ part,
                                               unsigned long long* __restrict__ masks) {
    const uint64_t start = (uint64_t)blockIdx.x * rows_per_block;
    uint64_t end = start + rows_per_block;
    if (end > n) end = n;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;

    unsigned int cnt = 0;
    long long sum = 0;
    int mn = INT_MAX, mx = INT_MIN;

    auto consume = [&](int4 v, uint64_t tile_row, bool full) {
        const uint64_t row = tile_row + (uint64_t)tid * 4;
        bool p0 = match(v.x, pred), p1 = match(v.y, pred), p2 = match(v.z, pred),
             p3 = match(v.w, pred);
        if (!full) {
            p0 = p0 && (row + 0 < end);
            p1 = p1 && (row + 1 < end);
            p2 = p2 && (row + 2 < end);
            p3 = p3 && (row + 3 < end);
        }
        cnt += (unsigned)p0 + (unsigned)p1 + (unsigned)p2 + (unsigned)p3;
        if constexpr (MASK) {
            const unsigned long long m0 = __ballot(p0), m1 = __ballot(p1), m2 = __ballot(p2),
                                     m3 = __ballot(p3);
            if (lane < 4) {
                const unsigned long long m = lane == 0 ? m0 : lane == 1 ? m1 : lane == 2 ? m2 : m3;
                masks[((tile_row / kTileRows) * kWaves + wave) * 4 + lane] = m;
            }
        } else {
            int a0 = v.x, a1 = v.y, a2 = v.z, a3 = v.w;
            if constexpr (AUX) {
                a0 = p0 ? aux[row + 0] : 0;
                a1 = p1 ? aux[row + 1] : 0;
                a2 = p2 ? aux[row + 2] : 0;
                a3 = p3 ? aux[row + 3] : 0;
            }
            sum += (long long)(p0 ? a0 : 0) + (long long)(p1 ? a1 : 0) +
                   (long long)(p2 ? a2 : 0) + (long long)(p3 ? a3 : 0);
            mn = min(mn, min(min(p0 ? a0 : INT_MAX, p1 ? a1 : INT_MAX),
                             min(p2 ? a2 : INT_MAX, p3 ? a3 : INT_MAX)));
            mx = max(mx, max(max(p0 ? a0 : INT_MIN, p1 ? a1 : INT_MIN),
                             max(p2 ? a2 : INT_MIN, p3 ? a3 : INT_MIN)));
        }
    };

    uint64_t t = start;
    // Full groups of kUnroll tiles: all loads issued before the first use.
    for (; t + (uint64_t)kUnroll * kTileRows <= end; t += (uint64_t)kUnroll * kTileRows) {
        int4 v[kUnroll];
#pragma unroll
        for (int u = 0; u < kUnroll; u++)
            v[u] = load4<VEC>(col + t + (uint64_t)u * kTileRows + (uint64_t)tid * 4);
#pragma unroll
        for (int u = 0; u < kUnroll; u++) consume(v[u], t + (uint64_t)u * kTileRows, true);
    }
    // Remaining tiles (the chunk tail), bounds-checked per row.
    for (; t < end; t += kTileRows) {
        const uint64_t row = t + (uint64_t)tid * 4;
        int4 v;
        if (row + 3 < end) {
            v = load4<VEC>(col + row);
        } else {
            v.x = row + 0 < end ? col[row + 0] : 0;
            v.y = row + 1 < end ? col[row + 1] : 0;
            v.z = row + 2 < end ? col[row + 2] : 0;
            v.w = row + 3 < end ? col[row + 3] : 0;
        }
        consume(v, t, row + 3 < end);
    }
    block_store_partial(cnt, sum, mn, mx, part);
}

// One block combines the per-block partials into the final aggregate.
__global__ __launch_bounds__(kTPB) void k_final(const Partial* __restrict__ part, uint32_t nparts,
                                                mq_agg* __restrict__ out) {
    unsigned long long cnt = 0;
    long long sum = 0;
    int mn = INT_MAX, mx = INT_MIN;
    for (uint32_t i = threadIdx.x; i < nparts; i += kTPB) {
        const Partial p = part[i];
        cnt += p.count;
        sum += p.sum;
        mn = min(mn, p.mn);
        mx = max(mx, p.mx);
    }
    __shared__ Partial sp[kWaves];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    cnt = wave_sum_u64(cnt);
    sum = wave_sum_i64(sum);
    mn = wave_min(mn);
    mx = wave_max(mx);
    if (lane == 0) sp[wave] = Partial{cnt, sum, mn, mx, 0ull};
    __syncthreads();
    if (threadIdx.x == 0) {
        Partial r = sp[0];
        for (int w = 1; w < kWaves; w++) {
            r.count += sp[w].count;
            r.sum += sp[w].sum;
            r.mn = min(r.mn, sp[w].mn);
            r.mx = max(r.mx, sp[w].mx);
        }
        out->count = r.count;
        out->sum = r.sum;
        out->min = r.mn;
        out->max = r.mx;
        out->_pad = 0;
    }
}

// ---------------------------------------------------------------------------
// k_compact: predicate bits -> ascending position list (second half of the
// ordered compaction). Block b re-walks the chunk of scan block b. Its output
// offset is the sum of the counts of blocks 0..b-1. Inside the block, 16 waves
// take contiguous runs of 256-row groups; a wave loads 16 groups (64 mask words)
// per instruction, popcounts them, and a wave-wide scan gives each group's
// offset. Every lane then writes its own rows' positions (or payload[row], for
// select_result's prior positions, query.c:38-86) in ascending row order.
// ---------------------------------------------------------------------------
template <bool PAYLOAD>
__global__ __launch_bounds__(kCompactTPB) void k_compact(
    const unsigned long long* __restrict__ masks, const Partial* __restrict__ part,
    const int* __restrict__ payload, uint64_t n, uint64_t rows_per_block, int* __restrict__ out,
    unsigned long long* __restrict__ d_count) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    __shared__ unsigned long long s_red[kCompactWaves];
    __shared__ unsigned long long s_wtot[kCompactWaves];

    // Output base = sum of the counts of the preceding blocks.
    unsigned long long acc = 0;
    for (uint32_t i = tid; i < blockIdx.x; i += kCompactTPB) acc += part[i].count;
    acc = wave_sum_u64(acc);
    if (lane == 0) s_red[wave] = acc;
    __syncthreads();
    unsigned long long base = 0;
#pragma unroll
    for (int w = 0; w < kCompactWaves; w++) base += s_red[w];
    const unsigned long long mine = part[blockIdx.x].count;
    if (blockIdx.x == gridDim.x - 1 && tid == 0) *d_count = base + mine;
    if (mine == 0) return;  // uniform across the block

    const uint64_t start = (uint64_t)blockIdx.x * rows_per_block;
    uint64_t end = start + rows_per_block;
    if (end > n) end = n;
    const uint64_t ngroups = ((end - start + kTileRows - 1) / kTileRows) * kWaves;
    const unsigned long long* cmask = masks + (start / kTileRows) * kWaves * 4;
    constexpr uint64_t kGroupsPerWave = (uint64_t)kGroupsPerBatch * kBatchesPerWave;
    constexpr uint64_t kGroupsPerRound = kGroupsPerWave * kCompactWaves;

    unsigned long long running = base;
    for (uint64_t r0 = 0; r0 < ngroups; r0 += kGroupsPerRound) {
        const uint64_t g0 = r0 + (uint64_t)wave * kGroupsPerWave;
        // Phase A: this wave's match total over its 128 groups (8 loads in flight).
        unsigned long long wtot = 0;
#pragma unroll
        for (int bb = 0; bb < kBatchesPerWave; bb++) {
            const uint64_t g = g0 + (uint64_t)bb * kGroupsPerBatch + (uint64_t)(lane >> 2);
            const unsigned long long w = g < ngroups ? cmask[g * 4 + (lane & 3)] : 0ull;
            wtot += (unsigned long long)__popcll(w);
        }
        wtot = wave_sum_u64(wtot);
        __syncthreads();  // s_wtot reuse across rounds
        if (lane == 0) s_wtot[wave] = wtot;
        __syncthreads();
        unsigned long long woff = running, rtot = 0;
#pragma unroll
        for (int w = 0; w < kCompactWaves; w++) {
            const unsigned long long x = s_wtot[w];
            if (w < wave) woff += x;
            rtot += x;
        }
        running += rtot;
        if (wtot == 0) continue;  // uniform within the wave

        // Phase B: write positions, batch by batch (mask words re-read from cache).
        for (int bb = 0; bb < kBatchesPerWave; bb++) {
            const uint64_t gb = g0 + (uint64_t)bb * kGroupsPerBatch;
            if (gb >= ngroups) break;
            const uint64_t g = gb + (uint64_t)(lane >> 2);
            const unsigned long long w = g < ngroups ? cmask[g * 4 + (lane & 3)] : 0ull;
            const unsigned int c = (unsigned int)__popcll(w);
            // inclusive scan of c across the 64 lanes (group-major, word-minor)
            unsigned int incl = c;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const unsigned int y = __shfl_up(incl, off, 64);
                if (lane >= off) incl += y;
            }
            const unsigned int btot = __shfl(incl, 63, 64);
            if (btot == 0) continue;
            const unsigned long long ltmask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
            for (int j = 0; j < kGroupsPerBatch; j++) {
                const unsigned int gend = __shfl(incl, 4 * j + 3, 64);
                const unsigned int gbeg = (j == 0) ? 0u : __shfl(incl, 4 * j - 1, 64);
                if (gend == gbeg) continue;
                const unsigned long long w0 = __shfl(w, 4 * j + 0, 64);
                const unsigned long long w1 = __shfl(w, 4 * j + 1, 64);
                const unsigned long long w2 = __shfl(w, 4 * j + 2, 64);
                const unsigned long long w3 = __shfl(w, 4 * j + 3, 64);
                const unsigned int b0 = (unsigned int)(w0 >> lane) & 1u;
                const unsigned int b1 = (unsigned int)(w1 >> lane) & 1u;
                const unsigned int b2 = (unsigned int)(w2 >> lane) & 1u;
                const unsigned int b3 = (unsigned int)(w3 >> lane) & 1u;
                const unsigned int pre = (unsigned int)(__popcll(w0 & ltmask) + __popcll(w1 & ltmask) +
                                                        __popcll(w2 & ltmask) + __popcll(w3 & ltmask));
                const uint64_t gidx = gb + (uint64_t)j;
                const uint64_t row = start + (gidx >> 2) * kTileRows + (gidx & 3) * 256 +
                                     (uint64_t)lane * 4;
                int* o = out + woff + gbeg + pre;
                unsigned int k = 0;
                if (b0) o[k++] = PAYLOAD ? payload[row + 0] : (int)(row + 0);
                if (b1) o[k++] = PAYLOAD ? payload[row + 1] : (int)(row + 1);
                if (b2) o[k++] = PAYLOAD ? payload[row + 2] : (int)(row + 2);
                if (b3) o[k++] = PAYLOAD ? payload[row + 3] : (int)(row + 3);
            }
            woff += btot;
        }
    }
}

// ---------------------------------------------------------------------------
// fetch (query.c:223-243): out[i] = col[pos[i]], 4 positions per lane.
// ---------------------------------------------------------------------------
template <bool VEC>
__global__ __launch_bounds__(kTPB) void k_fetch(const int* __restrict__ col,
                                                const int* __restrict__ pos, uint64_t k,
                                                int* __restrict__ out) {
    const uint64_t stride = (uint64_t)gridDim.x * kTPB;
    const uint64_t k4 = k / 4;
    for (uint64_t i = (uint64_t)blockIdx.x * kTPB + threadIdx.x; i < k4; i += stride) {
        const int4 p = load4<VEC>(pos + i * 4);
        int4 o;
        o.x = col[p.x];
        o.y = col[p.y];
        o.z = col[p.z];
        o.w = col[p.w];
        if constexpr (VEC) {
            *reinterpret_cast<int4*>(out + i * 4) = o;
        } else {
            out[i * 4 + 0] = o.x;
            out[i * 4 + 1] = o.y;
            out[i * 4 + 2] = o.z;
            out[i * 4 + 3] = o.w;
        }
    }
    if (blockIdx.x == 0 && threadIdx.x < (k & 3)) {
        const uint64_t i = k4 * 4 + threadIdx.x;
        out[i] = col[pos[i]];
    }
}

// add / sub (query.c:356-390), two's-complement wrap.
template <bool SUB, bool VEC>
__global__ __launch_bounds__(kTPB) void k_addsub(const int* __restrict__ a,
                                                 const int* __restrict__ b, uint64_t n,
                                                 int* __restrict__ out) {
    const uint64_t stride = (uint64_t)gridDim.x * kTPB;
    const uint64_t n4 = n / 4;
    for (uint64_t i = (uint64_t)blockIdx.x * kTPB + threadIdx.x; i < n4; i += stride) {
        const int4 x = load4<VEC>(a + i * 4), y = load4<VEC>(b + i * 4);
        int4 o;
        o.x = SUB ? (int)((uint32_t)x.x - (uint32_t)y.x) : (int)((uint32_t)x.x + (uint32_t)y.x);
        o.y = SUB ? (int)((uint32_t)x.y - (uint32_t)y.y) : (int)((uint32_t)x.y + (uint32_t)y.y);
        o.z = SUB ? (int)((uint32_t)x.z - (uint32_t)y.z) : (int)((uint32_t)x.z + (uint32_t)y.z);
        o.w = SUB ? (int)((uint32_t)x.w - (uint32_t)y.w) : (int)((uint32_t)x.w + (uint32_t)y.w);
        if constexpr (VEC) {
            *reinterpret_cast<int4*>(out + i * 4) = o;
        } else {
            out[i * 4 + 0] = o.x;
            out[i * 4 + 1] = o.y;
            out[i * 4 + 2] = o.z;
            out[i * 4 + 3] = o.w;
        }
    }
    if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
        const uint64_t i = n4 * 4 + threadIdx.x;
        out[i] = SUB ? (int)((uint32_t)a[i] - (uint32_t)b[i]) : (int)((uint32_t)a[i] + (uint32_t)b[i]);
    }
}

// ---------------------------------------------------------------------------
// select_column_sorted_index (query.c:143-198). The run search is O(log n) and
// runs in one lane; the run copy (size_t -> int32 positions) is the O(K) part.
// ---------------------------------------------------------------------------
// query.c:143-160 binary_search with signed indices. Where the reference's size_t
// `right` wraps below zero (target < values[0]) it reads out of bounds; here that
// case returns -1 and the caller treats it as "before the first row".
__device__ long long ref_binary_search(const int* __restrict__ a, long long size, int target) {
    long long left = 0, right = size - 1;
    while (left <= right) {
        const long long mid = (left + right) / 2;
        if (a[mid] == target) return mid;
        if (target < a[mid]) right = mid - 1;
        else left = mid + 1;
    }
    return right;
}

__global__ void k_index_bounds(const int* __restrict__ values, uint64_t n, int low, int high,
                               long long* __restrict__ run, unsigned long long* __restrict__ d_count) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    long long left = ref_binary_search(values, (long long)n, low);
    long long right = ref_binary_search(values, (long long)n, high);
    if (left < 0) {
        left = 0;  // low < values[0]: every row is >= low
    } else {
        while (left > 0 && values[left] >= low) left--;  // query.c:175-177
        if (values[left] != low) left++;                 // query.c:178-180
    }
    while (right > left && values[right] == high) right--;  // query.c:181-183
    const long long k = right >= left ? right - left + 1 : 0;
    run[0] = left;
    run[1] = k;
    *d_count = (unsigned long long)k;
}

__global__ __launch_bounds__(kTPB) void k_index_copy(const uint64_t* __restrict__ positions,
                                                     const long long* __restrict__ run,
                                                     int* __restrict__ out) {
    const long long left = run[0], k = run[1];
    const long long stride = (long long)gridDim.x * kTPB;
    for (long long i = (long long)blockIdx.x * kTPB + threadIdx.x; i < k; i += stride)
        out[i] = (int)positions[left + i];  // query.c:185-188 (size_t -> int)
}

// ---------------------------------------------------------------------------
// synthetic data: SURVEY.md §8(c) (bit-identical to oracle/refcpu.c)
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t sm64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

__device__ __forceinline__ uint32_t mix31(uint32_t x) {
    const uint32_t M = 0x7FFFFFFFu;
    x &= M;
    x = (uint32_t)(((uint64_t)x * 0x2545F491u) & M);
    x ^= x >> 15;
    x = (uint32_t)(((uint64_t)x * 0x4F6CDD1Du) & M);
    x ^= x >> 13;
    x = (uint32_t)(((uint64_t)x * 0x6A09E667u) & M);
    x ^= x >> 16;
    return x;
}

__global__ __launch_bounds__(kTPB) void k_gen_uniform(int* __restrict__ out, uint64_t n,
                                                      uint64_t base, uint64_t modulus) {
    const uint64_t stride = (uint64_t)gridDim.x * kTPB;
    for (uint64_t i = (uint64_t)blockIdx.x * kTPB + threadIdx.x; i < n; i += stride)
        out[i] = (int)(sm64(base + i) % modulus);
}

__global__ __launch_bounds__(kTPB) void k_gen_join(int* __restrict__ out, uint64_t n, int kind) {
    const uint64_t stride = (uint64_t)gridDim.x * kTPB;
    const uint64_t mask = 2 * n - 1;
    for (uint64_t i = (uint64_t)blockIdx.x * kTPB + threadIdx.x; i < n; i += stride) {
        if (kind == 0) out[i] = (int)mix31((uint32_t)i);
        else out[i] = (int)mix31((uint32_t)(sm64((7ull << 40) | i) & mask));
    }
}

__global__ __launch_bounds__(kTPB) void k_iota(int* __restrict__ out, uint64_t n) {
    const uint64_t stride = (uint64_t)gridDim.x * kTPB;
    for (uint64_t i = (uint64_t)blockIdx.x * kTPB + threadIdx.x; i < n; i += stride) out[i] = (int)i;
}

}  // namespace

// host runtime shared with mq_join.hip (mq_common.h)
namespace mqi {
thread_local char g_err[512] = "";

int set_err(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

DevState g_dev[kMaxDev];

int current_device(int* dev) {
    int d = -1;
    hipError_t e = hipGetDevice(&d);
    if (e != hipSuccess || d < 0 || d >= kMaxDev)
        return set_err(MQ_ENODEV, "no HIP device: %s", hipGetErrorString(e));
    *dev = d;
    return MQ_OK;
}

int ensure_ready(DevState** out) {
    int d;
    int rc = current_device(&d);
    if (rc) return rc;
    DevState& s = g_dev[d];
    if (!s.ready) {
        hipDeviceProp_t prop;
        HIPCHK(hipGetDeviceProperties(&prop, d));
        if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
            return set_err(MQ_ENODEV, "device %d is %s, libmq is built for gfx950 only", d,
                           prop.gcnArchName);
        s.cus = prop.multiProcessorCount;
        int occ = 0;
        HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(
            &occ, reinterpret_cast<const void*>(&k_scan<false, false, true>), kTPB, 0));
        if (occ < 1) occ = 1;
        s.scan_blocks_per_cu = occ;
        s.ready = true;
    }
    *out = &s;
    return MQ_OK;
}

uint32_t stream_grid(const DevState* s, uint64_t work_items) {
    uint64_t g = (work_items + kTPB - 1) / kTPB;
    const uint64_t cap = (uint64_t)s->cus * 8;
    if (g > cap) g = cap;
    return (uint32_t)(g == 0 ? 1 : g);
}

}  // namespace mqi

namespace {
using namespace mqi;

// Fold (has_low, low, has_high, high) into one unsigned range compare.
// Returns false for an empty range.
bool make_pred(int has_low, int32_t low, int has_high, int32_t high, Pred* p) {
    const int64_t lo = has_low ? (int64_t)low : (int64_t)INT32_MIN;
    const int64_t hi = has_high ? (int64_t)high : (int64_t)INT32_MAX + 1;
    const int64_t width = hi - lo;
    if (width <= 0) return false;
    p->lo = (uint32_t)lo;
    p->wm1 = (uint32_t)(width - 1);
    return true;
}

void geometry(const DevState* s, uint64_t n, uint32_t* blocks, uint64_t* rpb) {
    uint64_t gmax = (uint64_t)s->cus * (uint64_t)s->scan_blocks_per_cu;
    if (gmax > kMaxBlocks) gmax = kMaxBlocks;
    const uint64_t tiles = (n + kTileRows - 1) / kTileRows;
    uint64_t g = tiles < gmax ? tiles : gmax;
    if (g == 0) g = 1;
    const uint64_t tiles_per_block = (tiles + g - 1) / g;
    *rpb = (tiles_per_block == 0 ? 1 : tiles_per_block) * kTileRows;
    g = (n + *rpb - 1) / *rpb;
    *blocks = (uint32_t)(g == 0 ? 1 : g);
}

size_t partial_bytes() { return (size_t)kMaxBlocks * sizeof(Partial); }
size_t mask_bytes(uint64_t n) {
    return (size_t)((n + kTileRows - 1) / kTileRows) * kWaves * 4 * sizeof(unsigned long long);
}

inline bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }


int empty_agg(mq_agg* d_out, hipStream_t st) {
    mq_agg e;
    e.count = 0;
    e.sum = 0;
    e.min = INT32_MAX;
    e.max = INT32_MIN;
    e._pad = 0;
    HIPCHK(hipMemcpyAsync(d_out, &e, sizeof(e), hipMemcpyHostToDevice, st));
    HIPCHK(hipStreamSynchronize(st));  // e lives on this stack frame
    return MQ_OK;
}

int run_agg(const int32_t* col, const int32_t* aux, uint64_t n, Pred pred, mq_agg* d_out,
            void* d_ws, size_t ws_bytes, hipStream_t st, const DevState* s) {
    if (ws_bytes < partial_bytes() || !d_ws)
        return set_err(MQ_EINVAL, "workspace too small (%zu < %zu)", ws_bytes, partial_bytes());
    uint32_t g;
    uint64_t rpb;
    geometry(s, n, &g, &rpb);
    Partial* part = static_cast<Partial*>(d_ws);
    const bool vec = aligned16(col);
    if (aux) {
        if (vec)
            hipLaunchKernelGGL((k_scan<false, true, true>), dim3(g), dim3(kTPB), 0, st, col, aux, n,
                               rpb, pred, part, nullptr);
        else
            hipLaunchKernelGGL((k_scan<false, true, false>), dim3(g), dim3(kTPB), 0, st, col, aux,
                               n, rpb, pred, part, nullptr);
    } else {
        if (vec)
            hipLaunchKernelGGL((k_scan<false, false, true>), dim3(g), dim3(kTPB), 0, st, col,
                               nullptr, n, rpb, pred, part, nullptr);
        else
            hipLaunchKernelGGL((k_scan<false, false, false>), dim3(g), dim3(kTPB), 0, st, col,
                               nullptr, n, rpb, pred, part, nullptr);
    }
    LAUNCHCHK("k_scan");
    hipLaunchKernelGGL(k_final, dim3(1), dim3(kTPB), 0, st, part, g, d_out);
    LAUNCHCHK("k_final");
    return MQ_OK;
}

}  // namespace

// ===========================================================================
// C-ABI
// ===========================================================================
extern "C" {

const char* mq_last_error(void) { return g_err; }
const char* mq_version(void) { return "libmq 0.1 (gfx950)"; }

int mq_device_count(void) {
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) return 0;
    return c;
}

int mq_init(int device) {
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    if (e != hipSuccess || c == 0)
        return set_err(MQ_ENODEV, "no HIP device available (%s)", hipGetErrorString(e));
    if (device < 0 || device >= c) return set_err(MQ_EINVAL, "device %d out of range [0,%d)", device, c);
    HIPCHK(hipSetDevice(device));
    DevState* s;
    return ensure_ready(&s);
}

void* mq_default_stream(void) {
    DevState* s;
    if (ensure_ready(&s)) return nullptr;
    if (!s->stream) {
        if (hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) != hipSuccess) return nullptr;
    }
    return s->stream;
}

int mq_malloc(void** dptr, size_t bytes) {
    DevState* s;
    int rc = ensure_ready(&s);
    if (rc) return rc;
    if (!dptr) return set_err(MQ_EINVAL, "mq_malloc: NULL out pointer");
    *dptr = nullptr;
    if (bytes == 0) bytes = 16;
    hipError_t e = hipMalloc(dptr, bytes);
    if (e != hipSuccess)
        return set_err(MQ_ENOMEM, "hipMalloc(%zu) failed: %s", bytes, hipGetErrorString(e));
    return MQ_OK;
}

int mq_free(void* dptr) {
    if (!dptr) return MQ_OK;
    HIPCHK(hipFree(dptr));
    return MQ_OK;
}

int mq_memcpy_h2d(void* dst, const void* src, size_t bytes, void* stream) {
    if (bytes == 0) return MQ_OK;
    hipStream_t st = (hipStream_t)stream;
    HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, st));
    HIPCHK(hipStreamSynchronize(st));
    return MQ_OK;
}

int mq_memcpy_d2h(void* dst, const void* src, size_t bytes, void* stream) {
    if (bytes == 0) return MQ_OK;
    hipStream_t st = (hipStream_t)stream;
    HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    return MQ_OK;
}

int mq_memcpy_d2d(void* dst, const void* src, size_t bytes, void* stream) {
    if (bytes == 0) return MQ_OK;
    HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream));
    return MQ_OK;
}

int mq_memset(void* dptr, int value, size_t bytes, void* stream) {
    if (bytes == 0) return MQ_OK;
    HIPCHK(hipMemsetAsync(dptr, value, bytes, (hipStream_t)stream));
    return MQ_OK;
}

int mq_stream_sync(void* stream) {
    HIPCHK(hipStreamSynchronize((hipStream_t)stream));
    return MQ_OK;
}

size_t mq_scan_workspace_bytes(uint64_t n) { return partial_bytes() + mask_bytes(n); }

void mq_scan_geometry(uint64_t n, uint32_t* blocks, uint64_t* rows_per_block) {
    DevState* s;
    if (ensure_ready(&s)) {
        if (blocks) *blocks = 0;
        if (rows_per_block) *rows_per_block = 0;
        return;
    }
    uint32_t g;
    uint64_t r;
    geometry(s, n, &g, &r);
    if (blocks) *blocks = g;
    if (rows_per_block) *rows_per_block = r;
}

int mq_gen_uniform(int32_t* d_out, uint64_t n, uint64_t seed, uint64_t modulus, void* stream) {
    DevState* s;
    int rc = ensure_ready(&s);
    if (rc) return rc;
    if (n == 0) return MQ_OK;
    if (!d_out || modulus == 0) return set_err(MQ_EINVAL, "mq_gen_uniform: bad argument");
    hipLaunchKernelGGL(k_gen_uniform, dim3(stream_grid(s, n)), dim3(kTPB), 0, (hipStream_t)stream,
                       d_out, n, seed * 0x100000001B3ull, modulus);
    LAUNCHCHK("k_gen_uniform");
    return MQ_OK;
}

int mq_gen_join_keys(int32_t* d_out, uint64_t n, int kind, void* stream) {
    DevState* s;
    int rc = ensure_ready(&s);
    if (rc) return rc;
    if (n == 0) return MQ_OK;
    if (!d_out || kind < 0 || kind > 1) return set_err(MQ_EINVAL, "mq_gen_join_keys: bad argument");
    hipLaunchKernelGGL(k_gen_join, dim3(stream_grid(s, n)), dim3(kTPB), 0, (hipStream_t)stream,
                       d_out, n, kind);
    LAUNCHCHK("k_gen_join");
    return MQ_OK;
}

int mq_gen_iota(int32_t* d_out, uint64_t n, void* stream) {
    DevState* s;
    int rc = ensure_ready(&s);
    if (rc) return rc;
    if (n == 0) return MQ_OK;
    if (!d_out) return set_err(MQ_EINVAL, "mq_gen_iota: NULL output");
    hipLaunchKernelGGL(k_iota, dim3(stream_grid(s, n)), dim3(kTPB), 0, (hipStream_t)stream, d_out, n);
    LAUNCHCHK("k_iota");
    return MQ_OK;
}

int mq_select_agg(const int32_t* d_col, uint64_t n, int has_low, int32_t low, int has_high,
                  int32_t high, mq_agg* d_out, void* d_ws, size_t ws_bytes, void* stream) {
    DevState* s;
    int rc = ensure_ready(&s);
    if (rc) return rc;
    if (!d_out || (n && !d_col)) return set_err(MQ_EINVAL, "mq_select_agg: NULL pointer");
    if ((uintptr_t)d_col & 3u) return set_err(MQ_EINVAL, "mq_select_agg: column not 4-byte aligned");
    Pred p;
    hipStream_t st = (hipStream_t)stream;
    if (n == 0 || !make_pred(has_low, low, has_high, high, &p)) return empty_agg(d_out, st);
    return run_agg(d_col, nullptr, n, p, d_out, d_ws, ws_bytes, st, s);
}

int mq_select_fetch_agg(const int32_t* d_sel, const int32_t* d_val, uint64_t n, int has_low,
                        int32_t low, int has_high, int32_t high, mq_agg* d_out, void* d_ws,
                        size_t ws_bytes, void* stream) {
    DevState* s;
    int rc = ensure_ready(&s);
    if (rc) return rc;
    if (!d_out || (n && (!d_sel || !d_val)))
        return set_err(MQ_EINVAL, "mq_select_fetch_agg: NULL pointer");
    if (((uintptr_t)d_sel | (uintptr_t)d_val) & 3u)
        return set_err(MQ_EINVAL, "mq_select_fetch_agg: column not 4-byte aligned");
    Pred p;
    hipStream_t st = (hipStream_t)stream;
    if (n == 0 || !make_pred(has_low, low, has_high, high, &p)) return empty_agg(d_out, st);
    return run_agg(d_sel, d_val, n, p, d_out, d_ws, ws_bytes, st, s);
}

int mq_select_partials(const int32_t* d_col, uint64_t n, int has_low, int32_t low, int has_high,
                       int32_t high, void* d_ws, size_t ws_bytes, uint32_t* nblocks, void* stream) {
    DevState* s;
    int rc = ensure_ready(&s);
    if (rc) return rc;
    if (!nblocks || !d_ws || (n && !d_col)) return set_err(MQ_EINVAL, "mq_select_partials: NULL pointer");
    if ((uintptr_t)d_col & 3u) return set_err(MQ_EINVAL, "mq_select_partials: column not 4-byte aligned");
    if (ws_bytes < partial_bytes())
        return set_err(MQ_EINVAL, "workspace too small (%zu < %zu)", ws_bytes, partial_bytes());
    Pred p;
    hipStream_t st = (hipStream_t)stream;
    if (n == 0 || !make_pred(has_low, low, has_high, high, &p)) {
        Partial e{0ull, 0ll, INT_MAX, INT_MIN, 0ull};
        HIPCHK(hipMemcpyAsync(d_ws, &e, sizeof(e), hipMemcpyHostToDevice, st));
        HIPCHK(hipStreamSynchronize(st));
        *nblocks = 1;
        return MQ_OK;
    }
    uint32_t g;
    uint64_t rpb;
    geometry(s, n, &g, &rpb);
    Partial* part = static_cast<Partial*>(d_ws);
    if (aligned16(d_col))
        hipLaunchKernelGGL((k_scan<false, false, true>), dim3(g), dim3(kTPB), 0, st, d_col, nullptr,
                           n, rpb, p, part, nullptr);
    else
        hipLaunchKernelGGL((k_scan<false, false, false>), dim3(g), dim3(kTPB), 0, st, d_col,
                           nullptr, n, rpb, p, part, nullptr);
    LAUNCHCHK("k_scan");
    *nblocks = g;
    return MQ_OK;
}

int mq_combine_partials(const void* d_ws, uint32_t nblocks, mq_agg* d_out, void* stream) {
    DevState* s;
    int rc = ensure_ready(&s);
    if (rc) return rc;
    if (!d_ws || !d_out || nblocks == 0 || nblocks > (uint32_t)kMaxBlocks)
        return set_err(MQ_EINVAL, "mq_combine_partials: bad argument");
    hipLaunchKernelGGL(k_final, dim3(1), dim3(kTPB), 0, (hipStream_t)stream,
                       static_cast<const Partial*>(d_ws), nblocks, d_out);
    LAUNCHCHK("k_final");
    return MQ_OK;
}

int mq_reduce(const int32_t* d_vals, uint64_t n, mq_agg* d_out, void* d_ws, size_t ws_bytes,
              void* stream) {
    return mq_select_agg(d_vals, n, 0, 0, 0, 0, d_out, d_ws, ws_bytes, stream);
}

int mq_select_positions(const int32_t* d_col, const int32_t* d_payload, uint64_t n, int has_low,
                        int32_t low, int has_high, int32_t high, int32_t* d_pos_out,
                        uint64_t* d_count, void* d_ws, size_t ws_bytes, void* stream) {
    DevState* s;
    int rc = ensure_ready(&s);
    if (rc) return rc;
    if (!d_count || (n && (!d_col || !d_pos_out)))
        return set_err(MQ_EINVAL, "mq_select_positions: NULL pointer");
    if (n > (uint64_t)INT32_MAX)
        return set_err(MQ_EINVAL, "mq_select_positions: %llu rows exceed int32 positions",
                       (unsigned long long)n);
    if (((uintptr_t)d_col | (uintptr_t)d_pos_out) & 3u)
        return set_err(MQ_EINVAL, "mq_select_positions: pointers not 4-byte aligned");
    hipStream_t st = (hipStream_t)stream;
    Pred p;
    if (n == 0 || !make_pred(has_low, low, has_high, high, &p)) {
        HIPCHK(hipMemsetAsync(d_count, 0, sizeof(uint64_t), st));
        return MQ_OK;
    }
    if (!d_ws || ws_bytes < mq_scan_workspace_bytes(n))
        return set_err(MQ_EINVAL, "mq_select_positions: workspace too small (%zu < %zu)", ws_bytes,
                       mq_scan_workspace_bytes(n));
    uint32_t g;
    uint64_t rpb;
    geometry(s, n, &g, &rpb);
    Partial* part = static_cast<Partial*>(d_ws);
    unsigned long long* masks =
        reinterpret_cast<unsigned long long*>(static_cast<char*>(d_ws) + partial_bytes());
    if (aligned16(d_col))
        hipLaunchKernelGGL((k_scan<true, false, true>), dim3(g), dim3(kTPB), 0, st, d_col, nullptr,
                           n, rpb, p, part, masks);
    else
        hipLaunchKernelGGL((k_scan<true, false, false>), dim3(g), dim3(kTPB), 0, st, d_col,
                           nullptr, n, rpb, p, part, masks);
    LAUNCHCHK("k_scan<mask>");
    if (d_payload)
        hipLaunchKernelGGL(k_compact<true>, dim3(g), dim3(kCompactTPB), 0, st, masks, part,
                           d_payload, n, rpb, d_pos_out,
                           reinterpret_cast<unsigned long long*>(d_count));
    else
        hipLaunchKernelGGL(k_compact<false>, dim3(g), dim3(kCompactTPB), 0, st, masks, part,
                           nullptr, n, rpb, d_pos_out,
                           reinterpret_cast<unsigned long long*>(d_count));
    LAUNCHCHK("k_compact");
    return MQ_OK;
}

int mq_index_select(const int32_t* d_values, const uint64_t* d_positions, uint64_t n, int32_t low,
                    int32_t high, int32_t* d_pos_out, uint64_t* d_count, void* stream) {
    DevState* s;
    int rc = ensure_ready(&s);
    if (rc) return rc;
    hipStream_t st = (hipStream_t)stream;
    if (!d_count) return set_err(MQ_EINVAL, "mq_index_select: NULL count");
    if (n == 0) {
        HIPCHK(hipMemsetAsync(d_count, 0, sizeof(uint64_t), st));
        return MQ_OK;
    }
    if (!d_values || !d_positions || !d_pos_out)
        return set_err(MQ_EINVAL, "mq_index_select: NULL pointer");
    // run = {left, k}: 16 bytes of scratch kept with the device state.
    static thread_local long long* run_buf[kMaxDev];
    int d;
    if ((rc = current_device(&d))) return rc;
    if (!run_buf[d]) HIPCHK(hipMalloc(&run_buf[d], 2 * sizeof(long long)));
    hipLaunchKernelGGL(k_index_bounds, dim3(1), dim3(64), 0, st, d_values, n, low, high, run_buf[d],
                       reinterpret_cast<unsigned long long*>(d_count));
    LAUNCHCHK("k_index_bounds");
    hipLaunchKernelGGL(k_index_copy, dim3(stream_grid(s, n)), dim3(kTPB), 0, st, d_positions,
                       run_buf[d], d_pos_out);
    LAUNCHCHK("k_index_copy");
    return MQ_OK;
}

int mq_fetch(const int32_t* d_col, const int32_t* d_pos, uint64_t k, int32_t* d_out, void* stream) {
    DevState* s;
    int rc = ensure_ready(&s);
    if (rc) return rc;
    if (k == 0) return MQ_OK;
    if (!d_col || !d_pos || !d_out) return set_err(MQ_EINVAL, "mq_fetch: NULL pointer");
    const bool vec = aligned16(d_pos) && aligned16(d_out);
    const uint32_t g = stream_grid(s, (k + 3) / 4);
    if (vec)
        hipLaunchKernelGGL(k_fetch<true>, dim3(g), dim3(kTPB), 0, (hipStream_t)stream, d_col, d_pos,
                           k, d_out);
    else
        hipLaunchKernelGGL(k_fetch<false>, dim3(g), dim3(kTPB), 0, (hipStream_t)stream, d_col,
                           d_pos, k, d_out);
    LAUNCHCHK("k_fetch");
    return MQ_OK;
}

static int addsub(const int32_t* a, const int32_t* b, uint64_t n, int32_t* out, void* stream,
                  bool sub) {
    DevState* s;
    int rc = ensure_ready(&s);
    if (rc) return rc;
    if (n == 0) return MQ_OK;
    if (!a || !b || !out) return set_err(MQ_EINVAL, "mq_add/mq_sub: NULL pointer");
    const bool vec = aligned16(a) && aligned16(b) && aligned16(out);
    const uint32_t g = stream_grid(s, (n + 3) / 4);
    hipStream_t st = (hipStream_t)stream;
    if (sub) {
        if (vec) hipLaunchKernelGGL((k_addsub<true, true>), dim3(g), dim3(kTPB), 0, st, a, b, n, out);
        else hipLaunchKernelGGL((k_addsub<true, false>), dim3(g), dim3(kTPB), 0, st, a, b, n, out);
    } else {
        if (vec) hipLaunchKernelGGL((k_addsub<false, true>), dim3(g), dim3(kTPB), 0, st, a, b, n, out);
        else hipLaunchKernelGGL((k_addsub<false, false>), dim3(g), dim3(kTPB), 0, st, a, b, n, out);
    }
    LAUNCHCHK("k_addsub");
    return MQ_OK;
}

int mq_add(const int32_t* d_a, const int32_t* d_b, uint64_t n, int32_t* d_out, void* stream) {
    return addsub(d_a, d_b, n, d_out, stream, false);
}

int mq_sub(const int32_t* d_a, const int32_t* d_b, uint64_t n, int32_t* d_out, void* stream) {
    return addsub(d_a, d_b, n, d_out, stream, true);
}

size_t mq_shared_select_workspace_bytes(uint64_t n, int q) {
    (void)q;
    return mq_scan_workspace_bytes(n);
}

int mq_shared_select(const int32_t* d_col, uint64_t n, const int32_t* h_lows,
                     const int32_t* h_highs, int q, int32_t* const* d_pos_out,
                     uint64_t* d_counts, void* d_ws, size_t ws_bytes, void* stream) {
    if (q < 0 || (q > 0 && (!h_lows || !h_highs || !d_pos_out || !d_counts)))
        return set_err(MQ_EINVAL, "mq_shared_select: bad argument");
    for (int j = 0; j < q; j++) {
        int rc = mq_select_positions(d_col, nullptr, n, 1, h_lows[j], 1, h_highs[j], d_pos_out[j],
                                     d_counts + j, d_ws, ws_bytes, stream);
        if (rc) return rc;
    }
    return MQ_OK;
}


}  // extern "C"
