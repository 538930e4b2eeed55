// mq_join.hip — hash join (src/query.c:652-696 over src/multimap.c) for gfx950.
//
// Output contract (the reference's, verified in SURVEY.md §8(a) row J1): pairs
// (build position, probe position) in probe-major order and, for one probe row,
// in build-insertion order.
//
// Build:
//   * unique keys (the FK case, and config 5): one 64-bit word {key, build
//     position} per slot of an open-addressing table (4-slot buckets, linear
//     probing inside 8192-slot windows, all-ones = empty). Above 2^16 rows the
//     rows are radix-partitioned by window and each window is built in LDS by one
//     block (k_win_build), which also leaves overflow marks in full buckets' slot
//     order. A second sighting of a key, or the empty word, raises a flag.
//   * duplicate keys (a sampled duplicate check decides up front for 2^20 rows and
//     up, else the flag): a stable LSD radix sort of (key, position) makes each
//     key's rows one run in insertion order; the runs' distinct keys go into the
//     same windowed table with the run (start, length) packed as payload.
// Probe: one 32-byte bucket read per probe row; continuations past a full bucket
// ride along in later steps through a per-wave LDS queue. Unique table: a payload
// and one hit word per 64 rows, then a scan of the hit words; runs: each row's
// (start, length), then a scan of the lengths. The write kernels copy the pairs.
// No CPU work per row anywhere; the host reads back only the flags and M.

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <cstring>

#include "mq_common.h"
#include "mq_device.h"

namespace {

using namespace mqi;

constexpr int kTPB = 256;
constexpr int kScanItems = 16;
constexpr int kScanTile = kTPB * kScanItems;  // 4096
constexpr int kSortItems = 16;  // words per thread of a sort tile (8 and 32 measured slower)
constexpr int kRadix = 256;
constexpr int kSortTPB = 512;  // sort tile = kSortTPB x kSortItems words (radix_sort_tiles)
// Partition tiles (TPB x kSortItems rows). Round 6, 2^28 joins alternating on one box
// (unique / many-to-many ms): build words and probe keys in 4096-row tiles 8.68 / 10.47;
// probe keys of u32-result joins in 8192-key tiles (a digit's run of keys ~128 B, a whole
// line, not 64 B) 8.29 / 10.37; build words in 8192-word tiles as well 7.85 / 10.17; the
// probe passes recording their places (k_pwin_scatter, the inverse passes without keys,
// hashing or ranking: their LDS fell from 85 to 41-74 KB) 7.62 / 10.0, and then the u64-
// result probes in 8192-key tiles too 7.59 / 9.29. Not kept: u32 probes in 16384-key
// tiles 8.84.
template <typename RT>
constexpr int probe_tpb() { return 512; }
constexpr int kBTPB = 512;  // the build words' partition tile: kBTPB x kSortItems

typedef unsigned long long u64;

__device__ __forceinline__ u64 wave_incl_scan(u64 v, int lane) {
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const u64 y = __shfl_up(v, off, 64);
        if (lane >= off) v += y;
    }
    return v;
}

// ---------------------------------------------------------------------------
// exclusive scan: Tin[n] -> u64[n] (reduce-then-scan over 4096-element tiles)
// ---------------------------------------------------------------------------
template <typename Tin>
__global__ __launch_bounds__(kTPB) void k_tile_sum(const Tin* in, uint64_t n, u64* sums) {
    const uint64_t base = (uint64_t)blockIdx.x * kScanTile;
    u64 acc = 0;
    Tin v[kScanItems];  // all loads in flight first (clamped index, no branch)
#pragma unroll
    for (int k = 0; k < kScanItems; k++) {
        const uint64_t i = base + (uint64_t)k * kTPB + threadIdx.x;
        v[k] = in[i < n ? i : n - 1];
    }
#pragma unroll
    for (int k = 0; k < kScanItems; k++)
        if (base + (uint64_t)k * kTPB + threadIdx.x < n) acc += (u64)v[k];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
    __shared__ u64 ws[kTPB / 64];
    if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) sums[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
}

// in and out may alias (every element is read into LDS before any is written).
template <typename Tin, typename Tout = u64>
__global__ __launch_bounds__(kTPB) void k_tile_scan(const Tin* in, Tout* out, uint64_t n,
                                                    const u64* offs) {
    __shared__ u64 tile[kScanTile];
    __shared__ u64 ws[kTPB / 64];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint64_t base = (uint64_t)blockIdx.x * kScanTile;
    {
        Tin x[kScanItems];  // all loads in flight first (clamped index, no branch)
#pragma unroll
        for (int k = 0; k < kScanItems; k++) {
            const uint64_t i = base + (uint64_t)k * kTPB + tid;
            x[k] = in[i < n ? i : n - 1];
        }
#pragma unroll
        for (int k = 0; k < kScanItems; k++)
            tile[k * kTPB + tid] = base + (uint64_t)k * kTPB + tid < n ? (u64)x[k] : 0ull;
    }
    __syncthreads();
    u64 v[kScanItems];
    u64 acc = 0;
#pragma unroll
    for (int k = 0; k < kScanItems; k++) {
        v[k] = tile[tid * kScanItems + k];
        acc += v[k];
    }
    const u64 incl = wave_incl_scan(acc, lane);
    if (lane == 63) ws[wave] = incl;
    __syncthreads();
    u64 run = incl - acc + (offs ? offs[blockIdx.x] : 0ull);
    for (int w = 0; w < wave; w++) run += ws[w];
#pragma unroll
    for (int k = 0; k < kScanItems; k++) {
        tile[tid * kScanItems + k] = run;
        run += v[k];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kScanItems; k++) {
        const uint64_t i = base + (uint64_t)k * kTPB + tid;
        if (i < n) out[i] = (Tout)tile[k * kTPB + tid];
    }
}

uint64_t ceil_div(uint64_t a, uint64_t b) { return (a + b - 1) / b; }

// u64 elements of scratch needed by scan_exclusive(n).
uint64_t scan_scratch_elems(uint64_t n) {
    uint64_t total = 0;
    while (n > (uint64_t)kScanTile) {
        n = ceil_div(n, kScanTile);
        total += n;
    }
    return total + 1;
}

template <typename Tin, typename Tout = u64>
int scan_exclusive(const Tin* in, Tout* out, uint64_t n, u64* scratch, hipStream_t st) {
    if (n == 0) return MQ_OK;
    if (n <= (uint64_t)kScanTile) {
        hipLaunchKernelGGL((k_tile_scan<Tin, Tout>), dim3(1), dim3(kTPB), 0, st, in, out, n,
                           (const u64*)nullptr);
        LAUNCHCHK("k_tile_scan");
        return MQ_OK;
    }
    const uint64_t nb = ceil_div(n, kScanTile);
    hipLaunchKernelGGL(k_tile_sum<Tin>, dim3((uint32_t)nb), dim3(kTPB), 0, st, in, n, scratch);
    LAUNCHCHK("k_tile_sum");
    int rc = scan_exclusive<u64, u64>(scratch, scratch, nb, scratch + nb, st);
    if (rc) return rc;
    hipLaunchKernelGGL((k_tile_scan<Tin, Tout>), dim3((uint32_t)nb), dim3(kTPB), 0, st, in, out, n,
                       (const u64*)scratch);
    LAUNCHCHK("k_tile_scan");
    return MQ_OK;
}

// ---------------------------------------------------------------------------
// stable LSD radix sort of packed words {key ^ 2^31 (low 32), value (high 32)},
// 8-bit digits. Per tile of TPB x IT words (8192): an LDS histogram (k_sortw_hist), an exclusive
// scan over (digit, tile), then a scatter that ranks equal digits with 8 wave
// ballots (stable) and stages the tile in LDS, so every digit run leaves the block
// as contiguous stores. (Element-by-element scatter measured 0.5 TB/s at 1e9 rows.)
// FIRST: the words are built from the int32 keys (and values, or row ids).
// LAST : the sorted words are written split into key and value arrays.
// ---------------------------------------------------------------------------
template <bool FIRST>
__device__ __forceinline__ u64 sort_word(const int* c1, const int* p1, const u64* in, uint64_t i) {
    if constexpr (FIRST) {
        const uint32_t v = p1 ? (uint32_t)p1[i] : (uint32_t)i;
        return (u64)((uint32_t)c1[i] ^ 0x80000000u) | ((u64)v << 32);
    } else {
        return in[i];
    }
}

template <bool FIRST, int TPB, int IT>
__global__ __launch_bounds__(TPB) void k_sortw_hist(const int* __restrict__ c1, const u64* __restrict__ in,
                                                    uint64_t n, int shift, uint32_t kmin,
                                                    uint32_t* __restrict__ hist, uint32_t ntiles) {
    constexpr uint32_t kTile = TPB * IT;
    __shared__ uint32_t h[kRadix];
    if (threadIdx.x < kRadix) h[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t tile = xcd_tile(blockIdx.x, gridDim.x);
    const uint64_t base = (uint64_t)tile * kTile;
    // all of the lane's items are loaded before any is counted (indices clamped,
    // no branch), so the loads share one round trip instead of one each; the words
    // are read once, nontemporal (1.72 -> 1.62 ms per pass over 8 GB at 1e9 rows)
    uint32_t key[IT];
#pragma unroll
    for (int k = 0; k < IT; k++) {
        const uint64_t i = base + (uint64_t)k * TPB + threadIdx.x;
        const uint64_t ic = i < n ? i : n - 1;
        key[k] = (FIRST ? ((uint32_t)__builtin_nontemporal_load(c1 + ic) ^ 0x80000000u)
                        : (uint32_t)__builtin_nontemporal_load(in + ic)) - kmin;
    }
#pragma unroll
    for (int k = 0; k < IT; k++)
        if (base + (uint64_t)k * TPB + threadIdx.x < n) atomicAdd(&h[(key[k] >> shift) & 0xFF], 1u);
    __syncthreads();
    if (threadIdx.x < kRadix) hist[(uint64_t)threadIdx.x * ntiles + tile] = h[threadIdx.x];
}

// The same histogram from the digit bytes the previous scatter wrote (1 B per row
// instead of the 8-byte words): one 16-byte load per thread covers its 16 rows.
template <int TPB, int IT>
__global__ __launch_bounds__(TPB) void k_sortw_hist_bytes(const uint8_t* __restrict__ dig, uint64_t n,
                                                          uint32_t* __restrict__ hist, uint32_t ntiles) {
    constexpr uint32_t kTile = TPB * IT;
    __shared__ uint32_t h[kRadix];
    if (threadIdx.x < kRadix) h[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t tile = xcd_tile(blockIdx.x, gridDim.x);
    const uint64_t base = (uint64_t)tile * kTile + (uint64_t)threadIdx.x * IT;
    static_assert(IT == 16, "one 16-byte load per thread");
    if (base + IT <= n) {
        typedef unsigned int v4u __attribute__((ext_vector_type(4)));
        const v4u w = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(dig + base));
        const uint32_t x[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
        for (int k = 0; k < 4; k++) {
            atomicAdd(&h[x[k] & 0xFF], 1u);
            atomicAdd(&h[(x[k] >> 8) & 0xFF], 1u);
            atomicAdd(&h[(x[k] >> 16) & 0xFF], 1u);
            atomicAdd(&h[x[k] >> 24], 1u);
        }
    } else {
        for (uint64_t i = base; i < n && i < base + IT; i++) atomicAdd(&h[dig[i]], 1u);
    }
    __syncthreads();
    if (threadIdx.x < kRadix) hist[(uint64_t)threadIdx.x * ntiles + tile] = h[threadIdx.x];
}

// LAST: 0 = packed words to out, 1 = split into kout (flipped keys) / vout,
// 2 = an index: kout as int32 values (key ^ 2^31 undone), pout as size_t rows.
template <bool FIRST, int LAST, int TPB, int IT>
__global__ __launch_bounds__(TPB) void k_sortw_scatter(const int* __restrict__ c1, const int* __restrict__ p1,
                                                        const u64* __restrict__ in, uint64_t n, int shift,
                                                        uint32_t kmin, const u64* __restrict__ goff, uint32_t ntiles,
                                                        u64* __restrict__ out, uint32_t* __restrict__ kout,
                                                        uint32_t* __restrict__ vout, u64* __restrict__ pout,
                                                        uint8_t* __restrict__ dig) {
    constexpr int kW = TPB / 64;
    constexpr uint32_t kTile = TPB * IT;
    __shared__ uint32_t wcnt[kW][kRadix];
    __shared__ uint32_t loff[kRadix];
    __shared__ u64 gofs[kRadix];
    __shared__ u64 stage[kTile];
    __shared__ uint32_t wsum[kRadix / 64];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (int x = tid; x < kW * kRadix; x += TPB) (&wcnt[0][0])[x] = 0;
    const uint32_t tile = xcd_tile(blockIdx.x, gridDim.x);
    if (tid < kRadix) gofs[tid] = goff[(uint64_t)tid * ntiles + tile];
    __syncthreads();
    const uint64_t tile0 = (uint64_t)tile * kTile;
    const uint64_t seg = tile0 + (uint64_t)wave * (64 * IT);
    u64 el[IT];
    uint32_t dr[IT];
    // all items loaded first (indices clamped, no branch): one round trip, not one
    // per item (the ranking's ballots kept the compiler from hoisting the loads)
#pragma unroll
    for (int k = 0; k < IT; k++) {
        const uint64_t i = seg + (uint64_t)k * 64 + lane;
        el[k] = sort_word<FIRST>(c1, p1, in, i < n ? i : n - 1);
    }
#pragma unroll
    for (int k = 0; k < IT; k++) {
        const uint64_t i = seg + (uint64_t)k * 64 + lane;
        const bool valid = i < n;
        const uint32_t d = (((uint32_t)el[k] - kmin) >> shift) & 0xFF;
        const u64 peers = match_any8(d, __ballot(valid));
        const uint32_t lt = lanes_below(peers);
        const uint32_t cur = wcnt[wave][d];
        __builtin_amdgcn_wave_barrier();
        if (valid && lt == 0) wcnt[wave][d] = cur + (uint32_t)__popcll(peers);
        __builtin_amdgcn_wave_barrier();
        dr[k] = valid ? ((d << 16) | (cur + lt)) : 0xFFFFFFFFu;
    }
    __syncthreads();
    // per digit (thread tid < 256): prefix over the waves, then the tile-local
    // exclusive scan of the digit totals (waves 0-3)
    uint32_t tot = 0, incl = 0;
    if (tid < kRadix) {
#pragma unroll
        for (int w = 0; w < kW; w++) {
            const uint32_t c = wcnt[w][tid];
            wcnt[w][tid] = tot;
            tot += c;
        }
        incl = tot;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t y = __shfl_up(incl, off, 64);
            if (lane >= off) incl += y;
        }
        if (lane == 63) wsum[wave] = incl;
    }
    __syncthreads();
    if (tid < kRadix) {
        uint32_t excl = incl - tot;
        for (int w = 0; w < wave; w++) excl += wsum[w];
        loff[tid] = excl;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < IT; k++) {
        if (dr[k] != 0xFFFFFFFFu) {
            const uint32_t d = dr[k] >> 16, r = dr[k] & 0xFFFF;
            stage[loff[d] + wcnt[wave][d] + r] = el[k];
        }
    }
    __syncthreads();
    const uint64_t tn = n - tile0 < (uint64_t)kTile ? n - tile0 : (uint64_t)kTile;
#pragma unroll
    for (int k = 0; k < IT; k++) {
        const uint32_t e = (uint32_t)(k * TPB + tid);
        if (e < tn) {
            const u64 v = stage[e];
            const uint32_t d = (((uint32_t)v - kmin) >> shift) & 0xFF;
            const u64 dst = gofs[d] + (e - loff[d]);
            if constexpr (LAST == 1) {
                kout[dst] = (uint32_t)v;
                vout[dst] = (uint32_t)(v >> 32);
            } else if constexpr (LAST == 2) {
                if (kout) kout[dst] = (uint32_t)v ^ 0x80000000u;
                if (pout) pout[dst] = v >> 32;
            } else {
                out[dst] = v;
                if (dig) dig[dst] = (uint8_t)(((uint32_t)v - kmin) >> (shift + 8));  // the next pass's digit
            }
        }
    }
}

// ---------------------------------------------------------------------------
// hash table: 64-bit slot words {key (low 32), occupied (bit 32)}, linear probing
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t hash32(uint32_t k) {  // murmur3 finaliser
    k ^= k >> 16;
    k *= 0x85EBCA6Bu;
    k ^= k >> 13;
    k *= 0xC2B2AE35u;
    k ^= k >> 16;
    return k;
}

__device__ __forceinline__ u64 pack_key(int key) { return (u64)(uint32_t)key | (1ull << 32); }

// Claim (or find) key's slot. Returns slot; *fresh = true if this call claimed it.
__device__ __forceinline__ uint64_t ht_claim(u64* words, uint64_t mask, int key, bool* fresh) {
    const u64 w = pack_key(key);
    uint64_t h = hash32((uint32_t)key) & mask;
    for (uint64_t step = 0; step <= mask; step++) {
        const u64 old = atomicCAS(&words[h], 0ull, w);
        if (old == 0ull) {
            *fresh = true;
            return h;
        }
        if (old == w) {
            *fresh = false;
            return h;
        }
        h = (h + 1) & mask;
    }
    *fresh = false;
    return ~0ull;  // unreachable: the table is at most half full
}

__device__ __forceinline__ uint64_t ht_find(const u64* words, uint64_t mask, int key) {
    const u64 w = pack_key(key);
    uint64_t h = hash32((uint32_t)key) & mask;
    for (uint64_t step = 0; step <= mask; step++) {
        const u64 cur = words[h];
        if (cur == w) return h;
        if (cur == 0ull) return ~0ull;
        h = (h + 1) & mask;
    }
    return ~0ull;
}

// Unique-key table: one 64-bit word per slot, {key (low 32), build payload = the
// build position p1[row] (high 32)}; all-ones = empty. One CAS per build row, and a
// probe hit yields out1's value directly (no gather from p1). A build row whose
// word equals the empty marker (key = p1 = -1) sends the build to the general path.
constexpr u64 kEmpty = ~0ull;
__device__ __forceinline__ u64 pack_pair(int key, int payload) {
    return (u64)(uint32_t)key | ((u64)(uint32_t)payload << 32);
}

// Windowed open addressing: the table is cut into windows of W = min(8192, slots)
// slots and linear probing wraps inside the key's home window, so a window can be
// built in LDS (64 KB) and written out with one coalesced sweep.
constexpr int kWinLog = 13;
constexpr int kWinTPB = 1024;

struct Win {
    uint64_t mask;   // slots - 1
    uint64_t wmask;  // W - 1
    int wlog;        // log2 W
};

__device__ __forceinline__ uint64_t win_next(uint64_t h, const Win& t) {
    return (h & ~t.wmask) | ((h + 1) & t.wmask);
}
__device__ __forceinline__ uint32_t win_id(uint32_t key, const Win& t) {
    return (uint32_t)((hash32(key) & t.mask) >> t.wlog);
}

// Unique-key tables start a key's linear probe at the first slot of its aligned
// 4-slot bucket (32 B), not at its own slot: a probe then reads the whole bucket
// with two 16-byte loads and rarely needs a second, dependent read (with the probe
// starting at the hashed slot itself, about every other probe at load 1/2 went on
// to the next slot after its first read returned).
constexpr uint32_t kBucket = 4;
__device__ __forceinline__ uint64_t ht_home(uint32_t key, uint64_t mask) {
    return hash32(key) & mask & ~(uint64_t)(kBucket - 1);
}
// a full bucket's overflow mark (windowed builds, k_win_build): slot order
__device__ __forceinline__ bool bucket_ovf(u64 s0, u64 s1) { return (uint32_t)s0 > (uint32_t)s1; }

// Global-CAS insert (builds below kWindowBuildRows): sets *general on a duplicate
// key, the empty marker, or a full window.
__global__ __launch_bounds__(kTPB) void k_ht_insert_unique(const int* __restrict__ keys,
                                                           const int* __restrict__ pay, uint64_t n,
                                                           u64* words, Win t,
                                                           uint32_t* __restrict__ general) {
    const uint64_t stride = (uint64_t)gridDim.x * kTPB;
    for (uint64_t i = (uint64_t)blockIdx.x * kTPB + threadIdx.x; i < n; i += stride) {
        const u64 w = pack_pair(keys[i], pay[i]);
        if (w == kEmpty) {
            *general = 1;
            continue;
        }
        const uint32_t key = (uint32_t)w;
        uint64_t h = ht_home(key, t.mask);
        bool placed = false;
        for (uint64_t step = 0; step <= t.wmask; step++) {
            const u64 old = atomicCAS(&words[h], kEmpty, w);
            if (old == kEmpty) {
                placed = true;
                break;
            }
            if ((uint32_t)old == key) break;  // second sighting of the key
            h = win_next(h, t);
        }
        if (!placed) *general = 1;
    }
}

// ---- window build: stable LSD radix partition of the (key, payload) words by
// window id (8 bits per pass), then one block per window builds it in LDS ----
template <bool FROM_COLS>
__device__ __forceinline__ u64 win_elem(const int* c1, const int* p1, const u64* in, uint64_t i) {
    if constexpr (FROM_COLS) return pack_pair(c1[i], p1[i]);
    else return in[i];
}

// Tiles of TPB x kSortItems rows: the build's words in tiles of kBTPB threads, the
// probe keys in tiles of probe_tpb<RT>().
template <bool FROM_COLS, int TPB = kBTPB>
__global__ __launch_bounds__(TPB) void k_win_hist(const int* __restrict__ c1,
                                                  const u64* __restrict__ in, uint64_t n, Win t,
                                                  int shift, uint32_t* __restrict__ hist,
                                                  uint32_t ntiles) {
    __shared__ uint32_t h[kRadix];
    if (threadIdx.x < kRadix) h[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t tile = xcd_tile(blockIdx.x, gridDim.x);
    const uint64_t base = (uint64_t)tile * (TPB * kSortItems);
    uint32_t key[kSortItems];  // loaded before any is counted, as in k_sortw_hist
#pragma unroll
    for (int k = 0; k < kSortItems; k++) {
        const uint64_t i = base + (uint64_t)k * TPB + threadIdx.x;
        const uint64_t ic = i < n ? i : n - 1;
        key[k] = FROM_COLS ? (uint32_t)__builtin_nontemporal_load(c1 + ic)
                           : (uint32_t)__builtin_nontemporal_load(in + ic);
    }
#pragma unroll
    for (int k = 0; k < kSortItems; k++)
        if (base + (uint64_t)k * TPB + threadIdx.x < n) atomicAdd(&h[(win_id(key[k], t) >> shift) & 0xFF], 1u);
    __syncthreads();
    if (threadIdx.x < kRadix) hist[(uint64_t)threadIdx.x * ntiles + tile] = h[threadIdx.x];
}

// After a tile's items are ranked per wave (wcnt[w][d] = wave w's count of digit d):
// wcnt[w][d] becomes the count of d in the waves before w, loff[d] the tile-local start
// of digit d. Threads 0..255 (waves 0-3) own the digits; every thread takes the barriers.
template <int TPB>
__device__ __forceinline__ void tile_digit_offsets(uint32_t (*wcnt)[kRadix], uint32_t* loff, uint32_t* wsum,
                                                   int tid) {
    const int lane = tid & 63, wave = tid >> 6;
    uint32_t tot = 0, incl = 0;
    if (tid < kRadix) {
#pragma unroll
        for (int w = 0; w < TPB / 64; w++) {
            const uint32_t c = wcnt[w][tid];
            wcnt[w][tid] = tot;
            tot += c;
        }
        incl = tot;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t y = __shfl_up(incl, off, 64);
            if (lane >= off) incl += y;
        }
        if (lane == 63) wsum[wave] = incl;
    }
    __syncthreads();
    if (tid < kRadix) {
        uint32_t excl = incl - tot;
        for (int w = 0; w < wave; w++) excl += wsum[w];
        loff[tid] = excl;
    }
    __syncthreads();
}

// Stable scatter (k_sortw_scatter's ballot ranking), staged through LDS so that each
// digit's run leaves the block as contiguous, coalesced stores.
template <bool FROM_COLS, int TPB = kBTPB>
__global__ __launch_bounds__(TPB) void k_win_scatter(const int* __restrict__ c1,
                                                      const int* __restrict__ p1,
                                                      const u64* __restrict__ in, uint64_t n, Win t,
                                                      int shift, const u64* __restrict__ goff,
                                                      uint32_t ntiles, u64* __restrict__ out,
                                                      int* __restrict__ pmm = nullptr) {
    constexpr int kTile = TPB * kSortItems;
    __shared__ uint32_t wcnt[TPB / 64][kRadix];
    __shared__ uint32_t loff[kRadix];
    __shared__ u64 gofs[kRadix];
    __shared__ u64 stage[kTile];
    __shared__ uint32_t wsum[kRadix / 64];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (int x = tid; x < (TPB / 64) * kRadix; x += TPB) (&wcnt[0][0])[x] = 0;
    const uint32_t tile = xcd_tile(blockIdx.x, gridDim.x);
    if (tid < kRadix) gofs[tid] = goff[(uint64_t)tid * ntiles + tile];
    __syncthreads();
    const uint64_t tile0 = (uint64_t)tile * kTile;
    const uint64_t seg = tile0 + (uint64_t)wave * (64 * kSortItems);
    u64 el[kSortItems];
    uint32_t dr[kSortItems];
    // all items loaded first (indices clamped, no branch): one round trip, not one
    // per item (the ranking's ballots kept the compiler from hoisting the loads)
#pragma unroll
    for (int k = 0; k < kSortItems; k++) {
        const uint64_t i = seg + (uint64_t)k * 64 + lane;
        el[k] = win_elem<FROM_COLS>(c1, p1, in, i < n ? i : n - 1);
    }
    if (FROM_COLS && pmm) {
        // the payloads' range (a value outside it marks a miss, k_win_join): per block,
        // then one atomic pair into 64 spread slots (one address for every wave made the
        // pass 5.5x slower); the host folds the slots
        int mn = INT32_MAX, mx = INT32_MIN;
#pragma unroll
        for (int k = 0; k < kSortItems; k++) {  // (clamped rows repeat row n - 1: harmless)
            const int v = (int)(el[k] >> 32);
            mn = v < mn ? v : mn;
            mx = v > mx ? v : mx;
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const int a = __shfl_xor(mn, o, 64), b = __shfl_xor(mx, o, 64);
            mn = a < mn ? a : mn;
            mx = b > mx ? b : mx;
        }
        __shared__ int smm[2][TPB / 64];
        if (lane == 0) smm[0][wave] = mn, smm[1][wave] = mx;
        __syncthreads();
        if (tid == 0) {
#pragma unroll
            for (int w = 1; w < TPB / 64; w++) {
                mn = smm[0][w] < mn ? smm[0][w] : mn;
                mx = smm[1][w] > mx ? smm[1][w] : mx;
            }
            atomicMin(pmm + (tile & 63), mn);
            atomicMax(pmm + 64 + (tile & 63), mx);
        }
    }
#pragma unroll
    for (int k = 0; k < kSortItems; k++) {
        const uint64_t i = seg + (uint64_t)k * 64 + lane;
        const bool valid = i < n;
        const uint32_t d = (win_id((uint32_t)el[k], t) >> shift) & 0xFF;
        const u64 peers = match_any8(d, __ballot(valid));
        const uint32_t lt = lanes_below(peers);
        const uint32_t cur = wcnt[wave][d];
        __builtin_amdgcn_wave_barrier();
        if (valid && lt == 0) wcnt[wave][d] = cur + (uint32_t)__popcll(peers);
        __builtin_amdgcn_wave_barrier();
        dr[k] = valid ? ((d << 16) | (cur + lt)) : 0xFFFFFFFFu;
    }
    __syncthreads();
    tile_digit_offsets<TPB>(wcnt, loff, wsum, tid);
#pragma unroll
    for (int k = 0; k < kSortItems; k++) {
        if (dr[k] != 0xFFFFFFFFu) {
            const uint32_t d = dr[k] >> 16, r = dr[k] & 0xFFFF;
            stage[loff[d] + wcnt[wave][d] + r] = el[k];
        }
    }
    __syncthreads();
    const uint64_t tn = n - tile0 < (uint64_t)kTile ? n - tile0 : (uint64_t)kTile;
#pragma unroll
    for (int k = 0; k < kSortItems; k++) {
        const uint32_t e = (uint32_t)(k * TPB + tid);
        if (e < tn) {
            const u64 v = stage[e];
            const uint32_t d = (win_id((uint32_t)v, t) >> shift) & 0xFF;
            out[gofs[d] + (e - loff[d])] = v;
        }
    }
}

// wstart[w] = first index of window w in the partitioned words (wstart[nw] = n):
// the words are sorted by window id, so one binary search per window boundary
// (nw + 1 threads, ~28 dependent reads whose upper levels sit in L2) instead of a
// pass over all n words (0.48 ms at 2^28).
template <typename T>
__global__ __launch_bounds__(kTPB) void k_win_bounds(const T* __restrict__ in, uint64_t n, Win t,
                                                     uint32_t nw, uint32_t* __restrict__ wstart) {
    const uint32_t x = blockIdx.x * kTPB + threadIdx.x;
    if (x > nw) return;
    uint64_t lo = 0, hi = n;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (win_id((uint32_t)in[mid], t) < x) lo = mid + 1;
        else hi = mid;
    }
    wstart[x] = (uint32_t)lo;
}

// One block per window: insert the window's words into an LDS table with LDS CAS,
// 1024 threads so two 64 KB-LDS blocks still fill a CU with 32 waves (measured
// 3.3 ms at 256 threads for 2^28 rows),
// then store the whole window (coalesced). Duplicates, the empty marker and an
// overfull window set *general.
template <bool STORE>
__global__ __launch_bounds__(kWinTPB) void k_win_build(const u64* __restrict__ in,
                                                    const uint32_t* __restrict__ wstart,
                                                    u64* __restrict__ words, Win t,
                                                    uint32_t* __restrict__ general) {
    __shared__ u64 tab[1 << kWinLog];
    // A full bucket records in its slot order whether any key homed there went on
    // past it (then key(slot 0) > key(slot 1), else <; the keys are distinct), so a
    // probe that misses in a full bucket without overflow ends there (bucket_ovf).
    // An insert that lands outside its home bucket marks that bucket.
    __shared__ uint8_t ovf[(1 << kWinLog) / kBucket];
    const uint32_t W = (uint32_t)t.wmask + 1;
    const uint32_t w = blockIdx.x;
    for (uint32_t x = threadIdx.x; x < W; x += kWinTPB) tab[x] = kEmpty;
    for (uint32_t x = threadIdx.x; x < W / kBucket; x += kWinTPB) ovf[x] = 0;
    __syncthreads();
    const uint32_t b = wstart[w], e = wstart[w + 1];
    if (e - b > W - W / 4) {  // over 3/4 full: probes would run long (adversarial keys)
        if (threadIdx.x == 0) *general = 1;
    } else {
        // at most 3/4 of W words: every thread's (<= W / kWinTPB) words are loaded
        // before any is inserted (one round trip, not one per word)
        constexpr int kPer = (1 << kWinLog) / kWinTPB;
        u64 vs[kPer];
#pragma unroll
        for (int k = 0; k < kPer; k++) {
            const uint32_t i = b + threadIdx.x + (uint32_t)k * kWinTPB;
            vs[k] = i < e ? in[i] : kEmpty;
        }
#pragma unroll
        for (int k = 0; k < kPer; k++) {
            if (b + threadIdx.x + (uint32_t)k * kWinTPB >= e) break;
            const u64 v = vs[k];
            if (v == kEmpty) {
                *general = 1;
                continue;
            }
            const uint32_t key = (uint32_t)v;
            const uint32_t h0 = (uint32_t)ht_home(key, t.wmask);
            uint32_t h = h0;
            for (uint32_t step = 0; step < W; step++) {
                const u64 old = atomicCAS(&tab[h], kEmpty, v);
                if (old == kEmpty) {
                    if (step >= kBucket) ovf[h0 / kBucket] = 1;
                    break;
                }
                if ((uint32_t)old == key) {
                    *general = 1;
                    break;
                }
                h = (h + 1) & (W - 1);
            }
        }
    }
    if constexpr (!STORE) return;  // the check alone (partitioned probe: no global table)
    __syncthreads();
    for (uint32_t bk = threadIdx.x; bk < W / kBucket; bk += kWinTPB) {
        const uint32_t s0 = bk * kBucket;
        const u64 a = tab[s0], c = tab[s0 + 1];
        if (a == kEmpty || c == kEmpty || tab[s0 + 2] == kEmpty || tab[s0 + 3] == kEmpty) continue;
        if (((uint32_t)a > (uint32_t)c) != (ovf[bk] != 0)) tab[s0] = c, tab[s0 + 1] = a;
    }
    __syncthreads();
    u64* dst = words + (uint64_t)w * W;
    for (uint32_t x = threadIdx.x; x < W; x += kWinTPB) dst[x] = tab[x];
}

// ---- the partitioned unique probe (round 5) ----
// A probe row's bucket read is a random 128-B line fetch from a table far beyond the
// Infinity Cache: 2^28 probes moved ~34 GB for 8 GB of buckets (PMC). Instead the probe
// keys take the build's window partition (the same LSD passes, u32 keys), one block per
// window builds the window's table in LDS from the build's partitioned words and probes
// it with the window's probe keys (k_win_join: no global table is ever written or
// read), and the results go back to probe order by running the passes backwards
// (k_pwin_gather). Everything moves as streams.

// Exclusive scan of a tile's 256 digit counts (threads 0..255 own the digits; every
// thread takes the barriers): loff[d] = the tile-local start of digit d.
__device__ __forceinline__ void digit_scan(const uint32_t* cnt, uint32_t* loff, uint32_t* wsum, int tid) {
    const int lane = tid & 63, wave = tid >> 6;
    uint32_t c = 0, incl = 0;
    if (tid < kRadix) {
        c = cnt[tid];
        incl = c;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t y = __shfl_up(incl, off, 64);
            if (lane >= off) incl += y;
        }
        if (lane == 63) wsum[wave] = incl;
    }
    __syncthreads();
    if (tid < kRadix) {
        uint32_t ex = incl - c;
        for (int w = 0; w < wave; w++) ex += wsum[w];
        loff[tid] = ex;
    }
    __syncthreads();
}

// One pass of the probe keys by window-id digit (round 6 form). The pass records each
// row's place in its tile's digit order (perm, u16) for the inverse passes, which then
// neither hash nor rank: they read 2 B a row instead of the 4-B keys. STABLE: rows of a
// digit keep their order (ballot match-any ranks), which every pass after the first
// needs, so that the windows come out whole (LSD); the first pass's keys need no order
// within a digit (each key's result is its own), so there a key takes its place by one
// LDS atomic.
template <int TPB, bool STABLE>
__global__ __launch_bounds__(TPB) void k_pwin_scatter(const uint32_t* __restrict__ in, uint64_t n, Win t, int shift,
                                                      const u64* __restrict__ goff, uint32_t ntiles,
                                                      uint32_t* __restrict__ out, uint16_t* __restrict__ perm) {
    constexpr int kTile = TPB * kSortItems, kW = STABLE ? TPB / 64 : 1;
    static_assert(kTile <= 65536, "u16 places");
    __shared__ uint32_t wcnt[kW][kRadix];  // per wave (STABLE) or per tile
    __shared__ uint32_t loff[kRadix];
    __shared__ u64 gofs[kRadix];
    __shared__ uint32_t stage[kTile];
    __shared__ uint8_t sdig[kTile];
    __shared__ uint32_t wsum[kRadix / 64];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t tile = xcd_tile(blockIdx.x, gridDim.x);
    for (int x = tid; x < kW * kRadix; x += TPB) (&wcnt[0][0])[x] = 0;
    if (tid < kRadix) gofs[tid] = goff[(uint64_t)tid * ntiles + tile];
    __syncthreads();
    const uint64_t tile0 = (uint64_t)tile * kTile;
    // rows: STABLE, wave w owns 64 * kSortItems consecutive rows (ranks in row order);
    // else thread-strided
    auto row = [&](int k) -> uint64_t {
        return STABLE ? tile0 + (uint64_t)wave * (64 * kSortItems) + (uint64_t)k * 64 + lane
                      : tile0 + (uint64_t)k * TPB + tid;
    };
    uint32_t el[kSortItems], dr[kSortItems];
#pragma unroll
    for (int k = 0; k < kSortItems; k++) {
        const uint64_t i = row(k);
        el[k] = __builtin_nontemporal_load(in + (i < n ? i : n - 1));
    }
#pragma unroll
    for (int k = 0; k < kSortItems; k++) {
        const uint64_t i = row(k);
        const bool valid = i < n;
        const uint32_t d = (win_id(el[k], t) >> shift) & 0xFF;
        if constexpr (STABLE) {
            const u64 peers = match_any8(d, __ballot(valid));
            const uint32_t lt = lanes_below(peers);
            const uint32_t cur = wcnt[wave][d];
            __builtin_amdgcn_wave_barrier();
            if (valid && lt == 0) wcnt[wave][d] = cur + (uint32_t)__popcll(peers);
            __builtin_amdgcn_wave_barrier();
            dr[k] = valid ? ((d << 16) | (cur + lt)) : 0xFFFFFFFFu;
        } else {
            dr[k] = valid ? (d << 16) | atomicAdd(&wcnt[0][d], 1u) : 0xFFFFFFFFu;
        }
    }
    __syncthreads();
    if constexpr (STABLE) tile_digit_offsets<TPB>(wcnt, loff, wsum, tid);
    else digit_scan(wcnt[0], loff, wsum, tid);
#pragma unroll
    for (int k = 0; k < kSortItems; k++) {
        const uint64_t i = row(k);
        if (dr[k] != 0xFFFFFFFFu) {
            const uint32_t d = dr[k] >> 16;
            const uint32_t sp = loff[d] + (STABLE ? wcnt[wave][d] : 0u) + (dr[k] & 0xFFFF);
            stage[sp] = el[k];
            sdig[sp] = (uint8_t)d;
            perm[i] = (uint16_t)sp;
        }
    }
    __syncthreads();
    const uint64_t tn = n - tile0 < (uint64_t)kTile ? n - tile0 : (uint64_t)kTile;
#pragma unroll
    for (int k = 0; k < kSortItems; k++) {
        const uint32_t e = (uint32_t)(k * TPB + tid);
        if (e < tn) {
            const uint32_t d = sdig[e];
            out[gofs[d] + (e - loff[d])] = stage[e];
        }
    }
}

// The inverse passes' view of a tile: gofs[d] = where digit d's run of the tile starts in
// the pass's output, loff[d] its tile-local start (from the pass's scanned offsets: a
// run's length is the next offset's distance), sdig[e] = the digit of place e.
__device__ __forceinline__ void tile_runs(const u64* __restrict__ goff, uint32_t ntiles, uint32_t tile, uint64_t n,
                                          u64* gofs, uint32_t* cnt, uint32_t* loff, uint8_t* sdig, uint32_t* wsum,
                                          int tid) {
    if (tid < kRadix) {
        const uint64_t x = (uint64_t)tid * ntiles + tile;
        const u64 g = goff[x], gn = x + 1 < (uint64_t)kRadix * ntiles ? goff[x + 1] : n;
        gofs[tid] = g;
        cnt[tid] = (uint32_t)(gn - g);
    }
    __syncthreads();
    digit_scan(cnt, loff, wsum, tid);
    if (tid < kRadix)
        for (uint32_t e = loff[tid], e1 = loff[tid] + cnt[tid]; e < e1; e++) sdig[e] = (uint8_t)tid;
    __syncthreads();
}

// Persistent window kernels (round 5): a window is a small job (8192 slots' worth of
// build words, ~4096 on average, and ~4096 probe keys), so a block walks windows w,
// w + G, ... (G = two blocks a CU). kWinPer build words and kJoinPer probe keys a thread
// cover 8192 / 5120 per window; probe keys past that are loaded in place. Round 5 issued
// the next window's loads into registers before the current window's LDS work; that
// took the kernels to 88-90 VGPRs, so only one 1024-lane block fitted a CU (the grid's
// second half waited for the first). Round 6 drops the register prefetch and caps the
// kernels at 8 waves a SIMD (64 VGPRs, no spills): two blocks share a CU and cover each
// other's loads. 2^28, alternating on one box: unique 7.59 -> 7.43 ms, many-to-many
// 9.18 -> 8.74 ms; the prefetch kept under the same cap spilled (40-52 B a lane) and
// measured 7.72 / 9.86.
//
// In LDS a window is not an open-addressing table but its words grouped by bucket (a
// counting sort, CSR): kCsrBuckets buckets by hash, one LDS atomic add per word gives
// its rank, a scan the buckets' starts, a store its place. A lookup reads its bucket's
// bounds and then the bucket's words (about one), which are independent reads. The
// table's CAS insert and linear probe were chains of dependent LDS round trips: the
// first form of these kernels (one window per block, k_win_build's CAS insert) took
// 1.6 ms for the check and 3.3 ms for the join at 2^28 rows.
constexpr int kJoinPer = 5;
constexpr int kWinPer = (1 << kWinLog) / kWinTPB;
constexpr uint32_t kCsrBuckets = 1u << (kWinLog - 1);        // 4096: about one word a bucket
constexpr uint32_t kCsrCap = (1u << kWinLog) - (1u << kWinLog) / 4;  // 6144 words: the 3/4 rule

__device__ __forceinline__ uint32_t csr_bucket(uint32_t key, const Win& t) {
    return (uint32_t)((hash32(key) & t.wmask) >> 1);
}

__device__ __forceinline__ void win_load(const u64* __restrict__ in, uint32_t b, uint32_t e, u64 (&v)[kWinPer]) {
#pragma unroll
    for (int k = 0; k < kWinPer; k++) {
        const uint32_t i = b + threadIdx.x + (uint32_t)k * kWinTPB;
        v[k] = i < e ? __builtin_nontemporal_load(in + i) : kEmpty;
    }
}

// The window's c words (c <= kCsrCap, threads' words vs[k] = word threadIdx + k * kWinTPB)
// grouped by bucket into csr; boff[b] .. boff[b + 1] = bucket b's words. Ends synced.
// cidx (when not null): each grouped word's index in the window's stretch (input order).
__device__ __forceinline__ void csr_build(const u64 (&vs)[kWinPer], uint32_t c, const Win& t, u64* csr,
                                          uint32_t* boff, uint32_t* wsum, uint16_t* cidx = nullptr) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (uint32_t x = tid; x <= kCsrBuckets; x += kWinTPB) boff[x] = 0;
    __syncthreads();
    uint32_t rk[kWinPer];
#pragma unroll
    for (int k = 0; k < kWinPer; k++) {
        const uint32_t i = (uint32_t)tid + (uint32_t)k * kWinTPB;
        rk[k] = i < c ? atomicAdd(&boff[csr_bucket((uint32_t)vs[k], t)], 1u) : 0u;
    }
    __syncthreads();
    // exclusive scan of the kCsrBuckets counts: 4 consecutive a thread
    constexpr int kQ = (int)(kCsrBuckets / kWinTPB);
    uint32_t cnt[kQ], tot = 0;
#pragma unroll
    for (int q = 0; q < kQ; q++) {
        cnt[q] = boff[tid * kQ + q];
        tot += cnt[q];
    }
    uint32_t incl = tot;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(incl, off, 64);
        if (lane >= off) incl += y;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    uint32_t run = incl - tot;
    for (int w = 0; w < wave; w++) run += wsum[w];
#pragma unroll
    for (int q = 0; q < kQ; q++) {
        boff[tid * kQ + q] = run;
        run += cnt[q];
    }
    if (tid == kWinTPB - 1) boff[kCsrBuckets] = run;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kWinPer; k++) {
        const uint32_t i = (uint32_t)tid + (uint32_t)k * kWinTPB;
        if (i < c) {
            const uint32_t x = boff[csr_bucket((uint32_t)vs[k], t)] + rk[k];
            csr[x] = vs[k];
            if (cidx) cidx[x] = (uint16_t)i;
        }
    }
    __syncthreads();
}

// One window at a time per block: the window's build words grouped in LDS, then each of
// the window's probe keys (partitioned order) looks itself up in its bucket. r[i] =
// payload << 32 | 1 on a hit, 0 on a miss. The build was not checked: a probe key that
// finds two build words sets bit 0 of *flag (the caller probes again with the duplicate-
// capable k_win_join_runs), a window over kCsrCap words bit 1 (the caller rebuilds
// without the partition; the table's empty word is an ordinary word here).
template <typename RT>
__global__ __launch_bounds__(kWinTPB) __attribute__((amdgpu_waves_per_eu(8))) void k_win_join(const u64* __restrict__ bwords,
                                                      const uint32_t* __restrict__ bstart,
                                                      const uint32_t* __restrict__ pkeys,
                                                      const uint32_t* __restrict__ pstartw, uint32_t nwin, Win t,
                                                      RT* __restrict__ r, uint32_t* __restrict__ flag,
                                                      uint32_t sentinel, unsigned long long* __restrict__ mtot) {
    __shared__ u64 csr[kCsrCap];
    __shared__ uint32_t boff[kCsrBuckets + 1];
    __shared__ uint32_t wsum[kWinTPB / 64];
    const uint32_t G = gridDim.x;
    uint32_t w = blockIdx.x;
    if (w >= nwin) return;
    auto key_load = [&](uint32_t pb, uint32_t pe, uint32_t (&key)[kJoinPer]) {
#pragma unroll
        for (int k = 0; k < kJoinPer; k++) {
            const uint32_t i = pb + threadIdx.x + (uint32_t)k * kWinTPB;
            key[k] = i < pe ? __builtin_nontemporal_load(pkeys + i) : 0u;
        }
    };
    bool dup = false, overfull = false;
    unsigned long long nhit = 0;  // the window joins' pairs (M, for the fused write)
    // a key on two build words shows up only where a probe key matches it (duplicates no
    // probe row meets do not change the unique output): then the flag
    auto lookup = [&](uint32_t key) -> RT {
        const uint32_t bk = csr_bucket(key, t);
        const uint32_t x0 = boff[bk], x1 = boff[bk + 1];
        u64 out = 0;
        uint32_t hits = 0;
        for (uint32_t x = x0; x < x1; x++) {
            const u64 v = csr[x];
            if ((uint32_t)v == key) out = (v & 0xFFFFFFFF00000000ull) | 1ull, hits++;
        }
        dup |= hits > 1;
        nhit += hits ? 1u : 0u;
        if constexpr (sizeof(RT) == 4) return hits ? (uint32_t)(out >> 32) : sentinel;
        else return out;
    };
    // The loads' order decides what the wait-count pass can overlap (it waits for a
    // register's load with vmcnt(n), n = the younger memory operations, unknown past a
    // data-dependent number of stores): the next window's build words are issued at the
    // top and waited for after this window's grouping, the next window's probe keys
    // after this window's stores; nothing waits on this window's stores.
    for (; w < nwin; w += G) {
        const uint32_t b = bstart[w], e = bstart[w + 1], pb = pstartw[w], pe = pstartw[w + 1];
        u64 vs[kWinPer];
        uint32_t key[kJoinPer];
        win_load(bwords, b, e, vs);
        key_load(pb, pe, key);
        const bool over = e - b > kCsrCap;  // uniform: an overfull window (its results are dropped)
        if (!over) csr_build(vs, e - b, t, csr, boff, wsum);
        if (over) {
            overfull = true;
        } else {
#pragma unroll
            for (int k = 0; k < kJoinPer; k++) {
                const uint32_t i = pb + threadIdx.x + (uint32_t)k * kWinTPB;
                if (i < pe) __builtin_nontemporal_store(lookup(key[k]), r + i);
            }
            for (uint32_t i = pb + threadIdx.x + (uint32_t)kJoinPer * kWinTPB; i < pe; i += kWinTPB)
                __builtin_nontemporal_store(lookup(__builtin_nontemporal_load(pkeys + i)), r + i);
            __syncthreads();
        }
    }
    if (dup || overfull) atomicOr(flag, (dup ? 1u : 0u) | (overfull ? 2u : 0u));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) nhit += __shfl_xor(nhit, o, 64);
    if ((threadIdx.x & 63) == 0 && nhit) atomicAdd(mtot, nhit);
}

// The partitioned probe of a windowed RUNS table (duplicate keys, k_win_build_runs: the
// window's slots hold {key, start << 4 | length}): the window's 64 KB slice of the
// global table is loaded into LDS whole (coalesced) and each of the window's probe keys
// follows the table's own probe sequence there (home bucket, linear inside the window,
// an empty slot ends it). r[i] = the slot's packed run, 0 = no match (a run is never
// empty, so a hit's payload is never 0). (Round 5's u64 form carried short runs' build
// positions from the run array; round 6's k_win_join_runs does that without the table.)
template <typename RT>
__global__ __launch_bounds__(kWinTPB) void k_win_probe_tab(const u64* __restrict__ words,
                                                           const uint32_t* __restrict__ pkeys,
                                                           const uint32_t* __restrict__ pstartw, uint32_t nwin, Win t,
                                                           RT* __restrict__ r) {
    static_assert(sizeof(RT) == 4, "packed runs");
    __shared__ u64 tab[1 << kWinLog];
    const uint32_t W = (uint32_t)t.wmask + 1, G = gridDim.x;
    uint32_t w = blockIdx.x;
    if (w >= nwin) return;
    auto key_load = [&](uint32_t pb, uint32_t pe, uint32_t (&key)[kJoinPer]) {
#pragma unroll
        for (int k = 0; k < kJoinPer; k++) {
            const uint32_t i = pb + threadIdx.x + (uint32_t)k * kWinTPB;
            key[k] = i < pe ? __builtin_nontemporal_load(pkeys + i) : 0u;
        }
    };
    auto lookup = [&](uint32_t key) -> RT {
        uint32_t h = (uint32_t)ht_home(key, t.wmask);
        uint32_t pk = 0;
        for (uint32_t step = 0; step < W; step++) {
            const u64 v = tab[h];
            if (v == kEmpty) break;
            if ((uint32_t)v == key) {
                pk = (uint32_t)(v >> 32);
                break;
            }
            h = (h + 1) & (W - 1);
        }
        return pk;
    };
    uint32_t pb = pstartw[w], pe = pstartw[w + 1];
    u64 vs[kWinPer];
    uint32_t key[kJoinPer];
    win_load(words + (uint64_t)w * W, 0, W, vs);
    key_load(pb, pe, key);
    uint32_t pbn = 0, pen = 0;
    if (w + G < nwin) pbn = pstartw[w + G], pen = pstartw[w + G + 1];
    __builtin_amdgcn_s_waitcnt(0);  // (see k_win_join)
    for (; w < nwin; w += G) {
        u64 vn[kWinPer];
        win_load(words + (uint64_t)(w + G < nwin ? w + G : w) * W, 0, w + G < nwin ? W : 0, vn);
        uint32_t pbnn = 0, penn = 0;
        if (w + 2 * G < nwin) pbnn = pstartw[w + 2 * G], penn = pstartw[w + 2 * G + 1];
#pragma unroll
        for (int k = 0; k < kWinPer; k++) tab[threadIdx.x + (uint32_t)k * kWinTPB] = vs[k];
        __syncthreads();
#pragma unroll
        for (int k = 0; k < kWinPer; k++) {
            asm volatile("" : "+v"(vn[k]));  // the next slice waited for here, not behind the stores
            vs[k] = vn[k];
        }
#pragma unroll
        for (int k = 0; k < kJoinPer; k++) {
            const uint32_t i = pb + threadIdx.x + (uint32_t)k * kWinTPB;
            if (i < pe) __builtin_nontemporal_store(lookup(key[k]), r + i);
        }
        for (uint32_t i = pb + threadIdx.x + (uint32_t)kJoinPer * kWinTPB; i < pe; i += kWinTPB)
            __builtin_nontemporal_store(lookup(__builtin_nontemporal_load(pkeys + i)), r + i);
        __syncthreads();
        key_load(pbn, pen, key);
        pb = pbn, pe = pen, pbn = pbnn, pen = penn;
    }
}

// The partitioned probe for DUPLICATE build keys (round 6): no runs table. The build
// words stay partitioned by window as for unique keys (the stable LSD passes keep a
// window's words in input order, their stretch index i); per window the block groups
// them by bucket in LDS (csr_build, with each word's i) and answers each probe key of
// the window from its bucket: the words of equal key are the key's build rows, ordered
// by i (build-insertion order, query.c:669-681). r[k] is the run2 record the gathers
// and the write read: {p0, S} for one row, {p0, p1} for two (in order), {S, (b + s) << 4
// | L} for L = 3..14 rows, whose build positions are in bpos[b + s ...] in insertion
// order (s = the run's place when the bucket is ordered by (key, i), so every run has its
// own stretch inside the window's; written by the probe keys that meet the run, each the
// same values), and {S, 0} for a miss. S: a value outside the build payloads (the host
// checks one exists). A window over kCsrCap words or a probed key on 15+ rows sets *flag
// (the caller rebuilds on the sorted runs); *mtot += the pairs (sum of L over the probe
// keys).
// Replaces k_win_build_runs (the 4 GB runs table written by the build, 1.9 ms at 2^28)
// and k_win_probe_tab (reading it back, 1.76 ms).
__global__ __launch_bounds__(kWinTPB) __attribute__((amdgpu_waves_per_eu(8))) void k_win_join_runs(const u64* __restrict__ bwords,
                                                           const uint32_t* __restrict__ bstart,
                                                           const uint32_t* __restrict__ pkeys,
                                                           const uint32_t* __restrict__ pstartw, uint32_t nwin, Win t,
                                                           u64* __restrict__ r, int* __restrict__ bpos,
                                                           uint32_t* __restrict__ flag, unsigned long long* mtot,
                                                           uint32_t S) {
    __shared__ u64 csr[kCsrCap];
    __shared__ uint32_t boff[kCsrBuckets + 1];
    __shared__ uint16_t cidx[kCsrCap];
    __shared__ uint32_t wsum[kWinTPB / 64];
    const uint32_t G = gridDim.x;
    uint32_t w = blockIdx.x;
    if (w >= nwin) return;
    auto key_load = [&](uint32_t pb, uint32_t pe, uint32_t (&key)[kJoinPer]) {
#pragma unroll
        for (int k = 0; k < kJoinPer; k++) {
            const uint32_t i = pb + threadIdx.x + (uint32_t)k * kWinTPB;
            key[k] = i < pe ? __builtin_nontemporal_load(pkeys + i) : 0u;
        }
    };
    bool bad = false;
    unsigned long long pairs = 0;
    // key k's words in bucket [x0, x1): count L, those below k (its run's place in the
    // bucket ordered by (key, i)), and the first two by i
    auto scan_bucket = [&](uint32_t key, uint32_t b, uint32_t x0, uint32_t x1, uint32_t& L, uint32_t& lt,
                           uint32_t& p0, uint32_t& p1) {
        // the first two matches in bucket order, then put in input order (selects, no
        // array: an insertion by index compiled to a scratch array)
        uint32_t n = 0, ia = 0, ib = 0, pa = S, pb = S;
        for (uint32_t x = x0; x < x1; x++) {
            const u64 v = csr[x];
            if ((uint32_t)v == key) {
                const uint32_t i = cidx[x], p = (uint32_t)(v >> 32);
                ia = n == 0 ? i : ia;
                pa = n == 0 ? p : pa;
                ib = n == 1 ? i : ib;
                pb = n == 1 ? p : pb;
                n++;
            }
        }
        const bool sw = n == 2 && ib < ia;
        p0 = sw ? pb : pa;
        p1 = sw ? pa : pb;
        L = n;
        lt = 0;
        if (n >= 3u) {
            // a long run: its place in the bucket ordered by (key, i), and its rows' payloads
            // written there in insertion order by every probe key that meets it (the same
            // values to the same places: no race); no key of the window pays otherwise
            for (uint32_t x = x0; x < x1; x++) lt += (uint32_t)csr[x] < key ? 1u : 0u;
            if (n < 15u)
                for (uint32_t x = x0; x < x1; x++) {
                    const u64 v = csr[x];
                    if ((uint32_t)v != key) continue;
                    const uint32_t me = cidx[x];
                    uint32_t rk = 0;
                    for (uint32_t y = x0; y < x1; y++)
                        rk += ((uint32_t)csr[y] == key && cidx[y] < me) ? 1u : 0u;
                    bpos[b + x0 + lt + rk] = (int)(uint32_t)(v >> 32);
                }
            else
                bad = true;  // not packable: the caller takes the sorted runs
        }
    };
    auto lookup = [&](uint32_t key, uint32_t b) -> u64 {
        const uint32_t bk = csr_bucket(key, t);
        const uint32_t x0 = boff[bk], x1 = boff[bk + 1];
        uint32_t L, lt, p0, p1;
        scan_bucket(key, b, x0, x1, L, lt, p0, p1);
        pairs += L;
        if (L == 0) return (u64)S;
        if (L <= 2) return (u64)p0 | ((u64)p1 << 32);
        return (u64)S | ((u64)(((b + x0 + lt) << 4) | (L < 15u ? L : 15u)) << 32);
    };
    for (; w < nwin; w += G) {  // (no register prefetch of the next window: see k_win_join)
        const uint32_t b = bstart[w], e = bstart[w + 1], pb = pstartw[w], pe = pstartw[w + 1];
        u64 vs[kWinPer];
        uint32_t key[kJoinPer];
        win_load(bwords, b, e, vs);
        key_load(pb, pe, key);
        const uint32_t c = e - b;
        const bool over = c > kCsrCap;  // uniform
        if (!over) csr_build(vs, c, t, csr, boff, wsum, cidx);
        if (over) {
            bad = true;
        } else {
#pragma unroll
            for (int k = 0; k < kJoinPer; k++) {
                const uint32_t i = pb + threadIdx.x + (uint32_t)k * kWinTPB;
                if (i < pe) __builtin_nontemporal_store(lookup(key[k], b), r + i);
            }
            for (uint32_t i = pb + threadIdx.x + (uint32_t)kJoinPer * kWinTPB; i < pe; i += kWinTPB)
                __builtin_nontemporal_store(lookup(__builtin_nontemporal_load(pkeys + i), b), r + i);
            __syncthreads();
        }
    }
    if (bad) *flag = 1;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) pairs += __shfl_xor(pairs, o, 64);
    if ((threadIdx.x & 63) == 0 && pairs) atomicAdd(mtot, pairs);
}

// The inverse of one k_pwin_scatter pass: perm = that pass's places (a row's place in
// its tile's digit order), rin = per-row results in the pass's output order; rout[i] =
// the result of input row i. Each digit's run of the tile is read from rin as a
// contiguous stretch (staged in LDS by place) and every row takes its own value back.
// FINAL (the pass over the probe column itself): per row the payload (pstart) and, per
// 64 rows, the hit word.
// RUNS (with FINAL): rin holds packed runs (0 = no match); per row pstart = the packed
// run and per 64 rows wcnt = the sum of their run lengths, as k_ht_probe_unique<true>
// leaves them for the packed-runs write (hits is then that wcnt, as u32).
template <bool FINAL, typename RT, bool RUNS, int TPB>
__global__ __launch_bounds__(TPB) void k_pwin_gather(const uint16_t* __restrict__ perm, uint64_t n,
                                                     const u64* __restrict__ goff, uint32_t ntiles,
                                                     const RT* __restrict__ rin, RT* __restrict__ rout,
                                                     uint32_t* __restrict__ pstart, u64* __restrict__ hits,
                                                     uint32_t sentinel) {
    constexpr int kTile = TPB * kSortItems;
    __shared__ uint32_t cnt[kRadix];
    __shared__ uint32_t loff[kRadix];
    __shared__ u64 gofs[kRadix];
    __shared__ RT stage[kTile];
    __shared__ uint8_t sdig[kTile];
    __shared__ uint32_t wsum[kRadix / 64];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t tile = xcd_tile(blockIdx.x, gridDim.x);
    const uint64_t tile0 = (uint64_t)tile * kTile;
    const uint64_t seg = tile0 + (uint64_t)wave * (64 * kSortItems);
    uint32_t sp[kSortItems];  // each row's place in the tile's digit order
#pragma unroll
    for (int k = 0; k < kSortItems; k++) {
        const uint64_t i = seg + (uint64_t)k * 64 + lane;
        sp[k] = __builtin_nontemporal_load(perm + (i < n ? i : n - 1));
    }
    tile_runs(goff, ntiles, tile, n, gofs, cnt, loff, sdig, wsum, tid);
    const uint64_t tn = n - tile0 < (uint64_t)kTile ? n - tile0 : (uint64_t)kTile;
    {
        RT v[kSortItems];  // all reads in flight first
#pragma unroll
        for (int k = 0; k < kSortItems; k++) {
            const uint32_t e = (uint32_t)(k * TPB + tid);
            const uint32_t d = e < tn ? sdig[e] : 0u;
            v[k] = e < tn ? __builtin_nontemporal_load(rin + gofs[d] + (e - loff[d])) : (RT)0;
        }
#pragma unroll
        for (int k = 0; k < kSortItems; k++) stage[k * TPB + tid] = v[k];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kSortItems; k++) {
        const uint64_t i = seg + (uint64_t)k * 64 + lane;
        const bool in = i < n;
        const RT v = in ? stage[sp[k]] : (RT)0;
        if constexpr (FINAL && RUNS && sizeof(RT) == 8) {
            // run2 records: pstart = a packed run (long) or just its length (one or two rows,
            // whose positions go to rout = p01), as k_join_write_runs16 reads them
            const uint32_t lo = (uint32_t)v, hi = (uint32_t)((u64)v >> 32);
            const bool direct = lo != sentinel;
            const uint32_t pk = !in ? 0u : direct ? (hi == sentinel ? 1u : 2u) : hi;
            uint32_t L = pk & 15u;
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) L += __shfl_xor(L, o, 64);
            if (i < n) {
                __builtin_nontemporal_store(pk, pstart + i);
                __builtin_nontemporal_store((in && direct) ? (u64)v : 0ull, reinterpret_cast<u64*>(rout) + i);
            }
            if (lane == 0 && i < n) reinterpret_cast<uint32_t*>(hits)[i >> 6] = L;
        } else if constexpr (FINAL && RUNS) {
            const uint32_t pay = (uint32_t)v;
            uint32_t L = pay & 15u;  // (a windowed runs table: every run shorter than 15)
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) L += __shfl_xor(L, o, 64);
            if (i < n) __builtin_nontemporal_store(pay, pstart + i);
            if (lane == 0 && i < n) reinterpret_cast<uint32_t*>(hits)[i >> 6] = L;
        } else if constexpr (FINAL) {
            bool hit;
            uint32_t pay;
            if constexpr (sizeof(RT) == 4) {
                hit = in && (uint32_t)v != sentinel;
                pay = (uint32_t)v;
            } else {
                hit = ((u64)v & 1ull) != 0;
                pay = (uint32_t)((u64)v >> 32);
            }
            const u64 m = __ballot(hit);
            if (i < n) __builtin_nontemporal_store(pay, pstart + i);
            if (lane == 0 && i < n) hits[i >> 6] = m;
        } else {
            if (i < n) __builtin_nontemporal_store(v, rout + i);
        }
    }
}

// The last inverse pass fused with the pair write (round 6): k_pwin_gather<true>'s tile
// (its probe rows in row order; each row's result taken back from the window join's
// order) counts its pairs, learns the pairs of every earlier tile by decoupled look-back
// and writes its rows' pairs straight to out1 / out2, so neither the per-row results
// (pstart, p01: 4-12 B a row written and read back) nor the hit words, their scan and a
// separate write pass exist. MODE 0: unique, u32 results (sentinel = miss); 1: unique,
// u64 {payload << 32 | 1} (0 = miss); 2: run2 records (k_win_join_runs), runs of 3-14
// rows read from bpos. status[t] = kLbAgg | the tile's pairs, then kLbPre | the pairs of
// tiles 0..t.
// Tile order (kGwGroup): a digit's runs of neighbouring tiles share cache lines of rin,
// so neighbours should run on one XCD. Blocks are dispatched in blockIdx order, dealt
// round-robin over the 8 XCDs; in each group of 8 * kGwGroup blocks, the kGwGroup blocks
// of one XCD take kGwGroup consecutive tiles (a partial last group keeps blockIdx order).
// A tile waits only on lower tiles, whose blocks come earlier in dispatch order or in the
// same group (as k_select_stage relies on lower blocks being dispatched first). Round 6,
// 2^28 joins alternating on one box: tiles by an atomic ticket (order of block start, any
// XCD) 8.78 / 10.58 ms, groups of 4 8.70 / 10.47 (reads 1.75x -> 1.59x the design bytes,
// unique), groups of 8 8.77 / 10.62; 4 tiles a ticket in one block serialised the chain.
constexpr u64 kLbAgg = 1ull << 62, kLbPre = 2ull << 62, kLbVal = (1ull << 62) - 1;
constexpr uint32_t kGwGroup = 4;

__device__ __forceinline__ u64 lb_load(const u64* p) {
    return __hip_atomic_load(const_cast<u64*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void lb_store(u64* p, u64 v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <typename RT, int MODE, int TPB>
__global__ __launch_bounds__(TPB) void k_pwin_gather_write(const uint16_t* __restrict__ perm, uint64_t n,
                                                            const u64* __restrict__ goff, uint32_t ntiles,
                                                            const RT* __restrict__ rin, const int* __restrict__ p2,
                                                            const int* __restrict__ bpos, uint32_t sentinel,
                                                            int* __restrict__ out1, int* __restrict__ out2,
                                                            u64* status, uint32_t* err) {
    constexpr int kTile = TPB * kSortItems;
    __shared__ uint32_t cnt[kRadix];
    __shared__ uint32_t loff[kRadix];
    __shared__ u64 gofs[kRadix];
    __shared__ RT stage[kTile];
    __shared__ uint8_t sdig[kTile];
    __shared__ uint32_t wsum[TPB / 64];
    __shared__ u64 s_excl;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint32_t tile = blockIdx.x;  // (see kGwGroup)
    {
        constexpr uint32_t kSpan = 8u * kGwGroup;
        const uint32_t g0 = tile - tile % kSpan;
        if (g0 + kSpan <= ntiles) tile = g0 + (tile & 7u) * kGwGroup + (tile % kSpan) / 8u;
    }
    const uint64_t tile0 = (uint64_t)tile * kTile;
    const uint64_t seg = tile0 + (uint64_t)wave * (64 * kSortItems);
    uint32_t sp[kSortItems];  // each row's place in the tile's digit order
    int pv[kSortItems];       // the rows' probe positions, loaded with the places (a load at
                              // each store serialised 16 round trips a wave)
#pragma unroll
    for (int k = 0; k < kSortItems; k++) {
        const uint64_t i = seg + (uint64_t)k * 64 + lane;
        sp[k] = __builtin_nontemporal_load(perm + (i < n ? i : n - 1));
        pv[k] = out2 ? __builtin_nontemporal_load(p2 + (i < n ? i : n - 1)) : 0;
    }
    tile_runs(goff, ntiles, tile, n, gofs, cnt, loff, sdig, wsum, tid);
    const uint64_t tn = n - tile0 < (uint64_t)kTile ? n - tile0 : (uint64_t)kTile;
    {
        RT v[kSortItems];
#pragma unroll
        for (int k = 0; k < kSortItems; k++) {
            const uint32_t e = (uint32_t)(k * TPB + tid);
            const uint32_t d = e < tn ? sdig[e] : 0u;
            v[k] = e < tn ? __builtin_nontemporal_load(rin + gofs[d] + (e - loff[d])) : (RT)0;
        }
#pragma unroll
        for (int k = 0; k < kSortItems; k++) stage[k * TPB + tid] = v[k];
    }
    __syncthreads();
    // each row's pair count (from its result, read from stage twice: once for the wave's
    // total, once for the write, instead of holding results, counts and prefixes in
    // registers: 229 VGPRs, 2 waves a SIMD). Counts are below 16, so a wave's prefix and
    // total are 4 bit-ballots (1 for unique keys). Row order: wave, item, lane.
    auto count_of = [&](RT v) -> uint32_t {
        if constexpr (MODE == 0) {
            return (uint32_t)v != sentinel ? 1u : 0u;
        } else if constexpr (MODE == 1) {
            return (uint32_t)((u64)v & 1ull);
        } else {
            const uint32_t lo = (uint32_t)v, hi = (uint32_t)((u64)v >> 32);
            return lo != sentinel ? (hi == sentinel ? 1u : 2u) : (hi & 15u);
        }
    };
    constexpr int kBits = MODE == 2 ? 4 : 1;
    auto wave_prefix = [&](uint32_t c, uint32_t& tot) -> uint32_t {
        uint32_t pre = 0;
        tot = 0;
#pragma unroll
        for (int b = 0; b < kBits; b++) {
            const u64 m = __ballot((c >> b) & 1u);
            pre += lanes_below(m) << b;
            tot += (uint32_t)__popcll(m) << b;
        }
        return pre;
    };
    uint32_t wrun = 0;
#pragma unroll
    for (int k = 0; k < kSortItems; k++) {
        const uint64_t i = seg + (uint64_t)k * 64 + lane;
        const uint32_t c = i < n ? count_of(stage[sp[k]]) : 0u;
        uint32_t tot;
        (void)wave_prefix(c, tot);
        wrun += tot;
    }
    __syncthreads();  // (wsum reused)
    if (lane == 0) wsum[wave] = wrun;
    __syncthreads();
    uint32_t wbase = 0, ttot = 0;
#pragma unroll
    for (int w = 0; w < TPB / 64; w++) {
        wbase += w < wave ? wsum[w] : 0u;
        ttot += wsum[w];
    }
    // decoupled look-back over the earlier tiles (wave 0)
    if (wave == 0) {
        if (lane == 0) lb_store(&status[tile], (tile ? kLbAgg : kLbPre) | (u64)ttot);
        u64 acc = 0;
        int64_t j = (int64_t)tile - 1;
        uint32_t spins = 0;
        while (j >= 0) {
            const int64_t idx = j - lane;
            u64 x = idx >= 0 ? lb_load(&status[idx]) : kLbPre;
            // every lane's status published (bounded: never expected to run long)
            while (__ballot((x & ~kLbVal) == 0)) {
                if (++spins > (1u << 24)) {
                    if (lane == 0) atomicOr(err, 1u);
                    x = kLbPre;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
                if ((x & ~kLbVal) == 0) x = lb_load(&status[idx]);
            }
            const u64 pm = __ballot((x & kLbPre) != 0);
            const int stop = pm ? __ffsll((long long)pm) - 1 : 64;  // the nearest inclusive prefix
            u64 val = lane <= stop ? (x & kLbVal) : 0ull;
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) val += __shfl_xor(val, o, 64);
            acc += val;
            if (pm) break;
            j -= 64;
        }
        if (lane == 0) {
            if (tile) lb_store(&status[tile], kLbPre | (acc + ttot));
            s_excl = acc;
        }
    }
    __syncthreads();
    u64 o = s_excl + wbase;  // (wave-uniform) the first pair of this wave's next item
#pragma unroll
    for (int k = 0; k < kSortItems; k++) {
        const uint64_t i = seg + (uint64_t)k * 64 + lane;
        const RT v = i < n ? stage[sp[k]] : (RT)0;
        const uint32_t c = i < n ? count_of(v) : 0u;
        uint32_t tot;
        const uint32_t pre = wave_prefix(c, tot);
        if (c) {
            const u64 q = o + pre;
            const int pp = pv[k];
            if constexpr (MODE == 0) {
                out1[q] = (int)(uint32_t)v;
                if (out2) out2[q] = pp;
            } else if constexpr (MODE == 1) {
                out1[q] = (int)(uint32_t)((u64)v >> 32);
                if (out2) out2[q] = pp;
            } else {
                const uint32_t lo = (uint32_t)v, hi = (uint32_t)((u64)v >> 32);
                if (lo != sentinel) {
                    out1[q] = (int)lo;
                    if (out2) out2[q] = pp;
                    if (c == 2u) {
                        out1[q + 1] = (int)hi;
                        if (out2) out2[q + 1] = pp;
                    }
                } else {
                    const uint32_t a = hi >> 4;
                    for (uint32_t e = 0; e < c; e++) {
                        out1[q + e] = bpos[a + e];
                        if (out2) out2[q + e] = pp;
                    }
                }
            }
        }
        o += tot;
    }
}

// Duplicate keys without a sort (round 3): the build rows are partitioned by window
// like the unique build's (stable, so a window's rows keep their input order), and
// one block per window finds the runs itself. In LDS: its keys go into the window's
// slots by CAS (u32 keys; the key -1, the u32 empty marker, flags), a u16 count per
// slot, one scan over the slots in slot order gives each slot's run its place in
// the window's stretch of the run array, and each row takes a place in its run by
// one atomic; rows of a key arrive at their places in any order, so a row's final
// place is its run's start + the number of the run's rows before it in input order
// (their input indices sit in LDS by place). The row writes its payload there (the
// key's build positions in insertion order, bpos), and the window's table words
// carry {key, start << 4 | length} with the unique build's overflow marks. A window
// of more than kRunRows rows or a key on 15 rows or more (not packable) flags
// *general; the caller then takes the sorted-runs build. Replaces, at 2^28 rows with
// every key twice, the 4-pass sort of the pairs, the run extraction and the
// partition of the distinct keys.
constexpr uint32_t kRunRows = 6144;  // rows a window block takes (3/4 of its slots)
constexpr uint32_t kEmpty32 = ~0u;

__global__ __launch_bounds__(kWinTPB) void k_win_build_runs(const u64* __restrict__ in,
                                                            const uint32_t* __restrict__ wstart,
                                                            u64* __restrict__ words, int* __restrict__ bpos, Win t,
                                                            uint32_t* __restrict__ general) {
    constexpr uint32_t W = 1u << kWinLog;
    constexpr int kPer = (int)(kRunRows / kWinTPB);  // rows per thread
    constexpr int kW = kWinTPB / 64;
    __shared__ uint32_t tab[W];          // keys by slot
    __shared__ uint32_t c32[W / 2];      // u16 per slot: counts, then run places
    __shared__ uint16_t pidx[kRunRows];  // input index (within the window) by place
    __shared__ uint8_t ovf[W / kBucket];
    __shared__ uint32_t wsum[kW + 1];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t w = blockIdx.x;
    const uint32_t b = wstart[w], e = wstart[w + 1], c = e - b;
    if (W != (uint32_t)t.wmask + 1 || c > kRunRows) {  // (a table smaller than one window: never here)
        if (tid == 0) *general = 1;
        return;
    }
    for (uint32_t x = tid; x < W; x += kWinTPB) tab[x] = kEmpty32;
    for (uint32_t x = tid; x < W / 2; x += kWinTPB) c32[x] = 0;
    for (uint32_t x = tid; x < W / kBucket; x += kWinTPB) ovf[x] = 0;
    if (tid == 0) wsum[kW] = 0;
    __syncthreads();
    uint32_t key[kPer], pay[kPer], slot[kPer];
#pragma unroll
    for (int k = 0; k < kPer; k++) {
        const uint32_t i = (uint32_t)k * kWinTPB + tid;
        const u64 v = i < c ? in[b + i] : 0ull;
        key[k] = (uint32_t)v;
        pay[k] = (uint32_t)(v >> 32);
    }
    bool bad = false;
#pragma unroll
    for (int k = 0; k < kPer; k++) {
        slot[k] = 0;
        if ((uint32_t)k * kWinTPB + tid >= c) continue;
        if (key[k] == kEmpty32) {
            bad = true;
            continue;
        }
        const uint32_t h0 = (uint32_t)ht_home(key[k], t.wmask);
        uint32_t h = h0;
        for (uint32_t step = 0; step < W; step++) {
            const uint32_t old = atomicCAS(&tab[h], kEmpty32, key[k]);
            if (old == kEmpty32 || old == key[k]) {
                if (old == kEmpty32 && step >= kBucket) ovf[h0 / kBucket] = 1;
                break;
            }
            h = (h + 1) & (W - 1);
        }
        slot[k] = h;
        atomicAdd(&c32[h >> 1], 1u << (16 * (h & 1)));
    }
    if (bad) wsum[kW] = 1;
    __syncthreads();
    // exclusive scan of the counts in slot order: lane-consecutive words, 4 a thread
    constexpr int kQ = (int)(W / 2 / kWinTPB);
    uint32_t* mine = c32 + (uint32_t)tid * kQ;
    uint32_t tot = 0, mx = 0;
#pragma unroll
    for (int j = 0; j < kQ; j++) {
        const uint32_t cell = mine[j], lo = cell & 0xFFFFu, hi = cell >> 16;
        mx = lo > mx ? lo : mx;
        mx = hi > mx ? hi : mx;
        tot += lo + hi;
    }
    uint32_t incl = tot;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(incl, off, 64);
        if (lane >= off) incl += y;
    }
    if (lane == 63) wsum[wave] = incl;
    if (__ballot(mx >= 15u)) wsum[kW] = 1;  // a run the packed payload cannot hold
    __syncthreads();
    if (wsum[kW]) {
        if (tid == 0) *general = 1;
        return;
    }
    uint32_t run = incl - tot;
    for (int v = 0; v < wave; v++) run += wsum[v];
#pragma unroll
    for (int j = 0; j < kQ; j++) {
        const uint32_t cell = mine[j], lo = cell & 0xFFFFu;
        mine[j] = run | ((run + lo) << 16);
        run += lo + (cell >> 16);
    }
    __syncthreads();
    uint32_t place[kPer];
#pragma unroll
    for (int k = 0; k < kPer; k++) {
        place[k] = 0;
        const uint32_t i = (uint32_t)k * kWinTPB + tid;
        if (i >= c) continue;
        const uint32_t h = slot[k], sh = 16 * (h & 1);
        place[k] = (atomicAdd(&c32[h >> 1], 1u << sh) >> sh) & 0xFFFFu;
        pidx[place[k]] = (uint16_t)i;
    }
    __syncthreads();
    // c32 now holds each slot's run end; its run starts where slot h - 1's ends.
    // The window's table words first, a bucket (4 slots) per thread, with the overflow
    // marks; then tab's space stages the payloads by final place, so the run array
    // leaves in one coalesced copy (the rows' own stores were scattered 4-byte writes)
    const uint16_t* c16 = reinterpret_cast<const uint16_t*>(c32);
    u64* dst = words + (uint64_t)w * W;
    for (uint32_t bk = tid; bk < W / kBucket; bk += kWinTPB) {
        u64 o[kBucket];
        bool full = true;
#pragma unroll
        for (uint32_t q = 0; q < kBucket; q++) {
            const uint32_t h = bk * kBucket + q;
            const uint32_t k = tab[h];
            if (k == kEmpty32) {
                o[q] = kEmpty;
                full = false;
            } else {
                const uint32_t s0 = h ? c16[h - 1] : 0u, s1 = c16[h];
                o[q] = (u64)k | ((u64)(((b + s0) << 4) | (s1 - s0)) << 32);
            }
        }
        if (full && (((uint32_t)o[0] > (uint32_t)o[1]) != (ovf[bk] != 0))) {
            const u64 x = o[0];
            o[0] = o[1];
            o[1] = x;
        }
#pragma unroll
        for (uint32_t q = 0; q < kBucket; q++) dst[bk * kBucket + q] = o[q];
    }
    __syncthreads();
    uint32_t* stage = tab;  // (W >= kRunRows)
#pragma unroll
    for (int k = 0; k < kPer; k++) {
        const uint32_t i = (uint32_t)k * kWinTPB + tid;
        if (i >= c) continue;
        const uint32_t h = slot[k];
        const uint32_t s0 = h ? c16[h - 1] : 0u, s1 = c16[h];
        uint32_t r = 0;
        for (uint32_t q = s0; q < s1; q++) r += pidx[q] < i;
        stage[s0 + r] = pay[k];
    }
    __syncthreads();
    for (uint32_t x = tid; x < c; x += kWinTPB) bpos[b + x] = (int)stage[x];
}

// 2 probes per thread per step: with whole-bucket loads 2 beat 8 (8.25 vs 8.8 ms at
// 2^28, same box: fewer VGPRs, more waves); with single-slot loads 8 had beaten 1.
constexpr int kProbeILP = 2;
constexpr uint32_t kContCap = 320;  // queued continuations per wave (64 taken + 2 x 128 new fit)

// One probe row's outputs. RUNS: the run start and length (0 = no match), from the
// packed payload or, for a long run (or unpacked), from rs. Unique: the payload (the
// build position), whose hit bit is the caller's.
template <bool RUNS>
__device__ __forceinline__ void probe_emit(uint64_t j, bool hit, uint32_t payload, uint32_t* __restrict__ pstart,
                                           const uint32_t* __restrict__ rs, uint32_t* __restrict__ cnt,
                                           bool packed) {
    if constexpr (RUNS) {
        if (!cnt) {  // packed runs: the payload itself (0 = miss), decoded by the write
            pstart[j] = hit ? payload : 0u;
            return;
        }
        uint32_t a = 0, L = 0;
        if (hit) {
            L = packed ? payload & 15u : 15u;
            a = packed ? payload >> 4 : payload;
            if (L == 15u) {
                L = rs[a + 1] - rs[a];
                a = rs[a];
            }
        }
        pstart[j] = a;
        cnt[j] = L;
    } else {
        pstart[j] = payload;  // (misses store 0: whole lines)
    }
}

// A packed run payload's length (a hit's payload is never 0; 15 = look the run up).
__device__ __forceinline__ uint32_t run_len(uint32_t payload, const uint32_t* __restrict__ rs) {
    const uint32_t L = payload & 15u;
    if (L != 15u) return L;
    const uint32_t r = payload >> 4;
    return rs[r + 1] - rs[r];
}

// kProbeILP probes per thread per step: the keys are loaded coalesced, then all
// their home buckets (4 slots, 32 B, two 16-byte loads) are requested before any
// is examined. Random reads cost per 32-B sector (tools/random_read: a 64-B bucket
// takes 10.4 ms at 2^28 where 32 B take 5.6), so every slot read past the bucket
// costs about as much as the bucket itself; a line is long gone from L2 by the
// time a wave comes back to it. Two things keep those reads rare:
//  * overflow marks (windowed builds): a full bucket's slot order says whether any
//    key homed there lies past it; a miss in a full bucket without one ends there
//    (continuations at load 1/2: 10 % of probes -> 5 %; 8.2 -> 6.8 ms);
//  * the rest are not followed on the spot, where the wave would wait for one
//    dependent read per slot: the row goes to a per-wave queue in LDS, and each
//    step the wave takes up to 64 queued rows and requests their next slot with
//    the new buckets, in the same round trip (an unresolved row is requeued).
// RUNS (duplicate keys as runs, the payload a packed run, see run_payload): per row
// the run's start in pstart and its length in cnt (0 = no match) instead of hit
// words. Row indices and steps are kept as u32 (n2 <= 2^31 rows).
template <bool RUNS>
__global__ __launch_bounds__(kTPB) void k_ht_probe_unique(const int* __restrict__ pkeys, uint64_t n2,
                                                          const u64* __restrict__ words, Win t,
                                                          uint32_t* __restrict__ pstart,
                                                          u64* __restrict__ hits, const uint32_t* __restrict__ rs,
                                                          uint32_t* __restrict__ cnt, bool packed, bool marks,
                                                          uint32_t* __restrict__ wcnt) {
    constexpr uint32_t kB = kBucket;
    auto home = [&](uint32_t key) { return ht_home(key, t.mask); };
    __shared__ uint32_t q_j[kTPB / 64][kContCap], q_h[kTPB / 64][kContCap], q_k[kTPB / 64][kContCap];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t* const qj = q_j[wave];
    uint32_t* const qh = q_h[wave];
    uint32_t* const qk = q_k[wave];
    uint32_t nq = 0;  // queued rows (wave-uniform)
    const uint64_t lt = (1ull << lane) - 1;
    const uint64_t stride = (uint64_t)gridDim.x * kTPB * kProbeILP;
    uint64_t j0 = (uint64_t)blockIdx.x * kTPB * kProbeILP + threadIdx.x;
    // the next step's keys are loaded while this step's buckets are in flight;
    // indices are clamped (no branch) so nothing serialises the loads
    uint32_t knext[kProbeILP];
#pragma unroll
    for (int u = 0; u < kProbeILP; u++) {
        const uint64_t j = j0 + (uint64_t)u * kTPB;
        knext[u] = (uint32_t)pkeys[j < n2 ? j : n2 - 1];
    }
    // a queued row: cj, its key ck and ch, the slot it is at as steps from its home
    // slot (kBucket.. W-1); the slot itself is recomputed from the key
    auto cont_slot = [&](uint32_t ck, uint32_t ch) {
        const uint64_t hh = home(ck);
        return (hh & ~t.wmask) | ((hh + ch) & t.wmask);
    };
    // a continuation: row cj at step ch with key ck (lanes < ntake hold one)
    auto cont_resolve = [&](bool has, uint32_t cj, uint32_t ch, uint32_t ck, u64 c) {
        // c: the slot's word. Resolved on the key or an empty slot; otherwise requeued.
        bool again = false;
        if (has) {
            if (c == kEmpty || (uint32_t)c == ck || ch >= t.wmask) {  // (a full window: a miss)
                const bool hit = c != kEmpty && (uint32_t)c == ck;
                const uint32_t payload = hit ? (uint32_t)(c >> 32) : 0u;
                if (RUNS || hit) probe_emit<RUNS>(cj, hit, payload, pstart, rs, cnt, packed);
                if (!RUNS && hit) atomicOr(&hits[cj >> 6], 1ull << (cj & 63));  // word stored in an earlier step
                if (RUNS && wcnt && hit) atomicAdd(&wcnt[cj >> 6], run_len(payload, rs));  // likewise
            } else {
                again = true;
            }
        }
        const u64 am = __ballot(again);
        if (again) {
            const uint32_t at = nq + (uint32_t)__popcll(am & lt);
            qj[at] = cj;
            qh[at] = ch + 1;
            qk[at] = ck;
        }
        nq += (uint32_t)__popcll(am);
    };
    // the loop runs while the wave's first row is in range, so all 64 lanes take
    // every step together (the queue count is per wave)
    for (; j0 - (uint64_t)lane < n2; j0 += stride) {
        uint32_t key[kProbeILP];
        uint64_t h[kProbeILP];
        ulonglong2 b0[kProbeILP], b1[kProbeILP];  // the home bucket, slots 0-1 and 2-3
        // up to 64 queued rows from the back of the queue, their slots requested
        // with this step's buckets
        const uint32_t ntake = nq < 64 ? nq : 64;
        const bool has = (uint32_t)lane < ntake;
        uint32_t cj = 0, ch = 0, ck = 0;
        if (has) {
            const uint32_t e = nq - ntake + (uint32_t)lane;
            cj = qj[e];
            ch = qh[e];
            ck = qk[e];
        }
        nq -= ntake;
        u64 c = 0;
        if (has) c = words[cont_slot(ck, ch)];
#pragma unroll
        for (int u = 0; u < kProbeILP; u++) {
            key[u] = knext[u];
            h[u] = home(key[u]);
            const ulonglong2* q = reinterpret_cast<const ulonglong2*>(words + h[u]);
            b0[u] = q[0];
            b1[u] = q[1];
        }
#pragma unroll
        for (int u = 0; u < kProbeILP; u++) {
            const uint64_t j = j0 + stride + (uint64_t)u * kTPB;
            knext[u] = (uint32_t)pkeys[j < n2 ? j : n2 - 1];
        }
        cont_resolve(has, cj, ch, ck, c);
#pragma unroll
        for (int u = 0; u < kProbeILP; u++) {
            const uint64_t j = j0 + (uint64_t)u * kTPB;
            const u64 sl[4] = {b0[u].x, b0[u].y, b1[u].x, b1[u].y};
            bool hit = false, done = j >= n2;
            uint32_t payload = 0;
#pragma unroll
            for (uint32_t i = 0; i < kB; i++) {
                if (done) break;
                const u64 w = sl[i];
                if (w == kEmpty) done = true;
                else if ((uint32_t)w == key[u]) hit = done = true, payload = (uint32_t)(w >> 32);
            }
            // a full bucket without the key: on along the window, unless its mark
            // says no key homed here went on (j < n2 here)
            const bool defer = !done && !(marks && !bucket_ovf(sl[0], sl[1]));
            const u64 dm = __ballot(defer);
            if (defer) {
                const uint32_t at = nq + (uint32_t)__popcll(dm & lt);
                qj[at] = (uint32_t)j;
                qh[at] = kB;
                qk[at] = key[u];
            }
            nq += (uint32_t)__popcll(dm);
            if (j < n2 && !defer) probe_emit<RUNS>(j, hit, payload, pstart, rs, cnt, packed);
            if (RUNS && wcnt) {
                // packed runs: the word's run lengths, summed over the wave (a deferred
                // row adds its own when it resolves), so no pass re-reads the payloads
                uint32_t L = (j < n2 && !defer && hit) ? run_len(payload, rs) : 0u;
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) L += __shfl_xor(L, o, 64);
                if (j < n2 && lane == 0) wcnt[j >> 6] = L;
            }
            if constexpr (!RUNS) {
                // a wave's 64 lanes hold 64 consecutive rows: their hits are one word
                // (a deferred row's bit is set when it resolves)
                const u64 m = __ballot(hit);
                if (j < n2 && lane == 0) hits[j >> 6] = m;
            }
        }
        // keep room for a step's worst case (64 requeued + 64 x kProbeILP new):
        // drain in place when the queue runs long
        while (nq > kContCap - 64 - 64 * kProbeILP) {
            const uint32_t nt = nq < 64 ? nq : 64;
            const bool hs = (uint32_t)lane < nt;
            uint32_t dj = 0, dh = 0, dk = 0;
            u64 dc = 0;
            if (hs) {
                const uint32_t e = nq - nt + (uint32_t)lane;
                dj = qj[e], dh = qh[e], dk = qk[e];
                dc = words[cont_slot(dk, dh)];
            }
            nq -= nt;
            cont_resolve(hs, dj, dh, dk, dc);
        }
    }
    // the queue's rest
    while (nq) {
        const uint32_t nt = nq < 64 ? nq : 64;
        const bool hs = (uint32_t)lane < nt;
        uint32_t dj = 0, dh = 0, dk = 0;
        u64 dc = 0;
        if (hs) {
            const uint32_t e = nq - nt + (uint32_t)lane;
            dj = qj[e], dh = qh[e], dk = qk[e];
            dc = words[cont_slot(dk, dh)];
        }
        nq -= nt;
        cont_resolve(hs, dj, dh, dk, dc);
    }
}

// Unique path, after the probe: matches per 64-row hit word (scanned into the
// words' output offsets), then each matching row j writes its pair at its word's
// offset + the matches below it in the word. Output in ascending j, as J1.
__global__ __launch_bounds__(kTPB) void k_hits_count(const u64* __restrict__ hits, uint64_t nw,
                                                     uint32_t* __restrict__ cnt) {
    const uint64_t stride = (uint64_t)gridDim.x * kTPB;
    for (uint64_t w = (uint64_t)blockIdx.x * kTPB + threadIdx.x; w < nw; w += stride)
        cnt[w] = (uint32_t)__popcll(hits[w]);
}

__global__ __launch_bounds__(kTPB) void k_join_write_hits(const u64* __restrict__ hits,
                                                          const u64* __restrict__ woffs,
                                                          const uint32_t* __restrict__ pstart,
                                                          const int* __restrict__ p2, uint64_t n2,
                                                          int* __restrict__ out1, int* __restrict__ out2) {
    const uint64_t stride = (uint64_t)gridDim.x * kTPB;
    for (uint64_t j = (uint64_t)blockIdx.x * kTPB + threadIdx.x; j < n2; j += stride) {
        const u64 m = hits[j >> 6];
        const uint32_t b = (uint32_t)(j & 63);
        if (!((m >> b) & 1)) continue;
        const u64 o = woffs[j >> 6] + (u64)__popcll(m & ((1ull << b) - 1));
        out1[o] = (int)pstart[j];
        if (out2) out2[o] = (p2 ? p2[j] : 0);
    }
}

// The same with 4 rows a lane (round 5): payloads and probe positions read as 16-byte
// loads (p2 and pstart 16-byte aligned; else the 1-row kernel), a lane's hits are 4
// bits of its word, its output slot the word's offset plus the hits below them. The
// 1-row form moved its 3 GB at ~3 TB/s (one 4-byte load per thread and iteration).
__global__ __launch_bounds__(kTPB) void k_join_write_hits4(const u64* __restrict__ hits,
                                                           const u64* __restrict__ woffs,
                                                           const uint32_t* __restrict__ pstart,
                                                           const int* __restrict__ p2, uint64_t n2,
                                                           int* __restrict__ out1, int* __restrict__ out2) {
    const uint64_t stride = (uint64_t)gridDim.x * kTPB * 4;
    for (uint64_t j = ((uint64_t)blockIdx.x * kTPB + threadIdx.x) * 4; j < n2; j += stride) {
        const u64 m = hits[j >> 6];
        const uint32_t sh = (uint32_t)(j & 63);
        const uint32_t bits = (uint32_t)(m >> sh) & 0xFu;
        if (!bits) continue;
        u64 o = woffs[j >> 6] + (u64)__popcll(m & ((1ull << sh) - 1));
        uint4 pv;
        int4 qv = make_int4(0, 0, 0, 0);
        if (j + 3 < n2) {
            pv = *reinterpret_cast<const uint4*>(pstart + j);
            if (out2 && p2) qv = *reinterpret_cast<const int4*>(p2 + j);
        } else {
            pv.x = pstart[j];
            pv.y = j + 1 < n2 ? pstart[j + 1] : 0u;
            pv.z = j + 2 < n2 ? pstart[j + 2] : 0u;
            pv.w = 0u;
            if (out2 && p2) {
                qv.x = p2[j];
                qv.y = j + 1 < n2 ? p2[j + 1] : 0;
                qv.z = j + 2 < n2 ? p2[j + 2] : 0;
            }
        }
        const uint32_t pa[4] = {pv.x, pv.y, pv.z, pv.w};
        const int qa[4] = {qv.x, qv.y, qv.z, qv.w};
#pragma unroll
        for (int e = 0; e < 4; e++)
            if (bits & (1u << e)) {
                out1[o] = (int)pa[e];
                if (out2) out2[o] = qa[e];
                o++;
            }
    }
}

// Diagnostic: k_ht_probe_unique's memory pattern alone (mq_random_read). Read j
// goes to slot hash32(j) of a 2^k-slot table; 8 reads per lane in flight.
__global__ __launch_bounds__(kTPB) void k_random_read(const u64* __restrict__ t, uint64_t mask, uint64_t n,
                                                      u64* __restrict__ out) {
    u64 acc = 0;
    const uint64_t stride = (uint64_t)gridDim.x * kTPB * kProbeILP;
    for (uint64_t j0 = (uint64_t)blockIdx.x * kTPB * kProbeILP + threadIdx.x; j0 < n; j0 += stride) {
        u64 v[kProbeILP];
#pragma unroll
        for (int u = 0; u < kProbeILP; u++) {
            const uint64_t j = j0 + (uint64_t)u * kTPB;
            v[u] = j < n ? t[hash32((uint32_t)j ^ (uint32_t)(j >> 32)) & mask] : 0;
        }
#pragma unroll
        for (int u = 0; u < kProbeILP; u++) acc ^= v[u];
    }
    if (acc == 0x5EED5EED5EED5EEDull) out[0] = acc;  // keeps the loads; never true for a memset table
}

// sorted keys are (key ^ 0x80000000); a run head claims its slot and stores the start
__global__ __launch_bounds__(kTPB) void k_ht_insert_heads(const uint32_t* __restrict__ skeys,
                                                          uint64_t n, u64* words,
                                                          uint32_t* __restrict__ start,
                                                          uint64_t mask) {
    const uint64_t stride = (uint64_t)gridDim.x * kTPB;
    for (uint64_t i = (uint64_t)blockIdx.x * kTPB + threadIdx.x; i < n; i += stride) {
        const uint32_t k = skeys[i];
        if (i == 0 || skeys[i - 1] != k) {
            bool fresh;
            const uint64_t h = ht_claim(words, mask, (int)(k ^ 0x80000000u), &fresh);
            start[h] = (uint32_t)i;
        }
    }
}

__global__ __launch_bounds__(kTPB) void k_ht_set_len(const uint32_t* __restrict__ skeys, uint64_t n,
                                                     const u64* words,
                                                     const uint32_t* __restrict__ start,
                                                     uint32_t* __restrict__ len, uint64_t mask) {
    const uint64_t stride = (uint64_t)gridDim.x * kTPB;
    for (uint64_t i = (uint64_t)blockIdx.x * kTPB + threadIdx.x; i < n; i += stride) {
        const uint32_t k = skeys[i];
        if (i == n - 1 || skeys[i + 1] != k) {
            const uint64_t h = ht_find(words, mask, (int)(k ^ 0x80000000u));
            len[h] = (uint32_t)(i + 1 - start[h]);
        }
    }
}

__global__ __launch_bounds__(kTPB) void k_ht_probe(const int* __restrict__ pkeys, uint64_t n2,
                                                   const u64* words,
                                                   const uint32_t* __restrict__ start,
                                                   const uint32_t* __restrict__ len, uint64_t mask,
                                                   uint32_t* __restrict__ pstart,
                                                   uint32_t* __restrict__ plen) {
    const uint64_t stride = (uint64_t)gridDim.x * kTPB;
    for (uint64_t j = (uint64_t)blockIdx.x * kTPB + threadIdx.x; j < n2; j += stride) {
        const uint64_t h = ht_find(words, mask, pkeys[j]);
        const bool hit = h != ~0ull;
        pstart[j] = hit ? start[h] : 0u;
        plen[j] = hit ? len[h] : 0u;
    }
}

// Per-row runs (the sorted-runs and global-CAS builds). A run longer than kLongRun
// rows (a hot key) is not copied by its one lane: the lane lists it as chunks of
// kLongChunk pairs (entry = row << 32 | chunk) and k_join_write_long copies each chunk
// with a whole block, coalesced. (One lane writing a 2^26-row run alone took the wave
// 2^26 dependent iterations.)
constexpr uint32_t kLongRun = 4096;
constexpr uint32_t kLongChunk = 65536;

__global__ __launch_bounds__(kTPB) void k_join_write(const uint32_t* __restrict__ pstart,
                                                     const uint32_t* __restrict__ plen,
                                                     const u64* __restrict__ offs,
                                                     const int* __restrict__ p2,
                                                     const int* __restrict__ bpos, uint64_t n2,
                                                     int* __restrict__ out1, int* __restrict__ out2,
                                                     u64* __restrict__ longq, uint32_t* __restrict__ nlong) {
    const uint64_t stride = (uint64_t)gridDim.x * kTPB;
    for (uint64_t j = (uint64_t)blockIdx.x * kTPB + threadIdx.x; j < n2; j += stride) {
        const uint32_t L = plen[j];
        if (!L) continue;
        if (L > kLongRun) {
            const uint32_t nch = (L + kLongChunk - 1) / kLongChunk;
            const uint32_t at = atomicAdd(nlong, nch);
            for (uint32_t c = 0; c < nch; c++) longq[at + c] = (j << 32) | c;
            continue;
        }
        const u64 o = offs[j];
        const uint32_t s = pstart[j];
        const int pp = (p2 ? p2[j] : 0);
        for (uint32_t t = 0; t < L; t++) {
            out1[o + t] = bpos[s + t];
            if (out2) out2[o + t] = pp;
        }
    }
}

// The listed chunks of long runs, one block per chunk (grid-stride over the list,
// whose length k_join_write left in *nlong).
__global__ __launch_bounds__(kTPB) void k_join_write_long(const uint32_t* __restrict__ pstart,
                                                          const uint32_t* __restrict__ plen,
                                                          const u64* __restrict__ offs, const int* __restrict__ p2,
                                                          const int* __restrict__ bpos, const u64* __restrict__ longq,
                                                          const uint32_t* __restrict__ nlong, int* __restrict__ out1,
                                                          int* __restrict__ out2) {
    const uint32_t n = *nlong;
    for (uint32_t e = blockIdx.x; e < n; e += gridDim.x) {
        const u64 q = longq[e];
        const uint64_t j = q >> 32;
        const uint32_t c = (uint32_t)q;
        const uint32_t L = plen[j];
        const uint32_t a = c * kLongChunk, b = L - a < kLongChunk ? L : a + kLongChunk;
        const u64 o = offs[j];
        const uint32_t s = pstart[j];
        const int pp = (p2 ? p2[j] : 0);
        for (uint32_t t = a + threadIdx.x; t < b; t += kTPB) {
            out1[o + t] = bpos[s + t];
            if (out2) out2[o + t] = pp;
        }
    }
}

// Packed runs (n1 <= 2^28): the probe stores each row's table payload as it is (0 for
// a miss; a hit's payload is never 0: start << 4 | length with length >= 1, or
// r << 4 | 15 for a long run, whose bounds are rs[r], rs[r + 1]). Then per 64-row word
// the sum of the rows' run lengths, a scan over those n2/64 sums, and the write: each
// wave takes one word, its lanes the word's 64 consecutive rows, and a row's output
// offset is the word's offset plus the lengths of the rows below it (a wave prefix).
// (Was: per row a start and a length from the probe and a scan of n2 lengths into
// 8-byte offsets, 16 B more per probe row written and read again, plus the n2 scan.)
__device__ __forceinline__ void run_decode(uint32_t pk, const uint32_t* __restrict__ rs, uint32_t* a, uint32_t* L) {
    uint32_t l = pk & 15u, s = pk >> 4;
    if (l == 15u) {
        l = rs[s + 1] - rs[s];
        s = rs[s];
    }
    *a = pk ? s : 0u;
    *L = pk ? l : 0u;
}

// The packed-runs write (a wave's 64 rows = one word; a row's offset = the word's + a
// wave prefix of the lengths), with more reads in flight: a wave takes kWriteWords words
// at a time (2^28 many-to-many, alternating on one box: 1 word 4.30, 4 words 4.00 ms; on
// another 1 / 4 / 8 words 3.63-4.24 / 3.65-4.03 / 3.58-3.94 ms), and every row's first
// two run positions (all of config 5's runs) are requested for
// all of them before any pair is stored; longer runs finish in a loop. The run reads
// are random (one line of the key-sorted positions per hit row), so the kernel is
// bound by how many of them are outstanding.
template <int kWriteWords>
__global__ __launch_bounds__(kTPB) void k_join_write_runs_mlp(const uint32_t* __restrict__ pk, uint64_t n2,
                                                              const uint32_t* __restrict__ rs,
                                                              const u64* __restrict__ woffs,
                                                              const int* __restrict__ p2,
                                                              const int* __restrict__ bpos, int* __restrict__ out1,
                                                              int* __restrict__ out2) {
    const int lane = threadIdx.x & 63;
    const uint64_t nw = (n2 + 63) / 64;
    const uint64_t wstride = (uint64_t)gridDim.x * (kTPB / 64) * kWriteWords;
    for (uint64_t w0 = ((uint64_t)blockIdx.x * (kTPB / 64) + (threadIdx.x >> 6)) * kWriteWords; w0 < nw;
         w0 += wstride) {
        uint32_t pv[kWriteWords], a[kWriteWords], L[kWriteWords];
        u64 o[kWriteWords];
        int pp[kWriteWords], b0[kWriteWords], b1[kWriteWords];
#pragma unroll
        for (int u = 0; u < kWriteWords; u++) {
            const uint64_t j = (w0 + u) * 64 + (uint64_t)lane;
            pv[u] = j < n2 ? pk[j] : 0u;
            pp[u] = j < n2 ? (p2 ? p2[j] : 0) : 0;
        }
#pragma unroll
        for (int u = 0; u < kWriteWords; u++) {
            run_decode(pv[u], rs, &a[u], &L[u]);
            uint32_t incl = L[u];
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t y = __shfl_up(incl, d, 64);
                if (lane >= d) incl += y;
            }
            o[u] = (w0 + u < nw ? woffs[w0 + u] : 0ull) + (u64)(incl - L[u]);
        }
#pragma unroll
        for (int u = 0; u < kWriteWords; u++) {
            b0[u] = L[u] ? bpos[a[u]] : 0;
            b1[u] = L[u] > 1u ? bpos[a[u] + 1] : 0;
        }
#pragma unroll
        for (int u = 0; u < kWriteWords; u++) {
            if (!L[u]) continue;
            out1[o[u]] = b0[u];
            if (out2) out2[o[u]] = pp[u];
            if (L[u] > 1u) {
                out1[o[u] + 1] = b1[u];
                if (out2) out2[o[u] + 1] = pp[u];
            }
            for (uint32_t t = 2; t < L[u]; t++) {
                out1[o[u] + t] = bpos[a[u] + t];
                if (out2) out2[o[u] + t] = pp[u];
            }
        }
    }
}

// The write after a run2 probe (the partitioned runs probe, k_win_probe_tab<u64>): a run
// of one or two rows comes from the probe's per-row positions (p01, a stream), a longer
// one (3..14 rows) from the run array as before.
template <int kWriteWords>
__global__ __launch_bounds__(kTPB) void k_join_write_runs16(const uint32_t* __restrict__ pk, uint64_t n2,
                                                            const u64* __restrict__ woffs, const int* __restrict__ p2,
                                                            const u64* __restrict__ p01, const int* __restrict__ bpos,
                                                            int* __restrict__ out1, int* __restrict__ out2) {
    const int lane = threadIdx.x & 63;
    const uint64_t nw = (n2 + 63) / 64;
    const uint64_t wstride = (uint64_t)gridDim.x * (kTPB / 64) * kWriteWords;
    for (uint64_t w0 = ((uint64_t)blockIdx.x * (kTPB / 64) + (threadIdx.x >> 6)) * kWriteWords; w0 < nw;
         w0 += wstride) {
        uint32_t L[kWriteWords], a[kWriteWords];
        u64 o[kWriteWords], pq[kWriteWords];
        int pp[kWriteWords];
#pragma unroll
        for (int u = 0; u < kWriteWords; u++) {
            const uint64_t j = (w0 + u) * 64 + (uint64_t)lane;
            const uint32_t m = j < n2 ? pk[j] : 0u;
            pq[u] = j < n2 ? p01[j] : 0ull;
            pp[u] = j < n2 ? (p2 ? p2[j] : 0) : 0;
            L[u] = m & 15u;
            a[u] = m >> 4;
        }
#pragma unroll
        for (int u = 0; u < kWriteWords; u++) {
            uint32_t incl = L[u];
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t y = __shfl_up(incl, d, 64);
                if (lane >= d) incl += y;
            }
            o[u] = (w0 + u < nw ? woffs[w0 + u] : 0ull) + (u64)(incl - L[u]);
        }
#pragma unroll
        for (int u = 0; u < kWriteWords; u++) {
            if (!L[u]) continue;
            if (L[u] <= 2u) {
                out1[o[u]] = (int)(uint32_t)pq[u];
                if (out2) out2[o[u]] = pp[u];
                if (L[u] == 2u) {
                    out1[o[u] + 1] = (int)(uint32_t)(pq[u] >> 32);
                    if (out2) out2[o[u] + 1] = pp[u];
                }
            } else {
                for (uint32_t t = 0; t < L[u]; t++) {
                    out1[o[u] + t] = bpos[a[u] + t];
                    if (out2) out2[o[u] + t] = pp[u];
                }
            }
        }
    }
}

// ---- duplicate keys as runs (the build sorted by key, stable: a key's rows are one
// run in insertion order); the distinct keys go into the windowed unique table with
// their run index as payload ----
// Runs of the key-sorted build in two passes over the keys: k_run_count counts the
// run heads (a row whose key differs from the row before) per 4096-row tile, an
// exclusive scan of those counts gives each tile its first run, and k_run_emit
// ranks the heads inside the tile (each thread 16 consecutive rows, a block scan of
// the per-thread counts) and writes run r's key dk[r] (unflipped) and first sorted
// row rs[r]; rs[R] = n. k_run_payload then gives every run its payload rid[r]. (Was: a head flag per row, a scan of
// 2^28 flags into 8-byte ranks and a compaction: ≈ 10 GB of traffic, 2.2 ms.)
constexpr int kRunPer = 16;
constexpr uint64_t kRunTile = (uint64_t)kTPB * kRunPer;  // 4096

__device__ __forceinline__ uint32_t run_heads16(const uint32_t* __restrict__ skeys, uint64_t n, uint64_t i0,
                                                uint32_t (&k)[kRunPer]) {
    // bit m set <=> row i0 + m (< n) starts a run; k[] = the 16 keys
    uint32_t prev = i0 ? skeys[i0 - 1] : 0u, bits = 0;
    if (i0 + kRunPer <= n) {
        const uint4* q = reinterpret_cast<const uint4*>(skeys + i0);
#pragma unroll
        for (int v = 0; v < kRunPer / 4; v++) {
            const uint4 x = q[v];
            k[4 * v] = x.x, k[4 * v + 1] = x.y, k[4 * v + 2] = x.z, k[4 * v + 3] = x.w;
        }
    } else {
#pragma unroll
        for (int m = 0; m < kRunPer; m++) k[m] = i0 + m < n ? skeys[i0 + m] : 0u;
    }
#pragma unroll
    for (int m = 0; m < kRunPer; m++) {
        if (i0 + m < n && (i0 + m == 0 || k[m] != prev)) bits |= 1u << m;
        prev = k[m];
    }
    return bits;
}

__global__ __launch_bounds__(kTPB) void k_run_count(const uint32_t* __restrict__ skeys, uint64_t n,
                                                    uint32_t* __restrict__ tcount) {
    __shared__ uint32_t s_w[kTPB / 64];
    const uint64_t i0 = (uint64_t)blockIdx.x * kRunTile + (uint64_t)threadIdx.x * kRunPer;
    uint32_t k[kRunPer];
    uint32_t c = i0 < n ? (uint32_t)__popc(run_heads16(skeys, n, i0, k)) : 0u;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (int w = 0; w < kTPB / 64; w++) t += s_w[w];
        tcount[blockIdx.x] = t;
    }
}

// (the heads go through LDS: written straight from the ranks, a wave's stores
// scattered over ~2 KB, the emit took 1.03 ms at 2^28)
__global__ __launch_bounds__(kTPB) void k_run_emit(const uint32_t* __restrict__ skeys, uint64_t n,
                                                   const u64* __restrict__ toff, int* __restrict__ dk,
                                                   uint32_t* __restrict__ rs) {
    __shared__ uint32_t s_w[kTPB / 64];
    __shared__ uint32_t s_dk[kRunTile], s_rs[kRunTile];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t i0 = (uint64_t)blockIdx.x * kRunTile + (uint64_t)threadIdx.x * kRunPer;
    uint32_t k[kRunPer];
    const uint32_t bits = i0 < n ? run_heads16(skeys, n, i0, k) : 0u;
    const uint32_t c = (uint32_t)__popc(bits);
    uint32_t incl = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    if (lane == 63) s_w[wave] = incl;
    __syncthreads();
    uint32_t at = incl - c, tot = 0;
    for (int w = 0; w < kTPB / 64; w++) {
        if (w < wave) at += s_w[w];
        tot += s_w[w];
    }
#pragma unroll
    for (int m = 0; m < kRunPer; m++) {
        if (bits & (1u << m)) {
            s_dk[at] = k[m] ^ 0x80000000u;
            s_rs[at] = (uint32_t)(i0 + m);
            at++;
        }
    }
    __syncthreads();
    const u64 r0 = toff[blockIdx.x];
    for (uint32_t x = threadIdx.x; x < tot; x += kTPB) {
        dk[r0 + x] = (int)s_dk[x];
        rs[r0 + x] = s_rs[x];
    }
    if (i0 < n && n - i0 <= (uint64_t)kRunPer) rs[r0 + tot] = (uint32_t)n;  // the block holding row n-1
}

// The table payload of run r: (start << 4) | length for runs shorter than 15 rows
// (one probe then yields both), (r << 4) | 15 otherwise (the probe reads rs). Packed
// only while starts and run indexes fit 28 bits (n <= 2^28), else always via rs.
__global__ __launch_bounds__(kTPB) void k_run_payload(const uint32_t* __restrict__ rs, uint64_t R, bool packed,
                                                      int* __restrict__ rid) {
    const uint64_t stride = (uint64_t)gridDim.x * kTPB;
    for (uint64_t r = (uint64_t)blockIdx.x * kTPB + threadIdx.x; r < R; r += stride) {
        const uint32_t a = rs[r], L = rs[r + 1] - a;
        rid[r] = (int)(!packed ? (uint32_t)r : L < 15u ? (a << 4) | L : ((uint32_t)r << 4) | 15u);
    }
}

// Per probe row, the number of pairs the last probe found for it (mq_join_counts),
// from whichever per-row state the probe left: the unique table's hit words (0/1), a
// packed payload per row (its length, < 15 on the per-word path), or a length per row.
__global__ __launch_bounds__(kTPB) void k_join_counts(const u64* __restrict__ hits, const uint32_t* __restrict__ pk,
                                                      const uint32_t* __restrict__ plen, uint64_t n2,
                                                      uint32_t* __restrict__ cnt) {
    const uint64_t stride = (uint64_t)gridDim.x * kTPB;
    for (uint64_t j = (uint64_t)blockIdx.x * kTPB + threadIdx.x; j < n2; j += stride) {
        uint32_t c;
        if (hits) c = (uint32_t)(hits[j >> 6] >> (j & 63)) & 1u;
        else if (pk) c = pk[j] & 15u;
        else c = plen[j];
        cnt[j] = c;
    }
}

}  // namespace

namespace mqi {
uint64_t scan_u32_scratch_elems(uint64_t n) { return scan_scratch_elems(n); }
int scan_u32_exclusive(const uint32_t* in, unsigned long long* out, uint64_t n,
                       unsigned long long* scratch, hipStream_t st) {
    return scan_exclusive<uint32_t>(in, out, n, scratch, st);
}
int scan_u32_exclusive_u32(const uint32_t* in, uint32_t* out, uint64_t n, unsigned long long* scratch,
                           hipStream_t st) {
    return scan_exclusive<uint32_t, uint32_t>(in, out, n, scratch, st);
}
int scan_u64_exclusive(const unsigned long long* in, unsigned long long* out, uint64_t n,
                       unsigned long long* scratch, hipStream_t st) {
    return scan_exclusive<u64>(in, out, n, scratch, st);
}
}  // namespace mqi

// ===========================================================================
// handle
// ===========================================================================
struct mq_join {
    int device;
    int unique;            // 1: windowed {key, payload} table (words only); 0: words/start/len;
                           // 2: windowed table of distinct keys -> run index, runs in rs
    const uint32_t* rs;    // unique == 2: first sorted row of each run, + n1
    bool marks;            // the unique table's full buckets carry overflow marks (k_win_build)
    bool packed;           // unique == 2: payloads carry start << 4 | length (k_run_payload)
    uint64_t n1, mask;
    Win win;               // unique table geometry
    u64* words;
    uint32_t* start;
    uint32_t* len;
    const int* bpos;       // build positions in run order (p1 itself, or sorted copy)
    void* owned[16];       // device allocations owned by the handle
    int nowned;
    bool pruns;            // the last probe took the per-64-row-word form (packed runs of < 15 rows)
    // probe state
    uint64_t n2, m;
    u64* p01;              // run2: per probe row, a short run's build positions
    uint32_t* pstart;
    uint32_t* plen;
    u64* offs;
    u64* scan_scratch;
    u64* longq;            // per-row write: chunks of the long runs (k_join_write_long)
    hipStream_t stream;    // the stream of the handle's last queued work (juse)
    // partitioned unique build (round 5): no global table; the build's words partitioned
    // by window (pwords) and each window's first word (pwstart, nwin + 1 entries); the
    // probe partitions its keys the same way (passes LSD passes) and joins window by
    // window in LDS (probe_partitioned). words == nullptr until a probe asks for the table.
    bool part;
    const int32_t* c1;     // the build inputs (valid until mq_join_free): a partitioned build
    const int32_t* p1;     // that meets a duplicate key or an overfull window is rebuilt
    uint32_t* pflag;       // the window join's flag (a duplicate met, a window overfull)
    bool narrow;           // the window join's results as u32 payloads, `sentinel` = a miss
    bool run2;             // the last probe left short runs' positions in p01 (k_join_write_runs16)
    // deferred (round 6): the partitioned probe stopped before its last inverse pass, which
    // mq_join_write runs fused with the pair write (dmode: 0 unique u32 results, 1 unique
    // u64, 2 run2 records); dperm = pass 0's places of the probe rows (pool, owned),
    // dhs0 = pass 0's tile offsets, dres = the results in pass-0 order (pool, owned)
    bool deferred;
    int dmode;
    uint16_t* dperm;
    u64* dhs0;
    void* dres;
    bool dupw;             // a partitioned build whose probe answers duplicate keys window by
                           // window (k_win_join_runs: run2 records, long runs into bpos)
    unsigned long long* mtot;  // the window joins' pair count (device)
    bool rsent_ok;         // windowed runs: `sentinel` is outside the payloads (the partitioned
                           // runs probe then carries short runs' positions, run2)
    uint32_t sentinel;     // (a value outside the build payloads' range)
    u64* pwords;
    uint32_t* pwstart;
    uint32_t nwin;
    int passes;
    uint64_t slots;
};

namespace {

int jown(mq_join* j, void* p) {
    if (j->nowned >= (int)(sizeof(j->owned) / sizeof(j->owned[0]))) {
        pool_free_on(p, j->stream);  // (stream-ordered: queued work may still write it)
        return set_err(MQ_EINVAL, "join: handle owns too many allocations");
    }
    j->owned[j->nowned++] = p;
    return MQ_OK;
}

int jalloc(mq_join* j, void** p, size_t bytes) {
    *p = pool_alloc(bytes);
    if (!*p) return set_err(MQ_ENOMEM, "join: device allocation of %zu bytes failed", bytes);
    const int rc = jown(j, *p);
    if (rc) *p = nullptr;
    return rc;
}

// Every call queues its work on the stream it is given; one on a different stream than
// the last first waits for that stream, so the handle's queued work is always ordered
// on j->stream and the stream-ordered frees below (pool_free_on) cover all of it: no
// host sync, and shard workers sharing a device do not wait for each other.
int juse(mq_join* j, hipStream_t st) {
    if (j->stream != st) HIPCHK(hipStreamSynchronize(j->stream));
    j->stream = st;
    return MQ_OK;
}

void jfree_all(mq_join* j) {
    for (int i = 0; i < j->nowned; i++) pool_free_on(j->owned[i], j->stream);
    j->nowned = 0;
}

// Give one owned allocation back (stream-ordered).
void jdrop(mq_join* j, void* p) {
    for (int i = 0; i < j->nowned; i++)
        if (j->owned[i] == p) {
            j->owned[i] = j->owned[--j->nowned];
            pool_free_on(p, j->stream);
            return;
        }
}

// The partitioned probe from this many build rows (MQ_JOIN_PART_MIN; MQ_JOIN_PART=0: off).
uint64_t part_min_rows() {
    const char* e = getenv("MQ_JOIN_PART");
    if (e && e[0] == '0') return ~0ull;
    const char* m = getenv("MQ_JOIN_PART_MIN");
    return m ? strtoull(m, nullptr, 10) : (1ull << 20);
}

// Unique-path build.
//  * below kWindowBuildRows: one global CAS per build row (the table is small);
//  * above: stable LSD radix partition of the (key, payload) words by window id,
//    then one block per window builds it in LDS and stores it whole (no global
//    atomics; every window is written, so the table needs no memset).
// (A partition by table window feeding the global-CAS insert measured 20.3 vs
// 21.0 ms at 2^28 rows plus the partition pass: device-scope CAS costs the same
// wherever the line lives, so the atomics themselves have to go.)
constexpr uint64_t kWindowBuildRows = 1ull << 16;

// Duplicate keys in a strided sample of the build side (a CAS set of the sampled
// keys): when the sample already has one, the build has many and goes straight to
// the runs build instead of attempting (and abandoning) the unique table.
__global__ __launch_bounds__(kTPB) void k_sample_dups(const int* __restrict__ keys, uint64_t stride, uint32_t ns,
                                                      u64* tab, uint32_t tmask, uint32_t* __restrict__ flag) {
    for (uint32_t i = blockIdx.x * kTPB + threadIdx.x; i < ns; i += gridDim.x * kTPB) {
        const uint32_t key = (uint32_t)keys[(uint64_t)i * stride];
        const u64 w = (u64)key | (1ull << 32);
        uint32_t h = hash32(key) & tmask;
        for (uint32_t step = 0; step <= tmask; step++) {
            const u64 old = atomicCAS(&tab[h], 0ull, w);
            if (old == 0) break;
            if (old == w) {
                *flag = 1;
                break;
            }
            h = (h + 1) & tmask;
        }
    }
}

// 1 when a sample of the build keys holds a duplicate (builds of 2^20 rows and up;
// MQ_JOIN_SAMPLE=0 turns the check off)
int sample_has_dups(const int* c1, uint64_t n, uint32_t* dflag, hipStream_t st, const DevState* s, bool* dups) {
    *dups = false;
    const char* e = getenv("MQ_JOIN_SAMPLE");
    if (n < (1ull << 20) || (e && e[0] == '0')) return MQ_OK;
    constexpr uint32_t kSample = 1u << 18;
    u64* tab = (u64*)pool_alloc((size_t)2 * kSample * 8);
    if (!tab) return set_err(MQ_ENOMEM, "join: sample set");
    HIPCHK(hipMemsetAsync(tab, 0, (size_t)2 * kSample * 8, st));
    HIPCHK(hipMemsetAsync(dflag + 1, 0, 4, st));
    hipLaunchKernelGGL(k_sample_dups, dim3(stream_grid(s, kSample)), dim3(kTPB), 0, st, c1, n / kSample, kSample, tab,
                       2 * kSample - 1, dflag + 1);
    if (hipGetLastError() != hipSuccess) {
        pool_free_on(tab, st);
        return set_err(MQ_EHIP, "join: sample launch");
    }
    uint32_t f = 0;
    HIPCHK(hipMemcpyAsync(&f, dflag + 1, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    pool_free_on(tab, st);
    *dups = f != 0;
    return MQ_OK;
}

int insert_unique(mq_join* j, const int* c1, const int* p1, uint64_t n, uint64_t slots,
                  uint32_t* general, hipStream_t st, const DevState* s, bool keep = false, int* pmm = nullptr) {
    const Win t = j->win;
    j->marks = n >= kWindowBuildRows;
    if (n < kWindowBuildRows) {
        HIPCHK(hipMemsetAsync(j->words, 0xFF, slots * 8, st));
        hipLaunchKernelGGL(k_ht_insert_unique, dim3(stream_grid(s, n)), dim3(kTPB), 0, st, c1, p1,
                           n, j->words, t, general);
        LAUNCHCHK("k_ht_insert_unique");
        return MQ_OK;
    }
    int lg = 0;
    while ((1ull << lg) < slots) lg++;
    const int wid_bits = lg - t.wlog;
    const int passes = (wid_bits + 7) / 8;
    const uint32_t nw = (uint32_t)(slots >> t.wlog);
    const uint64_t ntiles = ceil_div(n, (uint64_t)kBTPB * kSortItems);
    const uint64_t nh = ntiles * kRadix;
    u64 *a = nullptr, *b = nullptr, *hscan = nullptr, *scratch = nullptr;
    uint32_t *hist = nullptr, *wstart = nullptr;
    auto done = [&](int rc) {
        pool_free_on(a, st);
        pool_free_on(b, st);
        pool_free_on(hist, st);
        pool_free_on(hscan, st);
        pool_free_on(scratch, st);
        pool_free_on(wstart, st);
        return rc;
    };
    a = (u64*)pool_alloc(n * 8);
    b = passes > 1 ? (u64*)pool_alloc(n * 8) : nullptr;
    hist = (uint32_t*)pool_alloc(nh * 4);
    hscan = (u64*)pool_alloc(nh * 8);
    scratch = (u64*)pool_alloc(scan_scratch_elems(nh) * 8);
    wstart = (uint32_t*)pool_alloc(((uint64_t)nw + 1) * 4);
    if (!a || (passes > 1 && !b) || !hist || !hscan || !scratch || !wstart)
        return done(set_err(MQ_ENOMEM, "join: window build buffers (%llu rows)", (unsigned long long)n));
    u64* src = nullptr;
    u64* dst = a;
    for (int pass = 0; pass < passes; pass++) {
        const int shift = 8 * pass;
        // (round 6 measured digit bytes for the next pass's histogram, as the index sort
        // writes them: the byte stores cost the scatter 0.2-0.4 ms at 2^28 against the
        // histogram's 0.32 ms saved; not kept)
        if (pass == 0) {
            hipLaunchKernelGGL(k_win_hist<true>, dim3((uint32_t)ntiles), dim3(kBTPB), 0, st, c1,
                               (const u64*)nullptr, n, t, shift, hist, (uint32_t)ntiles);
        } else {
            hipLaunchKernelGGL(k_win_hist<false>, dim3((uint32_t)ntiles), dim3(kBTPB), 0, st,
                               (const int*)nullptr, src, n, t, shift, hist, (uint32_t)ntiles);
        }
        int rc = scan_exclusive<uint32_t>(hist, hscan, nh, scratch, st);
        if (rc) return done(rc);
        if (pass == 0) {
            hipLaunchKernelGGL(k_win_scatter<true>, dim3((uint32_t)ntiles), dim3(kBTPB), 0, st, c1, p1,
                               (const u64*)nullptr, n, t, shift, hscan, (uint32_t)ntiles, dst, keep ? pmm : nullptr);
        } else {
            hipLaunchKernelGGL(k_win_scatter<false>, dim3((uint32_t)ntiles), dim3(kBTPB), 0, st,
                               (const int*)nullptr, (const int*)nullptr, src, n, t, shift, hscan,
                               (uint32_t)ntiles, dst, (int*)nullptr);
        }
        if (hipGetLastError() != hipSuccess) return done(set_err(MQ_EHIP, "join: window partition"));
        src = dst;
        dst = (dst == a) ? b : a;
    }
    hipLaunchKernelGGL(k_win_bounds<u64>, dim3(nw / kTPB + 1), dim3(kTPB), 0, st, src, n, t, nw, wstart);
    if (keep) {  // the partitioned build: the words and window bounds kept (checked by the probe)
        int rc = jown(j, src);
        if (rc) {  // (jown freed src, stream-ordered: not again here)
            if (src == a) a = nullptr; else b = nullptr;
            return done(rc);
        }
        if ((rc = jown(j, wstart))) {
            if (src == a) a = nullptr; else b = nullptr;
            wstart = nullptr;
            return done(rc);
        }
        j->pwords = src;
        j->pwstart = wstart;
        j->nwin = nw;
        j->passes = passes;
        if (src == a) a = nullptr; else b = nullptr;
        wstart = nullptr;
        return done(MQ_OK);
    }
    hipLaunchKernelGGL(k_win_build<true>, dim3(nw), dim3(kWinTPB), 0, st, src, wstart, j->words, t, general);
    if (hipGetLastError() != hipSuccess) return done(set_err(MQ_EHIP, "join: window build"));
    // the temporaries are released only after the build has run
    if (hipStreamSynchronize(st) != hipSuccess) return done(set_err(MQ_EHIP, "join: build sync"));
    return done(MQ_OK);
}

// Duplicate keys, windowed (k_win_build_runs): the build rows partitioned by window
// (the unique build's passes), then each window's runs found in LDS. Returns 0
// (j->unique = 2, packed payloads, j->bpos the runs), 1 when it does not apply or a
// window flagged (the caller takes the sorted-runs build), or an error.
int build_window_runs(mq_join* j, const int* c1, const int* p1, uint64_t n, uint64_t slots, uint32_t* general,
                      hipStream_t st, const DevState* s, int* pmm = nullptr) {
    (void)s;
    const char* e = getenv("MQ_JOIN_WINRUNS");  // "0": the sorted-runs build (A/B, tests)
    const char* r = getenv("MQ_JOIN_RUNS");     // "0": the global-CAS run table (tests)
    if ((e && e[0] == '0') || (r && r[0] == '0') || n < kWindowBuildRows || n > (1ull << 28) || j->win.wlog != kWinLog) return 1;
    const Win t = j->win;
    const uint64_t nslot = slots;
    int lg = 0;
    while ((1ull << lg) < nslot) lg++;
    const int passes = (lg - t.wlog + 7) / 8;
    const uint32_t nw = (uint32_t)(nslot >> t.wlog);
    const uint64_t ntiles = ceil_div(n, (uint64_t)kBTPB * kSortItems);
    const uint64_t nh = ntiles * kRadix;
    u64 *a = nullptr, *b = nullptr, *hscan = nullptr, *scratch = nullptr;
    uint32_t *hist = nullptr, *wstart = nullptr;
    auto done = [&](int rc) {
        pool_free_on(a, st);
        pool_free_on(b, st);
        pool_free_on(hist, st);
        pool_free_on(hscan, st);
        pool_free_on(scratch, st);
        pool_free_on(wstart, st);
        return rc;
    };
    a = (u64*)pool_alloc(n * 8);
    b = passes > 1 ? (u64*)pool_alloc(n * 8) : nullptr;
    hist = (uint32_t*)pool_alloc(nh * 4);
    hscan = (u64*)pool_alloc(nh * 8);
    scratch = (u64*)pool_alloc(scan_scratch_elems(nh) * 8);
    wstart = (uint32_t*)pool_alloc(((uint64_t)nw + 1) * 4);
    if (!a || (passes > 1 && !b) || !hist || !hscan || !scratch || !wstart)
        return done(set_err(MQ_ENOMEM, "join: window runs buffers (%llu rows)", (unsigned long long)n));
    // bp joins the handle only when the build takes this path
    int* bp = (int*)pool_alloc(n * 4);
    auto drop = [&](int rc) {
        pool_free_on(bp, st);  // (stream-ordered: launched work may still use it)
        return done(rc);
    };
    int rc = MQ_OK;
    if (!bp) return drop(set_err(MQ_ENOMEM, "join: window runs outputs (%llu rows)", (unsigned long long)n));
    u64* src = nullptr;
    u64* dst = a;
    for (int pass = 0; pass < passes; pass++) {
        const int shift = 8 * pass;
        if (pass == 0)
            hipLaunchKernelGGL(k_win_hist<true>, dim3((uint32_t)ntiles), dim3(kBTPB), 0, st, c1, (const u64*)nullptr, n,
                               t, shift, hist, (uint32_t)ntiles);
        else
            hipLaunchKernelGGL(k_win_hist<false>, dim3((uint32_t)ntiles), dim3(kBTPB), 0, st, (const int*)nullptr, src,
                               n, t, shift, hist, (uint32_t)ntiles);
        if ((rc = scan_exclusive<uint32_t>(hist, hscan, nh, scratch, st))) return drop(rc);
        if (pass == 0)
            hipLaunchKernelGGL(k_win_scatter<true>, dim3((uint32_t)ntiles), dim3(kBTPB), 0, st, c1, p1,
                               (const u64*)nullptr, n, t, shift, hscan, (uint32_t)ntiles, dst, pmm);
        else
            hipLaunchKernelGGL(k_win_scatter<false>, dim3((uint32_t)ntiles), dim3(kBTPB), 0, st, (const int*)nullptr,
                               (const int*)nullptr, src, n, t, shift, hscan, (uint32_t)ntiles, dst, (int*)nullptr);
        if (hipGetLastError() != hipSuccess) return drop(set_err(MQ_EHIP, "join: window partition"));
        src = dst;
        dst = (dst == a) ? b : a;
    }
    uint32_t flag = 0;
    if (hipMemsetAsync(general, 0, 4, st) != hipSuccess) return drop(set_err(MQ_EHIP, "join: memset"));
    hipLaunchKernelGGL(k_win_bounds<u64>, dim3(nw / kTPB + 1), dim3(kTPB), 0, st, src, n, t, nw, wstart);
    hipLaunchKernelGGL(k_win_build_runs, dim3(nw), dim3(kWinTPB), 0, st, src, wstart, j->words, bp, t, general);
    if (hipGetLastError() != hipSuccess) return drop(set_err(MQ_EHIP, "join: window runs build"));
    int sl[128];
    if (hipMemcpyAsync(&flag, general, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
        (pmm && hipMemcpyAsync(sl, pmm, sizeof sl, hipMemcpyDeviceToHost, st) != hipSuccess) ||
        hipStreamSynchronize(st) != hipSuccess)
        return drop(set_err(MQ_EHIP, "join: window runs sync"));
    if (flag) return drop(1);
    if (pmm) {  // a value outside the payloads' range: the partitioned probe's marker (rsent)
        int mn = INT32_MAX, mx = INT32_MIN;
        for (int q = 0; q < 64; q++) {
            mn = sl[q] < mn ? sl[q] : mn;
            mx = sl[64 + q] > mx ? sl[64 + q] : mx;
        }
        const char* nw = getenv("MQ_JOIN_NARROW");
        j->rsent_ok = !(nw && nw[0] == '0') && (mx < INT32_MAX || mn > INT32_MIN);
        j->sentinel = (uint32_t)(mx < INT32_MAX ? INT32_MAX : INT32_MIN);
    }
    int* const bpos = bp;
    bp = nullptr;  // (jown frees it itself when it fails)
    if ((rc = jown(j, bpos))) return drop(rc);
    j->unique = 2;
    j->packed = true;
    j->rs = nullptr;  // packed lengths stay below 15: no run is looked up
    j->bpos = bpos;
    j->marks = true;
    return done(0);
}

// Duplicate keys: runs of the sorted build, their distinct keys into the windowed
// unique table (payload: run index). Returns 0 (j->unique = 2), 1 when the windowed
// build flagged (the caller takes the global-CAS run table), or an error.
int build_runs(mq_join* j, const uint32_t* skeys, uint64_t n, uint64_t slots, uint32_t* dflag, hipStream_t st,
               const DevState* s) {
    const char* e = getenv("MQ_JOIN_RUNS");  // "0": the global-CAS run table (A/B, tests)
    if (e && e[0] == '0') return 1;
    const uint64_t ntiles = ceil_div(n, kRunTile);
    uint32_t* tcount = (uint32_t*)pool_alloc(ntiles * 4);
    u64* toff = (u64*)pool_alloc(ntiles * 8);
    u64* scratch = (u64*)pool_alloc(scan_scratch_elems(ntiles) * 8);
    auto fail = [&](int rc) {
        pool_free_on(tcount, st);
        pool_free_on(toff, st);
        pool_free_on(scratch, st);
        return rc;
    };
    if (!tcount || !toff || !scratch) return fail(set_err(MQ_ENOMEM, "join: run buffers"));
    hipLaunchKernelGGL(k_run_count, dim3((uint32_t)ntiles), dim3(kTPB), 0, st, skeys, n, tcount);
    int rc = scan_exclusive<uint32_t>(tcount, toff, ntiles, scratch, st);
    if (rc) return fail(rc);
    u64 last = 0;
    uint32_t lastc = 0;
    HIPCHK(hipMemcpyAsync(&last, toff + (ntiles - 1), 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(&lastc, tcount + (ntiles - 1), 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    const uint64_t R = last + lastc;
    int* dk = (int*)pool_alloc(R * 4);
    int* rid = (int*)pool_alloc(R * 4);
    uint32_t* rs = nullptr;
    if (!dk || !rid || (rc = jalloc(j, (void**)&rs, (R + 1) * 4))) {
        pool_free_on(dk, st);
        pool_free_on(rid, st);
        return fail(rc ? rc : set_err(MQ_ENOMEM, "join: run keys"));
    }
    hipLaunchKernelGGL(k_run_emit, dim3((uint32_t)ntiles), dim3(kTPB), 0, st, skeys, n, toff, dk, rs);
    hipLaunchKernelGGL(k_run_payload, dim3(stream_grid(s, R)), dim3(kTPB), 0, st, rs, R, n <= (1ull << 28), rid);
    if (hipGetLastError() != hipSuccess) rc = set_err(MQ_EHIP, "join: run compaction");
    uint32_t flag = 0;
    if (!rc) HIPCHK(hipMemsetAsync(dflag, 0, 4, st));
    if (!rc) rc = insert_unique(j, dk, rid, R, slots, dflag, st, s);
    if (!rc) {
        HIPCHK(hipMemcpyAsync(&flag, dflag, 4, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
    }
    pool_free_on(dk, st);
    pool_free_on(rid, st);
    if (rc) return fail(rc);
    fail(0);
    if (flag) return 1;
    j->unique = 2;
    j->rs = rs;
    j->packed = n <= (1ull << 28);
    return 0;
}

}  // namespace

namespace mqi {

template <int TPB, int IT>
int radix_sort_tiles(const int* c1, const int* p1, uint64_t n, int mode, uint32_t kmin, int npass, uint32_t* kout,
                     uint32_t* vout, u64* pout, hipStream_t st);

int radix_sort_run(const int* c1, const int* p1, uint64_t n, int mode, uint32_t* kout, uint32_t* vout,
                   u64* pout, hipStream_t st) {
    // (A onesweep form, decoupled look-back instead of a histogram pass per pass, measured
    // slower and was removed in round 6: 1e9-row index 27.9 vs 22.3 ms, its scatter passes
    // 6.3-7.1 ms against 3.7-4.4 + 1.6 ms of histogram; right after launch every resident
    // tile walked back over ~2000 unfinished predecessors through cross-XCD status loads.)
    // tiles of 512 x 16 words: 18.7 ms for the 1e9-row index, against 21.6 with
    // 256 x 16 (digit runs of 16 words leave the block as 128-B pieces), 25.9 with
    // 1024 x 8 and 22.3 with 512 x 8 (tools/sorttpb_cmd.sh)
    return radix_sort_tiles<kSortTPB, kSortItems>(c1, p1, n, mode, 0, 4, kout, vout, pout, st);
}

// npass 8-bit digits of (key ^ 2^31) - kmin, lowest first (1 <= npass <= 4): a key
// range of at most 8 * npass bits sorts in npass passes.
template <int TPB, int IT>
int radix_sort_tiles(const int* c1, const int* p1, uint64_t n, int mode, uint32_t kmin, int npass, uint32_t* kout,
                     uint32_t* vout, u64* pout, hipStream_t st) {
    constexpr uint64_t kTile = (uint64_t)TPB * IT;
    u64 *w0 = nullptr, *w1 = nullptr, *hscan = nullptr, *scratch = nullptr;
    uint32_t* hist = nullptr;
    uint8_t* dig = nullptr;  // the next pass's digit of every row, written by the scatter
    const uint64_t ntiles = ceil_div(n, kTile);
    const uint64_t nh = ntiles * kRadix;
    auto done = [&](int rc) {
        pool_free_on(w0, st);
        pool_free_on(w1, st);
        pool_free_on(hist, st);
        pool_free_on(hscan, st);
        pool_free_on(scratch, st);
        pool_free_on(dig, st);
        return rc;
    };
    if (npass < 1 || npass > 4) return set_err(MQ_EINVAL, "sort: %d passes", npass);
    w0 = (u64*)pool_alloc(n * 8);
    const bool use_dig = npass > 1;
    if (use_dig) dig = (uint8_t*)pool_alloc(n + 16);
    w1 = (u64*)pool_alloc(n * 8);
    hist = (uint32_t*)pool_alloc(nh * 4);
    hscan = (u64*)pool_alloc(nh * 8);
    scratch = (u64*)pool_alloc(scan_scratch_elems(nh) * 8);
    if (!w0 || !w1 || !hist || !hscan || !scratch || (use_dig && !dig))
        return done(set_err(MQ_ENOMEM, "sort: buffers (%llu rows)", (unsigned long long)n));
    const dim3 g((uint32_t)ntiles), b(TPB);
    const uint32_t nt = (uint32_t)ntiles;
    for (int pass = 0; pass < npass; pass++) {
        const int shift = 8 * pass;
        const bool first = pass == 0, last = pass == npass - 1;
        uint8_t* dnext = last ? nullptr : dig;
        if (first)
            hipLaunchKernelGGL((k_sortw_hist<true, TPB, IT>), g, b, 0, st, c1, nullptr, n, shift, kmin, hist, nt);
        else if (use_dig)
            hipLaunchKernelGGL((k_sortw_hist_bytes<TPB, IT>), g, b, 0, st, dig, n, hist, nt);
        else
            hipLaunchKernelGGL((k_sortw_hist<false, TPB, IT>), g, b, 0, st, nullptr, w0, n, shift, kmin, hist, nt);
        int rc = scan_exclusive<uint32_t>(hist, hscan, nh, scratch, st);
        if (rc) return done(rc);
        if (first && !last)
            hipLaunchKernelGGL((k_sortw_scatter<true, 0, TPB, IT>), g, b, 0, st, c1, p1, nullptr, n, shift, kmin, hscan,
                               nt, w1, nullptr, nullptr, nullptr, dnext);
        else if (!last)
            hipLaunchKernelGGL((k_sortw_scatter<false, 0, TPB, IT>), g, b, 0, st, nullptr, nullptr, w0, n, shift, kmin,
                               hscan, nt, w1, nullptr, nullptr, nullptr, dnext);
        else if (mode == 1 && first)
            hipLaunchKernelGGL((k_sortw_scatter<true, 1, TPB, IT>), g, b, 0, st, c1, p1, nullptr, n, shift, kmin, hscan,
                               nt, nullptr, kout, vout, nullptr, nullptr);
        else if (mode == 1)
            hipLaunchKernelGGL((k_sortw_scatter<false, 1, TPB, IT>), g, b, 0, st, nullptr, nullptr, w0, n, shift, kmin,
                               hscan, nt, nullptr, kout, vout, nullptr, nullptr);
        else if (first)
            hipLaunchKernelGGL((k_sortw_scatter<true, 2, TPB, IT>), g, b, 0, st, c1, p1, nullptr, n, shift, kmin, hscan,
                               nt, nullptr, kout, nullptr, pout, nullptr);
        else
            hipLaunchKernelGGL((k_sortw_scatter<false, 2, TPB, IT>), g, b, 0, st, nullptr, nullptr, w0, n, shift, kmin,
                               hscan, nt, nullptr, kout, nullptr, pout, nullptr);
        if (hipGetLastError() != hipSuccess) return done(set_err(MQ_EHIP, "sort: launch"));
        u64* t = w0;
        w0 = w1;
        w1 = t;
    }
    // the temporaries go back to the pool only after the passes have run
    if (hipStreamSynchronize(st) != hipSuccess) return done(set_err(MQ_EHIP, "sort: sync"));
    return done(MQ_OK);
}

int radix_sort_pairs(const int* c1, const int* p1, uint64_t n, uint32_t** keys_out,
                     uint32_t** vals_out, hipStream_t st, const DevState* s) {
    (void)s;
    uint32_t* ko = (uint32_t*)pool_alloc(n ? n * 4 : 16);
    uint32_t* vo = (uint32_t*)pool_alloc(n ? n * 4 : 16);
    if (!ko || !vo) {
        pool_free_on(ko, st);
        pool_free_on(vo, st);
        return set_err(MQ_ENOMEM, "sort: outputs (%llu rows)", (unsigned long long)n);
    }
    int rc = n ? radix_sort_run(c1, p1, n, 1, ko, vo, nullptr, st) : MQ_OK;
    if (rc) {
        pool_free_on(ko, st);
        pool_free_on(vo, st);
        return rc;
    }
    *keys_out = ko;
    *vals_out = vo;
    return MQ_OK;
}

int radix_sort_lsd_index(const int* col, uint64_t n, uint32_t kmin, int npass, int32_t* values, uint64_t* positions,
                         hipStream_t st) {
    return n ? radix_sort_tiles<kSortTPB, kSortItems>(col, nullptr, n, 2, kmin, npass,
                                                      reinterpret_cast<uint32_t*>(values), nullptr,
                                                      reinterpret_cast<u64*>(positions), st)
             : MQ_OK;
}

}  // namespace mqi

namespace {

// defer (round 6): the last inverse pass is left to mq_join_write, fused with the pair
// write (k_pwin_gather_write); the handle keeps what it reads: pass 0's places of the
// probe rows, its tile offsets and the results in pass-0 order.
template <typename RT, bool RUNS = false>
int probe_partitioned_t(mq_join* j, const int32_t* d_c2, uint64_t n2, uint32_t* pstart, u64* hits, hipStream_t st,
                        bool defer = false) {
    const Win t = j->win;
    const int passes = j->passes;
    constexpr int PT = probe_tpb<RT>();  // the probe partition's tile width
    const uint64_t ntiles = ceil_div(n2, (uint64_t)PT * kSortItems), nh = ntiles * kRadix;
    uint32_t* K[4] = {reinterpret_cast<uint32_t*>(const_cast<int32_t*>(d_c2)), nullptr, nullptr, nullptr};
    u64* hs[3] = {nullptr, nullptr, nullptr};
    uint16_t* P[3] = {nullptr, nullptr, nullptr};  // each pass's places of its input rows
    RT* R[2] = {nullptr, nullptr};
    uint32_t *hist = nullptr, *pws = nullptr;
    u64* scratch = nullptr;
    auto done = [&](int rc) {
        for (int p = 1; p <= passes; p++) pool_free_on(K[p], st);
        for (int p = 0; p < passes; p++) pool_free_on(hs[p], st);
        for (int p = 0; p < passes; p++) pool_free_on(P[p], st);
        pool_free_on(R[0], st);
        pool_free_on(R[1], st);
        pool_free_on(hist, st);
        pool_free_on(pws, st);
        pool_free_on(scratch, st);
        return rc;
    };
    bool ok = true;
    for (int p = 1; p <= passes; p++) ok = ok && (K[p] = (uint32_t*)pool_alloc(n2 * 4));
    for (int p = 0; p < passes; p++) ok = ok && (hs[p] = (u64*)pool_alloc(nh * 8));
    for (int p = 0; p < passes; p++) ok = ok && (P[p] = (uint16_t*)pool_alloc(n2 * 2));
    ok = ok && (R[0] = (RT*)pool_alloc(n2 * sizeof(RT))) && (passes < 2 || (R[1] = (RT*)pool_alloc(n2 * sizeof(RT)))) &&
         (hist = (uint32_t*)pool_alloc(nh * 4)) && (pws = (uint32_t*)pool_alloc(((uint64_t)j->nwin + 1) * 4)) &&
         (scratch = (u64*)pool_alloc(scan_scratch_elems(nh) * 8));
    if (!ok) return done(set_err(MQ_ENOMEM, "join: partitioned probe buffers (%llu rows)", (unsigned long long)n2));
    for (int p = 0; p < passes; p++) {
        hipLaunchKernelGGL((k_win_hist<true, PT>), dim3((uint32_t)ntiles), dim3(PT), 0, st, (const int*)K[p],
                           (const u64*)nullptr, n2, t, 8 * p, hist, (uint32_t)ntiles);
        int rc = scan_exclusive<uint32_t>(hist, hs[p], nh, scratch, st);
        if (rc) return done(rc);
        if (p == 0)  // (the first pass needs no order within a digit)
            hipLaunchKernelGGL((k_pwin_scatter<PT, false>), dim3((uint32_t)ntiles), dim3(PT), 0, st, K[p], n2, t, 8 * p,
                               hs[p], (uint32_t)ntiles, K[p + 1], P[p]);
        else
            hipLaunchKernelGGL((k_pwin_scatter<PT, true>), dim3((uint32_t)ntiles), dim3(PT), 0, st, K[p], n2, t, 8 * p,
                               hs[p], (uint32_t)ntiles, K[p + 1], P[p]);
        if (hipGetLastError() != hipSuccess) return done(set_err(MQ_EHIP, "join: probe partition"));
    }
    hipLaunchKernelGGL(k_win_bounds<uint32_t>, dim3(j->nwin / kTPB + 1), dim3(kTPB), 0, st, K[passes], n2, t,
                       j->nwin, pws);
    DevState* s;
    if (int rc0 = ensure_ready(&s)) return done(rc0);
    const uint32_t gj = j->nwin < (uint32_t)s->cus * 2 ? j->nwin : (uint32_t)s->cus * 2;
    if constexpr (RUNS && sizeof(RT) == 8)  // duplicate keys on the partitioned words (run2 records)
        hipLaunchKernelGGL(k_win_join_runs, dim3(gj), dim3(kWinTPB), 0, st, j->pwords, j->pwstart, K[passes], pws,
                           j->nwin, t, reinterpret_cast<u64*>(R[0]), const_cast<int*>(j->bpos), j->pflag, j->mtot,
                           j->sentinel);
    else if constexpr (RUNS)  // a windowed runs table (k_win_build_runs), a slice per window in LDS
        hipLaunchKernelGGL(k_win_probe_tab<RT>, dim3(gj), dim3(kWinTPB), 0, st, (const u64*)j->words, K[passes], pws,
                           j->nwin, t, R[0]);
    else
        hipLaunchKernelGGL(k_win_join<RT>, dim3(gj), dim3(kWinTPB), 0, st, j->pwords, j->pwstart, K[passes], pws,
                           j->nwin, t, R[0], j->pflag, j->sentinel, j->mtot);
    if (hipGetLastError() != hipSuccess) return done(set_err(MQ_EHIP, "join: window join"));
    int cur = 0;
    for (int p = passes - 1; p >= 0; p--) {
        if (p == 0 && defer) {
            j->dperm = P[0];
            P[0] = nullptr;
            j->dhs0 = hs[0];
            j->dres = R[cur];
            hs[0] = nullptr;
            R[cur] = nullptr;
            j->deferred = true;
            break;
        }
        if (p == 0)
            hipLaunchKernelGGL((k_pwin_gather<true, RT, RUNS, PT>), dim3((uint32_t)ntiles), dim3(PT), 0, st, P[0], n2,
                               hs[0], (uint32_t)ntiles, (const RT*)R[cur], (RT*)(RUNS ? (void*)j->p01 : nullptr),
                               pstart, hits, j->sentinel);
        else
            hipLaunchKernelGGL((k_pwin_gather<false, RT, false, PT>), dim3((uint32_t)ntiles), dim3(PT), 0, st, P[p], n2,
                               hs[p], (uint32_t)ntiles, (const RT*)R[cur], R[cur ^ 1], (uint32_t*)nullptr,
                               (u64*)nullptr, j->sentinel);
        if (hipGetLastError() != hipSuccess) return done(set_err(MQ_EHIP, "join: probe unpartition"));
        cur ^= 1;
    }
    return done(MQ_OK);
}

// The same over a windowed runs table (j->words, built by k_win_build_runs): per row the
// packed run (pstart) and per 64 rows the run lengths' sum (wcnt).
int probe_partitioned_runs(mq_join* j, const int32_t* d_c2, uint64_t n2, uint32_t* pstart, uint32_t* wcnt,
                           hipStream_t st) {
    int lg = 0;
    while ((1ull << lg) < j->mask + 1) lg++;
    j->nwin = (uint32_t)((j->mask + 1) >> j->win.wlog);
    j->passes = (lg - j->win.wlog + 7) / 8;
    if (j->dupw)  // run2 records from the partitioned build words (j->p01: n2 u64)
        return probe_partitioned_t<u64, true>(j, d_c2, n2, pstart, reinterpret_cast<u64*>(wcnt), st);
    return probe_partitioned_t<uint32_t, true>(j, d_c2, n2, pstart, reinterpret_cast<u64*>(wcnt), st);
}

// A deferred probe's last inverse pass in the classic form (per-row results, hit words or
// per-word run lengths, their scan): for mq_join_counts, whose caller (the key-partitioned
// shard join) needs every row's pair count; mq_join_write then takes the classic kernels.
int finish_classic(mq_join* j, hipStream_t st) {
    DevState* s;
    if (int rc = ensure_ready(&s)) return rc;
    const int pt = j->dmode == 0 ? probe_tpb<uint32_t>() : probe_tpb<u64>();
    const uint64_t n2 = j->n2, nw = (n2 + 63) / 64, ntiles = ceil_div(n2, (uint64_t)pt * kSortItems);
    const bool runs = j->dmode == 2;
    j->pstart = (uint32_t*)pool_alloc(n2 * 4);
    j->plen = (uint32_t*)pool_alloc(runs ? nw * 4 : nw * 12);
    j->offs = (u64*)pool_alloc(nw * 8);
    j->scan_scratch = (u64*)pool_alloc(scan_scratch_elems(nw) * 8);
    if (runs) j->p01 = (u64*)pool_alloc(n2 * 8);
    if (!j->pstart || !j->plen || !j->offs || !j->scan_scratch || (runs && !j->p01))
        return set_err(MQ_ENOMEM, "mq_join_counts: buffers for %llu rows", (unsigned long long)n2);
    uint32_t* const cnt = runs ? j->plen : j->plen + 2 * nw;
    u64* const hits = reinterpret_cast<u64*>(j->plen);
    const dim3 g((uint32_t)ntiles), b(pt);
    if (runs)
        hipLaunchKernelGGL((k_pwin_gather<true, u64, true, probe_tpb<u64>()>), g, b, 0, st, j->dperm, n2, j->dhs0,
                           (uint32_t)ntiles, (const u64*)j->dres, j->p01, j->pstart, hits, j->sentinel);
    else if (j->dmode == 1)
        hipLaunchKernelGGL((k_pwin_gather<true, u64, false, probe_tpb<u64>()>), g, b, 0, st, j->dperm, n2, j->dhs0,
                           (uint32_t)ntiles, (const u64*)j->dres, (u64*)nullptr, j->pstart, hits, j->sentinel);
    else
        hipLaunchKernelGGL((k_pwin_gather<true, uint32_t, false, probe_tpb<uint32_t>()>), g, b, 0, st, j->dperm, n2,
                           j->dhs0, (uint32_t)ntiles, (const uint32_t*)j->dres, (uint32_t*)nullptr, j->pstart, hits,
                           j->sentinel);
    LAUNCHCHK("k_pwin_gather");
    if (!runs) {
        hipLaunchKernelGGL(k_hits_count, dim3(stream_grid(s, nw)), dim3(kTPB), 0, st, hits, nw, cnt);
        LAUNCHCHK("k_hits_count");
    }
    if (int rc = scan_exclusive<uint32_t>(cnt, j->offs, nw, j->scan_scratch, st)) return rc;
    pool_free_on(j->dhs0, st);
    pool_free_on(j->dres, st);
    pool_free_on(j->dperm, st);
    j->dhs0 = nullptr;
    j->dres = nullptr;
    j->dperm = nullptr;
    j->deferred = false;
    return MQ_OK;
}

// The global table of a partitioned build, for a probe too small to pay for its own
// partition (and the handle's later probes): the checked windows stored as k_win_build
// stores them.
// *flagged = 1 when the windows hold a duplicate key, the empty marker or an overfull
// window: the caller then rebuilds without the partition (rebuild_unpartitioned).
int materialize_table(mq_join* j, hipStream_t st, bool* flagged) {
    int rc = jalloc(j, (void**)&j->words, j->slots * 8);
    if (rc) return rc;
    HIPCHK(hipMemsetAsync(j->pflag, 0, 4, st));
    hipLaunchKernelGGL(k_win_build<true>, dim3(j->nwin), dim3(kWinTPB), 0, st, j->pwords, j->pwstart, j->words, j->win,
                       j->pflag);
    LAUNCHCHK("k_win_build");
    uint32_t f = 0;
    HIPCHK(hipMemcpyAsync(&f, j->pflag, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    *flagged = f != 0;
    jdrop(j, j->pwords);
    jdrop(j, j->pwstart);
    j->pwords = nullptr;
    j->pwstart = nullptr;
    j->part = false;
    return MQ_OK;
}

// The duplicate-key window join on the partitioned words (k_win_join_runs) unless a
// test forces one of the runs tables (MQ_JOIN_WINRUNS=0, MQ_JOIN_RUNS=0, MQ_JOIN_RUN2=0)
bool dupw_allowed() {
    const char* a = getenv("MQ_JOIN_WINRUNS");
    const char* b = getenv("MQ_JOIN_RUNS");
    const char* c = getenv("MQ_JOIN_RUN2");
    return !(a && a[0] == '0') && !(b && b[0] == '0') && !(c && c[0] == '0');
}

// A partitioned build (pwords, pwstart kept) turned into the duplicate-key form: packed
// run2 records, long runs' positions into bpos (n1 ints, written by the probe's windows).
int make_dupw(mq_join* j) {
    int* bp = nullptr;
    if (int rc = jalloc(j, (void**)&bp, (j->n1 ? j->n1 : 1) * 4)) return rc;
    j->bpos = bp;
    j->dupw = true;
    j->unique = 2;
    j->packed = true;
    j->rs = nullptr;
    j->marks = true;
    return MQ_OK;
}

// The build proper into a fresh handle (device and stream set). allow_part: a unique
// build of part_min_rows() rows and more keeps its window partition for the
// partitioned probe instead of building the table (a duplicate key or an overfull
// window found there later sends it back here with allow_part = false).
int build_into(mq_join* j, const int32_t* d_c1, const int32_t* d_p1, uint64_t n1, hipStream_t st, DevState* s,
               bool allow_part) {
    int rc;
    j->n1 = n1;
    j->c1 = d_c1;
    j->p1 = d_p1;
    uint64_t slots = 64;
    while (slots < 2 * n1) slots <<= 1;
    j->mask = slots - 1;
    j->win.mask = j->mask;
    j->win.wlog = 0;
    while (j->win.wlog < kWinLog && (1ull << (j->win.wlog + 1)) <= slots) j->win.wlog++;
    j->win.wmask = (1ull << j->win.wlog) - 1;
    j->slots = slots;
    // the partitioned build keeps no global table: allocated only if a path needs it
    const bool part = allow_part && n1 >= kWindowBuildRows && n1 >= part_min_rows() && j->win.wlog == kWinLog;
    uint32_t* dflag = nullptr;
    if ((!part && (rc = jalloc(j, (void**)&j->words, slots * 8))) || (rc = jalloc(j, (void**)&dflag, 16 + 512 + 16)))
        return rc;
    j->pflag = dflag + 2;  // (dflag[1] is the sampled duplicate check's)
    j->mtot = reinterpret_cast<unsigned long long*>(dflag + 132);  // (after the 128 range slots)
    j->bpos = nullptr;  // unique table carries the build positions itself
    j->unique = 1;
    if (n1) {
        HIPCHK(hipMemsetAsync(dflag, 0, 16, st));
        int* pmm = reinterpret_cast<int*>(dflag + 4);  // the payloads' range: 64 min, 64 max slots
        if (part) {  // (bounds at least as wide as the range: 0x7F7F7F7F / 0x80808080 start)
            HIPCHK(hipMemsetAsync(pmm, 0x7F, 64 * 4, st));
            HIPCHK(hipMemsetAsync(pmm + 64, 0x80, 64 * 4, st));
        }
        bool sampled = false;
        if ((rc = sample_has_dups(d_c1, n1, dflag, st, s, &sampled))) return rc;
        uint32_t dup = sampled ? 1u : 0u;
        // the partition alone when the probe will join window by window: unique keys, or
        // (round 6) sampled duplicates answered by k_win_join_runs
        const bool keep = part && (!sampled || dupw_allowed());
        if (keep) {
            if ((rc = insert_unique(j, d_c1, d_p1, n1, slots, dflag, st, s, true, pmm))) return rc;
            // the payloads' range: a value outside it marks a miss (u32 results; the run2
            // records of duplicate keys need one)
            int sl[128];
            HIPCHK(hipMemcpyAsync(sl, pmm, sizeof sl, hipMemcpyDeviceToHost, st));
            HIPCHK(hipStreamSynchronize(st));
            int mm[2] = {INT32_MAX, INT32_MIN};
            for (int q = 0; q < 64; q++) {
                mm[0] = sl[q] < mm[0] ? sl[q] : mm[0];
                mm[1] = sl[64 + q] > mm[1] ? sl[64 + q] : mm[1];
            }
            const char* nw = getenv("MQ_JOIN_NARROW");
            j->rsent_ok = mm[1] < INT32_MAX || mm[0] > INT32_MIN;
            j->narrow = !(nw && nw[0] == '0') && j->rsent_ok;
            j->sentinel = (uint32_t)(mm[1] < INT32_MAX ? INT32_MAX : INT32_MIN);
            j->part = true;
            if (!sampled) return MQ_OK;
            if (j->rsent_ok) return make_dupw(j);
            // duplicates but no free payload value: the runs tables below, from the inputs
            jdrop(j, j->pwords);
            jdrop(j, j->pwstart);
            j->pwords = nullptr;
            j->pwstart = nullptr;
            j->part = false;
        }
        if (!sampled) {
            if ((rc = insert_unique(j, d_c1, d_p1, n1, slots, dflag, st, s, false, pmm))) return rc;
            HIPCHK(hipMemcpyAsync(&dup, dflag, 4, hipMemcpyDeviceToHost, st));
            HIPCHK(hipStreamSynchronize(st));
        }
        if (part && (rc = jalloc(j, (void**)&j->words, slots * 8))) return rc;  // (sampled duplicates)
        if (dup) {  // the payloads' range for the runs probe's marker (the unique attempt's, if any, is spent)
            HIPCHK(hipMemsetAsync(pmm, 0x7F, 64 * 4, st));
            HIPCHK(hipMemsetAsync(pmm + 64, 0x80, 64 * 4, st));
        }
        if (dup && (rc = build_window_runs(j, d_c1, d_p1, n1, slots, dflag, st, s, pmm)) != 1)
            return rc;  // 0: the windowed runs build took it
        if (dup) {  // general path: stable sort by key, runs in insertion order
            j->unique = 0;
            j->bpos = d_p1;
            uint32_t *skeys, *svals;
            if ((rc = radix_sort_pairs(d_c1, d_p1, n1, &skeys, &svals, st, s))) return rc;
            if ((rc = jown(j, skeys)) || (rc = jown(j, svals))) {
                if (rc && j->owned[j->nowned - 1] != skeys) pool_free_on(svals, st);  // (skeys refused: svals still ours)
                return rc;
            }
            j->bpos = reinterpret_cast<const int*>(svals);
            if ((rc = build_runs(j, skeys, n1, slots, dflag, st, s)) != 1) return rc;  // 0: done, else an error
            // a window of the distinct keys overflowed: the global-CAS table of run heads
            j->unique = 0;
            if ((rc = jalloc(j, (void**)&j->start, slots * 4)) || (rc = jalloc(j, (void**)&j->len, slots * 4)))
                return rc;
            HIPCHK(hipMemsetAsync(j->words, 0, slots * 8, st));
            hipLaunchKernelGGL(k_ht_insert_heads, dim3(stream_grid(s, n1)), dim3(kTPB), 0, st, skeys,
                               n1, j->words, j->start, j->mask);
            LAUNCHCHK("k_ht_insert_heads");
            hipLaunchKernelGGL(k_ht_set_len, dim3(stream_grid(s, n1)), dim3(kTPB), 0, st, skeys, n1,
                               j->words, j->start, j->len, j->mask);
            LAUNCHCHK("k_ht_set_len");
        }
    }
    return MQ_OK;
}

// A partitioned build whose windows turned out to hold a duplicate key (or an overfull
// window, or the table's empty word): everything of the build dropped (stream-ordered)
// and built again from the inputs the old way. The probe arrays stay.
int rebuild_unpartitioned(mq_join* j, hipStream_t st) {
    DevState* s;
    int rc = ensure_ready(&s);
    if (rc) return rc;
    jfree_all(j);
    const int32_t *c1 = j->c1, *p1 = j->p1;
    const uint64_t n1 = j->n1;
    mq_join keep = *j;
    std::memset(j, 0, sizeof(*j));
    j->device = keep.device;
    j->stream = st;
    j->p01 = keep.p01;
    j->pstart = keep.pstart;
    j->plen = keep.plen;
    j->offs = keep.offs;
    j->scan_scratch = keep.scan_scratch;
    j->dhs0 = keep.dhs0;  // (freed by the probe that follows)
    j->dres = keep.dres;
    j->dperm = keep.dperm;
    j->longq = keep.longq;
    return build_into(j, c1, p1, n1, st, s, false);
}

}  // namespace

extern "C" {

int mq_join_build(const int32_t* d_c1, const int32_t* d_p1, uint64_t n1, mq_join** out,
                  void* stream) {
    DevState* s;
    int rc = ensure_ready(&s);
    if (rc) return rc;
    if (!out || (n1 && (!d_c1 || !d_p1))) return set_err(MQ_EINVAL, "mq_join_build: NULL pointer");
    if (n1 > 0x7FFFFFFFull) return set_err(MQ_EINVAL, "mq_join_build: build side over 2^31 rows");
    hipStream_t st = (hipStream_t)stream;
    mq_join* j = new mq_join();
    std::memset(j, 0, sizeof(*j));
    HIPCHK(hipGetDevice(&j->device));
    j->stream = st;
    if ((rc = build_into(j, d_c1, d_p1, n1, st, s, true))) {
        jfree_all(j);
        delete j;
        return rc;
    }
    *out = j;
    return MQ_OK;
}

int mq_join_probe(mq_join* j, const int32_t* d_c2, uint64_t n2, uint64_t* h_m, void* stream) {
    DevState* s;
    int rc = ensure_ready(&s);
    if (rc) return rc;
    if (!j || !h_m || (n2 && !d_c2)) return set_err(MQ_EINVAL, "mq_join_probe: bad argument");
    if (n2 > (1ull << 31)) return set_err(MQ_EINVAL, "mq_join_probe: %llu rows (int32 positions)", (unsigned long long)n2);
    hipStream_t st = (hipStream_t)stream;
    if ((rc = juse(j, st))) return rc;
    // a queued write may still read the last probe's arrays: freed in stream order
    pool_free_on(j->p01, st);
    j->p01 = nullptr;
    pool_free_on(j->pstart, st);
    pool_free_on(j->plen, st);
    pool_free_on(j->offs, st);
    pool_free_on(j->scan_scratch, st);
    pool_free_on(j->dhs0, st);
    pool_free_on(j->dres, st);
    j->pstart = j->plen = nullptr;
    j->offs = j->scan_scratch = nullptr;
    j->dhs0 = nullptr;
    j->dres = nullptr;
    pool_free_on(j->dperm, st);
    j->dperm = nullptr;
    j->deferred = false;
    j->n2 = n2;
    j->m = 0;
    *h_m = 0;
    if (n2 == 0 || j->n1 == 0) return MQ_OK;
    // a partitioned build and a probe side too small to pay for its own partition (its
    // passes and the window join read all n1 build words): the global table, once
    const uint64_t pdiv = getenv("MQ_JOIN_PART_DIV") ? strtoull(getenv("MQ_JOIN_PART_DIV"), nullptr, 10) : 16;
    if (j->dupw && n2 < j->n1 / (pdiv ? pdiv : 1)) {  // duplicate keys, a small probe: a runs table
        if ((rc = rebuild_unpartitioned(j, st))) return rc;
        return mq_join_probe(j, d_c2, n2, h_m, stream);
    }
    if (j->part && n2 < j->n1 / (pdiv ? pdiv : 1)) {
        bool flagged = false;
        if ((rc = materialize_table(j, st, &flagged))) return rc;
        if (flagged) {
            if ((rc = rebuild_unpartitioned(j, st))) return rc;
            return mq_join_probe(j, d_c2, n2, h_m, stream);
        }
    }
    // the partitioned probes of a unique build and of duplicate keys on the partitioned
    // words: up to the window join and all but the last inverse pass; M from the window
    // joins' pair count, the rest in mq_join_write (k_pwin_gather_write)
    if (j->dupw || (j->unique == 1 && j->part)) {
        j->pruns = j->run2 = j->dupw;
        HIPCHK(hipMemsetAsync(j->pflag, 0, 4, st));
        HIPCHK(hipMemsetAsync(j->mtot, 0, 8, st));
        if (j->dupw) {
            j->dmode = 2;
            rc = probe_partitioned_t<u64, true>(j, d_c2, n2, nullptr, nullptr, st, true);
        } else if (j->narrow) {
            j->dmode = 0;
            rc = probe_partitioned_t<uint32_t>(j, d_c2, n2, nullptr, nullptr, st, true);
        } else {
            j->dmode = 1;
            rc = probe_partitioned_t<u64>(j, d_c2, n2, nullptr, nullptr, st, true);
        }
        if (rc) return rc;
        uint32_t pf = 0;
        unsigned long long mm = 0;
        HIPCHK(hipMemcpyAsync(&pf, j->pflag, 4, hipMemcpyDeviceToHost, st));
        HIPCHK(hipMemcpyAsync(&mm, j->mtot, 8, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        if (pf) {
            // a probe key met a duplicate build key: the same partitioned words answer
            // duplicate keys (k_win_join_runs) when a payload value is free; otherwise, an
            // overfull window or a key on 15+ rows: rebuild from the inputs on the runs tables
            if (pf == 1u && !j->dupw && j->rsent_ok && dupw_allowed()) {
                if ((rc = make_dupw(j))) return rc;
            } else if ((rc = rebuild_unpartitioned(j, st))) {
                return rc;
            }
            return mq_join_probe(j, d_c2, n2, h_m, stream);
        }
        j->m = mm;
        *h_m = mm;
        return MQ_OK;
    }
    const uint64_t nwords = (n2 + 63) / 64;
    // packed runs: per-word lengths. Only for the windowed runs build (rs == nullptr:
    // every run shorter than 15 rows), where a word's 64 rows sum to < 2^10; a sorted
    // runs build may hold runs of up to n1 rows, whose sums over a word would wrap the
    // u32 word counts and the write's u32 wave prefix, so it takes the per-row form
    // (u32 lengths, u64 offsets).
    const bool pruns = j->unique == 2 && j->packed && j->rs == nullptr;
    j->pruns = pruns;
    j->run2 = false;
    const bool words_scan = j->unique == 1 || pruns;  // per 64-row word; else per row
    j->pstart = (uint32_t*)pool_alloc(n2 * 4);
    j->plen = (uint32_t*)pool_alloc(j->unique == 1 ? nwords * 12 : pruns ? nwords * 4 : n2 * 4);
    j->offs = (u64*)pool_alloc((words_scan ? nwords : n2) * 8);
    j->scan_scratch = (u64*)pool_alloc(scan_scratch_elems(words_scan ? nwords : n2) * 8);
    if (!j->pstart || !j->plen || !j->offs || !j->scan_scratch)
        return set_err(MQ_ENOMEM, "mq_join_probe: buffers for %llu rows", (unsigned long long)n2);
    // unique path: plen holds one 64-bit hit word per 64 rows, then those words'
    // popcounts; offs the words' output offsets. Otherwise both are per row.
    const uint64_t nw = (n2 + 63) / 64;
    const uint64_t nscan = words_scan ? nw : n2;
    uint32_t* const cnt = j->unique == 1 ? j->plen + 2 * nw : j->plen;
    if (pruns && j->win.wlog == kWinLog && j->n1 >= part_min_rows() && n2 >= j->n1 / (pdiv ? pdiv : 1)) {
        // packed runs, partitioned: the probe keys by window, each window's slice of the runs
        // table in LDS (no free payload value for run2 records, or forced by a test)
        if ((rc = probe_partitioned_runs(j, d_c2, n2, j->pstart, cnt, st))) return rc;
    } else if (pruns) {  // packed runs: each row's payload, then the per-word run lengths
        auto kern = k_ht_probe_unique<true>;
        hipLaunchKernelGGL(kern, dim3(resident_grid(s, (n2 + kProbeILP - 1) / kProbeILP, (const void*)kern)), dim3(kTPB), 0, st, d_c2, n2,
                           j->words, j->win, j->pstart, (u64*)nullptr, j->rs, (uint32_t*)nullptr, true, j->marks, cnt);
        LAUNCHCHK("k_ht_probe_unique");
    } else if (j->unique == 2) {  // runs: each row's run start and length straight from the probe
        auto kern = k_ht_probe_unique<true>;
        hipLaunchKernelGGL(kern, dim3(resident_grid(s, (n2 + kProbeILP - 1) / kProbeILP, (const void*)kern)), dim3(kTPB), 0, st, d_c2, n2,
                           j->words, j->win, j->pstart, (u64*)nullptr, j->rs, cnt, j->packed, j->marks,
                           (uint32_t*)nullptr);
        LAUNCHCHK("k_ht_probe_unique");
    } else if (j->unique) {
        u64* const hits = reinterpret_cast<u64*>(j->plen);
        auto kern = k_ht_probe_unique<false>;
        hipLaunchKernelGGL(kern, dim3(resident_grid(s, (n2 + kProbeILP - 1) / kProbeILP, (const void*)kern)), dim3(kTPB), 0, st, d_c2, n2,
                           j->words, j->win, j->pstart, hits, (const uint32_t*)nullptr, (uint32_t*)nullptr, false, j->marks,
                           (uint32_t*)nullptr);
        LAUNCHCHK("k_ht_probe_unique");
        hipLaunchKernelGGL(k_hits_count, dim3(stream_grid(s, nw)), dim3(kTPB), 0, st, hits, nw, cnt);
        LAUNCHCHK("k_hits_count");
    } else {
        hipLaunchKernelGGL(k_ht_probe, dim3(stream_grid(s, n2)), dim3(kTPB), 0, st, d_c2, n2,
                           j->words, j->start, j->len, j->mask, j->pstart, j->plen);
        LAUNCHCHK("k_ht_probe");
    }
    if ((rc = scan_exclusive<uint32_t>(cnt, j->offs, nscan, j->scan_scratch, st))) return rc;
    u64 last_off = 0;
    uint32_t last_len = 0;
    HIPCHK(hipMemcpyAsync(&last_off, j->offs + (nscan - 1), 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(&last_len, cnt + (nscan - 1), 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    j->m = last_off + last_len;
    *h_m = j->m;
    return MQ_OK;
}

int mq_join_write(mq_join* j, const int32_t* d_p2, int32_t* d_out1, int32_t* d_out2, void* stream) {
    DevState* s;
    int rc = ensure_ready(&s);
    if (rc) return rc;
    if (!j) return set_err(MQ_EINVAL, "mq_join_write: NULL handle");
    if (j->m == 0) return MQ_OK;
    if (!d_out1 || (d_out2 && !d_p2)) return set_err(MQ_EINVAL, "mq_join_write: NULL pointer");
    if ((rc = juse(j, (hipStream_t)stream))) return rc;
    if (j->deferred) {  // the last inverse pass fused with the pair write (look-back over tiles)
        hipStream_t st = (hipStream_t)stream;
        const int pt = j->dmode == 0 ? probe_tpb<uint32_t>() : probe_tpb<u64>();
        const uint64_t ntiles = ceil_div(j->n2, (uint64_t)pt * kSortItems);
        u64* stat = (u64*)pool_alloc(ntiles * 8 + 16);
        if (!stat) return set_err(MQ_ENOMEM, "mq_join_write: tile status");
        HIPCHK(hipMemsetAsync(stat, 0, ntiles * 8 + 16, st));
        HIPCHK(hipMemsetAsync(j->pflag + 1, 0, 4, st));
        const dim3 g((uint32_t)ntiles), b(pt);
        if (j->dmode == 2)
            hipLaunchKernelGGL((k_pwin_gather_write<u64, 2, probe_tpb<u64>()>), g, b, 0, st, j->dperm, j->n2, j->dhs0,
                               (uint32_t)ntiles, (const u64*)j->dres, d_p2, j->bpos, j->sentinel, d_out1, d_out2, stat,
                               j->pflag + 1);
        else if (j->dmode == 1)
            hipLaunchKernelGGL((k_pwin_gather_write<u64, 1, probe_tpb<u64>()>), g, b, 0, st, j->dperm, j->n2, j->dhs0,
                               (uint32_t)ntiles, (const u64*)j->dres, d_p2, j->bpos, j->sentinel, d_out1, d_out2, stat,
                               j->pflag + 1);
        else
            hipLaunchKernelGGL((k_pwin_gather_write<uint32_t, 0, probe_tpb<uint32_t>()>), g, b, 0, st, j->dperm, j->n2, j->dhs0,
                               (uint32_t)ntiles, (const uint32_t*)j->dres, d_p2, j->bpos, j->sentinel, d_out1, d_out2,
                               stat, j->pflag + 1);
        const hipError_t e = hipGetLastError();
        pool_free_on(stat, st);
        if (e != hipSuccess) return set_err(MQ_EHIP, "launch of k_pwin_gather_write failed: %s", hipGetErrorString(e));
        return MQ_OK;
    }
    if (j->unique == 1) {
        const bool v4 = ((reinterpret_cast<uintptr_t>(j->pstart) | reinterpret_cast<uintptr_t>(d_p2)) & 15u) == 0;
        if (v4)
            hipLaunchKernelGGL(k_join_write_hits4, dim3(stream_grid(s, (j->n2 + 3) / 4)), dim3(kTPB), 0,
                               (hipStream_t)stream, reinterpret_cast<const u64*>(j->plen), j->offs, j->pstart, d_p2,
                               j->n2, d_out1, d_out2);
        else
            hipLaunchKernelGGL(k_join_write_hits, dim3(stream_grid(s, j->n2)), dim3(kTPB), 0, (hipStream_t)stream,
                               reinterpret_cast<const u64*>(j->plen), j->offs, j->pstart, d_p2, j->n2, d_out1, d_out2);
        LAUNCHCHK("k_join_write_hits");
        return MQ_OK;
    }
    if (j->pruns && j->run2) {
        hipLaunchKernelGGL(k_join_write_runs16<8>, dim3(stream_grid(s, ((j->n2 + 63) / 64) * 64 / 8)), dim3(kTPB), 0,
                           (hipStream_t)stream, j->pstart, j->n2, j->offs, d_p2, j->p01, j->bpos, d_out1, d_out2);
        LAUNCHCHK("k_join_write_runs16");
        return MQ_OK;
    }
    if (j->pruns) {
        hipLaunchKernelGGL(k_join_write_runs_mlp<8>, dim3(stream_grid(s, ((j->n2 + 63) / 64) * 64 / 8)), dim3(kTPB), 0,
                           (hipStream_t)stream, j->pstart, j->n2, j->rs, j->offs, d_p2, j->bpos, d_out1, d_out2);
        LAUNCHCHK("k_join_write_runs");
        return MQ_OK;
    }
    // the long-run list: at most m / kLongRun chunks (+ one per run for the rounding)
    const uint64_t qcap = j->m / kLongRun + j->m / kLongChunk + 2;
    if (qcap > 0xFFFFFFF0ull) return set_err(MQ_EINVAL, "mq_join_write: %llu pairs", (unsigned long long)j->m);
    pool_free_on(j->longq, (hipStream_t)stream);
    if (!(j->longq = (u64*)pool_alloc(qcap * 8 + 16))) return set_err(MQ_ENOMEM, "mq_join_write: long-run list");
    uint32_t* const nlong = reinterpret_cast<uint32_t*>(j->longq + qcap);
    HIPCHK(hipMemsetAsync(nlong, 0, 4, (hipStream_t)stream));
    hipLaunchKernelGGL(k_join_write, dim3(stream_grid(s, j->n2)), dim3(kTPB), 0, (hipStream_t)stream,
                       j->pstart, j->plen, j->offs, d_p2,
                       j->bpos, j->n2, d_out1, d_out2, j->longq, nlong);
    LAUNCHCHK("k_join_write");
    hipLaunchKernelGGL(k_join_write_long, dim3(s->cus * 8), dim3(kTPB), 0, (hipStream_t)stream, j->pstart, j->plen,
                       j->offs, d_p2, j->bpos, j->longq, nlong, d_out1, d_out2);
    LAUNCHCHK("k_join_write_long");
    return MQ_OK;
}

int mq_join_counts(mq_join* j, uint32_t* d_cnt, void* stream) {
    DevState* s;
    int rc = ensure_ready(&s);
    if (rc) return rc;
    if (!j || (j->n2 && !d_cnt)) return set_err(MQ_EINVAL, "mq_join_counts: bad argument");
    if (j->n2 == 0) return MQ_OK;
    hipStream_t st = (hipStream_t)stream;
    if ((rc = juse(j, st))) return rc;
    if (j->n1 == 0) {  // the probe ran nothing: no row matched
        HIPCHK(hipMemsetAsync(d_cnt, 0, j->n2 * 4, st));
        return MQ_OK;
    }
    if (j->deferred && (rc = finish_classic(j, st))) return rc;
    const u64* hits = j->unique == 1 ? reinterpret_cast<const u64*>(j->plen) : nullptr;
    const uint32_t* pk = (!hits && j->pruns) ? j->pstart : nullptr;
    const uint32_t* plen = (!hits && !j->pruns) ? j->plen : nullptr;
    hipLaunchKernelGGL(k_join_counts, dim3(stream_grid(s, j->n2)), dim3(kTPB), 0, st, hits, pk, plen, j->n2, d_cnt);
    LAUNCHCHK("k_join_counts");
    return MQ_OK;
}

int mq_random_read(const uint64_t* d_table, int slots_log2, uint64_t n_reads, void* d_ws, void* stream) {
    DevState* s;
    int rc = ensure_ready(&s);
    if (rc) return rc;
    if (!d_table || !d_ws) return set_err(MQ_EINVAL, "mq_random_read: NULL pointer");
    if (slots_log2 < 0 || slots_log2 > 40) return set_err(MQ_EINVAL, "mq_random_read: slots_log2 %d", slots_log2);
    if (n_reads == 0) return MQ_OK;
    hipLaunchKernelGGL(k_random_read, dim3(stream_grid(s, (n_reads + kProbeILP - 1) / kProbeILP)), dim3(kTPB), 0,
                       (hipStream_t)stream, reinterpret_cast<const u64*>(d_table), (1ull << slots_log2) - 1,
                       n_reads, static_cast<u64*>(d_ws));
    LAUNCHCHK("k_random_read");
    return MQ_OK;
}

int mq_join_free(mq_join* j) {
    if (!j) return MQ_OK;
    // queued probe / write kernels may still use the buffers: freed in j->stream's order
    pool_free_on(j->p01, j->stream);
    pool_free_on(j->pstart, j->stream);
    pool_free_on(j->plen, j->stream);
    pool_free_on(j->offs, j->stream);
    pool_free_on(j->scan_scratch, j->stream);
    pool_free_on(j->longq, j->stream);
    pool_free_on(j->dhs0, j->stream);
    pool_free_on(j->dres, j->stream);
    pool_free_on(j->dperm, j->stream);
    jfree_all(j);
    delete j;
    return MQ_OK;
}

int mq_hash_join(const int32_t* d_c1, const int32_t* d_p1, uint64_t n1, const int32_t* d_c2,
                 const int32_t* d_p2, uint64_t n2, int32_t* d_out1, int32_t* d_out2,
                 uint64_t cap, uint64_t* h_m, void* stream) {
    if (!h_m) return set_err(MQ_EINVAL, "mq_hash_join: NULL h_m");
    mq_join* j = nullptr;
    int rc = mq_join_build(d_c1, d_p1, n1, &j, stream);
    if (rc) return rc;
    if ((rc = mq_join_probe(j, d_c2, n2, h_m, stream))) {
        mq_join_free(j);
        return rc;
    }
    if (*h_m > cap || !d_out1 || !d_out2) {
        mq_join_free(j);
        return *h_m == 0 ? MQ_OK : MQ_ECAP;
    }
    const bool fused = j->deferred;
    rc = mq_join_write(j, d_p2, d_out1, d_out2, stream);
    if (!rc) rc = mq_stream_sync(stream);
    if (!rc && fused) {  // the fused write's look-back gave up (never expected): fail loudly
        uint32_t e = 0;
        if (hipMemcpy(&e, j->pflag + 1, 4, hipMemcpyDeviceToHost) != hipSuccess || e)
            rc = set_err(MQ_EHIP, "mq_hash_join: the fused write's look-back failed");
    }
    mq_join_free(j);
    return rc;
}

}  // extern "C"
