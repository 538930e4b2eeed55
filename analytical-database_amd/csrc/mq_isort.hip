// mq_isort.hip — the (value, row) sort behind mq_index_build (build_index,
// src/index.c:152-178, whose quicksort :25-46 it replaces; equal values come out in
// ascending row order, the stable radix order).
//
// The key range picks the form. One read of the column (mq_reduce) gives min and max;
// keys are k = (value ^ 2^31) - min, b = bit length of max - min.
// * b <= 24, or fewer than 2^22 rows: the LSD radix sort of mq_join.hip with
//   ceil(b / 8) passes instead of 4 (every pass reads and writes all n words).
// * otherwise MSD levels, then one LDS pass per range:
//   - a level splits each of its ranges by the next w <= 8 key bits: per tile of 8192
//     words an LDS histogram, one exclusive scan over (range, digit, tile), a stable
//     ballot-ranked scatter staged in LDS (the LSD sort's scatter, tiles mapped onto
//     ranges). The first level reads the int32 column and builds {k + min, row}
//     words; later levels histogram the digit byte the previous scatter wrote.
//   - a child range of at most kCap = 16384 words, or one with no key bits left, is
//     finished by one 1024-lane block: the words go to registers, are sorted by the
//     remaining bits in LDS (ceil(bits / 8) stable ballot-ranked passes through one
//     128 KB buffer), and leave as the index's int32 values and size_t positions,
//     coalesced. Larger children form the next level.
//   At 1e9 uniform rows (b = 30): two levels (256, then 65536 ranges of ~15.3K rows)
//   and the finisher, ≈ 58 B of HBM traffic a row against 74 for four LSD passes.
// Ranges, tiles and finisher lists are built on the device (atomic appends: order
// among ranges does not matter, every range has its own place in the output and its
// own slice of the scan); the host reads three counters per level.

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <cstring>

#include "mq_common.h"
#include "mq_device.h"

namespace {

using namespace mqi;
typedef unsigned long long u64;

constexpr int kMT = 512;  // MSD tile: kMT x kMI words (the LSD sort's tile)
constexpr int kMI = 16;
constexpr uint32_t kMTile = (uint32_t)kMT * kMI;
constexpr int kFT = 1024;  // finisher block: one range of at most kCap words in LDS
constexpr int kFI = 16;
constexpr uint32_t kCap = (uint32_t)kFT * kFI;
constexpr int kCountBits = 14;  // the counting finisher: keys below 2^14 (a u32 count cell each)
constexpr uint32_t kTieMax = 24;  // ... and no key on more rows (ties are put in row order serially)

struct Seg {  // a range split by this level: rows [start, start + len), tiles t0 .. t0 + nt,
    u64 start;  // keys k - klo in [0, the level's R)
    uint32_t len, t0, nt, klo;
};
struct Fin {  // a range the finisher completes: keys k - klo below 2^s, words in buffer buf
    u64 start;
    uint32_t len, klo, meta, _pad;  // meta = s | buf << 8
};
struct Ctr {
    uint32_t nfin, nnext, tnext, maxlen;
    uint32_t nranked, nfb, _pad[2];  // ranges for the ranked finisher: wide keys, count fallbacks
};

__host__ __device__ inline uint64_t cdiv(uint64_t a, uint64_t b) { return (a + b - 1) / b; }

// A level's digit of key x = k - klo (x < R): floor(x * M / 2^32) with M = floor(2^32 P / R),
// monotone and below P. Digit d holds the keys x in [lo(d), lo(d + 1)), lo(d) =
// ceil(d 2^32 / M), at most floor(2^32 / M) + 1 of them: the next level's R.
__device__ __forceinline__ uint32_t digit_of(uint32_t x, u64 M) { return (uint32_t)(((u64)x * M) >> 32); }
// The same for M < 2^32 (P < R, every level that splits a range into more than single
// keys): one v_mul_hi_u32 instead of a 64-bit multiply.
template <bool WIDE>
__device__ __forceinline__ uint32_t digit_m(uint32_t x, u64 M) {
    if constexpr (WIDE) return digit_of(x, M);
    else return __umulhi(x, (uint32_t)M);
}
__host__ __device__ inline u64 digit_lo(uint32_t d, u64 M) { return cdiv((u64)d << 32, M); }

__global__ void k_tile_seg(const Seg* __restrict__ segs, uint32_t* __restrict__ tseg) {
    const Seg sg = segs[blockIdx.x];
    for (uint32_t i = threadIdx.x; i < sg.nt; i += blockDim.x) tseg[sg.t0 + i] = blockIdx.x;
}

// The tile's range, its tile index within the range and its row count.
__device__ __forceinline__ void tile_range(const Seg* segs, const uint32_t* tseg, uint32_t t, Seg& sg, uint32_t& tin,
                                           uint32_t& len) {
    sg = segs[tseg[t]];
    tin = t - sg.t0;
    const uint32_t r = sg.len - tin * kMTile;
    len = r < kMTile ? r : kMTile;
}

// Per tile: counts of the level's digit, into hist[t0 * P + d * nt + tin]: from the int32
// column (level 0) or from the digit bytes the previous scatter wrote. (Round 6 measured
// the histogram computing the digits from the previous scatter's words instead, with no
// digit bytes written: 14.77 ms against 14.23 at 1e9, alternating on one box.)
template <bool FIRST, bool WIDE>
__global__ __launch_bounds__(kMT) void k_msd_hist(const int* __restrict__ col, const uint8_t* __restrict__ dig,
                                                  const Seg* __restrict__ segs, const uint32_t* __restrict__ tseg,
                                                  uint32_t kmin, u64 M, uint32_t P, uint32_t* __restrict__ hist) {
    __shared__ uint32_t h[256];
    const int tid = threadIdx.x;
    if (tid < 256) h[tid] = 0;
    __syncthreads();
    Seg sg;
    uint32_t tin, len;
    tile_range(segs, tseg, xcd_tile(blockIdx.x, gridDim.x), sg, tin, len);
    const u64 e0 = sg.start + (u64)tin * kMTile;
    if constexpr (FIRST) {
        uint32_t d[kMI];
#pragma unroll
        for (int k = 0; k < kMI; k++) {
            const uint32_t i = (uint32_t)k * kMT + tid;
            const u64 ic = e0 + (i < len ? i : len - 1);
            d[k] = digit_m<WIDE>(((uint32_t)__builtin_nontemporal_load(col + ic) ^ 0x80000000u) - kmin, M);
        }
#pragma unroll
        for (int k = 0; k < kMI; k++)
            if ((uint32_t)k * kMT + tid < len) atomicAdd(&h[d[k]], 1u);
    } else {
        // (round 6) the tile's digit bytes as the dwords covering [e0, e0 + len): a byte
        // load a lane made the pass issue-bound (1 GB in 0.43 ms at 1e9 rows). dig holds
        // at least n + 3 bytes, so the last dword is inside it.
        constexpr int kDW = kMI / 4 + 1;
        const u64 a0 = e0 & ~3ull;
        const uint32_t lead = (uint32_t)(e0 - a0), nw = (lead + len + 3u) >> 2;
        const uint32_t* d32 = reinterpret_cast<const uint32_t*>(dig) + (a0 >> 2);
        uint32_t wv[kDW];
#pragma unroll
        for (int k = 0; k < kDW; k++) {
            const uint32_t i = (uint32_t)k * kMT + tid;
            wv[k] = i < nw ? __builtin_nontemporal_load(d32 + i) : 0u;
        }
#pragma unroll
        for (int k = 0; k < kDW; k++) {
            const uint32_t i = (uint32_t)k * kMT + tid;
            if (i < nw) {
#pragma unroll
                for (uint32_t j = 0; j < 4; j++) {
                    const uint32_t b = 4u * i + j;
                    if (b >= lead && b < lead + len) atomicAdd(&h[(wv[k] >> (8u * j)) & 0xFFu], 1u);
                }
            }
        }
    }
    __syncthreads();
    if (tid < (int)P) hist[(u64)sg.t0 * P + (u64)tid * sg.nt + tin] = h[tid];
}

// Ranks a wave's IT items by digit (stable: item order k, then lane), counting into
// wc[d] (the wave's row of the block's counters). dr[k] = d << 16 | rank within the
// wave's items of digit d. Digits: byte `sh` of key - kbase (DIG = false) or the
// level digit of key - kbase (DIG = true).
template <int IT, bool LEVEL, bool WIDE = true>
__device__ __forceinline__ void rank_items(const u64 (&el)[IT], uint32_t (&dr)[IT], uint32_t wbase, uint32_t len,
                                           uint32_t kbase, int sh, uint32_t wm, u64 M, uint32_t* wc, int lane) {
#pragma unroll
    for (int k = 0; k < IT; k++) {
        const bool valid = wbase + (uint32_t)k * 64 + lane < len;
        const uint32_t x = (uint32_t)el[k] - kbase;
        const uint32_t d = LEVEL ? digit_m<WIDE>(x, M) : (x >> sh) & wm;
        const u64 peers = match_any8(d, __ballot(valid));
        const uint32_t lt = lanes_below(peers);
        const uint32_t cur = wc[d];
        __builtin_amdgcn_wave_barrier();
        if (valid && lt == 0) wc[d] = cur + (uint32_t)__popcll(peers);
        __builtin_amdgcn_wave_barrier();
        dr[k] = valid ? ((d << 16) | (cur + lt)) : 0xFFFFFFFFu;
    }
}

// After rank_items in every wave: wcnt[w][d] becomes the count of digit d in waves
// before w, loff[d] the block-local start of digit d. Threads 0..255 (waves 0-3).
template <int NW>
__device__ __forceinline__ void digit_offsets(uint32_t (*wcnt)[256], uint32_t* loff, uint32_t* wsum, int tid) {
    const int lane = tid & 63, wave = tid >> 6;
    uint32_t tot = 0, incl = 0;
    if (tid < 256) {
#pragma unroll
        for (int w = 0; w < NW; w++) {
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
    if (tid < 256) {
        uint32_t excl = incl - tot;
        for (int w = 0; w < wave; w++) excl += wsum[w];
        loff[tid] = excl;
    }
    __syncthreads();
}

// Stable scatter of a level: each tile's words ranked by digit in LDS, then written
// as contiguous digit runs at the range's start + the scanned offsets. Mn != 0: also
// the next level's digit of every word (of its key relative to its child range).
template <bool FIRST, bool WIDE, bool NWIDE>
__global__ __launch_bounds__(kMT) void k_msd_scatter(const int* __restrict__ col, const u64* __restrict__ in,
                                                     const Seg* __restrict__ segs, const uint32_t* __restrict__ tseg,
                                                     const uint32_t* __restrict__ hscan, uint32_t kmin, u64 M,
                                                     uint32_t P, u64 Mn, u64* __restrict__ out,
                                                     uint8_t* __restrict__ dig) {
    constexpr int kW = kMT / 64;
    __shared__ uint32_t wcnt[kW][256];
    __shared__ uint32_t loff[256];
    __shared__ u64 gofs[256];
    __shared__ uint32_t clo[256];
    __shared__ u64 stage[kMTile];
    __shared__ uint32_t wsum[4];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (int x = tid; x < kW * 256; x += kMT) (&wcnt[0][0])[x] = 0;
    Seg sg;
    uint32_t tin, len;
    tile_range(segs, tseg, xcd_tile(blockIdx.x, gridDim.x), sg, tin, len);
    const u64 hb = (u64)sg.t0 * P;
    if (tid < (int)P) {
        gofs[tid] = sg.start + (u64)(hscan[hb + (u64)tid * sg.nt + tin] - hscan[hb]);
        clo[tid] = Mn ? (uint32_t)digit_lo(tid, M) : 0u;
    }
    __syncthreads();
    const u64 e0 = sg.start + (u64)tin * kMTile;
    const uint32_t wbase = (uint32_t)wave * (64 * kMI);
    const uint32_t kbase = kmin + sg.klo;
    u64 el[kMI];
    uint32_t dr[kMI];
#pragma unroll
    for (int k = 0; k < kMI; k++) {
        const uint32_t i = wbase + (uint32_t)k * 64 + lane;
        const u64 ic = e0 + (i < len ? i : len - 1);
        if constexpr (FIRST)
            el[k] = (u64)((uint32_t)col[ic] ^ 0x80000000u) | ((u64)ic << 32);
        else
            el[k] = in[ic];
    }
    rank_items<kMI, true, WIDE>(el, dr, wbase, len, kbase, 0, 0, M, wcnt[wave], lane);
    __syncthreads();
    digit_offsets<kW>(wcnt, loff, wsum, tid);
#pragma unroll
    for (int k = 0; k < kMI; k++) {
        if (dr[k] != 0xFFFFFFFFu) {
            const uint32_t d = dr[k] >> 16, r = dr[k] & 0xFFFF;
            stage[loff[d] + wcnt[wave][d] + r] = el[k];
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kMI; k++) {
        const uint32_t e = (uint32_t)k * kMT + tid;
        if (e < len) {
            const u64 v = stage[e];
            const uint32_t x = (uint32_t)v - kbase;
            const uint32_t d = digit_m<WIDE>(x, M);
            const u64 dst = gofs[d] + (e - loff[d]);
            out[dst] = v;
            // (round 6 measured the bytes leaving as dwords instead, through LDS and one
            // dword store per covered dword: the level-0 scatter took 5.09 ms against 4.00)
            if (Mn) dig[dst] = (uint8_t)digit_m<NWIDE>(x - clo[d], Mn);
        }
    }
}

// One thread per (range, digit): the child's rows from the scan, its keys from the
// digit bounds. A child of at most kCap rows, or of one key, goes to the finisher
// list; a larger one to the next level (its tiles appended by one atomic).
__global__ __launch_bounds__(256) void k_msd_children(const Seg* __restrict__ segs, uint32_t nseg,
                                                      const uint32_t* __restrict__ hscan, u64 M, uint32_t P, u64 R,
                                                      int buf, Fin* __restrict__ fins, Fin* __restrict__ ranked,
                                                      Seg* __restrict__ next, Ctr* __restrict__ ctr) {
    const uint32_t g = blockIdx.x * 256u + threadIdx.x;
    if (g >= nseg * P) return;
    const uint32_t si = g / P, d = g - si * P;
    const Seg sg = segs[si];
    const u64 hb = (u64)sg.t0 * P;
    const uint32_t base = hscan[hb];
    const uint32_t a = hscan[hb + (u64)d * sg.nt] - base;
    const uint32_t b = d + 1 < P ? hscan[hb + (u64)(d + 1) * sg.nt] - base : sg.len;
    const uint32_t cnt = b - a;
    if (!cnt) return;
    const u64 st = sg.start + a;
    const u64 lo = digit_lo(d, M), hi0 = digit_lo(d + 1, M), hi = hi0 < R ? hi0 : R;
    const u64 span = hi - lo - 1;  // the child's keys are x - lo in [0, span]
    const int s = span ? 64 - __builtin_clzll(span) : 0;
    const uint32_t klo = sg.klo + (uint32_t)lo;
    if (s == 0 || cnt <= kCap) {
        const Fin f{st, cnt, klo, (uint32_t)(cnt > 1 ? s : 0) | ((uint32_t)buf << 8), 0};
        if (cnt > 1 && s > kCountBits)
            ranked[atomicAdd(&ctr->nranked, 1u)] = f;
        else
            fins[atomicAdd(&ctr->nfin, 1u)] = f;
    } else {
        const uint32_t nt = (uint32_t)cdiv(cnt, kMTile);
        const uint32_t t0 = atomicAdd(&ctr->tnext, nt);
        const uint32_t idx = atomicAdd(&ctr->nnext, 1u);
        next[idx] = Seg{st, cnt, t0, nt, klo};
        atomicMax(&ctr->maxlen, cnt);
    }
}

__device__ __forceinline__ void emit(int32_t* vout, u64* pout, u64 i, u64 v) {
    if (vout) vout[i] = (int32_t)((uint32_t)v ^ 0x80000000u);
    if (pout) pout[i] = v >> 32;
}


// The counting finisher runs as T threads x I rows (T * I = kCap). BF: guards without
// branches (a lane past the range's end counts into a dummy cell word and places into
// a dummy slot): per-row `if`s cost ≈ 12 scalar instructions each for the exec mask,
// and scalar issue bound the 1024 x 16 form; at 1024 x 16 the branch-free form spills.
template <int T>
__device__ __forceinline__ uint32_t count_words(int s) {
    const uint32_t nw = (1u << s) / 2;  // cell words (two u16 cells each), whole waves
    return nw < (uint32_t)T ? (uint32_t)T : nw;
}

// The counting finisher of one range (keys x = k - kbase below 2^s, s <= kCountBits),
// el[] in round-major order (element k * T + tid). c32: a u16 cell per key, two to a
// word, zeroed by the caller (counts, then, after the scan, running slots relative to
// the scanning wave's start); rows / keys: the placed row ids and keys by slot. A row
// takes its slot by one atomic on its key's cell; a row whose key holds other rows
// (they took their slots in any order) is then written at the group's start + the
// number of the group's rows with a smaller id, values and positions slot by slot,
// and the range's cell words are zeroed again for the next range. Returns false,
// having written nothing outside LDS, when some key holds more than kTieMax rows
// (the cells are then left for the caller to zero).
template <int T, int I, bool BF>
__device__ __forceinline__ bool finish_counting(const u64 (&el)[I], uint32_t len, uint32_t kbase, int s,
                                                uint32_t* c32, uint32_t* rows, uint16_t* keys, uint32_t* wsum,
                                                int32_t* vout, u64* pout) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    constexpr int kW = T / 64;
    const uint32_t nw = count_words<T>(s);
#pragma unroll
    for (int k = 0; k < I; k++) {
        const uint32_t x = (uint32_t)el[k] - kbase;
        const bool v = (uint32_t)k * T + tid < len;
        if (BF)
            atomicAdd(&c32[v ? x >> 1 : kCap / 2], 1u << (16 * (x & 1)));
        else if (v)
            atomicAdd(&c32[x >> 1], 1u << (16 * (x & 1)));
    }
    __syncthreads();
    // each lane scans q consecutive words (wave w: words [w * nw / kW, (w + 1) * nw / kW))
    const uint32_t per = nw / kW, q = per / 64, lgper = 31 - __builtin_clz(per);
    uint32_t* mine = c32 + wave * per + lane * q;
    uint32_t tot = 0, mx = 0;
    for (uint32_t j = 0; j < q; j++) {
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
    uint32_t run = incl - tot;  // slots before this lane's words, within the wave
    for (uint32_t j = 0; j < q; j++) {
        const uint32_t cell = mine[j], lo = cell & 0xFFFFu;
        mine[j] = run | ((run + lo) << 16);
        run += lo + (cell >> 16);
    }
    if (lane == 63) wsum[wave] = incl;
    if (__ballot(mx > kTieMax)) wsum[kW] = 1;  // benign race: any writer stores 1
    __syncthreads();
    if (wsum[kW]) return false;
    // the slots before each wave's words: lane w of every wave holds those of wave w
    uint32_t wpre = lane < kW ? wsum[lane] : 0u;
#pragma unroll
    for (int off = 1; off < kW; off <<= 1) {
        const uint32_t y = __shfl_up(wpre, off, 64);
        if (lane >= off) wpre += y;
    }
    wpre = __shfl_up(wpre, 1, 64);
    wpre = lane ? wpre : 0u;
#pragma unroll
    for (int k = 0; k < I; k++) {
        const uint32_t x = (uint32_t)el[k] - kbase, sh = 16 * (x & 1);
        const uint32_t base = __shfl(wpre, (x >> 1) >> lgper, 64);
        const bool v = (uint32_t)k * T + tid < len;
        if (BF) {
            const uint32_t old = atomicAdd(&c32[v ? x >> 1 : kCap / 2], 1u << sh);
            const uint32_t slot = v ? ((old >> sh) & 0xFFFFu) + base : kCap;
            rows[slot] = (uint32_t)(el[k] >> 32);
            keys[slot] = (uint16_t)x;
        } else if (v) {
            const uint32_t slot = ((atomicAdd(&c32[x >> 1], 1u << sh) >> sh) & 0xFFFFu) + base;
            rows[slot] = (uint32_t)(el[k] >> 32);
            keys[slot] = (uint16_t)x;
        }
    }
    __syncthreads();
    // the cell of x now holds the end of its slots, the cell of x - 1 their start
    const uint16_t* c16 = reinterpret_cast<const uint16_t*>(c32);
#pragma unroll
    for (int k = 0; k < I; k++) {
        const uint32_t e = (uint32_t)k * T + tid;
        const uint32_t ec = e < len ? e : len - 1;
        const uint32_t x = keys[ec], r = rows[ec];
        const bool tied = (ec > 0 && keys[ec - 1] == x) | (ec + 1 < len && keys[ec + 1] == x);
        const uint32_t xp = x ? x - 1 : 0;
        const uint32_t b0 = __shfl(wpre, (xp >> 1) >> lgper, 64);
        uint32_t pos = ec;
        if (tied) {
            pos = x ? c16[xp] + b0 : 0u;
            for (uint32_t j = pos; j < len && keys[j] == x; j++) pos += rows[j] < r;
        }
        if (e < len) {
            if (vout) vout[e] = (int32_t)((kbase + x) ^ 0x80000000u);
            if (pout) pout[pos] = r;
        }
    }
    __syncthreads();
    for (uint32_t x = tid; x < nw; x += T) c32[x] = 0;
    if (tid == 0) wsum[kW] = 0;
    return true;
}

// The counting finisher, second form (round 4): the same sort with
// fewer scalar and LDS instructions. The first form's PMC at 1e9 rows: 2.5 G SALU
// (exec-mask bookkeeping of per-row guards) and 0.71 G LDS instructions with 1.35 G
// bank-conflict cycles. Here:
//  * after the scan every cell holds an absolute slot (each wave adds the slots of the
//    waves before it to its own words; one more barrier), so no row looks up its
//    wave's base with a lane shuffle (ds_bpermute, an LDS instruction);
//  * the placement has no branch: a row past the range's end takes the dummy cell word
//    and the dummy slot kCap;
//  * a row's tie rank is counted over its key's slot group [cell(x - 1), cell(x)), read
//    from the cells (an untied row's group is itself), instead of testing both
//    neighbours' keys for every row and walking the group by key.
// Static counts (hipcc -S): 905 SALU / 201 LDS / 90 exec saves against 1265 / 252 /
// 182, 128 VGPRs, no spills. (Branch-free counting, or per-round uniform guards, spilled
// the prefetched next range: tools-free A/B of 36 variants by the compiler's counts.)
template <int T, int I>
__device__ __forceinline__ bool finish_counting2(const u64 (&el)[I], uint32_t len, uint32_t kbase, int s,
                                                 uint32_t* c32, uint32_t* rows, uint16_t* keys, uint32_t* wsum,
                                                 int32_t* vout, u64* pout) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    constexpr int kW = T / 64;
    const uint32_t nw = count_words<T>(s);
#pragma unroll
    for (int k = 0; k < I; k++) {
        const uint32_t x = (uint32_t)el[k] - kbase;
        const bool v = (uint32_t)k * T + tid < len;
        if (v) atomicAdd(&c32[x >> 1], 1u << (16 * (x & 1)));
    }
    __syncthreads();
    const uint32_t per = nw / kW, q = per / 64;
    uint32_t* mine = c32 + wave * per + lane * q;
    uint32_t tot = 0, mx = 0;
    for (uint32_t j = 0; j < q; j++) {
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
    if (__ballot(mx > kTieMax)) wsum[kW] = 1;  // benign race: any writer stores 1
    __syncthreads();
    if (wsum[kW]) return false;
    uint32_t base = 0;  // the slots of the waves before this one (wave-uniform)
    for (int w = 0; w < wave; w++) base += wsum[w];
    uint32_t run = base + incl - tot;
    for (uint32_t j = 0; j < q; j++) {
        const uint32_t cell = mine[j], lo = cell & 0xFFFFu;
        mine[j] = run | ((run + lo) << 16);
        run += lo + (cell >> 16);
    }
    __syncthreads();
    // the slots by atomics in batches of kB, their results waited for once a batch (the
    // compiler keeps an LDS atomic ahead of the stores after it, which waited out every
    // atomic's round trip)
    constexpr int kB = 4;
#pragma unroll
    for (int k0 = 0; k0 < I; k0 += kB) {
        uint32_t old[kB];
#pragma unroll
        for (int u = 0; u < kB; u++) {
            const int k = k0 + u;
            const uint32_t x = (uint32_t)el[k] - kbase, sh = 16 * (x & 1);
            const bool v = (uint32_t)k * T + tid < len;
            old[u] = atomicAdd(&c32[v ? x >> 1 : kCap / 2], 1u << sh);
        }
#pragma unroll
        for (int u = 0; u < kB; u++) {
            const int k = k0 + u;
            const uint32_t x = (uint32_t)el[k] - kbase, sh = 16 * (x & 1);
            const bool v = (uint32_t)k * T + tid < len;
            const uint32_t slot = v ? ((old[u] >> sh) & 0xFFFFu) : kCap;
            rows[slot] = (uint32_t)(el[k] >> 32);
            keys[slot] = (uint16_t)x;
        }
    }
    __syncthreads();
    const uint16_t* c16 = reinterpret_cast<const uint16_t*>(c32);
    // rows in batches of kB: their slot reads, then their groups' bounds, issued together
    // (one row at a time waited out each read's latency twice a row), then the tie walk
    // for the rows that share their key
#pragma unroll
    for (int k0 = 0; k0 < I; k0 += kB) {
        uint32_t x[kB], r[kB], gs[kB], ge[kB];
#pragma unroll
        for (int u = 0; u < kB; u++) {
            const uint32_t e = (uint32_t)(k0 + u) * T + tid;
            const uint32_t ec = e < len ? e : len - 1;
            x[u] = keys[ec];
            r[u] = rows[ec];
        }
#pragma unroll
        for (int u = 0; u < kB; u++) {
            ge[u] = c16[x[u]];
            gs[u] = x[u] ? c16[x[u] - 1] : 0u;
        }
#pragma unroll
        for (int u = 0; u < kB; u++) {
            const uint32_t e = (uint32_t)(k0 + u) * T + tid;
            uint32_t pos = gs[u];
            if (ge[u] - gs[u] > 1) {
#pragma unroll 1
                for (uint32_t j = gs[u]; j < ge[u]; j++) pos += rows[j] < r[u];
            }
            if (e < len) {
                vout[e] = (int32_t)((kbase + x[u]) ^ 0x80000000u);
                pout[pos] = r[u];
            }
        }
    }
    __syncthreads();
    for (uint32_t x = tid; x < nw; x += T) c32[x] = 0;
    if (tid == 0) {
        wsum[kW] = 0;
        c32[kCap / 2] = 0;
    }
    return true;
}

// The counting finisher, persistent: a block per CU walks the list, and the next
// range's words are loaded into registers while the current one is sorted (a block
// holds 128 KB of LDS, so a CU runs one: without this its loads, LDS work and stores
// would take turns). A range it cannot take goes to the ranked finisher's list.
template <int T, int I, bool BF, bool V2 = false>
__global__ __launch_bounds__(T) void k_msd_finish_count(const u64* __restrict__ w0, const u64* __restrict__ w1,
                                                        const Fin* __restrict__ fins, uint32_t nfin, uint32_t kmin,
                                                        int32_t* __restrict__ vout, u64* __restrict__ pout,
                                                        Fin* __restrict__ fb, Ctr* __restrict__ ctr) {
    static_assert(T * I == (int)kCap, "a range of kCap rows per block");
    constexpr int kW = T / 64;
    __shared__ uint32_t c32[kCap / 2 + 1];  // u16 cells of 2^14 keys (+ BF's dummy word)
    __shared__ uint32_t rows[kCap + 1];     // by slot (+ BF's dummy slot)
    __shared__ uint16_t keys[kCap + 1];
    __shared__ uint32_t wsum[kW + 1];  // wave totals, then the fallback flag
    const int tid = threadIdx.x;
    u64 nx[I];
    auto prefetch = [&](uint32_t fi) {  // the words of range fi, if the counting path sorts it
        const Fin f = fins[fi];
        if ((f.meta & 0xFF) == 0) return;
        const u64* src = ((f.meta >> 8) ? w1 : w0) + f.start;
#pragma unroll
        for (int k = 0; k < I; k++) {
            const uint32_t i = (uint32_t)k * T + tid;
            nx[k] = src[i < f.len ? i : f.len - 1];
        }
    };
    if (blockIdx.x >= nfin) return;
    prefetch(blockIdx.x);
    for (uint32_t x = tid; x < kCap / 2; x += T) c32[x] = 0;
    if (tid == 0) wsum[kW] = 0;
    __syncthreads();
    for (uint32_t fi = blockIdx.x; fi < nfin; fi += gridDim.x) {
        const Fin f = fins[fi];
        const int s = (int)(f.meta & 0xFF);
        const u64* src = ((f.meta >> 8) ? w1 : w0) + f.start;
        int32_t* vo = vout ? vout + f.start : nullptr;
        u64* po = pout ? pout + f.start : nullptr;
        const uint32_t nxt = fi + gridDim.x;
        if (s == 0) {  // one key (or one row): already in row order; the cells stay zero
            for (uint32_t e = tid; e < f.len; e += T) emit(vo, po, e, src[e]);
            if (nxt < nfin) prefetch(nxt);
            continue;
        }
        u64 el[I];
#pragma unroll
        for (int k = 0; k < I; k++) el[k] = nx[k];
        if (nxt < nfin) prefetch(nxt);
        const bool ok = V2 ? finish_counting2<T, I>(el, f.len, kmin + f.klo, s, c32, rows, keys, wsum, vo, po)
                           : finish_counting<T, I, BF>(el, f.len, kmin + f.klo, s, c32, rows, keys, wsum, vo, po);
        if (!ok) {
            if (tid == 0) fb[atomicAdd(&ctr->nfb, 1u)] = f;
            __syncthreads();
            for (uint32_t x = tid; x < kCap / 2; x += T) c32[x] = 0;
            if (tid == 0) wsum[kW] = 0;
        }
        __syncthreads();  // LDS is reused by the next range
    }
}

// The ranked finisher: ceil(s / 8) stable ballot-ranked LDS passes of 8 bits over one
// range (keys wider than kCountBits, or a key on more than kTieMax rows).
__device__ __forceinline__ void finish_ranked(const u64* __restrict__ src, uint32_t len, uint32_t kbase, int s,
                                           int32_t* __restrict__ vo, u64* __restrict__ po, u64* stage,
                                           uint32_t (*wcnt)[256], uint32_t* loff, uint32_t* wsum) {
    constexpr int kW = kFT / 64;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t wbase = (uint32_t)wave * (64 * kFI);
    u64 el[kFI];
    uint32_t dr[kFI];
#pragma unroll
    for (int k = 0; k < kFI; k++) {
        const uint32_t i = wbase + (uint32_t)k * 64 + lane;
        el[k] = src[i < len ? i : len - 1];
    }
    const int npass = (s + 7) >> 3;
    for (int p = 0; p < npass; p++) {
        const int sh = 8 * p;
        const uint32_t wm = (1u << (s - sh < 8 ? s - sh : 8)) - 1;
        for (int x = tid; x < kW * 256; x += kFT) (&wcnt[0][0])[x] = 0;
        __syncthreads();
        rank_items<kFI, false>(el, dr, wbase, len, kbase, sh, wm, 0, wcnt[wave], lane);
        __syncthreads();
        digit_offsets<kW>(wcnt, loff, wsum, tid);
#pragma unroll
        for (int k = 0; k < kFI; k++) {
            if (dr[k] != 0xFFFFFFFFu) {
                const uint32_t d = dr[k] >> 16, r = dr[k] & 0xFFFF;
                stage[loff[d] + wcnt[wave][d] + r] = el[k];
            }
        }
        __syncthreads();
        if (p + 1 < npass) {
#pragma unroll
            for (int k = 0; k < kFI; k++) {
                const uint32_t i = wbase + (uint32_t)k * 64 + lane;
                el[k] = stage[i < len ? i : 0];
            }
            __syncthreads();
        }
    }
#pragma unroll
    for (int k = 0; k < kFI; k++) {
        const uint32_t e = (uint32_t)k * kFT + tid;
        if (e < len) emit(vo, po, e, stage[e]);
    }
    __syncthreads();  // the stage is reused by the next range
}

// A block per range of a ranked list of n ranges (FB = false), or (FB = true, the
// count finisher's rare fallbacks, their number only on the device) a block per CU
// walking the list.
template <bool FB>
__global__ __launch_bounds__(kFT) void k_msd_finish_ranked(const u64* __restrict__ w0, const u64* __restrict__ w1,
                                                           const Fin* __restrict__ fins, const Ctr* __restrict__ ctr,
                                                           uint32_t kmin, int32_t* __restrict__ vout,
                                                           u64* __restrict__ pout) {
    constexpr int kW = kFT / 64;
    __shared__ u64 stage[kCap];
    __shared__ uint32_t wcnt[kW][256];
    __shared__ uint32_t loff[256];
    __shared__ uint32_t wsum[4];
    const uint32_t nf = FB ? ctr->nfb : blockIdx.x + 1;
    for (uint32_t fi = blockIdx.x; fi < nf; fi += gridDim.x) {
        const Fin f = fins[fi];
        finish_ranked(((f.meta >> 8) ? w1 : w0) + f.start, f.len, kmin + f.klo, (int)(f.meta & 0xFF),
                      vout ? vout + f.start : nullptr, pout ? pout + f.start : nullptr, stage, wcnt, loff, wsum);
        if (!FB) break;
    }
}

constexpr uint32_t kFill = 12288;  // rows a finisher range is aimed at (kCap less ~ 30 sigma of 16K)
constexpr int kMaxLevels = 40;

int msd_index_sort(const int* col, uint64_t n, uint32_t kmin, u64 R0, int32_t* vout, u64* pout, hipStream_t st,
                   uint32_t cus) {
    const uint64_t tmax = cdiv(n, kMTile) + n / kCap + 2;  // tiles of any one level
    const uint64_t smax = n / kCap + 2;                     // ranges of any one level past the first
    u64* wb[2] = {(u64*)pool_alloc(n * 8), (u64*)pool_alloc(n * 8)};
    uint8_t* dig = (uint8_t*)pool_alloc(n + 16);
    uint32_t* hist = (uint32_t*)pool_alloc(tmax * 256 * 4);
    uint32_t* tseg = (uint32_t*)pool_alloc(tmax * 4);
    u64* scratch = (u64*)pool_alloc(scan_u32_scratch_elems(tmax * 256) * 8);
    Seg* sl[2] = {(Seg*)pool_alloc(smax * sizeof(Seg)), (Seg*)pool_alloc(smax * sizeof(Seg))};
    Ctr* ctr = (Ctr*)pool_alloc(sizeof(Ctr));
    // The counting finisher: 1024 x 16, the second form (V2) where both outputs are
    // wanted (512 x 32 shapes, with and without per-row guards, measured slower in round 4,
    // profiles/r04_isort_fin_ab.log, and removed in round 6)
    Fin* fl[kMaxLevels] = {};  // finisher lists of each level: counting
    Fin* rl[kMaxLevels] = {};  // ... ranked
    Fin* bl[kMaxLevels] = {};  // ... and the counting finisher's fallbacks
    auto done = [&](int rc) {
        for (int i = 0; i < 2; i++) {
            pool_free_on(wb[i], st);
            pool_free_on(sl[i], st);
        }
        for (Fin* f : fl) pool_free_on(f, st);
        for (Fin* f : rl) pool_free_on(f, st);
        for (Fin* f : bl) pool_free_on(f, st);
        pool_free_on(dig, st);
        pool_free_on(hist, st);
        pool_free_on(tseg, st);
        pool_free_on(scratch, st);
        pool_free_on(ctr, st);
        return rc;
    };
    if (!wb[0] || !wb[1] || !dig || !hist || !tseg || !scratch || !sl[0] || !sl[1] || !ctr)
        return done(set_err(MQ_ENOMEM, "index sort: buffers (%llu rows)", (unsigned long long)n));
    Seg s0{0, (uint32_t)n, 0, (uint32_t)cdiv(n, kMTile), 0};
    if (hipMemcpyAsync(sl[0], &s0, sizeof s0, hipMemcpyHostToDevice, st) != hipSuccess)
        return done(set_err(MQ_EHIP, "index sort: upload"));
    uint32_t nseg = 1, ntile = s0.nt;
    u64 R = R0;         // key range bound of this level's ranges
    uint32_t P = 256;   // digits of this level
    u64 M = ((u64)P << 32) / R;
    for (int level = 0; nseg; level++) {
        if (level >= kMaxLevels) return done(set_err(MQ_EHIP, "index sort: level %d", level));
        const int dst = (level & 1) ^ 1;
        Seg* cur = sl[level & 1];
        Seg* nxt = sl[(level & 1) ^ 1];
        const uint64_t nh = (uint64_t)ntile * P;
        const uint64_t nchild = (uint64_t)nseg * P;
        fl[level] = (Fin*)pool_alloc((nchild < n ? nchild : n) * sizeof(Fin));
        rl[level] = (Fin*)pool_alloc((nchild < n ? nchild : n) * sizeof(Fin));
        bl[level] = (Fin*)pool_alloc((nchild < n ? nchild : n) * sizeof(Fin));
        if (!fl[level] || !rl[level] || !bl[level]) return done(set_err(MQ_ENOMEM, "index sort: range list"));
        hipLaunchKernelGGL(k_tile_seg, dim3(nseg), dim3(256), 0, st, cur, tseg);
        const bool wide = M >> 32 != 0;
        if (level == 0 && wide)
            hipLaunchKernelGGL((k_msd_hist<true, true>), dim3(ntile), dim3(kMT), 0, st, col, nullptr, cur, tseg, kmin,
                               M, P, hist);
        else if (level == 0)
            hipLaunchKernelGGL((k_msd_hist<true, false>), dim3(ntile), dim3(kMT), 0, st, col, nullptr, cur, tseg, kmin,
                               M, P, hist);
        else
            hipLaunchKernelGGL((k_msd_hist<false, true>), dim3(ntile), dim3(kMT), 0, st, nullptr, dig, cur, tseg, kmin,
                               M, P, hist);
        if (hipGetLastError() != hipSuccess) return done(set_err(MQ_EHIP, "index sort: histogram launch"));
        int rc = scan_u32_exclusive_u32(hist, hist, nh, scratch, st);
        if (rc) return done(rc);
        Ctr hc{};
        if (hipMemsetAsync(ctr, 0, sizeof(Ctr), st) != hipSuccess) return done(set_err(MQ_EHIP, "index sort: memset"));
        hipLaunchKernelGGL(k_msd_children, dim3((uint32_t)cdiv(nchild, 256)), dim3(256), 0, st, cur, nseg, hist, M, P,
                           R, dst, fl[level], rl[level], nxt, ctr);
        if (hipGetLastError() != hipSuccess || hipMemcpyAsync(&hc, ctr, sizeof hc, hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess)
            return done(set_err(MQ_EHIP, "index sort: ranges"));
        // the next level: ranges of at most Rn keys, enough digits to bring the largest
        // to about kFill rows if its keys were spread evenly, and each child's keys
        // within the counting finisher's 2^kCountBits where 256 digits can
        const u64 Rn = (1ull << 32) / M + 1;
        u64 Pn = cdiv(hc.maxlen, kFill), Pk = cdiv(Rn, 1ull << kCountBits);  // ... and keys for counting
        if (Pk > Pn) Pn = Pk;
        Pn = Pn < 2 ? 2 : Pn > 256 ? 256 : Pn;
        if (Pn > Rn) Pn = Rn;
        const u64 Mn = hc.nnext ? (Pn << 32) / Rn : 0;
        // digits by one v_mul_hi_u32 where the multipliers fit 32 bits (the usual case)
        const u64* lin = level == 0 ? nullptr : wb[dst ^ 1];
        const int* lcol = level == 0 ? col : nullptr;
        if (!wide && !(Mn >> 32)) {
            if (level == 0)
                hipLaunchKernelGGL((k_msd_scatter<true, false, false>), dim3(ntile), dim3(kMT), 0, st, lcol, lin, cur,
                                   tseg, hist, kmin, M, P, Mn, wb[dst], dig);
            else
                hipLaunchKernelGGL((k_msd_scatter<false, false, false>), dim3(ntile), dim3(kMT), 0, st, lcol, lin,
                                   cur, tseg, hist, kmin, M, P, Mn, wb[dst], dig);
        } else if (level == 0) {
            hipLaunchKernelGGL((k_msd_scatter<true, true, true>), dim3(ntile), dim3(kMT), 0, st, lcol, lin, cur, tseg,
                               hist, kmin, M, P, Mn, wb[dst], dig);
        } else {
            hipLaunchKernelGGL((k_msd_scatter<false, true, true>), dim3(ntile), dim3(kMT), 0, st, lcol, lin, cur,
                               tseg, hist, kmin, M, P, Mn, wb[dst], dig);
        }
        if (hc.nranked)
            hipLaunchKernelGGL(k_msd_finish_ranked<false>, dim3(hc.nranked), dim3(kFT), 0, st, wb[0], wb[1], rl[level],
                               ctr, kmin, vout, pout);
        if (hc.nfin) {
            const uint32_t g = hc.nfin < cus ? hc.nfin : cus;
            if (vout && pout)  // (the second form writes both outputs)
                hipLaunchKernelGGL((k_msd_finish_count<1024, 16, false, true>), dim3(g), dim3(1024), 0, st, wb[0],
                                   wb[1], fl[level], hc.nfin, kmin, vout, pout, bl[level], ctr);
            else
                hipLaunchKernelGGL((k_msd_finish_count<1024, 16, false>), dim3(g), dim3(1024), 0, st, wb[0], wb[1],
                                   fl[level], hc.nfin, kmin, vout, pout, bl[level], ctr);
            hipLaunchKernelGGL(k_msd_finish_ranked<true>, dim3(cus), dim3(kFT), 0, st, wb[0], wb[1], bl[level], ctr,
                               kmin, vout, pout);
        }
        if (hipGetLastError() != hipSuccess) return done(set_err(MQ_EHIP, "index sort: launch"));
        nseg = hc.nnext;
        ntile = hc.tnext;
        R = Rn;
        P = (uint32_t)Pn;
        M = Mn;
    }
    if (hipStreamSynchronize(st) != hipSuccess) return done(set_err(MQ_EHIP, "index sort: sync"));
    return done(MQ_OK);
}

}  // namespace

namespace mqi {

int radix_sort_index(const int* col, uint64_t n, int32_t* values, uint64_t* positions, hipStream_t st) {
    if (n == 0) return MQ_OK;
    DevState* s;
    if (int rc0 = ensure_ready(&s)) return rc0;
    // MQ_INDEX_SORT=lsd4 / lsd: the four-pass LSD sort whatever the range, or the LSD form
    // with the range's passes where the MSD form would run (path-forcing, tests)
    const char* f = getenv("MQ_INDEX_SORT");
    if (f && strcmp(f, "lsd4") == 0) return radix_sort_lsd_index(col, n, 0, 4, values, positions, st);
    void* ws = pool_alloc(mq_scan_workspace_bytes(n));
    mq_agg* agg = (mq_agg*)pool_alloc(sizeof(mq_agg));
    mq_agg h{};
    int rc = (!ws || !agg) ? set_err(MQ_ENOMEM, "index sort: workspace") : MQ_OK;
    if (!rc) rc = mq_reduce(col, n, agg, ws, mq_scan_workspace_bytes(n), st);
    if (!rc && (hipMemcpyAsync(&h, agg, sizeof h, hipMemcpyDeviceToHost, st) != hipSuccess ||
                hipStreamSynchronize(st) != hipSuccess))
        rc = set_err(MQ_EHIP, "index sort: range");
    pool_free(ws);
    pool_free(agg);
    if (rc) return rc;
    const uint32_t kmin = (uint32_t)h.min ^ 0x80000000u;
    const uint32_t span = ((uint32_t)h.max ^ 0x80000000u) - kmin;
    const int b = span ? 32 - __builtin_clz(span) : 0;
    // MQ_INDEX_MSD_MIN: the row count from which the MSD form is used (tests force it;
    // from 2^24 rows it is the faster form, tools/index_sweep.sh)
    const char* mm = getenv("MQ_INDEX_MSD_MIN");
    const uint64_t msd_min = mm ? strtoull(mm, nullptr, 10) : (1ull << 24);
    if (b > 24 && n >= msd_min && !(f && strcmp(f, "lsd") == 0))
        return msd_index_sort(col, n, kmin, (u64)span + 1, values, reinterpret_cast<u64*>(positions), st, s->cus);
    return radix_sort_lsd_index(col, n, kmin, b ? (b + 7) / 8 : 1, values, positions, st);
}

}  // namespace mqi
