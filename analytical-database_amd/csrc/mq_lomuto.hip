// mq_lomuto.hip — the reference's exact quicksort order on gfx950 (src/index.c:25-46).
//
// quicksort(low, high) partitions [low, high] around values[high] (Lomuto) and
// recurses on both sides; disjoint ranges do not interact, so every range of one
// recursion depth can be partitioned at once. One partition of a range with c values
// below the pivot, restated without its sequential loop:
//   * the k-th value below the pivot (index j_k, in index order) is swapped with
//     index low + k, so it ends at low + k: the "<" side is a stable compaction;
//   * a value >= the pivot moves only when it sits at low + k as the k-th "<" value
//     is found (j_k is beyond it); it then jumps to j_k. From index x it therefore
//     follows x -> J[x] -> J[J[x]] ... (J[low + k] = j_k) until the index leaves
//     [low, low + c). Every step of every chain is one "<" value found while the
//     ">=" block is not empty, so one partition's chains total at most c steps;
//   * the final swap puts the pivot at low + c and the value that ended there at high.
// A range whose values all equal its pivot would recurse one element per level
// (O(n) depth); its outcome has a closed form: the last value first, then the others
// in order (by induction over the partitions), so it finishes at once.
//
// Two phases:
//   * large ranges (more than `small` indexes) are partitioned level by level over
//     items of kItem indexes aligned to kItem (a block per item, 8 indexes per lane):
//     count "<" / ">" per item, one scan over the items, the children, the back map R
//     (k_ld_less), and the placement, which pushes the "<" values and the pivot and
//     pulls every index of the ">=" side by walking the chains backwards. Only the
//     indexes of large ranges are read; a pivot, a child of one index and an all-equal
//     range go straight to the output; a child of 2..small indexes joins the small
//     list. A walk longer than kChainCap flags its range: R is pointer-doubled over
//     that range and the range placed again.
//   * each small range is finished by one wave with its values in LDS (one buffer,
//     updated in place from registers): the same partition with a ballot-ranked "<"
//     side and forward chains walked in LDS, a stack of the sub-ranges above kTiny, and
//     sub-ranges of 2..kTiny indexes run through the reference's own sequential
//     partition by one lane each.
// Values and row ids move as (int32, u32) pairs; the host reads one small record per
// level. DESIGN.md §3.7 has the cost.

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "mq_common.h"
#include "mq_device.h"

namespace {

using namespace mqi;

constexpr int kTPB = 256;
constexpr uint32_t kItem = 2048;   // indexes per item: 256 lanes x 8
constexpr uint32_t kEq = 0xFFFFFFFFu;

// chain steps walked before pointer doubling takes over (MQ_LQ_CAP)
constexpr int kChainCap = 512;
constexpr int kMaxJumps = 64;      // doubling steps per level (2^64 > any chain)
constexpr int kJumpBatch = 16;     // doubling steps launched per host check (4: 70.5 ms, 8: 69.6, 16: 68.6)
// Levels of at most kSmallItems items (late levels: few rows, where one walk of up to
// kChainCap steps set each level's time) walk at most kChainCapSmall steps before
// doubling: 70.5 -> 69.3 ms (with 8 steps a check, 68.0; profiles/r04_lomuto_knobs2.log)
constexpr int kChainCapSmall = 64;
constexpr uint64_t kSmallItems = 2048;

struct LSeg {
    uint32_t lo, hi;
};

__device__ __forceinline__ uint32_t lane_rank(uint64_t mask) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

// The range of an item and the first index of the item's aligned chunk.
struct ItemAt {
    uint32_t r, base;
    LSeg g;
};
__device__ __forceinline__ ItemAt item_at(uint32_t item, const uint32_t* __restrict__ imap,
                                          const LSeg* __restrict__ seg, const uint32_t* __restrict__ ioff) {
    ItemAt a;
    a.r = imap[item];
    a.g = seg[a.r];
    a.base = (a.g.lo / kItem + (item - ioff[a.r])) * kItem;
    return a;
}

__device__ __forceinline__ uint32_t items_of(uint32_t lo, uint32_t hi) { return hi / kItem - lo / kItem + 1; }

// the last k < F with off[k] <= b (off ascending, off[0] = 0)
__device__ __forceinline__ uint32_t upper_index(const uint32_t* __restrict__ off, uint32_t F, uint32_t b) {
    uint32_t lo = 0, hi = F;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (off[mid] <= b) lo = mid;
        else hi = mid;
    }
    return lo;
}

// the 8 values of this lane (indexes i0 .. i0+7 within [lo, hi]; others read as 0)
template <typename T>
__device__ __forceinline__ void load8(const T* __restrict__ a, uint32_t i0, uint32_t lo, uint32_t hi, T v[8]) {
    if (i0 >= lo && i0 + 7 <= hi) {
        const int4 x = *reinterpret_cast<const int4*>(a + i0);
        const int4 y = *reinterpret_cast<const int4*>(a + i0 + 4);
        v[0] = (T)x.x, v[1] = (T)x.y, v[2] = (T)x.z, v[3] = (T)x.w;
        v[4] = (T)y.x, v[5] = (T)y.y, v[6] = (T)y.z, v[7] = (T)y.w;
    } else {
#pragma unroll
        for (int k = 0; k < 8; k++) v[k] = (i0 + k >= lo && i0 + k <= hi) ? a[i0 + k] : (T)0;
    }
}

// The less-map and placement take an item's indexes round-major: index base + k * 256
// + tid in round k, so a wave's lanes hold consecutive indexes in every round and the
// swap chains of consecutive indexes read nearby J entries at each step (J is
// monotone): at p = 1/2 a wave's first chain step touches ≈ 8 lines instead of ≈ 32
// with 8 consecutive indexes per lane. rank[k] = r0 + the "<" indexes of the item
// before this lane's round-k index.
__device__ __forceinline__ void round_ranks(const bool (&lt)[8], uint32_t r0, uint32_t (&rank)[8],
                                            uint32_t (*s_cnt)[kTPB / 64]) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint64_t m[8];
#pragma unroll
    for (int k = 0; k < 8; k++) {
        m[k] = __ballot(lt[k]);
        if (lane == 0) s_cnt[k][w] = (uint32_t)__popcll(m[k]);
    }
    __syncthreads();
    uint32_t run = r0;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        uint32_t before = 0, tot = 0;
#pragma unroll
        for (int w2 = 0; w2 < kTPB / 64; w2++) {
            const uint32_t c = s_cnt[k][w2];
            before += w2 < w ? c : 0u;
            tot += c;
        }
        rank[k] = run + before + lane_rank(m[k]);
        run += tot;
    }
}

__global__ __launch_bounds__(kTPB) void k_ld_init(const int32_t* __restrict__ col, uint64_t n, int32_t* __restrict__ V,
                                                  uint32_t* __restrict__ P) {
    const uint64_t stride = (uint64_t)gridDim.x * kTPB;
    for (uint64_t i = (uint64_t)blockIdx.x * kTPB + threadIdx.x; i < n; i += stride) {
        V[i] = col[i];
        P[i] = (uint32_t)i;
    }
}

// per item: its range (the last r with ioff[r] <= item)
__global__ __launch_bounds__(kTPB) void k_ld_imap(const uint32_t* __restrict__ ioff, uint32_t S, uint32_t NI,
                                                  uint32_t* __restrict__ imap) {
    for (uint32_t b = blockIdx.x * kTPB + threadIdx.x; b < NI; b += gridDim.x * kTPB) imap[b] = upper_index(ioff, S, b);
}

// per item: ("<" pivot) | (">" pivot) << 32 over its indexes, the pivot excluded; cnt[NI] = 0
__global__ __launch_bounds__(kTPB) void k_ld_count(const int32_t* __restrict__ V, const LSeg* __restrict__ seg,
                                                   const uint32_t* __restrict__ ioff, const uint32_t* __restrict__ imap,
                                                   uint32_t NI, unsigned long long* __restrict__ cnt,
                                                   unsigned long long* __restrict__ ctl,
                                                   unsigned int* __restrict__ chg) {
    __shared__ unsigned long long s_acc;
    const uint32_t item = blockIdx.x;
    if (threadIdx.x == 0) s_acc = 0;
    if (item == 0) {  // this level's control words: next-level counter, flagged count, doubling flags
        if (threadIdx.x == 0) {
            cnt[NI] = 0;
            ctl[0] = 0;
            reinterpret_cast<unsigned int*>(ctl + 1)[1] = 0;
        }
        if (threadIdx.x < kMaxJumps) chg[threadIdx.x] = 0;
    }
    const ItemAt a = item_at(item, imap, seg, ioff);
    const int32_t piv = V[a.g.hi];
    const uint32_t i0 = a.base + threadIdx.x * 8;
    int32_t v[8];
    load8(V, i0, a.g.lo, a.g.hi, v);
    uint32_t lt = 0, gt = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const uint32_t i = i0 + k;
        const bool ok = i >= a.g.lo && i < a.g.hi;
        lt += ok && v[k] < piv;
        gt += ok && v[k] > piv;
    }
    unsigned long long x = lt | ((unsigned long long)gt << 32);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) atomicAdd(&s_acc, x);
    __syncthreads();
    if (threadIdx.x == 0) cnt[item] = s_acc;
}

// Per large range: c, all-equal, and its children: large ones (more than `small`
// indexes) appended to the next level with their items (one packed atomic, so ranges
// and their items keep one order), small ones (2..small) to the small list.
__global__ __launch_bounds__(kTPB) void k_ld_children(const LSeg* __restrict__ seg, const uint32_t* __restrict__ ioff,
                                                      uint32_t S, const unsigned long long* __restrict__ ex,
                                                      uint32_t small, uint32_t dbuf, uint32_t* __restrict__ segc,
                                                      uint32_t* __restrict__ segflag,
                                                      LSeg* __restrict__ seg_next, uint32_t* __restrict__ ioff_next,
                                                      unsigned long long* __restrict__ ctr, uint2* __restrict__ slist,
                                                      unsigned int* __restrict__ nsmall) {
    for (uint32_t r = blockIdx.x * kTPB + threadIdx.x; r < S; r += gridDim.x * kTPB) {
        const LSeg g = seg[r];
        const uint32_t f = ioff[r];
        const unsigned long long tot = ex[f + items_of(g.lo, g.hi)] - ex[f];
        const uint32_t c = (uint32_t)tot, gt = (uint32_t)(tot >> 32);
        const bool eq = c == 0 && gt == 0;
        segc[r] = eq ? kEq : c;
        segflag[r] = 0;
        if (eq) continue;
        const LSeg ch[2] = {{g.lo, g.lo + c - 1}, {g.lo + c + 1, g.hi}};
        const uint32_t sz[2] = {c, g.hi - g.lo - c};
        for (int k = 0; k < 2; k++) {
            if (sz[k] > small) {
                const uint32_t ni = items_of(ch[k].lo, ch[k].hi);
                const unsigned long long old = atomicAdd(ctr, (1ull << 40) | ni);
                const uint32_t idx = (uint32_t)(old >> 40);
                seg_next[idx] = ch[k];
                ioff_next[idx] = (uint32_t)(old & ((1ull << 40) - 1));
            } else if (sz[k] >= 2) {
                const unsigned int at = atomicAdd(nsmall, 1u);
                slist[at] = make_uint2(ch[k].lo, ch[k].hi | (dbuf << 31));
            }
        }
    }
}

// The back map R of one level, per index x of a large range (the pivot excluded):
// kGe for a value >= the pivot; for a "<" value, the index it was swapped with,
// lo + rank(x) (the front of the ">=" block when x was reached), with kDone set when
// that index holds a value >= the pivot. The value that ends at an index y of the
// ">=" side is found by walking back from y: y -> R[y] -> ... until an index whose own
// value is >= the pivot (it never moved before being swapped out, and each swap moves
// the block's front). Walking back contracts (R[x] - lo ≈ p (x - lo)), so consecutive
// indexes read nearby entries at every step, and every store of the placement goes to
// consecutive indexes (the forward walk, from the ">=" values to their destinations,
// expands: its loads and stores scattered).
constexpr uint32_t kGe = 0xFFFFFFFFu, kDone = 0x80000000u;

// blocked: a lane's 8 consecutive indexes (two 16-byte loads, two 16-byte stores);
// the map has no chains, so the placement's round-major order buys nothing here
__global__ __launch_bounds__(kTPB) void k_ld_less(const int32_t* __restrict__ V, const LSeg* __restrict__ seg,
                                                  const uint32_t* __restrict__ ioff, const uint32_t* __restrict__ imap,
                                                  const uint32_t* __restrict__ segc,
                                                  const unsigned long long* __restrict__ ex, uint32_t* __restrict__ R) {
    __shared__ uint32_t sh[kTPB / 64];
    const uint32_t item = blockIdx.x;
    const ItemAt a = item_at(item, imap, seg, ioff);
    if (segc[a.r] == kEq) return;
    const uint32_t lo = a.g.lo, hi = a.g.hi;
    const int32_t piv = V[hi];
    const uint32_t i0 = a.base + threadIdx.x * 8;
    int32_t v[8];
    load8(V, i0, lo, hi, v);
    uint32_t m = 0, nl = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const bool lt = i0 + k >= lo && i0 + k < hi && v[k] < piv;
        m |= (uint32_t)lt << k;
        nl += lt;
    }
    // exclusive prefix of nl over the block's lanes
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t inc = nl;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(inc, o, 64);
        if (lane >= o) inc += y;
    }
    if (lane == 63) sh[w] = inc;
    __syncthreads();
    uint32_t rank = inc - nl + ((uint32_t)ex[item] - (uint32_t)ex[ioff[a.r]]);
    for (int k = 0; k < w; k++) rank += sh[k];
    uint32_t t[8];
#pragma unroll
    for (int k = 0; k < 8; k++) {
        t[k] = lo + rank;
        rank += m >> k & 1;
    }
    int32_t vt[8];
#pragma unroll
    for (int k = 0; k < 8; k++) vt[k] = (m >> k & 1) ? V[t[k]] : 0;
    uint32_t out[8];
#pragma unroll
    for (int k = 0; k < 8; k++) out[k] = (m >> k & 1) ? (t[k] | (vt[k] < piv ? 0u : kDone)) : kGe;
    if (i0 >= lo && i0 + 7 < hi) {
        *reinterpret_cast<uint4*>(R + i0) = make_uint4(out[0], out[1], out[2], out[3]);
        *reinterpret_cast<uint4*>(R + i0 + 4) = make_uint4(out[4], out[5], out[6], out[7]);
    } else {
#pragma unroll
        for (int k = 0; k < 8; k++)
            if (i0 + k >= lo && i0 + k < hi) R[i0 + k] = out[k];
    }
}

// Placement of one item's indexes, as sources and as destinations:
//  * a "<" value goes to lo + rank (stable compaction); the pivot to lo + c; an
//    all-equal range in closed form (the last value first, then the others in order);
//  * index y of the ">=" side [lo + c + 1, hi] takes the value found by walking back
//    from y (from lo + c for y = hi: the final swap with the pivot).
// Finals (the pivot, a child of one index, an all-equal range) go to the output, the
// rest to the other buffer. A lane's 8 walks go together (loads in flight at once).
// USE_F = false: a walk longer than cap flags its range (listed once in flist) and
// leaves the index to the second placement; USE_F = true (after the doubling): block
// b places item b - foff[k] of flagged range flist[k].
template <bool USE_F>
__global__ __launch_bounds__(kTPB) void k_ld_final(const int32_t* __restrict__ V, const uint32_t* __restrict__ P,
                                                   const LSeg* __restrict__ seg, const uint32_t* __restrict__ ioff,
                                                   const uint32_t* __restrict__ imap, const uint32_t* __restrict__ segc,
                                                   const unsigned long long* __restrict__ ex,
                                                   const uint32_t* __restrict__ R, int32_t* __restrict__ Vd,
                                                   uint32_t* __restrict__ Pd, int32_t* __restrict__ vout,
                                                   unsigned long long* __restrict__ pout, uint32_t* __restrict__ segflag,
                                                   uint32_t* __restrict__ flist, unsigned int* __restrict__ nflag,
                                                   const uint32_t* __restrict__ foff, uint32_t F, int cap) {
    __shared__ uint32_t s_cnt[8][kTPB / 64];
    uint32_t item;
    ItemAt a;
    if (USE_F) {
        const uint32_t k = upper_index(foff, F, blockIdx.x);
        a.r = flist[k];
        item = ioff[a.r] + (blockIdx.x - foff[k]);
        a.g = seg[a.r];
        a.base = (a.g.lo / kItem + (blockIdx.x - foff[k])) * kItem;
    } else {
        item = blockIdx.x;
        a = item_at(item, imap, seg, ioff);
    }
    const uint32_t lo = a.g.lo, hi = a.g.hi, c = segc[a.r];
    const int32_t piv = V[hi];
    int32_t v[8];
    uint32_t p[8];
    bool lt[8];
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const uint32_t i = a.base + k * kTPB + threadIdx.x;
        const bool ok = i >= lo && i <= hi;
        v[k] = ok ? V[i] : 0;
        p[k] = ok ? P[i] : 0u;
        lt[k] = ok && c != kEq && i < hi && v[k] < piv;
    }
    uint32_t rank[8];
    round_ranks(lt, (uint32_t)ex[item] - (uint32_t)ex[ioff[a.r]], rank, s_cnt);
    const bool lfin = c == 1, rfin = c != kEq && hi - lo - c == 1;
    // sources: "<" values, the pivot, all-equal ranges
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const uint32_t i = a.base + k * kTPB + threadIdx.x;
        if (i < lo || i > hi) continue;
        uint32_t q;
        bool fin;
        if (c == kEq) {
            q = i == hi ? lo : i + 1;
            fin = true;
        } else if (i == hi) {
            q = lo + c;
            fin = true;
        } else if (lt[k]) {
            q = lo + rank[k];
            fin = lfin;
        } else {
            continue;
        }
        if (fin) {
            if (vout) vout[q] = v[k];
            if (pout) pout[q] = p[k];
        } else {
            Vd[q] = v[k];
            Pd[q] = p[k];
        }
    }
    if (c == kEq) return;
    // destinations: the ">=" side [lo + c + 1, hi], walked back
    uint32_t x[8], r[8], walk = 0, dst = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const uint32_t y = a.base + k * kTPB + threadIdx.x;
        x[k] = y;
        r[k] = kGe;
        if (y < lo || y > hi || y - lo <= c) continue;
        dst |= 1u << k;
        if (y == hi) x[k] = lo + c;
        if (y == hi || lt[k]) walk |= 1u << k;  // a ">=" value at y < hi stays
    }
#pragma unroll
    for (int k = 0; k < 8; k++)
        if (walk >> k & 1) r[k] = R[x[k]];
    for (int steps = 0;; steps++) {
        // r[k]: the back map at x[k]; kGe: x[k] holds its own value; kDone: the next index does
#pragma unroll
        for (int k = 0; k < 8; k++) {
            if (!(walk >> k & 1)) continue;
            if (r[k] == kGe) {
                walk &= ~(1u << k);
            } else {
                x[k] = r[k] & ~kDone;
                if (r[k] & kDone) walk &= ~(1u << k);
            }
        }
        if (!walk || (!USE_F && steps >= cap)) break;
#pragma unroll
        for (int k = 0; k < 8; k++)
            if (walk >> k & 1) r[k] = R[x[k]];
    }
    if (!USE_F && walk) {  // long walks: placed after the doubling
        dst &= ~walk;
        if (atomicExch(&segflag[a.r], 1u) == 0u) flist[atomicAdd(nflag, 1u)] = a.r;
    }
#pragma unroll
    for (int k = 0; k < 8; k++) {
        if (!(dst >> k & 1)) continue;
        const uint32_t y = a.base + k * kTPB + threadIdx.x;
        const bool own = x[k] == y;
        const int32_t val = own ? v[k] : V[x[k]];
        const uint32_t row = own ? p[k] : P[x[k]];
        if (rfin) {
            if (vout) vout[y] = val;
            if (pout) pout[y] = row;
        } else {
            Vd[y] = val;
            Pd[y] = row;
        }
    }
}

// flagged range k: its items (fi); entry F is 0
__global__ __launch_bounds__(kTPB) void k_ld_fitems(const LSeg* __restrict__ seg, const uint32_t* __restrict__ flist,
                                                    uint32_t F, uint32_t* __restrict__ fi) {
    for (uint32_t k = blockIdx.x * kTPB + threadIdx.x; k <= F; k += gridDim.x * kTPB)
        fi[k] = k == F ? 0u : items_of(seg[flist[k]].lo, seg[flist[k]].hi);
}

// Doubling step `it` of the back map R over the flagged ranges: block b takes item
// b - foff[k] of range flist[k]; an entry not yet at a ">=" index takes its target's
// entry. chg[it] records a change; a step whose predecessor changed nothing returns
// at once, so the host launches steps in batches and reads one flag per batch.
__global__ __launch_bounds__(kTPB) void k_ld_jump(const LSeg* __restrict__ seg, const uint32_t* __restrict__ flist,
                                                  const uint32_t* __restrict__ foff, uint32_t F, uint32_t* R,
                                                  unsigned int* __restrict__ chg, int it) {
    if (it > 0 && chg[it - 1] == 0u) return;
    unsigned int* changed = chg + it;
    const uint32_t k = upper_index(foff, F, blockIdx.x);
    const LSeg g = seg[flist[k]];
    const uint32_t base = (g.lo / kItem + (blockIdx.x - foff[k])) * kItem;
    // a lane's 8 entries are loaded, then their 8 targets, then stored: two round
    // trips per step, not two per entry
    uint32_t t[8];
    bool act[8];
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const uint32_t i = base + k * kTPB + threadIdx.x;
        t[k] = i >= g.lo && i < g.hi ? R[i] : kGe;
        act[k] = t[k] != kGe && !(t[k] & kDone);  // t holds a "<" value: a pointer
    }
    uint32_t u[8];
#pragma unroll
    for (int k = 0; k < 8; k++) u[k] = act[k] ? R[t[k]] : 0u;
    unsigned int any = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        if (act[k] && u[k] != t[k]) {
            R[base + k * kTPB + threadIdx.x] = u[k];
            any = 1;
        }
    }
    if (__ballot(any) && (threadIdx.x & 63) == 0) atomicOr(changed, 1u);
}

// ---------------------------------------------------------------------------
// Small ranges: one wave each, values in LDS. A (l, h, buffer) record packs into
// 32 bits as l | h << 12 | buffer << 24 (T <= 4096).
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t rec(int l, int h, int s) { return (uint32_t)l | (uint32_t)h << 12 | (uint32_t)s << 24; }

template <int T, int kTiny>
__global__ __launch_bounds__(64) void k_ld_small(const int32_t* __restrict__ V0, const uint32_t* __restrict__ P0,
                                                 const int32_t* __restrict__ V1, const uint32_t* __restrict__ P1,
                                                 const uint2* __restrict__ list, uint32_t count,
                                                 int32_t* __restrict__ vout, unsigned long long* __restrict__ pout) {
    static_assert(T <= 4096 && T >= 64 && T % 64 == 0, "record packing");
    constexpr int R = T / 64;       // a sub-range's indexes per lane, held in registers while it moves
    // One buffer, updated in place: a partition first reads its whole sub-range into
    // registers, then writes every value to its destination (12 KB of LDS a wave at
    // T = 1024 instead of 19 KB with two buffers: 13 waves per CU instead of 8).
    __shared__ int32_t av[T];
    __shared__ uint16_t ai[T];      // index within the range at the start (the row is read at the end)
    __shared__ uint16_t J[T];
    __shared__ uint32_t tiny[T / 2];
    __shared__ uint32_t stk[T / kTiny + 8];
    __shared__ uint16_t lstk[64][kTiny];
    const int lane = threadIdx.x;
    for (uint32_t r = blockIdx.x; r < count; r += gridDim.x) {
        const uint2 e = list[r];
        const uint32_t lo = e.x, hi = e.y & 0x7FFFFFFFu;
        const bool b1 = (e.y >> 31) != 0;
        const int32_t* Vs = b1 ? V1 : V0;
        const uint32_t* Ps = b1 ? P1 : P0;
        const int m = (int)(hi - lo) + 1;
        for (int k = lane; k < m; k += 64) {
            av[k] = Vs[lo + k];
            ai[k] = (uint16_t)k;
        }
        int sp = 0, nt = 0;
        if (m > kTiny) {
            if (lane == 0) stk[0] = rec(0, m - 1, 0);
            sp = 1;
        } else if (m >= 2) {
            if (lane == 0) tiny[0] = rec(0, m - 1, 0);
            nt = 1;
        }
        __syncthreads();
        while (sp > 0) {
            const uint32_t t = stk[--sp];
            const int l = t & 0xFFF, h = (t >> 12) & 0xFFF;
            const int32_t piv = av[h];
            uint32_t carry = 0;
            bool anygt = false;
            for (int base = l; base < h; base += 64) {
                const int i = base + lane;
                const bool ok = i < h;
                const int32_t v = ok ? av[i] : 0;
                const bool lt = ok && v < piv;
                anygt |= ok && v > piv;
                const uint64_t mk = __ballot(lt);
                if (lt) J[l + carry + lane_rank(mk)] = (uint16_t)i;
                carry += (uint32_t)__popcll(mk);
            }
            const int c = (int)carry;
            const bool eq = c == 0 && __ballot(anygt) == 0;
            const int rsz = h - l - c;  // the right child's size
            int32_t rv[R];
            uint32_t rx[R];
#pragma unroll
            for (int k = 0; k < R; k++) {
                const int i = l + k * 64 + lane;
                if (l + k * 64 <= h) {
                    rv[k] = i <= h ? av[i] : 0;
                    rx[k] = i <= h ? ai[i] : 0u;
                }
            }
            __syncthreads();  // J complete; every value of the sub-range read
            carry = 0;
#pragma unroll
            for (int k = 0; k < R; k++) {
                if (l + k * 64 > h) break;
                const int i = l + k * 64 + lane;
                const bool ok = i <= h;
                const bool lt = !eq && ok && i != h && rv[k] < piv;
                const uint64_t mk = __ballot(lt);
                if (ok) {
                    int q;
                    if (eq) {
                        q = i == h ? l : i + 1;
                    } else if (i == h) {
                        q = l + c;
                    } else if (lt) {
                        q = l + (int)(carry + lane_rank(mk));
                    } else {
                        q = i;
                        while (q - l < c) q = J[q];
                        if (q == l + c) q = h;
                    }
                    av[q] = rv[k];
                    ai[q] = (uint16_t)rx[k];
                }
                carry += (uint32_t)__popcll(mk);
            }
            if (!eq) {
                // children: the larger pushed first, so the stack stays shallow
                int cl[2] = {l, l + c + 1}, ch[2] = {l + c - 1, h}, cs[2] = {c, rsz};
                const int big = cs[0] >= cs[1] ? 0 : 1;
                for (int k = 0; k < 2; k++) {
                    const int j = k == 0 ? big : big ^ 1;
                    if (cs[j] > kTiny) {
                        if (lane == 0) stk[sp] = rec(cl[j], ch[j], 0);
                        sp++;
                    } else if (cs[j] >= 2) {
                        if (lane == 0) tiny[nt] = rec(cl[j], ch[j], 0);
                        nt++;
                    }
                }
            }
            __syncthreads();
        }
        // sub-ranges of 2..kTiny indexes: the reference's partition, one lane each, in place
        for (int tt = lane; tt < nt; tt += 64) {
            const uint32_t t = tiny[tt];
            const int l0 = t & 0xFFF, h0 = (t >> 12) & 0xFFF;
            uint16_t* st = lstk[lane];
            int top = 0;
            st[top++] = (uint16_t)(0 | (h0 - l0) << 8);
            while (top) {
                const uint16_t w = st[--top];
                const int lo2 = l0 + (w & 0xFF), hi2 = l0 + (w >> 8);
                const int32_t piv = av[hi2];
                int i = lo2 - 1;
                for (int j = lo2; j < hi2; j++) {
                    if (av[j] < piv) {
                        i++;
                        const int32_t tv = av[i];
                        av[i] = av[j];
                        av[j] = tv;
                        const uint16_t tx = ai[i];
                        ai[i] = ai[j];
                        ai[j] = tx;
                    }
                }
                {
                    const int32_t tv = av[i + 1];
                    av[i + 1] = av[hi2];
                    av[hi2] = tv;
                    const uint16_t tx = ai[i + 1];
                    ai[i + 1] = ai[hi2];
                    ai[hi2] = tx;
                }
                const int pv = i + 1;
                if (pv - 1 > lo2) st[top++] = (uint16_t)((lo2 - l0) | (pv - 1 - l0) << 8);
                if (hi2 > pv + 1) st[top++] = (uint16_t)((pv + 1 - l0) | (hi2 - l0) << 8);
            }
        }
        __syncthreads();
        for (int k = lane; k < m; k += 64) {
            if (vout) vout[lo + k] = av[k];
            if (pout) pout[lo + k] = Ps[lo + ai[k]];
        }
        __syncthreads();
    }
}

struct LdBufs {
    void* blk[24];
    int nb = 0, want = 0;
    hipStream_t st = nullptr;  // the sort's stream: buffers go back in its order (error paths included)
    ~LdBufs() {
        for (int i = 0; i < nb; i++) pool_free_on(blk[i], st);
    }
    template <typename T>
    T* get(size_t count) {
        want++;
        void* p = pool_alloc((count ? count : 1) * sizeof(T));
        if (p) blk[nb++] = p;
        return static_cast<T*>(p);
    }
};

int small_threshold() {
    static const int t = [] {
        const char* e = getenv("MQ_LQ_SMALL");
        const int v = e ? atoi(e) : 1024;
        return v == 256 || v == 512 || v == 2048 ? v : 1024;
    }();
    return t;
}

int tiny_threshold() {
    static const int t = [] {
        const char* e = getenv("MQ_LQ_TINY");
        const int v = e ? atoi(e) : 16;
        return v == 8 || v == 32 ? v : 16;
    }();
    return t;
}

template <int T>
void launch_small_t(uint32_t grid, hipStream_t st, const int32_t* V0, const uint32_t* P0, const int32_t* V1,
                    const uint32_t* P1, const uint2* list, uint32_t count, int32_t* vout, unsigned long long* pout) {
    const int tiny = tiny_threshold();
    if (tiny == 8)
        hipLaunchKernelGGL((k_ld_small<T, 8>), dim3(grid), dim3(64), 0, st, V0, P0, V1, P1, list, count, vout, pout);
    else if (tiny == 32)
        hipLaunchKernelGGL((k_ld_small<T, 32>), dim3(grid), dim3(64), 0, st, V0, P0, V1, P1, list, count, vout, pout);
    else
        hipLaunchKernelGGL((k_ld_small<T, 16>), dim3(grid), dim3(64), 0, st, V0, P0, V1, P1, list, count, vout, pout);
}

int launch_small(int T, uint32_t grid, hipStream_t st, const int32_t* V0, const uint32_t* P0, const int32_t* V1,
                 const uint32_t* P1, const uint2* list, uint32_t count, int32_t* vout, unsigned long long* pout) {
    if (T == 256)
        launch_small_t<256>(grid, st, V0, P0, V1, P1, list, count, vout, pout);
    else if (T == 512)
        launch_small_t<512>(grid, st, V0, P0, V1, P1, list, count, vout, pout);
    else if (T == 2048)
        launch_small_t<2048>(grid, st, V0, P0, V1, P1, list, count, vout, pout);
    else
        launch_small_t<1024>(grid, st, V0, P0, V1, P1, list, count, vout, pout);
    LAUNCHCHK("k_ld_small");
    return MQ_OK;
}

}  // namespace

namespace mqi {

int lomuto_sort(const int32_t* col, uint64_t n, int32_t* vout, uint64_t* pout64, hipStream_t st, const DevState* s) {
    const uint32_t T = (uint32_t)small_threshold();
    const uint64_t smax = n / (T + 1) + 2;            // large ranges are disjoint, > T indexes each
    const uint64_t nimax = n / kItem + 2 * smax + 2;  // items of one level
    unsigned long long* pout = reinterpret_cast<unsigned long long*>(pout64);
    LdBufs b;
    b.st = st;
    int32_t* V[2] = {b.get<int32_t>(n), b.get<int32_t>(n)};
    uint32_t* P[2] = {b.get<uint32_t>(n), b.get<uint32_t>(n)};
    uint32_t* R = b.get<uint32_t>(n);  // the back map of the current level
    LSeg* seg[2] = {b.get<LSeg>(smax), b.get<LSeg>(smax)};
    uint32_t* ioff[2] = {b.get<uint32_t>(smax), b.get<uint32_t>(smax)};
    uint32_t* segc = b.get<uint32_t>(smax);
    uint32_t* segflag = b.get<uint32_t>(smax);  // ranges with a long chain, listed once in flist
    uint32_t* flist = b.get<uint32_t>(smax);
    uint32_t* fi = b.get<uint32_t>(smax + 1);    // per flagged range: its items, then their prefix
    uint32_t* imap = b.get<uint32_t>(nimax);
    unsigned long long* cnt = b.get<unsigned long long>(nimax + 1);
    unsigned long long* scratch = b.get<unsigned long long>(scan_u32_scratch_elems(nimax + 1));
    uint2* slist = b.get<uint2>(n / 2 + 2);
    unsigned long long* ctl = b.get<unsigned long long>(4 + kMaxJumps / 2);  // see ctl32, chg
    if (b.nb != b.want) return set_err(MQ_ENOMEM, "mq_index_build_lomuto: device allocation failed");
    // ctl[0]: next level's ranges << 40 | items; ctl32: [0] small ranges so far, [1] flagged
    // ranges of this level; chg: one flag per doubling step of this level
    unsigned int* ctl32 = reinterpret_cast<unsigned int*>(ctl + 1);
    unsigned int* chg = reinterpret_cast<unsigned int*>(ctl + 4);
    static const bool stats = getenv("MQ_LQ_STATS") != nullptr;     // per-level diagnostics (stderr)
    static const int cap = getenv("MQ_LQ_CAP") ? atoi(getenv("MQ_LQ_CAP")) : kChainCap;
    // A/B knobs (round 4): doubling steps per host check, and a walk limit for levels of
    // at most MQ_LQ_SMALL_ITEMS items (late levels: a few rows, one long walk)
    static const int jbatch = getenv("MQ_LQ_JUMPS") ? atoi(getenv("MQ_LQ_JUMPS")) : kJumpBatch;
    static const int cap_small = getenv("MQ_LQ_CAP_SMALL") ? atoi(getenv("MQ_LQ_CAP_SMALL")) : kChainCapSmall;
    static const uint64_t small_items =
        getenv("MQ_LQ_SMALL_ITEMS") ? strtoull(getenv("MQ_LQ_SMALL_ITEMS"), nullptr, 10) : kSmallItems;
    HIPCHK(hipMemsetAsync(ctl, 0, 32, st));  // (ctl32[0] is never reset after this)
    hipLaunchKernelGGL(k_ld_init, dim3(stream_grid(s, n)), dim3(kTPB), 0, st, col, n, V[0], P[0]);
    LAUNCHCHK("k_ld_init");
    uint64_t S = 0, NI = 0;
    uint32_t nsmall = 0;
    if (n > T) {
        const LSeg root{0u, (uint32_t)(n - 1)};
        const uint32_t z = 0;
        HIPCHK(hipMemcpyAsync(seg[0], &root, sizeof root, hipMemcpyHostToDevice, st));
        HIPCHK(hipMemcpyAsync(ioff[0], &z, 4, hipMemcpyHostToDevice, st));
        S = 1;
        NI = (n - 1) / kItem + 1;
    } else {
        const uint2 one = make_uint2(0u, (uint32_t)(n - 1));
        HIPCHK(hipMemcpyAsync(slist, &one, sizeof one, hipMemcpyHostToDevice, st));
        nsmall = 1;
    }
    int cur = 0, level = 0;
    while (S) {
        const int d = cur ^ 1;
        hipLaunchKernelGGL(k_ld_imap, dim3(stream_grid(s, NI)), dim3(kTPB), 0, st, ioff[cur], (uint32_t)S,
                           (uint32_t)NI, imap);
        LAUNCHCHK("k_ld_imap");
        hipLaunchKernelGGL(k_ld_count, dim3((uint32_t)NI), dim3(kTPB), 0, st, V[cur], seg[cur], ioff[cur], imap,
                           (uint32_t)NI, cnt, ctl, chg);
        LAUNCHCHK("k_ld_count");
        int rc = scan_u64_exclusive(cnt, cnt, NI + 1, scratch, st);
        if (rc) return rc;
        hipLaunchKernelGGL(k_ld_children, dim3(stream_grid(s, S)), dim3(kTPB), 0, st, seg[cur], ioff[cur],
                           (uint32_t)S, cnt, T, (uint32_t)d, segc, segflag, seg[d], ioff[d], ctl, slist, ctl32);
        LAUNCHCHK("k_ld_children");
        hipLaunchKernelGGL(k_ld_less, dim3((uint32_t)NI), dim3(kTPB), 0, st, V[cur], seg[cur], ioff[cur], imap, segc,
                           cnt, R);
        LAUNCHCHK("k_ld_less");
        hipLaunchKernelGGL(k_ld_final<false>, dim3((uint32_t)NI), dim3(kTPB), 0, st, V[cur], P[cur], seg[cur],
                           ioff[cur], imap, segc, cnt, R, V[d], P[d], vout, pout, segflag, flist, ctl32 + 1,
                           (const uint32_t*)nullptr, 0u, NI <= small_items ? cap_small : cap);
        LAUNCHCHK("k_ld_final");
        unsigned long long h[2];
        HIPCHK(hipMemcpyAsync(h, ctl, 16, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        int jumps = 0;
        const uint32_t F = (uint32_t)(h[1] >> 32);
        if (F) {  // walks longer than cap: double R over the flagged ranges, then place them again
            hipLaunchKernelGGL(k_ld_fitems, dim3(stream_grid(s, F + 1)), dim3(kTPB), 0, st, seg[cur], flist, F, fi);
            LAUNCHCHK("k_ld_fitems");
            if ((rc = scan_u32_exclusive_u32(fi, fi, F + 1, scratch, st))) return rc;
            uint32_t nf = 0;
            HIPCHK(hipMemcpyAsync(&nf, fi + F, 4, hipMemcpyDeviceToHost, st));
            HIPCHK(hipStreamSynchronize(st));
            for (;;) {
                if (jumps >= kMaxJumps) return set_err(MQ_EHIP, "mq_index_build_lomuto: pointer doubling did not converge");
                for (int k = 0; k < jbatch && jumps < kMaxJumps; k++, jumps++) {
                    hipLaunchKernelGGL(k_ld_jump, dim3(nf), dim3(kTPB), 0, st, seg[cur], flist, fi, F, R, chg, jumps);
                    LAUNCHCHK("k_ld_jump");
                }
                unsigned int ch = 0;
                HIPCHK(hipMemcpyAsync(&ch, chg + jumps - 1, 4, hipMemcpyDeviceToHost, st));
                HIPCHK(hipStreamSynchronize(st));
                if (!ch) break;
            }
            hipLaunchKernelGGL(k_ld_final<true>, dim3(nf), dim3(kTPB), 0, st, V[cur], P[cur], seg[cur], ioff[cur], imap,
                               segc, cnt, R, V[d], P[d], vout, pout, segflag, flist, ctl32 + 1, (const uint32_t*)fi, F,
                               0);
            LAUNCHCHK("k_ld_final");
        }
        nsmall = (uint32_t)h[1];
        if (stats) {
            std::vector<LSeg> hs(S);
            HIPCHK(hipMemcpy(hs.data(), seg[cur], S * sizeof(LSeg), hipMemcpyDeviceToHost));
            uint64_t rows = 0;
            for (const LSeg& g : hs) rows += (uint64_t)g.hi - g.lo + 1;
            fprintf(stderr, "lq level %d: large ranges %llu rows %llu items %llu | small so far %u | flagged %u jumps %d\n",
                    level, (unsigned long long)S, (unsigned long long)rows, (unsigned long long)NI, nsmall,
                    F, jumps);
            if (F) {  // the flagged ranges' shape: rows, "<" side c and ">=" side m = rows - 1 - c
                std::vector<uint32_t> fl(F), sc(S);
                HIPCHK(hipMemcpy(fl.data(), flist, F * 4, hipMemcpyDeviceToHost));
                HIPCHK(hipMemcpy(sc.data(), segc, S * 4, hipMemcpyDeviceToHost));
                for (uint32_t k = 0; k < F; k++) {
                    const LSeg& g = hs[fl[k]];
                    const uint64_t r = (uint64_t)g.hi - g.lo + 1, c = sc[fl[k]];
                    fprintf(stderr, "lq   flagged rows %llu c %llu m %llu\n", (unsigned long long)r,
                            (unsigned long long)c, (unsigned long long)(r - 1 - c));
                }
            }
        }
        S = h[0] >> 40;
        NI = h[0] & ((1ull << 40) - 1);
        cur = d;
        level++;
    }
    if (nsmall) {
        const uint32_t grid = nsmall < 16384u ? nsmall : 16384u;
        int rc = launch_small((int)T, grid, st, V[0], P[0], V[1], P[1], slist, nsmall, vout, pout);
        if (rc) return rc;
    }
    HIPCHK(hipStreamSynchronize(st));  // the buffers go back to the pool
    return MQ_OK;
}

}  // namespace mqi
