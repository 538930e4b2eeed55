// mq_shared.hip — shared_select (src/query.c:439-583): Q range selects over one
// column with the column read once (the reference reads it once per thread with Q
// predicates per value, query.c:472-479; a per-query loop of mq_select_positions
// would read it Q times).
//
// Decomposition: the scan grid of mq_scan_common.h, but inside a block each WAVE
// owns a contiguous quarter of the block's chunk (a "wave-chunk"). The Q bounds cut
// the int32 line into elementary intervals (EIs); the count pass (k_ssk_count) finds
// each covered row's EI through an LDS cell table, counts per (query, wave-chunk) and
// lists every (query, row) pair of its wave-chunk into the wave's slice of the
// workspace; one kernel scans the counts into offsets and totals (k_ss_offsets); the
// scatter (k_ssp_scatter) sorts each slice by query in LDS and writes every query's
// run of rows. A slice that overflows (dense queries: more than a pair a row) sends
// the write to the column pass (k_ssi_write) on the same counts. DESIGN.md §3.4.
// HBM traffic: 4N + 4 sum(K_q) (pairs) + 4 sum(K_q) read + 4 sum(K_q) written.

#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "mq_common.h"
#include "mq_device.h"
#include "mq_scan_common.h"

namespace {

using namespace mqi;

constexpr int kMaxQ = 256;             // queries per launch (the server chunks at 150)
constexpr int kSsUnroll = 4;           // wave-tiles in flight per lane
constexpr uint64_t kWaveTile = 256;    // rows per wave-tile (64 lanes x dwordx4)
constexpr uint64_t kGranule = kWaves * kWaveTile * kSsUnroll;  // 4096 rows

__device__ __forceinline__ void wave_chunk(uint64_t n, uint64_t rpb, int wave, uint64_t* s,
                                           uint64_t* e) {
    const uint64_t wrows = rpb / kWaves;  // multiple of kWaveTile * kSsUnroll
    uint64_t a = (uint64_t)blockIdx.x * rpb + (uint64_t)wave * wrows;
    uint64_t b = a + wrows;
    if (a > n) a = n;
    if (b > n) b = n;
    *s = a;
    *e = b;
}

template <bool VEC>
__device__ __forceinline__ int4 load_row4(const int* __restrict__ col, uint64_t row, uint64_t end) {
    if (row + 3 < end) return load4_nt<VEC>(col + row);
    int4 v;
    v.x = row + 0 < end ? col[row + 0] : 0;
    v.y = row + 1 < end ? col[row + 1] : 0;
    v.z = row + 2 < end ? col[row + 2] : 0;
    v.w = row + 3 < end ? col[row + 3] : 0;
    return v;
}

__device__ __forceinline__ uint32_t match4(int4 v, Pred p, uint64_t row, uint64_t end) {
    uint32_t b = (((uint32_t)v.x - p.lo) <= p.wm1 ? 1u : 0u) | (((uint32_t)v.y - p.lo) <= p.wm1 ? 2u : 0u) |
                 (((uint32_t)v.z - p.lo) <= p.wm1 ? 4u : 0u) | (((uint32_t)v.w - p.lo) <= p.wm1 ? 8u : 0u);
    if (row + 3 >= end) {
        if (row + 0 >= end) b &= ~1u;
        if (row + 1 >= end) b &= ~2u;
        if (row + 2 >= end) b &= ~4u;
        if (row + 3 >= end) b &= ~8u;
    }
    return b;
}

// Output pointers come from a device array, so the compiler sees generic (flat)
// pointers; flat stores count in lgkmcnt and every later LDS wait would also wait
// for them to reach memory. The outputs are global memory: store through that.
typedef int __attribute__((address_space(1))) gint;
__device__ __forceinline__ gint* global_ptr(int* p) { return (gint*)p; }

// Writes one wave-tile's matches of one query; o advances by the match count.
__device__ __forceinline__ void ss_emit(gint* __restrict__ out, unsigned long long& o, uint64_t row,
                                       unsigned long long m0, unsigned long long m1,
                                       unsigned long long m2, unsigned long long m3, int lane,
                                       unsigned long long ltmask, int32_t base) {
    const unsigned int tot = (unsigned int)(__popcll(m0) + __popcll(m1) + __popcll(m2) + __popcll(m3));
    if (!tot) return;  // uniform
    const unsigned int pre = (unsigned int)(__popcll(m0 & ltmask) + __popcll(m1 & ltmask) +
                                            __popcll(m2 & ltmask) + __popcll(m3 & ltmask));
    const unsigned long long bit = 1ull << lane;
    gint* w = out + o + pre;
    unsigned int k = 0;
    if (m0 & bit) w[k++] = (int)(row + 0) + base;
    if (m1 & bit) w[k++] = (int)(row + 1) + base;
    if (m2 & bit) w[k++] = (int)(row + 2) + base;
    if (m3 & bit) w[k++] = (int)(row + 3) + base;
    o += tot;
}

// ---------------------------------------------------------------------------
// Elementary intervals. The 2q query bounds cut the
// int32 line into m+1 <= 2q+1 "elementary intervals" (EIs); every value lies in
// exactly one, e(v) = #{bounds <= v}, and query i covers the EIs [ea_i, eb_i).
// e(v) comes from a 4096-bucket table over [bmin, bmax] (each entry: the EI range
// [e0, e1] its values can fall in; one LDS read when the bucket holds no bound,
// a binary search over its few bounds otherwise).
//   count: per wave-chunk, an LDS histogram of e over the covered rows; query i's
//          count = P[eb_i] - P[ea_i] from the histogram's prefix. Cost per row: the
//          lookup, not q compares.
//   write: per 256-row wave-tile, the (query, row) pairs of its covered rows
//          (query lists per EI, CSR) are listed in LDS in row order; a pair's rank
//          among earlier pairs of its query (one broadcast LDS read per pair of
//          the tile) gives its slot after the query's running offset. Tiles with
//          many pairs (dense queries) take the per-query ballot loop instead.
// ---------------------------------------------------------------------------
// Per-query ballot kernels (every predicate on every row) ran up to round 5 for small Q.
// Against the single-pass k-major count (1e9 rows, count + write, one box,
// profiles/r05_ss_small_q.log) they lost from Q = 2: 0.1 % ranges Q = 2 / 4 / 8 0.96 /
// 1.38 / 2.38 vs 0.79 / 0.83 / 0.89 ms, 10 % ranges 1.90 / 3.17 / 6.0 vs 1.72 / 2.52 /
// 4.22 ms; only very dense sets (50 % ranges, a pair per row, the pair slices overflow)
// were faster with them (Q = 2 4.77 vs 5.17 ms). Removed in round 6.
constexpr int kEiMax = 2 * kMaxQ + 2;   // EIs (m + 1 <= 2 q + 1) + prefix slot
constexpr int kBuckets = 4096;
constexpr int kPairCap = 512;
// k_ssk_count prefetches the next group from this many queries (round 5, with the
// dynamic-LDS pass and 4 blocks a CU: off is faster at Q = 16 / 32 / 64 (0.88 / 0.94 /
// 1.13 against 0.90 / 0.97 / 1.18 ms), on at Q = 150 (1.567 against 1.612), three
// alternating rounds on one box, profiles/r05_ss_pf_ab.log; was 64)
constexpr int kSsPfMinQ = 100;
constexpr int kQlCap = 1024;  // per-EI query-list entries staged in LDS by k_ssk_count
constexpr int kCells = 4096;             // k_ssk_count's cell table (u16 per cell, 8 KB of LDS)
constexpr uint32_t kRingK = 320;         // k_ssk_count's queued rows per wave (< 64 + a 256-row tile)
// Pairs of one 1024-row wave-group held in LDS until the next group's loads are
// issued, then written with at most 4 straight-line coalesced stores: vmcnt retires
// loads and stores in order, so stores issued before a group's loads (or a
// data-dependent number of them, which makes the compiler wait for all) would put
// their round trip on every group (a count pass with direct per-pair stores ran at
// 2.3 ms, 1.2 without the stores, at Q = 150).
constexpr uint32_t kPb = 256;

struct EiMeta {
    int m;          // number of bounds
    int shift;      // bucket width 2^shift
    int bmin, bmax; // first / last bound
    int xshift;     // k_ssk_count's cell width 2^xshift
};

struct EiTables {  // device copies, filled by the host (ss_count)
    const int32_t* bounds;      // m sorted bounds
    const uint32_t* bucket;     // kBuckets x {e0 (low 16), e1 (high 16)}
    const uint32_t* qoff;       // m + 2: CSR offsets of the per-EI query lists
    const uint16_t* qlist;      // queries covering each EI, ascending
    const uint32_t* qab;        // per query: ea (low 16) | eb (high 16)
    const uint16_t* cell;       // kCells entries over [bmin, bmax] (k_ssk_count): 0 = no covered
                                // EI meets the cell; e + 1 (< 0x8000) = the cell lies in covered
                                // EI e; 0x8000 | e0 = bounds inside, e(v) >= e0: search
};

__device__ __forceinline__ int ei_of(int32_t v, const EiMeta& M, const uint32_t* s_bkt,
                                     const int32_t* s_b) {
    if (v < M.bmin) return 0;
    if (v > M.bmax) return M.m;
    const uint32_t ent = s_bkt[((uint32_t)v - (uint32_t)M.bmin) >> M.shift];
    int lo = (int)(ent & 0xFFFFu), hi = (int)(ent >> 16);  // e(v) in [lo, hi]
    while (lo < hi) {  // first j in [lo, hi) with bound[j] > v, else hi
        const int mid = (lo + hi) >> 1;
        if (s_b[mid] <= v) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// The bucket table into LDS: all of a thread's 16 entries are loaded before any
// is stored (a load/store loop paid 16 round trips per block before its scan).
__device__ __forceinline__ void stage_buckets(const uint32_t* __restrict__ g, uint32_t* s, int tid) {
    constexpr int kPer = kBuckets / kTPB;
    uint32_t v[kPer];
#pragma unroll
    for (int k = 0; k < kPer; k++) v[k] = g[tid + k * kTPB];
#pragma unroll
    for (int k = 0; k < kPer; k++) s[tid + k * kTPB] = v[k];
}

template <bool VEC>
__global__ __launch_bounds__(kTPB) void k_ssi_count(const int* __restrict__ col, uint64_t n, uint64_t rpb,
                                                    EiMeta M, EiTables T, int q,
                                                    uint32_t* __restrict__ counts, uint64_t nwc) {
    __shared__ uint32_t s_bkt[kBuckets];
    __shared__ int32_t s_b[kEiMax];
    __shared__ uint32_t s_qoff[kEiMax];
    __shared__ uint32_t hist[kWaves][kEiMax];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    stage_buckets(T.bucket, s_bkt, tid);
    for (int i = tid; i < M.m; i += kTPB) s_b[i] = T.bounds[i];
    for (int i = tid; i <= M.m + 1; i += kTPB) s_qoff[i] = T.qoff[i];
    for (int i = tid; i < kWaves * kEiMax; i += kTPB) (&hist[0][0])[i] = 0;
    __syncthreads();
    uint64_t s, e;
    wave_chunk(n, rpb, wave, &s, &e);
    for (uint64_t t = s; t < e; t += kWaveTile * kSsUnroll) {
        int4 v[kSsUnroll];
#pragma unroll
        for (int u = 0; u < kSsUnroll; u++)
            v[u] = load_row4<VEC>(col, t + (uint64_t)u * kWaveTile + (uint64_t)lane * 4, e);
#pragma unroll
        for (int u = 0; u < kSsUnroll; u++) {
            const uint64_t row = t + (uint64_t)u * kWaveTile + (uint64_t)lane * 4;
            const int x[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
            for (int k = 0; k < 4; k++) {
                if (row + k < e) {
                    const int ei = ei_of(x[k], M, s_bkt, s_b);
                    if (s_qoff[ei + 1] > s_qoff[ei]) atomicAdd(&hist[wave][ei], 1u);
                }
            }
        }
    }
    __builtin_amdgcn_wave_barrier();
    // exclusive prefix over the m+1 EIs, in place (P[m+1] = total): this wave only
    uint32_t* h = hist[wave];
    const int ne = M.m + 2;
    const int per = (ne + 63) / 64;
    uint32_t loc = 0;
    for (int i = 0; i < per; i++) {
        const int j = lane * per + i;
        if (j < ne) loc += h[j];
    }
    uint32_t incl = loc;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    uint32_t run = incl - loc;
    __builtin_amdgcn_wave_barrier();
    for (int i = 0; i < per; i++) {
        const int j = lane * per + i;
        if (j < ne) {
            const uint32_t c = h[j];
            h[j] = run;
            run += c;
        }
    }
    __builtin_amdgcn_wave_barrier();
    const uint64_t wc = (uint64_t)blockIdx.x * kWaves + wave;
    for (int i = lane; i < q; i += 64) {
        const uint32_t ab = T.qab[i];
        counts[(uint64_t)i * nwc + wc] = h[ab >> 16] - h[ab & 0xFFFFu];
    }
}

template <bool VEC>
__global__ __launch_bounds__(kTPB) void k_ssi_write(const int* __restrict__ col, uint64_t n, uint64_t rpb,
                                                    EiMeta M, EiTables T, const Pred* __restrict__ preds,
                                                    int q, const unsigned long long* __restrict__ offs,
                                                    uint64_t nwc, int* const* __restrict__ outs, int32_t base,
                                                    const unsigned int* __restrict__ only_if) {
    if (only_if && !*only_if) return;  // single pass without overflow: k_ssp_scatter wrote
    __shared__ uint32_t s_bkt[kBuckets];
    __shared__ int32_t s_b[kEiMax];
    __shared__ uint32_t s_qoff[kEiMax];
    __shared__ unsigned long long run[kWaves][kMaxQ];
    __shared__ uint32_t pairs[kWaves][kPairCap];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const unsigned long long ltmask = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    stage_buckets(T.bucket, s_bkt, tid);
    for (int i = tid; i < M.m; i += kTPB) s_b[i] = T.bounds[i];
    for (int i = tid; i <= M.m + 1; i += kTPB) s_qoff[i] = T.qoff[i];
    for (int i = tid; i < q; i += kTPB) {
        const unsigned long long base = offs[(uint64_t)i * nwc];
#pragma unroll
        for (int w = 0; w < kWaves; w++)
            run[w][i] = offs[(uint64_t)i * nwc + (uint64_t)blockIdx.x * kWaves + w] - base;
    }
    __syncthreads();
    // tiles with more pairs than this take the per-query ballot loop (cost ~ 12 q)
    int cap = (int)sqrtf(768.0f * (float)q);
    if (cap > kPairCap) cap = kPairCap;
    uint64_t s, e;
    wave_chunk(n, rpb, wave, &s, &e);
    uint32_t* pl = pairs[wave];
    for (uint64_t t = s; t < e; t += kWaveTile * kSsUnroll) {
        int4 v[kSsUnroll];
#pragma unroll
        for (int u = 0; u < kSsUnroll; u++)
            v[u] = load_row4<VEC>(col, t + (uint64_t)u * kWaveTile + (uint64_t)lane * 4, e);
#pragma unroll
        for (int u = 0; u < kSsUnroll; u++) {
            const uint64_t row = t + (uint64_t)u * kWaveTile + (uint64_t)lane * 4;
            const int x[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
            uint32_t qa[4], qn[4];
            uint32_t np = 0;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                qa[k] = 0;
                qn[k] = 0;
                if (row + k < e) {
                    const int ei = ei_of(x[k], M, s_bkt, s_b);
                    qa[k] = s_qoff[ei];
                    qn[k] = s_qoff[ei + 1] - qa[k];
                }
                np += qn[k];
            }
            uint32_t incl = np;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = __shfl_up(incl, o, 64);
                if (lane >= o) incl += y;
            }
            const uint32_t tot = __builtin_amdgcn_readfirstlane(__shfl(incl, 63, 64));
            if (tot == 0) continue;
            if (tot > (uint32_t)cap) {
                // dense tile: every query's ballot, as k_ss_write
                for (int j = 0; j < q; j++) {
                    const Pred p = preds[j];
                    unsigned long long o = run[wave][j];
                    const uint32_t b = match4(v[u], p, row, e);
                    ss_emit(global_ptr(outs[j]), o, row, __ballot(b & 1u), __ballot(b & 2u), __ballot(b & 4u),
                            __ballot(b & 8u), lane, ltmask, base);
                    if (lane == 0) run[wave][j] = o;
                }
                __builtin_amdgcn_wave_barrier();
                continue;
            }
            // list the pairs in row order: (query << 16) | row offset in the wave-tile
            uint32_t at = incl - np;
#pragma unroll
            for (int k = 0; k < 4; k++)
                for (uint32_t i = 0; i < qn[k]; i++) pl[at++] = ((uint32_t)T.qlist[qa[k] + i] << 16) | (uint32_t)(lane * 4 + k);
            __builtin_amdgcn_wave_barrier();
            // rank of each pair among earlier pairs of its query: 64 pairs at a time,
            // lanes holding the same query found by 8 ballots over its bits (was a
            // broadcast-read loop over all the tile's pairs: one dependent LDS
            // read per pair); the group's last pair of a query advances that
            // query's running offset, so later groups start after it
            const uint64_t tile0 = t + (uint64_t)u * kWaveTile;
            for (uint32_t i0 = 0; i0 < tot; i0 += 64) {
                const uint32_t i = i0 + (uint32_t)lane;
                const bool valid = i < tot;
                const uint32_t me = valid ? pl[i] : 0u;
                const uint32_t mq = me >> 16;  // < q <= kMaxQ = 256: 8 bits
                const unsigned long long peers = match_any8(mq, __ballot(valid));
                const uint32_t rank = lanes_below(peers);
                const bool last = (peers & ~ltmask & ~(1ull << lane)) == 0;
                unsigned long long at0 = 0;
                if (valid) {
                    at0 = run[wave][mq];
                    global_ptr(outs[mq])[at0 + rank] = (int)(tile0 + (me & 0xFFFFu)) + base;
                }
                __builtin_amdgcn_wave_barrier();
                if (valid && last) run[wave][mq] = at0 + rank + 1;
                __builtin_amdgcn_wave_barrier();
            }
        }
    }
}

// ---------------------------------------------------------------------------
// One read of the column (the usual case): the count pass also lists
// every (query, row) pair of its wave-chunk, in row order, into the wave's slice of
// the workspace (one u32 per pair: query << 24 | row offset in the wave-chunk);
// after the scan, k_ssp_scatter sorts each slice by query in LDS, 2048 pairs at a
// time (stable: 8-ballot match-any ranks), and writes every query's run of rows
// with consecutive stores. HBM: 4N + 4K (pairs) + 4K + 4K (scatter) instead of
// 8N + 4K, and no second pass of interval lookups. A slice holds one pair per row
// of its wave-chunk; a wave-chunk with more pairs (dense queries) flags an overflow
// and the write falls back to the column pass (k_ssi_write) on the same counts.
// ---------------------------------------------------------------------------
// The single pass, k-major (round 3): lane l of a wave-tile holds rows l, l + 64,
// l + 128, l + 192 (four coalesced dword loads instead of one dwordx4), so the rows of
// one load are 64 consecutive rows and a row's place in the wave's queue is one
// mbcnt of the ballot of "covered" (rows in row order, no per-lane prefix over four
// rows). A covered row is found with one LDS read of the cell table (kCells u16 over
// [bmin, bmax], ei_build), which also gives its EI unless a bound lies inside the
// cell; such rows are queued with a flag and their EI found from the cell's first EI
// by a short search. The round-2 form of this pass (a coverage bitmap test per row, a
// per-lane prefix over a lane's 4 consecutive rows, removed in round 6) spent 670 M
// VALU per pass at Q = 150 on that per-row work (PMC); this pass does it in fewer
// instructions (625 vs 720 M VALU before the cell table shrank to 4096 cells, which let
// 4 blocks share a CU).
__device__ __forceinline__ uint32_t mbcnt64(unsigned long long m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// (Round 5 measured a 16-bit list, query << 7 | the row in its 128-row tile plus tile
// tokens: half the bytes, yet the count pass 1.20 -> 1.28 ms and the scatter 0.51 -> 0.57
// at Q = 150, profiles/r05_ss_host_ab.log; removed in round 6.)
template <bool PF>
__global__ __launch_bounds__(kTPB) void k_ssk_count(const int* __restrict__ col, uint64_t n, uint64_t rpb,
                                                    EiMeta M, EiTables T, int q, uint32_t* __restrict__ counts,
                                                    uint64_t nwc, uint32_t* __restrict__ pairs, uint64_t cap,
                                                    uint32_t* __restrict__ npairs, unsigned int* __restrict__ overflow,
                                                    uint32_t qlcap) {
    __shared__ uint16_t s_cell[kCells];
    __shared__ uint32_t s_pb[kWaves][kPb];
    __shared__ int32_t s_qv[kWaves][kRingK];
    __shared__ uint32_t s_qr[kWaves][kRingK];
    // (round 5) the EI-sized tables in dynamic LDS, sized by this launch's m and list
    // length (ssk_dyn_bytes), and a queued row's cell entry read again from its value
    // instead of queued: 39.5 KB a block -> 31 KB at Q = 150 (the grid's blocks a CU are
    // then set by ss_count's policy, not by LDS)
    extern __shared__ __attribute__((aligned(16))) unsigned char s_dyn[];
    const uint32_t hs = (uint32_t)M.m + 2u;  // EIs 0 .. m, plus the prefix slot
    int32_t* const s_b = reinterpret_cast<int32_t*>(s_dyn);
    uint32_t* const s_qoff = reinterpret_cast<uint32_t*>(s_dyn) + hs;
    uint32_t* const hist = s_qoff + hs;  // [kWaves][hs]
    uint16_t* const s_ql = reinterpret_cast<uint16_t*>(hist + kWaves * hs);
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    {  // the cell table: 16 u16 per thread, loaded as two 16-byte words before any store
        const uint4* g = reinterpret_cast<const uint4*>(T.cell);
        uint4* d = reinterpret_cast<uint4*>(s_cell);
        constexpr int kPer = kCells * 2 / 16 / kTPB;
        uint4 u[kPer];
#pragma unroll
        for (int k = 0; k < kPer; k++) u[k] = g[tid + k * kTPB];
#pragma unroll
        for (int k = 0; k < kPer; k++) d[tid + k * kTPB] = u[k];
    }
    for (int i = tid; i < M.m; i += kTPB) s_b[i] = T.bounds[i];
    for (int i = tid; i <= M.m + 1; i += kTPB) s_qoff[i] = T.qoff[i];
    for (uint32_t i = tid; i < kWaves * hs; i += kTPB) hist[i] = 0;
    __syncthreads();
    const uint32_t nql = s_qoff[M.m + 1];
    const bool ql_lds = nql <= qlcap;
    if (ql_lds)
        for (uint32_t i = tid; i < nql; i += kTPB) s_ql[i] = T.qlist[i];
    __syncthreads();
    const uint32_t bmin = (uint32_t)M.bmin, xsh = (uint32_t)M.xshift, m = (uint32_t)M.m;
    uint64_t s, e;
    wave_chunk(n, rpb, wave, &s, &e);
    const uint64_t wc = (uint64_t)blockIdx.x * kWaves + wave;
    uint32_t* list = pairs + wc * cap;
    uint32_t* pb = s_pb[wave];
    int32_t* qv = s_qv[wave];
    uint32_t* qr = s_qr[wave];
    uint32_t run = 0, pend = 0, pend_at = 0, head = 0, tail = 0, fill = 0;
    bool direct = false;
    const __amdgpu_buffer_rsrc_t lrs =
        __builtin_amdgcn_make_buffer_rsrc((void*)list, 0, (int)(cap * 4u), 0x00020000);
    auto enc = [&](uint32_t qid, uint32_t r) { return (qid << 24) | r; };
    auto round = [&](uint32_t nr) {
        const bool has = (uint32_t)lane < nr;
        uint32_t qa = 0, qn = 0, r = 0;
        if (has) {
            const uint32_t slot = head + (uint32_t)lane;
            const int32_t x = qv[slot];
            const uint32_t ent = s_cell[min(((uint32_t)x - bmin) >> xsh, (uint32_t)kCells - 1u)];
            r = qr[slot];
            uint32_t ei = ent - 1u;
            if (ent & 0x8000u) {  // bounds inside the cell: b[e0 ..), e0 = its first EI
                ei = ent & 0xFFFu;
                const uint32_t nb = (ent >> 12) & 7u;  // their number when below 7, else 0
                if (nb) {
                    // (round 4) e(v) = e0 + the cell's bounds <= v: nb reads, no search.
                    // PMC at Q = 150: the search made every 64-row round pay ~130 VALU
                    // (almost every round holds a row of a flagged cell)
                    const uint32_t e0 = ei;
                    for (uint32_t i = 0; i < nb; i++) ei += s_b[e0 + i] <= x ? 1u : 0u;
                } else if (ei < m && s_b[ei] <= x) {
                    uint32_t lo = ei + 1, hi = m;
                    while (lo < hi) {
                        const uint32_t mid = (lo + hi) >> 1;
                        if (s_b[mid] <= x) lo = mid + 1;
                        else hi = mid;
                    }
                    ei = lo;
                }
            }
            qa = s_qoff[ei];
            qn = s_qoff[ei + 1] - qa;
            if (qn) atomicAdd(&hist[wave * hs + ei], 1u);
        }
        head += nr;
        const uint32_t ne = qn;  // entries this row writes
        uint32_t pre = 0, tot = 0;
        const bool single = !__ballot(ne > 1u);
        if (single) {  // the usual case: at most one entry per row
            const unsigned long long bm = __ballot(ne != 0u);
            pre = mbcnt64(bm);
            tot = (uint32_t)__popcll(bm);
        } else if (!__ballot(ne >= 8u)) {
#pragma unroll
            for (int bit = 0; bit < 3; bit++) {
                const unsigned long long bm = __ballot((ne >> bit) & 1u);
                pre += mbcnt64(bm) << bit;
                tot += (uint32_t)__popcll(bm) << bit;
            }
        } else {
            for (uint32_t t = 1;; t++) {
                const unsigned long long bm = __ballot(ne >= t);
                if (!bm) break;
                pre += mbcnt64(bm);
                tot += (uint32_t)__popcll(bm);
            }
        }
        if (tot == 0) return;
        if ((uint64_t)run + tot <= cap) {
            direct = direct || fill + tot > kPb;
            // (round 4) the query list read from LDS or global memory by a wave-uniform
            // branch, and one pair per row without a loop in the usual case: a ternary of
            // the two pointers compiled to flat loads (both memory paths, and waits on
            // both), in a per-lane loop
            // (the list by buffer stores: else the compiler selects between the two
            // pointers and stores through flat)
            auto put = [&](uint32_t i, uint32_t y) {
                if (!direct) pb[fill + pre + i] = y;
                else __builtin_amdgcn_raw_buffer_store_b32(y, lrs, (int)((run + pre + i) * 4u), 0, 0);
            };
            if (single && ql_lds) {
                if (qn) put(0, enc(s_ql[qa], r));
            } else if (ql_lds) {
                for (uint32_t i = 0; i < qn; i++) put(i, enc(s_ql[qa + i], r));
            } else {
                for (uint32_t i = 0; i < qn; i++) put(i, enc(T.qlist[qa + i], r));
            }
            if (!direct) fill += tot;
        }
        run += tot;
    };
    auto drain = [&]() {  // full rounds while 64 rows are queued, the rest to the front
        if (tail < 64u) return;
        do {
            round(64u);
            __builtin_amdgcn_wave_barrier();
        } while (tail - head >= 64u);
        const uint32_t rest = tail - head;
        int32_t mv = 0;
        uint32_t mr = 0;
        if ((uint32_t)lane < rest) mv = qv[head + lane], mr = qr[head + lane];
        __builtin_amdgcn_wave_barrier();
        if ((uint32_t)lane < rest) qv[lane] = mv, qr[lane] = mr;
        __builtin_amdgcn_wave_barrier();
        head = 0;
        tail = rest;
    };
    constexpr int kV = kSsUnroll * 4;
    constexpr uint64_t kG = kWaveTile * kSsUnroll;
    auto load_group = [&](uint64_t t0, int* x) {
        if (t0 + kG <= e) {
#pragma unroll
            for (int i = 0; i < kV; i++) x[i] = __builtin_nontemporal_load(col + t0 + (uint64_t)i * 64 + lane);
        } else {
#pragma unroll
            for (int i = 0; i < kV; i++) {
                const uint64_t row = t0 + (uint64_t)i * 64 + lane;
                x[i] = row < e ? col[row] : 0;
            }
        }
    };
    // PF (round 4): the next group's loads are issued before this group is queued and
    // drained, so a wave keeps a group in flight while its rounds run (without it the
    // wave's next loads wait for its whole drain)
    int v[kV];
    if (PF && s < e) {
        load_group(s, v);
        // the first group waited for here: otherwise the loop entry merges "v pending"
        // from here with "v copied" from the back edge, and the wait-count pass then
        // waits inside every iteration for the next group's loads
        __builtin_amdgcn_s_waitcnt(0);
    }
    for (uint64_t t = s; t < e; t += kG) {
        const bool whole = t + kG <= e;
        int vn[kV];
        if (PF) {
            if (t + kG < e) load_group(t + kG, vn);
        } else {
            load_group(t, v);
        }
        {  // the previous group's pairs, behind this group's loads
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int k = 0; k < (int)(kPb / 64); k++) {
                const uint32_t i = (uint32_t)(k * 64 + lane);
                const int off = i < pend ? (int)((pend_at + i) * 4u) : (int)0x80000000u;
                __builtin_amdgcn_raw_buffer_store_b32(pb[i], lrs, off, 0, 0);
            }
            __builtin_amdgcn_wave_barrier();
        }
        const uint32_t grp_at = run;
        fill = 0;
        direct = false;
        const uint32_t r0 = (uint32_t)(t - s) + (uint32_t)lane;
        // per 256-row tile: its 4 row slots queued, then one drain (a drain per row slot
        // inlined 16 copies of the round and overflowed the instruction cache)
#pragma unroll
        for (int u = 0; u < kSsUnroll; u++) {
            uint32_t ent[4];
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const int i = u * 4 + k;
                ent[k] = s_cell[min(((uint32_t)v[i] - bmin) >> xsh, (uint32_t)kCells - 1u)];
            }
            if (!whole) {  // (wave-uniform) rows past the chunk's end are not covered
#pragma unroll
                for (int k = 0; k < 4; k++)
                    if (r0 + (uint32_t)(u * 4 + k) * 64u >= (uint32_t)(e - s)) ent[k] = 0u;
            }
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const int i = u * 4 + k;
                const bool cov = ent[k] != 0u;
                const unsigned long long bm = __ballot(cov);
                if (cov) {
                    const uint32_t at = tail + mbcnt64(bm);
                    qv[at] = v[i];
                    qr[at] = r0 + (uint32_t)i * 64u;
                }
                tail += (uint32_t)__popcll(bm);
            }
            __builtin_amdgcn_wave_barrier();
            drain();
        }
        pend = fill;
        pend_at = grp_at;
        if (PF) {
#pragma unroll
            for (int i = 0; i < kV; i++) v[i] = vn[i];
        }
    }
    __builtin_amdgcn_wave_barrier();
    for (uint32_t i = (uint32_t)lane; i < pend; i += 64) list[pend_at + i] = pb[i];
    __builtin_amdgcn_wave_barrier();
    fill = 0;
    direct = true;
    while (tail != head) {
        round(tail - head < 64u ? tail - head : 64u);
        __builtin_amdgcn_wave_barrier();
    }
    if (lane == 0) {
        npairs[wc] = run;
        if ((uint64_t)run > cap) atomicOr(overflow, 1u);
    }
    __builtin_amdgcn_wave_barrier();
    uint32_t* h = hist + wave * hs;
    const int ne = (int)hs;
    const int per = (ne + 63) / 64;
    uint32_t loc = 0;
    for (int i = 0; i < per; i++) {
        const int j = lane * per + i;
        if (j < ne) loc += h[j];
    }
    uint32_t incl = loc;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    uint32_t acc = incl - loc;
    __builtin_amdgcn_wave_barrier();
    for (int i = 0; i < per; i++) {
        const int j = lane * per + i;
        if (j < ne) {
            const uint32_t c = h[j];
            h[j] = acc;
            acc += c;
        }
    }
    __builtin_amdgcn_wave_barrier();
    for (int i = lane; i < q; i += 64) {
        const uint32_t ab = T.qab[i];
        counts[(uint64_t)i * nwc + wc] = h[ab >> 16] - h[ab & 0xFFFFu];
    }
}

constexpr int kSpChunk = 4096;                  // pairs sorted in LDS at a time
constexpr int kSpPerWave = kSpChunk / kWaves;   // 1024: 16 rounds of 64
constexpr int kSpRounds = kSpPerWave / 64;
constexpr int kSpBatch = 4;                     // rounds whose pairs are loaded together

// Ranks go to LDS as they are made (the pair itself in s_buf, its rank among the
// wave's earlier pairs of its query in s_loc), not into registers held across the
// block's scan: 2048-pair chunks held that way needed 102 VGPRs, and 4096 / 8192
// 144 / 225. The placement reads a thread's entries, syncs, and writes them sorted
// into the same s_buf. Longer chunks make longer runs per query in the output
// (≈ 27 entries at Q = 150 instead of ≈ 14), fewer partial lines: 0.55 -> 0.52 ms
// at Q = 150 on 1e9 rows; 8192-pair chunks (2 waves per SIMD) took 0.77 ms.
// `pairs` is clobbered: the padding stores of a chunk land on pairs of that chunk
// already read (hence not const, not __restrict__).
// Up to kArgQ output pointers by value (the kernel's argument block): a write that runs
// only the scatter then needs no upload before it.
constexpr int kArgQ = kMaxQ;  // 2 KB of arguments (the limit is 4 KB)
struct SsArgOuts {
    int* p[kArgQ];
};

template <int SW>
__global__ __launch_bounds__(64 * SW, 4) void k_ssp_scatter(uint32_t* pairs, uint64_t cap,
                                                      const uint32_t* __restrict__ npairs,
                                                      const unsigned long long* __restrict__ offs, uint64_t nwc,
                                                      int q, int* const* __restrict__ outs, SsArgOuts ao,
                                                      bool by_arg, uint64_t rpb, int32_t base,
                                                      const unsigned int* __restrict__ overflow) {
    // SW waves a block, 1024 pairs a wave a chunk (round 5: SW = 8 sorts 8192-pair
    // chunks in 512 threads, same registers a thread, twice the LDS)
    constexpr int TPB = 64 * SW, CH = kSpPerWave * SW;
    if (*overflow) return;  // a slice overflowed: k_ssi_write's column pass writes
    __shared__ uint32_t s_buf[CH];
    __shared__ uint16_t s_loc[CH];
    __shared__ uint32_t s_cnt[SW][kMaxQ];
    __shared__ uint32_t s_tot[kMaxQ];
    // (round 5) a query's write base for this chunk, out + run - start: one LDS read a
    // pair in the write instead of three (out, run, start)
    __shared__ gint* s_dst[kMaxQ];
    __shared__ unsigned long long s_run[kMaxQ];
    __shared__ gint* s_out[kMaxQ];
    __shared__ uint32_t s_wsum[SW];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const unsigned long long ltmask = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    const uint64_t wc = blockIdx.x;
    const uint32_t np = npairs[wc];
    uint32_t* const list = pairs + wc * cap;
    const uint64_t row0 = (wc / kWaves) * rpb + (wc % kWaves) * (rpb / kWaves);
    for (int i = tid; i < q; i += TPB) {
        s_run[i] = offs[(uint64_t)i * nwc + wc] - offs[(uint64_t)i * nwc];
        s_out[i] = global_ptr(by_arg ? ao.p[i] : outs[i]);
    }
    // (round 4) the wave's 1024 pairs of the next chunk are loaded while this chunk is
    // ranked, sorted and written (the loads of a chunk used to open it: 9 chunks a block
    // at Q = 150, each waiting for its own round trip)
    uint32_t nx[kSpRounds];
    auto load_chunk = [&](uint32_t c0) {
#pragma unroll
        for (int r = 0; r < kSpRounds; r++) {
            const uint32_t idx = c0 + (uint32_t)(wave * kSpPerWave + r * 64 + lane);
            nx[r] = idx < np ? list[idx] : 0u;
        }
    };
    load_chunk(0);
    for (uint32_t c0 = 0; c0 < np; c0 += CH) {
        uint32_t cx[kSpRounds];
#pragma unroll
        for (int r = 0; r < kSpRounds; r++) cx[r] = nx[r];
        if (c0 + CH < np) load_chunk(c0 + CH);
        for (int i = tid; i < SW * kMaxQ; i += TPB) (&s_cnt[0][0])[i] = 0;
        __syncthreads();
        // this wave's 1024 pairs of the chunk
#pragma unroll
        for (int r0 = 0; r0 < kSpRounds; r0 += kSpBatch) {
            uint32_t x[kSpBatch];
#pragma unroll
            for (int b = 0; b < kSpBatch; b++) x[b] = cx[r0 + b];
#pragma unroll
            for (int b = 0; b < kSpBatch; b++) {
                const uint32_t li = (uint32_t)(wave * kSpPerWave + (r0 + b) * 64 + lane);
                const bool valid = c0 + li < np;
                const uint32_t qid = x[b] >> 24, y = x[b];
                const unsigned long long peers = match_any8(qid, __ballot(valid));
                const uint32_t before = valid ? s_cnt[wave][qid] : 0u;
                s_buf[li] = y;
                s_loc[li] = (uint16_t)(before + lanes_below(peers));
                __builtin_amdgcn_wave_barrier();
                if (valid && (peers & ~ltmask & ~(1ull << lane)) == 0)
                    s_cnt[wave][qid] = before + (uint32_t)__popcll(peers);
                __builtin_amdgcn_wave_barrier();
            }
        }
        __syncthreads();
        // bucket starts: queries in order, waves in order inside a query
        uint32_t tq = 0;
        if (tid < q) {
#pragma unroll
            for (int w = 0; w < SW; w++) tq += s_cnt[w][tid];
        }
        uint32_t incl = tq;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(incl, o, 64);
            if (lane >= o) incl += y;
        }
        if (lane == 63) s_wsum[wave] = incl;
        __syncthreads();
        if (tid < q) {
            uint32_t st0 = incl - tq;
            for (int w = 0; w < wave; w++) st0 += s_wsum[w];
            s_dst[tid] = s_out[tid] + ((long long)s_run[tid] - (long long)st0);
            s_tot[tid] = tq;
            uint32_t a = st0;
#pragma unroll
            for (int w = 0; w < SW; w++) {
                const uint32_t c = s_cnt[w][tid];
                s_cnt[w][tid] = a;
                a += c;
            }
        }
        __syncthreads();
        const uint32_t cn = np - c0 < (uint32_t)CH ? np - c0 : (uint32_t)CH;
        uint32_t px[(CH / TPB)], pd[(CH / TPB)];
#pragma unroll
        for (int k = 0; k < (CH / TPB); k++) {
            const uint32_t i = (uint32_t)(k * TPB + tid);
            px[k] = s_buf[i];
            pd[k] = i < cn ? s_cnt[i / kSpPerWave][px[k] >> 24] + s_loc[i] : 0xFFFFFFFFu;
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < (CH / TPB); k++)
            if (pd[k] != 0xFFFFFFFFu) s_buf[pd[k]] = px[k];
        __syncthreads();
        // (round 4) a fixed 16 stores a thread, the slots past the chunk's end going to a
        // pair of this chunk already read (the slice is not read again): with a
        // data-dependent count the wait for the next chunk's loads at the loop's top was
        // vmcnt(0), i.e. also for every store of this chunk
        gint* const dummy = (gint*)(list + c0);
#pragma unroll
        for (int k = 0; k < (CH / TPB); k++) {
            const uint32_t i = (uint32_t)(k * TPB + tid);
            const bool in = i < cn;
            const uint32_t y = s_buf[i], qid = in ? y >> 24 : 0u;
            gint* const dst = in ? s_dst[qid] + i : dummy;
            *dst = (int)(row0 + (y & 0xFFFFFFu)) + base;
        }
        __syncthreads();
        if (tid < q) s_run[tid] += s_tot[tid];
    }
}

// totals[j] = offs[j*nwc + nwc-1] + counts[j*nwc + nwc-1] - offs[j*nwc]
__global__ void k_ss_totals(const uint32_t* __restrict__ counts,
                            const unsigned long long* __restrict__ offs, uint64_t nwc, int q,
                            const int* __restrict__ slot, uint64_t* __restrict__ totals, int qall,
                            const unsigned int* __restrict__ flag, uint64_t* __restrict__ flag_out) {
    if (flag_out && threadIdx.x == 0) *flag_out = *flag;  // the pair slices' overflow word
    for (int i = threadIdx.x; i < qall; i += blockDim.x) {
        const int j = slot[i];
        totals[i] = j < 0 ? 0ull
                          : offs[(uint64_t)j * nwc + nwc - 1] + counts[(uint64_t)j * nwc + nwc - 1] -
                                offs[(uint64_t)j * nwc];
    }
}

// The count pass's offsets and totals in one launch (round 5; was a 3-kernel flat scan
// plus k_ss_totals, ≈ 21 µs): block j scans kernel query j's nwc wave-chunk counts into
// offsets that start at 0 (every reader subtracts the query's first offset), and writes
// the total of each query i with slot[i] == j; block 0 also writes the zero totals of
// the empty queries and, with flag_out, copies the overflow word.
constexpr int kOffTPB = 1024, kOffPer = 8;
__global__ __launch_bounds__(kOffTPB) void k_ss_offsets(const uint32_t* __restrict__ counts,
                                                       unsigned long long* __restrict__ offs, uint64_t nwc,
                                                       const int* __restrict__ slot, uint64_t* __restrict__ totals,
                                                       int qall, const unsigned int* __restrict__ flag,
                                                       uint64_t* __restrict__ flag_out) {
    __shared__ unsigned long long s_w[kOffTPB / 64];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint64_t j = blockIdx.x;
    const uint32_t* c = counts + j * nwc;
    unsigned long long* o = offs + j * nwc;
    unsigned long long carry = 0;
    for (uint64_t b0 = 0; b0 < nwc; b0 += (uint64_t)kOffTPB * kOffPer) {
        const uint64_t i0 = b0 + (uint64_t)tid * kOffPer;
        uint32_t x[kOffPer];
#pragma unroll
        for (int k = 0; k < kOffPer; k++) x[k] = i0 + k < nwc ? c[i0 + k] : 0u;
        unsigned long long t = 0;
#pragma unroll
        for (int k = 0; k < kOffPer; k++) t += x[k];
        unsigned long long incl = t;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const unsigned long long y = __shfl_up(incl, d, 64);
            if (lane >= d) incl += y;
        }
        if (lane == 63) s_w[wave] = incl;
        __syncthreads();
        unsigned long long before = carry, all = 0;
#pragma unroll
        for (int w = 0; w < kOffTPB / 64; w++) {
            const unsigned long long v = s_w[w];
            if (w < wave) before += v;
            all += v;
        }
        unsigned long long run = before + incl - t;
#pragma unroll
        for (int k = 0; k < kOffPer; k++) {
            if (i0 + k < nwc) o[i0 + k] = run;
            run += x[k];
        }
        carry += all;
        __syncthreads();  // s_w is rewritten by the next segment
    }
    for (int i = tid; i < qall; i += kOffTPB) {
        const int sj = slot[i];
        if (sj == (int)j) totals[i] = carry;
        else if (sj < 0 && j == 0) totals[i] = 0ull;
    }
    if (flag_out && j == 0 && tid == 0) *flag_out = *flag;
}

struct SsLayout {
    size_t preds, outs, slot, counts, offs, scratch, ei, flag, npairs, pairs, total;
};

// EI tables in the workspace: bounds, bucket table, qoff, qab, then qlist
constexpr size_t kEiBoundsB = (size_t)kEiMax * 4, kEiBucketB = (size_t)kBuckets * 4,
                 kEiQoffB = (size_t)kEiMax * 4, kEiQabB = (size_t)kMaxQ * 4,
                 kEiQlistB = (size_t)kEiMax * kMaxQ * 2, kEiCellB = (size_t)kCells * 2;
constexpr size_t kEiBytes = kEiBoundsB + kEiBucketB + kEiQoffB + kEiQabB + kEiCellB + kEiQlistB;

SsLayout ss_layout(uint64_t nwc, int q) {
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    SsLayout L;
    size_t at = 0;
    // preds, slot, the flag word and the EI tables are one host upload (ss_count), up to
    // the last query-list entry in use (the EI tables end with the lists)
    L.preds = at;
    at += al((size_t)kMaxQ * sizeof(Pred));
    L.slot = at;
    at += al((size_t)kMaxQ * sizeof(int));
    L.flag = at;
    at += 256;
    L.ei = at;
    at += al(kEiBytes);
    L.outs = at;
    at += al((size_t)kMaxQ * sizeof(int*));
    L.counts = at;
    at += al((size_t)q * nwc * sizeof(uint32_t));
    L.offs = at;
    at += al((size_t)q * nwc * sizeof(unsigned long long));
    L.scratch = at;
    at += al((size_t)scan_u32_scratch_elems((uint64_t)q * nwc) * sizeof(unsigned long long));
    L.npairs = at;
    at += al(nwc * sizeof(uint32_t));
    L.pairs = at;  // pair slices (single pass), when the workspace extends this far
    L.total = at;
    return L;
}

// Host staging for the uploads (pinned, per thread, device and use: 0 = count's
// tables, 1 = write's output pointers). A call waits for the previous call's copy
// out of its buffer (an event recorded behind the copy) before refilling it, so
// neither count nor write synchronises the stream for its uploads.
struct Staging {
    char* p = nullptr;
    size_t cap = 0;
    hipEvent_t ev = nullptr;
};
Staging& staging_slot(int dev, int which) {
    static thread_local Staging st[kMaxDev][3];  // count upload, write upload, count download
    return st[dev][which];
}
}  // namespace

namespace mqi {
// Frees the calling thread's pinned staging on every device (mq_thread_release).
void shared_staging_release() {
    int cur = 0;
    const bool have_cur = hipGetDevice(&cur) == hipSuccess;
    for (int d = 0; d < kMaxDev; d++)
        for (int w = 0; w < 3; w++) {
            Staging& S = staging_slot(d, w);
            if (!S.p && !S.ev) continue;
            if (hipSetDevice(d) != hipSuccess) continue;
            if (S.ev) {
                (void)hipEventSynchronize(S.ev);
                (void)hipEventDestroy(S.ev);
            }
            if (S.p) (void)hipHostFree(S.p);
            S = Staging{};
        }
    if (have_cur) (void)hipSetDevice(cur);
}
}  // namespace mqi

namespace {
int staging_get(int which, size_t bytes, char** p) {
    int dev;
    int rc = current_device(&dev);
    if (rc) return rc;
    Staging& S = staging_slot(dev, which);
    if (S.ev) HIPCHK(hipEventSynchronize(S.ev));
    else HIPCHK(hipEventCreateWithFlags(&S.ev, hipEventDisableTiming));
    if (S.cap < bytes) {
        if (S.p) HIPCHK(hipHostFree(S.p));
        S.p = nullptr;
        S.cap = 0;
        HIPCHK(hipHostMalloc((void**)&S.p, bytes, hipHostMallocDefault));
        S.cap = bytes;
    }
    *p = S.p;
    return MQ_OK;
}
// copies the staged bytes to the device and marks the buffer busy until they are out
int staging_put(int which, void* dst, size_t bytes, hipStream_t st) {
    int dev;
    int rc = current_device(&dev);
    if (rc) return rc;
    Staging& S = staging_slot(dev, which);
    HIPCHK(hipMemcpyAsync(dst, S.p, bytes, hipMemcpyHostToDevice, st));
    HIPCHK(hipEventRecord(S.ev, st));
    return MQ_OK;
}

// Pair-slice capacity: one u32 per row of the wave-chunk.
uint64_t pair_cap(uint64_t rpb) { return rpb / kWaves; }

uint64_t max_wave_chunks(const DevState* s) {
    return (uint64_t)s->cus * 8 * kWaves;  // <= 8 resident blocks per CU
}

}  // namespace

namespace {

// State left in the workspace by the count pass for the write pass.
struct SsState {
    uint32_t g;
    uint64_t rpb;
    int q, qk;
    uint64_t n;
    const int32_t* col;
    EiMeta meta;
    int32_t base;  // first row number of this (row-shard) column
    bool pairs;    // the count pass listed the pairs (single pass)
    bool flag_known;  // the host read the overflow word after the count (flag) ...
    unsigned int flag;
    uint64_t pairs_total;  // ... and the totals (their sum)
    int slot[kMaxQ];  // kernel index of query i, or -1
};

// k_ssk_count's dynamic LDS: bounds and EI offsets (m + 2 words each), the per-wave EI
// histograms, the query lists when they fit (qlcap u16); rounded up to 1 KB so that the
// occupancy cache sees few sizes.
size_t ssk_dyn_bytes(int m, uint32_t qlcap) {
    const size_t hs = (size_t)m + 2;
    const size_t b = hs * 4 * 2 + (size_t)kWaves * hs * 4 + (size_t)qlcap * 2;
    return (b + 1023) & ~(size_t)1023;
}

// Host side of the EI path: bounds, per-query EI ranges, per-EI query lists and
// the bucket table, written to region (pinned staging of the workspace's EI region,
// ss_layout); *used = the bytes in use from its start (the query lists come last, only
// `at` entries of them).
int ei_build(const Pred* hp, int qk, char* region, EiMeta* meta, size_t* used, uint32_t* nql) {
    std::vector<long long> L(qk), H(qk), b;
    b.reserve(2 * qk);
    for (int i = 0; i < qk; i++) {
        L[i] = (long long)(int32_t)hp[i].lo;
        H[i] = L[i] + (long long)hp[i].wm1;
        b.push_back(L[i]);
        if (H[i] + 1 <= (long long)INT32_MAX) b.push_back(H[i] + 1);
    }
    std::sort(b.begin(), b.end());
    b.erase(std::unique(b.begin(), b.end()), b.end());
    const int m = (int)b.size();
    auto eof = [&](long long x) { return (int)(std::upper_bound(b.begin(), b.end(), x) - b.begin()); };
    static thread_local int32_t hb[kEiMax];
    static thread_local uint32_t hbkt[kBuckets], hqoff[kEiMax], hqab[kMaxQ];
    static thread_local uint16_t hql[(size_t)kEiMax * kMaxQ];
    for (int j = 0; j < m; j++) hb[j] = (int32_t)b[j];
    std::vector<int> ea(qk), eb(qk);
    for (int i = 0; i < qk; i++) {
        ea[i] = eof(L[i]);
        eb[i] = eof(H[i]) + 1;
        hqab[i] = (uint32_t)ea[i] | ((uint32_t)eb[i] << 16);
    }
    // per-EI query lists, ascending query index within an EI: counts, offsets, then the
    // queries in index order (O(q + m + entries); a scan of every (EI, query) pair cost
    // m x q host steps a call, 45 K at Q = 150)
    static thread_local uint32_t qfill[kEiMax];
    std::fill(hqoff, hqoff + m + 2, 0u);
    for (int i = 0; i < qk; i++)
        for (int e = ea[i]; e < eb[i]; e++) hqoff[e + 1]++;
    for (int e = 0; e <= m; e++) hqoff[e + 1] += hqoff[e];
    const uint32_t at = hqoff[m + 1];
    std::copy(hqoff, hqoff + m + 1, qfill);
    for (int i = 0; i < qk; i++)
        for (int e = ea[i]; e < eb[i]; e++) hql[qfill[e]++] = (uint16_t)i;
    const long long bmin = b[0], bmax = b[m - 1];
    int shift = 0;
    while (((bmax - bmin) >> shift) >= kBuckets) shift++;
    {  // bucket k: e(its first value) | e(its last value) << 16, both monotone in k
        int el = 0, eh = 0;
        for (int k = 0; k < kBuckets; k++) {
            const long long lo = bmin + ((long long)k << shift);
            if (lo > bmax) {
                hbkt[k] = (uint32_t)m | ((uint32_t)m << 16);
                continue;
            }
            long long hi = lo + (1ll << shift) - 1;
            if (hi > bmax) hi = bmax;
            while (el < m && b[el] <= lo) el++;  // el = eof(lo)
            if (eh < el) eh = el;
            while (eh < m && b[eh] <= hi) eh++;  // eh = eof(hi)
            hbkt[k] = (uint32_t)el | ((uint32_t)eh << 16);
        }
    }
    // k_ssk_count's cell table: one u16 per cell of 2^xshift values from bmin (the last
    // cell also takes every value below bmin and past the table, by the clamp)
    int xshift = 0;
    while (((bmax - bmin) >> xshift) >= kCells - 1) xshift++;
    {
        static thread_local uint16_t hcell[kCells];
        static thread_local int cp[kEiMax + 1];  // covered EIs below e
        cp[0] = 0;
        for (int e = 0; e <= m; e++) cp[e + 1] = cp[e] + (hqoff[e + 1] > hqoff[e] ? 1 : 0);
        int pl = 0, ph = 0;  // e(cell start), e(cell end): monotone over the cells
        for (int c = 0; c < kCells - 1; c++) {
            const long long cs = bmin + ((long long)c << xshift), ce = cs + (1ll << xshift) - 1;
            while (pl < m && b[pl] <= cs) pl++;
            if (ph < pl) ph = pl;
            while (ph < m && b[ph] <= ce) ph++;
            const bool any = cp[ph + 1] - cp[pl] > 0;  // a covered EI among [pl, ph]
            // bounds inside the cell: b[pl .. ph) (ph - pl of them, in the entry when fewer
            // than 7: e(v) = pl + the ones <= v, no search)
            const int nb = ph - pl < 7 ? ph - pl : 0;
            hcell[c] = !any ? (uint16_t)0 : pl == ph ? (uint16_t)(pl + 1) : (uint16_t)(0x8000 | nb << 12 | pl);
        }
        // past bmax's cell every value is in EI m; below bmin (wrapped) in EI 0
        hcell[kCells - 1] = hqoff[m + 1] > hqoff[m] ? (uint16_t)0x8000 : (uint16_t)0;
        std::memcpy(region + kEiBoundsB + kEiBucketB + kEiQoffB + kEiQabB, hcell, kEiCellB);
    }
    *meta = EiMeta{m, shift, (int)bmin, (int)bmax, xshift};
    size_t o = 0;
    std::memcpy(region + o, hb, (size_t)m * 4);
    o += kEiBoundsB;
    std::memcpy(region + o, hbkt, kEiBucketB);
    o += kEiBucketB;
    std::memcpy(region + o, hqoff, (size_t)(m + 2) * 4);
    o += kEiQoffB;
    std::memcpy(region + o, hqab, (size_t)qk * 4);
    o += kEiQabB;
    o += kEiCellB;  // the cell table, written above
    if (at) std::memcpy(region + o, hql, (size_t)at * 2);
    *used = o + (size_t)at * 2;
    *nql = at;
    return MQ_OK;
}

EiTables ei_tables(char* region) {
    EiTables T;
    size_t o = 0;
    T.bounds = reinterpret_cast<const int32_t*>(region + o);
    o += kEiBoundsB;
    T.bucket = reinterpret_cast<const uint32_t*>(region + o);
    o += kEiBucketB;
    T.qoff = reinterpret_cast<const uint32_t*>(region + o);
    o += kEiQoffB;
    T.qab = reinterpret_cast<const uint32_t*>(region + o);
    o += kEiQabB;
    T.cell = reinterpret_cast<const uint16_t*>(region + o);
    o += kEiCellB;
    T.qlist = reinterpret_cast<const uint16_t*>(region + o);
    return T;
}

// d_totals: q totals, and when flag_out the overflow word after them (d_totals[q])
int ss_count(const int32_t* d_col, uint64_t n, int32_t row_base, const int32_t* h_lows,
             const int32_t* h_highs, int q, uint64_t* d_totals, void* d_ws, size_t ws_bytes, hipStream_t st,
             SsState* state, bool flag_out = false) {
    DevState* s;
    int rc = ensure_ready(&s);
    if (rc) return rc;
    if (q < 1 || q > kMaxQ || !h_lows || !h_highs || !d_totals)
        return set_err(MQ_EINVAL, "shared_select: bad argument (q = %d, 1..%d)", q, kMaxQ);
    if (row_base < 0 || (uint64_t)row_base + n > (uint64_t)INT32_MAX)
        return set_err(MQ_EINVAL, "shared_select: rows beyond int32 positions");
    if (!d_ws || ws_bytes < mq_shared_select_workspace_bytes(n, q))
        return set_err(MQ_EINVAL, "shared_select: workspace too small");
    // Queries whose range is empty (high <= low) match nothing and are left out of
    // the kernels; slot[i] = kernel index of query i, or -1.
    static thread_local Pred hp[kMaxQ];
    static thread_local int hslot[kMaxQ];
    int qk = 0;
    for (int i = 0; i < q; i++) {
        Pred p;
        if (n && make_pred(1, h_lows[i], 1, h_highs[i], &p)) {
            hp[qk] = p;
            hslot[i] = qk++;
        } else {
            hslot[i] = -1;
        }
    }
    char* w = static_cast<char*>(d_ws);
    const bool vec = aligned16(d_col);
    // the grid is sized for the kernel that reads the column: the single-pass count,
    // or (MQ_SS_TWOPASS=1: the column pass forced, as a pair-slice overflow takes it)
    // the write pass
    const bool kmajor = getenv("MQ_SS_TWOPASS") == nullptr;
    // k_ssk_count with the next group's loads issued ahead from kSsPfMinQ queries (1e9
    // rows, 0.1 % each, alternating on one box: Q = 150 1.85 -> 1.81 ms, Q = 16 0.93 ->
    // 0.96 ms, where the rounds are few and the stream alone sets the time);
    // MQ_SS_PF=0 / 1 forces it off / on (tuning)
    static const char* pfe = getenv("MQ_SS_PF");
    const bool pf = pfe ? pfe[0] != '0' : qk >= kSsPfMinQ;
    const void* fn = kmajor ? (pf ? (const void*)&k_ssk_count<true> : (const void*)&k_ssk_count<false>)
                            : (vec ? (const void*)&k_ssi_write<true> : (const void*)&k_ssi_write<false>);
    // preds, slot, EI tables and the zeroed flag: one upload from pinned staging (their
    // offsets do not depend on the grid, the EI tables size k_ssk_count's LDS)
    const SsLayout L0 = ss_layout(1, 1);
    char* up = nullptr;
    if ((rc = staging_get(0, L0.outs, &up))) return rc;
    std::memcpy(up + L0.preds, hp, sizeof(Pred) * (qk > 0 ? qk : 1));
    std::memcpy(up + L0.slot, hslot, sizeof(int) * q);
    std::memset(up + L0.flag, 0, 4);
    EiMeta meta{0, 0, 0, 0, 0};
    size_t ei_used = 0;
    uint32_t nql = 0;
    if (qk > 0 && (rc = ei_build(hp, qk, up + L0.ei, &meta, &ei_used, &nql))) return rc;
    const uint32_t qlcap = nql <= (uint32_t)kQlCap ? nql : 0u;
    const size_t dyn = kmajor ? ssk_dyn_bytes(meta.m, qlcap) : 0;
    // blocks a CU for the k-major pass: with the tables in dynamic LDS 5-6 fit, but fewer,
    // longer wave-chunks measured faster (1e9 rows, 0.1 % ranges, count + write, two
    // alternating rounds on one box, profiles/r05_ss_bpc_sweep.log): 3 blocks for Q <= 8
    // (Q = 4 / 8: 0.75 / 0.80 ms against 0.78 / 0.82 at 4), 4 above (Q = 16 / 150: 0.86 /
    // 1.63-1.65 against 0.90 / 1.81 at 3 and 0.89 / 1.65 at the occupancy limit; the
    // static-LDS pass before: 0.86 / 1.68). MQ_SS_BPC overrides (0: occupancy limit).
    const char* bpce = getenv("MQ_SS_BPC");
    const int bpc_cap = bpce ? atoi(bpce) : (qk <= 8 ? 3 : 4);
    uint32_t g = 1;
    uint64_t rpb = kGranule;
    if (n) geometry(s, n, fn, &g, &rpb, kGranule, dyn, kmajor ? bpc_cap : 0);
    const uint64_t nwc = (uint64_t)g * kWaves;
    const SsLayout L = ss_layout(nwc, qk > 0 ? qk : 1);
    const uint64_t cap = pair_cap(rpb);
    const bool single = n && getenv("MQ_SS_TWOPASS") == nullptr &&
                        ws_bytes >= L.pairs + (size_t)nwc * cap * sizeof(uint32_t) && cap < (1ull << 24);
    if ((rc = staging_put(0, w, L.ei + ei_used, st))) return rc;
    uint32_t* counts = reinterpret_cast<uint32_t*>(w + L.counts);
    unsigned long long* offs = reinterpret_cast<unsigned long long*>(w + L.offs);
    if (qk > 0) {
        const EiTables T = ei_tables(w + L.ei);
        if (single) {
            uint32_t* pr = reinterpret_cast<uint32_t*>(w + L.pairs);
            uint32_t* npr = reinterpret_cast<uint32_t*>(w + L.npairs);
            unsigned int* of = reinterpret_cast<unsigned int*>(w + L.flag);
            if (pf)
                hipLaunchKernelGGL((k_ssk_count<true>), dim3(g), dim3(kTPB), dyn, st, d_col, n, rpb, meta, T, qk, counts,
                                   nwc, pr, cap, npr, of, qlcap);
            else
                hipLaunchKernelGGL((k_ssk_count<false>), dim3(g), dim3(kTPB), dyn, st, d_col, n, rpb, meta, T, qk, counts,
                                   nwc, pr, cap, npr, of, qlcap);
            LAUNCHCHK("k_ssk_count");
        } else {
            if (vec)
                hipLaunchKernelGGL(k_ssi_count<true>, dim3(g), dim3(kTPB), 0, st, d_col, n, rpb, meta, T, qk, counts, nwc);
            else
                hipLaunchKernelGGL(k_ssi_count<false>, dim3(g), dim3(kTPB), 0, st, d_col, n, rpb, meta, T, qk, counts, nwc);
            LAUNCHCHK("k_ssi_count");
        }
        hipLaunchKernelGGL(k_ss_offsets, dim3((uint32_t)qk), dim3(kOffTPB), 0, st, counts, offs, nwc,
                           reinterpret_cast<const int*>(w + L.slot), d_totals, q,
                           reinterpret_cast<const unsigned int*>(w + L.flag), flag_out ? d_totals + q : nullptr);
        LAUNCHCHK("k_ss_offsets");
    } else {  // every query empty: zero totals
        hipLaunchKernelGGL(k_ss_totals, dim3(1), dim3(256), 0, st, counts, offs, nwc, qk,
                           reinterpret_cast<const int*>(w + L.slot), d_totals, q,
                           reinterpret_cast<const unsigned int*>(w + L.flag), flag_out ? d_totals + q : nullptr);
        LAUNCHCHK("k_ss_totals");
    }
    state->g = g;
    state->rpb = rpb;
    state->q = q;
    state->qk = qk;
    state->n = n;
    state->col = d_col;
    state->meta = meta;
    state->base = row_base;
    state->pairs = single && qk > 0;
    state->flag_known = false;
    state->flag = 0;
    state->pairs_total = 0;
    std::memcpy(state->slot, hslot, sizeof(int) * q);
    return MQ_OK;
}

// k_ssp_scatter's waves a block: 8 (8192-pair chunks: longer runs per query, half the
// chunks a slice) where the slices average at least 8192 pairs, else 4 (a half-empty
// 8192-pair chunk costs more than it saves). 1e9 rows, 0.1 % ranges, count + write,
// alternating on one box (profiles/r05_ss_scatter_waves_ab.log): Q = 150 1.756 ->
// 1.668 ms with 8; Q = 16 (3.9 K pairs a slice) 0.866 -> 0.890; 16 waves (16384-pair
// chunks, one block a CU) 1.755 / 0.977 (profiles/r05_ss_scatter_waves16_ab.log).
// MQ_SS_SCATTER_WAVES=4|8 forces one (A/B, tests).
int ss_scatter_waves(const SsState& S, uint64_t nwc) {
    const char* e = getenv("MQ_SS_SCATTER_WAVES");
    if (e) return atoi(e) == 8 ? 8 : 4;
    return S.flag_known && nwc && S.pairs_total / nwc >= 8192 ? 8 : 4;
}

int ss_write(const SsState& S, int32_t* const* d_pos_out, void* d_ws, hipStream_t st) {
    if (S.qk == 0) return MQ_OK;
    char* w = static_cast<char*>(d_ws);
    const uint64_t nwc = (uint64_t)S.g * kWaves;
    const SsLayout L = ss_layout(nwc, S.qk);
    // the pair scatter, or (a slice overflowed: the pairs are incomplete) the column
    // pass: both launched, each checks the flag on the device, unless the host read the
    // flag after the count (mq_shared_select_count), then only the one it selects
    const bool scatter = S.pairs && !(S.flag_known && S.flag);
    const bool column = !S.pairs || !S.flag_known || S.flag;
    // the output pointers: in the scatter's arguments when it runs alone on at most
    // kArgQ queries, else uploaded to the workspace
    SsArgOuts ao{};
    const bool by_arg = scatter && !column && S.qk <= kArgQ;
    int rc;
    if (by_arg) {
        for (int i = 0; i < S.q; i++)
            if (S.slot[i] >= 0) ao.p[S.slot[i]] = d_pos_out[i];
    } else {
        char* hp = nullptr;
        if ((rc = staging_get(1, sizeof(int*) * kMaxQ, &hp))) return rc;
        int32_t** hout = reinterpret_cast<int32_t**>(hp);
        for (int i = 0; i < S.q; i++)
            if (S.slot[i] >= 0) hout[S.slot[i]] = d_pos_out[i];
        if ((rc = staging_put(1, w + L.outs, sizeof(int*) * S.qk, st))) return rc;
    }
    const Pred* dp = reinterpret_cast<const Pred*>(w + L.preds);
    const unsigned long long* offs = reinterpret_cast<const unsigned long long*>(w + L.offs);
    int* const* outs = reinterpret_cast<int* const*>(w + L.outs);
    const unsigned int* of = reinterpret_cast<const unsigned int*>(w + L.flag);
    if (scatter) {
        if (ss_scatter_waves(S, nwc) == 8)
            hipLaunchKernelGGL((k_ssp_scatter<8>), dim3((uint32_t)nwc), dim3(512), 0, st,
                               reinterpret_cast<uint32_t*>(w + L.pairs), pair_cap(S.rpb),
                               reinterpret_cast<const uint32_t*>(w + L.npairs), offs, nwc, S.qk, outs, ao, by_arg,
                               S.rpb, S.base, of);
        else
            hipLaunchKernelGGL((k_ssp_scatter<4>), dim3((uint32_t)nwc), dim3(kTPB), 0, st,
                               reinterpret_cast<uint32_t*>(w + L.pairs), pair_cap(S.rpb),
                               reinterpret_cast<const uint32_t*>(w + L.npairs), offs, nwc, S.qk, outs, ao, by_arg,
                               S.rpb, S.base, of);
        LAUNCHCHK("k_ssp_scatter");
    }
    if (!column) return MQ_OK;
    const EiTables T = ei_tables(w + L.ei);
    if (aligned16(S.col))
        hipLaunchKernelGGL(k_ssi_write<true>, dim3(S.g), dim3(kTPB), 0, st, S.col, S.n, S.rpb, S.meta, T, dp, S.qk, offs, nwc, outs, S.base, S.pairs ? of : nullptr);
    else
        hipLaunchKernelGGL(k_ssi_write<false>, dim3(S.g), dim3(kTPB), 0, st, S.col, S.n, S.rpb, S.meta, T, dp, S.qk, offs, nwc, outs, S.base, S.pairs ? of : nullptr);
    LAUNCHCHK("k_ssi_write");
    return MQ_OK;
}

thread_local SsState g_last_state;
thread_local const void* g_last_ws = nullptr;

}  // namespace

extern "C" {

size_t mq_shared_select_workspace_bytes(uint64_t n, int q) {
    DevState* s;
    if (ensure_ready(&s)) return 0;
    if (q < 1) q = 1;
    if (q > kMaxQ) q = kMaxQ;
    const uint64_t nwc = max_wave_chunks(s);
    // + the pair slices of the single pass: one u32 per row, each wave-chunk rounded
    // up to whole granules
    const size_t a = ss_layout(nwc, q).total + (size_t)(n + nwc * kGranule) * sizeof(uint32_t);
    const size_t b = mq_scan_workspace_bytes(n);  // the Q = 1 path of mq_shared_select
    return a > b ? a : b;
}

int mq_shared_select_count(const int32_t* d_col, uint64_t n, const int32_t* h_lows,
                           const int32_t* h_highs, int q, uint64_t* h_counts, void* d_ws,
                           size_t ws_bytes, void* stream) {
    return mq_shared_select_count_at(d_col, n, 0, h_lows, h_highs, q, h_counts, d_ws, ws_bytes, stream);
}

int mq_shared_select_count_at(const int32_t* d_col, uint64_t n, int32_t row_base, const int32_t* h_lows,
                              const int32_t* h_highs, int q, uint64_t* h_counts, void* d_ws,
                              size_t ws_bytes, void* stream) {
    if (!h_counts) return set_err(MQ_EINVAL, "mq_shared_select_count: NULL counts");
    hipStream_t st = (hipStream_t)stream;
    // totals land in the preds region's tail? keep them in their own small buffer
    static thread_local uint64_t* d_tot[kMaxDev];
    int dev;
    int rc = current_device(&dev);
    if (rc) return rc;
    if (!d_tot[dev]) HIPCHK(hipMalloc(&d_tot[dev], (kMaxQ + 1) * sizeof(uint64_t)));
    SsState S;
    if ((rc = ss_count(d_col, n, row_base, h_lows, h_highs, q, d_tot[dev], d_ws, ws_bytes, st, &S, true)))
        return rc;
    // totals and the overflow word through pinned staging (h_counts is the caller's,
    // often pageable: a staged copy costs more); write then launches one kernel
    char* hp = nullptr;
    if (q > 0) {
        if ((rc = staging_get(2, sizeof(uint64_t) * (kMaxQ + 1), &hp))) return rc;
        HIPCHK(hipMemcpyAsync(hp, d_tot[dev], sizeof(uint64_t) * (q + 1), hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        std::memcpy(h_counts, hp, sizeof(uint64_t) * q);
        uint64_t fl;
        std::memcpy(&fl, hp + sizeof(uint64_t) * q, sizeof fl);
        S.flag_known = true;
        S.flag = (unsigned int)fl;
        for (int i = 0; i < q; i++) S.pairs_total += h_counts[i];
    }
    g_last_state = S;
    g_last_ws = d_ws;
    return MQ_OK;
}

int mq_shared_select_write(void* d_ws, int32_t* const* d_pos_out, void* stream) {
    if (!d_ws || d_ws != g_last_ws || !d_pos_out)
        return set_err(MQ_EINVAL, "mq_shared_select_write: no matching mq_shared_select_count");
    return ss_write(g_last_state, d_pos_out, d_ws, (hipStream_t)stream);
}

int mq_shared_select(const int32_t* d_col, uint64_t n, const int32_t* h_lows,
                     const int32_t* h_highs, int q, int32_t* const* d_pos_out,
                     uint64_t* d_counts, void* d_ws, size_t ws_bytes, void* stream) {
    DevState* s;
    int rc = ensure_ready(&s);
    if (rc) return rc;
    if (q < 0 || q > kMaxQ || (q > 0 && (!h_lows || !h_highs || !d_pos_out || !d_counts)))
        return set_err(MQ_EINVAL, "mq_shared_select: bad argument (q = %d, at most %d)", q, kMaxQ);
    if (q == 0) return MQ_OK;
    if (q <= 3) {  // a few queries into capacity-n outputs: one ordered compaction each
        for (int j = 0; j < q; j++)
            if ((rc = mq_select_positions(d_col, nullptr, n, 1, h_lows[j], 1, h_highs[j], d_pos_out[j],
                                          d_counts + j, d_ws, ws_bytes, stream)))
                return rc;
        return MQ_OK;
    }
    SsState S;
    hipStream_t st = (hipStream_t)stream;
    if ((rc = ss_count(d_col, n, 0, h_lows, h_highs, q, d_counts, d_ws, ws_bytes, st, &S))) return rc;
    return ss_write(S, d_pos_out, d_ws, st);
}

}  // extern "C"
