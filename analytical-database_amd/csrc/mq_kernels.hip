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
//   * per-block partial aggregates go to a workspace slab; the last block to
//     arrive folds them in a fixed order (or k_final does, for callers of
//     mq_select_partials), so results are bitwise deterministic.
// Ordered compaction (select_column_scan's ascending position list,
// query.c:92-137) is two kernels: k_scan<MASK> writes one predicate bit per row
// (wave ballots, N/8 bytes) plus per-block counts; k_compact turns the bits into
// positions at offsets from an in-block prefix over the block counts. HBM
// traffic is 4N + N/8 + N/8 + 4K bytes for N rows and K matches.

#include <hip/hip_runtime.h>

#include <atomic>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <vector>
#include <climits>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include <cerrno>
#include <pthread.h>
#include <sched.h>
#include <sys/mman.h>

#ifndef MADV_POPULATE_WRITE
#define MADV_POPULATE_WRITE 23
#endif

#include "mq_common.h"
#include "mq_device.h"
#include "mq_scan_common.h"

// v_writelane through the LLVM intrinsic (this clang has no builtin for it); the
// backend inserts the hazard waits that an inline-asm v_writelane does not.
__device__ int mq_writelane(int src, int lane, int old) __asm("llvm.amdgcn.writelane.i32");

namespace {

using namespace mqi;

__device__ __forceinline__ void store_agent(unsigned long long* p, unsigned long long v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long load_agent(const unsigned long long* p) {
    return __hip_atomic_load(const_cast<unsigned long long*>(p), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
}

// Block-wide combine of per-thread aggregates into part[blockIdx.x]. WT = true
// publishes it write-through (agent-scope relaxed atomic stores, global_store sc1)
// for block_arrive_last's reader on another XCD.
template <bool WT = false>
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
        if constexpr (WT) {
            unsigned long long* w = reinterpret_cast<unsigned long long*>(part + blockIdx.x);
            store_agent(w + 0, r.count);
            store_agent(w + 1, (unsigned long long)r.sum);
            store_agent(w + 2, (unsigned long long)(uint32_t)r.mn | ((unsigned long long)(uint32_t)r.mx << 32));
        } else {
            part[blockIdx.x] = r;
        }
    }
}

// In-kernel combine (replaces the k_final launch on the fused paths). Arrival
// counters: 8 shards (blockIdx % 8, one per XCD under round-robin placement, so no
// word takes more than 1/8 of the arrivals) + a top counter. Zero at module load;
// the last arriver resets them, so consecutive launches on a stream reuse a block
// without a memset. Each (device, stream) owns its own counter block
// (arrive_counters): launches on one stream run in order, so they can share it,
// and launches on different streams never do, however many are in flight.
// Ordering without an L2 writeback: the partial is stored write-through (sc1),
// `s_waitcnt vmcnt(0)` waits for those stores to be acknowledged before the
// arrival add is issued, and the last block reads the partials with sc1 loads.
// (A __threadfence() release here emits buffer_wbl2 per block: measured +70 us
// per 1e9-row launch.) Measured at 1e9 rows: write-through partials alone save
// the k_final launch (-4.5 us); arrivals cost ~6 us and the combine ~4 us, so the
// fused launch ties k_scan + k_final on big scans (both end on a ~5 us latency
// chain) and saves a launch on small ones.
// Each counter sits on its own 4 KiB line: atomics on one line serialise at about
// 12 ns each (2048 arrivals on one line measured +45 us per launch).
constexpr int kArriveStride = 1024;  // uints = 4 KiB
constexpr size_t kArriveBytes = 9 * kArriveStride * sizeof(unsigned int);

// Called by every block after block_store_partial; true in the last block to
// arrive, which then sees every block's partial.
__device__ __forceinline__ bool block_arrive_last(uint32_t nblocks, unsigned int* ctr) {
    __shared__ int s_last;
    if (threadIdx.x == 0) {
        const uint32_t shard = blockIdx.x & 7u;
        const uint32_t shard_n = (nblocks - shard + 7u) / 8u;  // blocks b < nblocks, b % 8 == shard
        __builtin_amdgcn_s_waitcnt(0x0F70);                      // vmcnt(0): partial stores acked
        int last = 0;
        if (__hip_atomic_fetch_add(ctr + shard * kArriveStride, 1u, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT) == shard_n - 1u) {
            const uint32_t nshards = nblocks < 8u ? nblocks : 8u;
            last = __hip_atomic_fetch_add(ctr + 8 * kArriveStride, 1u, __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_AGENT) == nshards - 1u;
        }
        if (last) {
#pragma unroll
            for (int i = 0; i < 9; i++)
                __hip_atomic_store(ctr + i * kArriveStride, 0u, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        }
        s_last = last;
    }
    __syncthreads();
    return s_last != 0;
}

// Block-wide fold of nparts partials into *out (the body of k_final).
__device__ __forceinline__ void block_combine(const Partial* __restrict__ part, uint32_t nparts,
                                              mq_agg* __restrict__ out) {
    unsigned long long cnt = 0;
    long long sum = 0;
    int mn = INT_MAX, mx = INT_MIN;
    // batches of 8 partials per thread with all 24 coherent (sc1) loads in flight
    for (uint32_t base = 0; base < nparts; base += 8 * blockDim.x) {
        unsigned long long c[8], sm[8], m[8];
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const uint32_t i = base + j * blockDim.x + threadIdx.x;
            const unsigned long long* w =  // clamped: unconditional loads, no branches
                reinterpret_cast<const unsigned long long*>(part + (i < nparts ? i : nparts - 1));
            c[j] = load_agent(w + 0);
            sm[j] = load_agent(w + 1);
            m[j] = load_agent(w + 2);
        }
#pragma unroll
        for (int j = 0; j < 8; j++) {
            if (base + j * blockDim.x + threadIdx.x >= nparts) {
                c[j] = 0ull;
                sm[j] = 0ull;
                m[j] = 0x800000007FFFFFFFull;  // {INT_MAX, INT_MIN}
            }
        }
#pragma unroll
        for (int j = 0; j < 8; j++) {
            cnt += c[j];
            sum += (long long)sm[j];
            mn = min(mn, (int)(uint32_t)m[j]);
            mx = max(mx, (int)(uint32_t)(m[j] >> 32));
        }
    }
    __shared__ Partial sc[kWaves];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    cnt = wave_sum_u64(cnt);
    sum = wave_sum_i64(sum);
    mn = wave_min(mn);
    mx = wave_max(mx);
    if (lane == 0) sc[wave] = Partial{cnt, sum, mn, mx, 0ull};
    __syncthreads();
    if (threadIdx.x == 0) {
        Partial r = sc[0];
#pragma unroll
        for (int w = 1; w < kWaves; w++) {
            r.count += sc[w].count;
            r.sum += sc[w].sum;
            r.mn = min(r.mn, sc[w].mn);
            r.mx = max(r.mx, sc[w].mx);
        }
        out->count = r.count;
        out->sum = r.sum;
        out->min = r.mn;
        out->max = r.mx;
        out->_pad = 0;
    }
}

// ---------------------------------------------------------------------------
// k_scan: one streaming pass over a contiguous chunk of the column.
//   kSum   : count + int64 sum of the matching values (select + sum, the metric)
//   kAgg   : count + sum + min + max                       (query.c:306-354, 392-437)
// (select -> fetch -> agg fused, config 3, is k_scan_gather below.)
// Loads are non-temporal dwordx4 (global_load_dwordx4 ... nt): the column is read
// once, and keeping it out of the caches measured 0.586 vs 0.631 ms per 1e9 rows.
// Arithmetic runs on d = v - low (unsigned): a row matches iff d <= wm1, so
//   sum = sum(d) + count * low,  min = low + min(d),  max = low + wm1 - min(wm1 - d)
// where the min()s run over ALL rows of a full tile unmasked: a non-matching row
// has d > wm1 and wm1 - d > wm1, so it can never win.
// ---------------------------------------------------------------------------
enum ScanMode { kSum = 0, kAgg = 1 };

template <int MODE>
struct ScanTraits {
    static constexpr int kUnrollM = MODE == kAgg ? 6 : kUnroll;
};

template <int MODE, bool VEC>
__global__ __launch_bounds__(kTPB, 8) void k_scan(const int* __restrict__ col, uint64_t n,
                                               uint64_t rows_per_block, Pred pred,
                                               Partial* __restrict__ part,
                                               mq_agg* __restrict__ out, unsigned int* __restrict__ arrive) {
    const uint64_t start = (uint64_t)blockIdx.x * rows_per_block;
    uint64_t end = start + rows_per_block;
    if (end > n) end = n;
    const int tid = threadIdx.x;
    const uint32_t lo = pred.lo, wm1 = pred.wm1;

    unsigned int cnt = 0;
    unsigned long long sumd = 0;       // kSum/kAgg: sum of d over matches
    uint32_t mind = 0xFFFFFFFFu;       // kAgg: min d
    uint32_t maxr = 0xFFFFFFFFu;       // kAgg: min (wm1 - d)

    // FULL: all 4 rows valid (no per-row bound check, unmasked min()s)
    auto consume = [&](int4 v, uint64_t tile_row, bool full) {
        const uint64_t row = tile_row + (uint64_t)tid * 4;
        const uint32_t d0 = (uint32_t)v.x - lo, d1 = (uint32_t)v.y - lo, d2 = (uint32_t)v.z - lo,
                       d3 = (uint32_t)v.w - lo;
        bool p0 = d0 <= wm1, p1 = d1 <= wm1, p2 = d2 <= wm1, p3 = d3 <= wm1;
        if (!full) {
            p0 = p0 && (row + 0 < end);
            p1 = p1 && (row + 1 < end);
            p2 = p2 && (row + 2 < end);
            p3 = p3 && (row + 3 < end);
        }
        cnt += (unsigned)p0 + (unsigned)p1 + (unsigned)p2 + (unsigned)p3;
        sumd += (unsigned long long)(p0 ? d0 : 0u) + (unsigned long long)(p1 ? d1 : 0u) +
                (unsigned long long)(p2 ? d2 : 0u) + (unsigned long long)(p3 ? d3 : 0u);
        if constexpr (MODE == kAgg) {
            if (full) {
                mind = min(mind, min(min(d0, d1), min(d2, d3)));
                maxr = min(maxr, min(min(wm1 - d0, wm1 - d1), min(wm1 - d2, wm1 - d3)));
            } else {
                mind = min(mind, min(min(p0 ? d0 : ~0u, p1 ? d1 : ~0u), min(p2 ? d2 : ~0u, p3 ? d3 : ~0u)));
                maxr = min(maxr, min(min(p0 ? wm1 - d0 : ~0u, p1 ? wm1 - d1 : ~0u),
                                     min(p2 ? wm1 - d2 : ~0u, p3 ? wm1 - d3 : ~0u)));
            }
        }
    };

    constexpr int U = ScanTraits<MODE>::kUnrollM;
    uint64_t t = start;
    // Full groups of U tiles: all loads issued before the first use.
    for (; t + (uint64_t)U * kTileRows <= end; t += (uint64_t)U * kTileRows) {
        int4 v[U];
#pragma unroll
        for (int u = 0; u < U; u++)
            v[u] = load4_nt<VEC>(col + t + (uint64_t)u * kTileRows + (uint64_t)tid * 4);
#pragma unroll
        for (int u = 0; u < U; u++) consume(v[u], t + (uint64_t)u * kTileRows, true);
    }
    // Remaining tiles (the chunk tail), bounds-checked per row.
    for (; t < end; t += kTileRows) {
        const uint64_t row = t + (uint64_t)tid * 4;
        int4 v;
        if (row + 3 < end) {
            v = load4_nt<VEC>(col + row);
        } else {
            v.x = row + 0 < end ? col[row + 0] : 0;
            v.y = row + 1 < end ? col[row + 1] : 0;
            v.z = row + 2 < end ? col[row + 2] : 0;
            v.w = row + 3 < end ? col[row + 3] : 0;
        }
        consume(v, t, row + 3 < end);
    }
    // Back from d-space to values (exact: low + d never wraps for a matching row).
    const long long sum = (long long)sumd + (long long)cnt * (long long)(int32_t)lo;
    int mn = INT_MAX, mx = INT_MIN;
    if (MODE == kAgg && cnt) {
        mn = (int)(lo + mind);
        mx = (int)(lo + (wm1 - maxr));
    }
    // out != nullptr: the last block to finish folds all partials (no k_final launch)
    if (out) {
        block_store_partial<true>(cnt, sum, mn, mx, part);
        if (block_arrive_last(gridDim.x, arrive)) block_combine(part, gridDim.x, out);
    } else {
        block_store_partial(cnt, sum, mn, mx, part);
    }
}

// k_stream_read: the achievable HBM read ceiling for this access pattern (SURVEY
// §8(d) "achievable peak"): k_scan's chunking, nt dwordx4 loads and 8 tiles in
// flight, with no predicate; each block stores the xor of its chunk so the loads
// are live. Rows past the last full 8-tile group are not read (n is the bench's
// 1e9 = a multiple of 8192 x blocks in practice; the byte count reported is the
// number actually read, see mq_stream_read).
template <bool VEC>
__global__ __launch_bounds__(kTPB, 8) void k_stream_read(const int* __restrict__ col, uint64_t n,
                                                         uint64_t rows_per_block,
                                                         uint32_t* __restrict__ out) {
    const uint64_t start = (uint64_t)blockIdx.x * rows_per_block;
    uint64_t end = start + rows_per_block;
    if (end > n) end = n;
    const int tid = threadIdx.x;
    uint32_t x = 0;
    for (uint64_t t = start; t + 8ull * kTileRows <= end; t += 8ull * kTileRows) {
        int4 v[8];
#pragma unroll
        for (int u = 0; u < 8; u++)
            v[u] = load4_nt<VEC>(col + t + (uint64_t)u * kTileRows + (uint64_t)tid * 4);
#pragma unroll
        for (int u = 0; u < 8; u++) x ^= (uint32_t)(v[u].x ^ v[u].y ^ v[u].z ^ v[u].w);
    }
    x = (uint32_t)wave_sum_u64(x);
    if ((tid & 63) == 0) atomicXor(out + blockIdx.x, x);
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
// k_select_stage: ordered compaction in ONE launch (select_column_scan /
// select_result, query.c:38-137). Default positions path.
//   * block b's 4 waves each own a contiguous run of rw rows (wave unit
//     u = 4b + w, rows [u*rw, (u+1)*rw)) and stream it like k_scan (nt dwordx4,
//     8 x 256-row wave tiles in flight);
//   * positions mode: a tile's matches are ranked by 4 ballots (mbcnt) and
//     appended in row order to the wave's 1024-entry LDS ring; when the ring is
//     full its oldest entries spill to the wave's own workspace slice, as long as
//     the spilled positions take no more bytes than the bitmap of the rows already
//     scanned would (match density below 1/32);
//   * bitmap mode: past that, the wave stores each tile's 4 ballot words (32 B per
//     256 rows) to the workspace instead, like k_mask, and counts;
//   * end: each block publishes its count ({done, count} in one 64-bit word) and
//     sums ALL lower blocks' words in one parallel sweep (blocks finish together,
//     so a look-back chain would serialise); each wave then writes its buffer to
//     out[D ...] and expands its bitmap tiles after it, like k_compact.
// Every output word is written once, at its final place (no staging in the output,
// so no write-after-read between blocks). HBM traffic: 4N + 4K + 2 x (N_b/8) where
// N_b is the rows scanned in bitmap mode (0 for sparse waves, ~N at high
// selectivity). Blocks wait only for blocks with lower blockIdx, at the very end:
// workgroups are dispatched in grid order, so those are running or done (spins are
// bounded; a timeout sets the error word and poisons the count).
// ---------------------------------------------------------------------------
constexpr int kStTiles = 8;                        // wave tiles (256 rows) in flight per lane
constexpr int kStGranule = 256 * kStTiles;         // rows per wave iteration
constexpr int kStBuf = 1024;                       // LDS positions per wave
constexpr unsigned long long kStDone = 1ull << 63;

__device__ __forceinline__ uint32_t rank_lt(unsigned long long m, uint32_t acc) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, acc));
}

struct StageState {
    uint32_t fill;     // matches appended in positions mode (monotonic)
    uint32_t flushed;  // ... of which the oldest `flushed` spilled to the workspace
    uint32_t nbm;      // matches recorded in the bitmap (bitmap mode)
    uint64_t sw;       // first row in bitmap mode (a tile boundary); E = never
    bool bmode;        // wave-uniform
};

// One 256-row wave tile starting at row t0: lane l holds rows t0+4l .. t0+4l+3.
// Positions mode: matches go to the wave's LDS ring (BUF entries, entry i at
// ring[i % BUF]); when a tile does not fit, the oldest entries spill, 64 at a time,
// to the start of the wave's own workspace slice (`spill`, the bytes its bitmap
// would use) while the spilled positions take no more room than the bitmap of the
// rows already finished (<= 8 per tile before the current iteration, tile r0):
// density < 1/32, where positions are the smaller form. Past that: bitmap mode.
// Bitmap mode inside the unrolled loop (J >= 0): tile J's ballot e goes to lane 4J+e
// of the iteration's 256-byte record (rlo/rhi), stored by the caller after the next
// iteration's loads are issued. J < 0 (the tail): stored at once.
// Rows are 32-bit here: positions are int32, so n < 2^31 (mq_select_positions).
template <bool PAYLOAD, int BUF, bool FULL, int J>
__device__ __forceinline__ void stage_tile(StageState& st, int4 v, uint32_t t0, uint32_t E, uint32_t lo,
                                           uint32_t wm1, int32_t base, int lane, int* buf,
                                           const int* __restrict__ payload,
                                           unsigned long long* __restrict__ bm, int* __restrict__ spill,
                                           uint32_t r0, int& rlo, int& rhi) {
    const uint32_t row0 = t0 + (uint32_t)lane * 4;
    bool p0 = ((uint32_t)v.x - lo) <= wm1, p1 = ((uint32_t)v.y - lo) <= wm1,
         p2 = ((uint32_t)v.z - lo) <= wm1, p3 = ((uint32_t)v.w - lo) <= wm1;
    if (!FULL) {
        p0 = p0 && row0 + 0 < E;
        p1 = p1 && row0 + 1 < E;
        p2 = p2 && row0 + 2 < E;
        p3 = p3 && row0 + 3 < E;
    }
    const unsigned long long m0 = __ballot(p0), m1 = __ballot(p1), m2 = __ballot(p2),
                             m3 = __ballot(p3);
    // all state is wave-uniform; readfirstlane keeps it in SGPRs
    const uint32_t c = __builtin_amdgcn_readfirstlane(
        (uint32_t)(__popcll(m0) + __popcll(m1) + __popcll(m2) + __popcll(m3)));
    if (!st.bmode) {
        if (c == 0) return;
        const uint32_t over = st.fill + c - st.flushed;
        const uint32_t need = __builtin_amdgcn_readfirstlane(
            over > (uint32_t)BUF ? ((over - (uint32_t)BUF + 63u) & ~63u) : 0u);
        if (st.flushed + need <= 8u * r0) {
            if (need) {
                __builtin_amdgcn_wave_barrier();
                for (uint32_t f = 0; f < need; f += 64u) {  // spill the oldest entries, 64 at a time
                    const uint32_t i = st.flushed + f + (uint32_t)lane;
                    spill[i] = buf[i % (uint32_t)BUF];
                }
                st.flushed = __builtin_amdgcn_readfirstlane(st.flushed + need);
            }
            uint32_t k = rank_lt(m3, rank_lt(m2, rank_lt(m1, rank_lt(m0, st.fill))));
            if (p0) buf[(k++) % (uint32_t)BUF] = PAYLOAD ? payload[row0 + 0] : (int)(row0 + 0) + base;
            if (p1) buf[(k++) % (uint32_t)BUF] = PAYLOAD ? payload[row0 + 1] : (int)(row0 + 1) + base;
            if (p2) buf[(k++) % (uint32_t)BUF] = PAYLOAD ? payload[row0 + 2] : (int)(row0 + 2) + base;
            if (p3) buf[(k++) % (uint32_t)BUF] = PAYLOAD ? payload[row0 + 3] : (int)(row0 + 3) + base;
            st.fill = __builtin_amdgcn_readfirstlane(st.fill + c);
            return;
        }
        st.bmode = true;
        st.sw = t0;
    }
    if (J >= 0) {
        rlo = mq_writelane((int)m0, 4 * J + 0, rlo);
        rhi = mq_writelane((int)(m0 >> 32), 4 * J + 0, rhi);
        rlo = mq_writelane((int)m1, 4 * J + 1, rlo);
        rhi = mq_writelane((int)(m1 >> 32), 4 * J + 1, rhi);
        rlo = mq_writelane((int)m2, 4 * J + 2, rlo);
        rhi = mq_writelane((int)(m2 >> 32), 4 * J + 2, rhi);
        rlo = mq_writelane((int)m3, 4 * J + 3, rlo);
        rhi = mq_writelane((int)(m3 >> 32), 4 * J + 3, rhi);
    } else if (lane < 4) {
        bm[(uint64_t)(t0 >> 8) * 4 + (uint64_t)lane] = lane == 0 ? m0 : lane == 1 ? m1 : lane == 2 ? m2 : m3;
    }
    st.nbm = __builtin_amdgcn_readfirstlane(st.nbm + c);
}

// select_result's payload rows r .. r+3 of a 256-row tile (r = tile * 256 + 4 lane):
// one nontemporal dwordx4 where the payload is 16-byte aligned and the rows exist (every
// tile but the column's last), else four dword loads with the indices clamped. Four
// dword loads per lane issued the same lines as 4 instructions; one dwordx4 moves the
// wave's 1 KiB in one.
__device__ __forceinline__ void load_pay4(int (&pv)[4], const int* __restrict__ payload, uint64_t r, uint64_t n,
                                          bool pal) {
    if (pal && r + 3 < n) {
        const int4 x = load4_nt<true>(payload + r);
        pv[0] = x.x;
        pv[1] = x.y;
        pv[2] = x.z;
        pv[3] = x.w;
    } else {
#pragma unroll
        for (int e = 0; e < 4; e++) pv[e] = payload[r + e < n ? r + e : n - 1];
    }
}

template <bool PAYLOAD, bool VEC, int BUF = kStBuf>
__global__ __launch_bounds__(kTPB, 8) void k_select_stage(
    const int* __restrict__ col, const int* __restrict__ payload, uint64_t n, uint64_t rw, Pred pred,
    unsigned long long* status, unsigned long long* __restrict__ bm, int* __restrict__ out,
    unsigned long long* __restrict__ d_count, unsigned int* err) {
    __shared__ __attribute__((aligned(16))) int s_buf[kWaves][BUF > 0 ? BUF : 1];
    __shared__ unsigned int s_cnt[kWaves];
    __shared__ unsigned long long s_red[kWaves];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t lo = pred.lo, wm1 = pred.wm1;
    const int32_t rbase = pred.base;
    const uint32_t b = blockIdx.x;
    uint64_t S = ((uint64_t)b * kWaves + (uint64_t)wave) * rw;
    if (S > n) S = n;
    uint64_t E = S + rw;
    if (E > n) E = n;
    StageState st{0u, 0u, 0u, E, false};
    int* spill = reinterpret_cast<int*>(bm + (S >> 8) * 4);  // this wave's workspace slice
    int rlo = 0, rhi = 0;           // bitmap record of the current iteration
    unsigned long long rec = 0;     // ... and of the previous one, pending store
    uint32_t rec_at = ~0u;          // its first tile (global index), ~0 = none
    const uint32_t S32 = (uint32_t)S, E32 = (uint32_t)E;
    uint32_t t = S32;
    for (; t + kStGranule <= E32; t += kStGranule) {
        const int* base = col + t;  // wave-uniform
        int4 v[kStTiles];
#pragma unroll
        for (int j = 0; j < kStTiles; j++) v[j] = load4_nt<VEC>(base + (uint32_t)(j * 256 + lane * 4));
        // vmcnt retires loads and stores in order: storing the previous record only
        // now keeps its write round trip off this iteration's first wait (k_mask)
        if (rec_at != ~0u && lane < 32) bm[(uint64_t)rec_at * 4 + (uint64_t)lane] = rec;
        rec_at = ~0u;
        const uint32_t r0 = (t - S32) >> 8;  // this iteration's first tile in the wave's slice
#pragma unroll
        for (int j = 0; j < kStTiles; j++) {
            switch (j) {  // J must be a constant for the writelane lane index
#define MQ_ST(JJ) case JJ: stage_tile<PAYLOAD, BUF, true, JJ>(st, v[JJ], t + JJ * 256, E32, lo, wm1, rbase, lane, s_buf[wave], payload, bm, spill, r0, rlo, rhi); break;
                MQ_ST(0) MQ_ST(1) MQ_ST(2) MQ_ST(3) MQ_ST(4) MQ_ST(5) MQ_ST(6) MQ_ST(7)
#undef MQ_ST
            }
        }
        if (st.bmode) {  // words of tiles before the switch are garbage and never read
            rec = (unsigned long long)(uint32_t)rlo | ((unsigned long long)(uint32_t)rhi << 32);
            rec_at = t >> 8;
        }
    }
    if (rec_at != ~0u && lane < 32) bm[(uint64_t)rec_at * 4 + (uint64_t)lane] = rec;
    for (; t < E32; t += 256) {  // the last unit's tail, one wave tile at a time
        const uint32_t row = t + (uint32_t)lane * 4;
        int4 v;
        v.x = row + 0 < E32 ? col[row + 0] : 0;
        v.y = row + 1 < E32 ? col[row + 1] : 0;
        v.z = row + 2 < E32 ? col[row + 2] : 0;
        v.w = row + 3 < E32 ? col[row + 3] : 0;
        stage_tile<PAYLOAD, BUF, false, -1>(st, v, t, E32, lo, wm1, rbase, lane, s_buf[wave], payload, bm, spill,
                                            (t - S32) >> 8, rlo, rhi);
    }
    int* buf = s_buf[wave];
    const uint32_t fill = st.fill, nbm = st.nbm, flushed = st.flushed;
    const uint64_t sw = st.sw;

    // ---- block count, then the exclusive prefix over every lower block
    const uint32_t mine = fill + nbm;
    if (lane == 0) s_cnt[wave] = mine;
    __syncthreads();
    unsigned long long blk = 0;
#pragma unroll
    for (int w = 0; w < kWaves; w++) blk += s_cnt[w];
    if (tid == 0) store_agent(&status[b], kStDone | blk);
    unsigned long long acc = 0;
    for (uint32_t i = tid; i < b; i += kTPB) {
        unsigned long long x;
        unsigned int spins = 0;
        while (!((x = load_agent(&status[i])) & kStDone)) {
            if (++spins > (1u << 26)) {  // never expected; fail loudly, never hang
                atomicOr(err, 1u);
                x = kStDone;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        acc += x & ~kStDone;
    }
    acc = wave_sum_u64(acc);
    if (lane == 0) s_red[wave] = acc;
    __syncthreads();
    unsigned long long D = 0;
#pragma unroll
    for (int w = 0; w < kWaves; w++) D += s_red[w];
    if (b == gridDim.x - 1 && tid == 0)
        *d_count = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ? ~0ull : D + blk;
#pragma unroll
    for (int w = 0; w < kWaves; w++)
        if (w < wave) D += s_cnt[w];

    // ---- positions mode part: the spilled entries, then the LDS ring, in order
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's spill/bitmap stores are done
    for (uint32_t i0 = 0; i0 < flushed; i0 += 64u * 8u) {  // 8 loads in flight per lane
        int x[8];
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const uint32_t i = i0 + (uint32_t)j * 64u + (uint32_t)lane;
            x[j] = i < flushed ? spill[i] : 0;
        }
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const uint32_t i = i0 + (uint32_t)j * 64u + (uint32_t)lane;
            if (i < flushed) out[D + i] = x[j];
        }
    }
    __builtin_amdgcn_wave_barrier();
    for (uint32_t i = flushed + (uint32_t)lane; i < fill; i += 64u) out[D + i] = buf[i % (uint32_t)BUF];
    if (sw >= E) return;
    // ---- bitmap mode part: 64 tiles per step, one lane per tile (k_compact's scheme)
    unsigned long long o = D + fill;
    const uint64_t T1 = (E + 255) >> 8;
    const bool pal = PAYLOAD && ((reinterpret_cast<uintptr_t>(payload) & 15u) == 0);
    // ring entries [bst, bst + bfill) go to out[ob ...]; bst = out + ob's
    // dword offset within its 16 bytes
    unsigned long long ob = o;
    uint32_t bfill = 0, bst = (uint32_t)(((uintptr_t)(out + ob) >> 2) & 3u);
    auto flush = [&]() {
        __builtin_amdgcn_wave_barrier();
        const uint32_t end = bst + bfill;
        int* base = out + ob - bst;  // base + q is 16-byte aligned for q % 4 == 0
        for (uint32_t q = 4u * (uint32_t)lane; q < end; q += 256u) {
            if (q >= bst && q + 4u <= end) {
                *reinterpret_cast<int4*>(base + q) = *reinterpret_cast<const int4*>(buf + q);
            } else {
#pragma unroll
                for (uint32_t e = 0; e < 4; e++)
                    if (q + e >= bst && q + e < end) base[q + e] = buf[q + e];
            }
        }
        __builtin_amdgcn_wave_barrier();
        ob += bfill;
        bfill = 0;
        bst = (uint32_t)(((uintptr_t)(out + ob) >> 2) & 3u);
    };
    for (uint64_t tb = sw >> 8; tb < T1; tb += 64) {
        const uint64_t T = tb + (uint64_t)lane;
        unsigned long long w0 = 0, w1 = 0, w2 = 0, w3 = 0;
        if (T < T1) {
            const ulonglong2 a = reinterpret_cast<const ulonglong2*>(bm + T * 4)[0];
            const ulonglong2 c2 = reinterpret_cast<const ulonglong2*>(bm + T * 4)[1];
            w0 = a.x;
            w1 = a.y;
            w2 = c2.x;
            w3 = c2.y;
        }
        const unsigned int c = (unsigned int)(__popcll(w0) + __popcll(w1) + __popcll(w2) + __popcll(w3));
        unsigned int tot = c;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) tot += __shfl_xor(tot, off, 64);
        // batched (round 4): tiles' outputs gathered in row order in the wave's LDS ring
        // (free now: its entries went out above), placed so that ring index and output
        // address agree mod 16 bytes, and flushed when the next tile would not fit as
        // 16-byte stores, 64 lanes per instruction. Stored straight from the lanes' rows,
        // every store instruction's addresses had gaps wherever a row does not match
        // (round 4: 1.064 / 1.475 / 1.84 -> 1.022 / 1.355 / 1.56 ms at 10 / 50 / 100 %,
        // profiles/r04_positions_batched_ab.log). select_result: the payload rows of 4
        // tiles are loaded before any of them is placed.
        constexpr int kPf = PAYLOAD ? 4 : 1;
        for (int j0 = 0; j0 < 64; j0 += kPf) {
            int pv[kPf][4];
            if constexpr (PAYLOAD) {
#pragma unroll
                for (int jj = 0; jj < kPf; jj++) {
                    const uint64_t r = (tb + (uint64_t)(j0 + jj)) * 256 + 4 * (uint64_t)lane;
                    const bool any = __builtin_amdgcn_readlane((int)c, j0 + jj) != 0;
                    if (any) load_pay4(pv[jj], payload, r, n, pal);
                }
            }
#pragma unroll
            for (int jj = 0; jj < kPf; jj++) {
                const int j = j0 + jj;
                const uint32_t cj = (uint32_t)__builtin_amdgcn_readlane((int)c, j);
                if (cj == 0) continue;
                if (bst + bfill + cj > (uint32_t)BUF) flush();
                auto rl64 = [&](unsigned long long x) {
                    return (unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, j) |
                           ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), j) << 32);
                };
                const unsigned long long x0 = rl64(w0), x1 = rl64(w1), x2 = rl64(w2), x3 = rl64(w3);
                const int rj = (int)((tb + (uint64_t)j) * 256 + 4 * (uint64_t)lane) + rbase;
                uint32_t k = bst + bfill + rank_lt(x3, rank_lt(x2, rank_lt(x1, rank_lt(x0, 0u))));
                if ((x0 >> lane) & 1ull) buf[k++] = PAYLOAD ? pv[jj][0] : rj + 0;
                if ((x1 >> lane) & 1ull) buf[k++] = PAYLOAD ? pv[jj][1] : rj + 1;
                if ((x2 >> lane) & 1ull) buf[k++] = PAYLOAD ? pv[jj][2] : rj + 2;
                if ((x3 >> lane) & 1ull) buf[k++] = PAYLOAD ? pv[jj][3] : rj + 3;
                bfill += cj;
            }
        }
        o += tot;
    }
    if (bfill) flush();
}

// ---------------------------------------------------------------------------
// hashset.c lookup (hashset.c:35-45): one probe per lane along the reference's
// linear sequence from key % size; 0 marks an empty slot.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kTPB) void k_hashset_lookup(const int32_t* __restrict__ table, int32_t size,
                                                         const int32_t* __restrict__ probe, uint64_t n,
                                                         uint8_t* __restrict__ found) {
    const uint64_t stride = (uint64_t)gridDim.x * kTPB;
    for (uint64_t i = (uint64_t)blockIdx.x * kTPB + threadIdx.x; i < n; i += stride) {
        const int32_t key = probe[i];
        int32_t idx = key % size;  // hash() of multimap.c:60-63
        if (idx < 0) idx += size;  // the reference indexes out of bounds here
        int32_t v = table[idx];
        for (int32_t step = 1; v != 0 && v != key && step < size; step++) {
            idx = idx + 1 == size ? 0 : idx + 1;
            v = table[idx];
        }
        found[i] = (v != 0 && v == key) ? 1 : 0;
    }
}

// ---------------------------------------------------------------------------
// fetch (query.c:223-243): out[i] = col[pos[i]], 4 positions per lane.
// ---------------------------------------------------------------------------
template <bool VEC>
__device__ __forceinline__ void store4(int* __restrict__ p, int4 v) {
    if constexpr (VEC) {
        *reinterpret_cast<int4*>(p) = v;
    } else {
        p[0] = v.x;
        p[1] = v.y;
        p[2] = v.z;
        p[3] = v.w;
    }
}

template <bool VEC>
__global__ __launch_bounds__(kTPB) void k_fetch(const int* __restrict__ col,
                                                const int* __restrict__ pos, uint64_t k,
                                                int* __restrict__ out) {
    // kFetchU groups of 4 positions per lane per step: all position loads, then all
    // 4 x kFetchU gathers, are in flight before any result is used (one group at a
    // time left the lane with two serial round trips per 4 gathers). The main loop
    // runs whole steps only: no guard inside, so the compiler cannot sink the loads
    // back to their stores.
    constexpr int kFetchU = 4;
    const uint64_t stride = (uint64_t)gridDim.x * kTPB;
    const uint64_t k4 = k / 4;
    uint64_t i0 = (uint64_t)blockIdx.x * kTPB + threadIdx.x;
    for (; i0 + (uint64_t)(kFetchU - 1) * stride < k4; i0 += stride * kFetchU) {
        int4 p[kFetchU], o[kFetchU];
#pragma unroll
        for (int u = 0; u < kFetchU; u++) p[u] = load4<VEC>(pos + (i0 + (uint64_t)u * stride) * 4);
#pragma unroll
        for (int u = 0; u < kFetchU; u++) {
            o[u].x = col[p[u].x];
            o[u].y = col[p[u].y];
            o[u].z = col[p[u].z];
            o[u].w = col[p[u].w];
        }
#pragma unroll
        for (int u = 0; u < kFetchU; u++) store4<VEC>(out + (i0 + (uint64_t)u * stride) * 4, o[u]);
    }
    for (; i0 < k4; i0 += stride) {  // the last partial step, one group at a time
        const int4 p = load4<VEC>(pos + i0 * 4);
        store4<VEC>(out + i0 * 4, make_int4(col[p.x], col[p.y], col[p.z], col[p.w]));
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

// ---------------------------------------------------------------------------
// k_scan_gather: config 3 fused (select col -> fetch aux -> agg; query.c:92-137,
// 223-243, 306-354) with the gather deferred. Loading aux[row] inline at each match
// made every tile with a match wait a full random-read latency before the next tile's
// loads went out (0.975 vs 0.779 ms at 1e9, 1 %; that form was removed in round 6).
// Here the scan streams like k_scan<kSum> (8 tiles of
// nt dwordx4 in flight) and each wave appends its matching rows (as offsets from
// the block's first row) to a 1024-entry LDS buffer, ranked with 4 ballots +
// mbcnt. When a tile would overflow the buffer, and at the end, the wave drains it:
// 8 independent aux loads per lane in flight, folded into count/sum/min/max, in
// k_scan's partial slab and in-kernel combine.
// ---------------------------------------------------------------------------
constexpr int kGBuf = 1024;

template <bool VEC>
__global__ __launch_bounds__(kTPB, 6) void k_scan_gather(const int* __restrict__ col,
                                                         const int* __restrict__ aux, uint64_t n,
                                                         uint64_t rows_per_block, Pred pred,
                                                         Partial* __restrict__ part,
                                                         mq_agg* __restrict__ out, unsigned int* __restrict__ arrive) {
    __shared__ uint32_t s_buf[kWaves][kGBuf];
    const uint64_t start = (uint64_t)blockIdx.x * rows_per_block;
    uint64_t end = start + rows_per_block;
    if (end > n) end = n;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t lo = pred.lo, wm1 = pred.wm1;
    uint32_t* buf = s_buf[wave];
    const int* auxb = aux + start;
    uint32_t fill = 0;  // wave-uniform
    unsigned long long cnt = 0;
    long long sumv = 0;
    int mnv = INT_MAX, mxv = INT_MIN;

    auto drain = [&]() {
        __builtin_amdgcn_wave_barrier();
        for (uint32_t i0 = 0; i0 < fill; i0 += 64u * 8u) {
            int x[8];
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const uint32_t i = i0 + (uint32_t)j * 64u + (uint32_t)lane;
                x[j] = i < fill ? auxb[buf[i]] : 0;
            }
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const uint32_t i = i0 + (uint32_t)j * 64u + (uint32_t)lane;
                if (i < fill) {
                    sumv += x[j];
                    mnv = min(mnv, x[j]);
                    mxv = max(mxv, x[j]);
                }
            }
        }
        __builtin_amdgcn_wave_barrier();
        fill = 0;
    };
    auto consume = [&](int4 v, uint64_t tile_row, bool full) {
        const uint64_t row = tile_row + (uint64_t)tid * 4;
        bool p0 = ((uint32_t)v.x - lo) <= wm1, p1 = ((uint32_t)v.y - lo) <= wm1,
             p2 = ((uint32_t)v.z - lo) <= wm1, p3 = ((uint32_t)v.w - lo) <= wm1;
        if (!full) {
            p0 = p0 && row + 0 < end;
            p1 = p1 && row + 1 < end;
            p2 = p2 && row + 2 < end;
            p3 = p3 && row + 3 < end;
        }
        const unsigned long long m0 = __ballot(p0), m1 = __ballot(p1), m2 = __ballot(p2),
                                 m3 = __ballot(p3);
        const uint32_t c = __builtin_amdgcn_readfirstlane(
            (uint32_t)(__popcll(m0) + __popcll(m1) + __popcll(m2) + __popcll(m3)));
        if (c == 0) return;
        cnt += c;
        if (fill + c > (uint32_t)kGBuf) drain();
        uint32_t k = rank_lt(m3, rank_lt(m2, rank_lt(m1, rank_lt(m0, fill))));
        const uint32_t r = (uint32_t)(row - start);
        if (p0) buf[k++] = r + 0;
        if (p1) buf[k++] = r + 1;
        if (p2) buf[k++] = r + 2;
        if (p3) buf[k++] = r + 3;
        fill = __builtin_amdgcn_readfirstlane(fill + c);
    };

    constexpr int U = 8;
    uint64_t t = start;
    for (; t + (uint64_t)U * kTileRows <= end; t += (uint64_t)U * kTileRows) {
        int4 v[U];
#pragma unroll
        for (int u = 0; u < U; u++)
            v[u] = load4_nt<VEC>(col + t + (uint64_t)u * kTileRows + (uint64_t)tid * 4);
#pragma unroll
        for (int u = 0; u < U; u++) consume(v[u], t + (uint64_t)u * kTileRows, true);
    }
    for (; t < end; t += kTileRows) {
        const uint64_t row = t + (uint64_t)tid * 4;
        int4 v;
        if (row + 3 < end) {
            v = load4_nt<VEC>(col + row);
        } else {
            v.x = row + 0 < end ? col[row + 0] : 0;
            v.y = row + 1 < end ? col[row + 1] : 0;
            v.z = row + 2 < end ? col[row + 2] : 0;
            v.w = row + 3 < end ? col[row + 3] : 0;
        }
        consume(v, t, row + 3 < end);
    }
    drain();
    // cnt is wave-uniform: count it once per wave (lane 0) in the block sum
    const unsigned long long c_lane = lane == 0 ? cnt : 0ull;
    if (out) {
        block_store_partial<true>(c_lane, sumv, mnv, mxv, part);
        if (block_arrive_last(gridDim.x, arrive)) block_combine(part, gridDim.x, out);
    } else {
        block_store_partial(c_lane, sumv, mnv, mxv, part);
    }
}

__global__ __launch_bounds__(kTPB) void k_gen_join(int* __restrict__ out, uint64_t n, int kind) {
    const uint64_t stride = (uint64_t)gridDim.x * kTPB;
    const uint64_t mask = 2 * n - 1;
    for (uint64_t i = (uint64_t)blockIdx.x * kTPB + threadIdx.x; i < n; i += stride) {
        if (kind == 0) out[i] = (int)mix31((uint32_t)i);
        else if (kind == 1) out[i] = (int)mix31((uint32_t)(sm64((7ull << 40) | i) & mask));
        else if (kind == 2) out[i] = (int)mix31((uint32_t)(i % (n / 2 ? n / 2 : 1)));  // every key twice
        else out[i] = (int)mix31((uint32_t)(sm64((7ull << 40) | i) & (n - 1)));       // about half hit
    }
}

// Device-to-device copy (mq_memcpy_d2d): 16-byte words grid-stride, 4 in flight per
// lane; the byte tail by the first threads. hipMemcpyAsync D2D measured 23 ms for
// 40 MB on the API path (an engine copy behind the stream); this runs at HBM speed.
__global__ __launch_bounds__(kTPB) void k_copy16(uint4* __restrict__ dst, const uint4* __restrict__ src,
                                                 uint64_t n16, unsigned char* __restrict__ dtail,
                                                 const unsigned char* __restrict__ stail, uint32_t ntail) {
    const uint64_t stride = (uint64_t)gridDim.x * kTPB;
    uint64_t i = (uint64_t)blockIdx.x * kTPB + threadIdx.x;
    for (; i + 3 * stride < n16; i += 4 * stride) {
        const uint4 a = src[i], b = src[i + stride], c = src[i + 2 * stride], d = src[i + 3 * stride];
        dst[i] = a;
        dst[i + stride] = b;
        dst[i + 2 * stride] = c;
        dst[i + 3 * stride] = d;
    }
    for (; i < n16; i += stride) dst[i] = src[i];
    const uint32_t t = blockIdx.x * kTPB + threadIdx.x;
    if (t < ntail) dtail[t] = stail[t];
}

__global__ __launch_bounds__(kTPB) void k_copy1(unsigned char* __restrict__ dst, const unsigned char* __restrict__ src,
                                                uint64_t n) {
    const uint64_t stride = (uint64_t)gridDim.x * kTPB;
    for (uint64_t i = (uint64_t)blockIdx.x * kTPB + threadIdx.x; i < n; i += stride) dst[i] = src[i];
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
        s.ready = true;
    }
    *out = &s;
    return MQ_OK;
}

namespace {
struct PoolBlock {
    void* p;
    size_t bytes;
    int dev;
    bool busy;
    bool pending;    // freed stream-ordered: reusable once ev has completed
    hipEvent_t ev;   // created on the block's device at its first ordered free
};
std::mutex g_pool_mu;
std::vector<PoolBlock> g_pool;

// An idle block whose ordered free has not yet completed on its stream.
bool pool_in_flight(PoolBlock& b) {
    if (!b.pending) return false;
    if (hipEventQuery(b.ev) == hipErrorNotReady) return true;
    (void)hipGetLastError();
    b.pending = false;
    return false;
}

void pool_release_idle_locked() {
    for (size_t i = 0; i < g_pool.size();) {
        if (!g_pool[i].busy) {
            if (g_pool[i].pending) (void)hipEventSynchronize(g_pool[i].ev);
            if (g_pool[i].ev) (void)hipEventDestroy(g_pool[i].ev);
            (void)hipFree(g_pool[i].p);
            g_pool[i] = g_pool.back();
            g_pool.pop_back();
        } else {
            i++;
        }
    }
}
}  // namespace

void* pool_alloc(size_t bytes) {
    if (bytes == 0) bytes = 16;
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::unique_lock<std::mutex> lk(g_pool_mu);
    PoolBlock *best = nullptr, *wait = nullptr;  // best: reusable now; wait: its free still in flight
    for (auto& b : g_pool)
        if (!b.busy && b.dev == dev && b.bytes >= bytes && b.bytes / 2 <= bytes) {
            PoolBlock*& slot = pool_in_flight(b) ? wait : best;
            if (!slot || b.bytes < slot->bytes) slot = &b;
        }
    if (best) {
        best->busy = true;
        return best->p;
    }
    void* p = nullptr;
    if (hipMalloc(&p, bytes) != hipSuccess) {
        (void)hipGetLastError();
        if (wait) {  // the only fit is still used by queued work, and no fresh block fits
                     // in HBM: wait for that one (outside the lock). (a fresh
                     // block first, so callers on other streams never wait on each other.)
            wait->busy = true;
            void* q = wait->p;
            hipEvent_t ev = wait->ev;
            wait->pending = false;
            lk.unlock();
            (void)hipEventSynchronize(ev);
            return q;
        }
        pool_release_idle_locked();  // give the cache back and retry once
        if (hipMalloc(&p, bytes) != hipSuccess) {
            (void)hipGetLastError();
            return nullptr;
        }
    }
    g_pool.push_back(PoolBlock{p, bytes, dev, true, false, nullptr});
    return p;
}

void pool_free(void* p) {
    if (!p) return;
    std::lock_guard<std::mutex> lk(g_pool_mu);
    for (auto& b : g_pool)
        if (b.p == p) {
            b.busy = false;
            return;
        }
    (void)hipFree(p);  // not from the pool
}

void pool_free_on(void* p, hipStream_t st) {
    if (!p) return;
    int dev = -1;
    (void)hipGetDevice(&dev);
    std::unique_lock<std::mutex> lk(g_pool_mu);
    for (auto& b : g_pool)
        if (b.p == p) {
            bool ok = b.dev == dev;  // events record on the current device's streams only
            if (ok && !b.ev) ok = hipEventCreateWithFlags(&b.ev, hipEventDisableTiming) == hipSuccess;
            if (ok) ok = hipEventRecord(b.ev, st) == hipSuccess;
            if (!ok) {  // cannot order it: wait for the stream instead
                (void)hipGetLastError();
                lk.unlock();
                (void)hipStreamSynchronize(st);
                pool_free(p);
                return;
            }
            b.pending = true;
            b.busy = false;
            return;
        }
    lk.unlock();
    (void)hipStreamSynchronize(st);
    (void)hipFree(p);
}

uint32_t stream_grid(const DevState* s, uint64_t work_items) {
    uint64_t g = (work_items + kTPB - 1) / kTPB;
    const uint64_t cap = (uint64_t)s->cus * 8;
    if (g > cap) g = cap;
    return (uint32_t)(g == 0 ? 1 : g);
}

uint32_t resident_grid(const DevState* s, uint64_t work_items, const void* fn) {
    const uint32_t g = stream_grid(s, work_items);
    const uint64_t cap = (uint64_t)s->cus * (uint64_t)blocks_per_cu(fn);
    return cap && g > cap ? (uint32_t)cap : g;
}

// Fold (has_low, low, has_high, high) into one unsigned range compare.
// Returns false for an empty range.
bool make_pred(int has_low, int32_t low, int has_high, int32_t high, Pred* p) {
    const int64_t lo = has_low ? (int64_t)low : (int64_t)INT32_MIN;
    const int64_t hi = has_high ? (int64_t)high : (int64_t)INT32_MAX + 1;
    const int64_t width = hi - lo;
    if (width <= 0) return false;
    p->lo = (uint32_t)lo;
    p->wm1 = (uint32_t)(width - 1);
    p->base = 0;
    return true;
}

// Resident 256-thread blocks per CU for one kernel (cached per device and kernel).
int blocks_per_cu(const void* fn, size_t dyn_lds) {
    struct Entry {
        int dev;
        const void* fn;
        size_t dyn;
        int occ;
    };
    static Entry cache[64];
    static int ncache = 0;
    static std::mutex mu;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    std::lock_guard<std::mutex> lk(mu);
    for (int i = 0; i < ncache; i++)
        if (cache[i].dev == dev && cache[i].fn == fn && cache[i].dyn == dyn_lds) return cache[i].occ;
    int occ = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, fn, kTPB, dyn_lds) != hipSuccess || occ < 1)
        occ = 1;
    if (ncache < 64) cache[ncache++] = Entry{dev, fn, dyn_lds, occ};
    return occ;
}

// One wave of resident blocks, each owning a contiguous chunk of whole tiles.
void geometry(const DevState* s, uint64_t n, const void* fn, uint32_t* blocks, uint64_t* rpb,
              uint64_t granule, size_t dyn_lds, int bpc_cap) {
    int bpc = blocks_per_cu(fn, dyn_lds);
    if (bpc_cap > 0 && bpc > bpc_cap) bpc = bpc_cap;
    uint64_t gmax = (uint64_t)s->cus * (uint64_t)bpc;
    if (gmax > kMaxBlocks) gmax = kMaxBlocks;
    const uint64_t tiles = (n + granule - 1) / granule;
    uint64_t g = tiles < gmax ? tiles : gmax;
    if (g == 0) g = 1;
    const uint64_t tiles_per_block = (tiles + g - 1) / g;
    *rpb = (tiles_per_block == 0 ? 1 : tiles_per_block) * granule;
    g = (n + *rpb - 1) / *rpb;
    *blocks = (uint32_t)(g == 0 ? 1 : g);
}

size_t partial_bytes() { return (size_t)kMaxBlocks * sizeof(Partial); }
}  // namespace mqi

namespace {
using namespace mqi;

template <int MODE>
const void* scan_fn(bool vec) {
    return vec ? reinterpret_cast<const void*>(&k_scan<MODE, true>)
               : reinterpret_cast<const void*>(&k_scan<MODE, false>);
}

// The arrival counters of block_arrive_last for launches on stream st of the
// current device: one zeroed 36 KiB block per (device, stream), made on first use
// (the zeroing memset is queued on st ahead of the first launch that uses it).
// Launches on one stream run in order and the last arriver of each resets the
// counters, so every launch on that stream finds them zero; launches on different
// streams use different blocks, so any number of them may be in flight. (A fixed
// pool of slots handed out in rotation let >16 concurrent launches, e.g. row shards
// on one device, share counters and fold wrong partials.) The per-thread default
// stream is one stream per thread, so its blocks are keyed by thread as well.
// The block lives on the stream's own device (hipStreamGetDevice; the null and
// per-thread streams belong to the current one). Entries are dropped when libmq
// destroys the stream (mq_stream_destroy) and, for the per-thread stream, when
// the thread releases its resources (mq_thread_release).
struct ArriveEntry {
    int dev;
    hipStream_t st;
    std::thread::id th;
    unsigned int* ctr;
};
std::mutex g_arrive_mu;
std::vector<ArriveEntry> g_arrive;

int stream_device(hipStream_t st, int* dev) {
    if (st != nullptr && st != hipStreamPerThread && hipStreamGetDevice(st, dev) == hipSuccess) return 0;
    return hipGetDevice(dev) == hipSuccess ? 0 : -1;
}

unsigned int* arrive_counters(hipStream_t st) {
    int dev = 0;
    if (stream_device(st, &dev)) return nullptr;
    const std::thread::id th = st == hipStreamPerThread ? std::this_thread::get_id() : std::thread::id();
    std::lock_guard<std::mutex> lk(g_arrive_mu);
    for (const ArriveEntry& e : g_arrive)
        if (e.dev == dev && e.st == st && e.th == th) return e.ctr;
    int cur = dev;
    (void)hipGetDevice(&cur);
    if (cur != dev && hipSetDevice(dev) != hipSuccess) return nullptr;
    void* p = nullptr;
    const bool ok = hipMalloc(&p, kArriveBytes) == hipSuccess;
    if (ok && hipMemsetAsync(p, 0, kArriveBytes, st) != hipSuccess) {
        (void)hipFree(p);
        p = nullptr;
    }
    if (cur != dev) (void)hipSetDevice(cur);
    if (!p) return nullptr;
    g_arrive.push_back(ArriveEntry{dev, st, th, static_cast<unsigned int*>(p)});
    return static_cast<unsigned int*>(p);
}

// Free the counter blocks of stream st (every thread's, for a real stream) or, with
// st == hipStreamPerThread, the calling thread's. The caller has synchronised the
// work that used them.
void arrive_forget(hipStream_t st) {
    const std::thread::id th = st == hipStreamPerThread ? std::this_thread::get_id() : std::thread::id();
    std::lock_guard<std::mutex> lk(g_arrive_mu);
    for (size_t i = 0; i < g_arrive.size();) {
        if (g_arrive[i].st == st && g_arrive[i].th == th) {
            (void)hipFree(g_arrive[i].ctr);
            g_arrive[i] = g_arrive.back();
            g_arrive.pop_back();
        } else {
            i++;
        }
    }
}

// Launch k_scan<MODE> over n rows; returns the number of blocks (partials) via *g_out.
// out != nullptr folds the partials inside the launch (block_arrive_last).
template <int MODE>
int launch_scan(const int32_t* col, uint64_t n, Pred p, Partial* part,
                mq_agg* out, hipStream_t st, const DevState* s, uint32_t* g_out,
                uint64_t* rpb_out = nullptr) {
    unsigned int* arrive = nullptr;
    if (out && !(arrive = arrive_counters(st)))
        return set_err(MQ_ENOMEM, "arrival counters for the stream could not be allocated");
    const bool vec = aligned16(col);
    uint32_t g;
    uint64_t rpb;
    geometry(s, n, scan_fn<MODE>(vec), &g, &rpb);
    if (vec)
        hipLaunchKernelGGL((k_scan<MODE, true>), dim3(g), dim3(kTPB), 0, st, col, n, rpb, p,
                           part, out, arrive);
    else
        hipLaunchKernelGGL((k_scan<MODE, false>), dim3(g), dim3(kTPB), 0, st, col, n, rpb, p,
                           part, out, arrive);
    LAUNCHCHK("k_scan");
    *g_out = g;
    if (rpb_out) *rpb_out = rpb;
    return MQ_OK;
}

// Launch k_scan_gather (config 3 fused, deferred gather) with the partials folded
// in-kernel into *out.
int launch_gather(const int32_t* col, const int32_t* aux, uint64_t n, Pred p, Partial* part,
                  mq_agg* out, hipStream_t st, const DevState* s) {
    unsigned int* arrive = arrive_counters(st);
    if (!arrive) return set_err(MQ_ENOMEM, "arrival counters for the stream could not be allocated");
    const bool vec = aligned16(col);
    const void* fn = vec ? (const void*)&k_scan_gather<true> : (const void*)&k_scan_gather<false>;
    uint32_t g;
    uint64_t rpb;
    geometry(s, n, fn, &g, &rpb);
    if (vec)
        hipLaunchKernelGGL((k_scan_gather<true>), dim3(g), dim3(kTPB), 0, st, col, aux, n, rpb, p, part, out, arrive);
    else
        hipLaunchKernelGGL((k_scan_gather<false>), dim3(g), dim3(kTPB), 0, st, col, aux, n, rpb, p, part, out, arrive);
    LAUNCHCHK("k_scan_gather");
    return MQ_OK;
}

size_t mask_bytes(uint64_t n) {  // k_select_stage's bitmap / spill area: 32 B per 256-row wave tile
    return (size_t)((n + 8 * kTileRows - 1) / (8 * kTileRows)) * kWaves * 32 * sizeof(unsigned long long);
}



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
    Partial* part = static_cast<Partial*>(d_ws);
    uint32_t g;
    if (!aux) return launch_scan<kAgg>(col, n, pred, part, d_out, st, s, &g);
    return launch_gather(col, aux, n, pred, part, d_out, st, s);
}

// Ordered compaction: k_select_stage, one pass, 4N + 4K (+ staging) bytes (DESIGN.md §3.2;
// round 6 removed the measured-slower k_mask + k_compact and look-back forms).
// k_select_stage state: [err u32 | pad][status u64 x G] in the partial slab; the
// bitmap (bitmap-mode tiles only) in the mask area after it.
size_t stage_state_bytes(uint32_t g) { return 64 + (size_t)g * 8; }
static_assert(64 + (size_t)kMaxBlocks * 8 <= (size_t)kMaxBlocks * sizeof(Partial),
              "stage state must fit the partial slab");

int run_select_stage(const int32_t* col, const int32_t* payload, uint64_t n, Pred p, int32_t* out,
                     uint64_t* d_count, void* d_ws, hipStream_t st, const DevState* s) {
    const bool vec = aligned16(col);
    const void* fn = payload ? (vec ? (const void*)&k_select_stage<true, true> : (const void*)&k_select_stage<true, false>)
                             : (vec ? (const void*)&k_select_stage<false, true> : (const void*)&k_select_stage<false, false>);
    uint64_t gmax = (uint64_t)s->cus * (uint64_t)blocks_per_cu(fn);
    if (gmax > kMaxBlocks) gmax = kMaxBlocks;
    const uint64_t granules = (n + kStGranule - 1) / kStGranule;
    const uint64_t units = gmax * kWaves;
    const uint64_t rw = ((granules + units - 1) / units) * kStGranule;
    const uint32_t g = (uint32_t)((n + rw * kWaves - 1) / (rw * kWaves));
    char* w = static_cast<char*>(d_ws);
    unsigned int* err = reinterpret_cast<unsigned int*>(w);
    unsigned long long* status = reinterpret_cast<unsigned long long*>(w + 64);
    unsigned long long* bm = reinterpret_cast<unsigned long long*>(w + partial_bytes());
    HIPCHK(hipMemsetAsync(w, 0, stage_state_bytes(g), st));
    unsigned long long* cnt = reinterpret_cast<unsigned long long*>(d_count);
    if (payload) {
        if (vec) hipLaunchKernelGGL((k_select_stage<true, true>), dim3(g), dim3(kTPB), 0, st, col, payload, n, rw, p, status, bm, out, cnt, err);
        else hipLaunchKernelGGL((k_select_stage<true, false>), dim3(g), dim3(kTPB), 0, st, col, payload, n, rw, p, status, bm, out, cnt, err);
    } else {
        if (vec) hipLaunchKernelGGL((k_select_stage<false, true>), dim3(g), dim3(kTPB), 0, st, col, payload, n, rw, p, status, bm, out, cnt, err);
        else hipLaunchKernelGGL((k_select_stage<false, false>), dim3(g), dim3(kTPB), 0, st, col, payload, n, rw, p, status, bm, out, cnt, err);
    }
    LAUNCHCHK("k_select_stage");
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

static int h2d_staged(void* dst, const void* src, size_t bytes, hipStream_t st);

// Large uploads (columns, CSV text) go through the pinned staging ring of the D2H
// path below, host copies by the copy pool: a pageable hipMemcpy moved mmap'd
// columns at 13-15 GB/s.
int mq_memcpy_h2d(void* dst, const void* src, size_t bytes, void* stream) {
    if (bytes == 0) return MQ_OK;
    hipStream_t st = (hipStream_t)stream;
    if (bytes >= ((size_t)64 << 20)) return h2d_staged(dst, src, bytes, st);
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

// D2H through pinned staging buffers: the DMA fills a ring of 4 x 8 MB pinned
// buffers and the host copies each chunk out while the next ones are in flight.
// A direct D2H into pageable memory makes the runtime register those pages with
// the driver; write-protecting them afterwards (mq_guard_arm) then costs the next
// kernel 17-30 ms (tools/guard_stall.hip). Staged, the destination is never
// registered.
namespace {
constexpr int kStageBufs = 4;
constexpr size_t kStageBytes = (size_t)8 << 20;
struct Staging {
    void* buf[kStageBufs];
    hipEvent_t ev[kStageBufs];
    bool ready;
};
thread_local Staging g_staging[kMaxDev];

// The host side of the staged D2H: each chunk copied out of the pinned buffer by
// the calling thread and MQ_COPY_THREADS - 1 helpers (one memcpy thread moved ~10 GB/s,
// a quarter of the DMA rate; 6 threads, round 4: see FaultPool). One pool per calling thread (row-shard workers copy
// concurrently); helpers are started on first use and joined at thread exit.
struct CopyPool {
    std::vector<std::thread> th;
    std::mutex mu;
    std::condition_variable go, done;
    char* dst = nullptr;
    const char* src = nullptr;
    size_t len = 0;
    unsigned long gen = 0;
    int pending = 0, parts = 1;
    bool quit = false;

    void start() {
        const char* e = getenv("MQ_COPY_THREADS");
        parts = e ? atoi(e) : 6;
        if (parts < 1) parts = 1;
        if (parts > 16) parts = 16;
        for (int i = 1; i < parts; i++) th.emplace_back([this, i] { loop(i); });
    }
    void slice(int i) {
        const size_t a = len * (size_t)i / (size_t)parts, b = len * (size_t)(i + 1) / (size_t)parts;
        if (b > a) memcpy(dst + a, src + a, b - a);
    }
    void loop(int i) {
        unsigned long seen = 0;
        for (;;) {
            std::unique_lock<std::mutex> lk(mu);
            go.wait(lk, [&] { return quit || gen != seen; });
            if (quit) return;
            seen = gen;
            lk.unlock();
            slice(i);
            lk.lock();
            if (--pending == 0) done.notify_one();
        }
    }
    void copy(void* d, const void* s, size_t n) {
        if (th.empty() && parts == 1 && gen == 0) start();
        if (parts == 1 || n < ((size_t)1 << 20)) {
            memcpy(d, s, n);
            return;
        }
        {
            std::lock_guard<std::mutex> lk(mu);
            dst = static_cast<char*>(d);
            src = static_cast<const char*>(s);
            len = n;
            pending = parts - 1;
            gen++;
        }
        go.notify_all();
        slice(0);
        std::unique_lock<std::mutex> lk(mu);
        done.wait(lk, [&] { return pending == 0; });
    }
    ~CopyPool() {
        {
            std::lock_guard<std::mutex> lk(mu);
            quit = true;
        }
        go.notify_all();
        for (auto& t : th) t.join();
    }
};
thread_local CopyPool g_copy;

// Background population of a fresh host destination (a Result payload the caller
// will free()): first touch of fresh pages costs more than the DMA that fills them
// (tools/pcie_probe, payload_probe: 40 MB take 0.9 ms to fault in with 4 threads and
// huge pages, 0.71 ms to cross the link). F threads populate it ahead of the staged
// copy with MADV_POPULATE_WRITE (content unchanged; a range that is no longer mapped
// just fails), in 8 MB chunks split into F slices taken in chunk order, so the copy of
// chunk c waits only until chunk c is in. One pool per calling thread, like CopyPool.
struct FaultPool {
    std::vector<std::thread> th;
    std::mutex mu;
    std::condition_variable go;
    char* base = nullptr;
    size_t bytes = 0, nchunks = 0;
    std::vector<std::atomic<int>> done;  // finished slices per chunk
    std::atomic<size_t> next{0};
    std::atomic<int> busy{0};
    unsigned long gen = 0;
    int F = 0;
    bool quit = false;
    std::atomic<bool> usable{true};

    void start() {
        const char* e = getenv("MQ_FAULT_THREADS");
        // 6 population + 6 copy threads (round 4; was 8 + 4): config 3's select_column
        // 1.82-1.87 ms in four runs on two boxes against 1.89-2.41 for 8 + 4
        // (profiles/r04_api_threads_ab.log)
        F = e ? atoi(e) : 6;
        if (F < 0) F = 0;
        if (F > 16) F = 16;
        for (int i = 0; i < F; i++) th.emplace_back([this] { loop(); });
    }
    void work() {
        const size_t pg = 4096;
        for (;;) {
            const size_t piece = next.fetch_add(1, std::memory_order_relaxed);
            if (piece >= nchunks * (size_t)F) return;
            const size_t c = piece / (size_t)F, sl = piece % (size_t)F;
            const size_t c0 = c * kStageBytes, clen = bytes - c0 < kStageBytes ? bytes - c0 : kStageBytes;
            const size_t a = c0 + clen * sl / (size_t)F, b = c0 + clen * (sl + 1) / (size_t)F;
            const uintptr_t pa = ((uintptr_t)base + a + pg - 1) & ~(uintptr_t)(pg - 1);
            const uintptr_t pb = ((uintptr_t)base + b) & ~(uintptr_t)(pg - 1);
            if (pb > pa && madvise((void*)pa, pb - pa, MADV_POPULATE_WRITE) != 0 && errno == EINVAL)
                usable.store(false, std::memory_order_relaxed);
            done[c].fetch_add(1, std::memory_order_release);
        }
    }
    void loop() {
        unsigned long seen = 0;
        for (;;) {
            {
                std::unique_lock<std::mutex> lk(mu);
                go.wait(lk, [&] { return quit || gen != seen; });
                if (quit) return;
                seen = gen;
            }
            work();
            busy.fetch_sub(1, std::memory_order_acq_rel);
        }
    }
    // wait for the job in flight, if any
    void finish() {
        while (busy.load(std::memory_order_acquire) > 0) std::this_thread::yield();
        base = nullptr;
        bytes = nchunks = 0;
    }
    void begin(void* p, size_t n) {
        if (th.empty() && F == 0 && gen == 0) start();
        finish();
        if (F == 0 || !usable.load(std::memory_order_relaxed) || n < ((size_t)4 << 20)) return;
        base = static_cast<char*>(p);
        bytes = n;
        nchunks = (n + kStageBytes - 1) / kStageBytes;
        if (done.size() < nchunks) done = std::vector<std::atomic<int>>(nchunks);
        for (size_t c = 0; c < nchunks; c++) done[c].store(0, std::memory_order_relaxed);
        next.store(0, std::memory_order_relaxed);
        busy.store(F, std::memory_order_release);
        {
            std::lock_guard<std::mutex> lk(mu);
            gen++;
        }
        go.notify_all();
    }
    // chunk c of [dst, dst + n) is populated (or no job covers it)
    void wait_chunk(const void* dst, size_t n, size_t c) {
        if (!base || dst != base || n != bytes || c >= nchunks) return;
        while (done[c].load(std::memory_order_acquire) < F) std::this_thread::yield();
    }
    bool covers(const void* dst, size_t n) const { return base && dst == base && n == bytes; }
    ~FaultPool() {
        finish();
        {
            std::lock_guard<std::mutex> lk(mu);
            quit = true;
        }
        go.notify_all();
        for (auto& t : th) t.join();
    }
};
thread_local FaultPool g_fault;
}  // namespace

// mq_host_prefault (mq_device.h): start populating [p, p + bytes) on the calling
// thread's fault pool; the next mq_memcpy_d2h_staged into exactly that range waits for
// each chunk's population before copying into it.
void mq_host_prefault(void* p, size_t bytes) {
    static const bool on = !(getenv("MQ_PREFAULT") && getenv("MQ_PREFAULT")[0] == '0');
    if (on && p && bytes) g_fault.begin(p, bytes);
}

// mq_host_prefault_wait (mq_device.h): wait for the calling thread's population job,
// so its range may be freed.
void mq_host_prefault_wait(void) { g_fault.finish(); }

int mq_memcpy_d2h_staged(void* dst, const void* src, size_t bytes, void* stream) {
    if (bytes == 0) return MQ_OK;
    int d;
    int rc = current_device(&d);
    if (rc) return rc;
    Staging& S = g_staging[d];
    if (!S.ready) {
        for (int i = 0; i < kStageBufs; i++) {
            HIPCHK(hipHostMalloc(&S.buf[i], kStageBytes, hipHostMallocDefault));
            HIPCHK(hipEventCreateWithFlags(&S.ev[i], hipEventDisableTiming));
        }
        S.ready = true;
    }
    hipStream_t st = (hipStream_t)stream;
    const size_t nchunks = (bytes + kStageBytes - 1) / kStageBytes;
    auto issue = [&](size_t c) -> int {
        const size_t off = c * kStageBytes, len = bytes - off < kStageBytes ? bytes - off : kStageBytes;
        const int b = (int)(c % kStageBufs);
        HIPCHK(hipMemcpyAsync(S.buf[b], static_cast<const char*>(src) + off, len, hipMemcpyDeviceToHost, st));
        HIPCHK(hipEventRecord(S.ev[b], st));
        return MQ_OK;
    };
    for (size_t c = 0; c < nchunks && c < (size_t)kStageBufs; c++)
        if ((rc = issue(c))) return rc;
    if (!g_fault.covers(dst, bytes)) mq_host_prefault(dst, bytes);
    for (size_t c = 0; c < nchunks; c++) {
        const int b = (int)(c % kStageBufs);
        HIPCHK(hipEventSynchronize(S.ev[b]));
        const size_t off = c * kStageBytes, len = bytes - off < kStageBytes ? bytes - off : kStageBytes;
        g_fault.wait_chunk(dst, bytes, c);
        g_copy.copy(static_cast<char*>(dst) + off, S.buf[b], len);
        if (c + kStageBufs < nchunks && (rc = issue(c + kStageBufs))) return rc;
    }
    g_fault.finish();
    return MQ_OK;
}

// mq_select_positions_download (mq_device.h): segment s's kernel writes its count into
// pinned, host-coherent memory (no D2H on the compute stream), an event marks its end;
// the host waits for segment s alone and stages its positions down on the thread's copy
// stream, overlapping the kernels of segments s+1.. (the SDMA engine reads HBM at the
// link's 57 GB/s, far below the scan's own traffic). The payload pages of segment s are
// populated by the staged copy's fault pool as it starts (mq_host_prefault).
namespace {
struct SegPipe {
    hipStream_t copy = nullptr;
    unsigned long long* cnt = nullptr;  // 64 pinned counts
    hipEvent_t ev[64];
    bool ready = false;
};
thread_local SegPipe g_segpipe[kMaxDev];
}  // namespace

int mq_select_positions_download(const int32_t* d_col, uint64_t n, int has_low, int32_t low, int has_high,
                                 int32_t high, int segs, int32_t* d_pos, int32_t* h_dst, uint64_t* h_seg,
                                 uint64_t* h_rows, void* d_ws, size_t ws_bytes, void* stream) {
    DevState* s;
    int rc = ensure_ready(&s);
    if (rc) return rc;
    if (segs < 1 || segs > 64 || !h_seg || !h_rows || (n && (!d_col || !d_pos || !h_dst)))
        return set_err(MQ_EINVAL, "mq_select_positions_download: bad argument");
    int d;
    if ((rc = current_device(&d))) return rc;
    SegPipe& P = g_segpipe[d];
    if (!P.ready) {
        HIPCHK(hipStreamCreateWithFlags(&P.copy, hipStreamNonBlocking));
        HIPCHK(hipHostMalloc((void**)&P.cnt, 64 * sizeof(unsigned long long), hipHostMallocCoherent));
        for (int i = 0; i < 64; i++) HIPCHK(hipEventCreateWithFlags(&P.ev[i], hipEventDisableTiming));
        P.ready = true;
    }
    // segment bounds: whole 1024-row tiles (16-byte aligned slices, as the row shards).
    // (round 6) The first segment is 3/4 of an equal share: its positions start down
    // sooner, and while they do the longer second segment scans. With the payload D2H at
    // ~33 GB/s (1.2 ms for 40 MB) and the scan at 0.68 ms, two segments take s1 + max(d1,
    // s2) + d2, least near a first share of 0.36 (1.45 ms) against 1.54 ms at halves.
    h_rows[0] = 0;
    const uint64_t first = segs > 1 ? (uint64_t)(((unsigned __int128)n * 3u) / (4u * (unsigned)segs)) : n;
    for (int g = 1; g < segs; g++) {
        uint64_t b = (first + (uint64_t)(((unsigned __int128)(n - first) * (unsigned)(g - 1)) / (unsigned)(segs - 1))) &
                     ~(uint64_t)1023;
        h_rows[g] = b < h_rows[g - 1] ? h_rows[g - 1] : b;
    }
    h_rows[segs] = n;
    hipStream_t st = (hipStream_t)stream;
    unsigned long long* dcnt = nullptr;
    HIPCHK(hipHostGetDevicePointer((void**)&dcnt, P.cnt, 0));
    for (int g = 0; g < segs; g++) {
        const uint64_t r0 = h_rows[g], ng = h_rows[g + 1] - r0;
        P.cnt[g] = 0;
        if (ng && (rc = mq_select_positions_at(d_col + r0, nullptr, ng, (int32_t)r0, has_low, low, has_high, high,
                                               d_pos + r0, reinterpret_cast<uint64_t*>(dcnt + g), d_ws, ws_bytes,
                                               stream)))
            return rc;
        HIPCHK(hipEventRecord(P.ev[g], st));
    }
    uint64_t off = 0;
    for (int g = 0; g < segs; g++) {
        HIPCHK(hipEventSynchronize(P.ev[g]));
        const uint64_t k = *reinterpret_cast<volatile unsigned long long*>(P.cnt + g);
        if (k > h_rows[g + 1] - h_rows[g]) {  // the select's own error word (~0): its spin timed out
            (void)hipStreamSynchronize(st);
            return set_err(MQ_EHIP, "mq_select_positions_download: segment %d count %llu", g, (unsigned long long)k);
        }
        h_seg[g] = k;
        if (k && (rc = mq_memcpy_d2h_staged(h_dst + off, d_pos + h_rows[g], k * sizeof(int32_t), P.copy))) {
            (void)hipStreamSynchronize(st);
            return rc;
        }
        off += k;
    }
    return MQ_OK;
}

// mq_thread_release (mq_device.h): the calling thread's pinned staging buffers and
// their events, on every device it staged through. A thread that exits without it
// leaks them (thread_local storage is not freed by the runtime).
void mq_thread_release(void) {
    int cur = 0;
    const bool have_cur = hipGetDevice(&cur) == hipSuccess;
    for (int d = 0; d < kMaxDev; d++) {
        Staging& S = g_staging[d];
        if (!S.ready) continue;
        if (hipSetDevice(d) != hipSuccess) continue;
        for (int i = 0; i < kStageBufs; i++) {
            (void)hipEventSynchronize(S.ev[i]);
            (void)hipEventDestroy(S.ev[i]);
            (void)hipHostFree(S.buf[i]);
        }
        S = Staging{};
    }
    for (int d = 0; d < kMaxDev; d++) {
        SegPipe& P = g_segpipe[d];
        if (!P.ready || hipSetDevice(d) != hipSuccess) continue;
        (void)hipStreamSynchronize(P.copy);
        (void)hipStreamDestroy(P.copy);
        for (int i = 0; i < 64; i++) (void)hipEventDestroy(P.ev[i]);
        (void)hipHostFree(P.cnt);
        P = SegPipe{};
    }
    if (have_cur) (void)hipSetDevice(cur);
    mqi::shared_staging_release();
    (void)hipStreamSynchronize(hipStreamPerThread);
    arrive_forget(hipStreamPerThread);
}

// The mirror of the staged D2H: the pool copies chunk c into pinned buffer c % 4
// while the DMA of the chunks before it runs; a buffer is refilled once its DMA
// has completed (its event).
static int h2d_staged(void* dst, const void* src, size_t bytes, hipStream_t st) {
    int d;
    int rc = current_device(&d);
    if (rc) return rc;
    Staging& S = g_staging[d];
    if (!S.ready) {
        for (int i = 0; i < kStageBufs; i++) {
            HIPCHK(hipHostMalloc(&S.buf[i], kStageBytes, hipHostMallocDefault));
            HIPCHK(hipEventCreateWithFlags(&S.ev[i], hipEventDisableTiming));
        }
        S.ready = true;
    }
    const size_t nchunks = (bytes + kStageBytes - 1) / kStageBytes;
    for (size_t c = 0; c < nchunks; c++) {
        const int b = (int)(c % kStageBufs);
        if (c >= (size_t)kStageBufs) HIPCHK(hipEventSynchronize(S.ev[b]));
        const size_t off = c * kStageBytes, len = bytes - off < kStageBytes ? bytes - off : kStageBytes;
        g_copy.copy(S.buf[b], static_cast<const char*>(src) + off, len);
        HIPCHK(hipMemcpyAsync(static_cast<char*>(dst) + off, S.buf[b], len, hipMemcpyHostToDevice, st));
        HIPCHK(hipEventRecord(S.ev[b], st));
    }
    HIPCHK(hipStreamSynchronize(st));
    return MQ_OK;
}

int mq_memcpy_d2d(void* dst, const void* src, size_t bytes, void* stream) {
    if (bytes == 0) return MQ_OK;
    DevState* s;
    int rc = ensure_ready(&s);
    if (rc) return rc;
    if (!dst || !src) return set_err(MQ_EINVAL, "mq_memcpy_d2d: NULL pointer");
    hipStream_t st = (hipStream_t)stream;
    if ((((uintptr_t)dst | (uintptr_t)src) & 15u) == 0) {
        const uint64_t n16 = bytes / 16;
        const uint32_t tail = (uint32_t)(bytes % 16);
        const uint32_t g = stream_grid(s, n16 > tail ? n16 : tail);
        hipLaunchKernelGGL(k_copy16, dim3(g), dim3(kTPB), 0, st, static_cast<uint4*>(dst),
                           static_cast<const uint4*>(src), n16, static_cast<unsigned char*>(dst) + n16 * 16,
                           static_cast<const unsigned char*>(src) + n16 * 16, tail);
        LAUNCHCHK("k_copy16");
    } else {
        hipLaunchKernelGGL(k_copy1, dim3(stream_grid(s, bytes)), dim3(kTPB), 0, st, static_cast<unsigned char*>(dst),
                           static_cast<const unsigned char*>(src), (uint64_t)bytes);
        LAUNCHCHK("k_copy1");
    }
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

int mq_pool_malloc(void** dptr, size_t bytes) {
    DevState* s;
    int rc = ensure_ready(&s);
    if (rc) return rc;
    if (!dptr) return set_err(MQ_EINVAL, "mq_pool_malloc: NULL out pointer");
    *dptr = pool_alloc(bytes);
    if (!*dptr) return set_err(MQ_ENOMEM, "mq_pool_malloc(%zu) failed", bytes);
    return MQ_OK;
}

int mq_pool_free(void* dptr) {
    pool_free(dptr);
    return MQ_OK;
}

int mq_pool_free_on(void* dptr, void* stream) {
    pool_free_on(dptr, (hipStream_t)stream);
    return MQ_OK;
}

int mq_device_sync(void) {
    HIPCHK(hipDeviceSynchronize());
    return MQ_OK;
}

void mq_trim(void) {
    (void)hipDeviceSynchronize();
    std::lock_guard<std::mutex> lk(g_pool_mu);
    pool_release_idle_locked();
}

size_t mq_scan_workspace_bytes(uint64_t n) {
    return partial_bytes() + mask_bytes(n);
}

void mq_scan_geometry(uint64_t n, uint32_t* blocks, uint64_t* rows_per_block) {
    DevState* s;
    if (ensure_ready(&s)) {
        if (blocks) *blocks = 0;
        if (rows_per_block) *rows_per_block = 0;
        return;
    }
    uint32_t g;
    uint64_t r;
    geometry(s, n, scan_fn<kSum>(true), &g, &r);
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
    if (!d_out || kind < 0 || kind > 3 || (kind == 3 && (n & (n - 1))))
        return set_err(MQ_EINVAL, "mq_gen_join_keys: bad argument");
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

int mq_select_sum(const int32_t* d_col, uint64_t n, int has_low, int32_t low, int has_high,
                  int32_t high, mq_agg* d_out, void* d_ws, size_t ws_bytes, void* stream) {
    DevState* s;
    int rc = ensure_ready(&s);
    if (rc) return rc;
    if (!d_out || !d_ws || (n && !d_col)) return set_err(MQ_EINVAL, "mq_select_sum: NULL pointer");
    if ((uintptr_t)d_col & 3u) return set_err(MQ_EINVAL, "mq_select_sum: column not 4-byte aligned");
    if (ws_bytes < partial_bytes())
        return set_err(MQ_EINVAL, "workspace too small (%zu < %zu)", ws_bytes, partial_bytes());
    Pred p;
    hipStream_t st = (hipStream_t)stream;
    if (n == 0 || !make_pred(has_low, low, has_high, high, &p)) return empty_agg(d_out, st);
    uint32_t g;
    return launch_scan<kSum>(d_col, n, p, static_cast<Partial*>(d_ws), d_out, st, s, &g);
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
                       int32_t high, int want_minmax, void* d_ws, size_t ws_bytes,
                       uint32_t* nblocks, void* stream) {
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
    Partial* part = static_cast<Partial*>(d_ws);
    return want_minmax ? launch_scan<kAgg>(d_col, n, p, part, nullptr, st, s, nblocks)
                       : launch_scan<kSum>(d_col, n, p, part, nullptr, st, s, nblocks);
}

int mq_stream_read(const int32_t* d_col, uint64_t n, void* d_ws, size_t ws_bytes,
                   uint64_t* bytes_read, void* stream) {
    DevState* s;
    int rc = ensure_ready(&s);
    if (rc) return rc;
    if (!d_ws || !bytes_read || (n && !d_col)) return set_err(MQ_EINVAL, "mq_stream_read: NULL pointer");
    if ((uintptr_t)d_col & 15u) return set_err(MQ_EINVAL, "mq_stream_read: column not 16-byte aligned");
    if (ws_bytes < (size_t)kMaxBlocks * sizeof(uint32_t))
        return set_err(MQ_EINVAL, "mq_stream_read: workspace too small");
    uint32_t g;
    uint64_t rpb;
    geometry(s, n, reinterpret_cast<const void*>(&k_stream_read<true>), &g, &rpb, 8 * kTileRows);
    uint64_t read = 0;
    for (uint32_t b = 0; b < g; b++) {
        const uint64_t a = (uint64_t)b * rpb, e = a + rpb < n ? a + rpb : n;
        read += e > a ? (e - a) / (8 * kTileRows) * (8 * kTileRows) : 0;
    }
    *bytes_read = read * 4;
    if (n == 0) return MQ_OK;
    hipLaunchKernelGGL((k_stream_read<true>), dim3(g), dim3(kTPB), 0, (hipStream_t)stream, d_col, n,
                       rpb, static_cast<uint32_t*>(d_ws));
    LAUNCHCHK("k_stream_read");
    return MQ_OK;
}

int mq_hashset_lookup(const int32_t* d_table, int32_t size, const int32_t* d_probe, uint64_t n,
                      uint8_t* d_found, void* stream) {
    DevState* s;
    int rc = ensure_ready(&s);
    if (rc) return rc;
    if (size <= 0) return set_err(MQ_EINVAL, "mq_hashset_lookup: size %d", size);
    if (n == 0) return MQ_OK;
    if (!d_table || !d_probe || !d_found) return set_err(MQ_EINVAL, "mq_hashset_lookup: NULL pointer");
    hipLaunchKernelGGL(k_hashset_lookup, dim3(stream_grid(s, n)), dim3(kTPB), 0, (hipStream_t)stream, d_table,
                       size, d_probe, n, d_found);
    LAUNCHCHK("k_hashset_lookup");
    return MQ_OK;
}

// get_hashset_elements (hashset.c:48-65): the nonzero slots in slot order, i.e. the
// ordered compaction of the table with itself as payload under v != 0, which is
// the unsigned range (uint32)(v - 1) <= 0xFFFFFFFE.
int mq_hashset_elements(const int32_t* d_table, uint64_t size, int32_t* d_out, uint64_t* d_count,
                        void* d_ws, size_t ws_bytes, void* stream) {
    DevState* s;
    int rc = ensure_ready(&s);
    if (rc) return rc;
    if (!d_count || (size && (!d_table || !d_out || !d_ws)))
        return set_err(MQ_EINVAL, "mq_hashset_elements: NULL pointer");
    if (size >= (1ull << 31)) return set_err(MQ_EINVAL, "mq_hashset_elements: size beyond int32 positions");
    hipStream_t st = (hipStream_t)stream;
    if (size == 0) {
        HIPCHK(hipMemsetAsync(d_count, 0, sizeof(uint64_t), st));
        return MQ_OK;
    }
    if (ws_bytes < mq_scan_workspace_bytes(size)) return set_err(MQ_EINVAL, "mq_hashset_elements: workspace too small");
    Pred p;
    p.lo = 1u;
    p.wm1 = 0xFFFFFFFEu;
    p.base = 0;
    return run_select_stage(d_table, d_table, size, p, d_out, d_count, d_ws, st, s);
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
    return mq_select_positions_at(d_col, d_payload, n, 0, has_low, low, has_high, high, d_pos_out, d_count,
                                  d_ws, ws_bytes, stream);
}

namespace {
int select_positions_impl(const int32_t* d_col, const int32_t* d_payload, uint64_t n, int32_t row_base,
                          int has_low, int32_t low, int has_high, int32_t high, int32_t* d_pos_out,
                          uint64_t* d_count, void* d_ws, size_t ws_bytes, void* stream);
}

int mq_select_positions_at(const int32_t* d_col, const int32_t* d_payload, uint64_t n, int32_t row_base,
                           int has_low, int32_t low, int has_high, int32_t high, int32_t* d_pos_out,
                           uint64_t* d_count, void* d_ws, size_t ws_bytes, void* stream) {
    if (row_base < 0 || (uint64_t)row_base + n > (uint64_t)INT32_MAX)
        return set_err(MQ_EINVAL, "mq_select_positions_at: rows [%d, %d + %llu) beyond int32 positions", row_base,
                       row_base, (unsigned long long)n);
    return select_positions_impl(d_col, d_payload, n, d_payload ? 0 : row_base, has_low, low, has_high, high,
                                 d_pos_out, d_count, d_ws, ws_bytes, stream);
}

namespace {
int select_positions_impl(const int32_t* d_col, const int32_t* d_payload, uint64_t n, int32_t row_base,
                          int has_low, int32_t low, int has_high, int32_t high, int32_t* d_pos_out,
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
    p.base = row_base;  // k_select_stage adds it as it writes
    return run_select_stage(d_col, d_payload, n, p, d_pos_out, d_count, d_ws, st, s);
}
}  // namespace

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

int mq_fetch_at(const int32_t* d_col, int32_t row_base, const int32_t* d_pos, uint64_t k, int32_t* d_out,
                void* stream) {
    if (row_base < 0) return set_err(MQ_EINVAL, "mq_fetch_at: negative row base");
    // k_fetch reads col[pos]; positions of this shard lie in [row_base, row_base + rows),
    // so the column pointer is taken row_base rows back (never dereferenced there)
    return mq_fetch(d_col - row_base, d_pos, k, d_out, stream);
}

int mq_stream_create(void** stream) {
    DevState* s;
    int rc = ensure_ready(&s);
    if (rc) return rc;
    if (!stream) return set_err(MQ_EINVAL, "mq_stream_create: NULL out pointer");
    hipStream_t st;
    HIPCHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    *stream = st;
    return MQ_OK;
}

int mq_stream_destroy(void* stream) {
    if (!stream) return MQ_OK;
    HIPCHK(hipStreamSynchronize((hipStream_t)stream));
    arrive_forget((hipStream_t)stream);
    HIPCHK(hipStreamDestroy((hipStream_t)stream));
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



}  // extern "C"
