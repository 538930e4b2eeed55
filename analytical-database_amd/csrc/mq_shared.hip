// mq_shared.hip — shared_select (src/query.c:439-583): Q range selects over one
// column with the column read twice, whatever Q is (the reference reads it once
// per thread with Q predicates per value, query.c:472-479; a per-query loop of
// mq_select_positions would read it Q times).
//
// Decomposition: the scan grid of mq_scan_common.h, but inside a block each WAVE
// owns a contiguous quarter of the block's chunk (a "wave-chunk"). Row order is
// then (block, wave, wave-tile, lane, element), so:
//   pass 1 (k_ss_count): per (query, wave-chunk) match counts;
//   scan: one flat exclusive scan over the query-major count array gives every
//         (query, wave-chunk) its output offset (minus the query's own base);
//   pass 2 (k_ss_write): each wave re-reads its wave-chunk, evaluates the Q
//         predicates per 256-row wave-tile and writes each query's positions at
//         running offsets it keeps in LDS (no barriers, no atomics).
// HBM traffic: 8N (two nt reads) + 4 * sum(K_q), plus Q x 4 x blocks counters.
// VALU: ~2 compares + 1 ballot per row per query, so Q >> 1 is VALU-bound.

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>

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

// Ballot of "row matches" straight off the compare (v_sub + v_cmp -> SGPR pair).
__device__ __forceinline__ unsigned long long bal(int x, uint32_t lo, uint32_t wm1) {
    return __ballot(((uint32_t)x - lo) <= wm1);
}

// counts[q * nwc + wc], wc = block * 4 + wave
template <bool VEC>
__global__ __launch_bounds__(kTPB) void k_ss_count(const int* __restrict__ col, uint64_t n,
                                                   uint64_t rpb, const Pred* __restrict__ preds,
                                                   int q, uint32_t* __restrict__ counts,
                                                   uint64_t nwc) {
    __shared__ uint32_t wcnt[kWaves][kMaxQ];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (int i = tid; i < q; i += kTPB) {
#pragma unroll
        for (int w = 0; w < kWaves; w++) wcnt[w][i] = 0;
    }
    __syncthreads();
    uint64_t s, e;
    wave_chunk(n, rpb, wave, &s, &e);
    for (uint64_t t = s; t < e; t += kWaveTile * kSsUnroll) {
        int4 v[kSsUnroll];
#pragma unroll
        for (int u = 0; u < kSsUnroll; u++)
            v[u] = load_row4<VEC>(col, t + (uint64_t)u * kWaveTile + (uint64_t)lane * 4, e);
        if (t + kWaveTile * kSsUnroll <= e) {  // full: ballots straight off the compares
            for (int j = 0; j < q; j++) {
                const Pred p = preds[j];  // uniform index: scalar-cache load
                uint32_t c = 0;
#pragma unroll
                for (int u = 0; u < kSsUnroll; u++)
                    c += (uint32_t)(__popcll(bal(v[u].x, p.lo, p.wm1)) + __popcll(bal(v[u].y, p.lo, p.wm1)) +
                                    __popcll(bal(v[u].z, p.lo, p.wm1)) + __popcll(bal(v[u].w, p.lo, p.wm1)));
                if (lane == 0) wcnt[wave][j] += c;  // this wave only: no atomics
            }
        } else {
            for (int j = 0; j < q; j++) {
                const Pred p = preds[j];
                uint32_t c = 0;
#pragma unroll
                for (int u = 0; u < kSsUnroll; u++) {
                    const uint32_t b = match4(v[u], p, t + (uint64_t)u * kWaveTile + (uint64_t)lane * 4, e);
                    c += (uint32_t)(__popcll(__ballot(b & 1u)) + __popcll(__ballot(b & 2u)) +
                                    __popcll(__ballot(b & 4u)) + __popcll(__ballot(b & 8u)));
                }
                if (lane == 0) wcnt[wave][j] += c;
            }
        }
    }
    __syncthreads();
    for (int i = tid; i < q; i += kTPB) {
#pragma unroll
        for (int w = 0; w < kWaves; w++)
            counts[(uint64_t)i * nwc + (uint64_t)blockIdx.x * kWaves + w] = wcnt[w][i];
    }
}

// Writes one wave-tile's matches of one query; o advances by the match count.
__device__ __forceinline__ void ss_emit(int* __restrict__ out, unsigned long long& o, uint64_t row,
                                       unsigned long long m0, unsigned long long m1,
                                       unsigned long long m2, unsigned long long m3, int lane,
                                       unsigned long long ltmask) {
    const unsigned int tot = (unsigned int)(__popcll(m0) + __popcll(m1) + __popcll(m2) + __popcll(m3));
    if (!tot) return;  // uniform
    const unsigned int pre = (unsigned int)(__popcll(m0 & ltmask) + __popcll(m1 & ltmask) +
                                            __popcll(m2 & ltmask) + __popcll(m3 & ltmask));
    const unsigned long long bit = 1ull << lane;
    int* w = out + o + pre;
    unsigned int k = 0;
    if (m0 & bit) w[k++] = (int)(row + 0);
    if (m1 & bit) w[k++] = (int)(row + 1);
    if (m2 & bit) w[k++] = (int)(row + 2);
    if (m3 & bit) w[k++] = (int)(row + 3);
    o += tot;
}

template <bool VEC>
__global__ __launch_bounds__(kTPB) void k_ss_write(const int* __restrict__ col, uint64_t n,
                                                   uint64_t rpb, const Pred* __restrict__ preds,
                                                   int q, const unsigned long long* __restrict__ offs,
                                                   uint64_t nwc, int* const* __restrict__ outs) {
    __shared__ unsigned long long run[kWaves][kMaxQ];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const unsigned long long ltmask = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    for (int i = tid; i < q; i += kTPB) {
        const unsigned long long base = offs[(uint64_t)i * nwc];  // query i's first offset
#pragma unroll
        for (int w = 0; w < kWaves; w++)
            run[w][i] = offs[(uint64_t)i * nwc + (uint64_t)blockIdx.x * kWaves + w] - base;
    }
    __syncthreads();
    uint64_t s, e;
    wave_chunk(n, rpb, wave, &s, &e);
    for (uint64_t t = s; t < e; t += kWaveTile * kSsUnroll) {
        int4 v[kSsUnroll];
#pragma unroll
        for (int u = 0; u < kSsUnroll; u++)
            v[u] = load_row4<VEC>(col, t + (uint64_t)u * kWaveTile + (uint64_t)lane * 4, e);
        const bool full = t + kWaveTile * kSsUnroll <= e;
        for (int j = 0; j < q; j++) {
            const Pred p = preds[j];  // uniform index: scalar-cache load
            unsigned long long o = run[wave][j];
            int* const out = outs[j];
#pragma unroll
            for (int u = 0; u < kSsUnroll; u++) {
                const uint64_t row = t + (uint64_t)u * kWaveTile + (uint64_t)lane * 4;
                if (full) {
                    ss_emit(out, o, row, bal(v[u].x, p.lo, p.wm1), bal(v[u].y, p.lo, p.wm1),
                            bal(v[u].z, p.lo, p.wm1), bal(v[u].w, p.lo, p.wm1), lane, ltmask);
                } else {
                    const uint32_t b = match4(v[u], p, row, e);
                    ss_emit(out, o, row, __ballot(b & 1u), __ballot(b & 2u), __ballot(b & 4u),
                            __ballot(b & 8u), lane, ltmask);
                }
            }
            if (lane == 0) run[wave][j] = o;
        }
    }
}

// totals[j] = offs[j*nwc + nwc-1] + counts[j*nwc + nwc-1] - offs[j*nwc]
__global__ void k_ss_totals(const uint32_t* __restrict__ counts,
                            const unsigned long long* __restrict__ offs, uint64_t nwc, int q,
                            const int* __restrict__ slot, uint64_t* __restrict__ totals, int qall) {
    for (int i = threadIdx.x; i < qall; i += blockDim.x) {
        const int j = slot[i];
        totals[i] = j < 0 ? 0ull
                          : offs[(uint64_t)j * nwc + nwc - 1] + counts[(uint64_t)j * nwc + nwc - 1] -
                                offs[(uint64_t)j * nwc];
    }
}

struct SsLayout {
    size_t preds, outs, slot, counts, offs, scratch, total;
};

SsLayout ss_layout(uint64_t nwc, int q) {
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    SsLayout L;
    size_t at = 0;
    L.preds = at;
    at += al((size_t)kMaxQ * sizeof(Pred));
    L.outs = at;
    at += al((size_t)kMaxQ * sizeof(int*));
    L.slot = at;
    at += al((size_t)kMaxQ * sizeof(int));
    L.counts = at;
    at += al((size_t)q * nwc * sizeof(uint32_t));
    L.offs = at;
    at += al((size_t)q * nwc * sizeof(unsigned long long));
    L.scratch = at;
    at += al((size_t)scan_u32_scratch_elems((uint64_t)q * nwc) * sizeof(unsigned long long));
    L.total = at;
    return L;
}

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
};

int ss_count(const int32_t* d_col, uint64_t n, const int32_t* h_lows, const int32_t* h_highs,
             int q, uint64_t* d_totals, void* d_ws, size_t ws_bytes, hipStream_t st,
             SsState* state) {
    DevState* s;
    int rc = ensure_ready(&s);
    if (rc) return rc;
    if (q < 1 || q > kMaxQ || !h_lows || !h_highs || !d_totals)
        return set_err(MQ_EINVAL, "shared_select: bad argument (q = %d, 1..%d)", q, kMaxQ);
    if (n > (uint64_t)INT32_MAX) return set_err(MQ_EINVAL, "shared_select: n over 2^31");
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
    const void* fn = vec ? (const void*)&k_ss_write<true> : (const void*)&k_ss_write<false>;
    uint32_t g = 1;
    uint64_t rpb = kGranule;
    if (n) geometry(s, n, fn, &g, &rpb, kGranule);
    const uint64_t nwc = (uint64_t)g * kWaves;
    const SsLayout L = ss_layout(nwc, qk > 0 ? qk : 1);
    HIPCHK(hipMemcpyAsync(w + L.preds, hp, sizeof(Pred) * (qk > 0 ? qk : 1), hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(w + L.slot, hslot, sizeof(int) * q, hipMemcpyHostToDevice, st));
    HIPCHK(hipStreamSynchronize(st));  // the staging arrays are reused by the next call
    const Pred* dp = reinterpret_cast<const Pred*>(w + L.preds);
    uint32_t* counts = reinterpret_cast<uint32_t*>(w + L.counts);
    unsigned long long* offs = reinterpret_cast<unsigned long long*>(w + L.offs);
    if (qk > 0) {
        if (vec)
            hipLaunchKernelGGL(k_ss_count<true>, dim3(g), dim3(kTPB), 0, st, d_col, n, rpb, dp, qk, counts, nwc);
        else
            hipLaunchKernelGGL(k_ss_count<false>, dim3(g), dim3(kTPB), 0, st, d_col, n, rpb, dp, qk, counts, nwc);
        LAUNCHCHK("k_ss_count");
        if ((rc = scan_u32_exclusive(counts, offs, (uint64_t)qk * nwc,
                                     reinterpret_cast<unsigned long long*>(w + L.scratch), st)))
            return rc;
    }
    hipLaunchKernelGGL(k_ss_totals, dim3(1), dim3(256), 0, st, counts, offs, nwc, qk,
                       reinterpret_cast<const int*>(w + L.slot), d_totals, q);
    LAUNCHCHK("k_ss_totals");
    *state = SsState{g, rpb, q, qk, n, d_col};
    return MQ_OK;
}

int ss_write(const SsState& S, int32_t* const* d_pos_out, void* d_ws, hipStream_t st) {
    if (S.qk == 0) return MQ_OK;
    static thread_local int32_t* hout[kMaxQ];
    static thread_local int hslot[kMaxQ];
    char* w = static_cast<char*>(d_ws);
    const uint64_t nwc = (uint64_t)S.g * kWaves;
    const SsLayout L = ss_layout(nwc, S.qk);
    HIPCHK(hipMemcpyAsync(hslot, w + L.slot, sizeof(int) * S.q, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    for (int i = 0; i < S.q; i++)
        if (hslot[i] >= 0) hout[hslot[i]] = d_pos_out[i];
    HIPCHK(hipMemcpyAsync(w + L.outs, hout, sizeof(int*) * S.qk, hipMemcpyHostToDevice, st));
    HIPCHK(hipStreamSynchronize(st));
    const Pred* dp = reinterpret_cast<const Pred*>(w + L.preds);
    const unsigned long long* offs = reinterpret_cast<const unsigned long long*>(w + L.offs);
    int* const* outs = reinterpret_cast<int* const*>(w + L.outs);
    if (aligned16(S.col))
        hipLaunchKernelGGL(k_ss_write<true>, dim3(S.g), dim3(kTPB), 0, st, S.col, S.n, S.rpb, dp, S.qk, offs, nwc, outs);
    else
        hipLaunchKernelGGL(k_ss_write<false>, dim3(S.g), dim3(kTPB), 0, st, S.col, S.n, S.rpb, dp, S.qk, offs, nwc, outs);
    LAUNCHCHK("k_ss_write");
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
    const size_t a = ss_layout(max_wave_chunks(s), q).total;
    const size_t b = mq_scan_workspace_bytes(n);  // the Q = 1 path of mq_shared_select
    return a > b ? a : b;
}

int mq_shared_select_count(const int32_t* d_col, uint64_t n, const int32_t* h_lows,
                           const int32_t* h_highs, int q, uint64_t* h_counts, void* d_ws,
                           size_t ws_bytes, void* stream) {
    if (!h_counts) return set_err(MQ_EINVAL, "mq_shared_select_count: NULL counts");
    hipStream_t st = (hipStream_t)stream;
    // totals land in the preds region's tail? keep them in their own small buffer
    static thread_local uint64_t* d_tot[kMaxDev];
    int dev;
    int rc = current_device(&dev);
    if (rc) return rc;
    if (!d_tot[dev]) HIPCHK(hipMalloc(&d_tot[dev], kMaxQ * sizeof(uint64_t)));
    SsState S;
    if ((rc = ss_count(d_col, n, h_lows, h_highs, q, d_tot[dev], d_ws, ws_bytes, st, &S))) return rc;
    HIPCHK(hipMemcpyAsync(h_counts, d_tot[dev], sizeof(uint64_t) * q, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
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
    if (q == 1)  // one query: the ordered-compaction path reads the column once
        return mq_select_positions(d_col, nullptr, n, 1, h_lows[0], 1, h_highs[0], d_pos_out[0],
                                   d_counts, d_ws, ws_bytes, stream);
    SsState S;
    hipStream_t st = (hipStream_t)stream;
    if ((rc = ss_count(d_col, n, h_lows, h_highs, q, d_counts, d_ws, ws_bytes, st, &S))) return rc;
    return ss_write(S, d_pos_out, d_ws, st);
}

}  // extern "C"
