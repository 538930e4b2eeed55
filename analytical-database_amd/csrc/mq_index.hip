// mq_index.hip — the sorted index build on gfx950 (src/index.c:89-178).
//
// The reference builds an index at load time (server.c:125 -> build_index):
//   init_column_index (:89-100): values = a copy of the column, positions = 0..n-1;
//   quicksort (:25-46, Lomuto, last element as pivot) of values, carrying positions;
//   clustered (:119-135): the permutation reorders every OTHER column of the table
//     (reorder_column :105-114, out[i] = in[perm[i]]), and index->positions stays
//     0..n-1 (the sort ran on a copy);
//   unclustered (:140-143): index->positions is the permutation; plus a 100-bin
//     histogram of the column (build_histogram :63-84).
// Here the sort is the stable LSD radix sort of (value, row) pairs shared with the
// join (4 passes of 8 bits: histogram, scan, ballot-ranked LDS-staged scatter; the
// last pass writes int32 values and size_t positions), so rows of equal
// value come out in ascending row order. The reference's quicksort leaves equal
// values in an order of its own making (Lomuto partitions rotate the >= side); the
// sorted values and, for distinct values, the positions are identical, and for
// equal values each value's set of positions is.
//   k_gather_u64 : reorder_column / fetch through size_t positions
//   k_histogram  : build_histogram's bins, LDS-privatised counts

#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "mq_common.h"
#include "mq_device.h"

namespace {

using namespace mqi;

constexpr int kTPB = 256;
constexpr int kBins = 100;  // BIN_NUM (cs165_api.h:46)

// kGatherU rows per lane per step: their positions are loaded, then all their
// random reads are in flight before any is stored (a plain grid-stride loop waits
// out two dependent HBM round trips per row). Full steps carry no guards; the one
// partial step at the end does.
constexpr int kGatherU = 8;
__global__ __launch_bounds__(kTPB) void k_gather_u64(const int32_t* __restrict__ col,
                                                      const unsigned long long* __restrict__ pos,
                                                      uint64_t n, int32_t* __restrict__ out) {
    const uint64_t step = (uint64_t)gridDim.x * kTPB * kGatherU;
    uint64_t i0 = (uint64_t)blockIdx.x * kTPB * kGatherU + threadIdx.x;
    for (; i0 + (uint64_t)(kGatherU - 1) * kTPB < n; i0 += step) {
        unsigned long long p[kGatherU];
        int32_t v[kGatherU];
#pragma unroll
        for (int u = 0; u < kGatherU; u++) p[u] = pos[i0 + (uint64_t)u * kTPB];
#pragma unroll
        for (int u = 0; u < kGatherU; u++) v[u] = col[p[u]];
#pragma unroll
        for (int u = 0; u < kGatherU; u++) out[i0 + (uint64_t)u * kTPB] = v[u];
    }
    // i0 + step > n here, so this partial step is the last one
#pragma unroll
    for (int u = 0; u < kGatherU; u++) {
        const uint64_t i = i0 + (uint64_t)u * kTPB;
        if (i < n) out[i] = col[pos[i]];
    }
}

// build_histogram (index.c:63-84): bin of a row = (data - min) / bin_size, an int
// division; rows whose bin falls outside [0, 100) are counted in out_of_range (the
// reference writes past its array there).
__global__ __launch_bounds__(kTPB) void k_histogram(const int32_t* __restrict__ col, uint64_t n, int32_t mn,
                                                     int32_t bin_size, unsigned long long* __restrict__ counts) {
    __shared__ unsigned int h[kBins + 1];
    for (int i = threadIdx.x; i <= kBins; i += kTPB) h[i] = 0;
    __syncthreads();
    const uint64_t stride = (uint64_t)gridDim.x * kTPB;
    for (uint64_t i = (uint64_t)blockIdx.x * kTPB + threadIdx.x; i < n; i += stride) {
        const int b = (int)((uint32_t)col[i] - (uint32_t)mn) / bin_size;  // two's-complement wrap
        atomicAdd(&h[(b >= 0 && b < kBins) ? b : kBins], 1u);
    }
    __syncthreads();
    for (int i = threadIdx.x; i <= kBins; i += kTPB)
        if (h[i]) atomicAdd(&counts[i], (unsigned long long)h[i]);
}

// ---------------------------------------------------------------------------
// The reference's quicksort order (index.c:25-46), level by level.
//
// quicksort(low, high) partitions [low, high] around values[high] (Lomuto) and
// recurses on both sides; disjoint ranges do not interact, so every range of one
// recursion depth is partitioned at once. One partition of a range with c values
// below the pivot, restated without its sequential loop:
//   * the k-th value below the pivot (index j_k, in index order) is swapped with
//     index low + k, so it ends at low + k: the "<" side is a stable compaction;
//   * a value >= the pivot moves only when it sits at low + k as the k-th "<" value
//     is found (j_k is beyond it); it then jumps to j_k. From index x it therefore
//     follows x -> J[x] -> J[J[x]] ... (J[low + k] = j_k) until the index leaves
//     [low, low + c): a chain walk, or pointer doubling when a chain is long;
//   * the final swap puts the pivot at low + c and the value that ended there at high.
// A range whose values all equal its pivot would recurse one element per level
// (O(n) depth); its outcome has a closed form: the last value first, then the
// others in order (by induction over the partitions), so it finishes at once.
// Values and row ids move as (int32, u32) pairs; SID is each index's range id at the
// current depth (-1: final). Levels cost a few passes over n each; the host reads
// one count per level.
// ---------------------------------------------------------------------------
struct LSeg {
    uint32_t lo, hi;
};

__global__ __launch_bounds__(kTPB) void k_lq_init(const int32_t* __restrict__ col, uint64_t n, int32_t* __restrict__ V,
                                                  uint32_t* __restrict__ P, int32_t* __restrict__ SID) {
    const uint64_t stride = (uint64_t)gridDim.x * kTPB;
    for (uint64_t i = (uint64_t)blockIdx.x * kTPB + threadIdx.x; i < n; i += stride) {
        V[i] = col[i];
        P[i] = (uint32_t)i;
        SID[i] = 0;
    }
}

// per index: (v < pivot) in the low 32 bits, (v > pivot) in the high 32 bits
__global__ __launch_bounds__(kTPB) void k_lq_flags(const int32_t* __restrict__ V, const int32_t* __restrict__ SID,
                                                   const LSeg* __restrict__ seg, uint64_t n,
                                                   unsigned long long* __restrict__ FL) {
    const uint64_t stride = (uint64_t)gridDim.x * kTPB;
    for (uint64_t i = (uint64_t)blockIdx.x * kTPB + threadIdx.x; i < n; i += stride) {
        const int32_t sid = SID[i];
        unsigned long long f = 0;
        if (sid >= 0) {
            const uint32_t hi = seg[sid].hi;
            if ((uint32_t)i != hi) {
                const int32_t piv = V[hi], v = V[i];
                f = (v < piv ? 1ull : 0ull) | (v > piv ? (1ull << 32) : 0ull);
            }
        }
        FL[i] = f;
    }
}

// per range: c, all-equal, children (ranges of >= 2 indexes)
__global__ __launch_bounds__(kTPB) void k_lq_segs(const LSeg* __restrict__ seg, uint32_t S,
                                                  const unsigned long long* __restrict__ EX,
                                                  uint32_t* __restrict__ segc, uint32_t* __restrict__ nchild) {
    for (uint32_t s = blockIdx.x * kTPB + threadIdx.x; s < S; s += gridDim.x * kTPB) {
        const LSeg g = seg[s];
        const unsigned long long tot = EX[g.hi] - EX[g.lo];  // the pivot's own flag is 0
        const uint32_t c = (uint32_t)tot, gt = (uint32_t)(tot >> 32), m = g.hi - g.lo;
        const bool eq = c == 0 && gt == 0;
        segc[s] = eq ? 0xFFFFFFFFu : c;
        nchild[s] = eq ? 0u : (uint32_t)(c >= 2) + (uint32_t)(m - c >= 2);
    }
}

__global__ __launch_bounds__(kTPB) void k_lq_children(const LSeg* __restrict__ seg, uint32_t S,
                                                      const uint32_t* __restrict__ segc,
                                                      const uint32_t* __restrict__ nchild,
                                                      const unsigned long long* __restrict__ cbase,
                                                      LSeg* __restrict__ next, int32_t* __restrict__ lid,
                                                      int32_t* __restrict__ rid, unsigned long long* __restrict__ d_snext) {
    for (uint32_t s = blockIdx.x * kTPB + threadIdx.x; s < S; s += gridDim.x * kTPB) {
        const LSeg g = seg[s];
        const uint32_t c = segc[s];
        uint32_t at = (uint32_t)cbase[s];
        int32_t l = -1, r = -1;
        if (c != 0xFFFFFFFFu) {
            const uint32_t m = g.hi - g.lo;
            if (c >= 2) {
                l = (int32_t)at;
                next[at++] = LSeg{g.lo, g.lo + c - 1};
            }
            if (m - c >= 2) {
                r = (int32_t)at;
                next[at] = LSeg{g.lo + c + 1, g.hi};
            }
        }
        lid[s] = l;
        rid[s] = r;
        if (s == S - 1) *d_snext = cbase[s] + nchild[s];
    }
}

// J[lo + rank] = index of the rank-th value below the pivot
__global__ __launch_bounds__(kTPB) void k_lq_less(const int32_t* __restrict__ V, const int32_t* __restrict__ SID,
                                                  const LSeg* __restrict__ seg, const unsigned long long* __restrict__ EX,
                                                  uint64_t n, uint32_t* __restrict__ J) {
    const uint64_t stride = (uint64_t)gridDim.x * kTPB;
    for (uint64_t i = (uint64_t)blockIdx.x * kTPB + threadIdx.x; i < n; i += stride) {
        const int32_t sid = SID[i];
        if (sid < 0) continue;
        const LSeg g = seg[sid];
        if ((uint32_t)i == g.hi || !(V[i] < V[g.hi])) continue;
        J[g.lo + ((uint32_t)EX[i] - (uint32_t)EX[g.lo])] = (uint32_t)i;
    }
}

// chain steps walked before pointer doubling takes over (MQ_LQ_CAP); 2^27 uniform rows:
// 64 -> 288 ms, 128 -> 254, 256 -> 238, 512 -> 231 (the doubling only over flagged ranges)
constexpr int kChainCap = 256;

// One index of k_lq_final (below). Returns false when USE_F is false and the index
// sits on a chain longer than kChainCap (it is placed later, after the doubling).
template <bool USE_F>
__device__ __forceinline__ bool lq_place(uint64_t i, const int32_t* __restrict__ V, const uint32_t* __restrict__ P,
                                         const int32_t* __restrict__ SID, const LSeg* __restrict__ seg,
                                         const unsigned long long* __restrict__ EX, const uint32_t* __restrict__ segc,
                                         const int32_t* __restrict__ lid, const int32_t* __restrict__ rid,
                                         const uint32_t* __restrict__ J, int32_t* __restrict__ Vn,
                                         uint32_t* __restrict__ Pn, int32_t* __restrict__ SIDn, int cap) {
    const int32_t sid = SID[i];
    const int32_t v = V[i];
    const uint32_t row = P[i];
    uint32_t q = (uint32_t)i;
    int32_t ns = -1;
    if (sid >= 0) {
        const LSeg g = seg[sid];
        const uint32_t c = segc[sid];
        if (c == 0xFFFFFFFFu) {                 // all equal: last first, then in order
            q = (uint32_t)i == g.hi ? g.lo : (uint32_t)i + 1;
        } else if ((uint32_t)i == g.hi) {       // the pivot
            q = g.lo + c;
        } else if (v < V[g.hi]) {              // stable compaction of the "<" side
            q = g.lo + ((uint32_t)EX[i] - (uint32_t)EX[g.lo]);
            ns = lid[sid];
        } else {                                // the >= side: follow the swaps
            int steps = 0;
            while (q - g.lo < c) {
                q = J[q];
                if (!USE_F && ++steps > cap) break;
            }
            if (!USE_F && q - g.lo < c) return false;  // long chain: doubling, then placed again
            if (q == g.lo + c) q = g.hi;        // the final swap with the pivot
            ns = rid[sid];
        }
    }
    Vn[q] = v;
    Pn[q] = row;
    SIDn[q] = ns;
    return true;
}

template <bool USE_F>
__global__ __launch_bounds__(kTPB) void k_lq_final(const int32_t* __restrict__ V, const uint32_t* __restrict__ P,
                                                   const int32_t* __restrict__ SID, const LSeg* __restrict__ seg,
                                                   const unsigned long long* __restrict__ EX,
                                                   const uint32_t* __restrict__ segc, const int32_t* __restrict__ lid,
                                                   const int32_t* __restrict__ rid, const uint32_t* __restrict__ J,
                                                   uint64_t n, int32_t* __restrict__ Vn, uint32_t* __restrict__ Pn,
                                                   int32_t* __restrict__ SIDn, unsigned int* __restrict__ long_chain,
                                                   uint8_t* __restrict__ segflag, int cap) {
    const uint64_t stride = (uint64_t)gridDim.x * kTPB;
    for (uint64_t i = (uint64_t)blockIdx.x * kTPB + threadIdx.x; i < n; i += stride) {
        if (!lq_place<USE_F>(i, V, P, SID, seg, EX, segc, lid, rid, J, Vn, Pn, SIDn, cap)) {
            atomicOr(long_chain, 1u);
            segflag[SID[i]] = 1;
        }
    }
}

// Long chains are rare and sit in a few ranges (MQ_LQ_STATS at 2^27: their "<" zones
// hold 20 % of the rows at the top levels and under 2 % below level 30), so the
// doubling and the second placement run only over those ranges: per flagged range,
// items of kZChunk indexes (of its zone for the doubling, of the whole range for the
// placement), a block per item; a block finds its range by a binary search over the
// items' prefix. (Was: both over all n rows, every doubling step and level: 0.42 ms
// a pass, 44 % of the 2^27 build.)
constexpr uint32_t kZChunk = 2048;

__global__ __launch_bounds__(kTPB) void k_lq_items(const LSeg* __restrict__ seg, uint32_t S,
                                                   const uint32_t* __restrict__ segc,
                                                   const uint8_t* __restrict__ segflag, uint32_t* __restrict__ zi,
                                                   uint32_t* __restrict__ fi) {
    for (uint32_t s = blockIdx.x * kTPB + threadIdx.x; s < S; s += gridDim.x * kTPB) {
        const bool f = segflag[s] != 0;
        const uint32_t c = segc[s], m = seg[s].hi - seg[s].lo + 1;
        zi[s] = f && c != 0xFFFFFFFFu ? (c + kZChunk - 1) / kZChunk : 0u;
        fi[s] = f ? (m + kZChunk - 1) / kZChunk : 0u;
    }
}

// the range of item b: the last s with off[s] <= b (off: exclusive prefix of items, S entries)
__device__ __forceinline__ uint32_t lq_item_range(const unsigned long long* __restrict__ off, uint32_t S, uint64_t b) {
    uint32_t lo = 0, hi = S;  // off[lo] <= b < off[hi] (off[S] taken as infinity)
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (off[mid] <= b) lo = mid;
        else hi = mid;
    }
    return lo;
}

__global__ __launch_bounds__(kTPB) void k_lq_jump_z(const LSeg* __restrict__ seg, const uint32_t* __restrict__ segc,
                                                    const unsigned long long* __restrict__ zoff, uint32_t S,
                                                    uint32_t* J, unsigned int* __restrict__ changed) {
    __shared__ uint32_t s_r;
    if (threadIdx.x == 0) s_r = lq_item_range(zoff, S, blockIdx.x);
    __syncthreads();
    const uint32_t r = s_r;
    const uint32_t lo = seg[r].lo, c = segc[r];
    const uint32_t k = blockIdx.x - (uint32_t)zoff[r];
    const uint32_t b = lo + k * kZChunk, e = min(lo + c, b + kZChunk);
    unsigned int any = 0;
    for (uint32_t i = b + threadIdx.x; i < e; i += kTPB) {
        const uint32_t f = J[i];
        if (f != i && f - lo < c) {
            J[i] = J[f];
            any = 1;
        }
    }
    if (__ballot(any) && (threadIdx.x & 63) == 0) atomicOr(changed, 1u);
}

__global__ __launch_bounds__(kTPB) void k_lq_final_z(const int32_t* __restrict__ V, const uint32_t* __restrict__ P,
                                                     const int32_t* __restrict__ SID, const LSeg* __restrict__ seg,
                                                     const unsigned long long* __restrict__ EX,
                                                     const uint32_t* __restrict__ segc, const int32_t* __restrict__ lid,
                                                     const int32_t* __restrict__ rid, const uint32_t* __restrict__ J,
                                                     const unsigned long long* __restrict__ foff, uint32_t S,
                                                     int32_t* __restrict__ Vn, uint32_t* __restrict__ Pn,
                                                     int32_t* __restrict__ SIDn) {
    __shared__ uint32_t s_r;
    if (threadIdx.x == 0) s_r = lq_item_range(foff, S, blockIdx.x);
    __syncthreads();
    const uint32_t r = s_r;
    const uint32_t lo = seg[r].lo, hi = seg[r].hi;
    const uint32_t k = blockIdx.x - (uint32_t)foff[r];
    const uint32_t b = lo + k * kZChunk;
    const uint32_t e = hi + 1 - b < kZChunk ? hi + 1 : b + kZChunk;
    for (uint32_t i = b + threadIdx.x; i < e; i += kTPB)
        (void)lq_place<true>(i, V, P, SID, seg, EX, segc, lid, rid, J, Vn, Pn, SIDn, 0);
}

__global__ __launch_bounds__(kTPB) void k_lq_emit(const int32_t* __restrict__ V, const uint32_t* __restrict__ P,
                                                  uint64_t n, int32_t* __restrict__ vout,
                                                  unsigned long long* __restrict__ pout) {
    const uint64_t stride = (uint64_t)gridDim.x * kTPB;
    for (uint64_t i = (uint64_t)blockIdx.x * kTPB + threadIdx.x; i < n; i += stride) {
        if (vout) vout[i] = V[i];
        if (pout) pout[i] = P[i];
    }
}

// any i with v[i] == v[i+1] in a sorted array
__global__ __launch_bounds__(kTPB) void k_has_ties(const int32_t* __restrict__ v, uint64_t n, unsigned int* __restrict__ flag) {
    const uint64_t stride = (uint64_t)gridDim.x * kTPB;
    unsigned int t = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * kTPB + threadIdx.x; i + 1 < n; i += stride) t |= v[i] == v[i + 1];
    if (__ballot(t) && (threadIdx.x & 63) == 0) atomicOr(flag, 1u);
}

struct LqBufs {
    void* blk[32];
    int nb;
    ~LqBufs() {
        for (int i = 0; i < nb; i++) pool_free(blk[i]);
    }
    template <typename T>
    T* get(size_t count) {
        void* p = pool_alloc((count ? count : 1) * sizeof(T));
        if (p) blk[nb++] = p;
        return static_cast<T*>(p);
    }
};

int lomuto_sort(const int32_t* col, uint64_t n, int32_t* vout, uint64_t* pout, hipStream_t st, const DevState* s) {
    const uint64_t smax = n / 2 + 2;
    LqBufs b;
    b.nb = 0;
    int32_t* V[2] = {b.get<int32_t>(n), b.get<int32_t>(n)};
    uint32_t* P[2] = {b.get<uint32_t>(n), b.get<uint32_t>(n)};
    int32_t* SID[2] = {b.get<int32_t>(n), b.get<int32_t>(n)};
    unsigned long long* EX = b.get<unsigned long long>(n);
    uint32_t* J = b.get<uint32_t>(n);
    LSeg* seg[2] = {b.get<LSeg>(smax), b.get<LSeg>(smax)};
    uint32_t* segc = b.get<uint32_t>(smax);
    uint32_t* nchild = b.get<uint32_t>(smax);
    unsigned long long* cbase = b.get<unsigned long long>(smax);
    int32_t* lid = b.get<int32_t>(smax);
    int32_t* rid = b.get<int32_t>(smax);
    unsigned long long* scratch = b.get<unsigned long long>(scan_u32_scratch_elems(n));
    unsigned long long* small = b.get<unsigned long long>(4);  // [S_next, long_chain | changed]
    uint8_t* segflag = b.get<uint8_t>(smax);                    // ranges with a long chain
    uint32_t* zi = b.get<uint32_t>(smax);                       // per range: doubling items
    uint32_t* fi = b.get<uint32_t>(smax);                       // per range: placement items
    unsigned long long* zoff = b.get<unsigned long long>(smax);
    unsigned long long* foff = b.get<unsigned long long>(smax);
    if (b.nb != 22) return set_err(MQ_ENOMEM, "mq_index_build_lomuto: device allocation failed");
    static const bool stats = getenv("MQ_LQ_STATS") != nullptr;  // per-level diagnostics (stderr)
    std::vector<LSeg> hseg;
    std::vector<uint32_t> hsegc;
    std::vector<uint8_t> hflag;
    int level = 0;
    static const int cap = getenv("MQ_LQ_CAP") ? atoi(getenv("MQ_LQ_CAP")) : kChainCap;
    unsigned int* flags = reinterpret_cast<unsigned int*>(small + 1);
    const uint32_t gn = stream_grid(s, n);
    hipLaunchKernelGGL(k_lq_init, dim3(gn), dim3(kTPB), 0, st, col, n, V[0], P[0], SID[0]);
    LAUNCHCHK("k_lq_init");
    const LSeg root{0u, (uint32_t)(n - 1)};
    HIPCHK(hipMemcpyAsync(seg[0], &root, sizeof root, hipMemcpyHostToDevice, st));
    uint64_t S = n >= 2 ? 1 : 0;
    int cur = 0;
    while (S) {
        const uint32_t gs = stream_grid(s, S);
        hipLaunchKernelGGL(k_lq_flags, dim3(gn), dim3(kTPB), 0, st, V[cur], SID[cur], seg[cur], n, EX);
        LAUNCHCHK("k_lq_flags");
        int rc = scan_u64_exclusive(EX, EX, n, scratch, st);
        if (rc) return rc;
        hipLaunchKernelGGL(k_lq_segs, dim3(gs), dim3(kTPB), 0, st, seg[cur], (uint32_t)S, EX, segc, nchild);
        LAUNCHCHK("k_lq_segs");
        if ((rc = scan_u32_exclusive(nchild, cbase, S, scratch, st))) return rc;
        hipLaunchKernelGGL(k_lq_children, dim3(gs), dim3(kTPB), 0, st, seg[cur], (uint32_t)S, segc, nchild, cbase,
                           seg[cur ^ 1], lid, rid, small);
        LAUNCHCHK("k_lq_children");
        hipLaunchKernelGGL(k_lq_less, dim3(gn), dim3(kTPB), 0, st, V[cur], SID[cur], seg[cur], EX, n, J);
        LAUNCHCHK("k_lq_less");
        HIPCHK(hipMemsetAsync(flags, 0, 8, st));
        HIPCHK(hipMemsetAsync(segflag, 0, S, st));
        hipLaunchKernelGGL(k_lq_final<false>, dim3(gn), dim3(kTPB), 0, st, V[cur], P[cur], SID[cur], seg[cur], EX,
                           segc, lid, rid, J, n, V[cur ^ 1], P[cur ^ 1], SID[cur ^ 1], flags, segflag, cap);
        LAUNCHCHK("k_lq_final");
        unsigned long long h[2];
        HIPCHK(hipMemcpyAsync(h, small, 16, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        int jumps = 0;
        if ((uint32_t)h[1]) {  // chains longer than kChainCap: double J, then place again, flagged ranges only
            const uint32_t gs2 = stream_grid(s, S);
            hipLaunchKernelGGL(k_lq_items, dim3(gs2), dim3(kTPB), 0, st, seg[cur], (uint32_t)S, segc, segflag, zi, fi);
            LAUNCHCHK("k_lq_items");
            if ((rc = scan_u32_exclusive(zi, zoff, S, scratch, st))) return rc;
            if ((rc = scan_u32_exclusive(fi, foff, S, scratch, st))) return rc;
            unsigned long long t[2];
            uint32_t l[2];
            HIPCHK(hipMemcpyAsync(&t[0], zoff + (S - 1), 8, hipMemcpyDeviceToHost, st));
            HIPCHK(hipMemcpyAsync(&t[1], foff + (S - 1), 8, hipMemcpyDeviceToHost, st));
            HIPCHK(hipMemcpyAsync(&l[0], zi + (S - 1), 4, hipMemcpyDeviceToHost, st));
            HIPCHK(hipMemcpyAsync(&l[1], fi + (S - 1), 4, hipMemcpyDeviceToHost, st));
            HIPCHK(hipStreamSynchronize(st));
            const uint64_t nz = t[0] + l[0], nf = t[1] + l[1];
            for (int it = 0; nz; it++, jumps++) {
                if (it > 40) return set_err(MQ_EHIP, "mq_index_build_lomuto: pointer doubling did not converge");
                HIPCHK(hipMemsetAsync(flags + 1, 0, 4, st));
                hipLaunchKernelGGL(k_lq_jump_z, dim3((uint32_t)nz), dim3(kTPB), 0, st, seg[cur], segc, zoff,
                                   (uint32_t)S, J, flags + 1);
                LAUNCHCHK("k_lq_jump_z");
                unsigned int ch = 0;
                HIPCHK(hipMemcpyAsync(&ch, flags + 1, 4, hipMemcpyDeviceToHost, st));
                HIPCHK(hipStreamSynchronize(st));
                if (!ch) break;
            }
            if (nf) {
                hipLaunchKernelGGL(k_lq_final_z, dim3((uint32_t)nf), dim3(kTPB), 0, st, V[cur], P[cur], SID[cur],
                                   seg[cur], EX, segc, lid, rid, J, foff, (uint32_t)S, V[cur ^ 1], P[cur ^ 1],
                                   SID[cur ^ 1]);
                LAUNCHCHK("k_lq_final_z");
            }
        }
        if (stats) {
            hseg.resize(S);
            hsegc.resize(S);
            hflag.resize(S);
            HIPCHK(hipMemcpy(hseg.data(), seg[cur], S * sizeof(LSeg), hipMemcpyDeviceToHost));
            HIPCHK(hipMemcpy(hsegc.data(), segc, S * 4, hipMemcpyDeviceToHost));
            HIPCHK(hipMemcpy(hflag.data(), segflag, S, hipMemcpyDeviceToHost));
            uint64_t act = 0, big = 0, nbig = 0, nfl = 0, zfl = 0, efl = 0, maxm = 0;
            for (uint64_t k = 0; k < S; k++) {
                const uint64_t m = (uint64_t)hseg[k].hi - hseg[k].lo + 1;
                act += m;
                if (m > maxm) maxm = m;
                if (m > 2048) big += m, nbig++;
                if (hflag[k]) nfl++, efl += m, zfl += hsegc[k] == 0xFFFFFFFFu ? 0 : hsegc[k];
            }
            fprintf(stderr, "lq level %d: ranges %llu active %llu max %llu | >2048: %llu ranges %llu rows | long: %llu ranges, "
                    "%llu rows, zones %llu, jumps %d\n", level, (unsigned long long)S, (unsigned long long)act,
                    (unsigned long long)maxm, (unsigned long long)nbig, (unsigned long long)big, (unsigned long long)nfl,
                    (unsigned long long)efl, (unsigned long long)zfl, jumps);
        }
        level++;
        S = h[0];
        cur ^= 1;
    }
    hipLaunchKernelGGL(k_lq_emit, dim3(gn), dim3(kTPB), 0, st, V[cur], P[cur], n, vout,
                       reinterpret_cast<unsigned long long*>(pout));
    LAUNCHCHK("k_lq_emit");
    HIPCHK(hipStreamSynchronize(st));  // the scratch goes back to the pool
    return MQ_OK;
}

}  // namespace

extern "C" {

int mq_index_build_lomuto(const int32_t* d_col, uint64_t n, int32_t* d_values_out, uint64_t* d_positions_out,
                          void* stream) {
    DevState* s;
    int rc = ensure_ready(&s);
    if (rc) return rc;
    if (n && (!d_col || (!d_values_out && !d_positions_out)))
        return set_err(MQ_EINVAL, "mq_index_build_lomuto: NULL pointer");
    if (n >= (1ull << 31)) return set_err(MQ_EINVAL, "mq_index_build_lomuto: n >= 2^31");
    if (n == 0) return MQ_OK;
    return lomuto_sort(d_col, n, d_values_out, d_positions_out, (hipStream_t)stream, s);
}

int mq_index_build_ref(const int32_t* d_col, uint64_t n, int32_t* d_values_out, uint64_t* d_positions_out,
                       uint64_t exact_max, int* h_exact, void* stream) {
    DevState* s;
    int rc = ensure_ready(&s);
    if (rc) return rc;
    if (!d_values_out || (n && !d_col)) return set_err(MQ_EINVAL, "mq_index_build_ref: NULL pointer");
    if (h_exact) *h_exact = 1;
    if ((rc = mq_index_build(d_col, n, d_values_out, d_positions_out, stream)) || n < 2) return rc;
    // distinct values: the sort order is unique, the radix result is the reference's
    hipStream_t st = (hipStream_t)stream;
    unsigned int* flag = static_cast<unsigned int*>(pool_alloc(4));
    if (!flag) return set_err(MQ_ENOMEM, "mq_index_build_ref: allocation failed");
    unsigned int ties = 0;
    int e = hipMemsetAsync(flag, 0, 4, st) == hipSuccess ? 0 : 1;
    if (!e) {
        hipLaunchKernelGGL(k_has_ties, dim3(stream_grid(s, n)), dim3(kTPB), 0, st, d_values_out, n, flag);
        e = hipGetLastError() != hipSuccess || hipMemcpyAsync(&ties, flag, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess;
    }
    pool_free(flag);
    if (e) return set_err(MQ_EHIP, "mq_index_build_ref: tie check failed");
    if (!ties) return MQ_OK;
    if (n > exact_max || n >= (1ull << 31)) {
        if (h_exact) *h_exact = 0;  // equal values stay in ascending row order
        return MQ_OK;
    }
    return lomuto_sort(d_col, n, d_values_out, d_positions_out, st, s);
}

int mq_index_build(const int32_t* d_col, uint64_t n, int32_t* d_values_out,
                   uint64_t* d_positions_out, void* stream) {
    DevState* s;
    int rc = ensure_ready(&s);
    if (rc) return rc;
    if (n && (!d_col || (!d_values_out && !d_positions_out)))
        return set_err(MQ_EINVAL, "mq_index_build: NULL pointer");
    if (n >= (1ull << 32)) return set_err(MQ_EINVAL, "mq_index_build: n >= 2^32");
    if (n == 0) return MQ_OK;
    // the last radix pass writes the values and size_t positions directly
    return radix_sort_index(d_col, n, d_values_out, d_positions_out, (hipStream_t)stream);
}

int mq_gather_u64(const int32_t* d_col, const uint64_t* d_positions, uint64_t n, int32_t* d_out,
                  void* stream) {
    DevState* s;
    int rc = ensure_ready(&s);
    if (rc) return rc;
    if (n && (!d_col || !d_positions || !d_out)) return set_err(MQ_EINVAL, "mq_gather_u64: NULL pointer");
    if (n == 0) return MQ_OK;
    hipLaunchKernelGGL(k_gather_u64, dim3(stream_grid(s, (n + kGatherU - 1) / kGatherU)), dim3(kTPB), 0, (hipStream_t)stream, d_col,
                       reinterpret_cast<const unsigned long long*>(d_positions), n, d_out);
    LAUNCHCHK("k_gather_u64");
    return MQ_OK;
}

int mq_histogram(const int32_t* d_col, uint64_t n, int32_t col_min, int32_t bin_size,
                 uint64_t* d_counts, void* stream) {
    DevState* s;
    int rc = ensure_ready(&s);
    if (rc) return rc;
    if (!d_counts || (n && !d_col)) return set_err(MQ_EINVAL, "mq_histogram: NULL pointer");
    if (bin_size == 0) return set_err(MQ_EINVAL, "mq_histogram: bin_size 0 (the reference divides by it)");
    hipStream_t st = (hipStream_t)stream;
    HIPCHK(hipMemsetAsync(d_counts, 0, (kBins + 1) * 8, st));
    if (n == 0) return MQ_OK;
    hipLaunchKernelGGL(k_histogram, dim3(stream_grid(s, n)), dim3(kTPB), 0, st, d_col, n, col_min, bin_size,
                       reinterpret_cast<unsigned long long*>(d_counts));
    LAUNCHCHK("k_histogram");
    return MQ_OK;
}

}  // extern "C"
