// mq_scan_common.h — internal (not exported) pieces shared by libmq's scan kernels:
// the tile geometry, the predicate fold, per-block partials and the nt loads.
#pragma once

#include <hip/hip_runtime.h>

#include <climits>
#include <cstddef>
#include <cstdint>

#include "mq_common.h"

namespace mqi {

constexpr int kTPB = 256;                 // scan block: 4 wave64
constexpr int kWaves = kTPB / 64;
constexpr int kTileRows = kTPB * 4;       // 1024 rows per tile (one dwordx4 per lane)
constexpr int kUnroll = 8;                // tiles in flight per thread (128 B/lane)
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
    int32_t base;  // added to emitted row positions (a row shard's first row; 0 otherwise)
};

template <bool VEC>
__device__ __forceinline__ int4 load4(const int* __restrict__ p) {  // cached (fetch / add / sub)
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

typedef int v4i __attribute__((ext_vector_type(4)));

template <bool VEC>
__device__ __forceinline__ int4 load4_nt(const int* __restrict__ p) {
    if constexpr (VEC) {
        const v4i t = __builtin_nontemporal_load(reinterpret_cast<const v4i*>(p));
        return make_int4(t.x, t.y, t.z, t.w);
    } else {
        return make_int4(__builtin_nontemporal_load(p), __builtin_nontemporal_load(p + 1),
                         __builtin_nontemporal_load(p + 2), __builtin_nontemporal_load(p + 3));
    }
}

// Per-mode tiles in flight and occupancy target (waves per SIMD): 8 waves/SIMD
// means <= 64 VGPRs, chosen where it fits without spills.

inline bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

// Fold (has_low, low, has_high, high) into one unsigned range compare; false = empty.
bool make_pred(int has_low, int32_t low, int has_high, int32_t high, Pred* p);
// Resident blocks of kTPB threads per CU for one kernel with dyn_lds bytes of dynamic
// LDS (cached per kernel and size).
int blocks_per_cu(const void* fn, size_t dyn_lds = 0);
// One wave of resident blocks, each owning a contiguous chunk of whole granules
// (bpc_cap > 0: at most that many blocks a CU).
void geometry(const DevState* s, uint64_t n, const void* fn, uint32_t* blocks, uint64_t* rpb,
              uint64_t granule = kTileRows, size_t dyn_lds = 0, int bpc_cap = 0);
// Bytes of the per-block partial slab at the start of every scan workspace.
size_t partial_bytes();

}  // namespace mqi
