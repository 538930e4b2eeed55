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

// any i with v[i] == v[i+1] in a sorted array
__global__ __launch_bounds__(kTPB) void k_has_ties(const int32_t* __restrict__ v, uint64_t n, unsigned int* __restrict__ flag) {
    const uint64_t stride = (uint64_t)gridDim.x * kTPB;
    unsigned int t = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * kTPB + threadIdx.x; i + 1 < n; i += stride) t |= v[i] == v[i + 1];
    if (__ballot(t) && (threadIdx.x & 63) == 0) atomicOr(flag, 1u);
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
