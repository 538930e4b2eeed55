// mq_format.hip — result serialisation for print (src/query.c:245-304) on gfx950.
//
// The reference formats every value with sprintf("%d") and joins them with "\n"
// (query.c:262-268). After a GPU select of 1e7 rows that host loop is the
// slowest step of the query; here it is three data-parallel passes:
//   k_fmt_len   : bytes per value (sign + digits, + 1 for the "\n" separator);
//   exclusive scan of the lengths (the u32 scan shared with the join);
//   k_fmt_write : each thread writes its digits at its offset.
// The bytes are exactly glibc's "%d" output (INT_MIN included).

#include <hip/hip_runtime.h>

#include <cstdint>

#include "mq_common.h"
#include "mq_device.h"

namespace {

using namespace mqi;

constexpr int kTPB = 256;

__device__ __forceinline__ uint32_t magnitude(int32_t v) {
    return v < 0 ? 0u - (uint32_t)v : (uint32_t)v;  // INT_MIN -> 2147483648
}

__device__ __forceinline__ uint32_t ndigits(uint32_t m) {
    uint32_t d = 1;
    d += m >= 10u;
    d += m >= 100u;
    d += m >= 1000u;
    d += m >= 10000u;
    d += m >= 100000u;
    d += m >= 1000000u;
    d += m >= 10000000u;
    d += m >= 100000000u;
    d += m >= 1000000000u;
    return d;
}

__global__ __launch_bounds__(kTPB) void k_fmt_len(const int32_t* __restrict__ v, uint64_t n,
                                                  uint32_t* __restrict__ len) {
    const uint64_t stride = (uint64_t)gridDim.x * kTPB;
    for (uint64_t i = (uint64_t)blockIdx.x * kTPB + threadIdx.x; i < n; i += stride) {
        const int32_t x = v[i];
        len[i] = ndigits(magnitude(x)) + (x < 0 ? 1u : 0u) + (i + 1 < n ? 1u : 0u);
    }
}

__global__ __launch_bounds__(kTPB) void k_fmt_write(const int32_t* __restrict__ v, uint64_t n,
                                                    const unsigned long long* __restrict__ offs,
                                                    char* __restrict__ out) {
    const uint64_t stride = (uint64_t)gridDim.x * kTPB;
    for (uint64_t i = (uint64_t)blockIdx.x * kTPB + threadIdx.x; i < n; i += stride) {
        const int32_t x = v[i];
        uint32_t m = magnitude(x);
        const uint32_t nd = ndigits(m);
        char* p = out + offs[i];
        if (x < 0) *p++ = '-';
        char buf[10];
#pragma unroll
        for (int k = 9; k >= 0; k--) {
            buf[k] = (char)('0' + m % 10u);
            m /= 10u;
        }
        for (uint32_t k = 0; k < nd; k++) p[k] = buf[10 - nd + k];
        if (i + 1 < n) p[nd] = '\n';
    }
}

// ---- a table as CSV rows: "%d" per cell, ',' between columns, '\n' after each row
__device__ __forceinline__ uint32_t cell_len(int32_t x) { return ndigits(magnitude(x)) + (x < 0 ? 1u : 0u); }

__device__ __forceinline__ char* put_int(char* p, int32_t x) {
    uint32_t m = magnitude(x);
    const uint32_t nd = ndigits(m);
    if (x < 0) *p++ = '-';
    for (uint32_t k = nd; k-- > 0;) {
        p[k] = (char)('0' + m % 10u);
        m /= 10u;
    }
    return p + nd;
}

__global__ __launch_bounds__(kTPB) void k_csv_row_len(const int32_t* const* __restrict__ cols, int ncols,
                                                      uint64_t rows, uint32_t* __restrict__ len) {
    const uint64_t stride = (uint64_t)gridDim.x * kTPB;
    for (uint64_t r = (uint64_t)blockIdx.x * kTPB + threadIdx.x; r < rows; r += stride) {
        uint32_t l = 0;
        for (int j = 0; j < ncols; j++) l += cell_len(cols[j][r]) + 1u;
        len[r] = l;
    }
}

__global__ __launch_bounds__(kTPB) void k_csv_row_write(const int32_t* const* __restrict__ cols, int ncols,
                                                        uint64_t rows, const unsigned long long* __restrict__ offs,
                                                        char* __restrict__ out) {
    const uint64_t stride = (uint64_t)gridDim.x * kTPB;
    for (uint64_t r = (uint64_t)blockIdx.x * kTPB + threadIdx.x; r < rows; r += stride) {
        char* p = out + offs[r];
        for (int j = 0; j < ncols; j++) {
            p = put_int(p, cols[j][r]);
            *p++ = j + 1 < ncols ? ',' : '\n';
        }
    }
}

}  // namespace

extern "C" {

size_t mq_format_csv_workspace_bytes(uint64_t rows, int ncols) {
    (void)ncols;
    return 8192 + (size_t)rows * 4 + 16 + (size_t)rows * 8 + 16 + (size_t)scan_u32_scratch_elems(rows) * 8 + 16;
}

int mq_format_csv_int32(const int32_t* const* d_cols, int ncols, uint64_t rows, char* d_out,
                        uint64_t* h_len, void* d_ws, size_t ws_bytes, void* stream) {
    DevState* s;
    int rc = ensure_ready(&s);
    if (rc) return rc;
    if (!h_len || ncols < 1 || ncols > 1024 || (rows && (!d_cols || !d_out || !d_ws)))
        return set_err(MQ_EINVAL, "mq_format_csv_int32: bad argument");
    *h_len = 0;
    if (rows == 0) return MQ_OK;
    if (ws_bytes < mq_format_csv_workspace_bytes(rows, ncols))
        return set_err(MQ_EINVAL, "mq_format_csv_int32: workspace too small");
    hipStream_t st = (hipStream_t)stream;
    char* w = static_cast<char*>(d_ws);
    const int32_t** dcols = reinterpret_cast<const int32_t**>(w);
    w += 8192;
    uint32_t* len = reinterpret_cast<uint32_t*>(w);
    w += ((size_t)rows * 4 + 15) & ~(size_t)15;
    unsigned long long* offs = reinterpret_cast<unsigned long long*>(w);
    w += (size_t)rows * 8 + 16;
    unsigned long long* scratch = reinterpret_cast<unsigned long long*>(w);
    HIPCHK(hipMemcpyAsync(dcols, d_cols, (size_t)ncols * 8, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_csv_row_len, dim3(stream_grid(s, rows)), dim3(kTPB), 0, st, dcols, ncols, rows, len);
    LAUNCHCHK("k_csv_row_len");
    if ((rc = scan_u32_exclusive(len, offs, rows, scratch, st))) return rc;
    hipLaunchKernelGGL(k_csv_row_write, dim3(stream_grid(s, rows)), dim3(kTPB), 0, st, dcols, ncols, rows,
                       offs, d_out);
    LAUNCHCHK("k_csv_row_write");
    unsigned long long last_off = 0;
    uint32_t last_len = 0;
    HIPCHK(hipMemcpyAsync(&last_off, offs + (rows - 1), 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(&last_len, len + (rows - 1), 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    *h_len = last_off + last_len;
    return MQ_OK;
}


size_t mq_format_workspace_bytes(uint64_t n) {
    return (size_t)n * 4 + 16 + (size_t)n * 8 + 16 + (size_t)scan_u32_scratch_elems(n) * 8 + 16;
}

int mq_format_int32(const int32_t* d_vals, uint64_t n, char* d_out, uint64_t* h_len, void* d_ws,
                    size_t ws_bytes, void* stream) {
    DevState* s;
    int rc = ensure_ready(&s);
    if (rc) return rc;
    if (!h_len || (n && (!d_vals || !d_out || !d_ws)))
        return set_err(MQ_EINVAL, "mq_format_int32: NULL pointer");
    *h_len = 0;
    if (n == 0) return MQ_OK;
    if (ws_bytes < mq_format_workspace_bytes(n))
        return set_err(MQ_EINVAL, "mq_format_int32: workspace too small");
    hipStream_t st = (hipStream_t)stream;
    char* w = static_cast<char*>(d_ws);
    uint32_t* len = reinterpret_cast<uint32_t*>(w);
    w += ((size_t)n * 4 + 15) & ~(size_t)15;
    unsigned long long* offs = reinterpret_cast<unsigned long long*>(w);
    w += (size_t)n * 8 + 16;
    unsigned long long* scratch = reinterpret_cast<unsigned long long*>(w);
    hipLaunchKernelGGL(k_fmt_len, dim3(stream_grid(s, n)), dim3(kTPB), 0, st, d_vals, n, len);
    LAUNCHCHK("k_fmt_len");
    if ((rc = scan_u32_exclusive(len, offs, n, scratch, st))) return rc;
    hipLaunchKernelGGL(k_fmt_write, dim3(stream_grid(s, n)), dim3(kTPB), 0, st, d_vals, n, offs,
                       d_out);
    LAUNCHCHK("k_fmt_write");
    unsigned long long last_off = 0;
    uint32_t last_len = 0;
    HIPCHK(hipMemcpyAsync(&last_off, offs + (n - 1), 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(&last_len, len + (n - 1), 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    *h_len = last_off + last_len;
    return MQ_OK;
}

}  // extern "C"
