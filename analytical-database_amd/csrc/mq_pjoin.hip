// mq_pjoin.hip — the device pieces of the key-partitioned hash join (SURVEY.md §8(e):
// "radix-partitioning by key with an all-to-all"), for src/query.c:652-696 over G
// devices.
//
// Protocol. The build side and the probe side are each split into G
// contiguous row ranges in row order, range s on device s ("shard s").
//  1. partition: shard s splits its build rows (key, build position) and its probe
//     keys into G buckets by a hash of the key, stably (mq_pjoin_partition); for the
//     probe side it also records where each row went (inv[r] = its partitioned index).
//  2. exchange: device g takes bucket g of every shard, in shard order. Its build
//     input is then bucket g's rows in ascending global build order, its probe input
//     bucket g's rows in ascending global probe order, and every row of a key is on
//     the key's one device.
//  3. local join on device g (mq_join_build / probe): its pairs are exactly the
//     reference's pairs of those probe rows, in the reference's order restricted to
//     them (probe-major; a key's build rows in insertion order). mq_join_counts gives
//     each of its probe rows its match count; mq_join_write the build positions.
//  4. return exchange: shard s takes back, from every device g, the counts of its own
//     bucket-g rows and the pairs of those rows (out1 only), in g order: that is its
//     probe rows' counts and pairs in its partitioned order.
//  5. place (mq_pjoin_place): shard s gives each of its probe rows r its output
//     offset (a scan of the counts in row order) and copies the row's pairs there from
//     the partitioned stream, with out2 = p2[r]. Shard s's output is the reference's
//     output for probe rows of range s; the concatenation over s is the whole output.
// Nothing in the protocol sorts: both exchanges keep every row's relative order.
//
// The in-process driver over the row-shard workers is mq_shard_join (mq_shard.c, peer
// copies); analytical-database_amd/dist.py runs the same steps one process per GPU
// with all_to_all exchanges.

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>

#include "mq_common.h"
#include "mq_device.h"

namespace {

using namespace mqi;

constexpr int kTPB = 256;
constexpr int kWaves = kTPB / 64;
constexpr uint32_t kItems = 16;                // 64-row items per wave chunk
constexpr uint32_t kChunk = 64 * kItems;       // 1024 rows: one wave's contiguous rows
constexpr uint32_t kLongRun = 4096;            // a run longer than this is copied by a block
constexpr uint32_t kLongChunk = 65536;

typedef unsigned long long u64;

// The bucket of a key: a hash independent of the join table's (hash32, a murmur3
// finaliser on the key), so that one device's keys still spread over its table.
// "lowbias32" mix of key ^ golden ratio, then the multiply-shift range map to [0, G).
__host__ __device__ __forceinline__ uint32_t pj_part(uint32_t key, uint32_t G) {
    uint32_t h = key ^ 0x9E3779B9u;
    h ^= h >> 16;
    h *= 0x7feb352du;
    h ^= h >> 15;
    h *= 0x846ca68bu;
    h ^= h >> 16;
    return (uint32_t)(((uint64_t)h * G) >> 32);
}

// Per wave chunk of 1024 rows, the rows of each bucket: lane b holds bucket b's count
// (G <= 64), stored bucket-major (hist[b * nchunks + c]) so that one exclusive scan gives
// every (bucket, chunk) its first output index, chunks in row order within a bucket.
__global__ __launch_bounds__(kTPB) void k_pj_hist(const int* __restrict__ keys, uint64_t n, uint32_t G,
                                                  uint64_t nchunks, uint32_t* __restrict__ hist) {
    const int lane = threadIdx.x & 63;
    const uint64_t c = (uint64_t)blockIdx.x * kWaves + (threadIdx.x >> 6);
    if (c >= nchunks) return;
    const uint64_t r0 = c * kChunk;
    uint32_t p[kItems];
#pragma unroll
    for (uint32_t k = 0; k < kItems; k++) {
        const uint64_t r = r0 + k * 64 + (uint64_t)lane;
        p[k] = r < n ? pj_part((uint32_t)keys[r], G) : 0xFFFFFFFFu;
    }
    uint32_t mine = 0;
#pragma unroll
    for (uint32_t k = 0; k < kItems; k++)
        for (uint32_t b = 0; b < G; b++) {
            const uint32_t cb = (uint32_t)__popcll(__ballot(p[k] == b));
            if ((uint32_t)lane == b) mine += cb;
        }
    if ((uint32_t)lane < G) hist[(uint64_t)lane * nchunks + c] = mine;
}

// The stable scatter: row r of chunk c with bucket b goes to base(b, c) + the rows of
// bucket b before it in the chunk (lane b of the wave carries bucket b's running
// index). keys_out / pay_out / inv receive key, payload and the row's new index.
__global__ __launch_bounds__(kTPB) void k_pj_scatter(const int* __restrict__ keys, const int* __restrict__ pay,
                                                     uint64_t n, uint32_t G, uint64_t nchunks,
                                                     const u64* __restrict__ base, int* __restrict__ keys_out,
                                                     int* __restrict__ pay_out, uint32_t* __restrict__ inv) {
    const int lane = threadIdx.x & 63;
    const uint64_t c = (uint64_t)blockIdx.x * kWaves + (threadIdx.x >> 6);
    if (c >= nchunks) return;
    const uint64_t r0 = c * kChunk;
    const u64 lt = (1ull << lane) - 1;
    u64 run = (uint32_t)lane < G ? base[(uint64_t)lane * nchunks + c] : 0;
    int kv[kItems], pv[kItems];
#pragma unroll
    for (uint32_t k = 0; k < kItems; k++) {
        const uint64_t r = r0 + k * 64 + (uint64_t)lane;
        const uint64_t rc = r < n ? r : n - 1;  // clamped: every load issued before any is used
        kv[k] = keys[rc];
        pv[k] = pay ? pay[rc] : 0;
    }
#pragma unroll
    for (uint32_t k = 0; k < kItems; k++) {
        const uint64_t r = r0 + k * 64 + (uint64_t)lane;
        const uint32_t p = r < n ? pj_part((uint32_t)kv[k], G) : 0xFFFFFFFFu;
        u64 dst = 0;
        for (uint32_t b = 0; b < G; b++) {
            const u64 m = __ballot(p == b);
            const u64 rb = __shfl(run, (int)b, 64);
            if (p == b) dst = rb + (u64)__popcll(m & lt);
            if ((uint32_t)lane == b) run += (u64)__popcll(m);
        }
        if (r < n) {
            keys_out[dst] = kv[k];
            if (pay_out) pay_out[dst] = pv[k];
            if (inv) inv[r] = (uint32_t)dst;
        }
    }
}

// counts[b] = rows of bucket b: the difference of consecutive bucket bases
__global__ void k_pj_counts(const u64* __restrict__ base, uint64_t nchunks, uint32_t G, uint64_t n,
                            u64* __restrict__ counts) {
    const uint32_t b = threadIdx.x;
    if (b >= G) return;
    const u64 a = base[(uint64_t)b * nchunks];
    const u64 e = b + 1 < G ? base[(uint64_t)(b + 1) * nchunks] : n;
    counts[b] = e - a;
}

// cnt_row[r] = cntp[inv[r]]: each probe row's count back in row order. The reads are
// G interleaved forward streams (a bucket's rows keep their order), not random.
__global__ __launch_bounds__(kTPB) void k_pj_row_counts(const uint32_t* __restrict__ cntp,
                                                        const uint32_t* __restrict__ inv, uint64_t n,
                                                        uint32_t* __restrict__ cnt_row) {
    const uint64_t stride = (uint64_t)gridDim.x * kTPB;
    for (uint64_t r = (uint64_t)blockIdx.x * kTPB + threadIdx.x; r < n; r += stride) cnt_row[r] = cntp[inv[r]];
}

// Row r's pairs: cnt_row[r] build positions from the partitioned stream at poff[inv[r]],
// to the output at roff[r], each with out2 = p2[r]. A run past kLongRun rows is listed
// (row << 32 | chunk) for k_pj_place_long, one block per 64K-pair chunk.
__global__ __launch_bounds__(kTPB) void k_pj_place(const uint32_t* __restrict__ cnt_row,
                                                   const uint32_t* __restrict__ inv, const u64* __restrict__ poff,
                                                   const u64* __restrict__ roff, const int* __restrict__ out1p,
                                                   const int* __restrict__ p2, uint64_t n, int* __restrict__ out1,
                                                   int* __restrict__ out2, u64* __restrict__ longq,
                                                   uint32_t* __restrict__ nlong) {
    const uint64_t stride = (uint64_t)gridDim.x * kTPB;
    for (uint64_t r = (uint64_t)blockIdx.x * kTPB + threadIdx.x; r < n; r += stride) {
        const uint32_t L = cnt_row[r];
        if (!L) continue;
        if (L > kLongRun) {
            const uint32_t nch = (L + kLongChunk - 1) / kLongChunk;
            const uint32_t at = atomicAdd(nlong, nch);
            for (uint32_t c = 0; c < nch; c++) longq[at + c] = (r << 32) | c;
            continue;
        }
        const u64 src = poff[inv[r]], dst = roff[r];
        const int pp = p2[r];
        for (uint32_t t = 0; t < L; t++) {
            out1[dst + t] = out1p[src + t];
            out2[dst + t] = pp;
        }
    }
}

__global__ __launch_bounds__(kTPB) void k_pj_place_long(const uint32_t* __restrict__ cnt_row,
                                                        const uint32_t* __restrict__ inv,
                                                        const u64* __restrict__ poff, const u64* __restrict__ roff,
                                                        const int* __restrict__ out1p, const int* __restrict__ p2,
                                                        const u64* __restrict__ longq,
                                                        const uint32_t* __restrict__ nlong, int* __restrict__ out1,
                                                        int* __restrict__ out2) {
    const uint32_t nq = *nlong;
    for (uint32_t e = blockIdx.x; e < nq; e += gridDim.x) {
        const u64 q = longq[e];
        const uint64_t r = q >> 32;
        const uint32_t c = (uint32_t)q;
        const uint32_t L = cnt_row[r];
        const uint32_t a = c * kLongChunk, b = L - a < kLongChunk ? L : a + kLongChunk;
        const u64 src = poff[inv[r]], dst = roff[r];
        const int pp = p2[r];
        for (uint32_t t = a + threadIdx.x; t < b; t += kTPB) {
            out1[dst + t] = out1p[src + t];
            out2[dst + t] = pp;
        }
    }
}

}  // namespace

extern "C" {

uint32_t mq_pjoin_bucket(int32_t key, int G) { return G > 0 ? pj_part((uint32_t)key, (uint32_t)G) : 0u; }

int mq_pjoin_partition(const int32_t* d_keys, const int32_t* d_pay, uint64_t n, int G, int32_t* d_keys_out,
                       int32_t* d_pay_out, uint32_t* d_inv, uint64_t* h_counts, void* stream) {
    DevState* s;
    int rc = ensure_ready(&s);
    if (rc) return rc;
    if (G < 1 || G > 64 || !h_counts) return set_err(MQ_EINVAL, "mq_pjoin_partition: G = %d", G);
    if (n >= (1ull << 32)) return set_err(MQ_EINVAL, "mq_pjoin_partition: %llu rows", (unsigned long long)n);
    if (n && (!d_keys || !d_keys_out || (d_pay_out && !d_pay)))
        return set_err(MQ_EINVAL, "mq_pjoin_partition: NULL pointer");
    for (int b = 0; b < G; b++) h_counts[b] = 0;
    if (n == 0) return MQ_OK;
    hipStream_t st = (hipStream_t)stream;
    const uint64_t nchunks = (n + kChunk - 1) / kChunk;
    const uint64_t nh = nchunks * (uint64_t)G;
    uint32_t* hist = (uint32_t*)pool_alloc(nh * 4);
    u64* base = (u64*)pool_alloc(nh * 8 + 64 * 8);
    u64* scratch = (u64*)pool_alloc(scan_u32_scratch_elems(nh) * 8);
    auto done = [&](int r) {  // stream-ordered: queued kernels may still use them on an error path
        pool_free_on(hist, st);
        pool_free_on(base, st);
        pool_free_on(scratch, st);
        return r;
    };
    if (!hist || !base || !scratch) return done(set_err(MQ_ENOMEM, "mq_pjoin_partition: %llu rows", (unsigned long long)n));
    u64* counts = base + nh;
    const dim3 grid((uint32_t)((nchunks + kWaves - 1) / kWaves));
    hipLaunchKernelGGL(k_pj_hist, grid, dim3(kTPB), 0, st, d_keys, n, (uint32_t)G, nchunks, hist);
    if (hipGetLastError() != hipSuccess) return done(set_err(MQ_EHIP, "k_pj_hist launch"));
    if ((rc = scan_u32_exclusive(hist, base, nh, scratch, st))) return done(rc);
    hipLaunchKernelGGL(k_pj_scatter, grid, dim3(kTPB), 0, st, d_keys, d_pay_out ? d_pay : nullptr, n, (uint32_t)G,
                       nchunks, (const u64*)base, d_keys_out, d_pay_out, d_inv);
    hipLaunchKernelGGL(k_pj_counts, dim3(1), dim3(64), 0, st, (const u64*)base, nchunks, (uint32_t)G, n, counts);
    if (hipGetLastError() != hipSuccess) return done(set_err(MQ_EHIP, "k_pj_scatter launch"));
    if (hipMemcpyAsync(h_counts, counts, (size_t)G * 8, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
        return done(set_err(MQ_EHIP, "mq_pjoin_partition: counts"));
    return done(MQ_OK);
}

int mq_pjoin_place(const uint32_t* d_cntp, const int32_t* d_out1p, const uint32_t* d_inv, const int32_t* d_p2,
                   uint64_t n, uint64_t m, int32_t* d_out1, int32_t* d_out2, void* stream) {
    DevState* s;
    int rc = ensure_ready(&s);
    if (rc) return rc;
    if (n == 0 || m == 0) return MQ_OK;
    if (!d_cntp || !d_out1p || !d_inv || !d_p2 || !d_out1 || !d_out2)
        return set_err(MQ_EINVAL, "mq_pjoin_place: NULL pointer");
    if (n >= (1ull << 32)) return set_err(MQ_EINVAL, "mq_pjoin_place: %llu rows", (unsigned long long)n);
    const uint64_t qcap = m / kLongRun + m / kLongChunk + 2;
    if (qcap > 0xFFFFFFF0ull) return set_err(MQ_EINVAL, "mq_pjoin_place: %llu pairs", (unsigned long long)m);
    hipStream_t st = (hipStream_t)stream;
    uint32_t* cnt_row = (uint32_t*)pool_alloc(n * 4);
    u64* poff = (u64*)pool_alloc(n * 8);
    u64* roff = (u64*)pool_alloc(n * 8);
    u64* scratch = (u64*)pool_alloc(scan_u32_scratch_elems(n) * 8);
    u64* longq = (u64*)pool_alloc(qcap * 8 + 16);
    auto done = [&](int r) {  // the temporaries go back to the pool in stream order (no host wait)
        pool_free_on(cnt_row, st);
        pool_free_on(poff, st);
        pool_free_on(roff, st);
        pool_free_on(scratch, st);
        pool_free_on(longq, st);
        return r;
    };
    if (!cnt_row || !poff || !roff || !scratch || !longq)
        return done(set_err(MQ_ENOMEM, "mq_pjoin_place: %llu rows", (unsigned long long)n));
    uint32_t* nlong = reinterpret_cast<uint32_t*>(longq + qcap);
    if ((rc = scan_u32_exclusive(d_cntp, poff, n, scratch, st))) return done(rc);
    hipLaunchKernelGGL(k_pj_row_counts, dim3(stream_grid(s, n)), dim3(kTPB), 0, st, d_cntp, d_inv, n, cnt_row);
    if (hipGetLastError() != hipSuccess) return done(set_err(MQ_EHIP, "k_pj_row_counts launch"));
    if ((rc = scan_u32_exclusive(cnt_row, roff, n, scratch, st))) return done(rc);
    if (hipMemsetAsync(nlong, 0, 4, st) != hipSuccess) return done(set_err(MQ_EHIP, "mq_pjoin_place: memset"));
    hipLaunchKernelGGL(k_pj_place, dim3(stream_grid(s, n)), dim3(kTPB), 0, st, cnt_row, d_inv, poff, roff, d_out1p,
                       d_p2, n, d_out1, d_out2, longq, nlong);
    hipLaunchKernelGGL(k_pj_place_long, dim3(s->cus * 8), dim3(kTPB), 0, st, cnt_row, d_inv, poff, roff, d_out1p,
                       d_p2, longq, nlong, d_out1, d_out2);
    if (hipGetLastError() != hipSuccess) return done(set_err(MQ_EHIP, "k_pj_place launch"));
    return done(MQ_OK);
}

int mq_memcpy_peer(void* dst, int dst_dev, const void* src, int src_dev, size_t bytes, void* stream) {
    if (bytes == 0) return MQ_OK;
    if (!dst || !src) return set_err(MQ_EINVAL, "mq_memcpy_peer: NULL pointer");
    if (dst_dev == src_dev)
        HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream));
    else
        HIPCHK(hipMemcpyPeerAsync(dst, dst_dev, src, src_dev, bytes, (hipStream_t)stream));
    return MQ_OK;
}

int mq_enable_peer(int peer) {
    int cur = 0;
    HIPCHK(hipGetDevice(&cur));
    if (peer == cur) return MQ_OK;
    int can = 0;
    HIPCHK(hipDeviceCanAccessPeer(&can, cur, peer));
    if (!can) return MQ_OK;  // peer copies still work, staged by the runtime
    const hipError_t e = hipDeviceEnablePeerAccess(peer, 0);
    if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled)
        return set_err(MQ_EHIP, "hipDeviceEnablePeerAccess(%d): %s", peer, hipGetErrorString(e));
    (void)hipGetLastError();
    return MQ_OK;
}

}  // extern "C"
