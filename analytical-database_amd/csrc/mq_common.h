// mq_common.h — internal (not exported) runtime shared by libmq's HIP sources.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "mq_device.h"

namespace mqi {

constexpr int kMaxDev = 64;

struct DevState {
    bool ready;
    int cus;                 // compute units (256 on MI355X)
    hipStream_t stream;      // library stream (mq_default_stream)
};

// Records a message for mq_last_error() and returns code.
int set_err(int code, const char* fmt, ...);
int current_device(int* dev);
// Device checks (gfx950) and per-device constants, once per device.
int ensure_ready(DevState** out);
// Grid for a grid-stride streaming kernel of 256-thread blocks.
uint32_t stream_grid(const DevState* s, uint64_t work_items);
// The same, capped at the blocks of fn that are resident at once (a grid-stride
// kernel whose registers allow fewer than 8 blocks per CU would otherwise run a
// second, partial round of blocks).
uint32_t resident_grid(const DevState* s, uint64_t work_items, const void* fn);
// Device exclusive scan u32[n] -> u64[n] (mq_join.hip); scratch holds
// scan_u32_scratch_elems(n) u64.
uint64_t scan_u32_scratch_elems(uint64_t n);
int scan_u32_exclusive(const uint32_t* in, unsigned long long* out, uint64_t n,
                       unsigned long long* scratch, hipStream_t st);
// The same with u32 sums (n < 2^32 and a total below 2^32; in and out may alias).
int scan_u32_exclusive_u32(const uint32_t* in, uint32_t* out, uint64_t n, unsigned long long* scratch,
                           hipStream_t st);
// The same over u64 elements (in and out may alias); scratch as above.
int scan_u64_exclusive(const unsigned long long* in, unsigned long long* out, uint64_t n,
                       unsigned long long* scratch, hipStream_t st);

// Stable LSD radix sort (4 x 8-bit digits) of (int32 key, u32 value) pairs by key
// (mq_join.hip). vals == nullptr sorts (key, row id). *keys_out receives the keys
// as (uint32)key ^ 0x80000000 (ascending as unsigned), *vals_out the values; both
// are pool_alloc'd (the caller pool_frees them). Synchronises the stream.
int radix_sort_pairs(const int* keys, const int* vals, uint64_t n, uint32_t** keys_out,
                     uint32_t** vals_out, hipStream_t st, const DevState* s);
// The same sort of (col[i], i) written straight out as an index: values ascending
// (int32, may be NULL) and positions (size_t rows, may be NULL), equal values in
// ascending row order. Synchronises. Picks the form by the key range (mq_isort.hip).
int radix_sort_index(const int* col, uint64_t n, int32_t* values, uint64_t* positions, hipStream_t st);
// Its LSD form (mq_join.hip): npass 8-bit digits of (col ^ 2^31) - kmin.
int radix_sort_lsd_index(const int* col, uint64_t n, uint32_t kmin, int npass, int32_t* values, uint64_t* positions,
                         hipStream_t st);

// Frees the calling thread's pinned upload staging of shared_select (mq_shared.hip).
void shared_staging_release();

// The reference's exact quicksort order (index.c:25-46) of col[0..n), n < 2^31, into
// vout (values) and pout (size_t positions), either may be NULL (mq_lomuto.hip).
int lomuto_sort(const int32_t* col, uint64_t n, int32_t* vout, uint64_t* pout, hipStream_t st, const DevState* s);
// Caching device allocator for per-call scratch (join tables and partitions,
// probe arrays): grow-only, blocks are reused for requests of 1/2..1x their size,
// idle blocks are released by mq_trim(). A freed block may be handed out again at
// once, so callers free only what no queued kernel still uses (sync first);
// pool_free_on(p, st) is the stream-ordered free: an event recorded on st marks
// when the block may be reused: pool_alloc hands it out only once that has passed,
// takes a fresh block while it is pending, and waits for it only when no fresh block
// fits in HBM. Call it with the block's device current.
void* pool_alloc(size_t bytes);
void pool_free(void* p);
void pool_free_on(void* p, hipStream_t st);

// Lanes of the wave (within `among`) whose 8-bit value d equals this lane's: a
// match-any from 8 ballots. Per bit: one v_bfe_i32 (the bit as 0 / all-ones), one
// ballot, and per half one v_bitop3 accumulating acc | (bit ^ ballot), the lanes that
// differ from this lane in some bit: 4 VALU a bit (the or-of-xor the compiler formed
// took 5; `peers &= bit ? m : ~m` took 9). v_bitop3's table is indexed by
// (src0, src1, src2) bits as 4 s0 + 2 s1 + s2: a | (b ^ c) = 0xF0 | (0xCC ^ 0xAA) = 0xF6.
__device__ __forceinline__ unsigned long long match_any8(uint32_t d, unsigned long long among) {
    uint32_t sb[8];
#pragma unroll
    for (int b = 0; b < 8; b++) sb[b] = (uint32_t)(((int32_t)(d << (31 - b))) >> 31);  // bit b as 0 / ~0
    // opaque (else each ballot is rebuilt from a second shift), all eight at once so
    // the ballots and their uses interleave (a VALU-written SGPR needs wait states)
    asm("" : "+v"(sb[0]), "+v"(sb[1]), "+v"(sb[2]), "+v"(sb[3]), "+v"(sb[4]), "+v"(sb[5]), "+v"(sb[6]), "+v"(sb[7]));
    unsigned long long m[8];
#pragma unroll
    for (int b = 0; b < 8; b++) m[b] = __ballot(sb[b] != 0);
    uint32_t dlo = 0, dhi = 0;
#pragma unroll
    for (int b = 0; b < 8; b++) {
        dlo = __builtin_amdgcn_bitop3_b32(dlo, sb[b], (uint32_t)m[b], 0xF6);
        dhi = __builtin_amdgcn_bitop3_b32(dhi, sb[b], (uint32_t)(m[b] >> 32), 0xF6);
    }
    return among & ~(((unsigned long long)dhi << 32) | dlo);
}

// Lanes below this one in mask m (v_mbcnt: 2 VALU, against and + popcount of both halves).
__device__ __forceinline__ uint32_t lanes_below(unsigned long long m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// XCD-aware tile of block b in a grid of g blocks (cdna_hip_programming.md T1):
// blocks are dealt round-robin over the 8 XCDs, so block b runs on XCD b % 8;
// this bijection gives each XCD a contiguous range of tiles instead. Tiles whose
// outputs share cache lines (adjacent digit runs of a radix scatter) then meet in
// one L2 and leave it as whole lines. Speed only: any bijection is correct.
__device__ __forceinline__ uint32_t xcd_tile(uint32_t b, uint32_t g) {
    const uint32_t q = g >> 3, r = g & 7u, x = b & 7u;
    return x * q + (x < r ? x : r) + (b >> 3);
}

}  // namespace mqi

#define HIPCHK(expr)                                                                         \
    do {                                                                                     \
        hipError_t e_ = (expr);                                                              \
        if (e_ != hipSuccess)                                                                \
            return mqi::set_err(MQ_EHIP, "%s failed: %s", #expr, hipGetErrorString(e_));     \
    } while (0)

#define LAUNCHCHK(what)                                                                      \
    do {                                                                                     \
        hipError_t e_ = hipGetLastError();                                                   \
        if (e_ != hipSuccess)                                                                \
            return mqi::set_err(MQ_EHIP, "launch of %s failed: %s", what,                    \
                                hipGetErrorString(e_));                                      \
    } while (0)
