// mq_csv.hip — the load path on gfx950: CSV text in HBM -> int32 columns.
//
// Restates the data loop of load_db (src/db_manager.c:304-318) with insert_row
// (:164-199), the step that feeds every column the select/fetch/aggregate path reads:
//   * a row is one fgets(line, MAX_LINE_SIZE = 1024) piece (db_manager.c:23,306):
//     the bytes through the next '\n', at most 1023 of them, or up to EOF;
//   * the piece is split by strsep(",") and the first ncols tokens go through atoi
//     (= (int)strtol(tok, NULL, 10): leading isspace, sign, digits, saturation at
//     LONG_MIN/LONG_MAX, then the low 32 bits);
//   * tokens past ncols are ignored; a token missing from a piece keeps the
//     previous row's value (row[] is reused across lines; before the first line the
//     reference reads an uninitialised VLA, here 0); a NUL byte ends the string
//     strsep sees;
//   * min/max per column fold over the rows as insert_row does (:193-194).
//
// Layout: the text is cut into 16 KB chunks, one block each.
//   k_csv_count : every thread owns 64 bytes; a row starts at p when p == 0 or
//                 text[p-1] == '\n' (plus, inside lines longer than 1023 bytes,
//                 every 1023 bytes: "long mode"). Counts per chunk; in the first
//                 pass also the first/last start per chunk and a long-line flag.
//   scan        : chunk counts -> first row of each chunk (the shared u32 scan).
//   k_csv_parse : the chunk plus a 1 KB halo (a piece is <= 1023 bytes) is staged
//                 in LDS; the starts are enumerated again into an LDS list and each
//                 thread parses whole pieces from LDS, writing column j of row r to
//                 cols[j][r] (consecutive lanes -> consecutive rows, coalesced).
//                 min/max per column: lane registers (first 8 columns) or LDS
//                 atomics, one partial per block, folded by k_csv_minmax.
//   missing-token fix-up (only when a piece had fewer than ncols tokens): tokens
//                 per row, then per column a max-scan of "last row that had the
//                 token" over 1024-row tiles, and the copy.
// HBM traffic: 2 reads of the text (count + parse, +6 % halo) + 4 B per cell.

#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <vector>

#include "mq_common.h"
#include "mq_device.h"

namespace {

using namespace mqi;

constexpr int kTPB = 256;
constexpr int kWaves = kTPB / 64;
constexpr int kChunk = 16384;            // text bytes per block (12 KB chunks measured 5 % slower)
constexpr int kSeg = kChunk / kTPB;      // 64 bytes per thread
static_assert(kSeg % 16 == 0 && kSeg <= 64 && kChunk % 4096 == 0, "segments of 16-byte pieces");
constexpr int kPre = 16;                 // LDS bytes before the chunk (byte cs-1 at kPre-1)
constexpr int kHalo = 1024;              // after the chunk: a piece has <= 1023 bytes
constexpr int kLds = kPre + kChunk + kHalo;
constexpr int kPiece = 1023;             // fgets(line, 1024)
constexpr int kList = 4096;              // piece / token starts listed in LDS
constexpr int kRegCols = 8;              // columns whose min/max live in lane registers
constexpr int kMaxCols = 1024;
constexpr int kFillTile = 1024;          // rows per tile in the missing-token fix-up

enum { F_LONG = 0, F_MISSING = 1, F_MAYBE_LONG = 2 };

typedef unsigned v4u __attribute__((ext_vector_type(4)));

struct CsvWs {  // carved from the caller's workspace (mq_csv_workspace_bytes)
    unsigned* flags;
    uint32_t* cnt;
    long long* first;
    long long* last;
    long long* prev;
    unsigned long long* row_base;
    unsigned long long* scratch;
    int32_t** colptr;
    int2* partial;
};

size_t align16(size_t x) { return (x + 15) & ~(size_t)15; }
bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

uint64_t nchunks_of(uint64_t n) { return (n + kChunk - 1) / kChunk; }

size_t carve(void* ws, uint64_t n, int ncols, CsvWs* w) {
    const uint64_t c = nchunks_of(n) + 1;
    size_t o = 0;
    char* b = static_cast<char*>(ws);
    auto take = [&](size_t bytes) {
        char* p = b ? b + o : nullptr;
        o += align16(bytes);
        return p;
    };
    CsvWs t;
    t.flags = reinterpret_cast<unsigned*>(take(64));
    t.cnt = reinterpret_cast<uint32_t*>(take(c * 4));
    t.first = reinterpret_cast<long long*>(take(c * 8));
    t.last = reinterpret_cast<long long*>(take(c * 8));
    t.prev = reinterpret_cast<long long*>(take(c * 8));
    t.row_base = reinterpret_cast<unsigned long long*>(take(c * 8));
    t.scratch = reinterpret_cast<unsigned long long*>(take(scan_u32_scratch_elems(c) * 8));
    t.colptr = reinterpret_cast<int32_t**>(take((size_t)kMaxCols * 8));
    t.partial = reinterpret_cast<int2*>(take(c * (size_t)(ncols > 0 ? ncols : 1) * 8));
    if (w) *w = t;
    return o;
}

// A column pointer read from the workspace is a generic (flat) pointer to the
// compiler; its stores would be flat_store, which count in lgkmcnt, so every later
// LDS read of the parse waited for them to reach memory. The columns are global.
typedef int32_t __attribute__((address_space(1))) gint32;
__device__ __forceinline__ gint32* global_ptr(int32_t* p) { return (gint32*)p; }

// ---- staging: text[cs - kPre, cs + kChunk + kHalo) -> s (0 outside [0, n), except
// that the byte before position 0 reads as '\n': position 0 starts a row). Every
// lane issues all of its 16-byte loads before it stores any (a load/store loop
// left one HBM round trip per piece on the block's critical path).
constexpr int kPieces = kLds / 16;                  // 16-byte pieces staged per chunk
constexpr int kPf = (kPieces + kTPB - 1) / kTPB;    // ... per lane
static_assert(kLds % 16 == 0, "staging is in 16-byte pieces");

// Whole 16-byte pieces inside the text are loaded (nt, dwordx4) into registers;
// the others (before position 0, across or past EOF, or all of them when the text
// is not 16-byte aligned) are filled byte by byte straight into LDS at store time.
template <bool VEC>
__device__ __forceinline__ bool piece_vec(uint64_t n, long long g) {
    return VEC && g >= 0 && (uint64_t)g + 16 <= n;
}

// text[cs - kPre, cs + kChunk + kHalo) -> registers (stage_chunk's bytes)
template <bool VEC>
__device__ __forceinline__ void prefetch_chunk(const char* __restrict__ text, uint64_t n, uint64_t cs,
                                               uint4 (&pf)[kPf]) {
    const long long base = (long long)cs - kPre;
#pragma unroll
    for (int q = 0; q < kPf; q++) {
        const int i = threadIdx.x + q * kTPB;
        const long long g = base + (long long)i * 16;
        if (i < kPieces && piece_vec<VEC>(n, g)) {
            const v4u t = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(text + g));
            pf[q] = make_uint4(t.x, t.y, t.z, t.w);
        }
    }
}

// registers -> LDS; the byte before position 0 reads as '\n', bytes past EOF as 0
template <bool VEC>
__device__ __forceinline__ void store_chunk(const char* __restrict__ text, uint64_t n, uint64_t cs,
                                            const uint4 (&pf)[kPf], uint8_t* s) {
    const long long base = (long long)cs - kPre;
#pragma unroll
    for (int q = 0; q < kPf; q++) {
        const int i = threadIdx.x + q * kTPB;
        if (i >= kPieces) continue;
        const long long g = base + (long long)i * 16;
        if (piece_vec<VEC>(n, g)) {
            *reinterpret_cast<uint4*>(s + i * 16) = pf[q];
        } else {
            for (int k = 0; k < 16; k++) {
                const long long x = g + k;
                s[i * 16 + k] = x == -1 ? (uint8_t)'\n' : (x >= 0 && (uint64_t)x < n) ? (uint8_t)text[x] : 0;
            }
        }
    }
}

#ifndef MQ_CSV_STAGE_FAST
#define MQ_CSV_STAGE_FAST 1
#endif
template <bool VEC>
__device__ __forceinline__ void stage_chunk(const char* __restrict__ text, uint64_t n, uint64_t cs,
                                            uint8_t* s) {
    if (MQ_CSV_STAGE_FAST && VEC && cs >= (uint64_t)kPre && cs - kPre + kLds <= n) {
        // an interior chunk (all but the first and the last ones): every piece is a
        // whole 16-byte load, no per-piece bounds tests (~40 VALU and 5 branches a lane)
        const v4u* src = reinterpret_cast<const v4u*>(text + (cs - kPre));
        v4u pv[kPf];
#pragma unroll
        for (int q = 0; q < kPf; q++) {
            const int i = threadIdx.x + q * kTPB;
            if (q < kPf - 1 || i < kPieces) pv[q] = __builtin_nontemporal_load(src + i);
        }
#pragma unroll
        for (int q = 0; q < kPf; q++) {
            const int i = threadIdx.x + q * kTPB;
            if (q < kPf - 1 || i < kPieces) *reinterpret_cast<v4u*>(s + i * 16) = pv[q];
        }
        return;
    }
    uint4 pf[kPf];
    prefetch_chunk<VEC>(text, n, cs, pf);
    store_chunk<VEC>(text, n, cs, pf, s);
}

// bit k set <=> byte k of the 4 is '\n' (exact SWAR zero-byte test)
__device__ __forceinline__ uint32_t nl4(uint32_t w) {
    const uint32_t x = w ^ 0x0A0A0A0Au;
    const uint32_t z = ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u;
    return ((z >> 7) | (z >> 14) | (z >> 21) | (z >> 28)) & 0xFu;
}

// Real starts of this thread's segment [a, a+kSeg): bit k <=> a+k starts a
// line (byte a+k-1 is '\n'); bytes at or past ce are masked off.
__device__ __forceinline__ unsigned long long real_starts(const uint8_t* s, uint64_t cs, uint64_t ce,
                                                          int tid) {
    const int off = kPre + tid * kSeg;  // LDS index of byte a
    unsigned long long nl = 0;
#pragma unroll
    for (int q = 0; q < kSeg / 16; q++) {
        const uint4 v = *reinterpret_cast<const uint4*>(s + off + q * 16);
        nl |= (unsigned long long)(nl4(v.x) | (nl4(v.y) << 4) | (nl4(v.z) << 8) | (nl4(v.w) << 12))
              << (q * 16);
    }
    unsigned long long st = (nl << 1) | (s[off - 1] == '\n' ? 1ull : 0ull);
    if (kSeg < 64) st &= (1ull << (kSeg & 63)) - 1;  // (bit kSeg is the next segment's)
    const uint64_t a = cs + (uint64_t)tid * kSeg;
    if (a >= ce) return 0;
    if (ce - a < (uint64_t)kSeg) st &= (1ull << (ce - a)) - 1;
    return st;
}

__device__ __forceinline__ int wave_min_i(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ int wave_max_i(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
    return v;
}

template <typename T>
__device__ __forceinline__ T wave_incl_max(T v, int lane) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const T u = __shfl_up(v, o, 64);
        if (lane >= o) v = v > u ? v : u;
    }
    return v;
}
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
// Inclusive sum over the wave by DPP (row shifts within 16 lanes, then the row
// broadcasts of lanes 15 and 31): 6 adds instead of 6 ds_bpermute round trips.
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t v, int) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);  // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);  // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);  // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);  // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);  // row_bcast:15
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);  // row_bcast:31
    return v;
}

// Exclusive max over the block's threads (in order), seeded with `seed`.
__device__ __forceinline__ long long block_excl_max(long long x, long long seed, long long* s_w) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const long long inc = wave_incl_max(x, lane);
    if (lane == 63) s_w[wave] = inc;
    __syncthreads();
    long long carry = seed;
    for (int w = 0; w < wave; w++) carry = carry > s_w[w] ? carry : s_w[w];
    long long ex = __shfl_up(inc, 1, 64);
    if (lane == 0) ex = LLONG_MIN;
    __syncthreads();
    return carry > ex ? carry : ex;
}

// Exclusive sum over the block's threads; *total receives the block sum. TRAIL = false
// drops the closing barrier (s_w is not written again before the caller's next one).
template <bool TRAIL = true>
__device__ __forceinline__ uint32_t block_excl_sum(uint32_t x, uint32_t* s_w, uint32_t* total) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t inc = wave_incl_sum(x, lane);
    if (lane == 63) s_w[wave] = inc;
    __syncthreads();
    uint32_t carry = 0, tot = 0;
    for (int w = 0; w < kWaves; w++) {
        if (w < wave) carry += s_w[w];
        tot += s_w[w];
    }
    if (TRAIL) __syncthreads();
    *total = tot;
    return carry + inc - x;
}

// Row starts of the segment, in long mode: the real starts plus, inside a line that
// is longer than 1023 bytes, every 1023rd byte after its start (fgets pieces).
// ls_in = last real start before the segment (global). Between two real starts of
// one segment there is no room for 1023 bytes, so only the part before
// the first real start can hold a piece start.
__device__ __forceinline__ unsigned long long piece_starts(unsigned long long real, uint64_t a,
                                                           long long ls_in, uint64_t ce) {
    if (ls_in < 0 || a >= ce) return real;
    const uint64_t q = (a - (uint64_t)ls_in) % kPiece;
    const uint64_t p = q == 0 ? 0 : kPiece - q;  // first piece boundary at or after a
    const int rf = real ? __builtin_ctzll(real) : kSeg;
    if (p < (uint64_t)rf && a + p < ce) real |= 1ull << p;
    return real;
}

// ---- pass 1: row starts per chunk ----
//   LONG = false: real starts; also first/last start (global) per chunk and the
//                 long-line flag for gaps inside the chunk.
//   LONG = true : piece starts, given prev[c] = last real start before the chunk.
template <bool VEC, bool LONG>
__global__ __launch_bounds__(kTPB) void k_csv_count(const char* __restrict__ text, uint64_t n,
                                                     uint32_t* __restrict__ cnt, long long* __restrict__ first,
                                                     long long* __restrict__ last,
                                                     const long long* __restrict__ prev, unsigned* flags) {
    __shared__ __attribute__((aligned(16))) uint8_t s[kLds];
    __shared__ long long s_w[kWaves];
    __shared__ uint32_t s_u[kWaves];
    const uint64_t c = blockIdx.x, cs = c * kChunk;
    const uint64_t ce = cs + kChunk < n ? cs + kChunk : n;
    const int tid = threadIdx.x;
    stage_chunk<VEC>(text, n, cs, s);
    __syncthreads();
    unsigned long long st = real_starts(s, cs, ce, tid);
    const uint64_t a = cs + (uint64_t)tid * kSeg;
    const long long mylast = st ? (long long)(a + 63 - __builtin_clzll(st)) : -1;
    if (LONG) {
        const long long ls = block_excl_max(mylast, prev[c], s_w);
        st = piece_starts(st, a, ls, ce);
    } else {
        const long long ls = block_excl_max(mylast, -1, s_w);
        if (st && ls >= 0) {
            const long long f = (long long)(a + __builtin_ctzll(st));
            if (f - ls > kPiece) atomicOr(&flags[F_LONG], 1u);
        }
    }
    uint32_t tot;
    block_excl_sum((uint32_t)__popcll(st), s_u, &tot);
    if (!LONG) {  // first / last start of the chunk
        const long long myfirst = st ? (long long)(a + __builtin_ctzll(st)) : LLONG_MAX;
        long long f = myfirst;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const long long u = __shfl_xor(f, o, 64);
            f = f < u ? f : u;
        }
        long long l = mylast;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const long long u = __shfl_xor(l, o, 64);
            l = l > u ? l : u;
        }
        __syncthreads();
        if ((tid & 63) == 0) s_w[tid >> 6] = f;
        __syncthreads();
        if (tid == 0) {
            long long m = s_w[0];
            for (int w = 1; w < kWaves; w++) m = m < s_w[w] ? m : s_w[w];
            first[c] = m == LLONG_MAX ? -1 : m;
        }
        __syncthreads();
        if ((tid & 63) == 0) s_w[tid >> 6] = l;
        __syncthreads();
        if (tid == 0) {
            long long m = s_w[0];
            for (int w = 1; w < kWaves; w++) m = m > s_w[w] ? m : s_w[w];
            last[c] = m;
        }
    }
    if (tid == 0) cnt[c] = tot;
}

// ---- pass 1, streaming form (the default): row starts per chunk straight from
// the loaded registers, no LDS. Starts in [cs, ce) are the '\n' bytes in
// [cs-1, ce-1) (+ position 0). A line over 1023 bytes contains a whole aligned
// 512-byte block without '\n', so "some such block has no '\n'" flags a possible
// long line (never misses one); only then does the exact k_csv_count<., false>
// run (and long mode if it confirms).
template <bool VEC>
__global__ __launch_bounds__(kTPB) void k_csv_count_stream(const char* __restrict__ text, uint64_t n,
                                                            uint32_t* __restrict__ cnt, unsigned* flags) {
    __shared__ uint32_t s_c[kWaves];
    const uint64_t c = blockIdx.x, cs = c * kChunk;
    const uint64_t ce = cs + kChunk < n ? cs + kChunk : n;
    const int tid = threadIdx.x, lane = tid & 63;
    constexpr int kQ = kChunk / 4096;
    uint32_t w[kQ][4];
#pragma unroll
    for (int q = 0; q < kQ; q++) {  // kQ x 16 B per lane, 4 KB apart: coalesced
        const uint64_t g = cs + (uint64_t)q * 4096 + (uint64_t)tid * 16;
        if (VEC && g + 16 <= ce) {
            const v4u t = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(text + g));
            w[q][0] = t.x, w[q][1] = t.y, w[q][2] = t.z, w[q][3] = t.w;
        } else {
            uint8_t t[16];
#pragma unroll
            for (int k = 0; k < 16; k++) t[k] = g + k < ce ? (uint8_t)text[g + k] : 0;
            memcpy(w[q], t, 16);
        }
    }
    uint32_t cntl = 0;
    bool nolf_block = false;
#pragma unroll
    for (int q = 0; q < kQ; q++) {
        const uint32_t m = nl4(w[q][0]) | (nl4(w[q][1]) << 4) | (nl4(w[q][2]) << 8) | (nl4(w[q][3]) << 12);
        cntl += __popc(m);
        // 32 lanes x 16 B = one aligned 512-byte block; count only blocks wholly in the text
        const unsigned long long b = __ballot(m != 0);
        const uint64_t g = cs + (uint64_t)q * 4096 + (uint64_t)(tid & ~31) * 16;
        const uint32_t half = (uint32_t)(b >> (lane & 32));
        if (g + 512 <= n && half == 0) nolf_block = true;
    }
    cntl = (uint32_t)wave_sum_u32(cntl);
    if (lane == 0) s_c[tid >> 6] = cntl;
    if (__ballot(nolf_block) && lane == 0) atomicOr(&flags[F_MAYBE_LONG], 1u);
    __syncthreads();
    if (tid == 0) {
        uint32_t t = s_c[0] + s_c[1] + s_c[2] + s_c[3];
        // starts = '\n' in [cs-1, ce-1), plus position 0
        if (cs == 0) t += 1;
        else t += text[cs - 1] == '\n';
        t -= text[ce - 1] == '\n';
        cnt[c] = t;
    }
}

// Long lines across chunks: a full chunk without a start lies inside a line of
// more than 16 KB; otherwise compare each chunk's first start with the previous
// chunk's last, and the text end with the final start.
__global__ __launch_bounds__(kTPB) void k_csv_long_check(const uint32_t* __restrict__ cnt,
                                                          const long long* __restrict__ first,
                                                          const long long* __restrict__ last,
                                                          uint64_t nch, uint64_t n, unsigned* flags) {
    const uint64_t c = (uint64_t)blockIdx.x * kTPB + threadIdx.x;
    if (c >= nch) return;
    bool lng = false;
    if (cnt[c] == 0) {
        lng = c + 1 < nch;  // a full 16 KB chunk inside one line
    } else {
        if (c > 0 && cnt[c - 1] > 0 && first[c] - last[c - 1] > kPiece) lng = true;
        const bool final_start = c + 1 == nch || (c + 2 == nch && cnt[c + 1] == 0);
        if (final_start && (long long)n - last[c] > kPiece) lng = true;
    }
    if (lng) atomicOr(&flags[F_LONG], 1u);
}

// prev[c] = last real start before chunk c (-1 for none): one block, exclusive max
// over the chunks (long mode only).
__global__ __launch_bounds__(1024) void k_csv_prev_start(const long long* __restrict__ last,
                                                          uint64_t nch, long long* __restrict__ prev) {
    __shared__ long long s_w[16];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    long long carry = -1;
    for (uint64_t b = 0; b < nch; b += 1024) {
        const uint64_t c = b + tid;
        const long long x = c < nch ? last[c] : -1;
        const long long inc = wave_incl_max(x, lane);
        if (lane == 63) s_w[wave] = inc;
        __syncthreads();
        long long pre = carry, all = carry;
        for (int w = 0; w < 16; w++) {
            if (w < wave) pre = pre > s_w[w] ? pre : s_w[w];
            all = all > s_w[w] ? all : s_w[w];
        }
        long long ex = __shfl_up(inc, 1, 64);
        if (lane == 0) ex = LLONG_MIN;
        if (c < nch) prev[c] = pre > ex ? pre : ex;
        carry = all;
        __syncthreads();
    }
}

__device__ __forceinline__ bool is_space(uint32_t b) {  // isspace() in the C locale
    return b == ' ' || (b >= '\t' && b <= '\r');
}

// atoi of the token starting at LDS index k (its piece ends at index kend, the
// first '\n' included). Returns the value; *k is left on the byte that ended the
// token; *more is false when the piece ended (a '\n', a NUL, or kend), true when
// a ',' ended it.
__device__ __forceinline__ int32_t parse_token(const uint8_t* __restrict__ s, int& k, int kend,
                                               bool& more) {
    // leading isspace ('\n' included: it is the piece's last byte)
    uint32_t b = 0;
    while (k < kend) {
        b = s[k];
        if (!is_space(b) || b == '\n') break;
        k++;
    }
    bool neg = false;
    if (k < kend && (b == '+' || b == '-')) {
        neg = b == '-';
        k++;
    }
    unsigned long long acc = 0;
    int nd = 0;  // significant digits
    bool sat = false;
    while (k < kend) {
        b = s[k];
        const uint32_t d = b - '0';
        if (d > 9) break;
        if (acc != 0 || d != 0) {
            if (nd >= 19) sat = true;
            else acc = acc * 10 + d, nd++;
        }
        k++;
    }
    // rest of the token: up to ',', '\n', NUL or the piece end
    while (k < kend) {
        b = s[k];
        if (b == ',' || b == '\n' || b == 0) break;
        k++;
    }
    more = k < kend && b == ',';
    if (more) k++;
    if (!sat && nd == 19 && acc > (neg ? 0x8000000000000000ull : 0x7FFFFFFFFFFFFFFFull)) sat = true;
    if (sat) return neg ? 0 : -1;  // (int)LONG_MIN, (int)LONG_MAX
    return (int32_t)(uint32_t)(neg ? 0ull - acc : acc);
}

// Bytes of a word that are not ASCII digits: bit 7 of each such byte (exact, no
// carries across bytes).
__device__ __forceinline__ unsigned long long nondigit8(unsigned long long w) {
    const unsigned long long y = w ^ 0x3030303030303030ull;
    return (((y & 0x7F7F7F7F7F7F7F7Full) + 0x7676767676767676ull) | y) & 0x8080808080808080ull;
}

// The common token, from registers: [-]digits{0..10} ended by ',', '\n', NUL or the
// piece end. The 16 bytes at k come from 5 aligned LDS dwords + alignbyte; the
// non-digit flags of two 64-bit words locate the end (ctz), and the digits are
// converted SWAR-style (8 at once: x*10 + x>>8, then two 64-bit multiplies).
// Anything else (leading isspace, '+', junk after the digits, more than 10 digits)
// returns false and the caller runs parse_token, the byte-at-a-time restatement
// of strtol.
__device__ __forceinline__ bool token_fast(const uint8_t* __restrict__ s, int& k, int kend, bool& more,
                                           int32_t& out) {
    const uint32_t* d = reinterpret_cast<const uint32_t*>(s) + (k >> 2);
    const uint32_t d0 = d[0], d1 = d[1], d2 = d[2], d3 = d[3], d4 = d[4];
    const uint32_t r = (uint32_t)k & 3u;
    unsigned long long lo = (unsigned long long)__builtin_amdgcn_alignbyte(d1, d0, r) |
                            ((unsigned long long)__builtin_amdgcn_alignbyte(d2, d1, r) << 32);
    unsigned long long hi = (unsigned long long)__builtin_amdgcn_alignbyte(d3, d2, r) |
                            ((unsigned long long)__builtin_amdgcn_alignbyte(d4, d3, r) << 32);
    const int lim = kend - k;  // bytes left in the piece (>= 0)
    unsigned long long nlo = nondigit8(lo), nhi = nondigit8(hi);
    constexpr unsigned long long kHi = 0x8080808080808080ull;
    if (lim < 8) nlo |= kHi << (8 * lim), nhi = kHi;  // past the piece: terminators
    else if (lim < 16) nhi |= kHi << (8 * (lim - 8));
    const bool neg = lim > 0 && (lo & 0xFFu) == '-';
    if (neg) nlo &= ~0x80ull;
    const int e = nlo ? (__builtin_ctzll(nlo) >> 3) : nhi ? 8 + (__builtin_ctzll(nhi) >> 3) : 16;
    const int L = e - (neg ? 1 : 0);
    if (L > 10) return false;
    bool m = false;
    if (e < lim) {
        const uint32_t c = (uint32_t)((e < 8 ? lo >> (8 * e) : hi >> (8 * (e - 8))) & 0xFFu);
        if (c == ',') m = true;
        else if (c != '\n' && c != 0) return false;  // isspace / '+' / junk: the slow path
    }
    if (neg) lo = (lo >> 8) | (hi << 56), hi >>= 8;
    const int l8 = L < 8 ? L : 8;
    unsigned long long x = lo - 0x3030303030303030ull;
    x = l8 ? x << (8 * (8 - l8)) : 0ull;  // the first l8 digits, right-aligned
    x = x * 10 + (x >> 8);
    x = (((x & 0x000000FF000000FFull) * (100 + (1000000ull << 32))) +
         (((x >> 16) & 0x000000FF000000FFull) * (1 + (10000ull << 32)))) >> 32;
    unsigned long long v = x;
    if (L > 8) v = v * 10 + ((hi & 0xFFu) - '0');
    if (L > 9) v = v * 10 + (((hi >> 8) & 0xFFu) - '0');
    out = (int32_t)(uint32_t)(neg ? 0ull - v : v);
    more = m;
    k += e + (m ? 1 : 0);
    return true;
}

__device__ __forceinline__ int32_t next_token(const uint8_t* __restrict__ s, int& k, int kend,
                                              bool& more) {
    int32_t v;
    if (token_fast(s, k, kend, more, v)) return v;
    return parse_token(s, k, kend, more);
}

// Non-digit flags of a word: bit 7 of byte b set when byte b is not an ASCII digit.
// Exact up to and including the first flagged byte (a carry leaves a byte only when
// that byte is itself flagged, and only toward later bytes), which is all the
// token scan needs.
__device__ __forceinline__ uint32_t nondigit_first(uint32_t w) {
    const uint32_t y = w ^ 0x30303030u;
    return ((y + 0x76767676u) | y) & 0x80808080u;
}

// The value mod 2^32 of 12 ASCII digits (x0 byte 0 the most significant) whose
// first two are '0' (at most 10 significant digits): digit pairs by v_dot4 on
// byte ^ '0', then ((p1 * 10^4 + B) * 10^4 + C) in 24-bit multiplies (a chain of
// (a & 0xFFFFFF) * b + c compiled to quarter-rate 64-bit mads).
__device__ __forceinline__ uint32_t digits12_d(uint32_t d0, uint32_t d1, uint32_t d2) {
    // (each pair is <= 99 for digits, so no masking: the callers have checked them)
    const uint32_t p1 = __builtin_amdgcn_udot4(d0, 0x010A0000u, 0u, false);
    const uint32_t hb = __builtin_amdgcn_udot4(d1, 0x0000010Au, 0u, false);
    const uint32_t lb = __builtin_amdgcn_udot4(d1, 0x010A0000u, 0u, false);
    const uint32_t hc = __builtin_amdgcn_udot4(d2, 0x0000010Au, 0u, false);
    const uint32_t lc = __builtin_amdgcn_udot4(d2, 0x010A0000u, 0u, false);
    uint32_t hi = p1 * 10000u + hb * 100u + lb;  // < 2^24
    asm volatile("" : "+v"(hi));                 // (keeps the next product 24-bit)
    return (hi & 0xFFFFFFu) * 10000u + (hc * 100u + lc);
}
__device__ __forceinline__ uint32_t digits12(uint32_t x0, uint32_t x1, uint32_t x2) {
    return digits12_d(x0 ^ 0x30303030u, x1 ^ 0x30303030u, x2 ^ 0x30303030u);
}

// Index of the lowest set bit, or 0xFFFFFFFF for 0 (v_ffbl_b32 as it is).
__device__ __forceinline__ uint32_t ffbl(uint32_t x) { return (uint32_t)__builtin_ctzg(x, -1); }

// next_token for the usual case, where every piece ends with its '\n' or at EOF
// (no line over 1023 bytes: a token never runs past its piece, and past EOF the
// staged bytes are NUL). The fast rule is token_fast's: [-]digits{0..10} then ',',
// '\n' or NUL; anything else goes to parse_token (the strtol restatement). Written
// branch-free up to that one decision:
//   * 12 bytes at k (4 aligned LDS dwords + alignbyte): the first non-digit byte
//     after an optional '-' is the end e (min3 over the three words' ffbl);
//   * the 12 bytes ENDING at k+e are read again, so the digits sit right-aligned;
//     the bytes before them become '0' (one bitfield insert per word) and the value
//     is digits12 of the three words, mod 2^32: strtol
//     saturates only past 18 digits, so (int)strtol is the low 32 bits.
__device__ __forceinline__ int32_t next_token_nl(const uint8_t* __restrict__ s, int& k, int kend,
                                                 bool& more) {
    const uint32_t* d = reinterpret_cast<const uint32_t*>(s);
    const int a = k >> 2;
    const uint32_t r = (uint32_t)k & 3u;
    const uint32_t d0 = d[a], d1 = d[a + 1], d2 = d[a + 2], d3 = d[a + 3];
    const uint32_t w0 = __builtin_amdgcn_alignbyte(d1, d0, r), w1 = __builtin_amdgcn_alignbyte(d2, d1, r),
                   w2 = __builtin_amdgcn_alignbyte(d3, d2, r);
    const uint32_t neg = (w0 & 0xFFu) == '-' ? 1u : 0u;
    const uint32_t f0 = nondigit_first(w0) & ~(neg << 7), f1 = nondigit_first(w1),
                   f2 = nondigit_first(w2) | 0x80000000u;  // byte 11 ends the scan
    const uint32_t bit = min(min(ffbl(f0), ffbl(f1) | 32u), ffbl(f2) | 64u);
    const int e = (int)(bit >> 3);
    const uint32_t L = (uint32_t)e - neg;  // digits
    const uint32_t c = s[k + e];
    const bool ok = (L <= 10u) & ((c == (uint32_t)',') | (c == (uint32_t)'\n') | (c == 0u));
    if (!ok) return parse_token(s, k, kend, more);  // isspace / '+' / junk / 11+ digits
    const int b = k + e - 12;  // >= kPre - 12 >= 0
    const int a2 = b >> 2;
    const uint32_t r2 = (uint32_t)b & 3u;
    const uint32_t e0 = d[a2], e1 = d[a2 + 1], e2 = d[a2 + 2], e3 = d[a2 + 3];
    const uint32_t z8 = 8u * (12u - L);  // leading bits that are not digits: 16..96
    const uint64_t m01 = z8 >= 64u ? 0ull : (~0ull << z8);
    const uint32_t m2 = (uint32_t)(0xFFFFFFFFull << (z8 > 64u ? z8 - 64u : 0u));
    const uint32_t m0 = (uint32_t)m01, m1 = (uint32_t)(m01 >> 32);
    const uint32_t x0 = (__builtin_amdgcn_alignbyte(e1, e0, r2) & m0) | (0x30303030u & ~m0);
    const uint32_t x1 = (__builtin_amdgcn_alignbyte(e2, e1, r2) & m1) | (0x30303030u & ~m1);
    const uint32_t x2 = (__builtin_amdgcn_alignbyte(e3, e2, r2) & m2) | (0x30303030u & ~m2);
    const uint32_t v = digits12(x0, x1, x2);
    more = c == ',';
    k += e + (more ? 1 : 0);
    return (int32_t)(neg ? 0u - v : v);
}

// ---- pass 2, token-parallel form (the usual text): every row is ncols tokens
// [-]digits{0..10}, ',' between them and '\n' after the last, no line over 1023
// bytes. Then token t of the chunk is the text between separators t and t+1 of the
// chunk's list, counted from the '\n' that ends the previous chunk's last row, and
// it belongs to row t / ncols, column t % ncols. So:
//   * every lane classifies 68 staged bytes: a byte below '-' (0x2D) is a candidate
//     separator ('\n' and ',' are; digits and '-' are not): 4 ops a word, and the
//     flag bytes become a bit mask by v_dot4 with weights 1, 2, 4, 8 (16, ..., 128);
//   * the candidates' LDS offsets are listed in text order (one block scan of the
//     counts); wave 0 also finds the first '\n' of the chunk (entry f0);
//   * lane i takes tokens i, i + S, ... with S the largest multiple of ncols up to
//     256, so its column is fixed: one pointer, one min and one max per lane. The
//     token's bytes are its two list entries apart; the 12 bytes ending at the
//     separator are read from LDS, bytes before the digits become '0', and the
//     value is digits12 of three words (next_token_nl's arithmetic).
// Each token checks its own separator byte exactly (',' or, for the last column,
// '\n') and its digits; together with the candidate list (every ',' and '\n' is a
// candidate) that proves the chunk is R rows of the fast form. Anything else (a
// space, '+', '\r', a missing or extra token, 11+ digits, a NUL) makes the block
// return false before anything but its own rows' columns was written; the row-wise
// parse then rewrites those rows.
constexpr int kTokSeg = (kChunk + kHalo) / kTPB;  // 68 bytes classified per lane
constexpr int kTokMaxCols = 16;
static_assert((kChunk + kHalo) % kTPB == 0 && kTokSeg % 4 == 0 && kTokSeg < 64 + 32, "classification in words");

__device__ __forceinline__ uint32_t below_2d(uint32_t x) {  // 0x80 in each byte < 0x2D
    return ~(((x | 0x80808080u) - 0x2D2D2D2Du) | x) & 0x80808080u;
}

__device__ bool parse_chunk_tokens(const uint8_t* __restrict__ s, uint16_t* __restrict__ list,
                                   uint32_t* s_u, int* s_f0, int* s_mm, uint4* s_lead, uint64_t r0, uint32_t R,
                                   int ncols, int32_t* const* __restrict__ cols) {
    const int tid = threadIdx.x, lane = tid & 63;
    const int base = kPre + tid * kTokSeg;
    const uint32_t* d = reinterpret_cast<const uint32_t*>(s + base);
    constexpr int kW = kTokSeg / 4;
    uint32_t f[kW];
#pragma unroll
    for (int k = 0; k < kW; k++) f[k] = below_2d(d[k]);
    // flag bytes -> bits: v_dot4 with weights 1, 2, 4, 8 (and 16, ..., 128 for the
    // next word) gives 128 x the bits of two words
    unsigned long long m = 0;
#pragma unroll
    for (int g = 0; g < kW / 4 && g < 4; g++) {
        const uint32_t lo = __builtin_amdgcn_udot4(f[4 * g + 1], 0x80402010u,
                                                   __builtin_amdgcn_udot4(f[4 * g], 0x08040201u, 0u, false), false);
        const uint32_t hi = __builtin_amdgcn_udot4(f[4 * g + 3], 0x80402010u,
                                                   __builtin_amdgcn_udot4(f[4 * g + 2], 0x08040201u, 0u, false), false);
        m |= (unsigned long long)((lo | (hi << 8)) >> 7) << (16 * g);
    }
#pragma unroll
    for (int k = kW / 4 * 4; k < kW && k < 16; k++)
        m |= (unsigned long long)(__builtin_amdgcn_udot4(f[k], 0x08040201u, 0u, false) >> 7) << (4 * k);
    uint32_t mt = 0;  // the words past the first 64 bytes
#pragma unroll
    for (int k = 16; k < kW; k++) mt |= (__builtin_amdgcn_udot4(f[k], 0x08040201u, 0u, false) >> 7) << (4 * (k - 16));
    const bool pre = tid == 0 && s[kPre - 1] == '\n';  // byte cs-1: a row starts at cs
    if (tid == 0) s_f0[1] = 0;  // "not the fast form"
    if (tid < 13) {  // s_lead[z]: byte masks of a 12-byte window that clear its first z bytes
        const uint32_t z8 = 8u * (uint32_t)tid;
        const uint64_t m01 = z8 >= 64u ? 0ull : (~0ull << z8);
        s_lead[tid] = make_uint4((uint32_t)m01, (uint32_t)(m01 >> 32),
                                 z8 >= 96u ? 0u : (uint32_t)(0xFFFFFFFFull << (z8 > 64u ? z8 - 64u : 0u)), 0u);
    }
    uint32_t ntot;
    // (no closing barrier: the list barrier below orders the reads of s_u)
    uint32_t o = block_excl_sum<false>((uint32_t)(__popcll(m) + __popc(mt) + (pre ? 1 : 0)), s_u, &ntot);
    if (ntot > (uint32_t)kList) {
        __syncthreads();  // (the row-wise parse writes s_u next)
        return false;
    }
    if (pre) list[o++] = (uint16_t)(kPre - 1);
    // (three 32-bit loops: a 64-bit find-first and clear cost twice the VALU)
    const uint32_t mw[3] = {(uint32_t)m, (uint32_t)(m >> 32), mt};
#pragma unroll
    for (int h = 0; h < 3; h++) {
        for (uint32_t x = mw[h]; x; x &= x - 1) list[o++] = (uint16_t)(base + 32 * h + __builtin_ctz(x));
    }
    __syncthreads();
    // f0 = the first '\n' of the list. In the fast form a row has at most ncols <= 16
    // separators, so it is among the first 64 entries; every wave finds it by one
    // ballot (a search inside the list loop held wave 0, and the block, ~1000 cycles).
    const bool isnl = (uint32_t)lane < ntot && s[list[lane]] == '\n';
    const unsigned long long bnl = __ballot(isnl);
    const uint32_t T = R * (uint32_t)ncols;
    if (!bnl) return false;
    const int f0 = __builtin_ctzll(bnl);
    if ((uint64_t)f0 + T >= ntot) return false;

    const uint32_t S = (uint32_t)(kTPB - kTPB % ncols);
    bool bad = false;
    int mn = INT_MAX, mx = INT_MIN;
    int col = 0;
    if ((uint32_t)tid < S) {
        // tid / ncols by a 16-bit reciprocal (exact for tid < 256, ncols <= 16),
        // not the ~20-instruction integer division
        const uint32_t magic = (65536u + (uint32_t)ncols - 1u) / (uint32_t)ncols;
        uint32_t rr = ((uint32_t)tid * magic) >> 16;
        col = tid - (int)rr * ncols;
        const uint32_t expect = col == ncols - 1 ? (uint32_t)'\n' : (uint32_t)',';
        gint32* op = global_ptr(cols[col]) + r0 + rr;  // this lane's next row of its column
        const uint32_t rstep = S / (uint32_t)ncols;
        const uint32_t* w = reinterpret_cast<const uint32_t*>(s);
        const uint16_t* lt = list + f0;
        // (pointer steps: no separate token / row counters in the loop)
        for (const uint16_t *q = lt + tid, *qe = lt + T; q < qe; q += S, op += rstep) {
            const uint32_t pb = q[0], pe = q[1];  // the separators before / after the token
            const uint32_t L = pe - pb - 1u;
            const uint32_t a2 = (pe - 12u) >> 2, r2 = pe & 3u;  // the 12 bytes before pe, and pe
            const uint32_t e0 = w[a2], e1 = w[a2 + 1], e2 = w[a2 + 2], e3 = w[a2 + 3];
            const uint32_t x0 = __builtin_amdgcn_alignbyte(e1, e0, r2), x1 = __builtin_amdgcn_alignbyte(e2, e1, r2),
                           x2 = __builtin_amdgcn_alignbyte(e3, e2, r2);
            const uint32_t neg = s[pb + 1] == '-' ? 1u : 0u;  // (L == 0: that byte is the separator)
            const uint32_t Ld = L - neg;  // digits
            const uint4 mk = s_lead[12u - min(Ld, 12u)];  // keeps the last Ld bytes of 12
            // digit values: byte ^ '0' (no borrows: a digit byte is 0x30 | d), the bytes
            // before the digits cleared; a byte that is not a digit gives a value > 9
            const uint32_t d0 = (x0 ^ 0x30303030u) & mk.x;
            const uint32_t d1 = (x1 ^ 0x30303030u) & mk.y;
            const uint32_t d2 = (x2 ^ 0x30303030u) & mk.z;
            const uint32_t sep = __builtin_amdgcn_alignbyte(e3, e3, r2) & 0xFFu;  // byte pe
            const uint32_t nd = ((d0 + 0x76767676u) | d0 | (d1 + 0x76767676u) | d1 | (d2 + 0x76767676u) | d2) &
                                0x80808080u;
            bad |= (sep != expect) | (Ld > 10u) | (nd != 0u);
            const uint32_t v = digits12_d(d0, d1, d2);
            const int32_t y = (int32_t)(neg ? 0u - v : v);
            *op = y;
            mn = min(mn, y);
            mx = max(mx, y);
        }
    }
    // min/max go to LDS before the one barrier that also publishes the flag (a chunk
    // that fails re-initialises them for the row-wise parse)
    if ((uint32_t)tid < S) {  // LDS atomics (a shuffle tree cost ~50 VALU a wave)
        atomicMin(&s_mm[2 * col], mn);
        atomicMax(&s_mm[2 * col + 1], mx);
    }
    if (bad) s_f0[1] = 1;  // (__syncthreads_or costs ~26 VALU a wave)
    __syncthreads();
    return s_f0[1] == 0;
}

// ---- pass 2: parse. One block per chunk. The chunk's row starts stay as one
// 64-bit mask per thread segment plus the exclusive prefix of their counts; lane i
// takes pieces i, i+256, ... and finds piece i's byte by a binary search over the
// prefix and a select in the mask (2 KB of LDS instead of a 32 KB start list).
template <bool VEC>
__global__ __launch_bounds__(kTPB) void k_csv_parse(const char* __restrict__ text, uint64_t n,
                                                     const unsigned long long* __restrict__ row_base,
                                                     const long long* __restrict__ prev, int ncols,
                                                     int32_t* const* __restrict__ cols,
                                                     int2* __restrict__ partial, uint16_t* __restrict__ nf,
                                                     unsigned* flags, uint64_t rows, int tok) {
    __shared__ __attribute__((aligned(16))) uint8_t s[kLds + 32];  // + token_fast's over-read
    // the start list, or (more starts than it holds) the per-segment masks and
    // prefix it is searched in: one is written per chunk, so they share LDS (26 KB
    // a block: 6 blocks per CU instead of 5)
    __shared__ __attribute__((aligned(16))) unsigned long long s_lu[kList * 2 / 8];
    static_assert(kTPB * 12 <= kList * 2, "masks + prefix fit the list's bytes");
    uint16_t* const s_list = reinterpret_cast<uint16_t*>(s_lu);
    unsigned long long* const s_mask = s_lu;
    uint32_t* const s_off = reinterpret_cast<uint32_t*>(s_lu + kTPB);
    __shared__ long long s_w[kWaves];
    __shared__ uint32_t s_u[kWaves];
    __shared__ int s_f0[2];
    __shared__ uint4 s_lead[13];
    extern __shared__ int s_mm[];  // 2 * ncols: min, max
    const uint64_t c = xcd_tile(blockIdx.x, gridDim.x), cs = c * kChunk;  // XCD-contiguous chunks: halo reads and shared column lines meet in one L2
    const uint64_t ce = cs + kChunk < n ? cs + kChunk : n;
    const int tid = threadIdx.x, lane = tid & 63;
    const bool lmode = __builtin_amdgcn_readfirstlane(flags[F_LONG]) != 0;
    stage_chunk<VEC>(text, n, cs, s);
    for (int j = tid; j < ncols; j += kTPB) {
        s_mm[2 * j] = INT_MAX;
        s_mm[2 * j + 1] = INT_MIN;
    }
    __syncthreads();
    if (tok && !lmode && !nf && ncols <= kTokMaxCols) {
        const uint64_t rb = row_base[c];
        const uint64_t R = (c + 1 < gridDim.x ? row_base[c + 1] : rows) - rb;
        if (parse_chunk_tokens(s, s_list, s_u, s_f0, s_mm, s_lead, rb, (uint32_t)R, ncols, cols)) {
            for (int j = tid; j < ncols; j += kTPB)  // (after the flag barrier: every atomic is in)
                partial[c * (uint64_t)ncols + j] = make_int2(s_mm[2 * j], s_mm[2 * j + 1]);
            return;
        }
        for (int j = tid; j < ncols; j += kTPB) {  // (ordered before the row-wise atomics by its scan)
            s_mm[2 * j] = INT_MAX;
            s_mm[2 * j + 1] = INT_MIN;
        }
    }
    unsigned long long st = real_starts(s, cs, ce, tid);
    const uint64_t a = cs + (uint64_t)tid * kSeg;
    if (lmode) {
        const long long mylast = st ? (long long)(a + 63 - __builtin_clzll(st)) : -1;
        st = piece_starts(st, a, block_excl_max(mylast, prev[c], s_w), ce);
    }
    uint32_t nst;
    const uint32_t o = block_excl_sum((uint32_t)__popcll(st), s_u, &nst);
    if (nst > (uint32_t)kList) {
        s_off[tid] = o;
        s_mask[tid] = st;
    } else {  // the usual case: an explicit start list
        uint32_t q = o;
        for (unsigned long long m = st; m; m &= m - 1) s_list[q++] = (uint16_t)(tid * kSeg + __builtin_ctzll(m));
    }
    __syncthreads();

    const uint64_t r0 = row_base[c];
    int mn[kRegCols], mx[kRegCols];
#pragma unroll
    for (int j = 0; j < kRegCols; j++) mn[j] = INT_MAX, mx[j] = INT_MIN;
    bool missing = false;
    for (uint32_t i = tid; i < nst; i += kTPB) {
        int off;  // piece start within the chunk
        if (nst <= (uint32_t)kList) {
            off = s_list[i];
        } else {  // more starts than the list holds: search the per-segment prefix
            int t = 0;  // last segment whose prefix is <= i
#pragma unroll
            for (int step = kTPB / 2; step > 0; step >>= 1)
                if (s_off[t + step] <= i) t += step;
            unsigned long long m = s_mask[t];
            for (uint32_t r = s_off[t]; r < i; r++) m &= m - 1;
            off = t * kSeg + __builtin_ctzll(m);
        }
        const uint64_t p = cs + (uint64_t)off;
        const uint64_t pe = p + kPiece < n ? p + kPiece : n;  // fgets cap / EOF
        int k = kPre + off;
        const int kend = k + (int)(pe - p);
        const uint64_t row = r0 + i;
        bool more = true;
        int got = 0;
#pragma unroll
        for (int j = 0; j < kRegCols; j++) {
            if (j < ncols && more) {
                const int32_t v = lmode ? next_token(s, k, kend, more) : next_token_nl(s, k, kend, more);
                global_ptr(cols[j])[row] = v;
                mn[j] = min(mn[j], v);
                mx[j] = max(mx[j], v);
                got = j + 1;
            }
        }
        for (int j = kRegCols; j < ncols && more; j++) {
            const int32_t v = lmode ? next_token(s, k, kend, more) : next_token_nl(s, k, kend, more);
            global_ptr(cols[j])[row] = v;
            atomicMin(&s_mm[2 * j], v);
            atomicMax(&s_mm[2 * j + 1], v);
            got = j + 1;
        }
        if (got < ncols) missing = true;
        if (nf) nf[row] = (uint16_t)got;
    }
    if (__ballot(missing) && lane == 0) atomicOr(&flags[F_MISSING], 1u);
#pragma unroll
    for (int j = 0; j < kRegCols; j++) {
        if (j < ncols) {
            const int a0 = wave_min_i(mn[j]), a1 = wave_max_i(mx[j]);
            if (lane == 0) {
                atomicMin(&s_mm[2 * j], a0);
                atomicMax(&s_mm[2 * j + 1], a1);
            }
        }
    }
    __syncthreads();
    for (int j = tid; j < ncols; j += kTPB)
        partial[c * (uint64_t)ncols + j] = make_int2(s_mm[2 * j], s_mm[2 * j + 1]);
}

// min/max per column over the chunk partials (one block per column); zfill[j]
// set = the fix-up wrote 0s into column j (rows before its first token), which
// count as values like every other row.
__global__ __launch_bounds__(kTPB) void k_csv_minmax_init(int ncols, const unsigned* __restrict__ zfill,
                                                           int32_t* __restrict__ out) {
    for (int j = threadIdx.x; j < ncols; j += kTPB) {
        const bool z = zfill && zfill[j];
        out[2 * j] = z ? 0 : INT_MAX;
        out[2 * j + 1] = z ? 0 : INT_MIN;
    }
}

// Fold of the per-chunk partials (flat [chunk][column] int2) into out, which
// k_csv_minmax_init seeded: each block a contiguous range of the flat array (one
// read, coalesced), per column in registers when kTPB % ncols == 0 (a thread's
// column is then fixed), else through LDS atomics; one global atomic per column
// and block. (One block per column read 583K strided partials each: 2.4 ms at 1e9
// rows.)
__global__ __launch_bounds__(kTPB) void k_csv_minmax(const int2* __restrict__ partial, uint64_t nch,
                                                      int ncols, uint64_t per, int32_t* __restrict__ out) {
    extern __shared__ int s_mm[];  // 2 * ncols
    const int tid = threadIdx.x, lane = tid & 63;
    const uint64_t tot = nch * (uint64_t)ncols;
    const uint64_t i0 = (uint64_t)blockIdx.x * per, i1 = i0 + per < tot ? i0 + per : tot;
    if (kTPB % ncols == 0) {
        int mn = INT_MAX, mx = INT_MIN;
        for (uint64_t i = i0 + (uint64_t)tid; i < i1; i += kTPB) {
            const int2 v = partial[i];
            mn = min(mn, v.x);
            mx = max(mx, v.y);
        }
        const int col = (int)((i0 + (uint64_t)tid) % (uint64_t)ncols);  // per % ncols == 0
        for (int o = 32; o >= ncols; o >>= 1) {  // lanes l and l ^ o share the column
            mn = min(mn, __shfl_xor(mn, o, 64));
            mx = max(mx, __shfl_xor(mx, o, 64));
        }
        if (ncols > 64 || lane < ncols) {
            atomicMin(&out[2 * col], mn);
            atomicMax(&out[2 * col + 1], mx);
        }
        return;
    }
    for (int j = tid; j < ncols; j += kTPB) s_mm[2 * j] = INT_MAX, s_mm[2 * j + 1] = INT_MIN;
    __syncthreads();
    for (uint64_t i = i0 + (uint64_t)tid; i < i1; i += kTPB) {
        const int2 v = partial[i];
        const int col = (int)(i % (uint64_t)ncols);
        atomicMin(&s_mm[2 * col], v.x);
        atomicMax(&s_mm[2 * col + 1], v.y);
    }
    __syncthreads();
    for (int j = tid; j < ncols; j += kTPB) {
        atomicMin(&out[2 * j], s_mm[2 * j]);
        atomicMax(&out[2 * j + 1], s_mm[2 * j + 1]);
    }
}

// ---- missing-token fix-up: a row whose piece had got = nf[r] tokens keeps, for
// every column j >= got, the value of the last earlier row that had token j
// (0 when there is none). Tiles of kFillTile rows, 4 per thread.
__global__ __launch_bounds__(kTPB) void k_fill_tile_last(const uint16_t* __restrict__ nf, uint64_t rows,
                                                          int ncols, long long* __restrict__ tile_last) {
    __shared__ long long s_w[kWaves];
    const uint64_t t = blockIdx.x, r0 = t * kFillTile + (uint64_t)threadIdx.x * 4;
    const int lane = threadIdx.x & 63;
    uint16_t g[4];
#pragma unroll
    for (int e = 0; e < 4; e++) g[e] = r0 + e < rows ? nf[r0 + e] : 0;
    for (int j = 0; j < ncols; j++) {
        long long l = -1;
#pragma unroll
        for (int e = 0; e < 4; e++)
            if (r0 + e < rows && g[e] > j) l = (long long)(r0 + e);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const long long u = __shfl_xor(l, o, 64);
            l = l > u ? l : u;
        }
        if (lane == 0) s_w[threadIdx.x >> 6] = l;
        __syncthreads();
        if (threadIdx.x == 0) {
            long long m = s_w[0];
            for (int w = 1; w < kWaves; w++) m = m > s_w[w] ? m : s_w[w];
            tile_last[t * (uint64_t)ncols + j] = m;
        }
        __syncthreads();
    }
}

// carry[t][j] = last row with token j in tiles < t (exclusive max; one block per column)
__global__ __launch_bounds__(1024) void k_fill_carry(const long long* __restrict__ tile_last,
                                                      uint64_t ntiles, int ncols,
                                                      long long* __restrict__ carry) {
    __shared__ long long s_w[16];
    const int j = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    long long run = -1;
    for (uint64_t b = 0; b < ntiles; b += 1024) {
        const uint64_t t = b + tid;
        const long long x = t < ntiles ? tile_last[t * (uint64_t)ncols + j] : -1;
        const long long inc = wave_incl_max(x, lane);
        if (lane == 63) s_w[wave] = inc;
        __syncthreads();
        long long pre = run, all = run;
        for (int w = 0; w < 16; w++) {
            if (w < wave) pre = pre > s_w[w] ? pre : s_w[w];
            all = all > s_w[w] ? all : s_w[w];
        }
        long long ex = __shfl_up(inc, 1, 64);
        if (lane == 0) ex = LLONG_MIN;
        if (t < ntiles) carry[t * (uint64_t)ncols + j] = pre > ex ? pre : ex;
        run = all;
        __syncthreads();
    }
}

__global__ __launch_bounds__(kTPB) void k_fill_apply(const uint16_t* __restrict__ nf, uint64_t rows,
                                                      int ncols, int32_t* const* __restrict__ cols,
                                                      const long long* __restrict__ carry,
                                                      unsigned* __restrict__ zfill) {
    __shared__ long long s_w[kWaves];
    const uint64_t t = blockIdx.x, r0 = t * kFillTile + (uint64_t)threadIdx.x * 4;
    uint16_t g[4];
#pragma unroll
    for (int e = 0; e < 4; e++) g[e] = r0 + e < rows ? nf[r0 + e] : 0xFFFF;
    for (int j = 0; j < ncols; j++) {
        long long l = -1;
#pragma unroll
        for (int e = 0; e < 4; e++)
            if (r0 + e < rows && g[e] > j) l = (long long)(r0 + e);
        long long src = block_excl_max(l, carry[t * (uint64_t)ncols + j], s_w);
        int32_t* col = cols[j];
#pragma unroll
        for (int e = 0; e < 4; e++) {
            if (r0 + e >= rows) break;
            if (g[e] > j) {
                src = (long long)(r0 + e);
            } else {
                col[r0 + e] = src >= 0 ? col[src] : 0;
                if (src < 0) atomicOr(&zfill[j], 1u);
            }
        }
    }
}

int launch_count(const char* text, uint64_t n, const CsvWs& w, bool lng, hipStream_t st) {
    const uint64_t nch = nchunks_of(n);
    const bool vec = aligned16(text);
    const dim3 g((unsigned)nch);
    if (lng) {
        if (vec) hipLaunchKernelGGL((k_csv_count<true, true>), g, dim3(kTPB), 0, st, text, n, w.cnt, w.first, w.last, w.prev, w.flags);
        else hipLaunchKernelGGL((k_csv_count<false, true>), g, dim3(kTPB), 0, st, text, n, w.cnt, w.first, w.last, w.prev, w.flags);
    } else {
        if (vec) hipLaunchKernelGGL((k_csv_count<true, false>), g, dim3(kTPB), 0, st, text, n, w.cnt, w.first, w.last, w.prev, w.flags);
        else hipLaunchKernelGGL((k_csv_count<false, false>), g, dim3(kTPB), 0, st, text, n, w.cnt, w.first, w.last, w.prev, w.flags);
    }
    LAUNCHCHK("k_csv_count");
    return MQ_OK;
}

int launch_parse(const char* text, uint64_t n, int ncols, uint64_t rows, const CsvWs& w, uint16_t* nf,
                 hipStream_t st) {
    const uint64_t nch = nchunks_of(n);
    const size_t dyn = (size_t)ncols * 8;
    static const int tok = !(getenv("MQ_CSV_TOKENS") && getenv("MQ_CSV_TOKENS")[0] == '0');  // 0: row-wise only (A/B)
    if (aligned16(text))
        hipLaunchKernelGGL((k_csv_parse<true>), dim3((unsigned)nch), dim3(kTPB), dyn, st, text, n, w.row_base, w.prev, ncols, w.colptr, w.partial, nf, w.flags, rows, tok);
    else
        hipLaunchKernelGGL((k_csv_parse<false>), dim3((unsigned)nch), dim3(kTPB), dyn, st, text, n, w.row_base, w.prev, ncols, w.colptr, w.partial, nf, w.flags, rows, tok);
    LAUNCHCHK("k_csv_parse");
    return MQ_OK;
}

int check_args(const char* text, uint64_t n, void* ws, size_t ws_bytes, int ncols) {
    if (n && !text) return set_err(MQ_EINVAL, "mq_csv: NULL text");
    if (!ws) return set_err(MQ_EINVAL, "mq_csv: NULL workspace");
    if (ncols < 0 || ncols > kMaxCols) return set_err(MQ_EINVAL, "mq_csv: ncols %d outside [0, %d]", ncols, kMaxCols);
    if (nchunks_of(n) >= (1ull << 31)) return set_err(MQ_EINVAL, "mq_csv: text too large");
    if (ws_bytes < carve(nullptr, n, ncols, nullptr)) return set_err(MQ_EINVAL, "mq_csv: workspace too small");
    return MQ_OK;
}

}  // namespace

extern "C" {

size_t mq_csv_workspace_bytes(uint64_t n, int ncols) {
    return carve(nullptr, n, ncols < 0 ? 0 : (ncols > kMaxCols ? kMaxCols : ncols), nullptr);
}

int mq_csv_count_rows(const char* d_text, uint64_t n, int ncols, uint64_t* h_rows, void* d_ws,
                      size_t ws_bytes, void* stream) {
    DevState* s;
    int rc = ensure_ready(&s);
    if (rc) return rc;
    if (!h_rows) return set_err(MQ_EINVAL, "mq_csv_count_rows: NULL h_rows");
    *h_rows = 0;
    if ((rc = check_args(d_text, n, d_ws, ws_bytes, ncols))) return rc;
    hipStream_t st = (hipStream_t)stream;
    CsvWs w;
    carve(d_ws, n, ncols, &w);
    HIPCHK(hipMemsetAsync(w.flags, 0, 64, st));
    if (n == 0) return MQ_OK;
    const uint64_t nch = nchunks_of(n);
    if (aligned16(d_text))
        hipLaunchKernelGGL((k_csv_count_stream<true>), dim3((unsigned)nch), dim3(kTPB), 0, st, d_text, n, w.cnt, w.flags);
    else
        hipLaunchKernelGGL((k_csv_count_stream<false>), dim3((unsigned)nch), dim3(kTPB), 0, st, d_text, n, w.cnt, w.flags);
    LAUNCHCHK("k_csv_count_stream");
    unsigned flags[4] = {0, 0, 0, 0};
    HIPCHK(hipMemcpyAsync(flags, w.flags, 16, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (flags[F_MAYBE_LONG]) {  // exact check: a gap of more than 1023 bytes between starts?
        if ((rc = launch_count(d_text, n, w, false, st))) return rc;
        hipLaunchKernelGGL(k_csv_long_check, dim3((unsigned)((nch + kTPB - 1) / kTPB)), dim3(kTPB), 0, st,
                           w.cnt, w.first, w.last, nch, n, w.flags);
        LAUNCHCHK("k_csv_long_check");
        HIPCHK(hipMemcpyAsync(flags, w.flags, 16, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
    }
    if (flags[F_LONG]) {  // lines over 1023 bytes: rows are fgets pieces
        hipLaunchKernelGGL(k_csv_prev_start, dim3(1), dim3(1024), 0, st, w.last, nch, w.prev);
        LAUNCHCHK("k_csv_prev_start");
        if ((rc = launch_count(d_text, n, w, true, st))) return rc;
    }
    if ((rc = scan_u32_exclusive(w.cnt, w.row_base, nch, w.scratch, st))) return rc;
    unsigned long long base = 0;
    uint32_t last = 0;
    HIPCHK(hipMemcpyAsync(&base, w.row_base + (nch - 1), 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(&last, w.cnt + (nch - 1), 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    *h_rows = base + last;
    return MQ_OK;
}

int mq_csv_parse_int32(const char* d_text, uint64_t n, int ncols, int32_t* const* d_cols,
                       uint64_t rows, int32_t* d_minmax, void* d_ws, size_t ws_bytes, void* stream) {
    DevState* s;
    int rc = ensure_ready(&s);
    if (rc) return rc;
    if ((rc = check_args(d_text, n, d_ws, ws_bytes, ncols))) return rc;
    if (ncols && (!d_cols || !d_minmax)) return set_err(MQ_EINVAL, "mq_csv_parse_int32: NULL columns");
    for (int j = 0; j < ncols; j++)
        if (rows && !d_cols[j]) return set_err(MQ_EINVAL, "mq_csv_parse_int32: NULL column %d", j);
    hipStream_t st = (hipStream_t)stream;
    CsvWs w;
    carve(d_ws, n, ncols, &w);
    if (ncols == 0) return MQ_OK;
    if (rows == 0 || n == 0) {
        std::vector<int32_t> mm(2 * (size_t)ncols);
        for (int j = 0; j < ncols; j++) mm[2 * j] = INT_MAX, mm[2 * j + 1] = INT_MIN;
        HIPCHK(hipMemcpyAsync(d_minmax, mm.data(), mm.size() * 4, hipMemcpyHostToDevice, st));
        HIPCHK(hipStreamSynchronize(st));
        return MQ_OK;
    }
    const uint64_t nch = nchunks_of(n);
    HIPCHK(hipMemcpyAsync(w.colptr, d_cols, (size_t)ncols * 8, hipMemcpyHostToDevice, st));
    if ((rc = launch_parse(d_text, n, ncols, rows, w, nullptr, st))) return rc;
    unsigned flags[2] = {0, 0};
    HIPCHK(hipMemcpyAsync(flags, w.flags, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    unsigned* zfill = nullptr;
    void* scratch = nullptr;
    if (flags[F_MISSING]) {  // rows with fewer than ncols tokens: the stale-value copy
        const uint64_t ntiles = (rows + kFillTile - 1) / kFillTile;
        const size_t b_nf = align16(rows * 2), b_t = align16(ntiles * (size_t)ncols * 8);
        scratch = pool_alloc(b_nf + 2 * b_t + align16((size_t)ncols * 4));
        if (!scratch) return set_err(MQ_ENOMEM, "mq_csv_parse_int32: fix-up scratch");
        char* p = static_cast<char*>(scratch);
        uint16_t* nf = reinterpret_cast<uint16_t*>(p);
        long long* tl = reinterpret_cast<long long*>(p + b_nf);
        long long* carry = reinterpret_cast<long long*>(p + b_nf + b_t);
        zfill = reinterpret_cast<unsigned*>(p + b_nf + 2 * b_t);
        HIPCHK(hipMemsetAsync(zfill, 0, (size_t)ncols * 4, st));
        if ((rc = launch_parse(d_text, n, ncols, rows, w, nf, st))) return rc;
        hipLaunchKernelGGL(k_fill_tile_last, dim3((unsigned)ntiles), dim3(kTPB), 0, st, nf, rows, ncols, tl);
        LAUNCHCHK("k_fill_tile_last");
        hipLaunchKernelGGL(k_fill_carry, dim3((unsigned)ncols), dim3(1024), 0, st, tl, ntiles, ncols, carry);
        LAUNCHCHK("k_fill_carry");
        hipLaunchKernelGGL(k_fill_apply, dim3((unsigned)ntiles), dim3(kTPB), 0, st, nf, rows, ncols,
                           w.colptr, carry, zfill);
        LAUNCHCHK("k_fill_apply");
    }
    hipLaunchKernelGGL(k_csv_minmax_init, dim3(1), dim3(kTPB), 0, st, ncols, zfill, d_minmax);
    LAUNCHCHK("k_csv_minmax_init");
    {
        const uint64_t tot = nch * (uint64_t)ncols;
        uint64_t per = (tot + 1023) / 1024;                            // <= 1024 blocks
        per = (per + 8ull * kTPB - 1) / (8ull * kTPB) * (8ull * kTPB);  // 8 partials a thread at least
        per = (per + ncols - 1) / ncols * ncols;                       // whole chunks: a thread's column is fixed
        const unsigned g = (unsigned)((tot + per - 1) / per);
        hipLaunchKernelGGL(k_csv_minmax, dim3(g), dim3(kTPB), (size_t)ncols * 8, st, w.partial, nch, ncols, per,
                           d_minmax);
        LAUNCHCHK("k_csv_minmax");
    }
    if (scratch) {
        HIPCHK(hipStreamSynchronize(st));
        pool_free(scratch);
    }
    return MQ_OK;
}

}  // extern "C"
