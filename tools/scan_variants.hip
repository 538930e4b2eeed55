// scan_variants.hip — tuning harness for the select+count+sum scan (not product code).
// Times variants of the streaming kernel interleaved in one process
// (cdna_hip_programming.md §5.4 rule 24) on a 1e9-row int32 column and prints
// GB/s of algorithmic bytes (4N) per variant: median and best of R rounds.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/scan_variants.hip -o tools/scan_variants
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                     \
    do {                                                                          \
        hipError_t e = (x);                                                       \
        if (e != hipSuccess) {                                                    \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                \
            exit(1);                                                              \
        }                                                                         \
    } while (0)

struct Partial {
    unsigned long long count;
    long long sum;
    int mn, mx;
    unsigned long long pad;
};

__device__ __forceinline__ int4 ld(const int* p, bool nt) {
    if (nt) {
        int4 v;
        v.x = __builtin_nontemporal_load(p + 0);
        v.y = __builtin_nontemporal_load(p + 1);
        v.z = __builtin_nontemporal_load(p + 2);
        v.w = __builtin_nontemporal_load(p + 3);
        return v;
    }
    return *reinterpret_cast<const int4*>(p);
}

typedef int v4i __attribute__((ext_vector_type(4)));
__device__ __forceinline__ int4 ld_nt4(const int4* p) {
    v4i t = __builtin_nontemporal_load(reinterpret_cast<const v4i*>(p));
    return make_int4(t.x, t.y, t.z, t.w);
}

// MODE 0: contiguous chunk per block; MODE 1: grid-stride (grid covers a contiguous span per iter)
// MINMAX: also track min/max
template <int TPB, int UNROLL, bool NT, int MODE, bool MINMAX>
__global__ __launch_bounds__(TPB) void k_var(const int* __restrict__ col, unsigned long long n,
                                             unsigned long long rpb, unsigned lo, unsigned wm1,
                                             Partial* __restrict__ part) {
    constexpr int TILE = TPB * 4;
    unsigned cnt = 0;
    long long sum = 0;
    int mn = INT_MAX, mx = INT_MIN;
    auto eat = [&](int4 v) {
        bool p0 = ((unsigned)v.x - lo) <= wm1, p1 = ((unsigned)v.y - lo) <= wm1,
             p2 = ((unsigned)v.z - lo) <= wm1, p3 = ((unsigned)v.w - lo) <= wm1;
        cnt += p0 + p1 + p2 + p3;
        sum += (long long)(p0 ? v.x : 0) + (long long)(p1 ? v.y : 0) + (long long)(p2 ? v.z : 0) +
               (long long)(p3 ? v.w : 0);
        if (MINMAX) {
            mn = min(mn, min(min(p0 ? v.x : INT_MAX, p1 ? v.y : INT_MAX), min(p2 ? v.z : INT_MAX, p3 ? v.w : INT_MAX)));
            mx = max(mx, max(max(p0 ? v.x : INT_MIN, p1 ? v.y : INT_MIN), max(p2 ? v.z : INT_MIN, p3 ? v.w : INT_MIN)));
        }
    };
    if (MODE == 0) {
        const unsigned long long start = (unsigned long long)blockIdx.x * rpb;
        unsigned long long end = min(start + rpb, n);
        unsigned long long t = start;
        for (; t + (unsigned long long)UNROLL * TILE <= end; t += (unsigned long long)UNROLL * TILE) {
            int4 v[UNROLL];
#pragma unroll
            for (int u = 0; u < UNROLL; u++) {
                const int* p = col + t + (unsigned long long)u * TILE + threadIdx.x * 4;
                v[u] = NT ? ld_nt4(reinterpret_cast<const int4*>(p)) : ld(p, false);
            }
#pragma unroll
            for (int u = 0; u < UNROLL; u++) eat(v[u]);
        }
        for (; t < end; t += TILE) {
            unsigned long long r = t + threadIdx.x * 4;
            if (r + 3 < end) eat(ld(col + r, false));
        }
    } else {
        const unsigned long long span = (unsigned long long)gridDim.x * TILE * UNROLL;
        unsigned long long t = (unsigned long long)blockIdx.x * TILE * UNROLL;
        for (; t + (unsigned long long)UNROLL * TILE <= n; t += span) {
            int4 v[UNROLL];
#pragma unroll
            for (int u = 0; u < UNROLL; u++) {
                const int* p = col + t + (unsigned long long)u * TILE + threadIdx.x * 4;
                v[u] = NT ? ld_nt4(reinterpret_cast<const int4*>(p)) : ld(p, false);
            }
#pragma unroll
            for (int u = 0; u < UNROLL; u++) eat(v[u]);
        }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        cnt += __shfl_xor(cnt, off, 64);
        sum += __shfl_xor(sum, off, 64);
    }
    __shared__ unsigned long long sc[TPB / 64];
    __shared__ long long ss[TPB / 64];
    if ((threadIdx.x & 63) == 0) {
        sc[threadIdx.x >> 6] = cnt;
        ss[threadIdx.x >> 6] = sum;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long c = 0;
        long long s = 0;
        for (int w = 0; w < TPB / 64; w++) {
            c += sc[w];
            s += ss[w];
        }
        part[blockIdx.x] = Partial{c, s, mn, mx, 0};
    }
}

// buffer_load_dwordx4 with explicit aux (cache policy) bits; per-block descriptor at the chunk base
template <int TPB, int UNROLL, int AUX>
__global__ __launch_bounds__(TPB) void k_buf(const int* __restrict__ col, unsigned long long n,
                                             unsigned long long rpb, unsigned lo, unsigned wm1,
                                             Partial* __restrict__ part) {
    constexpr int TILE = TPB * 4;
    const unsigned long long start = (unsigned long long)blockIdx.x * rpb;
    unsigned long long end = min(start + rpb, n);
    const unsigned bytes = (unsigned)((end - start) * 4);
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)(col + start), 0, bytes, 0x00020000);
    unsigned cnt = 0;
    long long sum = 0;
    unsigned len = (unsigned)(end - start);
    unsigned t = 0;
    for (; t + UNROLL * TILE <= len; t += UNROLL * TILE) {
        v4i v[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; u++)
            v[u] = __builtin_bit_cast(v4i, __builtin_amdgcn_raw_buffer_load_b128(rs, (t + u * TILE + threadIdx.x * 4) * 4, 0, AUX));
#pragma unroll
        for (int u = 0; u < UNROLL; u++) {
            bool p0 = ((unsigned)v[u].x - lo) <= wm1, p1 = ((unsigned)v[u].y - lo) <= wm1,
                 p2 = ((unsigned)v[u].z - lo) <= wm1, p3 = ((unsigned)v[u].w - lo) <= wm1;
            cnt += p0 + p1 + p2 + p3;
            sum += (long long)(p0 ? v[u].x : 0) + (long long)(p1 ? v[u].y : 0) +
                   (long long)(p2 ? v[u].z : 0) + (long long)(p3 ? v[u].w : 0);
        }
    }
    for (; t < len; t += TILE) {
        unsigned r = t + threadIdx.x * 4;
        if (r + 3 < len) {
            v4i w = __builtin_bit_cast(v4i, __builtin_amdgcn_raw_buffer_load_b128(rs, r * 4, 0, AUX));
            bool p0 = ((unsigned)w.x - lo) <= wm1, p1 = ((unsigned)w.y - lo) <= wm1,
                 p2 = ((unsigned)w.z - lo) <= wm1, p3 = ((unsigned)w.w - lo) <= wm1;
            cnt += p0 + p1 + p2 + p3;
            sum += (long long)(p0 ? w.x : 0) + (long long)(p1 ? w.y : 0) + (long long)(p2 ? w.z : 0) + (long long)(p3 ? w.w : 0);
        }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        cnt += __shfl_xor(cnt, off, 64);
        sum += __shfl_xor(sum, off, 64);
    }
    if ((threadIdx.x & 63) == 0) atomicAdd(&part[blockIdx.x].count, (unsigned long long)cnt);
}

template <int TPB, int UNROLL, int AUX>
void launch_buf(const int* col, unsigned long long n, unsigned lo, unsigned wm1, Partial* part,
                hipStream_t st, int blocks) {
    constexpr int TILE = TPB * 4;
    unsigned long long tiles = (n + TILE - 1) / TILE;
    unsigned long long tpb = (tiles + blocks - 1) / blocks;
    unsigned long long rpb = tpb * TILE;
    unsigned g = (unsigned)((n + rpb - 1) / rpb);
    hipLaunchKernelGGL((k_buf<TPB, UNROLL, AUX>), dim3(g), dim3(TPB), 0, st, col, n, rpb, lo, wm1, part);
}

// mask-pass variants: STORE 0 = no mask store, 1 = transpose only (kept live), 2 = transpose + store
template <int STORE>
__global__ __launch_bounds__(256, 8) void k_maskv(const int* __restrict__ col, unsigned long long n,
                                                  unsigned long long rpb, unsigned lo, unsigned wm1,
                                                  Partial* __restrict__ part, unsigned long long* __restrict__ masks) {
    const unsigned long long start = (unsigned long long)blockIdx.x * rpb;
    unsigned long long end = min(start + rpb, n);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    unsigned cnt = 0;
    unsigned long long acc = 0;
    unsigned long long pending = 0, pat = ~0ull;
    __shared__ unsigned long long sbuf[(STORE == 7 || STORE == 8) ? 16 * 128 : 1];
    int nbuf = 0;
    unsigned long long fbase = 0;
    for (unsigned long long t = start; t + 8192 <= end; t += 8192) {
        int4 v[8];
#pragma unroll
        for (int u = 0; u < 8; u++) v[u] = ld_nt4(reinterpret_cast<const int4*>(col + t + u * 1024 + tid * 4));
        if (STORE == 3) {
            asm volatile("" ::: "memory");  // loads of this iteration are issued before the store
            if (pat != ~0ull && lane < 32) masks[pat + lane] = pending;
        }
        unsigned pbits = 0;
#pragma unroll
        for (int u = 0; u < 8; u++) {
            unsigned b = (((unsigned)v[u].x - lo) <= wm1 ? 1u : 0u) | (((unsigned)v[u].y - lo) <= wm1 ? 2u : 0u) |
                         (((unsigned)v[u].z - lo) <= wm1 ? 4u : 0u) | (((unsigned)v[u].w - lo) <= wm1 ? 8u : 0u);
            pbits |= b << (4 * u);
        }
        cnt += __popc(pbits);
        if (STORE >= 1) {
            unsigned long long w = 0;
#pragma unroll
            for (int k = 0; k < 32; k++) {
                unsigned long long m = __ballot((pbits >> k) & 1u);
                w = lane == k ? m : w;
            }
            if (STORE == 2) {
                if (lane < 32) masks[((t >> 13) * 4 + wave) * 32 + lane] = w;
            } else if (STORE == 4) {
                if (lane < 32) __builtin_nontemporal_store(w, &masks[((t >> 13) * 4 + wave) * 32 + lane]);
            } else if (STORE == 5) {
                if (lane < 32) __hip_atomic_store(&masks[((t >> 13) * 4 + wave) * 32 + lane], w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else if (STORE == 6) {
                // 16 lanes x 16 B
                unsigned long long w2 = __shfl(w, (lane * 2 + 1) & 63, 64);
                unsigned long long w1 = __shfl(w, (lane * 2) & 63, 64);
                if (lane < 16) {
                    ulonglong2 q; q.x = w1; q.y = w2;
                    reinterpret_cast<ulonglong2*>(&masks[((t >> 13) * 4 + wave) * 32])[lane] = q;
                }
            } else if (STORE == 3) {
                pending = w;
                pat = ((t >> 13) * 4 + wave) * 32;
            } else if (STORE == 7 || STORE == 8) {
                // LDS-buffered: 16 super-tiles (16 KB contiguous) per flush, 16 B per lane
                if (nbuf == 0) fbase = (t >> 13) * 128;
                if (lane < 32) sbuf[nbuf * 128 + wave * 32 + lane] = w;
                if (++nbuf == 16) {
                    __syncthreads();
                    for (int k = tid; k < 16 * 64; k += 256) {
                        ulonglong2 q;
                        q.x = sbuf[2 * k];
                        q.y = sbuf[2 * k + 1];
                        ulonglong2* d = reinterpret_cast<ulonglong2*>(masks + fbase) + k;
                        if (STORE == 8) {
                            typedef unsigned long long v2u __attribute__((ext_vector_type(2)));
                            v2u qq = {q.x, q.y};
                            __builtin_nontemporal_store(qq, reinterpret_cast<v2u*>(d));
                        } else {
                            *d = q;
                        }
                    }
                    __syncthreads();
                    nbuf = 0;
                }
            } else {
                acc ^= w;
            }
        }
    }
    if (STORE == 3 && pat != ~0ull && lane < 32) masks[pat + lane] = pending;
    if ((STORE == 7 || STORE == 8) && nbuf) {
        __syncthreads();
        for (int k = tid; k < nbuf * 64; k += 256)
            reinterpret_cast<ulonglong2*>(masks + fbase)[k] = make_ulonglong2(sbuf[2 * k], sbuf[2 * k + 1]);
    }
    if (threadIdx.x == 0) part[blockIdx.x].count = cnt + (unsigned)acc;
}

// v_writelane via the LLVM intrinsic (no clang builtin in this toolchain); the backend
// inserts the hazard waits an inline-asm writelane would not.
__device__ int mq_writelane(int src, int lane, int old) __asm("llvm.amdgcn.writelane.i32");

// direct-ballot mask pass: the row compares ARE the ballots; each goes straight into
// its record lane with v_writelane (no bit packing, no 32-ballot transpose).
// GRID 0: contiguous chunk per block; GRID 1: grid-stride super-tiles.
template <int GRID>
__global__ __launch_bounds__(256, 8) void k_maskw(const int* __restrict__ col, unsigned long long n,
                                                  unsigned long long rpb, unsigned lo, unsigned wm1,
                                                  Partial* __restrict__ part,
                                                  unsigned long long* __restrict__ masks) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    unsigned long long cnt = 0;
    unsigned long long s0, s1, step;
    if (GRID) {
        s0 = blockIdx.x;
        s1 = n / 8192;
        step = gridDim.x;
    } else {
        const unsigned long long start = (unsigned long long)blockIdx.x * rpb;
        s0 = start / 8192;
        s1 = min(start + rpb, n) / 8192;
        step = 1;
    }
    for (unsigned long long st = s0; st < s1; st += step) {
        const unsigned long long t = st * 8192;
        int4 v[8];
#pragma unroll
        for (int u = 0; u < 8; u++) v[u] = ld_nt4(reinterpret_cast<const int4*>(col + t + u * 1024 + tid * 4));
        int wlo = 0, whi = 0;
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const unsigned long long m0 = __ballot(((unsigned)v[u].x - lo) <= wm1);
            const unsigned long long m1 = __ballot(((unsigned)v[u].y - lo) <= wm1);
            const unsigned long long m2 = __ballot(((unsigned)v[u].z - lo) <= wm1);
            const unsigned long long m3 = __ballot(((unsigned)v[u].w - lo) <= wm1);
            cnt += __popcll(m0) + __popcll(m1) + __popcll(m2) + __popcll(m3);
            wlo = mq_writelane((int)m0, 4 * u + 0, wlo);
            whi = mq_writelane((int)(m0 >> 32), 4 * u + 0, whi);
            wlo = mq_writelane((int)m1, 4 * u + 1, wlo);
            whi = mq_writelane((int)(m1 >> 32), 4 * u + 1, whi);
            wlo = mq_writelane((int)m2, 4 * u + 2, wlo);
            whi = mq_writelane((int)(m2 >> 32), 4 * u + 2, whi);
            wlo = mq_writelane((int)m3, 4 * u + 3, wlo);
            whi = mq_writelane((int)(m3 >> 32), 4 * u + 3, whi);
        }
        const unsigned long long w = (unsigned long long)(unsigned)wlo | ((unsigned long long)(unsigned)whi << 32);
        if (lane < 32) masks[(st * 4 + wave) * 32 + lane] = w;
    }
    if (threadIdx.x == 0) part[blockIdx.x].count = cnt;
}

template <int GRID>
void launch_maskw(const int* col, unsigned long long n, unsigned lo, unsigned wm1, Partial* part,
                  hipStream_t st, int blocks) {
    static unsigned long long* masks = nullptr;
    if (!masks) hipMalloc(&masks, n / 8 + 65536);
    unsigned long long tiles = (n + 8191) / 8192;
    unsigned long long tpb = (tiles + blocks - 1) / blocks;
    unsigned long long rpb = tpb * 8192;
    unsigned g = GRID ? (unsigned)blocks : (unsigned)((n + rpb - 1) / rpb);
    hipLaunchKernelGGL((k_maskw<GRID>), dim3(g), dim3(256), 0, st, col, n, rpb, lo, wm1, part, masks);
}

// grid-stride mask pass: super-tile s handled by block s % G; records indexed by s (contiguous over the grid)
template <int STORE>
__global__ __launch_bounds__(256, 8) void k_maskg(const int* __restrict__ col, unsigned long long n,
                                                  unsigned lo, unsigned wm1, Partial* __restrict__ part,
                                                  unsigned long long* __restrict__ masks, unsigned* __restrict__ counts) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    unsigned long long nst = n / 8192;
    for (unsigned long long st = blockIdx.x; st < nst; st += gridDim.x) {
        unsigned long long t = st * 8192;
        int4 v[8];
#pragma unroll
        for (int u = 0; u < 8; u++) v[u] = ld_nt4(reinterpret_cast<const int4*>(col + t + u * 1024 + tid * 4));
        unsigned pbits = 0;
#pragma unroll
        for (int u = 0; u < 8; u++) {
            unsigned b = (((unsigned)v[u].x - lo) <= wm1 ? 1u : 0u) | (((unsigned)v[u].y - lo) <= wm1 ? 2u : 0u) |
                         (((unsigned)v[u].z - lo) <= wm1 ? 4u : 0u) | (((unsigned)v[u].w - lo) <= wm1 ? 8u : 0u);
            pbits |= b << (4 * u);
        }
        unsigned long long w = 0;
        unsigned c = 0;
#pragma unroll
        for (int k = 0; k < 32; k++) {
            unsigned long long m = __ballot((pbits >> k) & 1u);
            c += __popcll(m);
            w = lane == k ? m : w;
        }
        if (lane < 32) masks[(st * 4 + wave) * 32 + lane] = w;
        if (STORE == 1 && lane == 0) counts[st * 4 + wave] = c;
    }
}

template <int STORE>
void launch_maskg(const int* col, unsigned long long n, unsigned lo, unsigned wm1, Partial* part,
                  hipStream_t st, int blocks) {
    static unsigned long long* masks = nullptr;
    static unsigned* counts = nullptr;
    if (!masks) { hipMalloc(&masks, n / 8 + 65536); hipMalloc(&counts, n / 512 + 4096); }
    hipLaunchKernelGGL((k_maskg<STORE>), dim3(blocks), dim3(256), 0, st, col, n, lo, wm1, part, masks, counts);
}

template <int STORE>
void launch_mask(const int* col, unsigned long long n, unsigned lo, unsigned wm1, Partial* part,
                 hipStream_t st, int blocks) {
    static unsigned long long* masks = nullptr;
    if (!masks) hipMalloc(&masks, n / 8 + 65536);
    unsigned long long tiles = (n + 8191) / 8192;
    unsigned long long tpb = (tiles + blocks - 1) / blocks;
    unsigned long long rpb = tpb * 8192;
    unsigned g = (unsigned)((n + rpb - 1) / rpb);
    hipLaunchKernelGGL((k_maskv<STORE>), dim3(g), dim3(256), 0, st, col, n, rpb, lo, wm1, part, masks);
}

__global__ void k_gen(int* out, unsigned long long n) {
    for (unsigned long long i = (unsigned long long)blockIdx.x * 256 + threadIdx.x; i < n;
         i += (unsigned long long)gridDim.x * 256) {
        unsigned long long x = 42ull * 0x100000001B3ull + i + 0x9E3779B97F4A7C15ull;
        x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
        x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
        x ^= x >> 31;
        out[i] = (int)(x % n);
    }
}

struct Var {
    const char* name;
    void (*launch)(const int*, unsigned long long, unsigned, unsigned, Partial*, hipStream_t, int);
    int bpc;  // blocks per CU
};

template <int TPB, int UNROLL, bool NT, int MODE, bool MM>
void launch(const int* col, unsigned long long n, unsigned lo, unsigned wm1, Partial* part,
            hipStream_t st, int blocks) {
    constexpr int TILE = TPB * 4;
    unsigned long long tiles = (n + TILE - 1) / TILE;
    unsigned long long tpb = (tiles + blocks - 1) / blocks;
    unsigned long long rpb = tpb * TILE;
    unsigned g = (unsigned)((n + rpb - 1) / rpb);
    if (MODE == 1) g = blocks;
    hipLaunchKernelGGL((k_var<TPB, UNROLL, NT, MODE, MM>), dim3(g), dim3(TPB), 0, st, col, n, rpb,
                       lo, wm1, part);
}

int main(int argc, char** argv) {
    unsigned long long n = argc > 1 ? strtoull(argv[1], 0, 10) : 1000000000ull;
    int rounds = argc > 2 ? atoi(argv[2]) : 7;
    int cus;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    int* col;
    Partial* part;
    CK(hipMalloc(&col, n * 4));
    CK(hipMalloc(&part, 65536 * sizeof(Partial)));
    hipLaunchKernelGGL(k_gen, dim3(cus * 8), dim3(256), 0, 0, col, n);
    CK(hipDeviceSynchronize());
    unsigned lo = (unsigned)(n / 4), wm1 = (unsigned)(n / 100) - 1;
    std::vector<Var> vars = {
        {"ref t256 u8 chunk nt 8/CU", launch<256, 8, true, 0, false>, 8},
        {"mask: bits only", launch_mask<0>, 8},
        {"mask: + transpose", launch_mask<1>, 8},
        {"mask: + transpose + store", launch_mask<2>, 8},
        {"mask: + transpose + deferred store", launch_mask<3>, 8},
        {"mask: writelane chunk + store", launch_maskw<0>, 8},
        {"mask: writelane grid-stride + store", launch_maskw<1>, 8},
        {"mask: LDS-buffered 16KB flush", launch_mask<7>, 8},
        {"mask: LDS-buffered 16KB flush nt", launch_mask<8>, 8},
        {"mask: + transpose + store (again)", launch_mask<2>, 8},
        {"ref t256 u8 chunk nt 8/CU (again)", launch<256, 8, true, 0, false>, 8},
        {"mask grid-stride + store", launch_maskg<0>, 8},
        {"mask grid-stride + store + counts", launch_maskg<1>, 8},
    };
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    std::vector<std::vector<float>> ms(vars.size());
    const int reps = 10;
    for (int r = 0; r < rounds; r++) {
        for (size_t v = 0; v < vars.size(); v++) {
            vars[v].launch(col, n, lo, wm1, part, 0, cus * vars[v].bpc);  // warm
            CK(hipEventRecord(a, 0));
            for (int i = 0; i < reps; i++) vars[v].launch(col, n, lo, wm1, part, 0, cus * vars[v].bpc);
            CK(hipEventRecord(b, 0));
            CK(hipEventSynchronize(b));
            float t;
            CK(hipEventElapsedTime(&t, a, b));
            ms[v].push_back(t / reps);
        }
    }
    CK(hipGetLastError());
    printf("n=%llu rounds=%d reps=%d CUs=%d\n", n, rounds, reps, cus);
    for (size_t v = 0; v < vars.size(); v++) {
        std::sort(ms[v].begin(), ms[v].end());
        float med = ms[v][ms[v].size() / 2], best = ms[v][0];
        printf("%-32s median %.4f ms  %.1f GB/s   best %.4f ms  %.1f GB/s\n", vars[v].name, med,
               4.0 * n / (med * 1e-3) / 1e9, best, 4.0 * n / (best * 1e-3) / 1e9);
    }
    return 0;
}
