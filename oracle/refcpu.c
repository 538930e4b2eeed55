/*
 * refcpu.c — CPU restatement of siyaoL1/Analytical-Database's select / fetch /
 * aggregate / join hot path. ORACLE AND CPU BASELINE ONLY: this file is test
 * infrastructure (tests/, __graft_entry__.smoke(), bench.py cpu_baseline). It is
 * never linked into libmq and the product path never calls it.
 *
 * Each function cites the reference loop it restates (paths relative to the
 * reference repository root). Semantics kept exactly:
 *   - select is half-open  low <= v < high, NULL bound = unbounded
 *     (src/query.c:97-127), positions are int32 in ascending row order;
 *   - sum accumulates int32 into a 64-bit `long` (src/query.c:325-354);
 *   - avg = (double)int64_sum / (double)n (src/query.c:306-323);
 *   - hash_join emits (build_pos, probe_pos) in probe-major, build-insertion
 *     order (src/query.c:652-696 over src/multimap.c:41-102).
 * The restatement is pinned against oracle/_ref/libref.so (the reference's own
 * query.c/multimap.c compiled by oracle/Makefile) by tests/test_oracle.py.
 */
#define _GNU_SOURCE
#include "refcpu.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ */
/* synthetic data: SURVEY.md §8(c)                                     */
/* ------------------------------------------------------------------ */

uint64_t rc_sm64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

uint32_t rc_mix31(uint32_t x) {
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

typedef struct {
    int32_t* out;
    size_t lo, hi;
    uint64_t base, modulus;
} gen_arg;

static void* gen_worker(void* p) {
    gen_arg* a = (gen_arg*)p;
    for (size_t i = a->lo; i < a->hi; i++)
        a->out[i] = (int32_t)(rc_sm64(a->base + (uint64_t)i) % a->modulus);
    return NULL;
}

void rc_gen_uniform(int32_t* out, size_t n, uint64_t seed, uint64_t modulus, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    gen_arg args[256];
    uint64_t base = seed * 0x100000001B3ull;
    size_t chunk = (n + (size_t)nthreads - 1) / (size_t)nthreads;
    for (int t = 0; t < nthreads; t++) {
        size_t lo = (size_t)t * chunk, hi = lo + chunk;
        if (lo > n) lo = n;
        if (hi > n) hi = n;
        args[t] = (gen_arg){out, lo, hi, base, modulus};
        pthread_create(&th[t], NULL, gen_worker, &args[t]);
    }
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
}

void rc_gen_join_build(int32_t* out, size_t n) {
    for (size_t i = 0; i < n; i++) out[i] = (int32_t)rc_mix31((uint32_t)i);
}

void rc_gen_join_probe(int32_t* out, size_t n) {
    uint64_t mask = 2 * (uint64_t)n - 1;
    for (size_t j = 0; j < n; j++)
        out[j] = (int32_t)rc_mix31((uint32_t)(rc_sm64((7ull << 40) | (uint64_t)j) & mask));
}

/* config 5, many-to-many variant: every build key twice,
 * a[i] = mix31(i mod n/2) (rows i and i + n/2, spread over the build order), probe
 * keys mix31(sm64((7 << 40) | j) mod n): about half the probes hit a key, each with
 * two matches, so M ~ n; the reference multimap's probing stays linear. */
void rc_gen_join_build_dup(int32_t* out, size_t n) {
    const size_t h = n / 2 ? n / 2 : 1;
    for (size_t i = 0; i < n; i++) out[i] = (int32_t)rc_mix31((uint32_t)(i % h));
}

void rc_gen_join_probe_dup(int32_t* out, size_t n) {
    uint64_t mask = (uint64_t)n - 1;  /* n a power of two */
    for (size_t j = 0; j < n; j++)
        out[j] = (int32_t)rc_mix31((uint32_t)(rc_sm64((7ull << 40) | (uint64_t)j) & mask));
}

void rc_iota(int32_t* out, size_t n) {
    for (size_t i = 0; i < n; i++) out[i] = (int32_t)i;
}

uint64_t rc_fnv1a64(const void* p, size_t bytes) {
    const unsigned char* b = (const unsigned char*)p;
    uint64_t h = 0xcbf29ce484222325ull;
    for (size_t i = 0; i < bytes; i++) {
        h ^= b[i];
        h *= 0x100000001B3ull;
    }
    return h;
}

uint64_t rc_fnv1a64_pairs(const int32_t* a, const int32_t* b, size_t m) {
    uint64_t h = 0xcbf29ce484222325ull;
    for (size_t i = 0; i < m; i++) {
        int32_t pr[2] = {a[i], b[i]};
        const unsigned char* c = (const unsigned char*)pr;
        for (int k = 0; k < 8; k++) {
            h ^= c[k];
            h *= 0x100000001B3ull;
        }
    }
    return h;
}

/* ------------------------------------------------------------------ */
/* select                                                              */
/* ------------------------------------------------------------------ */

/* src/query.c:92-137 select_column_scan: four bound cases, positions in row order. */
size_t rc_select_scan(const int32_t* data, size_t n, const int32_t* low, const int32_t* high,
                      int32_t* pos_out) {
    size_t k = 0;
    if (low && high) {                               /* query.c:97-104 */
        int32_t lo = *low, hi = *high;
        for (size_t i = 0; i < n; i++)
            if (data[i] >= lo && data[i] < hi) pos_out[k++] = (int32_t)i;
    } else if (!low && high) {                       /* query.c:105-112 */
        int32_t hi = *high;
        for (size_t i = 0; i < n; i++)
            if (data[i] < hi) pos_out[k++] = (int32_t)i;
    } else if (low && !high) {                       /* query.c:113-120 */
        int32_t lo = *low;
        for (size_t i = 0; i < n; i++)
            if (data[i] >= lo) pos_out[k++] = (int32_t)i;
    } else {                                         /* query.c:121-127 */
        for (size_t i = 0; i < n; i++) pos_out[i] = (int32_t)i;
        k = n;
    }
    return k;
}

typedef struct {
    const int32_t* data;
    size_t lo, hi;
    const int32_t *low, *high;
    int32_t* buf;
    size_t k;
} scan_arg;

static void* scan_worker(void* p) {
    scan_arg* a = (scan_arg*)p;
    size_t k = rc_select_scan(a->data + a->lo, a->hi - a->lo, a->low, a->high, a->buf);
    for (size_t i = 0; i < k; i++) a->buf[i] += (int32_t)a->lo;
    a->k = k;
    return NULL;
}

/* Row-balanced nthreads split of select_column_scan; per-thread lists are
 * concatenated in thread order, as shared_select does (query.c:563-574). */
size_t rc_select_scan_mt(const int32_t* data, size_t n, const int32_t* low, const int32_t* high,
                         int32_t* pos_out, int nthreads) {
    if (nthreads <= 1) return rc_select_scan(data, n, low, high, pos_out);
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    scan_arg args[256];
    size_t chunk = (n + (size_t)nthreads - 1) / (size_t)nthreads;
    for (int t = 0; t < nthreads; t++) {
        size_t lo = (size_t)t * chunk, hi = lo + chunk;
        if (lo > n) lo = n;
        if (hi > n) hi = n;
        /* thread t writes into pos_out+lo (its rows' own slice), compacted below */
        args[t] = (scan_arg){data, lo, hi, low, high, pos_out + lo, 0};
        pthread_create(&th[t], NULL, scan_worker, &args[t]);
    }
    size_t k = 0;
    for (int t = 0; t < nthreads; t++) {
        pthread_join(th[t], NULL);
        if (pos_out + k != args[t].buf) memmove(pos_out + k, args[t].buf, args[t].k * sizeof(int32_t));
        k += args[t].k;
    }
    return k;
}

/* src/query.c:38-86 select_result: filter fetched values, emit the matching prior positions. */
size_t rc_select_result(const int32_t* vals, const int32_t* prev_pos, size_t n,
                        const int32_t* low, const int32_t* high, int32_t* pos_out) {
    size_t k = 0;
    if (low && high) {                               /* query.c:45-52 */
        int32_t lo = *low, hi = *high;
        for (size_t i = 0; i < n; i++)
            if (vals[i] >= lo && vals[i] < hi) pos_out[k++] = prev_pos[i];
    } else if (!low && high) {                       /* query.c:53-60 */
        int32_t hi = *high;
        for (size_t i = 0; i < n; i++)
            if (vals[i] < hi) pos_out[k++] = prev_pos[i];
    } else if (low && !high) {                       /* query.c:61-68 */
        int32_t lo = *low;
        for (size_t i = 0; i < n; i++)
            if (vals[i] >= lo) pos_out[k++] = prev_pos[i];
    } else {                                         /* query.c:69-75 */
        for (size_t i = 0; i < n; i++) pos_out[i] = prev_pos[i];
        k = n;
    }
    return k;
}

/* ------------------------------------------------------------------ */
/* fetch / aggregates / elementwise                                    */
/* ------------------------------------------------------------------ */

/* src/query.c:223-243 fetch_column: values[i] = column->data[position[i]] */
void rc_fetch(const int32_t* col, const int32_t* pos, size_t k, int32_t* out) {
    for (size_t i = 0; i < k; i++) out[i] = col[pos[i]];
}

/* src/query.c:325-354 sum: `long` (int64) accumulator over int32 */
int64_t rc_sum(const int32_t* v, size_t n) {
    int64_t s = 0;
    for (size_t i = 0; i < n; i++) s += v[i];
    return s;
}

/* src/query.c:306-323 average: one double division of the int64 sum (n=0 -> NaN) */
double rc_avg(const int32_t* v, size_t n) {
    int64_t s = rc_sum(v, n);
    return (double)s / (double)n;
}

/* src/query.c:392-415 min. The reference seeds from payload[0] even when n == 0
 * (reads uninitialised memory); the restatement returns INT32_MAX for n == 0. */
int32_t rc_min(const int32_t* v, size_t n) {
    if (n == 0) return INT32_MAX;
    int32_t m = v[0];
    for (size_t i = 0; i < n; i++)
        if (m > v[i]) m = v[i];
    return m;
}

/* src/query.c:417-437 max (n == 0: INT32_MIN, see rc_min) */
int32_t rc_max(const int32_t* v, size_t n) {
    if (n == 0) return INT32_MIN;
    int32_t m = v[0];
    for (size_t i = 0; i < n; i++)
        if (m < v[i]) m = v[i];
    return m;
}

/* src/query.c:356-372 add (two's-complement wrap; the reference's signed overflow is UB) */
void rc_add(const int32_t* a, const int32_t* b, size_t n, int32_t* out) {
    for (size_t i = 0; i < n; i++) out[i] = (int32_t)((uint32_t)a[i] + (uint32_t)b[i]);
}

/* src/query.c:374-390 sub (wrap, as rc_add) */
void rc_sub(const int32_t* a, const int32_t* b, size_t n, int32_t* out) {
    for (size_t i = 0; i < n; i++) out[i] = (int32_t)((uint32_t)a[i] - (uint32_t)b[i]);
}

typedef struct {
    const int32_t* data;
    size_t lo, hi;
    int has_lo, has_hi;
    int32_t low, high;
    uint64_t count;
    int64_t sum;
} cs_arg;

static void* cs_worker(void* p) {
    cs_arg* a = (cs_arg*)p;
    uint64_t c = 0;
    int64_t s = 0;
    for (size_t i = a->lo; i < a->hi; i++) {
        int32_t v = a->data[i];
        int ok = (!a->has_lo || v >= a->low) && (!a->has_hi || v < a->high);
        if (ok) {
            c++;
            s += v;
        }
    }
    a->count = c;
    a->sum = s;
    return NULL;
}

/* The composition select_column_scan -> fetch_column -> sum over the same
 * column (query.c:92-137, 223-243, 325-354) collapsed into one pass. */
void rc_select_count_sum(const int32_t* data, size_t n, const int32_t* low, const int32_t* high,
                         uint64_t* count, int64_t* sum, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    cs_arg args[256];
    size_t chunk = (n + (size_t)nthreads - 1) / (size_t)nthreads;
    for (int t = 0; t < nthreads; t++) {
        size_t lo = (size_t)t * chunk, hi = lo + chunk;
        if (lo > n) lo = n;
        if (hi > n) hi = n;
        args[t] = (cs_arg){data, lo, hi, low != NULL, high != NULL, low ? *low : 0, high ? *high : 0, 0, 0};
        if (nthreads == 1) cs_worker(&args[t]);
        else pthread_create(&th[t], NULL, cs_worker, &args[t]);
    }
    uint64_t c = 0;
    int64_t s = 0;
    for (int t = 0; t < nthreads; t++) {
        if (nthreads > 1) pthread_join(th[t], NULL);
        c += args[t].count;
        s += args[t].sum;
    }
    *count = c;
    *sum = s;
}

/* ------------------------------------------------------------------ */
/* shared_select (batched scan)                                        */
/* ------------------------------------------------------------------ */

typedef struct {
    const int32_t* data;
    size_t lo, hi;
    const int32_t *lows, *highs;
    int q;
    int32_t** bufs;  /* q buffers of (hi-lo) entries */
    size_t* ks;
} ss_arg;

/* src/query.c:450-494 select_task: row-major loop, q predicates per value
 * (has_low/has_high are ignored there; lows/highs are used as given). */
static void* ss_worker(void* p) {
    ss_arg* a = (ss_arg*)p;
    for (int qq = 0; qq < a->q; qq++) a->ks[qq] = 0;
    for (size_t row = a->lo; row < a->hi; row++) {
        int32_t v = a->data[row];
        for (int qq = 0; qq < a->q; qq++)
            if (v >= a->lows[qq] && v < a->highs[qq]) a->bufs[qq][a->ks[qq]++] = (int32_t)row;
    }
    return NULL;
}

/* src/query.c:496-583 shared_select. split=1 reproduces the value-range split
 * of query.c:506-522 (3 tasks of (max-min)/3 rows, the last to row_count);
 * split=0 uses nthreads row-balanced tasks. Results concatenate in task
 * order (query.c:563-574), i.e. ascending rows. Returns 0, or -1 on an
 * invalid value-range split (the reference reads past the column there). */
int rc_shared_select(const int32_t* data, size_t n, const int32_t* lows, const int32_t* highs,
                     int q, int32_t** pos_out, size_t* counts, int nthreads, int split,
                     int32_t col_min, int32_t col_max) {
    size_t starts[257], ends[257];
    int T;
    if (split == 1) {
        T = 3;
        size_t task = (size_t)((col_max - col_min) / 3);
        size_t cur = 0;
        for (int t = 0; t < T; t++) {
            starts[t] = cur;
            cur += task;
            ends[t] = (t == T - 1) ? n : cur;
            if (starts[t] > n || ends[t] > n || ends[t] < starts[t]) return -1;
        }
    } else {
        T = nthreads < 1 ? 1 : (nthreads > 256 ? 256 : nthreads);
        size_t chunk = (n + (size_t)T - 1) / (size_t)T;
        for (int t = 0; t < T; t++) {
            starts[t] = (size_t)t * chunk;
            ends[t] = starts[t] + chunk;
            if (starts[t] > n) starts[t] = n;
            if (ends[t] > n) ends[t] = n;
        }
    }
    pthread_t th[256];
    ss_arg args[256];
    int32_t** bufs = (int32_t**)malloc(sizeof(int32_t*) * (size_t)T * (size_t)q);
    size_t* ks = (size_t*)calloc((size_t)T * (size_t)q, sizeof(size_t));
    for (int t = 0; t < T; t++) {
        for (int qq = 0; qq < q; qq++)
            bufs[t * q + qq] = (int32_t*)malloc(sizeof(int32_t) * (ends[t] - starts[t] + 1));
        args[t] = (ss_arg){data, starts[t], ends[t], lows, highs, q, bufs + t * q, ks + t * q};
        pthread_create(&th[t], NULL, ss_worker, &args[t]);
    }
    for (int t = 0; t < T; t++) pthread_join(th[t], NULL);
    for (int qq = 0; qq < q; qq++) {
        size_t cur = 0;
        for (int t = 0; t < T; t++) {
            memcpy(pos_out[qq] + cur, bufs[t * q + qq], ks[t * q + qq] * sizeof(int32_t));
            cur += ks[t * q + qq];
        }
        counts[qq] = cur;
    }
    for (int i = 0; i < T * q; i++) free(bufs[i]);
    free(bufs);
    free(ks);
    return 0;
}

/* ------------------------------------------------------------------ */
/* joins                                                               */
/* ------------------------------------------------------------------ */

/* src/multimap.c:15-27 prime(): trial division; n < 2 counts as prime there. */
static int is_prime(int32_t n) {
    if (n < 2) return 1;
    for (int64_t i = 2; i * i <= n; i++)
        if (n % i == 0) return 0;
    return 1;
}

/* src/multimap.c:30-38 get_proper_size: smallest prime >= (int)(1.3 * n) */
int32_t rc_multimap_size(int32_t tuple_num) {
    int32_t s = (int32_t)(1.3 * tuple_num);
    while (!is_prime(s)) s++;
    return s;
}

/* src/multimap.c:60-63 hash = key % size; the reference's negative index for a
 * negative key is UB, the restatement wraps it into [0, size). */
static inline int32_t mm_hash(int32_t key, int32_t size) {
    int32_t h = key % size;
    return h < 0 ? h + size : h;
}

/* src/query.c:652-696 hash_join over src/multimap.c:41-102. The multimap's
 * per-slot growable lists are restated as one CSR array filled in insertion
 * order, which preserves lookup_multimap's value order exactly. */
size_t rc_hash_join(const int32_t* c1, const int32_t* p1, size_t n1,
                    const int32_t* c2, const int32_t* p2, size_t n2,
                    int32_t* out1, int32_t* out2, size_t cap) {
    if (n1 == 0 || n2 == 0) return 0;
    int32_t size = rc_multimap_size((int32_t)n1);
    int32_t* keys = (int32_t*)malloc(sizeof(int32_t) * (size_t)size);
    uint32_t* cnt = (uint32_t*)calloc((size_t)size, sizeof(uint32_t));
    int32_t* slot_of = (int32_t*)malloc(sizeof(int32_t) * n1);
    for (size_t i = 0; i < n1; i++) {                 /* insert_multimap, multimap.c:74-89 */
        int32_t h = mm_hash(c1[i], size);
        while (cnt[h] != 0 && keys[h] != c1[i]) h = (h + 1) % size;  /* find_index :65-71 */
        keys[h] = c1[i];
        cnt[h]++;
        slot_of[i] = h;
    }
    uint32_t* off = (uint32_t*)malloc(sizeof(uint32_t) * ((size_t)size + 1));
    uint32_t acc = 0;
    for (int32_t s = 0; s < size; s++) {
        off[s] = acc;
        acc += cnt[s];
    }
    off[size] = acc;
    int32_t* vals = (int32_t*)malloc(sizeof(int32_t) * n1);
    uint32_t* cur = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)size);
    memcpy(cur, off, sizeof(uint32_t) * (size_t)size);
    for (size_t i = 0; i < n1; i++) vals[cur[slot_of[i]]++] = p1[i];
    free(cur);
    free(slot_of);
    size_t m = 0;
    int overflow = 0;
    for (size_t j = 0; j < n2; j++) {                 /* probe loop, query.c:669-681 */
        int32_t h = mm_hash(c2[j], size);
        /* find_index (multimap.c:65-71) never terminates when every slot is taken
         * and the key is absent (size == n1 for n1 <= 3 distinct keys); the
         * restatement stops after one lap: the key is not in the map. */
        int32_t steps = 0;
        while (cnt[h] != 0 && keys[h] != c2[j] && steps < size) {
            h = (h + 1) % size;
            steps++;
        }
        if (steps == size || keys[h] != c2[j]) continue;
        for (uint32_t e = off[h]; e < off[h] + cnt[h]; e++) {
            if (out1) {
                if (m >= cap) {
                    overflow = 1;
                    break;
                }
                out1[m] = vals[e];
                out2[m] = p2[j];
            }
            m++;
        }
        if (overflow) break;
    }
    free(keys);
    free(cnt);
    free(off);
    free(vals);
    return overflow ? (size_t)-1 : m;
}

/* The same join over `nthreads` host threads (the config-5 host-cores baseline, SURVEY
 * §8(d) "CPU threadpool"; the reference's hash_join is single-threaded). Output
 * identical to rc_hash_join: probe-major, a key's build rows in insertion order.
 *   build: the build rows split by key hash into P partitions (a per-thread histogram
 *   over contiguous row ranges, a prefix in (partition, thread) order, a scatter: every
 *   partition holds its rows in input order); each partition then gets its own
 *   open-addressing CSR multimap (as rc_hash_join's), partitions spread over threads;
 *   probe: contiguous probe ranges per thread, a count pass, a prefix, a write pass. */
#define MJ_P 256
typedef struct {
    const int32_t *c1, *p1, *c2, *p2;
    size_t n1, n2;
    int T;
    size_t (*hist)[MJ_P];     /* [T][P] build rows of thread t's range in partition p */
    int32_t *pk, *pp;          /* build rows partitioned (key, payload) */
    size_t poff[MJ_P + 1];     /* partition starts in pk / pp */
    uint32_t tmask[MJ_P];      /* partition tables: 2^k slots, mask */
    int32_t* tkey[MJ_P];
    uint32_t* tcnt[MJ_P];
    uint32_t* toff[MJ_P];
    int32_t* tval[MJ_P];
    size_t* pcount;            /* per thread: pairs of its probe range */
    int32_t *out1, *out2;
} mj_ctx;
typedef struct {
    mj_ctx* c;
    int t, phase;
} mj_arg;

static inline uint32_t mj_hash(int32_t k) { return rc_mix31((uint32_t)k) ^ ((uint32_t)k * 0x9E3779B1u); }

static void mj_range(size_t n, int T, int t, size_t* lo, size_t* hi) {
    size_t ch = (n + (size_t)T - 1) / (size_t)T;
    *lo = (size_t)t * ch;
    *hi = *lo + ch;
    if (*lo > n) *lo = n;
    if (*hi > n) *hi = n;
}

static void mj_build_part(mj_ctx* c, int p) {
    size_t a = c->poff[p], b = c->poff[p + 1], n = b - a;
    uint32_t slots = 16;
    while (slots < 2 * n) slots <<= 1;
    uint32_t mask = slots - 1;
    int32_t* keys = (int32_t*)malloc(sizeof(int32_t) * slots);
    uint32_t* cnt = (uint32_t*)calloc(slots, sizeof(uint32_t));
    uint32_t* slot_of = (uint32_t*)malloc(sizeof(uint32_t) * (n ? n : 1));
    for (size_t i = 0; i < n; i++) {
        int32_t k = c->pk[a + i];
        uint32_t h = (mj_hash(k) >> 8) & mask;
        while (cnt[h] != 0 && keys[h] != k) h = (h + 1) & mask;
        keys[h] = k;
        cnt[h]++;
        slot_of[i] = h;
    }
    uint32_t* off = (uint32_t*)malloc(sizeof(uint32_t) * (slots + 1));
    uint32_t acc = 0;
    for (uint32_t s = 0; s < slots; s++) {
        off[s] = acc;
        acc += cnt[s];
    }
    off[slots] = acc;
    int32_t* vals = (int32_t*)malloc(sizeof(int32_t) * (n ? n : 1));
    uint32_t* cur = (uint32_t*)malloc(sizeof(uint32_t) * slots);
    memcpy(cur, off, sizeof(uint32_t) * slots);
    for (size_t i = 0; i < n; i++) vals[cur[slot_of[i]]++] = c->pp[a + i];
    free(cur);
    free(slot_of);
    c->tmask[p] = mask;
    c->tkey[p] = keys;
    c->tcnt[p] = cnt;
    c->toff[p] = off;
    c->tval[p] = vals;
}

/* the build rows of key k: *len of them from tval[p] + the returned start */
static inline uint32_t mj_find(const mj_ctx* c, int32_t k, uint32_t* len, int* part) {
    uint32_t hh = mj_hash(k);
    int p = (int)(hh & (MJ_P - 1));
    uint32_t mask = c->tmask[p], h = (hh >> 8) & mask;
    const uint32_t* cnt = c->tcnt[p];
    const int32_t* keys = c->tkey[p];
    while (cnt[h] != 0 && keys[h] != k) h = (h + 1) & mask;
    *part = p;
    *len = cnt[h];
    return c->toff[p][h];
}

static void* mj_worker(void* v) {
    mj_arg* g = (mj_arg*)v;
    mj_ctx* c = g->c;
    const int t = g->t, T = c->T;
    size_t lo, hi;
    if (g->phase == 0) {  /* build histogram */
        mj_range(c->n1, T, t, &lo, &hi);
        for (int p = 0; p < MJ_P; p++) c->hist[t][p] = 0;
        for (size_t i = lo; i < hi; i++) c->hist[t][mj_hash(c->c1[i]) & (MJ_P - 1)]++;
    } else if (g->phase == 1) {  /* build scatter (hist now holds offsets) */
        mj_range(c->n1, T, t, &lo, &hi);
        for (size_t i = lo; i < hi; i++) {
            size_t o = c->hist[t][mj_hash(c->c1[i]) & (MJ_P - 1)]++;
            c->pk[o] = c->c1[i];
            c->pp[o] = c->p1[i];
        }
    } else if (g->phase == 2) {  /* partition tables */
        for (int p = t; p < MJ_P; p += T) mj_build_part(c, p);
    } else if (g->phase == 3) {  /* probe count */
        mj_range(c->n2, T, t, &lo, &hi);
        size_t m = 0;
        for (size_t j = lo; j < hi; j++) {
            uint32_t len;
            int p;
            (void)mj_find(c, c->c2[j], &len, &p);
            m += len;
        }
        c->pcount[t] = m;
    } else {  /* probe write (pcount now holds offsets) */
        mj_range(c->n2, T, t, &lo, &hi);
        size_t o = c->pcount[t];
        for (size_t j = lo; j < hi; j++) {
            uint32_t len;
            int p;
            uint32_t a = mj_find(c, c->c2[j], &len, &p);
            for (uint32_t e = 0; e < len; e++) {
                c->out1[o] = c->tval[p][a + e];
                c->out2[o] = c->p2[j];
                o++;
            }
        }
    }
    return NULL;
}

static void mj_phase(mj_ctx* c, int phase) {
    pthread_t th[256];
    mj_arg a[256];
    for (int t = 0; t < c->T; t++) {
        a[t] = (mj_arg){c, t, phase};
        pthread_create(&th[t], NULL, mj_worker, &a[t]);
    }
    for (int t = 0; t < c->T; t++) pthread_join(th[t], NULL);
}

/* Returns M; writes the pairs when out1 != NULL and M <= cap, else (size_t)-1. */
size_t rc_hash_join_mt(const int32_t* c1, const int32_t* p1, size_t n1, const int32_t* c2, const int32_t* p2,
                       size_t n2, int32_t* out1, int32_t* out2, size_t cap, int nthreads) {
    if (n1 == 0 || n2 == 0) return 0;
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    mj_ctx* c = (mj_ctx*)calloc(1, sizeof(mj_ctx));
    c->c1 = c1, c->p1 = p1, c->c2 = c2, c->p2 = p2, c->n1 = n1, c->n2 = n2, c->T = nthreads;
    c->hist = (size_t(*)[MJ_P])malloc(sizeof(size_t) * MJ_P * (size_t)nthreads);
    c->pk = (int32_t*)malloc(sizeof(int32_t) * n1);
    c->pp = (int32_t*)malloc(sizeof(int32_t) * n1);
    c->pcount = (size_t*)malloc(sizeof(size_t) * (size_t)nthreads);
    mj_phase(c, 0);
    size_t acc = 0;
    for (int p = 0; p < MJ_P; p++) {  /* partition p's rows: thread 0's range first */
        c->poff[p] = acc;
        for (int t = 0; t < nthreads; t++) {
            size_t h = c->hist[t][p];
            c->hist[t][p] = acc;
            acc += h;
        }
    }
    c->poff[MJ_P] = acc;
    mj_phase(c, 1);
    mj_phase(c, 2);
    mj_phase(c, 3);
    size_t m = 0;
    for (int t = 0; t < nthreads; t++) {
        size_t x = c->pcount[t];
        c->pcount[t] = m;
        m += x;
    }
    size_t ret = m;
    if (out1) {
        if (m > cap) ret = (size_t)-1;
        else {
            c->out1 = out1, c->out2 = out2;
            mj_phase(c, 4);
        }
    }
    for (int p = 0; p < MJ_P; p++) {
        free(c->tkey[p]);
        free(c->tcnt[p]);
        free(c->toff[p]);
        free(c->tval[p]);
    }
    free(c->hist);
    free(c->pk);
    free(c->pp);
    free(c->pcount);
    free(c);
    return ret;
}

/* src/query.c:585-650 nested_loop_join: outer column_one, inner column_two. */
size_t rc_nested_loop_join(const int32_t* c1, const int32_t* p1, size_t n1,
                           const int32_t* c2, const int32_t* p2, size_t n2,
                           int32_t* out1, int32_t* out2, size_t cap) {
    size_t m = 0;
    for (size_t i = 0; i < n1; i++)
        for (size_t j = 0; j < n2; j++)
            if (c1[i] == c2[j]) {
                if (out1) {
                    if (m >= cap) return (size_t)-1;
                    out1[m] = p1[i];
                    out2[m] = p2[j];
                }
                m++;
            }
    return m;
}

/* ------------------------------------------------------------------ */
/* load path: src/db_manager.c:240-322 load_db + :164-199 insert_row    */
/* ------------------------------------------------------------------ */

/* fgets(line, MAX_LINE_SIZE = 1024, stream) over a memory buffer
 * (db_manager.c:23,263,306): up to 1023 bytes, through the first '\n'. */
static size_t csv_fgets(const char* text, size_t n, size_t at, char line[1024]) {
    size_t k = 0;
    while (at + k < n && k < 1023) {
        line[k] = text[at + k];
        k++;
        if (line[k - 1] == '\n') break;
    }
    line[k] = '\0';
    return k;
}

size_t rc_csv_header_len(const char* text, size_t n) {
    char line[1024];
    return csv_fgets(text, n, 0, line);
}

/* The data lines of load_db (db_manager.c:304-318): every fgets piece is one row;
 * strsep(",") tokens, atoi, the first ncols tokens fill row[], a token missing from
 * a line keeps the previous line's value (row[] is reused; the reference leaves it
 * uninitialised before the first line, this restatement starts it at 0). Each row
 * is appended to the columns and folds into min/max as insert_row does
 * (db_manager.c:189-195). cols == NULL counts rows only. */
size_t rc_load_csv(const char* text, size_t n, int ncols, int32_t** cols, size_t cap,
                   int32_t* minmax) {
    char line[1024];
    int* row = calloc((size_t)(ncols > 0 ? ncols : 1), sizeof(int));
    for (int j = 0; j < ncols && minmax; j++) {
        minmax[2 * j] = INT32_MAX;
        minmax[2 * j + 1] = INT32_MIN;
    }
    size_t rows = 0, at = 0;
    while (at < n) {
        at += csv_fgets(text, n, at, line);
        char* temp = line;
        char* token;
        int index = 0;
        while ((token = strsep(&temp, ",")) != NULL && index < ncols) row[index++] = atoi(token);
        if (cols) {
            if (rows >= cap) {
                free(row);
                return (size_t)-1;
            }
            for (int j = 0; j < ncols; j++) {
                cols[j][rows] = row[j];
                if (minmax) {
                    if (row[j] < minmax[2 * j]) minmax[2 * j] = row[j];
                    if (row[j] > minmax[2 * j + 1]) minmax[2 * j + 1] = row[j];
                }
            }
        }
        rows++;
    }
    free(row);
    return rows;
}

/* ------------------------------------------------------------------ */
/* index build: src/index.c:25-143 (sorted copy + positions)           */
/* ------------------------------------------------------------------ */

typedef struct {
    int32_t v;
    uint64_t row;
} IdxPair;

static int idx_cmp(const void* a, const void* b) {
    const IdxPair* x = a;
    const IdxPair* y = b;
    if (x->v != y->v) return x->v < y->v ? -1 : 1;
    return x->row < y->row ? -1 : (x->row > y->row);
}

/* init_column_index + quicksort (index.c:89-100, :25-46): the values sorted
 * ascending and the row each came from. Equal values in ascending row order — the
 * reference's Lomuto quicksort leaves them in an order of its own; the restatement
 * pins the values exactly and, per value, the set of rows. */
void rc_index_build(const int32_t* col, size_t n, int32_t* values, uint64_t* positions) {
    IdxPair* p = malloc((n ? n : 1) * sizeof(IdxPair));
    for (size_t i = 0; i < n; i++) p[i] = (IdxPair){col[i], i};
    qsort(p, n, sizeof(IdxPair), idx_cmp);
    for (size_t i = 0; i < n; i++) {
        values[i] = p[i].v;
        positions[i] = p[i].row;
    }
    free(p);
}

/* quicksort + partition exactly as index.c:25-46 (Lomuto, values[high] as the pivot,
 * `<` sends a value left, the >= side rotated by the swaps), so equal values end in
 * the reference's own order. Iterative (an explicit stack of [low, high] ranges in
 * the order the recursion visits them) so that deep recursions (sorted or
 * duplicate-heavy input: depth n) do not overflow the C stack; the result does not
 * depend on the order disjoint ranges are visited. Positions start as 0..n-1
 * (init_column_index :97-99). O(n^2) on duplicates, as the reference. */
void rc_index_build_lomuto(const int32_t* col, size_t n, int32_t* values, uint64_t* positions) {
    for (size_t i = 0; i < n; i++) {
        values[i] = col[i];
        positions[i] = i;
    }
    if (n < 2) return;
    size_t cap = 64, top = 0;
    int64_t* stk = malloc(cap * 2 * sizeof(int64_t));
    stk[0] = 0;
    stk[1] = (int64_t)n - 1;
    top = 1;
    while (top) {
        top--;
        const int64_t low = stk[2 * top], high = stk[2 * top + 1];
        if (low >= high) continue;
        const int32_t pivot = values[high];
        int64_t i = low - 1;
        for (int64_t j = low; j < high; j++) {
            if (values[j] < pivot) {
                i++;
                int32_t tv = values[i];
                values[i] = values[j];
                values[j] = tv;
                uint64_t tp = positions[i];
                positions[i] = positions[j];
                positions[j] = tp;
            }
        }
        int32_t tv = values[i + 1];
        values[i + 1] = values[high];
        values[high] = tv;
        uint64_t tp = positions[i + 1];
        positions[i + 1] = positions[high];
        positions[high] = tp;
        const int64_t pv = i + 1;
        if (top + 2 > cap) {
            cap *= 2;
            stk = realloc(stk, cap * 2 * sizeof(int64_t));
        }
        /* the recursion sorts [low, pv-1] first, then [pv+1, high]: push in reverse */
        stk[2 * top] = pv + 1;
        stk[2 * top + 1] = high;
        top++;
        stk[2 * top] = low;
        stk[2 * top + 1] = pv - 1;
        top++;
    }
    free(stk);
}

/* build_histogram (index.c:63-84): counts[(v - min) / bin_size]; rows whose bin is
 * outside [0, 100) go to counts[100] (the reference writes past its array). */
void rc_histogram(const int32_t* col, size_t n, int32_t mn, int32_t bin_size, uint64_t* counts) {
    memset(counts, 0, 101 * sizeof(uint64_t));
    for (size_t i = 0; i < n; i++) {
        const int b = (int)((uint32_t)col[i] - (uint32_t)mn) / bin_size;
        counts[(b >= 0 && b < 100) ? b : 100]++;
    }
}
