/*
 * refcpu.h — CPU restatement of the reference hot path (ORACLE / TEST INFRASTRUCTURE ONLY).
 *
 * This library is the parity checker and the CPU baseline timed by bench.py's
 * cpu_baseline leg. It is NEVER linked into libmq and never called by the
 * product path. Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it.
 *
 * Every function restates one loop of siyaoL1/Analytical-Database
 * (src/query.c, src/multimap.c) on plain pointers; the file:line each one
 * follows is given at its definition in refcpu.c. The restatement is pinned
 * against the reference itself (oracle/_ref/libref.so, compiled from
 * /root/reference/src by oracle/Makefile) and against the golden vectors in
 * tests/golden/ (see tests/test_oracle.py).
 */
#ifndef MQ_REFCPU_H
#define MQ_REFCPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- synthetic data (SURVEY.md §8(c) generator) ---- */
uint64_t rc_sm64(uint64_t x);
uint32_t rc_mix31(uint32_t x);
/* out[i] = (int32)(sm64(seed*0x100000001B3 + i) % modulus), i in [0,n) */
void rc_gen_uniform(int32_t* out, size_t n, uint64_t seed, uint64_t modulus, int nthreads);
/* hash-join keys of SURVEY §8(c) config 5: build a[i]=mix31(i);
 * probe b[j]=mix31(sm64((7<<40)|j) & (2n-1)) */
void rc_gen_join_build(int32_t* out, size_t n);
void rc_gen_join_probe(int32_t* out, size_t n);
void rc_gen_join_build_dup(int32_t* out, size_t n);
void rc_gen_join_probe_dup(int32_t* out, size_t n);
void rc_iota(int32_t* out, size_t n);
uint64_t rc_fnv1a64(const void* p, size_t bytes);
uint64_t rc_fnv1a64_pairs(const int32_t* a, const int32_t* b, size_t m);

/* ---- operators (NULL bound = unbounded, half-open [low, high)) ---- */
size_t rc_select_scan(const int32_t* data, size_t n, const int32_t* low, const int32_t* high,
                      int32_t* pos_out);
size_t rc_select_scan_mt(const int32_t* data, size_t n, const int32_t* low, const int32_t* high,
                         int32_t* pos_out, int nthreads);
size_t rc_select_result(const int32_t* vals, const int32_t* prev_pos, size_t n,
                        const int32_t* low, const int32_t* high, int32_t* pos_out);
void rc_fetch(const int32_t* col, const int32_t* pos, size_t k, int32_t* out);
int64_t rc_sum(const int32_t* v, size_t n);
double rc_avg(const int32_t* v, size_t n);
int32_t rc_min(const int32_t* v, size_t n);
int32_t rc_max(const int32_t* v, size_t n);
void rc_add(const int32_t* a, const int32_t* b, size_t n, int32_t* out);
void rc_sub(const int32_t* a, const int32_t* b, size_t n, int32_t* out);
/* fused count+sum of values in [low,high): the scalar loop the GPU fused kernel replaces */
void rc_select_count_sum(const int32_t* data, size_t n, const int32_t* low, const int32_t* high,
                         uint64_t* count, int64_t* sum, int nthreads);

/* shared_select: q predicates [lows[i], highs[i]) over one column in one pass.
 * pos_out[i] must hold n entries; counts[i] receives K_i.
 * split = 0: row-balanced nthreads split; split = 1: the reference's
 * value-range split into 3 tasks (query.c:506-522; requires 2*((max-min)/3) <= n). */
int rc_shared_select(const int32_t* data, size_t n, const int32_t* lows, const int32_t* highs,
                     int q, int32_t** pos_out, size_t* counts, int nthreads, int split,
                     int32_t col_min, int32_t col_max);

/* hash_join: build on (c1,p1), probe with (c2,p2); output pairs in probe-major,
 * build-insertion order. Returns M (number of pairs) or (size_t)-1 when the
 * output capacity cap is exceeded. Pass out1=out2=NULL to count only. */
size_t rc_hash_join(const int32_t* c1, const int32_t* p1, size_t n1,
                    const int32_t* c2, const int32_t* p2, size_t n2,
                    int32_t* out1, int32_t* out2, size_t cap);
/* The same over nthreads host threads (partitioned build, range-split probe): the
 * config-5 host-cores baseline; output identical to rc_hash_join. */
size_t rc_hash_join_mt(const int32_t* c1, const int32_t* p1, size_t n1, const int32_t* c2, const int32_t* p2,
                       size_t n2, int32_t* out1, int32_t* out2, size_t cap, int nthreads);
size_t rc_nested_loop_join(const int32_t* c1, const int32_t* p1, size_t n1,
                           const int32_t* c2, const int32_t* p2, size_t n2,
                           int32_t* out1, int32_t* out2, size_t cap);
int32_t rc_multimap_size(int32_t tuple_num);

/* ---- load path (db_manager.c:240-322 load_db, :164-199 insert_row) ----
 * rc_csv_header_len: bytes the header fgets consumes (<= 1023, through '\n').
 * rc_load_csv: rows of the data text (header excluded); cols[j] (capacity cap)
 * receive column j and minmax[2j], [2j+1] its min / max (INT32_MAX / INT32_MIN
 * when there are no rows). cols == NULL counts only; (size_t)-1 when rows > cap. */
size_t rc_csv_header_len(const char* text, size_t n);

/* ---- index build (index.c:25-143): stable sort of (value, row) ---- */
void rc_index_build(const int32_t* col, size_t n, int32_t* values, uint64_t* positions);
void rc_index_build_lomuto(const int32_t* col, size_t n, int32_t* values, uint64_t* positions);
/* build_histogram counts (index.c:63-84); counts has 101 entries, [100] = out of range */
void rc_histogram(const int32_t* col, size_t n, int32_t mn, int32_t bin_size, uint64_t* counts);
size_t rc_load_csv(const char* text, size_t n, int ncols, int32_t** cols, size_t cap,
                   int32_t* minmax);

#ifdef __cplusplus
}
#endif
#endif
