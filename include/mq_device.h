/*
 * mq_device.h — device-level C-ABI of libmq (MI355X / gfx950 column-scan executor).
 *
 * Plain pointers, sizes and a `void* stream` (a hipStream_t; NULL = the HIP null
 * stream; mq_default_stream() returns the library's own non-blocking stream). Every column / position pointer below is a DEVICE
 * pointer into HBM. All functions return 0 (MQ_OK) on success or a negative
 * MQ_E* code; mq_last_error() returns a message for the calling thread's last
 * failure. Nothing here falls back to the CPU: without a usable gfx950 device
 * every entry point returns MQ_ENODEV.
 *
 * Predicates are the reference's half-open range select: a row v matches when
 * (!has_low || v >= low) && (!has_high || v < high)  (src/query.c:97-127).
 *
 * The reference-facing drop-in (select_column, fetch_column, sum, ...) is in
 * mq_query.h; it is implemented in C on top of these entry points.
 */
#ifndef MQ_DEVICE_H
#define MQ_DEVICE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
    MQ_OK = 0,
    MQ_ENODEV = -1,   /* no gfx950 device / HIP runtime unusable */
    MQ_EINVAL = -2,   /* bad argument (NULL, misaligned, size out of range) */
    MQ_EHIP = -3,     /* a HIP runtime call or kernel launch failed */
    MQ_ENOMEM = -4,   /* device allocation failed */
    MQ_ECAP = -5      /* output capacity exceeded (join) */
};

/* Aggregates returned by the reductions (device-resident, 32 bytes). */
typedef struct mq_agg {
    uint64_t count;   /* rows that matched */
    int64_t sum;      /* exact int64 sum of the matched int32 values (query.c:325-354) */
    int32_t min;      /* INT32_MAX when count == 0 */
    int32_t max;      /* INT32_MIN when count == 0 */
    uint64_t _pad;
} mq_agg;

/* ---- runtime ---- */
int mq_init(int device);                 /* select/initialise a device; idempotent */
int mq_device_count(void);
const char* mq_last_error(void);
const char* mq_version(void);
int mq_malloc(void** dptr, size_t bytes);
int mq_free(void* dptr);
int mq_memcpy_h2d(void* dst, const void* src, size_t bytes, void* stream);
int mq_memcpy_d2h(void* dst, const void* src, size_t bytes, void* stream);
/* D2H through the library's pinned staging buffers (synchronous): dst is never
 * registered with the driver, so it can be write-protected afterwards without
 * stalling later GPU work (a direct pageable D2H followed by mprotect does). */
int mq_memcpy_d2h_staged(void* dst, const void* src, size_t bytes, void* stream);
/* Start populating the fresh host pages of [p, p + bytes) in the background (helper
 * threads of the calling thread, MADV_POPULATE_WRITE: content unchanged). The next
 * mq_memcpy_d2h_staged into exactly that range copies each chunk as soon as its pages
 * are in; it also starts this itself when nothing covers its range. Callers that know
 * a result's size before its kernel runs start it first, so the page faults overlap
 * the kernel. MQ_PREFAULT=0 disables it, MQ_FAULT_THREADS (default 6) sizes it; the
 * staged copies' host memcpy runs on MQ_COPY_THREADS threads (default 6: the calling
 * thread and 5 helpers). */
void mq_host_prefault(void* p, size_t bytes);
/* Wait until the calling thread's population job (if any) has finished: call it
 * before freeing a range handed to mq_host_prefault that no staged copy consumed. */
void mq_host_prefault_wait(void);
int mq_memcpy_d2d(void* dst, const void* src, size_t bytes, void* stream);
int mq_memset(void* dptr, int value, size_t bytes, void* stream);
int mq_stream_sync(void* stream);
void* mq_default_stream(void);
/* A non-blocking stream of its own on the calling thread's current device. */
int mq_stream_create(void** stream);
int mq_stream_destroy(void* stream);
/* Release the device scratch libmq keeps cached between calls (join tables and
 * partition buffers, probe arrays); the next call allocates afresh. */
void mq_trim(void);
/* Free the calling thread's pinned host staging buffers (the staged D2H/H2D ring
 * and shared_select's upload staging) on every device. A thread that stops using
 * libmq calls it before it exits (the row-shard workers do); later staged copies
 * on the thread allocate afresh. */
void mq_thread_release(void);
/* The same caching allocator for callers (the query layer keeps result shadows
 * and column copies in it). mq_pool_free hands the block out again at once, so it
 * frees only what no queued work still uses; mq_pool_free_on is the stream-ordered
 * free: the block is reused only after the work queued on `stream` so far has
 * finished (an event recorded on it; an allocation meanwhile gets a fresh block and
 * waits for the event only when no fresh block fits in HBM), so a caller frees right
 * after queueing the last kernel that reads it, with no host sync. Both also accept pointers from mq_malloc (freed at once;
 * mq_pool_free_on syncs the stream first). Call mq_pool_free_on with the block's
 * device current. */
int mq_pool_malloc(void** dptr, size_t bytes);
int mq_pool_free(void* dptr);
int mq_pool_free_on(void* dptr, void* stream);
/* Wait for all work queued on the calling thread's current device, on every stream
 * including the null stream (hipDeviceSynchronize). */
int mq_device_sync(void);

/* Workspace (device bytes) needed by the scan entry points for n rows. */
size_t mq_scan_workspace_bytes(uint64_t n);
/* The library's grid for a scan of n rows: blocks launched and rows per block. */
void mq_scan_geometry(uint64_t n, uint32_t* blocks, uint64_t* rows_per_block);

/* ---- synthetic data (bench/tests; SURVEY.md §8(c) generator) ---- */
/* out[i] = (int32)(sm64(seed*0x100000001B3 + i) % modulus) */
int mq_gen_uniform(int32_t* d_out, uint64_t n, uint64_t seed, uint64_t modulus, void* stream);
/* hash-join keys of SURVEY §8(c) config 5 (kind 0 = build mix31(i), 1 = probe) and its
 * many-to-many variant (2 = build mix31(i mod n/2): every key twice; 3 = probe
 * mix31(sm64((7<<40)|j) mod n), n a power of two: about half hit), and iota */
int mq_gen_join_keys(int32_t* d_out, uint64_t n, int kind, void* stream);
int mq_gen_iota(int32_t* d_out, uint64_t n, void* stream);

/* ---- S1/S7 fused, one launch: count + int64 sum of rows of d_col in range ----
 * (select_column -> fetch_column -> sum, query.c:92-137 + 223-243 + 325-354, with
 * the positions never materialised). min/max are left INT32_MAX / INT32_MIN.
 * This is the bench's headline step. d_ws: >= mq_scan_workspace_bytes(0). */
int mq_select_sum(const int32_t* d_col, uint64_t n, int has_low, int32_t low, int has_high,
                  int32_t high, mq_agg* d_out, void* d_ws, size_t ws_bytes, void* stream);

/* ---- S1/S7 fused: count + int64 sum (+min/max) of rows of d_col in range ----
 * One HBM pass over d_col (4n bytes). *d_out receives the aggregate. */
int mq_select_agg(const int32_t* d_col, uint64_t n, int has_low, int32_t low, int has_high,
                  int32_t high, mq_agg* d_out, void* d_ws, size_t ws_bytes, void* stream);

/* The two launches of mq_select_agg, for callers that time the scan kernel alone:
 * mq_select_partials writes one partial per block into d_ws (and *nblocks);
 * mq_combine_partials folds nblocks partials from d_ws into *d_out.
 * want_minmax = 0 computes count + sum only (select + sum; min/max left at
 * INT32_MAX / INT32_MIN), 1 also min/max. */
int mq_select_partials(const int32_t* d_col, uint64_t n, int has_low, int32_t low, int has_high,
                       int32_t high, int want_minmax, void* d_ws, size_t ws_bytes,
                       uint32_t* nblocks, void* stream);
int mq_combine_partials(const void* d_ws, uint32_t nblocks, mq_agg* d_out, void* stream);

/* Diagnostic (no reference counterpart): the achievable HBM read rate for the
 * scan's access pattern (SURVEY.md §8(d) "achievable peak"). Streams d_col with
 * k_scan's loads and no predicate; *bytes_read receives the bytes the launch reads
 * (whole 8192-row groups of each block's chunk). d_ws: >= 8192 * 4 bytes. */
int mq_stream_read(const int32_t* d_col, uint64_t n, void* d_ws, size_t ws_bytes,
                   uint64_t* bytes_read, void* stream);

/* Diagnostic (no reference counterpart): the random-access ceiling of the join
 * probe. n_reads 8-byte reads of d_table (2^slots_log2
 * u64 slots) at hashed slots, 8 per lane in flight: k_ht_probe_unique's pattern
 * without the key compare or the output. d_ws: >= 8 bytes. */
int mq_random_read(const uint64_t* d_table, int slots_log2, uint64_t n_reads, void* d_ws, void* stream);

/* ---- J4 hashset.c (src/hashset.c:11-65) on the device ----
 * The set is the reference's own table: `size` int32 slots, 0 = empty, a key's
 * linear probe starting at hash(key, size) = key % size (multimap.c:60-63; a
 * negative key, an out-of-bounds index in the reference, starts at the wrapped
 * remainder here).
 * mq_hashset_lookup: d_found[i] = lookup_hashset(set, d_probe[i]) (hashset.c:35-45)
 *   for n probes; a full table without the key answers 0 after one lap (the
 *   reference loops forever).
 * mq_hashset_elements: the nonzero slots in slot order (get_hashset_elements,
 *   hashset.c:48-65) into d_out (capacity size); *d_count (device) receives their
 *   number. d_ws: mq_scan_workspace_bytes(size) bytes. */
int mq_hashset_lookup(const int32_t* d_table, int32_t size, const int32_t* d_probe, uint64_t n,
                      uint8_t* d_found, void* stream);
int mq_hashset_elements(const int32_t* d_table, uint64_t size, int32_t* d_out, uint64_t* d_count,
                        void* d_ws, size_t ws_bytes, void* stream);

/* Config-3 fused: aggregate of d_val[i] over rows i where d_sel[i] is in range. */
int mq_select_fetch_agg(const int32_t* d_sel, const int32_t* d_val, uint64_t n, int has_low,
                        int32_t low, int has_high, int32_t high, mq_agg* d_out, void* d_ws,
                        size_t ws_bytes, void* stream);

/* ---- S1 select_column_scan / S4 select_result: ordered compaction ----
 * Writes, in ascending i, d_payload ? d_payload[i] : i for every i whose d_col[i]
 * is in range, into d_pos_out (capacity n). *d_count receives K.
 * n must be < 2^31 (positions are int32, query.c:94). */
int mq_select_positions(const int32_t* d_col, const int32_t* d_payload, uint64_t n, int has_low,
                        int32_t low, int has_high, int32_t high, int32_t* d_pos_out,
                        uint64_t* d_count, void* d_ws, size_t ws_bytes, void* stream);

/* The same over a row shard: the rows are d_col[0..n) but number from row_base, so
 * without a payload the positions written are row_base + i (a column split into row
 * ranges across devices concatenates its shards' outputs in shard order).
 * row_base + n must be < 2^31. */
int mq_select_positions_at(const int32_t* d_col, const int32_t* d_payload, uint64_t n, int32_t row_base,
                           int has_low, int32_t low, int has_high, int32_t high, int32_t* d_pos_out,
                           uint64_t* d_count, void* d_ws, size_t ws_bytes, void* stream);

/* select_column's download pipeline (the API path): the ordered positions
 * of d_col[0..n) selected in `segs` contiguous row segments (1..64) queued on `stream`,
 * and each segment's positions downloaded into h_dst as soon as ITS kernel has finished,
 * through the staged D2H on a copy stream of the calling thread, while the later
 * segments' kernels still run. h_dst must hold n int32 (the caller's payload; untouched
 * beyond the K written). d_pos (capacity n) receives segment s's positions from its
 * first row (d_pos[r_s ...], r_s = h_rows[s]); h_seg[s] receives segment s's count and
 * h_rows[s] its first row (segs + 1 entries, h_rows[segs] = n). Returns when every
 * download is complete; the segments' positions in h_dst are contiguous in order. */
int mq_select_positions_download(const int32_t* d_col, uint64_t n, int has_low, int32_t low, int has_high,
                                 int32_t high, int segs, int32_t* d_pos, int32_t* h_dst, uint64_t* h_seg,
                                 uint64_t* h_rows, void* d_ws, size_t ws_bytes, void* stream);

/* ---- S6 select_column_sorted_index (query.c:143-198) ----
 * d_values: n int32 sorted ascending; d_positions: n size_t row ids. Restates the
 * reference's binary_search + run adjustment exactly (including its low == high
 * quirk), writes the run's positions (as int32) to d_pos_out, K to *d_count. */
int mq_index_select(const int32_t* d_values, const uint64_t* d_positions, uint64_t n, int32_t low,
                    int32_t high, int32_t* d_pos_out, uint64_t* d_count, void* stream);

/* ---- index build (index.c:89-143) ----
 * Sorted copy of d_col (n < 2^32 rows): d_values_out ascending (may be NULL) and
 * d_positions_out[i] (size_t, may be NULL) the row it came from, equal values in
 * ascending row order. (The reference's quicksort orders equal values its own way;
 * the values, and the positions of distinct values, are identical.) */
int mq_index_build(const int32_t* d_col, uint64_t n, int32_t* d_values_out,
                   uint64_t* d_positions_out, void* stream);
/* The same in the reference quicksort's own order (index.c:25-46), equal values
 * included: a level-synchronous restatement of the Lomuto recursion (n < 2^31).
 * Costs a few passes over n per recursion depth (O(log n) depths on distinct-ish
 * data; a range of equal values finishes in one). */
int mq_index_build_lomuto(const int32_t* d_col, uint64_t n, int32_t* d_values_out,
                          uint64_t* d_positions_out, void* stream);
/* The build_index drop-in's policy: the radix sort; if the values hold ties and
 * n <= exact_max, the Lomuto order instead (distinct values have one order, so the
 * radix result is already the reference's). *h_exact = 0 when ties were left in
 * ascending row order (n > exact_max). d_values_out is required. */
int mq_index_build_ref(const int32_t* d_col, uint64_t n, int32_t* d_values_out, uint64_t* d_positions_out,
                       uint64_t exact_max, int* h_exact, void* stream);
/* reorder_column (index.c:105-114): d_out[i] = d_col[d_positions[i]] (size_t positions) */
int mq_gather_u64(const int32_t* d_col, const uint64_t* d_positions, uint64_t n, int32_t* d_out,
                  void* stream);
/* build_histogram's counts (index.c:63-84): d_counts[b] (101 u64) = rows with
 * (int)(v - col_min) / bin_size == b for b in [0, 100); d_counts[100] = rows outside
 * (the reference writes those past its 100-entry array). bin_size != 0. */
int mq_histogram(const int32_t* d_col, uint64_t n, int32_t col_min, int32_t bin_size,
                 uint64_t* d_counts, void* stream);

/* ---- S5 fetch_column: d_out[i] = d_col[d_pos[i]] ---- */
int mq_fetch(const int32_t* d_col, const int32_t* d_pos, uint64_t k, int32_t* d_out, void* stream);
/* the same from a row shard holding rows [row_base, row_base + rows) of the column:
 * d_out[i] = d_col[d_pos[i] - row_base] (every position must lie in the shard) */
int mq_fetch_at(const int32_t* d_col, int32_t row_base, const int32_t* d_pos, uint64_t k, int32_t* d_out,
                void* stream);

/* ---- S7/S8/S9 over a values vector (sum/avg/min/max of a Result) ---- */
int mq_reduce(const int32_t* d_vals, uint64_t n, mq_agg* d_out, void* d_ws, size_t ws_bytes,
              void* stream);

/* ---- P1 print (query.c:245-304): int32 values as decimal text ----
 * Writes "%d" of every value, joined by "\n" (no trailing separator, no NUL),
 * into d_out (capacity >= 12 * n bytes); *h_len receives the byte count. The
 * call synchronises the stream. d_ws: >= mq_format_workspace_bytes(n). */
size_t mq_format_workspace_bytes(uint64_t n);
int mq_format_int32(const int32_t* d_vals, uint64_t n, char* d_out, uint64_t* h_len, void* d_ws,
                    size_t ws_bytes, void* stream);

/* A table as CSV text, the way the reference's generators write the load files
 * (value of column 0, ',' ... column ncols-1, '\n' per row; "%d" each). d_cols: host
 * array of ncols device pointers; d_out capacity >= rows * ncols * 12 bytes; *h_len
 * receives the byte count. Synchronises the stream. (Bench/test data for the load
 * path; the reference loads such files with load_db.) */
size_t mq_format_csv_workspace_bytes(uint64_t rows, int ncols);
int mq_format_csv_int32(const int32_t* const* d_cols, int ncols, uint64_t rows, char* d_out,
                        uint64_t* h_len, void* d_ws, size_t ws_bytes, void* stream);

/* ---- load path: load_db's data loop (db_manager.c:304-318) + insert_row (:164-199) ----
 * d_text: n bytes of CSV data lines in HBM (the header line already consumed; the
 * header is what fgets returns first, <= 1023 bytes through '\n'). Rows are the
 * reference's fgets(line, 1024) pieces: through the next '\n', at most 1023 bytes.
 * Each row's first ncols ','-separated tokens go through atoi; a token missing from
 * a row keeps the previous row's value (0 before the first row); extra tokens are
 * ignored. Two steps on one workspace (mq_csv_workspace_bytes(n, ncols)):
 * count: *h_rows = rows (synchronous);
 * parse: d_cols[j] (host array of ncols device pointers, capacity >= rows) receive
 *        column j; d_minmax (device, 2*ncols int32) min/max per column (INT32_MAX /
 *        INT32_MIN when rows == 0), as insert_row folds them. ncols <= 1024. */
size_t mq_csv_workspace_bytes(uint64_t n, int ncols);
int mq_csv_count_rows(const char* d_text, uint64_t n, int ncols, uint64_t* h_rows, void* d_ws,
                      size_t ws_bytes, void* stream);
int mq_csv_parse_int32(const char* d_text, uint64_t n, int ncols, int32_t* const* d_cols,
                       uint64_t rows, int32_t* d_minmax, void* d_ws, size_t ws_bytes, void* stream);

/* ---- S10 add / sub (int32, two's-complement wrap) ---- */
int mq_add(const int32_t* d_a, const int32_t* d_b, uint64_t n, int32_t* d_out, void* stream);
int mq_sub(const int32_t* d_a, const int32_t* d_b, uint64_t n, int32_t* d_out, void* stream);

/* ---- S11 shared_select: q range predicates [lows[j], highs[j]) over one column ----
 * h_lows/h_highs: q host int32 bounds, used as given (has_low/has_high are ignored
 * there, query.c:472-479). d_pos_out[j] (host array of q device pointers, each of
 * capacity n) receives query j's ascending positions; d_counts[j] (device) its K_j.
 * q >= 2 reads the column twice in total (count pass + write pass), any q <= 256. */
size_t mq_shared_select_workspace_bytes(uint64_t n, int q);
int mq_shared_select(const int32_t* d_col, uint64_t n, const int32_t* h_lows,
                     const int32_t* h_highs, int q, int32_t* const* d_pos_out,
                     uint64_t* d_counts, void* d_ws, size_t ws_bytes, void* stream);
/* The same in two steps, so outputs can be sized exactly (q <= 256):
 * count: one pass, *h_counts[j] = K_j (host, synchronous); the workspace keeps the
 *        offsets for the next step;
 * write: the second pass into d_pos_out[j] (capacity K_j each), on the workspace
 *        of the immediately preceding count call of this thread. */
int mq_shared_select_count(const int32_t* d_col, uint64_t n, const int32_t* h_lows,
                           const int32_t* h_highs, int q, uint64_t* h_counts, void* d_ws,
                           size_t ws_bytes, void* stream);
int mq_shared_select_write(void* d_ws, int32_t* const* d_pos_out, void* stream);
/* count over a row shard whose rows number from row_base (the write then emits
 * row_base + i), as mq_select_positions_at */
int mq_shared_select_count_at(const int32_t* d_col, uint64_t n, int32_t row_base, const int32_t* h_lows,
                              const int32_t* h_highs, int q, uint64_t* h_counts, void* d_ws,
                              size_t ws_bytes, void* stream);

/* ---- J1 hash_join as three steps on a handle (lets the caller size the output) ----
 * build: table over (c1, p1); c1 and p1 must stay valid until mq_join_free (a unique
 *   build of 2^20 rows and more keeps only its window partition, and one whose probe
 *   meets a duplicate key is built again from them).
 * probe: per-probe match counts + output offsets for keys c2; *h_m = M. c2 is read
 *   only inside the call (a partitioned probe leaves its last inverse pass to the write,
 *   which reads the places that pass recorded, not the keys: DESIGN.md §3.3 round 6).
 * write: the M pairs (out1 = build positions, out2 = probe positions p2). */
typedef struct mq_join mq_join;
int mq_join_build(const int32_t* d_c1, const int32_t* d_p1, uint64_t n1, mq_join** out,
                  void* stream);
int mq_join_probe(mq_join* join, const int32_t* d_c2, uint64_t n2, uint64_t* h_m, void* stream);
int mq_join_write(mq_join* join, const int32_t* d_p2, int32_t* d_out1, int32_t* d_out2,
                  void* stream);
int mq_join_free(mq_join* join);
/* Per probe row of the last mq_join_probe, its number of pairs (d_cnt: n2 u32).
 * mq_join_write also accepts d_p2 = d_out2 = NULL: build positions only. */
int mq_join_counts(mq_join* join, uint32_t* d_cnt, void* stream);

/* ---- key-partitioned hash join over G devices ----
 * The device pieces; mq_shard_join (mq_query.h) runs them over the row-shard workers,
 * analytical-database_amd/dist.py one process per GPU.
 * mq_pjoin_bucket: the bucket (0..G-1) of a key, as the partition kernels compute it.
 * mq_pjoin_partition: stable split of n rows into G buckets by key: d_keys_out (and
 *   d_pay_out with d_pay, and d_inv[r] = row r's new index, when not NULL) hold bucket
 *   0's rows in row order, then bucket 1's, ...; h_counts[b] (host, G entries) their
 *   numbers. Synchronous. G <= 64, n < 2^32.
 * mq_pjoin_place: a probe shard's output from its partitioned counts d_cntp (n u32) and
 *   pairs d_out1p (m build positions, partitioned order): row r's pairs go to the offset
 *   of the rows before it, out2 = d_p2[r]. Asynchronous on stream (its temporaries are
 *   freed stream-ordered). */
uint32_t mq_pjoin_bucket(int32_t key, int G);
int mq_pjoin_partition(const int32_t* d_keys, const int32_t* d_pay, uint64_t n, int G, int32_t* d_keys_out,
                       int32_t* d_pay_out, uint32_t* d_inv, uint64_t* h_counts, void* stream);
int mq_pjoin_place(const uint32_t* d_cntp, const int32_t* d_out1p, const uint32_t* d_inv, const int32_t* d_p2,
                   uint64_t n, uint64_t m, int32_t* d_out1, int32_t* d_out2, void* stream);
/* Device-to-device copy between (or within) devices on stream (the destination's). */
int mq_memcpy_peer(void* dst, int dst_dev, const void* src, int src_dev, size_t bytes, void* stream);
/* Let the current device read and write peer's memory directly (a no-op where the
 * platform cannot; peer copies still work then). */
int mq_enable_peer(int peer);

/* ---- J1 hash_join in one call: build on (c1,p1) (n1 rows), probe with (c2,p2) (n2 rows) ----
 * Output pairs (out1[m], out2[m]) = (build position, probe position) in
 * probe-major, build-insertion order (query.c:652-696). *h_m receives M.
 * Returns MQ_ECAP (with *h_m = M) when M > cap. Allocates its own scratch. */
int mq_hash_join(const int32_t* d_c1, const int32_t* d_p1, uint64_t n1, const int32_t* d_c2,
                 const int32_t* d_p2, uint64_t n2, int32_t* d_out1, int32_t* d_out2,
                 uint64_t cap, uint64_t* h_m, void* stream);

#ifdef __cplusplus
}
#endif
#endif
