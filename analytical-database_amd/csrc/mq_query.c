/*
 * mq_query.c — the reference operator API (src/include/query.h:20-50) in C on
 * top of libmq's device layer (include/mq_device.h).
 *
 * This file is host control only: it keeps the reference's calling contract
 * (Column* and Result* in, malloc'd Result out, Status.code), decides what is
 * device-resident, and moves results between HBM and host memory. Every
 * row-proportional loop of the reference runs as a gfx950 kernel; there is no
 * CPU fallback — without a device every entry point sets Status ERROR and
 * returns NULL, after printing why to stderr.
 *
 * Residency:
 *   - Column rows (column->data, mmap'd host memory in the reference,
 *     db_manager.c:736-790) are uploaded once and cached by (Column*, data,
 *     row_count) until mq_column_invalidate(); mq_column_attach() adopts an
 *     existing HBM copy without any upload.
 *   - A Result made here keeps a device shadow keyed by its payload pointer, so
 *     the next operator on it (fetch, sum, avg, select_result, ...) reads HBM.
 *     The shadow is validated against num_tuples and the first/last element and
 *     is re-uploaded on mismatch. Shadows are evicted LRU beyond a byte budget
 *     (MQ_SHADOW_MB, default 65536 MB).
 */
#define _DEFAULT_SOURCE
#include "mq_query.h"

#include <fcntl.h>
#include <limits.h>
#include <malloc.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include "mq_device.h"
#include "mq_guard.h"
#include "mq_shim.h"

/* ---- ABI pins: x86-64 layouts of the reference structs ---- */
_Static_assert(sizeof(Result) == 24, "Result size");
_Static_assert(offsetof(Result, num_tuples) == 0, "Result.num_tuples");
_Static_assert(offsetof(Result, data_type) == 8, "Result.data_type");
_Static_assert(offsetof(Result, payload) == 16, "Result.payload");
_Static_assert(sizeof(Column) == 128, "Column size");
_Static_assert(offsetof(Column, data) == 64, "Column.data");
_Static_assert(offsetof(Column, fd) == 72, "Column.fd");
_Static_assert(offsetof(Column, row_count) == 80, "Column.row_count");
_Static_assert(offsetof(Column, sorted) == 88, "Column.sorted");
_Static_assert(offsetof(Column, clustered) == 89, "Column.clustered");
_Static_assert(offsetof(Column, has_index) == 90, "Column.has_index");
_Static_assert(offsetof(Column, index) == 96, "Column.index");
_Static_assert(offsetof(Column, btree_node) == 104, "Column.btree_node");
_Static_assert(offsetof(Column, histogram) == 112, "Column.histogram");
_Static_assert(offsetof(Column, max) == 120, "Column.max");
_Static_assert(offsetof(Column, min) == 124, "Column.min");
_Static_assert(sizeof(Status) == 16, "Status size");
_Static_assert(offsetof(Status, error_message) == 8, "Status.error_message");
_Static_assert(sizeof(GeneralizedColumn) == 16, "GeneralizedColumn size");
_Static_assert(offsetof(GeneralizedColumn, column_pointer) == 8, "GeneralizedColumn.pointer");
_Static_assert(sizeof(SelectOperator) == 136, "SelectOperator size");
_Static_assert(offsetof(SelectOperator, handle) == 4, "SelectOperator.handle");
_Static_assert(offsetof(SelectOperator, low) == 68, "SelectOperator.low");
_Static_assert(offsetof(SelectOperator, high) == 72, "SelectOperator.high");
_Static_assert(offsetof(SelectOperator, has_low) == 76, "SelectOperator.has_low");
_Static_assert(offsetof(SelectOperator, has_high) == 80, "SelectOperator.has_high");
_Static_assert(offsetof(SelectOperator, db) == 88, "SelectOperator.db");
_Static_assert(offsetof(SelectOperator, column) == 104, "SelectOperator.column");
_Static_assert(offsetof(SelectOperator, comparator) == 128, "SelectOperator.comparator");
_Static_assert(sizeof(ColumnIndex) == 16, "ColumnIndex size");
_Static_assert(sizeof(Table) == 96, "Table size");
_Static_assert(offsetof(Table, columns) == 64 && offsetof(Table, col_count) == 72, "Table.columns");
_Static_assert(offsetof(Table, row_count) == 80 && offsetof(Table, table_length) == 88, "Table rows");
_Static_assert(sizeof(Db) == 88, "Db size");
_Static_assert(offsetof(Db, tables) == 64 && offsetof(Db, tables_size) == 72, "Db.tables");
_Static_assert(INT == 0 && LONG == 1 && FLOAT == 2 && DOUBLE == 3, "DataType values");
_Static_assert(OK == 0 && ERROR == 1, "StatusCode values");

/* ------------------------------------------------------------------ */
/* state                                                              */
/* ------------------------------------------------------------------ */

/* Every entry remembers the operator that last used it (op == g_op: in use by
 * the current call, never evicted) and, for copies of host memory, the write
 * guard (mq_guard.c) that says whether that memory is still what was uploaded.
 * An entry without a guard (memory that cannot be guarded) serves only the
 * operator that uploaded it. */
typedef struct {
    const Column* col;
    const int* host;
    size_t rows;
    void* dev;
    int owned;                /* 0: attached by the caller (mq_column_attach), trusted */
    uint64_t guard;
    unsigned long long op;
} ColEntry;

typedef struct {
    const void* host;
    size_t n;
    size_t bytes;
    void* dev;
    uint64_t guard;
    unsigned long long stamp; /* LRU */
    unsigned long long op;
} ShadowEntry;

typedef struct {
    const ColumnIndex* index;
    const int* values;
    const size_t* positions;
    size_t rows;
    void* d_values;
    void* d_positions;
    uint64_t guard_v, guard_p;
    unsigned long long op;
} IndexEntry;

#define MAX_COLS 1024
#define MAX_SHADOWS 4096
#define MAX_INDEXES 256

static ColEntry g_cols[MAX_COLS];
static int g_ncols;
static ShadowEntry g_shadows[MAX_SHADOWS];
static int g_nshadows;
static size_t g_shadow_bytes;
static unsigned long long g_stamp;
static unsigned long long g_op;
static IndexEntry g_idx[MAX_INDEXES];
static int g_nidx;
static mq_residency g_res;

static void* g_ws;        /* scan workspace */
static size_t g_ws_bytes;
static void* g_scratch;   /* capacity-n int32 output staging */
static size_t g_scratch_bytes;
static void* g_small;     /* mq_agg + counts */
static int g_ready;       /* 1 ok, -1 failed */
static void* g_stream;
static double g_xfer_s;

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

/* MQ_TRACE=1: host-side phase times of the API path on stderr (diagnostics). */
static int trace_on(void) {
    static int v = -1;
    if (v < 0) {
        const char* e = getenv("MQ_TRACE");
        v = e && e[0] == '1';
    }
    return v;
}
#define TRACE(label, t0)                                                                    \
    do {                                                                                    \
        if (trace_on()) fprintf(stderr, "mq-trace %-24s %9.3f ms\n", label, 1e3 * (now_s() - (t0))); \
    } while (0)

static int fail(Status* st, const char* what, int rc) {
    fprintf(stderr, "libmq: %s failed (%d): %s\n", what, rc, mq_last_error());
    if (st) st->code = ERROR;
    return rc;
}

static void sweep(void);

static int ready(Status* st) {
    if (g_ready == 1) return 0;
    if (g_ready == -1) return fail(st, "device init (earlier)", MQ_ENODEV);
    const char* env = getenv("MQ_DEVICE");
    int dev = env ? atoi(env) : 0;
    int rc = mq_init(dev);
    if (rc) {
        g_ready = -1;
        return fail(st, "device init", rc);
    }
    /* Result payloads of >= 1 MB come from mmap (and go back to it on free), which
     * is what lets a write guard cover them; glibc's dynamic threshold would
     * otherwise rise to the last freed size (up to 32 MB) and serve them from the
     * heap. Affects only where large blocks of this process come from. */
    if (mq_guard_enabled()) mallopt(M_MMAP_THRESHOLD, (int)SHADOW_MIN_BYTES); /* not needed unguarded */
    g_stream = mq_default_stream();
    if (!g_stream) {
        g_ready = -1;
        return fail(st, "stream creation", MQ_EHIP);
    }
    rc = mq_malloc(&g_small, 4096);
    if (rc) {
        g_ready = -1;
        return fail(st, "small buffer", rc);
    }
    g_ready = 1;
    return 0;
}

/* Start of an operator of the reference API: a new op number (what the previous
 * operator held may now be evicted) and drop the copies no later call can use. */
static int op_begin(Status* st) {
    const double t0 = now_s();
    if (ready(st)) return -1;
    g_op++;
    sweep();
    shard_op_begin();
    TRACE("op_begin", t0);
    return 0;
}

static int h2d(void* d, const void* h, size_t bytes) {
    double t0 = now_s();
    int rc = mq_memcpy_h2d(d, h, bytes, g_stream);
    g_xfer_s += now_s() - t0;
    return rc;
}

/* The transfer clock starts once the stream is idle, so mq_transfer_seconds counts
 * the copies alone, not the kernels they wait for. */
static int d2h(void* h, const void* d, size_t bytes) {
    int rc = mq_stream_sync(g_stream);
    if (rc) return rc;
    double t0 = now_s();
    rc = mq_memcpy_d2h(h, d, bytes, g_stream);
    g_xfer_s += now_s() - t0;
    return rc;
}

/* D2H into memory that will be write-guarded: through pinned staging, so the
 * guard's mprotect does not stall the GPU (mq_memcpy_d2h_staged). */
static int d2h_staged(void* h, const void* d, size_t bytes) {
    int rc = mq_stream_sync(g_stream);
    if (rc) return rc;
    double t0 = now_s();
    rc = mq_memcpy_d2h_staged(h, d, bytes, g_stream);
    g_xfer_s += now_s() - t0;
    return rc;
}

/* ---- column residency ---- */

static ColEntry* col_find(const Column* c) {
    for (int i = 0; i < g_ncols; i++)
        if (g_cols[i].col == c) return &g_cols[i];
    return NULL;
}

/* Free an entry's device copy. Work queued on g_stream may still read it and the
 * pool hands blocks out again at once, so the stream is drained first. */
static void col_drop(ColEntry* e) {
    mq_guard_release(e->guard);
    if (e->owned && e->dev) {
        mq_stream_sync(g_stream);
        mq_pool_free(e->dev);
    }
    *e = g_cols[--g_ncols];
}

static int col_usable(const ColEntry* e, const Column* c) {
    if (e->host != c->data || e->rows != c->row_count) return 0;
    if (!e->owned || e->op == g_op || e->rows == 0) return 1;
    return e->guard && mq_guard_clean(e->guard, e->host, e->rows * sizeof(int32_t));
}

/* ---- result shadows ---- */

static void shadow_drop(int i) {
    mq_guard_release(g_shadows[i].guard);
    if (g_shadows[i].dev) {
        mq_stream_sync(g_stream);
        mq_pool_free(g_shadows[i].dev);
    }
    g_shadow_bytes -= g_shadows[i].bytes;
    g_shadows[i] = g_shadows[--g_nshadows];
}

static size_t shadow_budget(void) { /* read per call: tests change it at run time */
    const char* env = getenv("MQ_SHADOW_MB");
    size_t mb = env ? (size_t)strtoull(env, NULL, 10) : 65536;
    return mb << 20;
}

/* LRU eviction down to the budget; what the current operator holds stays (the
 * budget may be exceeded for the duration of one call). */
static void shadow_make_room(size_t bytes) {
    while (g_nshadows >= MAX_SHADOWS || g_shadow_bytes + bytes > shadow_budget()) {
        int lru = -1;
        for (int i = 0; i < g_nshadows; i++)
            if (g_shadows[i].op != g_op && (lru < 0 || g_shadows[i].stamp < g_shadows[lru].stamp)) lru = i;
        if (lru < 0) break;
        shadow_drop(lru);
    }
}

/* Entries that only the operator that made them could use (no guard, or the
 * guard saw a write) are dropped at the start of the next operator. */
static void sweep(void) {
    for (int i = g_nshadows - 1; i >= 0; i--)
        if (g_shadows[i].op != g_op && !g_shadows[i].guard) shadow_drop(i);
    shadow_make_room(0); /* back within the budget the last operator may have exceeded */
    for (int i = g_ncols - 1; i >= 0; i--)
        if (g_cols[i].owned && g_cols[i].op != g_op && g_cols[i].rows && !g_cols[i].guard) col_drop(&g_cols[i]);
}

/* Device allocation for copies: on failure, evict what the current operator does
 * not hold (shadows LRU, then columns), release the pool's idle blocks, retry. */
static int dev_alloc(void** p, size_t bytes) {
    int rc = mq_pool_malloc(p, bytes);
    while (rc == MQ_ENOMEM) {
        int lru = -1;
        for (int i = 0; i < g_nshadows; i++)
            if (g_shadows[i].op != g_op && (lru < 0 || g_shadows[i].stamp < g_shadows[lru].stamp)) lru = i;
        if (lru >= 0) {
            shadow_drop(lru);
        } else {
            int c = -1;
            for (int i = 0; i < g_ncols; i++)
                if (g_cols[i].owned && g_cols[i].op != g_op) c = i;
            if (c < 0) {
                mq_stream_sync(g_stream);
                mq_trim();
                return mq_pool_malloc(p, bytes);
            }
            col_drop(&g_cols[c]);
        }
        mq_stream_sync(g_stream);
        mq_trim();
        rc = mq_pool_malloc(p, bytes);
    }
    return rc;
}

static int grow(void** buf, size_t* have, size_t need) {
    if (*have >= need && *buf) return 0;
    if (*buf) {
        mq_stream_sync(g_stream);
        mq_pool_free(*buf);
    }
    *buf = NULL;
    *have = 0;
    size_t want = need + need / 8 + 4096;
    int rc = dev_alloc(buf, want);
    if (rc) return rc;
    *have = want;
    return 0;
}

/* Register a device copy of a column's rows (made here: owned) and guard the host
 * rows it mirrors (armed here unless the caller armed it already: guard != ~0). */
static ColEntry* col_put_armed(Column* c, void* dev, uint64_t guard) {
    ColEntry* e = col_find(c);
    if (e) col_drop(e);
    if (g_ncols == MAX_COLS) {
        int victim = 0;
        for (int i = 0; i < g_ncols; i++)
            if (g_cols[i].op != g_op) victim = i;
        col_drop(&g_cols[victim]);
    }
    const size_t bytes = c->row_count * sizeof(int32_t);
    if (guard == ~(uint64_t)0) guard = bytes ? mq_guard_arm(c->data, bytes, MQ_GUARD_FILE) : 0;
    g_cols[g_ncols++] = (ColEntry){c, c->data, c->row_count, dev, 1, guard, g_op};
    return &g_cols[g_ncols - 1];
}

static ColEntry* col_put(Column* c, void* dev) { return col_put_armed(c, dev, ~(uint64_t)0); }

/* Arming a guard is one mprotect over the whole column, 11-22 ms per GB of a file
 * mapping (tools/payload_probe); it runs on a thread of its own while the upload
 * copies. The staged upload only reads the rows, so read-only pages do not disturb it,
 * and no store can reach them meanwhile: the caller is inside this operator. */
typedef struct {
    const void* p;
    size_t bytes;
    uint64_t guard;
} ArmArg;

static void* arm_thread(void* a) {
    ArmArg* x = (ArmArg*)a;
    x->guard = mq_guard_arm(x->p, x->bytes, MQ_GUARD_FILE);
    return NULL;
}

static int column_device(Column* c, const int32_t** d, Status* st) {
    const double t0 = now_s();
    ColEntry* e = col_find(c);
    if (e && col_usable(e, c)) {
        e->op = g_op;
        *d = (const int32_t*)e->dev;
        TRACE("column_device(hit)", t0);
        return 0;
    }
    if (e) col_drop(e);
    size_t bytes = c->row_count * sizeof(int32_t);
    void* dev = NULL;
    int rc = dev_alloc(&dev, bytes);
    if (rc) return fail(st, "column allocation", rc);
    ArmArg arm = {c->data, bytes, ~(uint64_t)0};
    pthread_t th;
    const int async = bytes >= ((size_t)64 << 20) && mq_guard_enabled() &&
                      pthread_create(&th, NULL, arm_thread, &arm) == 0;
    if (c->row_count && (rc = h2d(dev, c->data, bytes))) {
        if (async) {
            pthread_join(th, NULL);
            mq_guard_release(arm.guard);
        }
        mq_pool_free(dev);
        return fail(st, "column upload", rc);
    }
    TRACE("column h2d", t0);
    if (async) pthread_join(th, NULL);
    TRACE("column h2d + guard", t0);
    g_res.column_uploads++;
    g_res.column_bytes += bytes;
    *d = (const int32_t*)col_put_armed(c, dev, async ? arm.guard : ~(uint64_t)0)->dev;
    TRACE("column_device(upload)", t0);
    return 0;
}

static int shadow_find(const void* host) {
    for (int i = 0; i < g_nshadows; i++)
        if (g_shadows[i].host == host) return i;
    return -1;
}

/* Register dev (owned, n int32) as the shadow of host payload, with its guard
 * (0: single-use). */
static void shadow_put(const void* host, size_t n, void* dev, uint64_t guard) {
    int i = shadow_find(host);
    if (i >= 0) shadow_drop(i);
    size_t bytes = n * sizeof(int32_t);
    shadow_make_room(bytes);
    if (g_nshadows == MAX_SHADOWS) { /* everything is held by the current operator */
        int v = 0;
        for (int j = 0; j < g_nshadows; j++)
            if (g_shadows[j].stamp < g_shadows[v].stamp) v = j;
        shadow_drop(v);
    }
    g_shadows[g_nshadows++] = (ShadowEntry){host, n, bytes, dev, guard, ++g_stamp, g_op};
    g_shadow_bytes += bytes;
}

/* Device view of an int32 Result payload: its shadow while the payload is
 * unchanged (guarded, or uploaded by this same operator), else a fresh upload. */
static int result_device(const Result* r, const int32_t** d, Status* st) {
    const double t0 = now_s();
    const int32_t* h = (const int32_t*)r->payload;
    size_t n = r->num_tuples;
    int i = shadow_find(h);
    if (i >= 0) {
        ShadowEntry* e = &g_shadows[i];
        if (e->n == n && (e->op == g_op || n == 0 || (e->guard && mq_guard_clean(e->guard, h, n * 4)))) {
            e->stamp = ++g_stamp;
            e->op = g_op;
            *d = (const int32_t*)e->dev;
            TRACE("result_device(hit)", t0);
            return 0;
        }
        shadow_drop(i);
    }
    void* dev = NULL;
    int rc = dev_alloc(&dev, n * sizeof(int32_t));
    if (rc) return fail(st, "result allocation", rc);
    if (n && (rc = h2d(dev, h, n * sizeof(int32_t)))) {
        mq_pool_free(dev);
        return fail(st, "result upload", rc);
    }
    g_res.result_uploads++;
    g_res.result_bytes += n * sizeof(int32_t);
    shadow_put(h, n, dev, 0); /* not libmq's memory: single-use */
    *d = (const int32_t*)dev;
    return 0;
}

/* A result payload: plain malloc (the caller free()s it, client_context.c:31-90).
 * Large ones are advised onto transparent huge pages first: the D2H that fills a
 * fresh buffer otherwise takes one page fault per 4 KB (tools/d2h_paths: 40 MB in
 * 2.0 ms plain, 1.7 ms advised). */
static void* payload_alloc(size_t bytes) {
    void* p = malloc(bytes ? bytes : 1);
    if (!p) return NULL;
    mq_guard_forget_range((uintptr_t)p, bytes ? bytes : 1); /* a guard left on recycled memory */
    if (bytes >= ((size_t)8 << 20)) {
        const uintptr_t a = ((uintptr_t)p + 4095) & ~(uintptr_t)4095;
        const uintptr_t e = ((uintptr_t)p + bytes) & ~(uintptr_t)4095;
        if (e > a) (void)madvise((void*)a, e - a, MADV_HUGEPAGE);
    }
    return p;
}

static Result* new_result(DataType t, size_t n, void* payload) {
    Result* r = (Result*)malloc(sizeof(Result));
    r->num_tuples = n;
    r->data_type = t;
    r->payload = payload;
    return r;
}

/* Host Result from n int32 on the device (d_src, staging memory): D2H into a
 * malloc'd payload. When the payload can be guarded (glibc served it with mmap, so
 * free() unmaps it) an HBM shadow of it is kept for the operators that follow;
 * otherwise they upload it again. */
static Result* int_result_into(int32_t* host, const void* d_src, size_t n, Status* st) {
    double t0;
    const size_t bytes = n * sizeof(int32_t);
    /* small payloads are cheaper to upload again than to guard */
    const int keep = bytes >= SHADOW_MIN_BYTES && mq_guard_enabled() && mq_guard_chunk_ok(host);
    int rc;
    t0 = now_s();
    if (n && (rc = keep ? d2h_staged(host, d_src, bytes) : d2h(host, d_src, bytes))) {
        free(host);
        fail(st, "result download", rc);
        return NULL;
    }
    TRACE("result d2h", t0);
    t0 = now_s();
    const uint64_t guard = keep ? mq_guard_arm(host, bytes, MQ_GUARD_CHUNK) : 0;
    TRACE("guard_arm(payload)", t0);
    t0 = now_s();
    if (guard) {
        void* dev = NULL;
        if ((rc = dev_alloc(&dev, n * sizeof(int32_t))) ||
            (rc = mq_memcpy_d2d(dev, d_src, n * sizeof(int32_t), g_stream))) {
            mq_guard_release(guard);
            mq_pool_free(dev);
            free(host);
            fail(st, "shadow copy", rc);
            return NULL;
        }
        if (trace_on()) {
            mq_stream_sync(g_stream);
            TRACE("shadow alloc+d2d", t0);
            t0 = now_s();
        }
        shadow_put(host, n, dev, guard);
    }
    TRACE("shadow put", t0);
    st->code = OK;
    return new_result(INT, n, host);
}

static Result* int_result_from_device(const void* d_src, size_t n, Status* st) {
    double t0 = now_s();
    int32_t* host = (int32_t*)payload_alloc(n * sizeof(int32_t));
    TRACE("payload_alloc", t0);
    return int_result_into(host, d_src, n, st);
}

static int read_count(uint64_t* k, Status* st) {
    int rc = d2h(k, g_small, sizeof(uint64_t));
    if (rc) return fail(st, "count download", rc);
    return 0;
}

static int read_agg(mq_agg* a, Status* st) {
    int rc = d2h(a, g_small, sizeof(mq_agg));
    if (rc) return fail(st, "aggregate download", rc);
    return 0;
}

static int ensure_ws(size_t n_rows, Status* st) {
    int rc = grow(&g_ws, &g_ws_bytes, mq_scan_workspace_bytes(n_rows));
    if (rc) return fail(st, "workspace allocation", rc);
    rc = grow(&g_scratch, &g_scratch_bytes, (n_rows ? n_rows : 1) * sizeof(int32_t));
    if (rc) return fail(st, "staging allocation", rc);
    return 0;
}

/* ------------------------------------------------------------------ */
/* the reference API                                                  */
/* ------------------------------------------------------------------ */

/* query.c:26-36: the reference returns before logging anything. */
void log_result(Result* result) { (void)result; }

/* index.c:180-185 — weak: the reference's index.o definition takes precedence. */
__attribute__((weak)) bool should_use_index(Column* column, int low, int high) {
    (void)column;
    (void)low;
    (void)high;
    return true;
}

/* Segments of the pipelined select (0 = off): MQ_SELECT_SEGS, default 2, for columns of
 * at least MQ_SELECT_PIPE_MIN rows (default 2^26). Read per call (tests change them).
 * Config 3's select_column (1e9 rows, 1 %), 15 reps over 3 processes each, one box
 * (profiles/r05_api_segs_sweep.log): medians 2 segments 1.54 ms, 4 1.71, 6 2.10; one
 * kernel then the D2H 1.89 ms (profiles/r05_api_numa_segs.log). Past the first segment
 * the host side of the staged copy (first touch of the payload, memcpy out of the pinned
 * buffers, ~35 GB/s) is the bound, so more segments only add launches and copy calls. */
static int pipe_segments(size_t n) {
    const char* e = getenv("MQ_SELECT_SEGS");
    int segs = e ? atoi(e) : 2;
    if (segs < 0 || segs > 64) segs = 0;
    const char* m = getenv("MQ_SELECT_PIPE_MIN");
    const size_t min_rows = m ? (size_t)strtoull(m, NULL, 10) : ((size_t)1 << 26);
    return segs >= 2 && n >= min_rows && mq_guard_enabled() ? segs : 0;
}

/* select_column_scan for long columns (round 5): the payload's size is unknown until the
 * select ends, so the one-kernel path pays select, then the whole D2H. Here the select
 * runs in `segs` row segments and segment s's positions go down while segments s+1..
 * scan (mq_select_positions_download). Their host destination must exist before K is
 * known: the payload is malloc'd for all n rows (an mmap'd chunk: address space, no
 * pages until written; advised onto huge pages), filled at the running offset, and
 * shrunk to K rows by realloc afterwards (glibc remaps an mmapped chunk in place, so it
 * stays guardable). The HBM shadow is the segments' pieces copied together on the device. */
static Result* scan_positions_piped(const int32_t* dcol, size_t n, int segs, int* low_pointer, int* high_pointer,
                                    int32_t* host, Status* st) {
    double t0 = now_s();
    uint64_t seg[65], rows[65];
    int rc = mq_stream_sync(g_stream);
    const double tx = now_s();
    if (!rc)
        rc = mq_select_positions_download(dcol, n, low_pointer != NULL, low_pointer ? *low_pointer : 0,
                                          high_pointer != NULL, high_pointer ? *high_pointer : 0, segs,
                                          (int32_t*)g_scratch, host, seg, rows, g_ws, g_ws_bytes, g_stream);
    g_xfer_s += now_s() - tx; /* (the kernels overlap the copies: counted as transfer) */
    if (rc) {
        free(host);
        fail(st, "select_column_scan", rc);
        return NULL;
    }
    TRACE("select segments + d2h", t0);
    size_t k = 0;
    for (int g = 0; g < segs; g++) k += (size_t)seg[g];
    const size_t bytes = k * sizeof(int32_t);
    int32_t* h2 = (int32_t*)realloc(host, bytes ? bytes : 1);
    if (h2) host = h2;
    const int keep = bytes >= SHADOW_MIN_BYTES && mq_guard_chunk_ok(host);
    const uint64_t guard = keep ? mq_guard_arm(host, bytes, MQ_GUARD_CHUNK) : 0;
    if (guard) {
        void* dev = NULL;
        rc = dev_alloc(&dev, bytes);
        size_t off = 0;
        for (int g = 0; g < segs && !rc; g++) {
            rc = mq_memcpy_d2d((int32_t*)dev + off, (const int32_t*)g_scratch + rows[g], seg[g] * sizeof(int32_t),
                               g_stream);
            off += seg[g];
        }
        if (rc) {
            mq_guard_release(guard);
            mq_pool_free(dev);
            free(host);
            fail(st, "shadow copy", rc);
            return NULL;
        }
        shadow_put(host, k, dev, guard);
    }
    TRACE("shrink + guard + shadow", t0);
    st->code = OK;
    return new_result(INT, k, host);
}

/* query.c:92-137 (the body; shared_select calls it inside its own operator) */
static Result* scan_positions(Column* column, int* low_pointer, int* high_pointer, Status* ret_status) {
    if (shard_wants(column)) return shard_select(column, low_pointer, high_pointer, ret_status);
    size_t n = column->row_count;
    const int32_t* dcol;
    if (column_device(column, &dcol, ret_status) || ensure_ws(n, ret_status)) return NULL;
    const int segs = pipe_segments(n);
    if (segs) {
        /* the n-row payload is address space only; where even that is refused (RLIMIT_AS,
         * strict overcommit) the one-kernel path below needs just K rows */
        int32_t* host = (int32_t*)payload_alloc(n * sizeof(int32_t));
        if (host) return scan_positions_piped(dcol, n, segs, low_pointer, high_pointer, host, ret_status);
    }
    const double t0 = now_s();
    int rc = mq_select_positions(dcol, NULL, n, low_pointer != NULL, low_pointer ? *low_pointer : 0,
                                 high_pointer != NULL, high_pointer ? *high_pointer : 0,
                                 (int32_t*)g_scratch, (uint64_t*)g_small, g_ws, g_ws_bytes, g_stream);
    if (rc) {
        fail(ret_status, "select_column_scan", rc);
        return NULL;
    }
    uint64_t k;
    if (read_count(&k, ret_status)) return NULL;
    TRACE("select kernel+count", t0);
    return int_result_from_device(g_scratch, (size_t)k, ret_status);
}

Result* select_column_scan(Column* column, int* low_pointer, int* high_pointer, Status* ret_status) {
    if (op_begin(ret_status)) return NULL;
    return scan_positions(column, low_pointer, high_pointer, ret_status);
}

/* ---- sorted-index residency: the index arrays' HBM copies ---- */

static void idx_drop(IndexEntry* e) {
    mq_guard_release(e->guard_v);
    mq_guard_release(e->guard_p);
    mq_stream_sync(g_stream);
    mq_pool_free(e->d_values);
    mq_pool_free(e->d_positions);
    *e = g_idx[--g_nidx];
}

static int idx_usable(const IndexEntry* e, const ColumnIndex* ix, size_t n) {
    if (e->values != ix->values || e->positions != ix->positions || e->rows != n) return 0;
    if (e->op == g_op || n == 0) return 1;
    return e->guard_v && e->guard_p && mq_guard_clean(e->guard_v, e->values, n * sizeof(int32_t)) &&
           mq_guard_clean(e->guard_p, e->positions, n * sizeof(size_t));
}

/* guarded: the arrays are libmq's own malloc'd memory (build_index) */
static IndexEntry* idx_put(ColumnIndex* ix, size_t n, void* d_values, void* d_positions, int guarded) {
    for (int i = 0; i < g_nidx; i++)
        if (g_idx[i].index == ix) {
            idx_drop(&g_idx[i]);
            break;
        }
    if (g_nidx == MAX_INDEXES) idx_drop(&g_idx[0]);
    uint64_t gv = 0, gp = 0;
    if (guarded && n) {
        gv = mq_guard_arm(ix->values, n * sizeof(int32_t), MQ_GUARD_CHUNK);
        gp = mq_guard_arm(ix->positions, n * sizeof(size_t), MQ_GUARD_CHUNK);
    }
    g_idx[g_nidx++] = (IndexEntry){ix, ix->values, ix->positions, n, d_values, d_positions, gv, gp, g_op};
    return &g_idx[g_nidx - 1];
}

/* query.c:165-198: sorted-index select, in value order. */
Result* select_column_sorted_index(Column* column, int low, int high, Status* ret_status) {
    if (op_begin(ret_status)) return NULL;
    ColumnIndex* ix = column->index;
    size_t n = column->row_count;
    IndexEntry* e = NULL;
    for (int i = 0; i < g_nidx; i++)
        if (g_idx[i].index == ix) e = &g_idx[i];
    if (e && !idx_usable(e, ix, n)) {
        idx_drop(e);
        e = NULL;
    }
    if (!e) {
        void *dv = NULL, *dp = NULL;
        int rc;
        if ((rc = dev_alloc(&dv, n * sizeof(int32_t))) || (rc = dev_alloc(&dp, n * sizeof(uint64_t))) ||
            (n && (rc = h2d(dv, ix->values, n * sizeof(int32_t)))) ||
            (n && (rc = h2d(dp, ix->positions, n * sizeof(uint64_t))))) {
            mq_pool_free(dv);
            mq_pool_free(dp);
            fail(ret_status, "index upload", rc);
            return NULL;
        }
        e = idx_put(ix, n, dv, dp, 0); /* the caller's arrays: single-use */
    }
    e->op = g_op;
    if (ensure_ws(n, ret_status)) return NULL;
    int rc = mq_index_select((const int32_t*)e->d_values, (const uint64_t*)e->d_positions, n, low, high,
                             (int32_t*)g_scratch, (uint64_t*)g_small, g_stream);
    if (rc) {
        fail(ret_status, "select_column_sorted_index", rc);
        return NULL;
    }
    uint64_t k;
    if (read_count(&k, ret_status)) return NULL;
    return int_result_from_device(g_scratch, (size_t)k, ret_status);
}

/* query.c:203-220: same dispatch as the reference (clustered or indexed columns
 * take the sorted-index path, which dereferences both bounds as it does). */
Result* select_column(Column* column, int* low_pointer, int* high_pointer, Status* ret_status) {
    if (column->clustered)
        return select_column_sorted_index(column, *low_pointer, *high_pointer, ret_status);
    if (column->has_index && should_use_index(column, *low_pointer, *high_pointer))
        return select_column_sorted_index(column, *low_pointer, *high_pointer, ret_status);
    return select_column_scan(column, low_pointer, high_pointer, ret_status);
}

/* query.c:38-86 */
Result* select_result(Result* column, Result* prev_position, int* low_pointer, int* high_pointer,
                      Status* ret_status) {
    if (op_begin(ret_status)) return NULL;
    size_t n = column->num_tuples;
    const int32_t *dval, *dpos;
    if (result_device(column, &dval, ret_status) || result_device(prev_position, &dpos, ret_status) ||
        ensure_ws(n, ret_status))
        return NULL;
    int rc = mq_select_positions(dval, dpos, n, low_pointer != NULL, low_pointer ? *low_pointer : 0,
                                 high_pointer != NULL, high_pointer ? *high_pointer : 0,
                                 (int32_t*)g_scratch, (uint64_t*)g_small, g_ws, g_ws_bytes, g_stream);
    if (rc) {
        fail(ret_status, "select_result", rc);
        return NULL;
    }
    uint64_t k;
    if (read_count(&k, ret_status)) return NULL;
    return int_result_from_device(g_scratch, (size_t)k, ret_status);
}

/* query.c:223-243 */
Result* fetch_column(Column* column, Result* position_result, Status* ret_status) {
    if (op_begin(ret_status)) return NULL;
    if (shard_wants(column)) {
        Result* r = NULL;
        const int h = shard_fetch(column, position_result, &r, ret_status);
        if (h) return h > 0 ? r : NULL;
    }
    size_t k = position_result->num_tuples;
    const int32_t *dcol, *dpos;
    if (column_device(column, &dcol, ret_status) || result_device(position_result, &dpos, ret_status) ||
        ensure_ws(k, ret_status))
        return NULL;
    /* K is known before the gather runs: the payload's pages fault in while it does.
     * Only a payload that takes the staged copy (which waits for the helper threads)
     * is handed to them; the plain copy would return with them still at work. */
    const size_t bytes = k * sizeof(int32_t);
    int32_t* host = (int32_t*)payload_alloc(bytes);
    if (!host) {
        fail(ret_status, "fetch_column payload", MQ_ENOMEM);
        return NULL;
    }
    const int staged = bytes >= SHADOW_MIN_BYTES && mq_guard_enabled() && mq_guard_chunk_ok(host);
    if (staged) mq_host_prefault(host, bytes);
    int rc = mq_fetch(dcol, dpos, k, (int32_t*)g_scratch, g_stream);
    if (rc) {
        fail(ret_status, "fetch_column", rc);
        if (staged) mq_host_prefault_wait();
        free(host);
        return NULL;
    }
    return int_result_into(host, g_scratch, k, ret_status);
}

static int reduce_result(Result* r, mq_agg* a, Status* st) {
    if (op_begin(st)) return -1;
    const int h = shard_reduce_result(r, a, st);
    if (h) return h > 0 ? 0 : -1;
    const int32_t* d;
    if (result_device(r, &d, st) || ensure_ws(0, st)) return -1;
    int rc = mq_reduce(d, r->num_tuples, (mq_agg*)g_small, g_ws, g_ws_bytes, g_stream);
    if (rc) return fail(st, "reduce", rc);
    return read_agg(a, st);
}

/* query.c:306-323: (double)int64_sum / (double)n; n == 0 gives NaN as there. */
Result* average(Result* column, Status* ret_status) {
    mq_agg a;
    if (reduce_result(column, &a, ret_status)) return NULL;
    double* out = (double*)malloc(sizeof(double));
    *out = (double)a.sum / (double)column->num_tuples;
    ret_status->code = OK;
    return new_result(DOUBLE, 1, out);
}

/* query.c:325-354: RESULT or COLUMN, int64 sum. */
Result* sum(GeneralizedColumn* column, Status* ret_status) {
    mq_agg a;
    if (column->column_type == RESULT) {
        if (reduce_result(column->column_pointer.result, &a, ret_status)) return NULL;
    } else {
        if (op_begin(ret_status)) return NULL;
        Column* c = column->column_pointer.column;
        if (shard_wants(c)) {
            if (shard_reduce_column(c, &a, ret_status)) return NULL;
            long* out = (long*)malloc(sizeof(long));
            *out = (long)a.sum;
            ret_status->code = OK;
            return new_result(LONG, 1, out);
        }
        const int32_t* d;
        if (column_device(c, &d, ret_status) || ensure_ws(0, ret_status)) return NULL;
        int rc = mq_reduce(d, c->row_count, (mq_agg*)g_small, g_ws, g_ws_bytes, g_stream);
        if (rc) {
            fail(ret_status, "sum(column)", rc);
            return NULL;
        }
        if (read_agg(&a, ret_status)) return NULL;
    }
    long* out = (long*)malloc(sizeof(long));
    *out = (long)a.sum;
    ret_status->code = OK;
    return new_result(LONG, 1, out);
}

static Result* elementwise(Result* a, Result* b, Status* st, int is_sub) {
    if (op_begin(st)) return NULL;
    size_t n = a->num_tuples;
    const int32_t *da, *db;
    if (result_device(a, &da, st) || result_device(b, &db, st) || ensure_ws(n, st)) return NULL;
    if (b->num_tuples < n) {
        fprintf(stderr, "libmq: %s: second operand has %zu < %zu rows\n", is_sub ? "sub" : "add",
                b->num_tuples, n);
        st->code = ERROR;
        return NULL;
    }
    int rc = is_sub ? mq_sub(da, db, n, (int32_t*)g_scratch, g_stream)
                    : mq_add(da, db, n, (int32_t*)g_scratch, g_stream);
    if (rc) {
        fail(st, is_sub ? "sub" : "add", rc);
        return NULL;
    }
    return int_result_from_device(g_scratch, n, st);
}

/* query.c:356-372 */
Result* add(Result* column_one, Result* column_two, Status* ret_status) {
    return elementwise(column_one, column_two, ret_status, 0);
}

/* query.c:374-390 */
Result* sub(Result* column_one, Result* column_two, Status* ret_status) {
    return elementwise(column_one, column_two, ret_status, 1);
}

/* query.c:392-415. The reference reads payload[0] of an empty result (garbage);
 * libmq returns INT_MAX for an empty input. */
Result* min(Result* column, Status* ret_status) {
    mq_agg a;
    if (reduce_result(column, &a, ret_status)) return NULL;
    int* out = (int*)malloc(sizeof(int));
    *out = a.min;
    ret_status->code = OK;
    return new_result(INT, 1, out);
}

/* query.c:417-437 (empty input: INT_MIN, see min) */
Result* max(Result* column, Status* ret_status) {
    mq_agg a;
    if (reduce_result(column, &a, ret_status)) return NULL;
    int* out = (int*)malloc(sizeof(int));
    *out = a.max;
    ret_status->code = OK;
    return new_result(INT, 1, out);
}

/* query.c:496-583. As in the reference, every query reads `column` and uses its
 * low/high fields as given (has_low/has_high are not consulted, query.c:474).
 * Positions per query are ascending, which is what the reference's thread-order
 * concatenation (query.c:563-574) produces. Two streaming passes over the column
 * serve all queries of a chunk (up to 256): count -> exact allocation -> write; each
 * query's device output becomes its result's HBM shadow. */
Result** shared_select(SelectOperator* operators, int query_count, Column* column, Status* ret_status) {
    if (op_begin(ret_status)) return NULL;
    size_t n = column->row_count;
    if (query_count > 1 && shard_wants(column)) return shard_shared_select(operators, query_count, column, ret_status);
    const int32_t* dcol = NULL;
    if (query_count > 1 && column_device(column, &dcol, ret_status)) return NULL;
    Result** out = (Result**)calloc((size_t)(query_count > 0 ? query_count : 1), sizeof(Result*));
    /* one query: the ordered-compaction pass. From two the shared pass is cheaper (round
     * 5: Q = 2 of 0.1 % 0.79 ms on the device against 2 x 0.68 ms; until round 4 the
     * ballot kernels below Q = 12 made it 0.96 and the split was at Q = 3) */
    if (query_count <= 1) {
        for (int j = 0; j < query_count; j++) {
            int lo = operators[j].low, hi = operators[j].high;
            if (!(out[j] = scan_positions(column, &lo, &hi, ret_status))) {
                for (int i = 0; i < j; i++) {
                    free(out[i]->payload);
                    free(out[i]);
                }
                free(out);
                ret_status->code = ERROR;
                return NULL;
            }
        }
        ret_status->code = OK;
        return out;
    }
    int done = 0;
    for (int q0 = 0; q0 < query_count; q0 += 256) {
        int q = query_count - q0 < 256 ? query_count - q0 : 256;
        int32_t lows[256], highs[256];
        uint64_t k[256];
        void* dev[256] = {0};
        for (int j = 0; j < q; j++) {
            lows[j] = operators[q0 + j].low;
            highs[j] = operators[q0 + j].high;
        }
        int rc = grow(&g_ws, &g_ws_bytes, mq_shared_select_workspace_bytes(n, q));
        if (!rc) rc = mq_shared_select_count(dcol, n, lows, highs, q, k, g_ws, g_ws_bytes, g_stream);
        for (int j = 0; !rc && j < q; j++) rc = dev_alloc(&dev[j], (size_t)k[j] * sizeof(int32_t));
        if (!rc) rc = mq_shared_select_write(g_ws, (int32_t* const*)dev, g_stream);
        for (int j = 0; !rc && j < q; j++) {
            const size_t bytes = (size_t)k[j] * sizeof(int32_t);
            int32_t* host = (int32_t*)payload_alloc(bytes);
            const int keep = bytes >= SHADOW_MIN_BYTES && mq_guard_enabled() && mq_guard_chunk_ok(host);
            if (k[j] && (rc = keep ? d2h_staged(host, dev[j], bytes) : d2h(host, dev[j], bytes))) {
                free(host);
                break;
            }
            const uint64_t guard = keep ? mq_guard_arm(host, bytes, MQ_GUARD_CHUNK) : 0;
            if (guard) {
                shadow_put(host, (size_t)k[j], dev[j], guard);
                dev[j] = NULL; /* owned by the shadow now */
            }
            out[q0 + j] = new_result(INT, (size_t)k[j], host);
            done = q0 + j + 1;
        }
        mq_stream_sync(g_stream);
        for (int j = 0; j < q; j++) mq_pool_free(dev[j]);
        if (rc) {
            fail(ret_status, "shared_select", rc);
            for (int j = 0; j < done; j++) {
                free(out[j]->payload);
                free(out[j]);
            }
            free(out);
            return NULL;
        }
    }
    ret_status->code = OK;
    return out;
}

static Result** join_pairs(const int32_t* d1, const int32_t* dp1, size_t n1, const int32_t* d2,
                           const int32_t* dp2, size_t n2, int swap, Status* st) {
    mq_join* jn = NULL;
    uint64_t m = 0;
    void *o1 = NULL, *o2 = NULL;
    int rc = mq_join_build(d1, dp1, n1, &jn, g_stream);
    if (!rc) rc = mq_join_probe(jn, d2, n2, &m, g_stream);
    if (!rc && m) {
        if (!(rc = mq_pool_malloc(&o1, m * sizeof(int32_t))) && !(rc = mq_pool_malloc(&o2, m * sizeof(int32_t))))
            rc = mq_join_write(jn, dp2, (int32_t*)o1, (int32_t*)o2, g_stream);
    }
    mq_join_free(jn);
    if (rc) {
        mq_pool_free(o1);
        mq_pool_free(o2);
        fail(st, "hash_join", rc);
        return NULL;
    }
    Result** out = (Result**)malloc(2 * sizeof(Result*));
    out[0] = int_result_from_device(swap ? o2 : o1, (size_t)m, st);
    out[1] = int_result_from_device(swap ? o1 : o2, (size_t)m, st);
    mq_stream_sync(g_stream);
    mq_pool_free(o1);
    mq_pool_free(o2);
    if (!out[0] || !out[1]) {
        st->code = ERROR;
        return NULL;
    }
    st->code = OK;
    return out;
}

/* query.c:652-696: build on column_one, probe with column_two; pairs in
 * probe-major, build-insertion order. */
Result** hash_join(Result* column_one, Result* position_one, Result* column_two, Result* position_two,
                   Status* ret_status) {
    if (op_begin(ret_status)) return NULL;
    if (shard_join_wants(column_one->num_tuples, column_two->num_tuples)) /* key-partitioned, DESIGN.md §6 */
        return shard_hash_join(column_one, position_one, column_two, position_two, 0, ret_status);
    const int32_t *d1, *dp1, *d2, *dp2;
    if (result_device(column_one, &d1, ret_status) || result_device(position_one, &dp1, ret_status) ||
        result_device(column_two, &d2, ret_status) || result_device(position_two, &dp2, ret_status))
        return NULL;
    return join_pairs(d1, dp1, column_one->num_tuples, d2, dp2, column_two->num_tuples, 0, ret_status);
}

/* query.c:585-650: outer column_one x inner column_two, outer-major with inner
 * ascending — exactly a hash join that builds on the inner side (insertion
 * order = inner order) and probes with the outer side, outputs swapped. */
Result** nested_loop_join(Result* column_one, Result* position_one, Result* column_two,
                          Result* position_two, Status* ret_status) {
    if (op_begin(ret_status)) return NULL;
    if (shard_join_wants(column_two->num_tuples, column_one->num_tuples))
        return shard_hash_join(column_two, position_two, column_one, position_one, 1, ret_status);
    const int32_t *d1, *dp1, *d2, *dp2;
    if (result_device(column_one, &d1, ret_status) || result_device(position_one, &dp1, ret_status) ||
        result_device(column_two, &d2, ret_status) || result_device(position_two, &dp2, ret_status))
        return NULL;
    return join_pairs(d2, dp2, column_two->num_tuples, d1, dp1, column_one->num_tuples, 1, ret_status);
}

/* query.c:245-304: host string formatting (stays on the CPU).
 * Same formats and separators; an all-empty input yields "" (the reference
 * returns an unterminated malloc(0) buffer there, query.c:253). */
/* Large INT results are formatted on the GPU from their HBM copy (mq_format_int32:
 * per-value lengths, a scan, a digit-writing pass) and copied back as text; the
 * bytes equal the reference's sprintf loop. Other results stay on the host. */
#define PRINT_GPU_MIN_TUPLES 32768 /* MQ_PRINT_GPU_MIN overrides */

static size_t print_gpu_min(void) {
    static size_t v = 0;
    if (!v) {
        const char* e = getenv("MQ_PRINT_GPU_MIN");
        v = (e && atoll(e) > 0) ? (size_t)atoll(e) : PRINT_GPU_MIN_TUPLES;
    }
    return v;
}

static void* g_print_out;
static void* g_print_ws;
static size_t g_print_out_cap, g_print_ws_cap;

static int print_gpu(const Result* r, char* dst, size_t* len, Status* st) {
    const uint64_t n = r->num_tuples;
    const int32_t* d;
    if (result_device(r, &d, st)) return -1;
    const size_t need_out = (size_t)n * 12, need_ws = mq_format_workspace_bytes(n);
    int rc;
    if (g_print_out_cap < need_out) {
        mq_pool_free(g_print_out);
        g_print_out = NULL;
        g_print_out_cap = 0;
        if ((rc = mq_malloc(&g_print_out, need_out))) return fail(st, "print: device buffer", rc);
        g_print_out_cap = need_out;
    }
    if (g_print_ws_cap < need_ws) {
        mq_pool_free(g_print_ws);
        g_print_ws = NULL;
        g_print_ws_cap = 0;
        if ((rc = mq_malloc(&g_print_ws, need_ws))) return fail(st, "print: workspace", rc);
        g_print_ws_cap = need_ws;
    }
    uint64_t h_len = 0;
    if ((rc = mq_format_int32(d, n, (char*)g_print_out, &h_len, g_print_ws, g_print_ws_cap, g_stream)) ||
        (rc = mq_memcpy_d2h(dst, g_print_out, h_len, g_stream)) || (rc = mq_stream_sync(g_stream)))
        return fail(st, "print: mq_format_int32", rc);
    *len = (size_t)h_len;
    return 0;
}

char* print(Result** results, int result_num, Status* ret_status) {
    size_t total = 0;
    int on_gpu = 0;
    for (int i = 0; i < result_num; i++) {
        total += results[i]->num_tuples;
        on_gpu |= results[i]->data_type == INT && results[i]->num_tuples >= print_gpu_min();
    }
    if (on_gpu && op_begin(ret_status)) return NULL;
    size_t cap = total * 24 + (size_t)result_num + 1;
    char* s = (char*)malloc(cap);
    size_t at = 0;
    s[0] = '\0';
    for (int i = 0; i < result_num; i++) {
        Result* r = results[i];
        if (i > 0) at += (size_t)snprintf(s + at, cap - at, ",");
        if (r->data_type == INT && r->num_tuples >= print_gpu_min()) {
            size_t len = 0;
            if (print_gpu(r, s + at, &len, ret_status)) {
                free(s);
                return NULL;
            }
            at += len;
            s[at] = '\0';
            continue;
        }
        for (size_t j = 0; j < r->num_tuples; j++) {
            switch (r->data_type) {
                case INT: at += (size_t)snprintf(s + at, cap - at, "%d", ((int*)r->payload)[j]); break;
                case LONG: at += (size_t)snprintf(s + at, cap - at, "%ld", ((long*)r->payload)[j]); break;
                case FLOAT: at += (size_t)snprintf(s + at, cap - at, "%.2f", (double)((float*)r->payload)[j]); break;
                case DOUBLE: at += (size_t)snprintf(s + at, cap - at, "%.2f", ((double*)r->payload)[j]); break;
            }
            if (j != r->num_tuples - 1) at += (size_t)snprintf(s + at, cap - at, "\n");
        }
    }
    ret_status->code = OK;
    return s;
}

/* ------------------------------------------------------------------ */
/* load path: db_manager.c:240-322 load_db + :164-199 insert_row      */
/* ------------------------------------------------------------------ */

/* ---- J4: hashset.c (src/hashset.c:11-65) ----
 * The reference's linear-probing int32 set, kept as its own host table so that
 * code written against hashset.h behaves the same; defined behaviour where the
 * reference has none (include/mq_query.h). get_hashset_elements lists large
 * tables on the GPU (mq_hashset_elements: ordered compaction of the nonzero
 * slots, in slot order). */
__attribute__((weak)) int hash(int key, int size) { return key % size; }  /* multimap.c:60-63 */

static int hs_home(int key, int size) {
    int idx = key % size;
    return idx < 0 ? idx + size : idx;  /* the reference reads keys[negative] here */
}

hashset* create_hashset(int size) {
    hashset* set = (hashset*)malloc(sizeof(hashset));
    set->keys = (int*)calloc(size > 0 ? (size_t)size : 1, sizeof(int));  /* reference: malloc */
    set->size = size;
    return set;
}

void free_hashset(hashset* set) {
    if (!set) return;
    free(set->keys);
    free(set);
}

void insert_hashset(hashset* set, int key) {
    if (!set || set->size <= 0) return;
    int idx = hs_home(key, set->size);
    for (int step = 0; set->keys[idx] != 0 && set->keys[idx] != key; step++) {
        if (step + 1 >= set->size) return;  /* full without the key: the reference spins */
        idx = idx + 1 == set->size ? 0 : idx + 1;
    }
    set->keys[idx] = key;
}

bool lookup_hashset(hashset* set, int key) {
    if (!set || set->size <= 0) return false;
    int idx = hs_home(key, set->size);
    for (int step = 0; set->keys[idx] != 0 && set->keys[idx] != key; step++) {
        if (step + 1 >= set->size) return false;
        idx = idx + 1 == set->size ? 0 : idx + 1;
    }
    return set->keys[idx] != 0;
}

static size_t hashset_gpu_min(void) {
    const char* e = getenv("MQ_HASHSET_GPU_MIN");
    return e ? (size_t)strtoull(e, NULL, 10) : (size_t)32768;
}

Result* get_hashset_elements(hashset* set) {
    const size_t size = set && set->size > 0 ? (size_t)set->size : 0;
    if (size >= hashset_gpu_min() && ready(NULL) == 0) {
        Status st = {OK, NULL};
        void* d_tab = NULL;
        int rc = mq_malloc(&d_tab, 2 * size * sizeof(int32_t));  /* table, then elements */
        if (!rc && !(rc = ensure_ws(size, &st)) && !(rc = h2d(d_tab, set->keys, size * sizeof(int32_t)))) {
            int32_t* d_out = (int32_t*)d_tab + size;
            uint64_t k = 0;
            if (!(rc = mq_hashset_elements((const int32_t*)d_tab, size, d_out, (uint64_t*)g_small, g_ws,
                                           g_ws_bytes, g_stream)) &&
                !(rc = read_count(&k, &st))) {
                int32_t* host = (int32_t*)malloc((k ? k : 1) * sizeof(int32_t));
                if (!(rc = k ? d2h(host, d_out, k * sizeof(int32_t)) : 0)) {
                    mq_pool_free(d_tab);
                    return new_result(INT, k, host);
                }
                free(host);
            }
        }
        if (d_tab) mq_pool_free(d_tab);
        fail(NULL, "get_hashset_elements on the GPU", rc ? rc : MQ_EHIP);
        return NULL;
    }
    size_t count = 0;
    for (size_t i = 0; i < size; i++) count += set->keys[i] != 0;
    int32_t* elements = (int32_t*)malloc((count ? count : 1) * sizeof(int32_t));  /* reference: 16 B */
    count = 0;
    for (size_t i = 0; i < size; i++)
        if (set->keys[i] != 0) elements[count++] = set->keys[i];
    return new_result(INT, count, elements);
}

/* The server's own capacity helpers (db_manager.c:430 save_data, :736 start_data),
 * resolved from the executable that links libmq; NULL when none does. */
extern void save_data(Table* table, Column* column, Status* ret_status) __attribute__((weak));
extern void start_data(Db* db, Table* table, Column* column, Status* ret_status)
    __attribute__((weak));

static void load_fail(Status* st, const char* msg) {
    fprintf(stderr, "libmq: load_db: %s\n", msg);
    st->code = ERROR;
    st->error_message = (char*)msg;
}

/* insert_row's growth (db_manager.c:168-187): the capacity doubles whenever a row
 * arrives at a full table, so after the load it is the first table_length * 2^k
 * that holds every row; reached here in one remap instead of k. */
static int grow_table(Db* db, Table* t, size_t total, Status* st) {
    size_t len = t->table_length;
    if (len == 0) return -1;
    while (len < total) len *= 2;
    if (len == t->table_length) return 0;
    if (!save_data || !start_data) {
        load_fail(st, "the table must grow and the server's save_data/start_data are not linked");
        return -1;
    }
    for (size_t i = 0; i < t->col_count; i++) {
        Status s = {OK, NULL};
        save_data(t, t->columns + i, &s);
        if (s.code != OK) return -1;
    }
    t->table_length = len;
    for (size_t i = 0; i < t->col_count; i++) {
        Status s = {OK, NULL};
        start_data(db, t, t->columns + i, &s);
        if (s.code != OK) return -1;
    }
    return 0;
}

void load_db(Db* db, const char* path, Status* ret_status) {
    ret_status->code = OK;
    int fd = open(path, O_RDONLY);
    if (fd < 0) {
        ret_status->code = ERROR;
        ret_status->error_message = "Failed to open file to load db";
        return;
    }
    struct stat sb;
    if (fstat(fd, &sb) != 0 || sb.st_size == 0) {
        close(fd);
        load_fail(ret_status, "empty or unreadable file");
        return;
    }
    const size_t n = (size_t)sb.st_size;
    const char* text = mmap(NULL, n, PROT_READ, MAP_PRIVATE, fd, 0);
    close(fd);
    if (text == MAP_FAILED) {
        load_fail(ret_status, "mmap failed");
        return;
    }
    /* header: fgets(line, MAX_LINE_SIZE) then strsep(".") twice (:263-268) */
    char line[1024];
    size_t h = 0;
    while (h < n && h < 1023) {
        line[h] = text[h];
        if (line[h++] == '\n') break;
    }
    line[h] = '\0';
    char* temp = line;
    const char* db_name = strsep(&temp, ".");
    const char* table_name = strsep(&temp, ".");
    Table* table = NULL;
    if (db && db_name && table_name && strcmp(db->name, db_name) == 0)
        for (size_t i = 0; i < db->tables_size; i++)
            if (!strcmp(db->tables[i].name, table_name)) {
                table = db->tables + i;
                break;
            }
    if (!table) { /* :273-295 */
        munmap((void*)text, n);
        ret_status->code = ERROR;
        return;
    }
    const int ncols = (int)table->col_count;
    const char* data = text + h;
    const size_t dn = n - h;
    void *d_text = NULL, *d_ws = NULL, *d_mm = NULL;
    void* dcol[1024] = {NULL};
    int32_t* dparse[1024];
    int32_t mm[2048];
    int rc = 0;
    if (table->col_count > 1024) {
        load_fail(ret_status, "more than 1024 columns");
        goto out;
    }
    if (op_begin(ret_status)) goto out;
    const size_t wsb = mq_csv_workspace_bytes(dn, ncols);
    if ((rc = mq_malloc(&d_text, dn ? dn : 16)) || (rc = mq_malloc(&d_ws, wsb)) ||
        (rc = mq_malloc(&d_mm, 8 * (size_t)(ncols ? ncols : 1)))) {
        fail(ret_status, "load_db allocation", rc);
        goto out;
    }
    if (dn && (rc = h2d(d_text, data, dn))) {
        fail(ret_status, "load_db upload", rc);
        goto out;
    }
    uint64_t rows = 0;
    if ((rc = mq_csv_count_rows(d_text, dn, ncols, &rows, d_ws, wsb, g_stream))) {
        fail(ret_status, "mq_csv_count_rows", rc);
        goto out;
    }
    const size_t old = table->row_count, total = old + rows;
    /* HBM copies of the whole columns: the resident rows, then the parsed ones */
    for (int j = 0; j < ncols; j++) {
        Column* c = table->columns + j;
        if ((rc = mq_malloc(&dcol[j], (total ? total : 1) * 4))) {
            fail(ret_status, "load_db column allocation", rc);
            goto out;
        }
        ColEntry* e = col_find(c);
        if (old && e && col_usable(e, c))
            rc = mq_memcpy_d2d(dcol[j], e->dev, old * 4, g_stream);
        else if (old)
            rc = h2d(dcol[j], c->data, old * 4);
        if (rc) {
            fail(ret_status, "load_db column copy", rc);
            goto out;
        }
        dparse[j] = (int32_t*)dcol[j] + old;
    }
    if ((rc = mq_csv_parse_int32(d_text, dn, ncols, dparse, rows, d_mm, d_ws, wsb, g_stream))) {
        fail(ret_status, "mq_csv_parse_int32", rc);
        goto out;
    }
    if (rows && grow_table(db, table, total, ret_status)) {
        ret_status->code = ERROR;
        goto out;
    }
    if (ncols && (rc = d2h(mm, d_mm, 8 * (size_t)ncols))) {
        fail(ret_status, "load_db min/max", rc);
        goto out;
    }
    for (int j = 0; j < ncols; j++) {
        Column* c = table->columns + j;
        mq_guard_forget_range((uintptr_t)c->data, total * 4); /* libmq writes the rows in place */
        if (rows && (rc = d2h(c->data + old, dparse[j], rows * 4))) {
            fail(ret_status, "load_db column download", rc);
            goto out;
        }
        c->row_count += rows;
        if (rows) { /* insert_row :193-194 */
            c->max = c->max > mm[2 * j + 1] ? c->max : mm[2 * j + 1];
            c->min = c->min < mm[2 * j] ? c->min : mm[2 * j];
        }
        col_put(c, dcol[j]); /* resident for the queries that follow */
        dcol[j] = NULL;
    }
    table->row_count = total;
out:
    for (int j = 0; j < ncols && j < 1024; j++)
        if (dcol[j]) mq_pool_free(dcol[j]);
    if (d_text) mq_pool_free(d_text);
    if (d_ws) mq_pool_free(d_ws);
    if (d_mm) mq_pool_free(d_mm);
    munmap((void*)text, n);
}

/* ------------------------------------------------------------------ */
/* index build: index.c:152-178 build_index                           */
/* ------------------------------------------------------------------ */

#define MQ_BIN_NUM 100 /* cs165_api.h:46 */
typedef struct MqHistogram { /* cs165_api.h:71-75 */
    int bin_size;
    int values[MQ_BIN_NUM];
    size_t counts[MQ_BIN_NUM];
} MqHistogram;
_Static_assert(sizeof(MqHistogram) == 1208, "Histogram size");

/* Up to this many rows an index over equal values reproduces the reference
 * quicksort's order of them exactly (mq_index_build_lomuto); beyond it (where the
 * reference's recursion and reorder_column's stack array cannot run) they keep
 * ascending row order. MQ_INDEX_EXACT_MAX overrides. */
static uint64_t index_exact_max(void) {
    const char* e = getenv("MQ_INDEX_EXACT_MAX");
    return e ? (uint64_t)strtoull(e, NULL, 10) : ((uint64_t)1 << 27);
}

/* One indexed column (index.c:119-143 + :63-84). Returns 0 or an MQ_E code. */
static int index_one(Table* t, Column* c, Status* st) {
    const size_t n = c->row_count;
    const int32_t* dcol;
    int rc;
    if ((rc = column_device(c, &dcol, st))) return rc;
    void *dv = NULL, *dp = NULL, *dh = NULL;
    ColumnIndex* ix = malloc(sizeof(ColumnIndex)); /* init_column_index :89-100 */
    int* hv = malloc((n ? n : 1) * sizeof(int));
    size_t* hp = malloc((n ? n : 1) * sizeof(size_t));
    if (!ix || !hv || !hp) {
        rc = MQ_ENOMEM;
        goto bad;
    }
    if ((rc = mq_malloc(&dv, (n ? n : 1) * 4)) || (rc = mq_malloc(&dp, (n ? n : 1) * 8))) goto bad;
    int exact = 1;
    if ((rc = mq_index_build_ref(dcol, n, dv, dp, index_exact_max(), &exact, g_stream))) goto bad;
    if (!exact)
        fprintf(stderr, "libmq: build_index: %zu rows of %s hold equal values beyond MQ_INDEX_EXACT_MAX; "
                        "they keep ascending row order instead of the reference quicksort's\n", n, c->name);
    if (n && (rc = d2h(hv, dv, n * 4))) goto bad;
    ix->values = hv;
    if (c->clustered) {
        /* build_clustered_index :119-135: the sort ran on a copy of the positions, so
         * index->positions stays 0..n-1; the permutation reorders every other column */
        for (size_t i = 0; i < n; i++) hp[i] = i;
        for (size_t j = 0; j < t->col_count; j++) {
            Column* o = t->columns + j;
            if (!strcmp(o->name, c->name)) continue;
            const int32_t* dsrc;
            void* dnew = NULL;
            if ((rc = column_device(o, &dsrc, st))) goto bad;
            if ((rc = mq_malloc(&dnew, (n ? n : 1) * 4))) goto bad;
            mq_guard_forget_range((uintptr_t)o->data, n * 4); /* reorder_column writes o->data in place */
            if ((rc = mq_gather_u64(dsrc, (const uint64_t*)dp, n, dnew, g_stream)) ||
                (n && (rc = d2h(o->data, dnew, n * 4)))) {
                mq_pool_free(dnew);
                goto bad;
            }
            col_put(o, dnew); /* the reordered rows stay resident */
        }
        if (n && (rc = mq_memcpy_h2d(dp, hp, n * 8, g_stream))) goto bad;
    } else {
        /* build_unclustered_index :140-143 + build_histogram :63-84 */
        if (n && (rc = d2h(hp, dp, n * 8))) goto bad;
        MqHistogram* h = malloc(sizeof(MqHistogram));
        if (!h) {
            rc = MQ_ENOMEM;
            goto bad;
        }
        h->bin_size = (c->max - c->min) / (MQ_BIN_NUM - 1);
        memset(h->values, 0, sizeof h->values);
        memset(h->counts, 0, sizeof h->counts);
        size_t bin_start = 0;
        for (int b = 0; b < MQ_BIN_NUM; b++) {
            h->values[b] = (int)bin_start;
            bin_start += (size_t)(long)h->bin_size;
        }
        if (h->bin_size == 0) {
            fprintf(stderr, "libmq: build_index: column %s spans < %d values; histogram counts left 0 "
                            "(the reference divides by zero here)\n", c->name, MQ_BIN_NUM - 1);
        } else {
            uint64_t counts[MQ_BIN_NUM + 1];
            if ((rc = mq_malloc(&dh, sizeof counts)) ||
                (rc = mq_histogram(dcol, n, c->min, h->bin_size, dh, g_stream)) ||
                (rc = d2h(counts, dh, sizeof counts))) {
                free(h);
                goto bad;
            }
            for (int b = 0; b < MQ_BIN_NUM; b++) h->counts[b] = counts[b];
        }
        c->histogram = (struct Histogram*)h;
    }
    ix->positions = hp;
    c->index = ix;
    idx_put(ix, n, dv, dp, 1); /* resident for select_column_sorted_index */
    mq_pool_free(dh);
    return 0;
bad:
    free(ix);
    free(hv);
    free(hp);
    mq_pool_free(dv);
    mq_pool_free(dp);
    mq_pool_free(dh);
    fail(st, "build_index", rc);
    return rc;
}

void build_index(Db* db) {
    Status st = {OK, NULL};
    if (!db || op_begin(&st)) return;
    for (size_t i = 0; i < db->tables_size; i++) {
        Table* t = db->tables + i;
        for (size_t j = 0; j < t->col_count; j++) {
            Column* c = t->columns + j;
            if (c->has_index && index_one(t, c, &st)) return; /* build_btree is a no-op */
        }
    }
}

/* ------------------------------------------------------------------ */
/* residency control                                                  */
/* ------------------------------------------------------------------ */

int mq_column_attach(Column* column, const int32_t* d_data) {
    Status st = {OK, NULL};
    if (ready(&st)) return MQ_ENODEV;
    ColEntry* e = col_find(column);
    if (e) col_drop(e);
    if (g_ncols == MAX_COLS) col_drop(&g_cols[0]);
    g_cols[g_ncols++] = (ColEntry){column, column->data, column->row_count, (void*)d_data, 0, 0, g_op};
    return MQ_OK;
}

int mq_column_upload(Column* column) {
    Status st = {OK, NULL};
    if (op_begin(&st)) return MQ_ENODEV;
    if (shard_wants(column)) return shard_upload(column, &st) ? MQ_EHIP : MQ_OK;
    const int32_t* d;
    return column_device(column, &d, &st) ? MQ_EHIP : MQ_OK;
}

void mq_column_invalidate(Column* column) {
    ColEntry* e = col_find(column);
    if (e) col_drop(e);
    shard_forget_column(column);
}

const void* mq_result_device_ptr(const Result* result) {
    int i = shadow_find(result->payload);
    if (i < 0) return NULL;
    const ShadowEntry* e = &g_shadows[i];
    if (e->n != result->num_tuples) return NULL;
    if (e->op == g_op || e->n == 0 || (e->guard && mq_guard_clean(e->guard, e->host, e->n * 4))) return e->dev;
    return NULL;
}

void mq_release_all(void) {
    if (g_stream) mq_stream_sync(g_stream);
    mq_pool_free(g_print_out);
    mq_pool_free(g_print_ws);
    g_print_out = g_print_ws = NULL;
    g_print_out_cap = g_print_ws_cap = 0;
    while (g_ncols) col_drop(&g_cols[g_ncols - 1]);
    while (g_nshadows) shadow_drop(g_nshadows - 1);
    while (g_nidx) idx_drop(&g_idx[g_nidx - 1]);
    shard_release_all();
    mq_trim();
}

void mq_residency_stats(mq_residency* out) {
    mq_guard_stats gs = mq_guard_get_stats();
    *out = g_res;
    out->guards_armed = gs.armed;
    out->guard_clean = gs.clean;
    out->guard_stale = gs.stale;
    out->guards_live = gs.live;
    out->remap_probe = gs.remap_probe;
    out->columns_resident = (uint64_t)g_ncols;
    out->shadows_resident = (uint64_t)g_nshadows;
    out->shadow_bytes = (uint64_t)g_shadow_bytes;
    shard_stats(out);
}

double mq_transfer_seconds(int reset) {
    double t = g_xfer_s;
    if (reset) g_xfer_s = 0;
    return t;
}

/* ------------------------------------------------------------------ */
/* internal interface for the row-shard executor (mq_shim.h)          */
/* ------------------------------------------------------------------ */

double shim_now(void) { return now_s(); }
int shim_trace_on(void) { return trace_on(); }
int shim_fail(Status* st, const char* what, int rc) { return fail(st, what, rc); }
void* shim_payload_alloc(size_t bytes) { return payload_alloc(bytes); }

Result* shim_new_result(DataType t, size_t n, void* payload) { return new_result(t, n, payload); }
unsigned long long shim_op(void) { return g_op; }
size_t shim_shadow_budget(void) { return shadow_budget(); }
mq_residency* shim_stats(void) { return &g_res; }
void shim_xfer_add(double seconds) { g_xfer_s += seconds; }
