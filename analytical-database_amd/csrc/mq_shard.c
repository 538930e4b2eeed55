/*
 * mq_shard.c — row shards: a long column split into G contiguous row ranges, shard g
 * resident on its own device and served by its own host thread and stream.
 *
 * scans, selects and aggregates partition by row range; per-shard
 * position lists use local rows plus the shard base, so the global ascending list is
 * the concatenation in shard order, which is also the order the reference's
 * shared_select threads concatenate in (src/query.c:563-574); {count, sum, min, max}
 * combine with one fold (avg = one double division after it, bit-identical to one
 * device). The fan-out sits inside the operators the server calls for one query or
 * one batch (server.c:360-399 batches into shared_select), so the reference server
 * links it unchanged.
 *
 * Data movement: each shard uploads its rows from the host column over its own PCIe
 * link, and downloads its part of every Result straight into the host payload at the
 * part's offset, so results are assembled in host memory with no device-to-device
 * exchange. The pieces stay resident as a sharded shadow of the payload: a following
 * fetch_column / sum / avg / min / max on that Result runs on the shards again.
 *
 * The aggregate combine is a host fold of G 32-byte partials: the Result the API returns
 * is host memory, so a collective would only add a hop (RCCL's all-reduce serves the
 * one-process-per-GPU bench, analytical-database_amd/dist.py).
 *
 * Threads: G workers, each bound to its shard's device for its lifetime; an operator
 * hands every worker the same task and waits for all (no work is queued across calls).
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mq_guard.h"
#include "mq_shim.h"

#define MAXS 64
#define MAX_SCOLS 256
#define MAX_SSHADOWS 2048
#define MAXQ 256

typedef struct Shard {
    int idx, dev;
    void* stream;
    void* ws;
    size_t ws_bytes;
    void* scratch;
    size_t scratch_bytes;
    void* small;  /* counts / aggregates */
    int rc, quit;
    double xfer;  /* PCIe seconds of the current task */
    unsigned long gen0;  /* task generation when the worker was started */
    pthread_t th;
    /* per-task outputs */
    uint64_t k;
    mq_agg agg;
    uint64_t kq[MAXQ];
    void* piece[MAXQ];
} Shard;

static Shard g_sh[MAXS];
static int g_G = -1;        /* shard count; 1 = off */
static size_t g_min_rows;
static int g_started;       /* 1 = workers up, -1 = start failed (one device from then on) */
static int g_live;          /* workers running: g_sh[0 .. g_live) */

static pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER;
static pthread_cond_t g_go = PTHREAD_COND_INITIALIZER, g_done = PTHREAD_COND_INITIALIZER;
static unsigned long g_gen;
static int g_pending;
static void (*g_fn)(Shard*, void*);
static void* g_arg;

/* ------------------------------------------------------------------ */
/* configuration and workers                                          */
/* ------------------------------------------------------------------ */

static void configure(void) {
    if (g_G >= 0) return;
    memset(g_sh, 0, sizeof g_sh);
    int devs[MAXS], nd = 0;
    const char* e = getenv("MQ_DEVICES");
    while (e && *e && nd < MAXS) {
        char* end;
        long v = strtol(e, &end, 10);
        if (end == e) break;
        devs[nd++] = (int)v;
        e = *end == ',' ? end + 1 : end;
    }
    const char* s = getenv("MQ_SHARDS");
    int G = s ? atoi(s) : (nd > 0 ? nd : 1);
    if (G < 1) G = 1;
    if (G > MAXS) G = MAXS;
    const char* pe = getenv("MQ_DEVICE");
    const int primary = pe ? atoi(pe) : 0;
    int count = mq_device_count();
    if (count < 1) count = 1;
    for (int g = 0; g < G; g++) {
        g_sh[g].idx = g;
        g_sh[g].dev = nd > 0 ? devs[g % nd] : (primary + g) % count;
        if (G > 1 && (g_sh[g].dev < 0 || g_sh[g].dev >= count)) { /* as mq_shard_config refuses */
            fprintf(stderr, "libmq: MQ_DEVICES names device %d of %d; row shards off\n", g_sh[g].dev, count);
            G = 1;
            break;
        }
    }
    const char* m = getenv("MQ_SHARD_MIN_ROWS");
    g_min_rows = m ? (size_t)strtoull(m, NULL, 10) : ((size_t)1 << 24);
    g_G = G;
}

static void* worker(void* p) {
    Shard* s = (Shard*)p;
    unsigned long seen = s->gen0; /* tasks before this worker existed are not its own */
    for (;;) {
        pthread_mutex_lock(&g_mu);
        while (g_gen == seen) pthread_cond_wait(&g_go, &g_mu);
        seen = g_gen;
        void (*fn)(Shard*, void*) = g_fn;
        void* arg = g_arg;
        pthread_mutex_unlock(&g_mu);
        s->rc = 0;
        fn(s, arg);
        const int quit = s->quit;
        pthread_mutex_lock(&g_mu);
        if (--g_pending == 0) pthread_cond_signal(&g_done);
        pthread_mutex_unlock(&g_mu);
        if (quit) return NULL;
    }
}

/* Run fn on every shard's worker and wait for all; the first nonzero rc, or 0. */
static int run_all(void (*fn)(Shard*, void*), void* arg) {
    pthread_mutex_lock(&g_mu);
    g_fn = fn;
    g_arg = arg;
    g_pending = g_live;
    g_gen++;
    pthread_cond_broadcast(&g_go);
    while (g_pending) pthread_cond_wait(&g_done, &g_mu);
    pthread_mutex_unlock(&g_mu);
    double x = 0; /* the shards copy in parallel: the task's transfer time is the longest */
    for (int g = 0; g < g_live; g++) {
        if (g_sh[g].xfer > x) x = g_sh[g].xfer;
        g_sh[g].xfer = 0;
    }
    shim_xfer_add(x);
    for (int g = 0; g < g_live; g++)
        if (g_sh[g].rc) return g_sh[g].rc;
    return 0;
}

static void t_init(Shard* s, void* arg) {
    (void)arg;
    if ((s->rc = mq_init(s->dev))) return;
    if ((s->rc = mq_stream_create(&s->stream))) return;
    if ((s->rc = mq_malloc(&s->small, 4096))) return;
    /* the join's exchanges copy between shard devices (mq_memcpy_peer) */
    for (int g = 0; g < g_G && !s->rc; g++) s->rc = mq_enable_peer(g_sh[g].dev);
}

static void t_stop(Shard* s, void* a);

/* Stop every running worker (each frees its stream, scratch and pinned staging). */
static void stop_workers(void) {
    if (g_live > 0) run_all(t_stop, NULL);
    g_live = 0;
}

/* Start the G workers and bind each to its device. On any failure the workers
 * already running are stopped again and row shards stay off for the process: the
 * operators then run on one device (shard_wants() is 0). */
static int start(Status* st) {
    if (g_started == 1) return 0;
    if (g_started == -1) return shim_fail(st, "row shards (earlier)", MQ_ENODEV);
    pthread_mutex_lock(&g_mu);
    const unsigned long gen0 = g_gen;
    pthread_mutex_unlock(&g_mu);
    for (int g = 0; g < g_G; g++) {
        g_sh[g].gen0 = gen0;
        g_sh[g].quit = 0;
        if (pthread_create(&g_sh[g].th, NULL, worker, &g_sh[g]) != 0) {
            stop_workers();
            g_started = -1;
            fprintf(stderr, "libmq: shard worker start failed; row shards off\n");
            return shim_fail(st, "shard worker start", MQ_EINVAL);
        }
        pthread_detach(g_sh[g].th);
        g_live = g + 1;
    }
    int rc = run_all(t_init, NULL);
    if (rc) {
        stop_workers();
        g_started = -1;
        fprintf(stderr, "libmq: shard device init failed (%s); row shards off\n", mq_last_error());
        return shim_fail(st, "shard device init", rc);
    }
    g_started = 1;
    return 0;
}

int shard_count(void) {
    configure();
    return g_G;
}

/* Whether an operator on column c fans out over the row shards. Starts the workers
 * on first use; a failed start turns shards off, and the operator (this one and every
 * later one) runs on the one-device path instead of failing. */
int shard_wants(const Column* c) {
    configure();
    if (!(g_G > 1 && c && c->row_count >= g_min_rows && c->row_count >= (size_t)g_G &&
          c->row_count <= (size_t)INT32_MAX))
        return 0;
    if (g_started == 0) {
        Status tmp;
        (void)start(&tmp);
    }
    return g_started == 1;
}

/* Per-shard scratch on the worker's device (grow-only, pool memory). */
static int grow(void** buf, size_t* have, size_t need) {
    if (*have >= need && *buf) return 0;
    if (*buf) mq_pool_free(*buf);
    *buf = NULL;
    *have = 0;
    size_t want = need + need / 8 + 4096;
    int rc = mq_pool_malloc(buf, want);
    if (rc) return rc;
    *have = want;
    return 0;
}

static int ensure(Shard* s, size_t rows) {
    int rc = grow(&s->ws, &s->ws_bytes, mq_scan_workspace_bytes(rows));
    if (!rc) rc = grow(&s->scratch, &s->scratch_bytes, (rows ? rows : 1) * sizeof(int32_t));
    return rc;
}

/* D2H of one piece of a Result into its slot of the host payload; staged (pinned
 * buffers) when the payload will be write-guarded, see mq_memcpy_d2h_staged. */
static int download(Shard* s, void* host, const void* dev, size_t bytes, int staged) {
    if (!bytes) return 0;
    int rc = mq_stream_sync(s->stream); /* the transfer clock counts the copy alone */
    if (rc) return rc;
    double t0 = shim_now();
    rc = staged ? mq_memcpy_d2h_staged(host, dev, bytes, s->stream) : mq_memcpy_d2h(host, dev, bytes, s->stream);
    s->xfer += shim_now() - t0;
    return rc;
}

/* ------------------------------------------------------------------ */
/* sharded columns                                                    */
/* ------------------------------------------------------------------ */

typedef struct {
    const Column* col;
    const int* host;
    size_t rows;
    size_t base[MAXS + 1];
    void* dev[MAXS];
    uint64_t guard;
    unsigned long long op;
} SCol;

static SCol g_scols[MAX_SCOLS];
static int g_nscols;

typedef struct {
    const void* host;  /* payload */
    size_t n;
    size_t rows;       /* > 0: the pieces are positions of a rows-row column split as split_of(rows) */
    size_t off[MAXS + 1];
    void* dev[MAXS];
    uint64_t guard;
    size_t bytes;
    unsigned long long stamp, op;
} SShadow;

static SShadow g_ssh[MAX_SSHADOWS];
static int g_nssh;
static size_t g_ssh_bytes;
static unsigned long long g_sstamp;
static uint64_t g_ops, g_uploads;

/* Row split of a column: whole 1024-row tiles per shard (16-byte aligned slices). */
static void split_of(size_t rows, size_t* base) {
    base[0] = 0;
    for (int g = 1; g < g_G; g++) {
        size_t b = (size_t)(((unsigned __int128)rows * (unsigned)g) / (unsigned)g_G) & ~(size_t)1023;
        base[g] = b < base[g - 1] ? base[g - 1] : b;
    }
    base[g_G] = rows;
}

/* Device memory is freed only between operators, when no worker has work queued. */
static void free_pieces(void* const* dev) {
    for (int g = 0; g < g_G; g++) mq_pool_free(dev[g]);
}

static void scol_drop(int i) {
    mq_guard_release(g_scols[i].guard);
    free_pieces(g_scols[i].dev);
    g_scols[i] = g_scols[--g_nscols];
}

static void ssh_drop(int i) {
    mq_guard_release(g_ssh[i].guard);
    free_pieces(g_ssh[i].dev);
    g_ssh_bytes -= g_ssh[i].bytes;
    g_ssh[i] = g_ssh[--g_nssh];
}

typedef struct {
    SCol* e;
    const int* host;
} UpArg;

static void t_upload(Shard* s, void* a) {
    UpArg* u = (UpArg*)a;
    const size_t b0 = u->e->base[s->idx], n = u->e->base[s->idx + 1] - b0;
    if ((s->rc = mq_pool_malloc(&u->e->dev[s->idx], (n ? n : 1) * 4))) return;
    double t0 = shim_now();
    if (n) s->rc = mq_memcpy_h2d(u->e->dev[s->idx], u->host + b0, n * 4, s->stream);
    s->xfer += shim_now() - t0;
}

static SCol* scol_get(Column* c, Status* st) {
    if (start(st)) return NULL;
    for (int i = 0; i < g_nscols; i++) {
        SCol* e = &g_scols[i];
        if (e->col != c) continue;
        if (e->host == c->data && e->rows == c->row_count &&
            (e->op == shim_op() || (e->guard && mq_guard_clean(e->guard, e->host, e->rows * 4)))) {
            e->op = shim_op();
            return e;
        }
        scol_drop(i);
        break;
    }
    if (g_nscols == MAX_SCOLS) {
        int v = 0;
        for (int i = 0; i < g_nscols; i++)
            if (g_scols[i].op != shim_op()) v = i;
        scol_drop(v);
    }
    SCol* e = &g_scols[g_nscols];
    memset(e, 0, sizeof *e);
    e->col = c;
    e->host = c->data;
    e->rows = c->row_count;
    e->op = shim_op();
    split_of(e->rows, e->base);
    UpArg u = {e, c->data};
    int rc = run_all(t_upload, &u);
    if (rc) {
        free_pieces(e->dev);
        shim_fail(st, "shard column upload", rc);
        return NULL;
    }
    e->guard = mq_guard_arm(c->data, e->rows * 4, MQ_GUARD_FILE);
    g_nscols++;
    g_uploads++;
    shim_stats()->column_uploads++;
    shim_stats()->column_bytes += e->rows * 4;
    return e;
}

static int ssh_find(const void* host, size_t n) {
    for (int i = 0; i < g_nssh; i++)
        if (g_ssh[i].host == host) {
            SShadow* e = &g_ssh[i];
            if (e->n == n && (e->op == shim_op() || n == 0 || (e->guard && mq_guard_clean(e->guard, host, n * 4)))) {
                e->op = shim_op();
                e->stamp = ++g_sstamp;
                return i;
            }
            ssh_drop(i);
            return -1;
        }
    return -1;
}

/* LRU down to the shadow budget; entries the current operator holds stay. */
static void ssh_make_room(size_t bytes) {
    while (g_nssh >= MAX_SSHADOWS || g_ssh_bytes + bytes > shim_shadow_budget()) {
        int v = -1;
        for (int i = 0; i < g_nssh; i++)
            if (g_ssh[i].op != shim_op() && (v < 0 || g_ssh[i].stamp < g_ssh[v].stamp)) v = i;
        if (v < 0) break;
        ssh_drop(v);
    }
}

/* Register the pieces (owned from now on) as the payload's sharded shadow. */
static void ssh_put(const void* host, size_t n, size_t rows, const size_t* off, void* const* dev, uint64_t guard) {
    for (int i = 0; i < g_nssh; i++)
        if (g_ssh[i].host == host) {
            ssh_drop(i);
            break;
        }
    ssh_make_room(n * 4);
    if (g_nssh == MAX_SSHADOWS) ssh_drop(0);
    SShadow* e = &g_ssh[g_nssh++];
    e->host = host;
    e->n = n;
    e->rows = rows;
    memcpy(e->off, off, sizeof(size_t) * (size_t)(g_G + 1));
    memcpy(e->dev, dev, sizeof(void*) * (size_t)g_G);
    e->guard = guard;
    e->bytes = n * 4;
    e->stamp = ++g_sstamp;
    e->op = shim_op();
    g_ssh_bytes += e->bytes;
}

/* Assemble a Result from per-shard pieces already downloaded: guard the payload and
 * keep the pieces as its shadow, or free them. */
static Result* finish(void* payload, size_t n, size_t rows, const size_t* off, void** pieces, int keep) {
    const uint64_t guard = keep && n ? mq_guard_arm(payload, n * 4, MQ_GUARD_CHUNK) : 0;
    if (guard) {
        ssh_put(payload, n, rows, off, pieces, guard);
    } else {
        free_pieces(pieces);
    }
    g_ops++;
    return shim_new_result(INT, n, payload);
}

static int keep_payload(const void* p, size_t bytes) {
    return bytes >= SHADOW_MIN_BYTES && mq_guard_enabled() && mq_guard_chunk_ok(p);
}

/* ------------------------------------------------------------------ */
/* operators                                                          */
/* ------------------------------------------------------------------ */

typedef struct {
    SCol* e;
    int has_low, has_high;
    int32_t low, high;
    /* download step */
    int32_t* payload;
    size_t off[MAXS + 1];
    void* pieces[MAXS];
    int staged, keep;
} SelArg;

static void t_select(Shard* s, void* a) {
    SelArg* x = (SelArg*)a;
    const size_t b0 = x->e->base[s->idx], n = x->e->base[s->idx + 1] - b0;
    if ((s->rc = ensure(s, n))) return;
    s->rc = mq_select_positions_at((const int32_t*)x->e->dev[s->idx], NULL, n, (int32_t)b0, x->has_low, x->low,
                                   x->has_high, x->high, (int32_t*)s->scratch, (uint64_t*)s->small, s->ws,
                                   s->ws_bytes, s->stream);
    if (!s->rc) s->rc = mq_memcpy_d2h(&s->k, s->small, sizeof(uint64_t), s->stream);
}

/* download shard g's k positions from its scratch; keep a copy as the shadow piece */
static void t_select_out(Shard* s, void* a) {
    SelArg* x = (SelArg*)a;
    const size_t k = x->off[s->idx + 1] - x->off[s->idx];
    x->pieces[s->idx] = NULL;
    if ((s->rc = download(s, x->payload + x->off[s->idx], s->scratch, k * 4, x->staged))) return;
    if (!x->keep) return;
    if ((s->rc = mq_pool_malloc(&x->pieces[s->idx], (k ? k : 1) * 4))) return;
    if (!(s->rc = mq_memcpy_d2d(x->pieces[s->idx], s->scratch, k * 4, s->stream))) s->rc = mq_stream_sync(s->stream);
}

Result* shard_select(Column* c, int* low, int* high, Status* st) {
    SCol* e = scol_get(c, st);
    if (!e) return NULL;
    const double t0 = shim_now();
    SelArg x;
    memset(&x, 0, sizeof x);
    x.e = e;
    x.has_low = low != NULL;
    x.low = low ? *low : 0;
    x.has_high = high != NULL;
    x.high = high ? *high : 0;
    int rc = run_all(t_select, &x);
    if (rc) {
        shim_fail(st, "shard select", rc);
        return NULL;
    }
    x.off[0] = 0;
    for (int g = 0; g < g_G; g++) x.off[g + 1] = x.off[g] + g_sh[g].k;
    const size_t K = x.off[g_G];
    x.payload = (int32_t*)shim_payload_alloc(K * 4);
    x.keep = x.staged = keep_payload(x.payload, K * 4);
    if ((rc = run_all(t_select_out, &x))) {
        free_pieces(x.pieces);
        free(x.payload);
        shim_fail(st, "shard select download", rc);
        return NULL;
    }
    Result* r = finish(x.payload, K, e->rows, x.off, x.pieces, x.keep);
    if (shim_trace_on()) fprintf(stderr, "mq-trace shard_select(G=%d)      %9.3f ms\n", g_G, 1e3 * (shim_now() - t0));
    st->code = OK;
    return r;
}

typedef struct {
    SCol* e;
    SShadow* pos;
    int32_t* payload;
    void* pieces[MAXS];
    int staged, keep;
} FetchArg;

static void t_fetch(Shard* s, void* a) {
    FetchArg* x = (FetchArg*)a;
    const size_t k = x->pos->off[s->idx + 1] - x->pos->off[s->idx];
    x->pieces[s->idx] = NULL;
    if ((s->rc = mq_pool_malloc(&x->pieces[s->idx], (k ? k : 1) * 4))) return;
    if ((s->rc = mq_fetch_at((const int32_t*)x->e->dev[s->idx], (int32_t)x->e->base[s->idx],
                             (const int32_t*)x->pos->dev[s->idx], k, (int32_t*)x->pieces[s->idx], s->stream)))
        return;
    s->rc = download(s, x->payload + x->pos->off[s->idx], x->pieces[s->idx], k * 4, x->staged);
    if (!s->rc) s->rc = mq_stream_sync(s->stream);
}

int shard_fetch(Column* c, Result* pos, Result** out, Status* st) {
    if (g_started != 1) return 0;
    const int i = ssh_find(pos->payload, pos->num_tuples);
    if (i < 0 || g_ssh[i].rows != c->row_count) return 0;
    SCol* e = scol_get(c, st);
    if (!e) return -1;
    const int j = ssh_find(pos->payload, pos->num_tuples); /* scol_get may have evicted */
    if (j < 0) return 0;
    const double t0 = shim_now();
    FetchArg x;
    memset(&x, 0, sizeof x);
    x.e = e;
    x.pos = &g_ssh[j];
    const size_t K = x.pos->n;
    x.payload = (int32_t*)shim_payload_alloc(K * 4);
    x.keep = x.staged = keep_payload(x.payload, K * 4);
    int rc = run_all(t_fetch, &x);
    if (rc) {
        free_pieces(x.pieces);
        free(x.payload);
        shim_fail(st, "shard fetch", rc);
        return -1;
    }
    size_t off[MAXS + 1];
    memcpy(off, x.pos->off, sizeof off);
    *out = finish(x.payload, K, 0, off, x.pieces, x.keep);
    if (shim_trace_on()) fprintf(stderr, "mq-trace shard_fetch(G=%d)       %9.3f ms\n", g_G, 1e3 * (shim_now() - t0));
    st->code = OK;
    return 1;
}

typedef struct {
    void* const* dev;    /* per shard */
    const size_t* len;   /* per shard rows: len[g+1] - len[g] */
} RedArg;

static void t_reduce(Shard* s, void* a) {
    RedArg* x = (RedArg*)a;
    const size_t n = x->len[s->idx + 1] - x->len[s->idx];
    if ((s->rc = ensure(s, 0))) return;
    if ((s->rc = mq_reduce((const int32_t*)x->dev[s->idx], n, (mq_agg*)s->small, s->ws, s->ws_bytes, s->stream)))
        return;
    s->rc = mq_memcpy_d2h(&s->agg, s->small, sizeof(mq_agg), s->stream);
}

/* {count, sum, min, max} of the shards, folded: sums add, extremes take min / max */
static void fold(mq_agg* a) {
    a->count = 0;
    a->sum = 0;
    a->min = INT32_MAX;
    a->max = INT32_MIN;
    a->_pad = 0;
    for (int g = 0; g < g_G; g++) {
        a->count += g_sh[g].agg.count;
        a->sum += g_sh[g].agg.sum;
        if (g_sh[g].agg.count) {
            if (g_sh[g].agg.min < a->min) a->min = g_sh[g].agg.min;
            if (g_sh[g].agg.max > a->max) a->max = g_sh[g].agg.max;
        }
    }
}

int shard_reduce_column(Column* c, mq_agg* a, Status* st) {
    SCol* e = scol_get(c, st);
    if (!e) return -1;
    RedArg x = {e->dev, e->base};
    int rc = run_all(t_reduce, &x);
    if (rc) return shim_fail(st, "shard sum", rc);
    fold(a);
    g_ops++;
    return 0;
}

int shard_reduce_result(const Result* r, mq_agg* a, Status* st) {
    if (g_started != 1) return 0;
    const int i = ssh_find(r->payload, r->num_tuples);
    if (i < 0) return 0;
    RedArg x = {g_ssh[i].dev, g_ssh[i].off};
    int rc = run_all(t_reduce, &x);
    if (rc) {
        shim_fail(st, "shard reduce", rc);
        return -1;
    }
    fold(a);
    g_ops++;
    return 1;
}

/* ---- shared_select ---- */

typedef struct {
    SCol* e;
    int q;
    int32_t lows[MAXQ], highs[MAXQ];
    int32_t* payload[MAXQ];
    size_t off[MAXQ][MAXS + 1];
    int keep[MAXQ];
} SsArg;

static void t_ss_count(Shard* s, void* a) {
    SsArg* x = (SsArg*)a;
    const size_t b0 = x->e->base[s->idx], n = x->e->base[s->idx + 1] - b0;
    if ((s->rc = grow(&s->ws, &s->ws_bytes, mq_shared_select_workspace_bytes(n, x->q)))) return;
    s->rc = mq_shared_select_count_at((const int32_t*)x->e->dev[s->idx], n, (int32_t)b0, x->lows, x->highs, x->q,
                                      s->kq, s->ws, s->ws_bytes, s->stream);
}

static void t_ss_write(Shard* s, void* a) {
    SsArg* x = (SsArg*)a;
    for (int j = 0; j < x->q; j++) s->piece[j] = NULL;
    for (int j = 0; j < x->q; j++)
        if ((s->rc = mq_pool_malloc(&s->piece[j], (s->kq[j] ? s->kq[j] : 1) * 4))) return;
    if ((s->rc = mq_shared_select_write(s->ws, (int32_t* const*)s->piece, s->stream))) return;
    for (int j = 0; j < x->q; j++)
        if ((s->rc = download(s, x->payload[j] + x->off[j][s->idx], s->piece[j], s->kq[j] * 4, x->keep[j]))) return;
    s->rc = mq_stream_sync(s->stream);
}

Result** shard_shared_select(SelectOperator* ops, int q, Column* c, Status* st) {
    SCol* e = scol_get(c, st);
    if (!e) return NULL;
    Result** out = (Result**)calloc((size_t)(q > 0 ? q : 1), sizeof(Result*));
    SsArg* x = (SsArg*)calloc(1, sizeof(SsArg));
    if (!out || !x) {
        free(out);
        free(x);
        shim_fail(st, "shard shared_select", MQ_ENOMEM);
        return NULL;
    }
    x->e = e;
    int done = 0, rc = 0;
    for (int q0 = 0; q0 < q && !rc; q0 += MAXQ) {
        const int m = q - q0 < MAXQ ? q - q0 : MAXQ;
        x->q = m;
        for (int j = 0; j < m; j++) { /* the fields as given (query.c:472-479) */
            x->lows[j] = ops[q0 + j].low;
            x->highs[j] = ops[q0 + j].high;
        }
        if ((rc = run_all(t_ss_count, x))) break;
        for (int j = 0; j < m; j++) {
            x->off[j][0] = 0;
            for (int g = 0; g < g_G; g++) x->off[j][g + 1] = x->off[j][g] + g_sh[g].kq[j];
            const size_t K = x->off[j][g_G];
            x->payload[j] = (int32_t*)shim_payload_alloc(K * 4);
            x->keep[j] = keep_payload(x->payload[j], K * 4);
        }
        rc = run_all(t_ss_write, x);
        for (int j = 0; j < m; j++) {
            void* pieces[MAXS];
            for (int g = 0; g < g_G; g++) pieces[g] = g_sh[g].piece[j];
            if (rc) {
                free_pieces(pieces);
                free(x->payload[j]);
                continue;
            }
            out[q0 + j] = finish(x->payload[j], x->off[j][g_G], e->rows, x->off[j], pieces, x->keep[j]);
            done = q0 + j + 1;
        }
    }
    free(x);
    if (rc) {
        for (int j = 0; j < done; j++) {
            free(out[j]->payload);
            free(out[j]);
        }
        free(out);
        shim_fail(st, "shard shared_select", rc);
        return NULL;
    }
    st->code = OK;
    return out;
}

/* ---- hash_join: key-partitioned over the shards (mq_pjoin.hip's protocol) ---- */

typedef struct {
    /* inputs: shard s's rows of each side, on its device */
    const int32_t* c1[MAXS];
    const int32_t* p1[MAXS];
    uint64_t n1[MAXS];
    const int32_t* c2[MAXS];
    const int32_t* p2[MAXS];
    uint64_t n2[MAXS];
    /* 1. partitioned sides on shard s, bucket sizes [s][b] */
    int32_t *bk[MAXS], *bp[MAXS], *pk[MAXS];
    uint32_t* inv[MAXS];
    uint64_t cb[MAXS][MAXS], cp[MAXS][MAXS];
    /* 2. on device g: per probe row counts, build positions of the pairs, pairs per
     *    source shard [g][s] */
    uint32_t* cnt[MAXS];
    int32_t* o1[MAXS];
    uint64_t mg[MAXS][MAXS];
    /* 3. outputs on shard s */
    int32_t *out1[MAXS], *out2[MAXS];
    uint64_t m[MAXS];
    double ms[4]; /* host wall time of the phases (partition, join, place, total) */
} PJ;

/* Test hook (mq_shard_join_inject_failure): the phase whose allocations fail (1 = the
 * partition, 2 = the local joins, 3 = the placement, 4 = the one-shard join; 0 = none). */
static volatile int g_pj_fail;

void mq_shard_join_inject_failure(int phase) { g_pj_fail = phase; }

static void* pj_alloc(int* rc, size_t bytes, int phase) {
    void* p = NULL;
    if (!*rc && g_pj_fail == phase) *rc = MQ_ENOMEM;
    if (!*rc) *rc = mq_pool_malloc(&p, bytes ? bytes : 4);
    return p;
}

/* The end of a worker's phase: its stream drained whatever rc is, so that on an error
 * path no queued peer copy or kernel still uses a buffer the caller's thread frees. */
static int pj_end(Shard* s, int rc) {
    const int r2 = mq_stream_sync(s->stream);
    return rc ? rc : r2;
}

/* Entry fence of mq_shard_join: its inputs are device pointers the caller may still be
 * writing on any stream of the shard's device (the null stream included; the workers'
 * own streams are non-blocking, so they would not wait for it). Each worker waits for
 * its whole device before the first read. */
static void t_pj_fence(Shard* s, void* a) {
    (void)a;
    s->rc = mq_device_sync();
}

/* G = 1: no partition, exchange or placement, the local join straight into the outputs. */
static void t_pj_single(Shard* s, void* a) {
    PJ* x = (PJ*)a;
    mq_join* j = NULL;
    uint64_t m = 0;
    int rc = mq_join_build(x->c1[0], x->p1[0], x->n1[0], &j, s->stream);
    if (!rc) rc = mq_join_probe(j, x->c2[0], x->n2[0], &m, s->stream);
    x->out1[0] = (int32_t*)pj_alloc(&rc, m * 4, 4);
    x->out2[0] = (int32_t*)pj_alloc(&rc, m * 4, 4);
    if (!rc && m) rc = mq_join_write(j, x->p2[0], x->out1[0], x->out2[0], s->stream);
    rc = pj_end(s, rc);
    if (j) mq_join_free(j);
    x->m[0] = m;
    x->mg[0][0] = m;
    s->rc = rc;
}


static void t_pj_part(Shard* s, void* a) {
    PJ* x = (PJ*)a;
    const int i = s->idx;
    int rc = 0;
    x->bk[i] = (int32_t*)pj_alloc(&rc, x->n1[i] * 4, 1);
    x->bp[i] = (int32_t*)pj_alloc(&rc, x->n1[i] * 4, 1);
    x->pk[i] = (int32_t*)pj_alloc(&rc, x->n2[i] * 4, 1);
    x->inv[i] = (uint32_t*)pj_alloc(&rc, x->n2[i] * 4, 1);
    if (!rc)
        rc = mq_pjoin_partition(x->c1[i], x->p1[i], x->n1[i], g_G, x->bk[i], x->bp[i], NULL, x->cb[i], s->stream);
    if (!rc)
        rc = mq_pjoin_partition(x->c2[i], NULL, x->n2[i], g_G, x->pk[i], NULL, x->inv[i], x->cp[i], s->stream);
    s->rc = pj_end(s, rc); /* pj_free_temps frees the outputs from the caller's thread */
}

/* first index of bucket b in shard s's partitioned side (cnt = cb or cp) */
static uint64_t pj_seg(uint64_t (*cnt)[MAXS], int s, int b) {
    uint64_t o = 0;
    for (int k = 0; k < b; k++) o += cnt[s][k];
    return o;
}

static void t_pj_join(Shard* s, void* a) {
    PJ* x = (PJ*)a;
    const int g = s->idx;
    uint64_t nb = 0, np = 0;
    for (int k = 0; k < g_G; k++) {
        nb += x->cb[k][g];
        np += x->cp[k][g];
    }
    int rc = 0;
    int32_t* jk = (int32_t*)pj_alloc(&rc, nb * 4, 2);
    int32_t* jp = (int32_t*)pj_alloc(&rc, nb * 4, 2);
    int32_t* jq = (int32_t*)pj_alloc(&rc, np * 4, 2);
    x->cnt[g] = (uint32_t*)pj_alloc(&rc, np * 4, 2);
    /* bucket g of every shard, in shard order */
    uint64_t ab = 0, ap = 0;
    for (int k = 0; k < g_G && !rc; k++) {
        const uint64_t ob = pj_seg(x->cb, k, g), op = pj_seg(x->cp, k, g);
        const int dv = g_sh[k].dev;
        rc = mq_memcpy_peer(jk + ab, s->dev, x->bk[k] + ob, dv, x->cb[k][g] * 4, s->stream);
        if (!rc) rc = mq_memcpy_peer(jp + ab, s->dev, x->bp[k] + ob, dv, x->cb[k][g] * 4, s->stream);
        if (!rc) rc = mq_memcpy_peer(jq + ap, s->dev, x->pk[k] + op, dv, x->cp[k][g] * 4, s->stream);
        ab += x->cb[k][g];
        ap += x->cp[k][g];
    }
    mq_join* j = NULL;
    uint64_t m = 0;
    if (!rc) rc = mq_join_build(jk, jp, nb, &j, s->stream);
    if (!rc) rc = mq_join_probe(j, jq, np, &m, s->stream);
    if (!rc) rc = mq_join_counts(j, x->cnt[g], s->stream);
    /* pairs per source shard: the sum of its segment's counts */
    if (!rc) rc = ensure(s, 0);
    uint64_t sp = 0;
    for (int k = 0; k < g_G && !rc; k++) {
        x->mg[g][k] = 0;
        if (x->cp[k][g] && m) {
            rc = mq_reduce((const int32_t*)(x->cnt[g] + sp), x->cp[k][g], (mq_agg*)s->small, s->ws, s->ws_bytes,
                           s->stream);
            mq_agg ag;
            if (!rc) rc = mq_memcpy_d2h(&ag, s->small, sizeof ag, s->stream);
            if (!rc) x->mg[g][k] = (uint64_t)ag.sum;
        }
        sp += x->cp[k][g];
    }
    x->o1[g] = (int32_t*)pj_alloc(&rc, m * 4, 2);
    if (!rc && m) rc = mq_join_write(j, NULL, x->o1[g], NULL, s->stream);
    rc = pj_end(s, rc);
    if (j) mq_join_free(j);
    /* stream-ordered: on an error path peer copies or the build may still be queued */
    mq_pool_free_on(jk, s->stream);
    mq_pool_free_on(jp, s->stream);
    mq_pool_free_on(jq, s->stream);
    s->rc = rc;
}

static void t_pj_place(Shard* s, void* a) {
    PJ* x = (PJ*)a;
    const int i = s->idx;
    const uint64_t n = x->n2[i];
    uint64_t M = 0;
    for (int g = 0; g < g_G; g++) M += x->mg[g][i];
    x->m[i] = M;
    int rc = 0;
    uint32_t* cntp = (uint32_t*)pj_alloc(&rc, n * 4, 3);
    int32_t* o1p = (int32_t*)pj_alloc(&rc, M * 4, 3);
    x->out1[i] = (int32_t*)pj_alloc(&rc, M * 4, 3);
    x->out2[i] = (int32_t*)pj_alloc(&rc, M * 4, 3);
    /* from every device g, in g order: this shard's bucket-g rows' counts and pairs */
    uint64_t ac = 0, am = 0;
    for (int g = 0; g < g_G && !rc; g++) {
        uint64_t oc = 0, om = 0; /* the segments of shards before this one on device g */
        for (int k = 0; k < i; k++) {
            oc += x->cp[k][g];
            om += x->mg[g][k];
        }
        const int dv = g_sh[g].dev;
        rc = mq_memcpy_peer(cntp + ac, s->dev, x->cnt[g] + oc, dv, x->cp[i][g] * 4, s->stream);
        if (!rc) rc = mq_memcpy_peer(o1p + am, s->dev, x->o1[g] + om, dv, x->mg[g][i] * 4, s->stream);
        ac += x->cp[i][g];
        am += x->mg[g][i];
    }
    if (!rc) rc = mq_pjoin_place(cntp, o1p, x->inv[i], x->p2[i], n, M, x->out1[i], x->out2[i], s->stream);
    rc = pj_end(s, rc);
    mq_pool_free_on(cntp, s->stream);
    mq_pool_free_on(o1p, s->stream);
    s->rc = rc;
}

static void pj_free_temps(PJ* x) {
    for (int g = 0; g < g_G; g++) {
        mq_pool_free(x->bk[g]);
        mq_pool_free(x->bp[g]);
        mq_pool_free(x->pk[g]);
        mq_pool_free(x->inv[g]);
        mq_pool_free(x->cnt[g]);
        mq_pool_free(x->o1[g]);
        x->bk[g] = x->bp[g] = x->pk[g] = x->o1[g] = NULL;
        x->inv[g] = x->cnt[g] = NULL;
    }
}

/* The three phases; every worker synchronises its stream before a phase ends, error or
 * not (pj_end), so the next phase's peer copies read finished data and, on error, the
 * caller's thread frees x's buffers only after every queued use of them has run. */
static int pj_run(PJ* x) {
    double t0 = shim_now();
    if (g_G == 1) { /* one shard: the local join alone (timed as the join phase) */
        int rc = run_all(t_pj_single, x);
        double t1 = shim_now();
        x->ms[0] = x->ms[2] = 0;
        x->ms[1] = x->ms[3] = 1e3 * (t1 - t0);
        if (rc) {
            mq_pool_free(x->out1[0]);
            mq_pool_free(x->out2[0]);
            x->out1[0] = x->out2[0] = NULL;
        }
        return rc;
    }
    int rc = run_all(t_pj_part, x);
    double t1 = shim_now();
    if (!rc) rc = run_all(t_pj_join, x);
    double t2 = shim_now();
    if (!rc) rc = run_all(t_pj_place, x);
    double t3 = shim_now();
    pj_free_temps(x);
    x->ms[0] = 1e3 * (t1 - t0);
    x->ms[1] = 1e3 * (t2 - t1);
    x->ms[2] = 1e3 * (t3 - t2);
    x->ms[3] = 1e3 * (t3 - t0);
    if (rc)
        for (int g = 0; g < g_G; g++) {
            mq_pool_free(x->out1[g]);
            mq_pool_free(x->out2[g]);
            x->out1[g] = x->out2[g] = NULL;
        }
    return rc;
}

static double g_pj_ms[4];

void mq_shard_join_times(double* ms) {
    for (int k = 0; k < 4; k++) ms[k] = g_pj_ms[k];
}

int mq_shard_join(const int32_t* const* d_c1, const int32_t* const* d_p1, const uint64_t* n1,
                  const int32_t* const* d_c2, const int32_t* const* d_p2, const uint64_t* n2, int32_t** d_out1,
                  int32_t** d_out2, uint64_t* h_m) {
    configure();
    Status st;
    if (g_G < 1) return MQ_EINVAL;
    if (start(&st)) return MQ_ENODEV;
    PJ* x = (PJ*)calloc(1, sizeof(PJ));
    if (!x) return MQ_ENOMEM;
    int rc = run_all(t_pj_fence, NULL);
    if (rc) {
        free(x);
        return rc;
    }
    for (int g = 0; g < g_G; g++) {
        x->c1[g] = d_c1[g];
        x->p1[g] = d_p1[g];
        x->n1[g] = n1[g];
        x->c2[g] = d_c2[g];
        x->p2[g] = d_p2[g];
        x->n2[g] = n2[g];
    }
    rc = pj_run(x);
    for (int k = 0; k < 4; k++) g_pj_ms[k] = x->ms[k];
    for (int g = 0; g < g_G && !rc; g++) {
        d_out1[g] = x->out1[g];
        d_out2[g] = x->out2[g];
        h_m[g] = x->m[g];
    }
    free(x);
    return rc;
}

int mq_shard_devices(int* devices, int max) {
    configure();
    for (int g = 0; g < g_G && g < max; g++) devices[g] = g_sh[g].dev;
    return g_G;
}

/* Whether hash_join / nested_loop_join fan out: shards on, and a probe side of at
 * least MQ_SHARD_MIN_ROWS rows (the row count columns shard at). */
int shard_join_wants(size_t n1, size_t n2) {
    configure();
    if (!(g_G > 1 && n2 >= g_min_rows && n1 <= (size_t)INT32_MAX && n2 <= (size_t)INT32_MAX)) return 0;
    if (g_started == 0) {
        Status tmp;
        (void)start(&tmp);
    }
    return g_started == 1;
}

/* one side's shard pieces (values a, positions b): the sharded shadows when both have
 * them with one split, else uploads of the split_of(n) row ranges */
typedef struct {
    const Result* r[2];
    size_t off[MAXS + 1];
    void* dev[2][MAXS];
    int owned;
} PjSide;

typedef struct {
    PjSide* side;
} PjUpArg;

static void t_pj_upload(Shard* s, void* a) {
    PjSide* x = ((PjUpArg*)a)->side;
    const size_t b0 = x->off[s->idx], n = x->off[s->idx + 1] - b0;
    for (int k = 0; k < 2; k++) {
        if ((s->rc = mq_pool_malloc(&x->dev[k][s->idx], (n ? n : 1) * 4))) return;
        double t0 = shim_now();
        if (n) s->rc = mq_memcpy_h2d(x->dev[k][s->idx], (const int32_t*)x->r[k]->payload + b0, n * 4, s->stream);
        s->xfer += shim_now() - t0;
        if (s->rc) return;
    }
    s->rc = mq_stream_sync(s->stream);
}

static int pj_side(PjSide* x, const Result* a, const Result* b) {
    memset(x, 0, sizeof *x);
    x->r[0] = a;
    x->r[1] = b;
    const size_t n = a->num_tuples;
    /* (a lookup may drop a stale entry and move another into its slot: look a up again) */
    int ia = ssh_find(a->payload, n);
    const int ib = ia >= 0 ? ssh_find(b->payload, n) : -1;
    if (ib >= 0) ia = ssh_find(a->payload, n);
    if (ia >= 0 && ib >= 0 && memcmp(g_ssh[ia].off, g_ssh[ib].off, sizeof(size_t) * (size_t)(g_G + 1)) == 0) {
        memcpy(x->off, g_ssh[ia].off, sizeof(size_t) * (size_t)(g_G + 1));
        memcpy(x->dev[0], g_ssh[ia].dev, sizeof(void*) * (size_t)g_G);
        memcpy(x->dev[1], g_ssh[ib].dev, sizeof(void*) * (size_t)g_G);
        return 0;
    }
    split_of(n, x->off);
    x->owned = 1;
    PjUpArg u = {x};
    int rc = run_all(t_pj_upload, &u);
    if (rc) {
        free_pieces(x->dev[0]);
        free_pieces(x->dev[1]);
    }
    return rc;
}

static void pj_side_free(PjSide* x) {
    if (!x->owned) return;
    free_pieces(x->dev[0]);
    free_pieces(x->dev[1]);
}

typedef struct {
    PJ* pj;
    int32_t* payload[2];
    size_t off[MAXS + 1];
    int keep[2];
} PjOutArg;

static void t_pj_download(Shard* s, void* a) {
    PjOutArg* x = (PjOutArg*)a;
    const size_t m = x->pj->m[s->idx];
    int32_t* dev[2] = {x->pj->out1[s->idx], x->pj->out2[s->idx]};
    for (int k = 0; k < 2 && !s->rc; k++)
        s->rc = download(s, x->payload[k] + x->off[s->idx], dev[k], m * 4, x->keep[k]);
    if (!s->rc) s->rc = mq_stream_sync(s->stream);
}

/* hash_join (query.c:652-696) with the build side (c1, p1) and the probe side (c2, p2)
 * over the shards; swap puts the probe positions first (nested_loop_join). */
Result** shard_hash_join(Result* c1, Result* p1, Result* c2, Result* p2, int swap, Status* st) {
    const double t0 = shim_now();
    PjSide bs, ps;
    int rc = pj_side(&bs, c1, p1);
    if (rc) {
        shim_fail(st, "shard join upload", rc);
        return NULL;
    }
    if ((rc = pj_side(&ps, c2, p2))) {
        pj_side_free(&bs);
        shim_fail(st, "shard join upload", rc);
        return NULL;
    }
    PJ* x = (PJ*)calloc(1, sizeof(PJ));
    PjOutArg* o = (PjOutArg*)calloc(1, sizeof(PjOutArg));
    if (!x || !o) {
        free(x);
        free(o);
        pj_side_free(&bs);
        pj_side_free(&ps);
        shim_fail(st, "shard join", MQ_ENOMEM);
        return NULL;
    }
    for (int g = 0; g < g_G; g++) {
        x->c1[g] = (const int32_t*)bs.dev[0][g];
        x->p1[g] = (const int32_t*)bs.dev[1][g];
        x->n1[g] = bs.off[g + 1] - bs.off[g];
        x->c2[g] = (const int32_t*)ps.dev[0][g];
        x->p2[g] = (const int32_t*)ps.dev[1][g];
        x->n2[g] = ps.off[g + 1] - ps.off[g];
    }
    rc = pj_run(x);
    for (int k = 0; k < 4; k++) g_pj_ms[k] = x->ms[k];
    pj_side_free(&bs);
    pj_side_free(&ps);
    Result** out = NULL;
    if (!rc) {
        o->pj = x;
        o->off[0] = 0;
        for (int g = 0; g < g_G; g++) o->off[g + 1] = o->off[g] + x->m[g];
        const size_t M = o->off[g_G];
        for (int k = 0; k < 2; k++) {
            o->payload[k] = (int32_t*)shim_payload_alloc(M * 4);
            o->keep[k] = o->payload[k] && keep_payload(o->payload[k], M * 4);
            if (!o->payload[k]) rc = MQ_ENOMEM;
        }
        if (!rc) rc = run_all(t_pj_download, o);
        if (!rc) {
            out = (Result**)malloc(2 * sizeof(Result*));
            /* the pieces stay as the payloads' sharded shadows (rows 0: not positions of a
             * column split, so fetch_column does not take them) */
            Result* r1 = finish(o->payload[0], M, 0, o->off, (void**)x->out1, o->keep[0]);
            Result* r2 = finish(o->payload[1], M, 0, o->off, (void**)x->out2, o->keep[1]);
            out[0] = swap ? r2 : r1;
            out[1] = swap ? r1 : r2;
        } else {
            free(o->payload[0]);
            free(o->payload[1]);
            free_pieces((void**)x->out1);
            free_pieces((void**)x->out2);
        }
    }
    free(x);
    free(o);
    if (rc) {
        shim_fail(st, "shard hash_join", rc);
        return NULL;
    }
    if (shim_trace_on()) fprintf(stderr, "mq-trace shard_hash_join(G=%d)  %9.3f ms\n", g_G, 1e3 * (shim_now() - t0));
    st->code = OK;
    return out;
}

/* ------------------------------------------------------------------ */
/* bookkeeping                                                        */
/* ------------------------------------------------------------------ */

void shard_op_begin(void) {
    if (g_started != 1) return;
    for (int i = g_nscols - 1; i >= 0; i--) /* unguardable host rows: single-use copies */
        if (g_scols[i].op != shim_op() && !g_scols[i].guard) scol_drop(i);
    for (int i = g_nssh - 1; i >= 0; i--)
        if (g_ssh[i].op != shim_op() && !g_ssh[i].guard) ssh_drop(i);
    ssh_make_room(0);
}

int shard_upload(Column* c, Status* st) { return scol_get(c, st) ? 0 : -1; }

void shard_forget_column(const Column* c) {
    for (int i = 0; i < g_nscols; i++)
        if (g_scols[i].col == c) {
            scol_drop(i);
            return;
        }
}

static void t_trim(Shard* s, void* a) {
    (void)a;
    mq_stream_sync(s->stream);
    mq_pool_free(s->ws);
    mq_pool_free(s->scratch);
    s->ws = s->scratch = NULL;
    s->ws_bytes = s->scratch_bytes = 0;
    mq_trim();
}

void shard_release_all(void) {
    if (g_started != 1) return;
    while (g_nscols) scol_drop(g_nscols - 1);
    while (g_nssh) ssh_drop(g_nssh - 1);
    run_all(t_trim, NULL);
}

void shard_stats(mq_residency* out) {
    configure();
    out->shards = (uint64_t)g_G;
    out->shard_columns = (uint64_t)g_nscols;
    out->shard_shadows = (uint64_t)g_nssh;
    out->shard_ops = g_ops;
    out->shard_uploads = g_uploads;
}

static void t_stop(Shard* s, void* a) {
    (void)a;
    if (s->stream) { /* a worker whose t_init failed early has nothing on its device */
        t_trim(s, NULL);
        mq_stream_destroy(s->stream);
    }
    mq_free(s->small);
    mq_thread_release(); /* the worker's pinned staging (it exits after this task) */
    s->stream = s->small = NULL;
    s->quit = 1;
}

/* mq_shard_config (mq_query.h): drop every sharded copy, stop the workers, then take
 * the new layout (G <= 0: back to the environment's). */
int mq_shard_config(int shards, const int* devices, int ndev, uint64_t min_rows) {
    if (g_started == 1) shard_release_all();
    stop_workers();
    g_started = 0;
    g_G = -1;
    if (shards <= 0) return MQ_OK;
    if (shards > MAXS || (ndev > 0 && !devices)) return MQ_EINVAL;
    memset(g_sh, 0, sizeof g_sh);
    const char* pe = getenv("MQ_DEVICE");
    const int primary = pe ? atoi(pe) : 0;
    int count = mq_device_count();
    if (count < 1) count = 1;
    for (int g = 0; g < shards; g++) {
        g_sh[g].idx = g;
        g_sh[g].dev = ndev > 0 ? devices[g % ndev] : (primary + g) % count;
        if (g_sh[g].dev < 0 || g_sh[g].dev >= count) return MQ_EINVAL;
    }
    g_min_rows = (size_t)min_rows;
    g_G = shards;
    return MQ_OK;
}
