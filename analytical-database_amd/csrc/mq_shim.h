/* mq_shim.h — internal interface between the query shim (mq_query.c) and its row-shard
 * executor (mq_shard.c). Not installed; nothing here is part of the C-ABI. */
#ifndef MQ_SHIM_H
#define MQ_SHIM_H

#include <stddef.h>
#include <stdint.h>

#include "mq_device.h"
#include "mq_query.h"

/* Payloads from this size on keep an HBM shadow (mq_query.c lowers glibc's mmap
 * threshold to it, so they are mmapped chunks, which a write guard can cover). */
#define SHADOW_MIN_BYTES ((size_t)1 << 20)

/* ---- provided by mq_query.c ---- */
double shim_now(void);
int shim_trace_on(void);
int shim_fail(Status* st, const char* what, int rc);
void* shim_payload_alloc(size_t bytes);
Result* shim_new_result(DataType t, size_t n, void* payload);
unsigned long long shim_op(void);          /* the current operator's number */
size_t shim_shadow_budget(void);           /* MQ_SHADOW_MB in bytes */
mq_residency* shim_stats(void);
void shim_xfer_add(double seconds);        /* PCIe time, mq_transfer_seconds */

/* ---- provided by mq_shard.c: long columns split into row shards over devices ----
 * MQ_SHARDS=G (default: the number of entries of MQ_DEVICES, else 1) row shards, shard g
 * on device MQ_DEVICES[g] (default: (primary + g) % device count); columns of at least
 * MQ_SHARD_MIN_ROWS rows (default 2^24) are served by the shards. */
int shard_count(void);
int shard_wants(const Column* c);
/* select_column_scan (query.c:92-137): each shard selects its rows; the position lists
 * are concatenated in shard order straight into the host payload. */
Result* shard_select(Column* c, int* low, int* high, Status* st);
/* fetch_column (query.c:223-243) when `pos` came from a sharded select over a column of
 * the same row count: each shard gathers its own positions. 1 = done (*out set), 0 =
 * not applicable (the caller takes the one-device path), -1 = error. */
int shard_fetch(Column* c, Result* pos, Result** out, Status* st);
/* sum of a column (query.c:336-342): per-shard partials folded on the host */
int shard_reduce_column(Column* c, mq_agg* a, Status* st);
/* sum/avg/min/max of a Result produced by the shards (query.c:306-437): 1 done, 0 not
 * sharded, -1 error */
int shard_reduce_result(const Result* r, mq_agg* a, Status* st);
/* shared_select (query.c:439-583) over a sharded column */
Result** shard_shared_select(SelectOperator* ops, int q, Column* c, Status* st);
/* hash_join (query.c:652-696) key-partitioned over the shards: the
 * build side (c1, p1), the probe side (c2, p2); swap = 1 returns the probe positions
 * first (nested_loop_join). */
int shard_join_wants(size_t n1, size_t n2);
Result** shard_hash_join(Result* c1, Result* p1, Result* c2, Result* p2, int swap, Status* st);
void shard_op_begin(void);                 /* sweep + budget at every operator start */
void shard_forget_column(const Column* c);
/* make c resident on the shards now (mq_column_upload of a sharded column): 0 or -1 */
int shard_upload(Column* c, Status* st);
void shard_release_all(void);
void shard_stats(mq_residency* out);

#endif
