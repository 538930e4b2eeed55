/*
 * mq_query.h — libmq's drop-in for the reference's operator API.
 *
 * libmq exports exactly the symbols of siyaoL1/Analytical-Database
 * src/include/query.h:20-50, with identical C signatures and struct layouts, so
 * the reference's server.o parse.o client_context.o db_manager.o index.o utils.o
 * link against libmq.so in place of query.o multimap.o (src/Makefile:62).
 * Each entry point below cites the reference function it replaces.
 *
 * The types are re-declared here layout-for-layout from
 * src/include/cs165_api.h:58-132,152-206 and src/include/db_manager.h:95-108;
 * mq_query.c pins every size and offset with _Static_assert (x86-64 SysV).
 * The reference's own headers stay authoritative for its translation units;
 * this header is what libmq itself is compiled against.
 *
 * Ownership (reference contract, client_context.c:31-90, server.c:432):
 * every returned Result / Result** and every payload is malloc'd host memory
 * that the caller frees with free(). Inputs are borrowed.
 * Device residency: a Column's rows are uploaded to HBM on first use and kept
 * while a write guard shows them unchanged; Results produced by libmq keep a
 * device shadow on the same terms (see "residency control" below).
 */
#ifndef MQ_QUERY_H
#define MQ_QUERY_H

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- reference ABI types (cs165_api.h) ---- */
#define MQ_MAX_SIZE_NAME 64
#define MQ_HANDLE_MAX_SIZE 64

typedef enum DataType { INT, LONG, FLOAT, DOUBLE } DataType;          /* cs165_api.h:58-63 */

typedef struct ColumnIndex {                                          /* cs165_api.h:65-68 */
    int* values;
    size_t* positions;
} ColumnIndex;

struct Node;       /* btree node, opaque here (btree.h) */
struct Histogram;  /* opaque here (cs165_api.h:71-75) */

typedef struct Column {                                               /* cs165_api.h:77-92 */
    char name[MQ_MAX_SIZE_NAME];
    int* data;
    int fd;
    size_t row_count;
    bool sorted;
    bool clustered;
    bool has_index;
    ColumnIndex* index;
    struct Node* btree_node;
    struct Histogram* histogram;
    int max;
    int min;
} Column;

typedef enum StatusCode { OK, ERROR } StatusCode;                    /* cs165_api.h:152-157 */

typedef struct Status {                                               /* cs165_api.h:160-163 */
    StatusCode code;
    char* error_message;
} Status;

typedef struct Result {                                               /* cs165_api.h:179-183 */
    size_t num_tuples;
    DataType data_type;
    void* payload;
} Result;

typedef enum GeneralizedColumnType { RESULT, COLUMN } GeneralizedColumnType;  /* cs165_api.h:188-191 */

typedef union GeneralizedColumnPointer {                              /* cs165_api.h:195-198 */
    Result* result;
    Column* column;
} GeneralizedColumnPointer;

typedef struct GeneralizedColumn {                                    /* cs165_api.h:203-206 */
    GeneralizedColumnType column_type;
    GeneralizedColumnPointer column_pointer;
} GeneralizedColumn;

typedef struct Table {                                                /* cs165_api.h:110-116 */
    char name[MQ_MAX_SIZE_NAME];
    Column* columns;
    size_t col_count;
    size_t row_count;
    size_t table_length;
} Table;

typedef struct Db {                                                   /* cs165_api.h:127-132 */
    char name[MQ_MAX_SIZE_NAME];
    Table* tables;
    size_t tables_size;
    size_t tables_capacity;
} Db;

/* db_manager.h:95-108; only low/high/column are read by libmq (shared_select). */
typedef struct SelectOperator {
    int select_type;            /* SelectType enum */
    char handle[MQ_HANDLE_MAX_SIZE];
    int low;
    int high;
    int has_low;
    int has_high;
    void* db;
    void* table;
    Column* column;
    Result* col_result;
    Result* pos_result;
    void* comparator;
} SelectOperator;

/* ---- the reference operator API (query.h:20-50) ---- */
Result* select_result(Result* column, Result* position, int* low_pointer, int* high_pointer,
                      Status* ret_status);                          /* query.c:38-86   */
Result* select_column(Column* column, int* low, int* high, Status* ret_status); /* :203-220 */
Result* fetch_column(Column* column, Result* position_result, Status* ret_status); /* :223-243 */
char* print(Result** result, int result_num, Status* ret_status);  /* query.c:245-304 */
Result* average(Result* column, Status* ret_status);                /* query.c:306-323 */
Result* sum(GeneralizedColumn* column, Status* ret_status);          /* query.c:325-354 */
Result* add(Result* column_one, Result* column_two, Status* ret_status);   /* :356-372 */
Result* sub(Result* column_one, Result* column_two, Status* ret_status);   /* :374-390 */
Result* min(Result* column, Status* ret_status);                    /* query.c:392-415 */
Result* max(Result* column, Status* ret_status);                    /* query.c:417-437 */
Result** shared_select(SelectOperator* operators, int query_count, Column* column,
                       Status* ret_status);                         /* query.c:496-583 */
Result** nested_loop_join(Result* column_one, Result* position_one, Result* column_two,
                          Result* position_two, Status* ret_status); /* query.c:585-650 */
Result** hash_join(Result* column_one, Result* position_one, Result* column_two,
                   Result* position_two, Status* ret_status);       /* query.c:652-696 */
void log_result(Result* result);                                    /* query.c:26-36   */
/* also global (undeclared in query.h) in the reference: */
Result* select_column_scan(Column* column, int* low_pointer, int* high_pointer,
                           Status* ret_status);                     /* query.c:92-137  */
Result* select_column_sorted_index(Column* column, int low, int high,
                                   Status* ret_status);             /* query.c:165-198 */
/* index.c:180-185 — exported weak so the reference's index.o definition wins. */
bool should_use_index(Column* column, int low, int high);

/* ---- J4: hashset.h (src/include/hashset.h:7-24) ----
 * hashset.c is not linked into the reference server and has no caller
 * (src/Makefile:62); libmq exports its API so that code
 * written against hashset.h links, with the reference's semantics: `size` int32
 * slots, 0 = empty (0 is never a member), linear probing from hash(key, size).
 * Defined where the reference leaves undefined behaviour: the slots start zeroed
 * (create_hashset mallocs them uninitialised, hashset.c:13), a negative key's probe
 * starts at the wrapped remainder (the reference indexes out of bounds), a full
 * table stops after one lap (it loops forever), and get_hashset_elements returns a
 * buffer sized for its elements (hashset.c:49 allocates 16 bytes). Its element
 * listing runs on the GPU for tables of >= 32768 slots (MQ_HASHSET_GPU_MIN);
 * mq_hashset_lookup (mq_device.h) is the batched device lookup. */
typedef struct hashset {                                              /* hashset.h:7-10 */
    int* keys;
    int size;
} hashset;
int hash(int key, int size);                       /* multimap.c:60-63, exported weak */
hashset* create_hashset(int size);                 /* hashset.c:11-16 */
void free_hashset(hashset* set);                   /* hashset.c:19-22 */
void insert_hashset(hashset* set, int key);        /* hashset.c:25-32 */
bool lookup_hashset(hashset* set, int key);        /* hashset.c:35-45 */
Result* get_hashset_elements(hashset* set);        /* hashset.c:48-65 */

/* ---- the load path (db_manager.h:254) ----
 * load_db (db_manager.c:240-322 with insert_row :164-199): same header check
 * (db name, table name), same rows, values, min/max and table_length growth, with
 * the data lines parsed on the GPU (mq_csv_parse_int32). Capacity grows through
 * the server's own save_data / start_data (db_manager.c:430,736), which libmq
 * references weakly: without them (no server linked) a load that must grow the
 * table fails with ERROR. The loaded columns stay resident in HBM for the queries
 * that follow. To use it, the server links this definition instead of
 * db_manager.o's. */
void load_db(Db* db, const char* path, Status* ret_status);

/* ---- the index build (index.c:152-178 build_index, db_manager.h:282) ----
 * For every column with has_index: the sorted copy and its positions on the GPU
 * (mq_index_build), then, as the reference does, clustered: index->positions left
 * 0..n-1 and every other column of the table reordered by the sort permutation;
 * unclustered: index->positions = the permutation plus the 100-bin histogram. The
 * index arrays, histogram and reordered rows are host memory as in the reference
 * (malloc'd / the mmap'd column data); their HBM copies stay resident. Equal values
 * come out in ascending row order (the reference's quicksort orders them its own
 * way). Used like load_db: the server links this definition
 * instead of index.o's. */
void build_index(Db* db);

/* ---- libmq residency control (not in the reference) ----
 * A device copy of host memory (a Column's rows, a Result payload, an index's
 * arrays) is reused by later operators only while a write guard proves the host
 * memory unchanged: the whole pages inside it are read-only, the
 * first write into them faults once and marks the copy stale. Guarded are the
 * reference's column files (any writable file-backed mapping, e.g. start_data's
 * MAP_SHARED column files, or a memfd) and the payloads libmq allocates when glibc
 * serves them with mmap. Any other memory is uploaded again by each operator that
 * reads it. MQ_GUARD=0 turns the guards off (every copy single-use). */
/* Use an existing device copy of column->data (row_count int32 rows in HBM); the
 * caller keeps ownership of d_data and must keep it alive while attached (attached
 * copies are trusted: not guarded). */
int mq_column_attach(Column* column, const int32_t* d_data);
/* Upload column->data now (otherwise done lazily on first use). */
int mq_column_upload(Column* column);
/* Forget the device copy (call after insert_row / reorder / remap of the column). */
void mq_column_invalidate(Column* column);
/* Device pointer of a libmq-produced Result's shadow copy, or NULL. */
const void* mq_result_device_ptr(const Result* result);
/* Row shards: columns of at least min_rows rows are split into `shards`
 * contiguous row ranges, range g resident on device devices[g % ndev] (ndev = 0: the
 * primary device + g, modulo the device count) and served by a host thread and stream
 * of its own; select_column, fetch_column, sum/avg/min/max and shared_select then run
 * on every shard and concatenate / fold in shard order. Replaces the MQ_SHARDS /
 * MQ_DEVICES / MQ_SHARD_MIN_ROWS environment (read at first use); drops every sharded
 * copy first. shards <= 0 returns to the environment's layout. Several shards may
 * share one device (a rehearsal of the split on a one-GPU machine). */
int mq_shard_config(int shards, const int* devices, int ndev, uint64_t min_rows);
/* The current layout: returns the shard count G, devices[g] (up to max) its devices. */
int mq_shard_devices(int* devices, int max);
/* hash_join (query.c:652-696) key-partitioned over the G shards (DESIGN.md
 * §6; hash_join / nested_loop_join take it for probe sides of at least min_rows rows).
 * Shard g holds build rows (d_c1[g], d_p1[g], n1[g]) and probe rows (d_c2[g], d_p2[g],
 * n2[g]) on its device, the ranges of each side in row order (any split). On return
 * shard g's device holds d_out1[g] / d_out2[g]: the h_m[g] pairs of probe rows of range
 * g, in the reference's order; their concatenation over g is hash_join's output. The
 * outputs are pool memory (mq_pool_free). Starts the shard workers if needed.
 * Stream contract: the inputs may still be being written by work the caller queued on
 * ANY stream of the shard devices, the null stream included: mq_shard_join first waits
 * for every shard device to go idle (mq_device_sync on each worker), because its
 * workers run on non-blocking streams of their own that would not wait for that work.
 * On return every output is complete (each worker has synchronised its stream). Work
 * the caller queues concurrently from other threads while the call runs is not
 * ordered against it. */
int mq_shard_join(const int32_t* const* d_c1, const int32_t* const* d_p1, const uint64_t* n1,
                  const int32_t* const* d_c2, const int32_t* const* d_p2, const uint64_t* n2,
                  int32_t** d_out1, int32_t** d_out2, uint64_t* h_m);
/* Host wall ms of the last partitioned join's phases: partition, exchange + local join,
 * return exchange + place, total. */
void mq_shard_join_times(double* ms);
/* Test hook (no reference counterpart): every device allocation of the next
 * mq_shard_join calls' phase `phase` fails with MQ_ENOMEM (1 partition, 2 exchange + local
 * join, 3 return + place, 4 the one-shard join; 0 turns it off). The error paths drain
 * every worker's stream before buffers go back to the pool. */
void mq_shard_join_inject_failure(int phase);
/* Drop every cached device copy. */
void mq_release_all(void);
/* Residency counters since load (tests and the bench read them). */
typedef struct mq_residency {
    uint64_t column_uploads, column_bytes;  /* H2D uploads of column rows */
    uint64_t result_uploads, result_bytes;  /* H2D uploads of Result payloads */
    uint64_t guards_armed, guard_clean, guard_stale, guards_live;
    uint64_t remap_probe;                   /* 1: a remapped range is told apart (MADV_POPULATE_WRITE) */
    uint64_t columns_resident, shadows_resident, shadow_bytes;
    /* row shards (MQ_SHARDS): shard count, sharded columns and result shadows held,
     * sharded operator calls served, sharded column uploads */
    uint64_t shards, shard_columns, shard_shadows, shard_ops, shard_uploads;
} mq_residency;
void mq_residency_stats(mq_residency* out);
/* Seconds spent in host<->device copies by the query API since the last reset. */
double mq_transfer_seconds(int reset);

#ifdef __cplusplus
}
#endif
#endif
