/* mq_guard.h — write guards on host memory mirrored in HBM (mq_guard.c). Internal. */
#ifndef MQ_GUARD_H
#define MQ_GUARD_H

#include <stddef.h>
#include <stdint.h>

typedef struct mq_guard_stats {
    uint64_t armed, clean, stale, live, remap_probe;
} mq_guard_stats;

enum { MQ_GUARD_FILE = 0, MQ_GUARD_CHUNK = 1 };

/* 0 when MQ_GUARD=0 (then nothing is guarded and host copies are single-use). */
int mq_guard_enabled(void);
/* 1 when p starts a malloc chunk glibc served with mmap (MQ_GUARD_CHUNK can cover it). */
int mq_guard_chunk_ok(const void* p);
/* Guard [p, p+bytes); returns a handle, or 0 when the memory is not guardable. */
uint64_t mq_guard_arm(const void* p, size_t bytes, int kind);
/* 1 when nothing wrote into [p, p+bytes) since the guard was armed. */
int mq_guard_clean(uint64_t handle, const void* p, size_t bytes);
/* Lift the guard (restores the pages' protection) and free the handle. */
void mq_guard_release(uint64_t handle);
/* Before libmq itself writes into host memory: lift any guard over the range and
 * mark it dirty. */
void mq_guard_forget_range(uintptr_t addr, size_t bytes);
mq_guard_stats mq_guard_get_stats(void);
/* Test hook for the fault handler's per-thread retry table: get = 0 records tag for
 * thread id tid (0 when the table has no live-free slot), get = 1 returns the tag
 * recorded for tid (0 = none, or dead). */
int mq_guard_retry_test(uint32_t tid, uint32_t tag, int get);

#endif
