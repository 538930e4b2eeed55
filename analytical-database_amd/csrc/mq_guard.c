/*
 * mq_guard.c — write guards on host memory that libmq mirrors in HBM.
 *
 * The reference hands libmq host memory that it may later rewrite in place: the
 * clustered index build reorders every other column through the same mmap'd
 * pointer (src/index.c:105-114, reorder_column), insert_row appends through it
 * (src/db_manager.c:190-197). A device copy keyed on (pointer, length) cannot see
 * that. A guard makes any such write visible:
 *
 *   arm    the whole pages inside [p, p+bytes) become read-only (mprotect); the
 *          partial pages at both ends (at most 2 x 4 KB) are copied aside;
 *   write  the first store into a guarded page faults; the SIGSEGV handler gives
 *          the pages their protection back, marks the guard dirty and returns, so
 *          the store re-executes and succeeds (one fault per guard, not per page);
 *   check  clean = not dirty, the edge bytes still equal their copies, and the
 *          read-only pages are still the ones armed (a munmap + fresh mapping at
 *          the same address is writable again: MADV_POPULATE_WRITE, which never
 *          changes content, fails on the armed pages and succeeds on a new map).
 *
 * Only memory whose lifetime ends in munmap is guarded, so a read-only page can
 * never be left behind inside the malloc heap (where a later read(2) into it would
 * fail with EFAULT):
 *   MQ_GUARD_FILE   every page is in a writable file-backed mapping (the
 *                   reference's column files, start_data db_manager.c:736-790, or
 *                   a memfd);
 *   MQ_GUARD_CHUNK  the caller's own malloc chunk that glibc served with mmap
 *                   (freed by munmap); checked from the chunk header.
 * Anything else is not guardable: arm returns 0 and the caller treats its copy as
 * single-use.
 *
 * Not seen: content changed through the page cache (write(2) to a column file)
 * rather than through the mapping; documented in DESIGN.md §1.
 */
#define _GNU_SOURCE
#include "mq_guard.h"

#include <errno.h>
#include <fcntl.h>
#include <signal.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#ifndef MADV_POPULATE_WRITE
#define MADV_POPULATE_WRITE 23
#endif

#define NGUARD 8192

enum { G_FREE = 0, G_ARMED = 1, G_DIRTY = 2 };

typedef struct {
    _Atomic int state;
    uintptr_t lo, hi;       /* read-only pages [lo, hi) (empty when no whole page) */
    int prot;               /* protection restored on a write or at release */
    uint32_t gen;
    const unsigned char* p; /* the guarded range */
    size_t bytes;
    unsigned char* edge;    /* [p, lo) then [hi, p + bytes); the whole range if lo == hi */
    size_t head, tail;
    _Atomic int refs;       /* owners of one handle: a range armed again while armed */
} Guard;

static Guard g_guard[NGUARD];
static _Atomic int g_hw;        /* slots [0, g_hw) may be in use */
static size_t g_page;
static struct sigaction g_prev;
static int g_installed;
static int g_probe = -1;        /* 1: MADV_POPULATE_WRITE tells armed pages apart; 0: not available */
static int g_probe_errno;
static int g_enabled = -1;
static mq_guard_stats g_stats;

static void on_segv(int sig, siginfo_t* si, void* uc);

static size_t page(void) {
    if (!g_page) g_page = (size_t)sysconf(_SC_PAGESIZE);
    return g_page;
}

int mq_guard_enabled(void) {
    if (g_enabled < 0) {
        const char* e = getenv("MQ_GUARD");
        g_enabled = !(e && e[0] == '0');
    }
    return g_enabled;
}

/* Keep the handler first in line: Python's faulthandler (pytest enables it) or
 * anything else installed later would otherwise see the guard faults first. */
static void install(void) {
    struct sigaction cur;
    sigaction(SIGSEGV, NULL, &cur);
    if (g_installed && (cur.sa_flags & SA_SIGINFO) && cur.sa_sigaction == on_segv) return;
    struct sigaction sa;
    memset(&sa, 0, sizeof sa);
    sa.sa_sigaction = on_segv;
    sa.sa_flags = SA_SIGINFO | SA_NODEFER | SA_ONSTACK;
    sigemptyset(&sa.sa_mask);
    if (sigaction(SIGSEGV, &sa, &g_prev) == 0) g_installed = 1;
}

/* Per thread, the address it last returned for without an armed guard (a second
 * fault there in a row is not a race with another handler, so it is handed on).
 * Kept in a lock-free table keyed by thread id rather than in TLS: libmq is
 * dlopen'd, so its TLS is dynamic, and a thread's first __tls_get_addr may allocate,
 * which a signal handler must not do (initial-exec TLS would move the library's
 * whole TLS block into the static surplus, which dlopen refuses). A slot is one
 * word, tid << 32 | h(address), h != 0, plus the CLOCK_MONOTONIC time it was
 * written. An entry only matters for the thread's very next fault (the store
 * re-executes within microseconds), so one older than RETRY_TTL_NS is dead: it is
 * never read back (a later thread that reuses the tid does not inherit its tag) and
 * any thread may take its slot over (a thread whose retried store succeeded never
 * comes back to clear its entry, so without this the table would fill for good).
 * A slot whose h is 0 is idle. Every update is a CAS. */
#define NRETRY 1024
#define RETRY_TTL_NS 250000000ull
static _Atomic uint64_t g_retry[NRETRY];
static _Atomic uint64_t g_retry_ns[NRETRY];

static uint32_t addr_tag(uintptr_t a) { return ((uint32_t)a ^ (uint32_t)((uint64_t)a >> 32)) | 1u; }

static uint64_t now_ns(void) { /* clock_gettime is async-signal-safe */
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

static int retry_live(int i, uint64_t now) {
    return now - atomic_load_explicit(&g_retry_ns[i], memory_order_acquire) < RETRY_TTL_NS;
}

static uint32_t retry_get(uint32_t tid) {
    const uint64_t now = now_ns();
    for (int i = 0; i < NRETRY; i++) {
        const uint64_t v = atomic_load_explicit(&g_retry[i], memory_order_acquire);
        if ((uint32_t)(v >> 32) == tid && (uint32_t)v && retry_live(i, now)) return (uint32_t)v;
    }
    return 0;
}

/* Record h for tid (h = 0: clear every entry of tid); 0 when there was no room (the
 * caller must not count on a retry being remembered then). */
static int retry_set(uint32_t tid, uint32_t h) {
    const uint64_t want = ((uint64_t)tid << 32) | h;
    const uint64_t now = now_ns();
    if (h == 0) {
        for (int i = 0; i < NRETRY; i++) {
            uint64_t v = atomic_load_explicit(&g_retry[i], memory_order_acquire);
            if ((uint32_t)(v >> 32) == tid && (uint32_t)v)
                (void)atomic_compare_exchange_strong(&g_retry[i], &v, (uint64_t)tid << 32);
        }
        return 1;
    }
    /* this thread's entry, else an idle or dead slot */
    for (int pass = 0; pass < 2; pass++)
        for (int i = 0; i < NRETRY; i++) {
            uint64_t v = atomic_load_explicit(&g_retry[i], memory_order_acquire);
            const int mine = (uint32_t)(v >> 32) == tid && (uint32_t)v;
            if (pass == 0 ? !mine : ((uint32_t)v && retry_live(i, now))) continue;
            /* the time first: between the CAS and a later store another thread would see
             * our word with the dead slot's old time and take it over */
            atomic_store_explicit(&g_retry_ns[i], now, memory_order_release);
            if (atomic_compare_exchange_strong(&g_retry[i], &v, want)) {
                if (pass == 1) /* an older entry of ours elsewhere must not shadow this one */
                    for (int k = 0; k < i; k++) {
                        uint64_t o = atomic_load_explicit(&g_retry[k], memory_order_acquire);
                        if ((uint32_t)(o >> 32) == tid && (uint32_t)o)
                            (void)atomic_compare_exchange_strong(&g_retry[k], &o, (uint64_t)tid << 32);
                    }
                return 1;
            }
        }
    return 0;
}

int mq_guard_retry_test(uint32_t tid, uint32_t tag, int get) {
    return get ? (int)retry_get(tid) : retry_set(tid, tag);
}

static void on_segv(int sig, siginfo_t* si, void* uc) {
    const uint32_t tid = (uint32_t)syscall(SYS_gettid);
    const uintptr_t a = (uintptr_t)si->si_addr;
    int hit = 0, covered = 0;
    if (si->si_code == SEGV_ACCERR) {
        const int hw = atomic_load_explicit(&g_hw, memory_order_acquire);
        for (int i = 0; i < hw; i++) {
            Guard* g = &g_guard[i];
            const int state = atomic_load_explicit(&g->state, memory_order_acquire);
            if (state == G_FREE || a < g->lo || a >= g->hi) continue;
            if (state != G_ARMED) {
                covered = 1;
                continue;
            }
            mprotect((void*)g->lo, g->hi - g->lo, g->prot);
            atomic_store_explicit(&g->state, G_DIRTY, memory_order_release);
            hit = 1;
        }
    }
    if (hit) {
        (void)retry_set(tid, 0);
        return;
    }
    /* Another thread's fault on the same guard (or a release) already gave the pages
     * their protection back between this fault and the scan: re-execute the store
     * once. A slot of any live state covering the address says so. */
    if (covered && retry_get(tid) != addr_tag(a) && retry_set(tid, addr_tag(a))) return;
    (void)retry_set(tid, 0);
    /* not ours: hand it on as if we were not here */
    if (g_prev.sa_flags & SA_SIGINFO) {
        if (g_prev.sa_sigaction) {
            g_prev.sa_sigaction(sig, si, uc);
            return;
        }
    } else if (g_prev.sa_handler != SIG_DFL && g_prev.sa_handler != SIG_IGN) {
        g_prev.sa_handler(sig);
        return;
    }
    signal(SIGSEGV, SIG_DFL); /* the faulting access re-executes and terminates the process */
}

/* Does MADV_POPULATE_WRITE distinguish a read-only page (armed) from a writable
 * one on this kernel? Calibrated once on a page of our own. */
static void calibrate(void) {
    if (g_probe >= 0) return;
    g_probe = 0;
    void* m = mmap(NULL, page(), PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (m == MAP_FAILED) return;
    if (madvise(m, page(), MADV_POPULATE_WRITE) == 0 && mprotect(m, page(), PROT_READ) == 0) {
        errno = 0;
        if (madvise(m, page(), MADV_POPULATE_WRITE) != 0 && errno != ENOMEM) {
            g_probe = 1;
            g_probe_errno = errno;
        }
    }
    munmap(m, page());
}

/* 1 when page lo is still a read-only page of ours (or the kernel cannot tell). */
static int still_armed(uintptr_t lo) {
    calibrate();
    if (!g_probe) return 1;
    errno = 0;
    int rc = madvise((void*)lo, page(), MADV_POPULATE_WRITE);
    return rc != 0 && errno == g_probe_errno;
}

/* Protection of [lo, hi) when every page of it lies in writable mappings that are
 * file-backed (want_file) or of any kind; -1 when not, or when they differ. */
static int vma_prot(uintptr_t lo, uintptr_t hi, int want_file) {
    int fd = open("/proc/self/maps", O_RDONLY | O_CLOEXEC);
    if (fd < 0) return -1;
    static char buf[1 << 16];
    size_t have = 0;
    uintptr_t covered = lo;
    int prot = -2, ok = 1, done = 0;
    while (!done && ok) {
        ssize_t r = read(fd, buf + have, sizeof buf - 1 - have);
        if (r <= 0) break;
        have += (size_t)r;
        buf[have] = '\0';
        char* line = buf;
        char* nl;
        while ((nl = strchr(line, '\n'))) {
            *nl = '\0';
            unsigned long s, e, off, ino;
            char perms[8] = {0}, dev[16] = {0};
            if (sscanf(line, "%lx-%lx %7s %lx %15s %lu", &s, &e, perms, &off, dev, &ino) == 6 && e > covered &&
                s < hi) {
                if (s > covered) { ok = 0; break; } /* a hole */
                int p = (perms[0] == 'r' ? PROT_READ : 0) | (perms[1] == 'w' ? PROT_WRITE : 0) |
                        (perms[2] == 'x' ? PROT_EXEC : 0);
                if (!(p & PROT_WRITE) || !(p & PROT_READ) || (want_file && ino == 0) ||
                    (prot != -2 && p != prot)) {
                    ok = 0;
                    break;
                }
                prot = p;
                covered = e;
                if (covered >= hi) { done = 1; break; }
            }
            line = nl + 1;
        }
        have = strlen(line);
        memmove(buf, line, have);
    }
    close(fd);
    return (ok && covered >= hi && prot >= 0) ? prot : -1;
}

static void restore(Guard* g) {
    if (g->hi > g->lo && atomic_load(&g->state) == G_ARMED && still_armed(g->lo))
        mprotect((void*)g->lo, g->hi - g->lo, g->prot);
}

static void slot_free(Guard* g) {
    free(g->edge);
    g->edge = NULL;
    g->gen++;
    atomic_store_explicit(&g->state, G_FREE, memory_order_release);
}

void mq_guard_forget_range(uintptr_t addr, size_t bytes) {
    const uintptr_t a = addr, b = a + bytes;
    const int hw = atomic_load(&g_hw);
    for (int i = 0; i < hw; i++) {
        Guard* g = &g_guard[i];
        if (atomic_load(&g->state) != G_ARMED) continue;
        const uintptr_t ga = (uintptr_t)g->p, gb = ga + g->bytes;
        if (ga < b && a < gb) {
            restore(g);
            atomic_store(&g->state, G_DIRTY); /* its owner sees it unclean */
        }
    }
}

int mq_guard_chunk_ok(const void* p) {
    /* glibc's mmapped chunk: the header (prev_size, size) sits at the start of its own
     * mapping, so p is 16 bytes past a page boundary, and the size word has IS_MMAPPED
     * (0x2) set and counts whole pages. A block from another allocator (a preloaded
     * malloc) almost never looks like that; one that does not is never guarded. */
    if (!p) return 0;
    const uintptr_t chunk = (uintptr_t)p - 2 * sizeof(size_t);
    const size_t sz = ((const size_t*)p)[-1];
    return (chunk & (page() - 1)) == 0 && (sz & 2) != 0 && ((sz & ~(size_t)7) & (page() - 1)) == 0 &&
           (sz & ~(size_t)7) >= page();
}

uint64_t mq_guard_arm(const void* p, size_t bytes, int kind) {
    if (!mq_guard_enabled() || !p || !bytes) return 0;
    const uintptr_t a = (uintptr_t)p, b = a + bytes;
    const uintptr_t pg = page();
    uintptr_t lo = (a + pg - 1) & ~(pg - 1), hi = b & ~(pg - 1);
    if (hi <= lo) lo = hi = 0;
    /* the same range already armed (a column resident both whole on one device and
     * split over the row shards): one more owner of that guard, since a second
     * mprotect-based guard cannot arm over read-only pages */
    const int hw0 = atomic_load(&g_hw);
    for (int i = 0; i < hw0; i++) {
        Guard* g = &g_guard[i];
        if (atomic_load(&g->state) == G_ARMED && g->p == (const unsigned char*)p && g->bytes == bytes &&
            (g->hi == g->lo || still_armed(g->lo))) {
            atomic_fetch_add(&g->refs, 1);
            g_stats.armed++;
            return ((uint64_t)g->gen << 32) | (uint32_t)i;
        }
    }
    int prot = PROT_READ | PROT_WRITE;
    if (kind == MQ_GUARD_CHUNK) {
        if (!mq_guard_chunk_ok(p)) return 0;
    } else {
        if (lo == hi) return 0;
        if ((prot = vma_prot(lo, hi, 1)) < 0) return 0;
    }
    mq_guard_forget_range((uintptr_t)p, bytes);
    int idx = -1;
    const int hw = atomic_load(&g_hw);
    for (int i = 0; i < hw; i++)
        if (atomic_load(&g_guard[i].state) == G_FREE) {
            idx = i;
            break;
        }
    if (idx < 0) {
        if (hw == NGUARD) return 0;
        idx = hw;
    }
    Guard* g = &g_guard[idx];
    const size_t head = lo == hi ? bytes : lo - a, tail = lo == hi ? 0 : b - hi;
    unsigned char* edge = (unsigned char*)malloc(head + tail + 1);
    if (!edge) return 0;
    memcpy(edge, p, head);
    if (tail) memcpy(edge + head, (const void*)hi, tail);
    g->lo = lo;
    g->hi = hi;
    g->prot = prot;
    g->p = (const unsigned char*)p;
    g->bytes = bytes;
    g->edge = edge;
    g->head = head;
    g->tail = tail;
    atomic_store(&g->refs, 1);
    if (!g->gen) g->gen = 1;
    install();
    atomic_store_explicit(&g->state, G_ARMED, memory_order_release);
    if (idx == hw) atomic_store_explicit(&g_hw, hw + 1, memory_order_release);
    if (hi > lo && mprotect((void*)lo, hi - lo, PROT_READ) != 0) {
        slot_free(g);
        return 0;
    }
    g_stats.armed++;
    return ((uint64_t)g->gen << 32) | (uint32_t)idx;
}

static Guard* lookup(uint64_t h) {
    if (!h) return NULL;
    const uint32_t idx = (uint32_t)h;
    if (idx >= NGUARD) return NULL;
    Guard* g = &g_guard[idx];
    return (g->gen == (uint32_t)(h >> 32) && atomic_load(&g->state) != G_FREE) ? g : NULL;
}

static double gnow(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

int mq_guard_clean(uint64_t h, const void* p, size_t bytes) {
    static int tr = -1;
    if (tr < 0) tr = getenv("MQ_TRACE") && getenv("MQ_TRACE")[0] == '1';
    const double t0 = tr ? gnow() : 0;
    Guard* g = lookup(h);
    int ok = g && g->p == (const unsigned char*)p && g->bytes == bytes && atomic_load(&g->state) == G_ARMED &&
             memcmp(g->edge, p, g->head) == 0 &&
             (!g->tail || memcmp(g->edge + g->head, (const void*)g->hi, g->tail) == 0) &&
             (g->hi == g->lo || still_armed(g->lo));
    if (ok) g_stats.clean++;
    else g_stats.stale++;
    if (tr) fprintf(stderr, "mq-trace guard_clean(%zu B)       %9.3f ms\n", bytes, 1e3 * (gnow() - t0));
    return ok;
}

void mq_guard_release(uint64_t h) {
    Guard* g = lookup(h);
    if (!g) return;
    if (atomic_fetch_sub(&g->refs, 1) > 1) return; /* another owner still holds it */
    restore(g);
    slot_free(g);
}

mq_guard_stats mq_guard_get_stats(void) {
    int n = 0;
    const int hw = atomic_load(&g_hw);
    for (int i = 0; i < hw; i++) n += atomic_load(&g_guard[i].state) != G_FREE;
    mq_guard_stats s = g_stats;
    s.live = (uint64_t)n;
    calibrate();
    s.remap_probe = (uint64_t)g_probe;
    return s;
}
