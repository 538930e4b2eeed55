// payload_probe.hip — host-memory costs around the drop-in API's transfers (not
// product code). Two questions:
//  1. a Result payload is fresh malloc'd memory the caller free()s: what do its page
//     faults and its free cost, with and without transparent huge pages, with and
//     without a write guard (mprotect) on it, faulted by 1 or 4 threads?
//  2. a column lives in a file mapping (start_data, here a memfd) that libmq uploads
//     and then write-protects: which upload path reaches the link rate without making
//     the later mprotect stall the GPU (a pageable hipMemcpy registers the pages)?
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/payload_probe.hip -o tools/payload_probe -lpthread
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <thread>
#include <vector>

#ifndef MADV_POPULATE_WRITE
#define MADV_POPULATE_WRITE 23
#endif

#define CK(x)                                                                    \
    do {                                                                         \
        hipError_t e = (x);                                                      \
        if (e != hipSuccess) {                                                   \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));               \
            exit(1);                                                             \
        }                                                                        \
    } while (0)

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static void par(int nt, size_t bytes, const std::function<void(size_t, size_t)>& f) {
    std::vector<std::thread> th;
    for (int i = 1; i < nt; i++) th.emplace_back([&, i] { f(bytes * i / nt, bytes * (i + 1) / nt); });
    f(0, bytes / nt);
    for (auto& x : th) x.join();
}

__global__ void k_tiny(int* p) {
    if (threadIdx.x == 0) p[0] += 1;
}

static double med(std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

int main(int argc, char** argv) {
    const size_t bytes = argc > 1 ? strtoull(argv[1], nullptr, 10) : 40000000ull;
    const size_t colb = argc > 2 ? strtoull(argv[2], nullptr, 10) : ((size_t)1 << 30);
    const long pg = sysconf(_SC_PAGESIZE);
    int* dtiny;
    CK(hipMalloc(&dtiny, 4096));
    CK(hipMemset(dtiny, 0, 4096));
    auto tiny_ms = [&] {
        double t0 = now();
        hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, 0, dtiny);
        CK(hipDeviceSynchronize());
        return 1e3 * (now() - t0);
    };
    tiny_ms();

    // ---- 1. payload lifecycle ----
    for (int thp : {0, 1})
        for (int nt : {1, 4})
            for (int guard : {0, 1}) {
                std::vector<double> ta, tf, tp, tfr;
                for (int r = 0; r < 9; r++) {
                    double t0 = now();
                    char* p = (char*)malloc(bytes);
                    const uintptr_t a = ((uintptr_t)p + pg - 1) & ~(uintptr_t)(pg - 1);
                    const uintptr_t e = ((uintptr_t)p + bytes) & ~(uintptr_t)(pg - 1);
                    if (thp) madvise((void*)a, e - a, MADV_HUGEPAGE);
                    double t1 = now();
                    par(nt, bytes, [&](size_t x, size_t y) { memset(p + x, 1, y - x); });
                    double t2 = now();
                    if (guard) mprotect((void*)a, e - a, PROT_READ);
                    double t3 = now();
                    free(p);
                    double t4 = now();
                    ta.push_back(t1 - t0);
                    tf.push_back(t2 - t1);
                    tp.push_back(t3 - t2);
                    tfr.push_back(t4 - t3);
                }
                printf("{\"probe\": \"payload\", \"bytes\": %zu, \"thp\": %d, \"threads\": %d, \"guard\": %d, "
                       "\"ms_alloc\": %.3f, \"ms_first_touch\": %.3f, \"ms_mprotect\": %.3f, \"ms_free\": %.3f}\n",
                       bytes, thp, nt, guard, 1e3 * med(ta), 1e3 * med(tf), 1e3 * med(tp), 1e3 * med(tfr));
                fflush(stdout);
            }

    // ---- 2. column upload from a populated file mapping ----
    void* dcol;
    CK(hipMalloc(&dcol, colb));
    auto memfd_col = [&] {
        int fd = memfd_create("col", 0);
        if (ftruncate(fd, (off_t)colb) != 0) exit(1);
        char* m = (char*)mmap(nullptr, colb, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        close(fd);
        par(8, colb, [&](size_t x, size_t y) { memset(m + x, 3, y - x); });
        return m;
    };
    struct Path {
        const char* name;
        int mode;
    };
    // 0: hipMemcpy then mprotect; 1: mprotect then hipMemcpy; 2: hipHostRegister(ReadOnly)
    // + DMA + unregister, then mprotect; 3: hipHostRegister default + DMA + unregister + mprotect
    for (Path P : {Path{"memcpy_then_guard", 0}, Path{"guard_then_memcpy", 1}, Path{"register_ro", 2},
                   Path{"register_default", 3}}) {
        for (int r = 0; r < 3; r++) {
            char* m = memfd_col();
            double t0 = now(), t1, t2, t3;
            hipError_t err = hipSuccess;
            if (P.mode == 0) {
                err = hipMemcpy(dcol, m, colb, hipMemcpyHostToDevice);
                t1 = now();
                mprotect(m, colb, PROT_READ);
            } else if (P.mode == 1) {
                mprotect(m, colb, PROT_READ);
                t1 = now();
                err = hipMemcpy(dcol, m, colb, hipMemcpyHostToDevice);
            } else {
                err = hipHostRegister(m, colb, P.mode == 2 ? hipHostRegisterReadOnly : hipHostRegisterDefault);
                if (err == hipSuccess) {
                    void* dp = nullptr;
                    CK(hipHostGetDevicePointer(&dp, m, 0));
                    err = hipMemcpy(dcol, m, colb, hipMemcpyHostToDevice);
                    CK(hipHostUnregister(m));
                }
                t1 = now();
                mprotect(m, colb, PROT_READ);
            }
            t2 = now();
            const double k1 = tiny_ms();
            const double k2 = tiny_ms();
            t3 = now();
            printf("{\"probe\": \"column_upload\", \"path\": \"%s\", \"bytes\": %zu, \"rep\": %d, \"err\": \"%s\", "
                   "\"ms_copy\": %.2f, \"gbs\": %.1f, \"ms_to_guarded\": %.2f, \"ms_next_kernel\": %.3f, "
                   "\"ms_second_kernel\": %.3f}\n",
                   P.name, colb, r, hipGetErrorString(err), 1e3 * (t1 - t0), colb / (t1 - t0) / 1e9,
                   1e3 * (t2 - t0), k1, k2);
            fflush(stdout);
            (void)t3;
            munmap(m, colb);
        }
    }
    return 0;
}
