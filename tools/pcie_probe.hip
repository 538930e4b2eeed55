// pcie_probe.hip — what the drop-in API's host transfers can reach on this box (not
// product code). The reference hands every Result to the server as a malloc'd host
// payload (client_context.c:31-90), so each select_column / fetch_column ends in a D2H
// into fresh, free()-able memory; columns arrive from mmap'd files (H2D). Measured:
//   pinned_d2h / pinned_h2d     hipMemcpy to / from hipHostMalloc memory: the link rate
//   fresh_fault_only            malloc + touch every page (the first-touch cost alone)
//   fresh_fault_<t>thr          the same touched by t threads (MADV_POPULATE_WRITE)
//   pageable_fresh              hipMemcpy D2H into fresh malloc'd memory
//   pageable_warm               hipMemcpy D2H into memory already faulted in
//   staged_warm_<t>thr          D2H into pinned, then t threads memcpy into faulted memory
//   staged_fresh_<t>thr         the same into fresh memory (the copy faults the pages)
//   staged_pipe_fresh_<t>thr    4 x 8 MB pinned ring, DMA of chunk c+1.. overlapping the
//                               t-thread copy of chunk c (what mq_memcpy_d2h_staged does)
//   prefault_then_pipe_<t>thr   fresh memory populated by t threads first, then the ring
//   h2d_pageable_warm           hipMemcpy H2D from faulted pageable memory
//   h2d_staged_pipe_<t>thr      t threads copy into the pinned ring, DMA overlapping
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/pcie_probe.hip -o tools/pcie_probe -lpthread
#include <hip/hip_runtime.h>
#include <sys/mman.h>

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

static void populate(void* h, size_t bytes, int nt) {
    par(nt, bytes, [&](size_t a, size_t b) {
        const uintptr_t pa = ((uintptr_t)h + a) & ~(uintptr_t)4095;
        const uintptr_t pb = ((uintptr_t)h + b + 4095) & ~(uintptr_t)4095;
        if (madvise((void*)pa, pb - pa, MADV_POPULATE_WRITE) != 0)
            for (uintptr_t p = pa; p < pb; p += 4096) *(volatile char*)p = 0;
    });
}

int main(int argc, char** argv) {
    const size_t bytes = (argc > 1 ? strtoull(argv[1], nullptr, 10) : 40000000ull);
    const size_t big = (argc > 2 ? strtoull(argv[2], nullptr, 10) : (size_t)256 << 20);
    void* d;
    CK(hipMalloc(&d, std::max(bytes, big)));
    CK(hipMemset(d, 7, std::max(bytes, big)));
    void* pin;
    CK(hipHostMalloc(&pin, std::max(bytes, big), 0));
    constexpr int kBufs = 4;
    constexpr size_t kChunk = (size_t)8 << 20;
    void* ring[kBufs];
    hipEvent_t ev[kBufs];
    for (int i = 0; i < kBufs; i++) {
        CK(hipHostMalloc(&ring[i], kChunk, 0));
        CK(hipEventCreateWithFlags(&ev[i], hipEventDisableTiming));
    }
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    CK(hipDeviceSynchronize());
    void* warm = malloc(std::max(bytes, big));
    memset(warm, 1, std::max(bytes, big));

    auto report = [&](const char* name, size_t nb, std::vector<double> t) {
        std::sort(t.begin() + 1, t.end());
        const double med = t[1 + (t.size() - 1) / 2];
        printf("{\"path\": \"%s\", \"bytes\": %zu, \"ms\": %.3f, \"gbs\": %.1f}\n", name, nb, 1e3 * med, nb / med / 1e9);
        fflush(stdout);
    };
    auto run = [&](const char* name, size_t nb, const std::function<void*()>& fn, bool check = true) {
        std::vector<double> t;
        for (int r = 0; r < 8; r++) {
            double t0 = now();
            void* h = fn();
            t.push_back(now() - t0);
            if (check && h && ((unsigned char*)h)[nb / 2] != 7) printf("BAD %s\n", name);
            if (h && h != warm && h != pin) free(h);
        }
        report(name, nb, t);
    };
    // staged ring D2H: chunk c DMA'd into ring[c % 4]; the copy of chunk c by nt threads
    // overlaps the DMA of chunks c+1..c+3
    auto ring_d2h = [&](void* h, size_t nb, int nt) {
        const size_t nc = (nb + kChunk - 1) / kChunk;
        auto issue = [&](size_t c) {
            const size_t off = c * kChunk, len = std::min(kChunk, nb - off);
            CK(hipMemcpyAsync(ring[c % kBufs], (char*)d + off, len, hipMemcpyDeviceToHost, st));
            CK(hipEventRecord(ev[c % kBufs], st));
        };
        for (size_t c = 0; c < nc && c < (size_t)kBufs; c++) issue(c);
        for (size_t c = 0; c < nc; c++) {
            CK(hipEventSynchronize(ev[c % kBufs]));
            const size_t off = c * kChunk, len = std::min(kChunk, nb - off);
            par(nt, len, [&](size_t a, size_t b) { memcpy((char*)h + off + a, (char*)ring[c % kBufs] + a, b - a); });
            if (c + kBufs < nc) issue(c + kBufs);
        }
    };

    for (size_t nb : {bytes, big}) {
        char name[96];
        snprintf(name, sizeof name, "pinned_d2h");
        run(name, nb, [&] { CK(hipMemcpy(pin, d, nb, hipMemcpyDeviceToHost)); return pin; });
        snprintf(name, sizeof name, "pinned_h2d");
        run(name, nb, [&] { CK(hipMemcpy(d, pin, nb, hipMemcpyHostToDevice)); return (void*)nullptr; }, false);
        snprintf(name, sizeof name, "pageable_warm");
        run(name, nb, [&] { CK(hipMemcpy(warm, d, nb, hipMemcpyDeviceToHost)); return warm; });
        snprintf(name, sizeof name, "h2d_pageable_warm");
        run(name, nb, [&] { CK(hipMemcpy(d, warm, nb, hipMemcpyHostToDevice)); return (void*)nullptr; }, false);
        for (int nt : {4, 8, 16}) {
            snprintf(name, sizeof name, "h2d_staged_pipe_%dthr", nt);
            run(name, nb, [&, nt] {
                const size_t nc = (nb + kChunk - 1) / kChunk;
                for (size_t c = 0; c < nc; c++) {
                    if (c >= (size_t)kBufs) CK(hipEventSynchronize(ev[c % kBufs]));
                    const size_t off = c * kChunk, len = std::min(kChunk, nb - off);
                    par(nt, len, [&](size_t a, size_t b) { memcpy((char*)ring[c % kBufs] + a, (char*)warm + off + a, b - a); });
                    CK(hipMemcpyAsync((char*)d + off, ring[c % kBufs], len, hipMemcpyHostToDevice, st));
                    CK(hipEventRecord(ev[c % kBufs], st));
                }
                CK(hipStreamSynchronize(st));
                return (void*)nullptr;
            }, false);
        }
        CK(hipMemset(d, 7, nb));
        CK(hipDeviceSynchronize());
    }
    // fresh-payload paths at the result size
    run("fresh_fault_only", bytes, [&] {
        void* h = malloc(bytes);
        for (size_t p = 0; p < bytes; p += 4096) ((char*)h)[p] = 7;
        ((char*)h)[bytes / 2] = 7;
        return h;
    });
    for (int nt : {4, 8, 16}) {
        char name[96];
        snprintf(name, sizeof name, "fresh_fault_%dthr", nt);
        run(name, bytes, [&, nt] {
            void* h = malloc(bytes);
            populate(h, bytes, nt);
            ((char*)h)[bytes / 2] = 7;
            return h;
        });
    }
    run("pageable_fresh", bytes, [&] {
        void* h = malloc(bytes);
        CK(hipMemcpy(h, d, bytes, hipMemcpyDeviceToHost));
        return h;
    });
    for (int nt : {4, 8, 16}) {
        char name[96];
        snprintf(name, sizeof name, "staged_warm_%dthr", nt);
        run(name, bytes, [&, nt] {
            CK(hipMemcpy(pin, d, bytes, hipMemcpyDeviceToHost));
            par(nt, bytes, [&](size_t a, size_t b) { memcpy((char*)warm + a, (char*)pin + a, b - a); });
            return warm;
        });
        snprintf(name, sizeof name, "staged_pipe_warm_%dthr", nt);
        run(name, bytes, [&, nt] { ring_d2h(warm, bytes, nt); return warm; });
        snprintf(name, sizeof name, "staged_pipe_fresh_%dthr", nt);
        run(name, bytes, [&, nt] {
            void* h = malloc(bytes);
            ring_d2h(h, bytes, nt);
            return h;
        });
        snprintf(name, sizeof name, "prefault_then_pipe_%dthr", nt);
        run(name, bytes, [&, nt] {
            void* h = malloc(bytes);
            populate(h, bytes, nt);
            ring_d2h(h, bytes, nt);
            return h;
        });
    }
    return 0;
}
