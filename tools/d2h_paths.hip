// d2h_paths.hip — D2H of a result into a fresh malloc'd (free()-able) payload, the
// way the drop-in API must hand results over (not product code). Compares plain
// hipMemcpy into fresh pageable memory with variants that avoid its costs.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/d2h_paths.hip -o tools/d2h_paths -lpthread
#include <hip/hip_runtime.h>
#include <sys/mman.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <algorithm>
#include <vector>

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

int main(int argc, char** argv) {
    const size_t bytes = (argc > 1 ? strtoull(argv[1], nullptr, 10) : 40000000ull);
    void* d;
    CK(hipMalloc(&d, bytes));
    CK(hipMemset(d, 7, bytes));
    void* pin;
    CK(hipHostMalloc(&pin, bytes, 0));
    CK(hipDeviceSynchronize());
    auto run = [&](const char* name, auto fn) {
        std::vector<double> t;
        for (int r = 0; r < 6; r++) {
            double t0 = now();
            void* h = fn();
            t.push_back(now() - t0);
            if (((unsigned char*)h)[bytes / 2] != 7) printf("BAD %s\n", name);
            free(h);
        }
        std::sort(t.begin() + 1, t.end());
        printf("{\"path\": \"%s\", \"bytes\": %zu, \"ms\": %.3f, \"gbs\": %.1f}\n", name, bytes, 1e3 * t[3],
               bytes / t[3] / 1e9);
    };
    run("pageable", [&] {
        void* h = malloc(bytes);
        CK(hipMemcpy(h, d, bytes, hipMemcpyDeviceToHost));
        return h;
    });
    run("pageable_thp", [&] {
        void* h = malloc(bytes);
        madvise((void*)(((uintptr_t)h + 4095) & ~(uintptr_t)4095), bytes - 4096, MADV_HUGEPAGE);
        CK(hipMemcpy(h, d, bytes, hipMemcpyDeviceToHost));
        return h;
    });
    run("register", [&] {
        void* h = malloc(bytes);
        CK(hipHostRegister(h, bytes, hipHostRegisterDefault));
        CK(hipMemcpy(h, d, bytes, hipMemcpyDeviceToHost));
        CK(hipHostUnregister(h));
        return h;
    });
    for (int nt : {1, 4, 8, 16}) {
        char name[64];
        snprintf(name, sizeof name, "pinned_staging_%dthr", nt);
        run(name, [&] {
            void* h = malloc(bytes);
            CK(hipMemcpy(pin, d, bytes, hipMemcpyDeviceToHost));
            std::vector<std::thread> th;
            for (int i = 0; i < nt; i++)
                th.emplace_back([&, i] {
                    const size_t a = bytes * i / nt, b = bytes * (i + 1) / nt;
                    memcpy((char*)h + a, (char*)pin + a, b - a);
                });
            for (auto& x : th) x.join();
            return h;
        });
    }
    return 0;
}
