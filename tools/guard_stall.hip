// guard_stall.hip — does write-protecting host memory that a HIP copy just used
// stall the next GPU work? (The API path's result shadows measured 11-28 ms for a
// 40 MB device copy right after mq_guard_arm's mprotect of the payload.)
//   hipcc --offload-arch=gfx950 -O2 tools/guard_stall.hip -o tools/guard_stall && tools/guard_stall
#include <hip/hip_runtime.h>
#include <sys/mman.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e = (x);                                                     \
        if (e != hipSuccess) {                                                  \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));              \
            exit(1);                                                            \
        }                                                                       \
    } while (0)

__global__ void k_touch(int* p, size_t n) {
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i < n) p[i] += 1;
}

static double ms(std::chrono::steady_clock::time_point a) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a).count();
}

int main() {
    const size_t bytes = 40u << 20, n = bytes / 4;
    int* d;
    CK(hipMalloc(&d, bytes));
    CK(hipMemset(d, 1, bytes));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    void* pinned;
    CK(hipHostMalloc(&pinned, bytes, 0));
    const char* names[] = {"d2h pageable, no mprotect", "d2h pageable, mprotect RO", "d2h pinned+memcpy, mprotect RO",
                           "d2h pageable, mprotect RO, munmap", "h2d pageable, mprotect RO"};
    for (int mode = 0; mode < 5; mode++) {
        for (int rep = 0; rep < 4; rep++) {
            char* h = (char*)mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
            memset(h, 0, bytes);
            auto t0 = std::chrono::steady_clock::now();
            if (mode == 2) {
                CK(hipMemcpyAsync(pinned, d, bytes, hipMemcpyDeviceToHost, st));
                CK(hipStreamSynchronize(st));
                memcpy(h, pinned, bytes);
            } else if (mode == 4) {
                CK(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, st));
                CK(hipStreamSynchronize(st));
            } else {
                CK(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, st));
                CK(hipStreamSynchronize(st));
            }
            const double t_copy = ms(t0);
            t0 = std::chrono::steady_clock::now();
            if (mode != 0) mprotect(h, bytes, PROT_READ);
            const double t_prot = ms(t0);
            t0 = std::chrono::steady_clock::now();
            hipLaunchKernelGGL(k_touch, dim3((n + 255) / 256), dim3(256), 0, st, d, n);
            CK(hipStreamSynchronize(st));
            const double t_k = ms(t0);
            t0 = std::chrono::steady_clock::now();
            hipLaunchKernelGGL(k_touch, dim3((n + 255) / 256), dim3(256), 0, st, d, n);
            CK(hipStreamSynchronize(st));
            const double t_k2 = ms(t0);
            t0 = std::chrono::steady_clock::now();
            munmap(h, bytes);
            const double t_un = ms(t0);
            t0 = std::chrono::steady_clock::now();
            hipLaunchKernelGGL(k_touch, dim3((n + 255) / 256), dim3(256), 0, st, d, n);
            CK(hipStreamSynchronize(st));
            const double t_k3 = ms(t0);
            printf("%-36s rep %d: copy %7.3f  mprotect %7.3f  kernel %7.3f  kernel2 %7.3f  munmap %7.3f  kernel3 %7.3f ms\n",
                   names[mode], rep, t_copy, t_prot, t_k, t_k2, t_un, t_k3);
        }
    }
    return 0;
}
