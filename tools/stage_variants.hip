// stage_variants.hip — tuning harness for the one-pass ordered compaction (not product
// code). Includes libmq's kernel source, so it times the product kernels themselves
// and variants of their template knobs, interleaved in one process, on a 1e9-row
// column (SURVEY §8(c) generator), and checks every variant's K against k_scan's.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/stage_variants.hip -o tools/stage_variants
#include "../analytical-database_amd/csrc/mq_kernels.hip"

#include <algorithm>
#include <functional>
#include <string>

#define CK(x)                                                                     \
    do {                                                                          \
        hipError_t e = (x);                                                       \
        if (e != hipSuccess) {                                                    \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                \
            exit(1);                                                              \
        }                                                                         \
    } while (0)

struct Var {
    std::string name;
    std::function<void(hipStream_t)> run;
};

int main(int argc, char** argv) {
    const uint64_t n = argc > 1 ? strtoull(argv[1], 0, 10) : 1000000000ull;
    const int rounds = argc > 2 ? atoi(argv[2]) : 5;
    CK(hipSetDevice(0));
    DevState* s;
    if (ensure_ready(&s)) return 1;
    int* col;
    int* out;
    void* ws;
    unsigned long long* cnt;
    CK(hipMalloc(&col, n * 4));
    CK(hipMalloc(&out, n * 4));
    const size_t wsb = mq_scan_workspace_bytes(n);
    CK(hipMalloc(&ws, wsb));
    CK(hipMalloc(&cnt, 64));
    if (mq_gen_uniform(col, n, 42, n, nullptr)) return 1;
    CK(hipDeviceSynchronize());
    hipStream_t st = nullptr;
    std::vector<double> sels = {0.0, 0.001, 0.01, 0.1, 0.5, 1.0};
    for (double sel : sels) {
        const int32_t lo = sel == 0.0 ? (int32_t)n : (int32_t)(n / 4);
        const int32_t hi = lo + (int32_t)(sel * n) + (sel == 0.0 ? 1 : 0);
        Pred p;
        make_pred(1, lo, 1, hi, &p);
        std::vector<Var> vars;
        vars.push_back({"k_scan<kSum> (count+sum)", [&](hipStream_t q) {
                            Partial* part = (Partial*)ws;
                            uint32_t g;
                            launch_scan<kSum>(col, nullptr, n, p, part, nullptr, q, s, &g);
                        }});
        vars.push_back({"k_select_stage", [&](hipStream_t q) {
                            run_select_stage(col, nullptr, n, p, out, (uint64_t*)cnt, ws, q, s);
                        }});
        auto stv = [&](int buf) {
            return [&, buf](hipStream_t q) {
                const uint64_t gmax = 2048;
                const uint64_t granules = (n + kStGranule - 1) / kStGranule;
                const uint64_t units = gmax * kWaves;
                const uint64_t rw = ((granules + units - 1) / units) * kStGranule;
                const uint32_t g = (uint32_t)((n + rw * kWaves - 1) / (rw * kWaves));
                char* w = (char*)ws;
                (void)hipMemsetAsync(w, 0, stage_state_bytes(g), q);
                unsigned* err = (unsigned*)w;
                unsigned long long* status = (unsigned long long*)(w + 64);
                unsigned long long* bm = (unsigned long long*)(w + partial_bytes());
#define L_(B) hipLaunchKernelGGL((k_select_stage<false, true, B>), dim3(g), dim3(kTPB), 0, q, col, nullptr, n, rw, p, status, bm, out, cnt, err)
                if (buf == 256) L_(256);
                else if (buf == 512) L_(512);
                else L_(1024);
#undef L_
            };
        };
        vars.push_back({"stage buf 256", stv(256)});
        vars.push_back({"stage buf 512", stv(512)});
        vars.push_back({"k_mask + k_compact", [&](hipStream_t q) {
                            setenv("MQ_POSITIONS_IMPL", "mask", 1);
                            mq_select_positions(col, nullptr, n, 1, lo, 1, hi, out, (uint64_t*)cnt, ws, wsb, q);
                            unsetenv("MQ_POSITIONS_IMPL");
                        }});
        vars.push_back({"memset only", [&](hipStream_t q) { (void)hipMemsetAsync(ws, 0, 50000, q); }});
        hipEvent_t a, b;
        CK(hipEventCreate(&a));
        CK(hipEventCreate(&b));
        std::vector<std::vector<float>> ms(vars.size());
        const int reps = 10;
        for (int r = 0; r < rounds; r++) {
            for (size_t v = 0; v < vars.size(); v++) {
                vars[v].run(st);
                CK(hipEventRecord(a, st));
                for (int i = 0; i < reps; i++) vars[v].run(st);
                CK(hipEventRecord(b, st));
                CK(hipEventSynchronize(b));
                float t;
                CK(hipEventElapsedTime(&t, a, b));
                ms[v].push_back(t / reps);
                if (v == 1) {
                    unsigned long long k = 0;
                    unsigned errw = 0;
                    CK(hipMemcpy(&k, cnt, 8, hipMemcpyDeviceToHost));
                    CK(hipMemcpy(&errw, (char*)ws + 4, 4, hipMemcpyDeviceToHost));
                    Partial part0;
                    (void)part0;
                    if (r == 0) printf("  sel %.3f %-16s K=%llu err=%u\n", sel, vars[v].name.c_str(), k, errw);
                }
            }
        }
        CK(hipGetLastError());
        for (size_t v = 0; v < vars.size(); v++) {
            std::sort(ms[v].begin(), ms[v].end());
            printf("sel %.3f %-28s median %.4f ms best %.4f ms\n", sel, vars[v].name.c_str(),
                   ms[v][ms[v].size() / 2], ms[v][0]);
        }
    }
    return 0;
}
