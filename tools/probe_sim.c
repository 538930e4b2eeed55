/* probe_sim.c: CPU simulation of the join's unique table at load 1/2 (not product
 * code). Builds 2^lg config-5 build keys into 2*2^lg slots (4-slot buckets, linear
 * probing inside 8192-slot windows, as k_win_build) and probes 2^lg config-5 probe
 * keys, counting the probes that go past their home bucket and the 32-byte bucket
 * reads per probe, without and with the overflow marks of k_win_build.
 *   gcc -O2 -o /tmp/probe_sim tools/probe_sim.c && /tmp/probe_sim 24 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

static uint32_t hash32(uint32_t k) {
    k ^= k >> 16;
    k *= 0x85EBCA6Bu;
    k ^= k >> 13;
    k *= 0xC2B2AE35u;
    k ^= k >> 16;
    return k;
}
static uint64_t sm64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
static uint32_t mix31(uint32_t x) { /* the k_gen_join generator */
    const uint32_t M = 0x7FFFFFFFu;
    x &= M;
    x = (uint32_t)(((uint64_t)x * 0x2545F491u) & M);
    x ^= x >> 15;
    x = (uint32_t)(((uint64_t)x * 0x4F6CDD1Du) & M);
    x ^= x >> 13;
    x = (uint32_t)(((uint64_t)x * 0x6A09E667u) & M);
    x ^= x >> 16;
    return x;
}

int main(int argc, char** argv) {
    const int lg = argc > 1 ? atoi(argv[1]) : 24;
    const uint64_t n = 1ull << lg, slots = 2 * n, mask = slots - 1, wmask = (1 << 13) - 1;
    uint64_t* t = malloc(slots * 8);
    uint8_t* ovf = calloc(slots / 4, 1);
    for (uint64_t i = 0; i < slots; i++) t[i] = ~0ull;
    for (uint64_t i = 0; i < n; i++) {
        const uint32_t k = mix31((uint32_t)i);
        const uint64_t h0 = hash32(k) & mask & ~3ull;
        uint64_t h = h0;
        while (t[h] != ~0ull) h = (h & ~wmask) | ((h + 1) & wmask);
        t[h] = k;
        if ((h >> 2) != (h0 >> 2)) ovf[h0 >> 2] = 1;
    }
    for (int marks = 0; marks < 2; marks++) {
        uint64_t cont = 0, reads = 0;
        for (uint64_t i = 0; i < n; i++) {
            const uint32_t k = mix31((uint32_t)(sm64((7ull << 40) | i) & (2 * n - 1)));
            const uint64_t h0 = hash32(k) & mask & ~3ull;
            int done = 0;
            for (int q = 0; q < 4 && !done; q++)
                if (t[h0 + q] == ~0ull || (uint32_t)t[h0 + q] == k) done = 1;
            if (!done && marks && !ovf[h0 >> 2]) done = 1;
            reads++;
            if (done) continue;
            cont++;
            uint64_t h = (h0 & ~wmask) | ((h0 + 4) & wmask), last = h0 >> 2;
            for (;;) {
                if ((h >> 2) != last) reads++, last = h >> 2;
                if (t[h] == ~0ull || (uint32_t)t[h] == k) break;
                h = (h & ~wmask) | ((h + 1) & wmask);
            }
        }
        printf("marks=%d: probes past the bucket %.4f, bucket reads per probe %.4f\n", marks, (double)cont / n,
               (double)reads / n);
    }
    free(t);
    free(ovf);
    return 0;
}
