// Probe (GPU box): cost of ONE blocks.Checksum call per leg, in C, without Python.
//   host leg   : stormck_checksum (= stormck_xxh64 on the calling thread)
//   device leg : stormck_checksum_gpu (k_xxh64_single up to 64 KiB, pipeline beyond)
// Lengths from storm's blocks (72 B singularity .. 32 KiB) up to 256 MiB. Prints one
// line per length with the median of 7 rounds and the crossover verdict.
//   g++ -O2 -std=c++17 -Iinclude tools/single_call_probe.cpp -Lstorm_amd/lib -lstormck \
//       -Wl,-rpath,$PWD/storm_amd/lib -o tools/single_call_probe
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "stormck.h"

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
    if (stormck_init(0) != STORMCK_OK) {
        std::fprintf(stderr, "init: %s\n", stormck_last_error());
        return 1;
    }
    const size_t lens[] = {72, 256, 4096, 28808, 30000, 32768, 65536, 1u << 20, 16u << 20, 256u << 20};
    std::vector<unsigned char> buf((256u << 20) + 64);
    uint64_t x = 0x9E3779B97F4A7C15ULL;
    for (auto& c : buf) {
        x ^= x << 13, x ^= x >> 7, x ^= x << 17;
        c = static_cast<unsigned char>(x);
    }
    uint64_t out = 0, sink = 0;
    // warm both legs (pinned staging, clocks)
    for (int i = 0; i < 2000; ++i) stormck_checksum_gpu(buf.data(), 32768, &out);
    std::printf("%10s %14s %14s %10s\n", "bytes", "host_us", "gpu_us", "gpu/host");
    for (size_t L : lens) {
        const int reps = L <= 65536 ? 2000 : (L <= (1u << 20) ? 200 : (L <= (16u << 20) ? 20 : 3));
        std::vector<double> h, g;
        for (int round = 0; round < 7; ++round) {
            double t0 = now_us();
            for (int i = 0; i < reps; ++i) {
                stormck_checksum(buf.data(), L, &out);
                sink += out;
            }
            h.push_back((now_us() - t0) / reps);
            const int greps = std::max(1, reps / 10);
            t0 = now_us();
            for (int i = 0; i < greps; ++i) {
                if (stormck_checksum_gpu(buf.data(), L, &out) != STORMCK_OK) {
                    std::fprintf(stderr, "gpu %zu: %s\n", L, stormck_last_error());
                    return 1;
                }
                sink += out;
            }
            g.push_back((now_us() - t0) / greps);
        }
        std::sort(h.begin(), h.end());
        std::sort(g.begin(), g.end());
        uint64_t a = 0, b = 0;
        stormck_checksum(buf.data(), L, &a);
        stormck_checksum_gpu(buf.data(), L, &b);
        std::printf("%10zu %14.3f %14.3f %10.1f %s\n", L, h[3], g[3], g[3] / h[3], a == b ? "" : "MISMATCH");
        std::fflush(stdout);
    }
    std::printf("sink %llu\n", static_cast<unsigned long long>(sink & 1));
    return 0;
}
