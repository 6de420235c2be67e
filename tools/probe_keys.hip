// A/B probe of the f4 key-tag kernels (48-byte keys, the keystore benchmark's shape,
// /root/reference/keystore/benchmark_test.go:27-32): lane kernel, per-wave double
// buffer (k_key_tags_lds) and the ring variants, interleaved over rounds, each checked
// bit-exact against a host XXH64 on the first keys.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/probe_keys tools/probe_keys.hip
//   tools/probe_keys [Mkeys=64] [reps=5] [rounds=3]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "../storm_amd/csrc/kernels.h"

using namespace stormck;

#define CK(x)                                                                     \
    do {                                                                          \
        hipError_t e = (x);                                                       \
        if (e != hipSuccess) {                                                    \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
            exit(1);                                                              \
        }                                                                         \
    } while (0)

static uint64_t rl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
static uint64_t hround(uint64_t a, uint64_t w) { return rl(a + w * kP2, 31) * kP1; }
static uint64_t hmerge(uint64_t h, uint64_t v) { return (h ^ hround(0, v)) * kP1 + kP4; }
static uint64_t rd64(const uint8_t* p) { uint64_t v; memcpy(&v, p, 8); return v; }
static uint64_t host_xxh64(const uint8_t* p, uint64_t n) {
    uint64_t h; const uint8_t* e = p + n;
    if (n >= 32) {
        uint64_t v1 = kV1, v2 = kV2, v3 = kV3, v4 = kV4;
        for (; p + 32 <= e; p += 32) { v1 = hround(v1, rd64(p)); v2 = hround(v2, rd64(p + 8)); v3 = hround(v3, rd64(p + 16)); v4 = hround(v4, rd64(p + 24)); }
        h = rl(v1, 1) + rl(v2, 7) + rl(v3, 12) + rl(v4, 18);
        h = hmerge(h, v1); h = hmerge(h, v2); h = hmerge(h, v3); h = hmerge(h, v4);
    } else h = kP5;
    h += n;
    for (; p + 8 <= e; p += 8) h = rl(h ^ hround(0, rd64(p)), 27) * kP1 + kP4;
    if (p + 4 <= e) { uint32_t w; memcpy(&w, p, 4); h = rl(h ^ (uint64_t)w * kP1, 23) * kP2 + kP3; p += 4; }
    for (; p < e; ++p) h = rl(h ^ (uint64_t)(*p) * kP5, 11) * kP1;
    h ^= h >> 33; h *= kP2; h ^= h >> 29; h *= kP3; h ^= h >> 32;
    return h;
}

struct Timer {
    hipEvent_t a, b;
    Timer() { CK(hipEventCreate(&a)); CK(hipEventCreate(&b)); }
    void start() { CK(hipEventRecord(a, 0)); }
    float stop() { CK(hipEventRecord(b, 0)); CK(hipEventSynchronize(b)); float ms; CK(hipEventElapsedTime(&ms, a, b)); return ms; }
};

int main(int argc, char** argv) {
    const uint64_t n = (uint64_t)((argc > 1 ? atof(argv[1]) : 64.0) * (1 << 20)) / 64 * 64;
    const int reps = argc > 2 ? atoi(argv[2]) : 5, rounds = argc > 3 ? atoi(argv[3]) : 3;
    constexpr uint32_t klen = 48;
    uint8_t* keys; CK(hipMalloc(&keys, n * klen));
    uint64_t* out; CK(hipMalloc(&out, n * 8));
    hipLaunchKernelGGL(k_fill_synthetic, dim3(8192), dim3(256), 0, 0, keys, 48ULL * 1024, n * klen / (48 * 1024), 0ULL, 0x53544f524dULL);
    CK(hipDeviceSynchronize());
    const uint64_t K = std::min<uint64_t>(n, 1 << 16);
    std::vector<uint8_t> hk(K * klen);
    CK(hipMemcpy(hk.data(), keys, K * klen, hipMemcpyDeviceToHost));
    std::vector<uint64_t> ref(K), got(K);
    for (uint64_t i = 0; i < K; ++i) ref[i] = host_xxh64(hk.data() + i * klen, klen);
    // also check the LAST keys (grid tail)
    std::vector<uint8_t> hk2(K * klen);
    CK(hipMemcpy(hk2.data(), keys + (n - K) * klen, K * klen, hipMemcpyDeviceToHost));
    std::vector<uint64_t> ref2(K), got2(K);
    for (uint64_t i = 0; i < K; ++i) ref2[i] = host_xxh64(hk2.data() + i * klen, klen);

    const uint64_t batches = n / 64;
    struct V { std::string name; std::function<void()> f; };
    std::vector<V> vs;
    vs.push_back({"lane k_key_tags", [&] {
        hipLaunchKernelGGL((k_key_tags<false, false>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, keys, (uint64_t)klen,
                           nullptr, nullptr, klen, n, out); }});
    vs.push_back({"lds double buffer pw8", [&] {
        const uint64_t waves = (batches + 7) / 8;
        hipLaunchKernelGGL(k_key_tags_lds<2>, dim3((unsigned)((waves + 3) / 4)), dim3(256), 4 * 2 * 64 * klen, 0, keys, klen, klen,
                           batches, 8u, out); }});
#define RV(RING, PW)                                                                                       \
    vs.push_back({"ring R=" #RING " PW=" #PW, [&] {                                                        \
        const uint64_t waves = (batches + PW - 1) / PW;                                                    \
        hipLaunchKernelGGL((k_key_tags_ring<2, 3, RING, PW>), dim3((unsigned)((waves + 3) / 4)), dim3(256), \
                           4 * RING * 64 * klen, 0, keys, klen, batches, out); }})
    RV(2, 8); RV(3, 8); RV(3, 16); RV(4, 8); RV(4, 16); RV(5, 16); RV(6, 16);
    std::vector<std::vector<double>> gks(vs.size());
    for (int r = 0; r < rounds; ++r)
        for (size_t v = 0; v < vs.size(); ++v) {
            CK(hipMemset(out, 0, n * 8));
            vs[v].f();
            CK(hipDeviceSynchronize());
            if (r == 0) {
                CK(hipMemcpy(got.data(), out, K * 8, hipMemcpyDeviceToHost));
                CK(hipMemcpy(got2.data(), out + (n - K), K * 8, hipMemcpyDeviceToHost));
                uint64_t bad = 0;
                for (uint64_t i = 0; i < K; ++i) bad += (got[i] != ref[i]) + (got2[i] != ref2[i]);
                if (bad) printf("  !! %s: %llu mismatches\n", vs[v].name.c_str(), (unsigned long long)bad);
            }
            Timer t;
            for (int k = 0; k < reps; ++k) { t.start(); vs[v].f(); gks[v].push_back(n / (t.stop() * 1e-3) / 1e9); }
        }
    printf("keys %llu x %u B (%.2f GB + %.2f GB out)\n", (unsigned long long)n, klen, n * klen / 1e9, n * 8 / 1e9);
    for (size_t v = 0; v < vs.size(); ++v) {
        auto g = gks[v]; std::sort(g.begin(), g.end());
        const double med = g[g.size() / 2];
        printf("%-26s max %7.2f  median %7.2f Gkeys/s  = %7.1f GB/s (%.3f of 8 TB/s)\n", vs[v].name.c_str(), g.back(), med,
               med * (klen + 8), med * (klen + 8) / 8000.0);
    }
    printf("done\n");
    return 0;
}
