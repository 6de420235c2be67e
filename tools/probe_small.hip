// Small-batch latency probe: time per launch of the streaming kernels (glds 8-wave,
// register quad) and the one-workgroup-per-block "wide" kernel on batches of
// n = 1 .. 32K device-resident blocks (32 KiB uniform, and storm's commit mix of
// 31808-byte objectlist blocks with per-block lengths), each checked bit-exact
// against a host XXH64. Picks the launch_checksum crossover.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/probe_small tools/probe_small.hip
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

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e = (x);                                                                     \
        if (e != hipSuccess) {                                                                  \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e));    \
            exit(1);                                                                            \
        }                                                                                       \
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

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 20;
    const uint64_t L = 32768, NMAX = 32768;
    uint8_t* d; CK(hipMalloc(&d, NMAX * L + 4096));
    uint64_t* out; CK(hipMalloc(&out, NMAX * 8));
    uint32_t* dl; CK(hipMalloc(&dl, NMAX * 4));
    uint64_t* doff; CK(hipMalloc(&doff, NMAX * 8));
    hipLaunchKernelGGL(k_fill_synthetic, dim3(8192), dim3(256), 0, 0, d, L, NMAX, 0ULL, 0x53544f524dULL);
    std::vector<uint32_t> hl(NMAX);
    std::vector<uint64_t> ho(NMAX);
    for (uint64_t i = 0; i < NMAX; ++i) { hl[i] = (i % 97 == 0) ? 30000 : ((i % 89 == 0) ? 72 : 31808); ho[i] = i * L + (i % 7 == 3 ? 5 : 0); }
    CK(hipMemcpy(dl, hl.data(), NMAX * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(doff, ho.data(), NMAX * 8, hipMemcpyHostToDevice));
    CK(hipDeviceSynchronize());
    const uint64_t K = 512;
    std::vector<uint8_t> hb(K * L + 64);
    CK(hipMemcpy(hb.data(), d, K * L + 64, hipMemcpyDeviceToHost));
    std::vector<uint64_t> ref_u(K), ref_m(K), got(K);
    for (uint64_t i = 0; i < K; ++i) { ref_u[i] = host_xxh64(hb.data() + i * L, L); ref_m[i] = host_xxh64(hb.data() + ho[i], hl[i]); }
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    auto timeit = [&](const std::function<void()>& f) {
        f(); CK(hipDeviceSynchronize());
        CK(hipEventRecord(a, 0));
        for (int r = 0; r < reps; ++r) f();
        CK(hipEventRecord(b, 0)); CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b));
        return ms * 1e3 / reps;  // us per launch
    };
    auto check = [&](const char* name, uint64_t n, const std::vector<uint64_t>& ref) {
        const uint64_t m = std::min(n, K);
        CK(hipMemcpy(got.data(), out, m * 8, hipMemcpyDeviceToHost));
        uint64_t bad = 0; for (uint64_t i = 0; i < m; ++i) bad += got[i] != ref[i];
        if (bad) printf("  !! %s n=%llu: %llu mismatches\n", name, (unsigned long long)n, (unsigned long long)bad);
        CK(hipMemset(out, 0, NMAX * 8));
    };
    printf("%8s %10s %10s %10s | %10s %10s   (us per launch; uniform 32 KiB | mixed lens+offsets)\n", "n", "glds8w", "quad", "wide", "quad", "wide");
    for (uint64_t n : {1ULL, 16ULL, 128ULL, 512ULL, 1024ULL, 1280ULL, 2048ULL, 3072ULL, 4096ULL, 6144ULL, 8192ULL, 16384ULL, 32768ULL}) {
        const dim3 g8((unsigned)((n + 127) / 128)), gq((unsigned)((n * 4 + 255) / 256)), gw((unsigned)n);
        auto f_glds = [&] { hipLaunchKernelGGL((k_xxh64_glds<16, 2, 2, true, false, 8>), g8, dim3(512), 0, 0, d, L, (uint32_t)L, n, out, nullptr, nullptr, nullptr); };
        auto f_quad = [&] { hipLaunchKernelGGL((k_xxh64_quad<16, false, false, false>), gq, dim3(256), 0, 0, d, L, nullptr, (uint32_t)L, nullptr, n, out, nullptr, nullptr, nullptr); };
        auto f_wide = [&] { hipLaunchKernelGGL((k_xxh64_wide<false, false, false>), gw, dim3(256), 0, 0, d, L, nullptr, (uint32_t)L, nullptr, n, out, nullptr, nullptr, nullptr); };
        auto m_quad = [&] { hipLaunchKernelGGL((k_xxh64_quad<16, true, true, false>), gq, dim3(256), 0, 0, d, 0, dl, 0u, doff, n, out, nullptr, nullptr, nullptr); };
        auto m_wide = [&] { hipLaunchKernelGGL((k_xxh64_wide<true, true, false>), gw, dim3(256), 0, 0, d, 0, dl, 0u, doff, n, out, nullptr, nullptr, nullptr); };
        const double t1 = timeit(f_glds); check("glds", n, ref_u);
        const double t2 = timeit(f_quad); check("quad", n, ref_u);
        const double t3 = timeit(f_wide); check("wide", n, ref_u);
        const double t4 = timeit(m_quad); check("quad mixed", n, ref_m);
        const double t5 = timeit(m_wide); check("wide mixed", n, ref_m);
        printf("%8llu %10.1f %10.1f %10.1f | %10.1f %10.1f\n", (unsigned long long)n, t1, t2, t3, t4, t5);
        fflush(stdout);
    }
    printf("done\n");
    return 0;
}
