// XXH64 stripe chain at small batch sizes (latency-bound: one block per quad), A/B in
// one process after a clock-settling warm-up, on n device-resident blocks of storm's
// commit mix (31808 B objectlist leaves, per-block lengths) and uniform 32 KiB blocks.
// Variants of k_xxh64_quad's register-quad mapping: the shipped 2-group pipeline
// ("classic"), D register groups in flight (k_deep), and two bound finders: synthetic
// words with no loads (VALU floor) and loads with no hash (load floor). All checked
// bit-exact against a host XXH64 (bound finders excepted). DESIGN_LOG.md §5 has results.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/chain_probe tools/chain_probe.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <utility>
#include <vector>

#include "../storm_amd/csrc/kernels.h"

using namespace stormck;

#define CK(x)                                                                                \
    do {                                                                                     \
        hipError_t e = (x);                                                                  \
        if (e != hipSuccess) {                                                               \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
            exit(1);                                                                         \
        }                                                                                    \
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

// ---- the stripe chain in folded form (measured, not adopted: DESIGN_LOG.md §4) -------
// round(acc, w) = rotl31(acc + w*P2) * P1 puts acc through both multiplies: the
// compiler folds acc into the w*P2 v_mad_u64_u32, so each round's dependent path is
// mad -> add3 -> alignbit -> mad -> add3. Carrying x = acc + w*P2 instead (the value
// before the rotate) gives x' = rotl31(x)*P1 + w'*P2, where w'*P2 depends on the data
// only and folds into the P1 multiply's v_mad_u64_u32 addend: alignbit -> mad -> add3
// per round. Latency-bound chains (one block per quad, small batches) run faster;
// the instruction count is unchanged. P1 is odd, hence invertible mod 2^64, so any
// acc enters the chain as x = rotr31(acc * P1^-1) and every stripe is the same step.
constexpr uint64_t inv_odd(uint64_t a) {
    uint64_t x = a;  // correct to 3 bits for odd a; each Newton step doubles that
    for (int i = 0; i < 5; ++i) x *= 2 - a * x;
    return x;
}
constexpr uint64_t kP1inv = inv_odd(kP1);
static_assert(kP1 * kP1inv == 1, "P1 inverse");

__device__ __forceinline__ uint64_t chain_in(uint64_t acc) {
    const uint64_t a = acc * kP1inv;
    return rotl<1>((a << 32) | (a >> 32));  // rotr31 = rotl33
}

// One round given t = w*P2 (computed elsewhere, e.g. by another wave).
__device__ __forceinline__ uint64_t chain_step_t(uint64_t x, uint64_t t) {
    const uint32_t xl = static_cast<uint32_t>(x), xh = static_cast<uint32_t>(x >> 32);
    const uint32_t rh = __builtin_amdgcn_alignbit(xh, xl, 1);  // rotl31
    const uint32_t rl = __builtin_amdgcn_alignbit(xl, xh, 1);
    // prod = rl * P1lo + t in one v_mad_u64_u32. Written as asm: in plain C the compiler
    // re-associates the two 64-bit products and rebuilds the long chain.
    uint64_t prod, carry;
    asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(prod), "=s"(carry) : "v"(rl), "s"(static_cast<uint32_t>(kP1)), "v"(t));
    (void)carry;
    const uint32_t hi = static_cast<uint32_t>(prod >> 32) + rl * static_cast<uint32_t>(kP1 >> 32) +
                        rh * static_cast<uint32_t>(kP1);
    return (static_cast<uint64_t>(hi) << 32) | static_cast<uint32_t>(prod);
}

__device__ __forceinline__ uint64_t chain_step(uint64_t x, uint64_t w) { return chain_step_t(x, w * kP2); }

__device__ __forceinline__ uint64_t chain_out(uint64_t x) { return rotl<31>(x) * kP1; }

// the classic form: acc = round(acc, w), same software pipeline as quad_stripes_aligned
template <int U>
__device__ __forceinline__ uint64_t stripes_classic(const uint64_t* __restrict__ p, uint32_t nst, uint64_t acc) {
    const uint32_t ngroups = nst / U;
    uint32_t s = 0;
    if (ngroups > 0) {
        uint64_t wa[U], wb[U];
#pragma unroll
        for (int u = 0; u < U; ++u) wa[u] = p[4 * u];
        for (uint32_t g = 1; g < ngroups; ++g) {
#pragma unroll
            for (int u = 0; u < U; ++u) wb[u] = p[4 * (g * U + u)];
#pragma unroll
            for (int u = 0; u < U; ++u) acc = round(acc, wa[u]);
#pragma unroll
            for (int u = 0; u < U; ++u) wa[u] = wb[u];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc = round(acc, wa[u]);
        s = ngroups * U;
    }
    for (; s < nst; ++s) acc = round(acc, p[4 * s]);
    return acc;
}

template <int U>
__device__ __forceinline__ uint64_t stripes_folded(const uint64_t* __restrict__ p, uint32_t nst, uint64_t acc) {
    uint64_t x = chain_in(acc);
    const uint32_t ngroups = nst / U;
    uint32_t s = 0;
    if (ngroups > 0) {
        uint64_t wa[U], wb[U];
#pragma unroll
        for (int u = 0; u < U; ++u) wa[u] = p[4 * u];
        for (uint32_t g = 1; g < ngroups; ++g) {
#pragma unroll
            for (int u = 0; u < U; ++u) wb[u] = p[4 * (g * U + u)];
#pragma unroll
            for (int u = 0; u < U; ++u) x = chain_step(x, wa[u]);
#pragma unroll
            for (int u = 0; u < U; ++u) wa[u] = wb[u];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) x = chain_step(x, wa[u]);
        s = ngroups * U;
    }
    for (; s < nst; ++s) x = chain_step(x, p[4 * s]);
    return chain_out(x);
}

template <bool FOLD, bool LENS>
__global__ __launch_bounds__(256) void k_quad(const uint8_t* __restrict__ base, uint64_t stride,
                                              const uint32_t* __restrict__ lens, uint32_t len, uint64_t n,
                                              uint64_t* __restrict__ out) {
    const uint64_t gtid = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x;
    const uint64_t blk_raw = gtid >> 2;
    const uint32_t j = threadIdx.x & 3;
    const bool live = blk_raw < n;
    const uint64_t blk = live ? blk_raw : n - 1;
    const uint8_t* src = base + blk * stride;
    const uint32_t L = LENS ? lens[blk] : len;
    const uint32_t nst = L >> 5;
    const uint64_t* p = reinterpret_cast<const uint64_t*>(src) + j;
    const uint64_t acc = FOLD ? stripes_folded<16>(p, nst, acc_seed(j)) : stripes_classic<16>(p, nst, acc_seed(j));
    const uint64_t v1 = quad_bcast<0>(acc), v2 = quad_bcast<1>(acc), v3 = quad_bcast<2>(acc), v4 = quad_bcast<3>(acc);
    if (j == 0 && live) {
        const uint64_t h0 = (L >= 32) ? converge(v1, v2, v3, v4) : kP5;
        out[blk] = finish_fast(h0, L, src + 32 * static_cast<uint64_t>(nst), L & 31);
    }
}

// Deep software pipeline: D register groups of U stripes in flight. A group's words
// are loaded D-1 groups of hashing before they are used, which must cover the load
// latency: one round costs ~27 cycles from registers (tools/round_probe.hip), so the
// U=16, 2-group pipeline leaves ~450 ns loads exposed every group.
template <int U, int D>
__device__ __forceinline__ uint64_t stripes_deep(const uint64_t* __restrict__ p, uint32_t nst, uint64_t acc) {
    const uint32_t ng = nst / U;
    if (ng >= D) {
        // straight-line loop body (unconditional refills from a per-group clamped pointer,
        // immediate offsets per load) so the waitcnt pass keeps D-1 groups outstanding
        uint64_t w[D][U];
#pragma unroll
        for (int d = 0; d < D; ++d) {
#pragma unroll
            for (int u = 0; u < U; ++u) w[d][u] = p[4 * (d * U + u)];
        }
        uint32_t g = 0;
        for (; g + D <= ng; g += D) {
#pragma unroll
            for (int d = 0; d < D; ++d) {
#pragma unroll
                for (int u = 0; u < U; ++u) acc = round(acc, w[d][u]);
                const uint64_t* q = p + 4 * U * min(g + d + D, ng - 1);
#pragma unroll
                for (int u = 0; u < U; ++u) w[d][u] = q[4 * u];
            }
        }
#pragma unroll
        for (int d = 0; d < D - 1; ++d) {
            if (g + d < ng) {
#pragma unroll
                for (int u = 0; u < U; ++u) acc = round(acc, w[d][u]);
            }
        }
        for (uint32_t s = ng * U; s < nst; ++s) acc = round(acc, p[4 * s]);
        return acc;
    }
    for (uint32_t s = 0; s < nst; ++s) acc = round(acc, p[4 * s]);
    return acc;
}

template <int U, int D, bool LENS>
__global__ __launch_bounds__(256) void k_deep(const uint8_t* __restrict__ base, uint64_t stride,
                                              const uint32_t* __restrict__ lens, uint32_t len, uint64_t n,
                                              uint64_t* __restrict__ out) {
    const uint64_t gtid = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x;
    const uint64_t blk_raw = gtid >> 2;
    const uint32_t j = threadIdx.x & 3;
    const bool live = blk_raw < n;
    const uint64_t blk = live ? blk_raw : n - 1;
    const uint8_t* src = base + blk * stride;
    const uint32_t L = LENS ? lens[blk] : len;
    const uint32_t nst = L >> 5;
    const uint64_t* p = reinterpret_cast<const uint64_t*>(src) + j;
    const uint64_t acc = stripes_deep<U, D>(p, nst, acc_seed(j));
    const uint64_t v1 = quad_bcast<0>(acc), v2 = quad_bcast<1>(acc), v3 = quad_bcast<2>(acc), v4 = quad_bcast<3>(acc);
    if (j == 0 && live) {
        const uint64_t h0 = (L >= 32) ? converge(v1, v2, v3, v4) : kP5;
        out[blk] = finish_fast(h0, L, src + 32 * static_cast<uint64_t>(nst), L & 31);
    }
}

// Bound finders for the register quad at small n: MODE 1 hashes synthetic words (no
// loads: the VALU floor of a full round), MODE 2 loads and XORs (no hash: load floor).
template <int MODE>
__global__ __launch_bounds__(256) void k_bound(const uint8_t* __restrict__ base, uint64_t stride, uint32_t len,
                                               uint64_t n, uint64_t* __restrict__ out) {
    const uint64_t gtid = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x;
    const uint64_t blk_raw = gtid >> 2;
    const uint32_t j = threadIdx.x & 3;
    const uint64_t blk = blk_raw < n ? blk_raw : n - 1;
    const uint64_t* p = reinterpret_cast<const uint64_t*>(base + blk * stride) + j;
    const uint32_t nst = len >> 5;
    uint64_t acc = acc_seed(j);
    if constexpr (MODE == 1) {
        uint64_t w = blk * 0x9E3779B97F4A7C15ULL + j;
        for (uint32_t s = 0; s < nst; s += 16) {
#pragma unroll
            for (int u = 0; u < 16; ++u) { acc = round(acc, w); w += 0x632BE59BD9B4E019ULL; }
        }
    } else {
        const uint32_t ngroups = nst / 16;
        uint64_t wa[16], wb[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) wa[u] = p[4 * u];
        for (uint32_t g = 1; g < ngroups; ++g) {
#pragma unroll
            for (int u = 0; u < 16; ++u) wb[u] = p[4 * (g * 16 + u)];
#pragma unroll
            for (int u = 0; u < 16; ++u) acc = rotl<1>(acc) ^ wa[u];
#pragma unroll
            for (int u = 0; u < 16; ++u) wa[u] = wb[u];
        }
#pragma unroll
        for (int u = 0; u < 16; ++u) acc ^= wa[u];
    }
    if (blk_raw < n && j == 0) out[blk] = acc;
}

// Mid-size batches (8K..128K blocks of 32 KiB): workgroup size of the LDS-DMA streaming
// kernel. 8 waves x 16 blocks put 128 blocks and 128 KiB of LDS ring on one CU, so a
// 16K-block batch occupies only 128 of 256 CUs.
static int mid_sweep(int reps) {
    const uint64_t L = 32768, NMAX = 131072;
    uint8_t* d; CK(hipMalloc(&d, NMAX * L));
    uint64_t* out; CK(hipMalloc(&out, NMAX * 8));
    hipLaunchKernelGGL(k_fill_synthetic, dim3(8192), dim3(256), 0, 0, d, L, NMAX, 0ULL, 0x53544f524dULL);
    CK(hipDeviceSynchronize());
    const uint64_t K = 256;
    std::vector<uint8_t> hb(L);
    std::vector<uint64_t> ref(K), got(K);
    std::vector<uint64_t> idx(K);
    for (uint64_t i = 0; i < K; ++i) idx[i] = (i * 2654435761ULL) % 8192;
    for (uint64_t i = 0; i < K; ++i) { CK(hipMemcpy(hb.data(), d + idx[i] * L, L, hipMemcpyDeviceToHost)); ref[i] = host_xxh64(hb.data(), L); }
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    auto timeit = [&](const std::function<void()>& f) {
        CK(hipEventRecord(a, 0));
        for (int r = 0; r < reps; ++r) f();
        CK(hipEventRecord(b, 0)); CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b));
        return ms * 1e3 / reps;
    };
    int bad_total = 0;
    printf("%7s %9s %9s %9s %9s %9s %9s   (us per launch; GB/s of the best in the last column)\n", "n", "quad", "glds8w",
           "glds4w", "glds2w", "glds1w", "glds1w-R4");
    for (uint64_t n : {8192ULL, 12288ULL, 16384ULL, 24576ULL, 32768ULL, 49152ULL, 65536ULL, 131072ULL}) {
        const unsigned gq = (unsigned)((n * 4 + 255) / 256);
        auto G = [&](unsigned bpw) { return dim3((unsigned)((n + bpw - 1) / bpw)); };
        std::vector<std::pair<const char*, std::function<void()>>> fs = {
            {"quad", [&] { hipLaunchKernelGGL((k_xxh64_quad<16, false, false, false>), dim3(gq), dim3(256), 0, 0, d, L, nullptr, (uint32_t)L, nullptr, n, out, nullptr, nullptr, nullptr); }},
            {"glds8w", [&] { hipLaunchKernelGGL((k_xxh64_glds<16, 2, 2, true, false, 8>), G(128), dim3(512), 0, 0, d, L, (uint32_t)L, n, out, nullptr, nullptr, nullptr); }},
            {"glds4w", [&] { hipLaunchKernelGGL((k_xxh64_glds<16, 2, 2, true, false, 4, false>), G(64), dim3(256), 0, 0, d, L, (uint32_t)L, n, out, nullptr, nullptr, nullptr); }},
            {"glds2w", [&] { hipLaunchKernelGGL((k_xxh64_glds<16, 2, 2, true, false, 2, false>), G(32), dim3(128), 0, 0, d, L, (uint32_t)L, n, out, nullptr, nullptr, nullptr); }},
            {"glds1w", [&] { hipLaunchKernelGGL((k_xxh64_glds<16, 2, 2, true, false, 1, false>), G(16), dim3(64), 0, 0, d, L, (uint32_t)L, n, out, nullptr, nullptr, nullptr); }},
            {"glds1w-R4", [&] { hipLaunchKernelGGL((k_xxh64_glds<16, 4, 2, true, false, 1, false>), G(16), dim3(64), 0, 0, d, L, (uint32_t)L, n, out, nullptr, nullptr, nullptr); }},
        };
        for (auto& f : fs) f.second();
        CK(hipDeviceSynchronize());
        std::vector<double> t(fs.size(), 1e30);
        for (int round = 0; round < 5; ++round)
            for (size_t i = 0; i < fs.size(); ++i) t[i] = std::min(t[i], timeit(fs[i].second));
        for (auto& f : fs) {
            CK(hipMemset(out, 0, NMAX * 8));
            f.second();
            CK(hipDeviceSynchronize());
            uint64_t bad = 0;
            for (uint64_t i = 0; i < K; ++i) {
                if (idx[i] >= n) continue;
                uint64_t g; CK(hipMemcpy(&g, out + idx[i], 8, hipMemcpyDeviceToHost));
                bad += g != ref[i];
            }
            if (bad) { printf("  !! %s n=%llu: %llu mismatches\n", f.first, (unsigned long long)n, (unsigned long long)bad); ++bad_total; }
        }
        double best = 1e30;
        printf("%7llu", (unsigned long long)n);
        for (size_t i = 0; i < fs.size(); ++i) { printf(" %9.2f", t[i]); best = std::min(best, t[i]); }
        printf("   %7.0f GB/s\n", n * (L + 8) / (best * 1e-6) / 1e9);
        fflush(stdout);
    }
    printf(bad_total ? "MISMATCH\n" : "all bit-exact\n");
    return bad_total ? 1 : 0;
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 50;
    if (argc > 2 && std::string(argv[2]) == "mid") return mid_sweep(reps);
    const uint64_t L = 32768, NMAX = 16384;
    uint8_t* d; CK(hipMalloc(&d, NMAX * L));
    uint64_t* out; CK(hipMalloc(&out, NMAX * 8));
    uint32_t* dl; CK(hipMalloc(&dl, NMAX * 4));
    hipLaunchKernelGGL(k_fill_synthetic, dim3(8192), dim3(256), 0, 0, d, L, NMAX, 0ULL, 0x53544f524dULL);
    std::vector<uint32_t> hl(NMAX);
    for (uint64_t i = 0; i < NMAX; ++i) hl[i] = (i % 1202 == 1200) ? 30000 : ((i % 1202 == 1201) ? 72 : 31808);
    CK(hipMemcpy(dl, hl.data(), NMAX * 4, hipMemcpyHostToDevice));
    CK(hipDeviceSynchronize());
    const uint64_t K = 2048;
    std::vector<uint8_t> hb(K * L);
    CK(hipMemcpy(hb.data(), d, K * L, hipMemcpyDeviceToHost));
    std::vector<uint64_t> ref_u(K), ref_m(K), got(K);
    for (uint64_t i = 0; i < K; ++i) { ref_u[i] = host_xxh64(hb.data() + i * L, L); ref_m[i] = host_xxh64(hb.data() + i * L, hl[i]); }
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    auto timeit = [&](const std::function<void()>& f) {
        CK(hipEventRecord(a, 0));
        for (int r = 0; r < reps; ++r) f();
        CK(hipEventRecord(b, 0)); CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b));
        return ms * 1e3 / reps;
    };
    int bad_total = 0;
    auto check = [&](const char* name, uint64_t n, const std::vector<uint64_t>& ref) {
        const uint64_t m = std::min(n, K);
        CK(hipMemcpy(got.data(), out, m * 8, hipMemcpyDeviceToHost));
        uint64_t bad = 0; for (uint64_t i = 0; i < m; ++i) bad += got[i] != ref[i];
        if (bad) { printf("  !! %s n=%llu: %llu mismatches\n", name, (unsigned long long)n, (unsigned long long)bad); ++bad_total; }
        CK(hipMemset(out, 0, NMAX * 8));
    };
    // settle the clocks: 2 s of back-to-back launches
    {
        auto t0 = std::chrono::steady_clock::now();
        while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < 2.0) {
            for (int r = 0; r < 20; ++r)
                hipLaunchKernelGGL((k_quad<false, false>), dim3(64), dim3(256), 0, 0, d, L, nullptr, (uint32_t)L, 4096ULL, out);
            CK(hipDeviceSynchronize());
        }
    }
    printf("%6s %9s %9s %9s %9s %9s %9s %9s %9s | %9s %9s %9s %9s   (us per launch, best of 5 alternating rounds of %d launches)\n",
           "n", "classic", "d16x4", "d16x3", "g1w16x2", "g1w16x4", "g1w8x6", "valu", "loads", "mix-cls", "mix16x4", "mix16x3", "mix8x6", reps);
    for (uint64_t n : {1ULL, 16ULL, 64ULL, 256ULL, 1202ULL, 2048ULL, 4096ULL, 8192ULL, 16384ULL}) {
        const dim3 g((unsigned)((n * 4 + 255) / 256));
#define KU(NAME, KERN) {NAME, [&] { hipLaunchKernelGGL(KERN, g, dim3(256), 0, 0, d, L, nullptr, (uint32_t)L, n, out); }}
#define KM(NAME, KERN) {NAME, [&] { hipLaunchKernelGGL(KERN, g, dim3(256), 0, 0, d, L, dl, 0u, n, out); }}
        std::vector<std::pair<const char*, std::function<void()>>> fs = {
            KU("classic", (k_quad<false, false>)), KU("d16x4", (k_deep<16, 4, false>)), KU("d16x3", (k_deep<16, 3, false>)),
            {"g1w16x2", [&] { hipLaunchKernelGGL((k_xxh64_glds<16, 2, 2, true, false, 1, false>), dim3((unsigned)((n + 15) / 16)), dim3(64), 0, 0, d, L, (uint32_t)L, n, out, nullptr, nullptr, nullptr); }},
            {"g1w16x4", [&] { hipLaunchKernelGGL((k_xxh64_glds<16, 4, 2, true, false, 1, false>), dim3((unsigned)((n + 15) / 16)), dim3(64), 0, 0, d, L, (uint32_t)L, n, out, nullptr, nullptr, nullptr); }},
            {"g1w8x6", [&] { hipLaunchKernelGGL((k_xxh64_glds<8, 6, 2, true, false, 1, false>), dim3((unsigned)((n + 15) / 16)), dim3(64), 0, 0, d, L, (uint32_t)L, n, out, nullptr, nullptr, nullptr); }},
            {"valu-only", [&] { hipLaunchKernelGGL(k_bound<1>, g, dim3(256), 0, 0, d, L, (uint32_t)L, n, out); }},
            {"loads-only", [&] { hipLaunchKernelGGL(k_bound<2>, g, dim3(256), 0, 0, d, L, (uint32_t)L, n, out); }},
            KM("mix classic", (k_quad<false, true>)), KM("mix d16x4", (k_deep<16, 4, true>)),
            KM("mix d16x3", (k_deep<16, 3, true>)), KM("mix d8x6", (k_deep<8, 6, true>)),
        };
#undef KU
#undef KM
        std::vector<double> t(fs.size(), 1e30);
        for (int round = 0; round < 5; ++round)
            for (size_t i = 0; i < fs.size(); ++i) t[i] = std::min(t[i], timeit(fs[i].second));
        for (size_t i = 0; i < fs.size(); ++i) { fs[i].second(); if (i == 6 || i == 7) continue; check(fs[i].first, n, i < 8 ? ref_u : ref_m); }
        printf("%6llu", (unsigned long long)n);
        for (size_t i = 0; i < fs.size(); ++i) printf(i == 8 ? " | %9.2f" : " %9.2f", t[i]);
        printf("\n");
        fflush(stdout);
    }
    printf(bad_total ? "MISMATCH\n" : "all bit-exact\n");
    return bad_total ? 1 : 0;
}
