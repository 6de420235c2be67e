// Design probe for the block-checksum kernels on MI355X (gfx950).
// Measures, in ONE process (guide §5.4 rule 24):
//   1. stream-read peak (dwordx4 grid-stride sum, plain / non-temporal)
//   2. hash-kernel mapping variants (quad / lane, unroll U, NT) on synthetic 32 KiB blocks
//   3. a compute-only hash loop (no loads) = the VALU ceiling in byte-equivalents
//   4. v_mul_lo_u32 / v_mad_u64_u32 issue rate vs v_add_u32
// Every hash variant is checked bit-exact against a host XXH64 of the first blocks.
// Usage: probe [GiB=64] [reps=5] [rounds=3]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>
#include <algorithm>
#include <string>
#include <functional>
#include "../storm_amd/csrc/kernels.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1);} } while (0)

using namespace stormck;

// Rejected alternative kept for the design comparison (DESIGN_LOG.md §4): one lane per
// block, all four accumulators in the lane, dwordx4 loads of whole stripes.
namespace stormck {
// ---------------------------------------------------------------------------
// Lane kernel: 1 lane per block, uniform length, 16-byte aligned blocks
// (base % 16 == 0, stride % 16 == 0). U stripes (2U dwordx4) per pipelined group.
}  // namespace stormck

namespace stormck {
// ---------------------------------------------------------------------------
// REJECTED (profiles/r01_probe_persist.txt: 0.884-0.886 vs 0.886 for the one-group-per-
// workgroup kernel; DESIGN_LOG.md §4). Persistent form of k_xxh64_glds (R = 2, barrier-synchronised ring): one workgroup per
// CU walks groups g = blockIdx.x, + gridDim.x, ... of 16*WAVES blocks, and the tile
// stream runs on across group boundaries, so the first tile of the next group is in
// flight while the current group's last tile hashes and its blocks finish. The
// one-group-per-workgroup kernel drains the ring at every group and pays a workgroup
// launch plus a memory round trip before the next group's first tile lands (1 WG per
// CU: the 128 KiB ring leaves no room for a second). At any time the resident
// workgroups cover a contiguous window of groups, as with the hardware's dispatch order.
// Requires nst / T >= 1 (the host checks).
// ---------------------------------------------------------------------------
template <int T, int AUX, bool HASH = true, bool VERIFY = false, int WAVES = 8>
__global__ __launch_bounds__(64 * WAVES) void k_xxh64_glds_p(const uint8_t* __restrict__ base, uint64_t stride,
                                                             uint32_t len, uint64_t n, uint64_t* __restrict__ out,
                                                             const uint64_t* __restrict__ expected = nullptr,
                                                             unsigned long long* __restrict__ first_bad = nullptr,
                                                             unsigned long long* __restrict__ n_bad = nullptr) {
    constexpr int BPW = 16 * WAVES;
    constexpr int ROW = 32 * T;
    constexpr int TILE = BPW * ROW;
    constexpr int INSTR = TILE / 1024;
    constexpr int PER_WAVE = INSTR / WAVES;
    static_assert(INSTR % WAVES == 0, "tile must split evenly over the waves");
    __shared__ __attribute__((aligned(16))) uint8_t lds[2 * TILE];

    const uint32_t tid = threadIdx.x;
    const uint32_t wave = tid >> 6, lane = tid & 63;
    const uint64_t ngroups = (n + BPW - 1) / BPW;
    const uint64_t G = gridDim.x;
    uint64_t g = blockIdx.x;
    if (g >= ngroups) return;
    const uint32_t nst = len >> 5, ntiles = nst / T;
    const uint64_t total = ((ngroups - g + G - 1) / G) * ntiles;

    // piece geometry, the same in every group: block row and source byte offset
    uint32_t prow[PER_WAVE], pofs[PER_WAVE];
#pragma unroll
    for (int k = 0; k < PER_WAVE; ++k) {
        const uint32_t off = (wave * PER_WAVE + k) * 1024 + lane * 16;
        const uint32_t b = off / ROW, q = (off % ROW) / 16;
        prow[k] = b;
        pofs[k] = ((q + glds_rot<T>(b)) % (2 * T)) * 16;
    }
    const uint8_t* src[PER_WAVE];
    auto set_src = [&](uint64_t grp) {
#pragma unroll
        for (int k = 0; k < PER_WAVE; ++k) {
            uint64_t gb = grp * BPW + prow[k];
            if (gb >= n) gb = n - 1;  // shadow the last block; never stored
            src[k] = base + gb * stride + pofs[k];
        }
    };

    const uint32_t b = tid >> 2, j = tid & 3;
    const uint32_t rot = glds_rot<T>(b);
    uint64_t acc = acc_seed(j);
    set_src(g);
    STORMCK_GLDS_ISSUE(src, lds + wave * PER_WAVE * 1024, 0u, PER_WAVE, ROW, AUX);
    uint32_t t = 0;
    for (uint64_t u = 0; u < total; ++u) {
        wait_vmcnt<0>();
        __builtin_amdgcn_s_barrier();
        if (u + 1 < total) {
            uint32_t tn = t + 1;
            if (tn == ntiles) {
                tn = 0;
                set_src(g + G);
            }
            STORMCK_GLDS_ISSUE(src, lds + ((u + 1) & 1) * TILE + wave * PER_WAVE * 1024, tn, PER_WAVE, ROW, AUX);
        }
        const uint8_t* row = lds + (u & 1) * TILE + b * ROW + (j & 1) * 8;
#pragma unroll
        for (int s = 0; s < T; ++s) {
            const uint32_t q = (2 * s + (j >> 1) + 2 * T - rot) % (2 * T);
            const uint64_t w = *reinterpret_cast<const uint64_t*>(row + q * 16);
            if constexpr (HASH) acc = round(acc, w);
            else acc ^= w;
        }
        if (++t == ntiles) {
            // this group's blocks are complete: remainder stripes and tail from global
            // memory (none for 32 KiB blocks), then the checksum
            const uint64_t gbk = g * BPW + b;
            const uint64_t gb = gbk < n ? gbk : n - 1;
            const uint8_t* blk_src = base + gb * stride;
            for (uint32_t s = ntiles * T; s < nst; ++s)
                acc = round(acc, reinterpret_cast<const uint64_t*>(blk_src)[4 * s + j]);
            const uint64_t v1 = quad_bcast<0>(acc), v2 = quad_bcast<1>(acc), v3 = quad_bcast<2>(acc),
                           v4 = quad_bcast<3>(acc);
            if (j == 0 && gbk < n) {
                const uint64_t h0 = converge(v1, v2, v3, v4);
                const uint64_t h = finish_fast(h0, len, blk_src + 32 * static_cast<uint64_t>(nst), len & 31);
                if constexpr (VERIFY) {
                    if (h != expected[gbk]) {
                        atomicMin(first_bad, static_cast<unsigned long long>(gbk));
                        atomicAdd(n_bad, 1ULL);
                    }
                } else {
                    out[gbk] = h;
                }
            }
            acc = acc_seed(j);
            t = 0;
            g += G;
        }
    }
}

}  // namespace stormck

namespace stormck {
// REJECTED, the north star's literal mapping (DESIGN_LOG.md §4): ONE WAVEFRONT PER BLOCK.
// The wave streams its block through a private 2 x 2 KiB LDS ring with coalesced
// LDS-DMA (64 lanes x 16 B per instruction), and quad 0 hashes each tile (XXH64's four
// serial accumulators leave no work for the other 60 lanes). Requires len % 2048 == 0.
template <int WPB>
__global__ __launch_bounds__(64 * WPB) void k_xxh64_wave(const uint8_t* __restrict__ base, uint64_t stride,
                                                         uint32_t len, uint64_t n, uint64_t* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[WPB * 2 * 2048];
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint64_t blk = static_cast<uint64_t>(blockIdx.x) * WPB + wave;
    if (blk >= n) return;
    const uint8_t* src = base + blk * stride + lane * 16;
    uint8_t* ring = lds + wave * 2 * 2048;
    const uint32_t ntiles = len / 2048;
    const uint8_t* s2[2] = {src, src + 1024};
    STORMCK_GLDS_ISSUE(s2, ring, 0u, 2, 2048, 2);
    uint64_t acc = acc_seed(lane & 3);
    for (uint32_t t = 0; t < ntiles; ++t) {
        wait_vmcnt<0>();
        wait_lgkm0();
        if (t + 1 < ntiles) STORMCK_GLDS_ISSUE(s2, ring + ((t + 1) & 1) * 2048, t + 1, 2, 2048, 2);
        if (lane < 4) {
            const uint8_t* tile = ring + (t & 1) * 2048 + lane * 8;
#pragma unroll 8
            for (int s = 0; s < 64; ++s) acc = round(acc, *reinterpret_cast<const uint64_t*>(tile + 32 * s));
        }
    }
    const uint64_t v1 = quad_bcast<0>(acc), v2 = quad_bcast<1>(acc), v3 = quad_bcast<2>(acc), v4 = quad_bcast<3>(acc);
    if (lane == 0) out[blk] = finish_fast(converge(v1, v2, v3, v4), len, base + blk * stride + len, 0);
}
}  // namespace stormck

// ---- host XXH64 (probe self-check only) ----
static inline uint64_t hrotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
static inline uint64_t hround(uint64_t a, uint64_t w) { a += w * kP2; a = hrotl(a, 31); return a * kP1; }
static uint64_t host_xxh64(const uint8_t* p, size_t n) {
    const uint8_t* e = p + n; uint64_t h;
    if (n >= 32) {
        uint64_t v1 = kV1, v2 = kV2, v3 = kV3, v4 = kV4;
        do { uint64_t w[4]; memcpy(w, p, 32); v1 = hround(v1, w[0]); v2 = hround(v2, w[1]); v3 = hround(v3, w[2]); v4 = hround(v4, w[3]); p += 32; } while (p + 32 <= e);
        h = hrotl(v1, 1) + hrotl(v2, 7) + hrotl(v3, 12) + hrotl(v4, 18);
        uint64_t vs[4] = {v1, v2, v3, v4};
        for (int i = 0; i < 4; ++i) { h ^= hround(0, vs[i]); h = h * kP1 + kP4; }
    } else h = kP5;
    h += n;
    while (p + 8 <= e) { uint64_t w; memcpy(&w, p, 8); h ^= hround(0, w); h = hrotl(h, 27) * kP1 + kP4; p += 8; }
    if (p + 4 <= e) { uint32_t w; memcpy(&w, p, 4); h ^= (uint64_t)w * kP1; h = hrotl(h, 23) * kP2 + kP3; p += 4; }
    while (p < e) { h ^= (*p) * kP5; h = hrotl(h, 11) * kP1; ++p; }
    h ^= h >> 33; h *= kP2; h ^= h >> 29; h *= kP3; h ^= h >> 32; return h;
}

// ---- read-peak kernels ----
template <bool NT>
__global__ __launch_bounds__(256) void k_readpeak(const u64x2* __restrict__ p, uint64_t n16, uint64_t* out) {
    u64x2 acc = {0, 0};
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    for (; i + 3 * stride < n16; i += 4 * stride) {
        u64x2 a = ldg<NT>(p + i), b = ldg<NT>(p + i + stride), c = ldg<NT>(p + i + 2 * stride), d = ldg<NT>(p + i + 3 * stride);
        acc ^= a ^ b ^ c ^ d;
    }
    for (; i < n16; i += stride) acc ^= ldg<NT>(p + i);
    if ((acc.x ^ acc.y) == 0x1234567) out[0] = acc.x;  // practically never: keeps loads live
}

// ---- compute-only ceiling: same quad loop with register-synthesised words ----
__global__ __launch_bounds__(256) void k_compute_only(uint32_t nst, uint64_t* out) {
    uint64_t acc = acc_seed(threadIdx.x & 3);
    uint64_t w = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    for (uint32_t s = 0; s < nst; s += 4) {
        acc = round(acc, w); acc = round(acc, w + 1); acc = round(acc, w + 2); acc = round(acc, w + 3);
        w += acc >> 60;
    }
    if (acc == 0x1234567) out[0] = acc;
}

// ---- multiply issue rate ----
template <int MODE>
__global__ __launch_bounds__(256) void k_mulrate(uint32_t iters, uint32_t* out) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 5, a5 = a0 + 7, a6 = a0 + 11, a7 = a0 + 13;
    const uint32_t c = 0x9E3779B1u + blockIdx.x;
    for (uint32_t i = 0; i < iters; ++i) {
        if (MODE == 0) {  // v_mul_lo_u32
            a0 *= c; a1 *= c; a2 *= c; a3 *= c; a4 *= c; a5 *= c; a6 *= c; a7 *= c;
        } else if (MODE == 1) {  // v_add_u32
            a0 += c; a1 += c; a2 += c; a3 += c; a4 += c; a5 += c; a6 += c; a7 += c;
        } else {  // v_mad_u64_u32 (64-bit product of 32-bit operands)
            uint64_t t0 = (uint64_t)a0 * c + a1, t1 = (uint64_t)a2 * c + a3, t2 = (uint64_t)a4 * c + a5, t3 = (uint64_t)a6 * c + a7;
            a0 = (uint32_t)t0; a1 = (uint32_t)(t0 >> 32); a2 = (uint32_t)t1; a3 = (uint32_t)(t1 >> 32);
            a4 = (uint32_t)t2; a5 = (uint32_t)(t2 >> 32); a6 = (uint32_t)t3; a7 = (uint32_t)(t3 >> 32);
        }
    }
    uint32_t r = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
    if (r == 0x1234567) out[0] = r;
}

struct Timer {
    hipEvent_t a, b;
    Timer() { CK(hipEventCreate(&a)); CK(hipEventCreate(&b)); }
    void start() { CK(hipEventRecord(a, 0)); }
    float stop() { CK(hipEventRecord(b, 0)); CK(hipEventSynchronize(b)); float ms; CK(hipEventElapsedTime(&ms, a, b)); return ms; }
};

static int g_reps = 5;

template <typename F>
static void bench(const char* name, double bytes, F launch) {
    Timer t;
    launch();  // warm
    CK(hipDeviceSynchronize());
    std::vector<float> ms;
    for (int r = 0; r < g_reps; ++r) { t.start(); launch(); ms.push_back(t.stop()); }
    std::sort(ms.begin(), ms.end());
    double best = bytes / (ms[0] * 1e-3) / 1e9, med = bytes / (ms[ms.size() / 2] * 1e-3) / 1e9;
    printf("%-34s best %8.3f ms  %8.1f GB/s (%.3f of 8 TB/s)   median %8.1f GB/s\n", name, ms[0], best, best / 8000.0, med);
    fflush(stdout);
}

int main(int argc, char** argv) {
    double gib = argc > 1 ? atof(argv[1]) : 64.0;
    g_reps = argc > 2 ? atoi(argv[2]) : 5;
    const uint64_t L = 32768;
    const uint64_t n = (uint64_t)(gib * 1073741824.0) / L;
    const uint64_t bytes = n * L;
    hipDeviceProp_t prop; CK(hipGetDeviceProperties(&prop, 0));
    printf("device %s  CUs %d  clock %d kHz  blocks %llu (%.1f GiB)\n", prop.gcnArchName, prop.multiProcessorCount, prop.clockRate, (unsigned long long)n, bytes / 1073741824.0);
    uint8_t* d; CK(hipMalloc(&d, bytes));
    uint64_t* out; CK(hipMalloc(&out, n * 8));
    uint64_t* sink; CK(hipMalloc(&sink, 64));
    const uint64_t seed = 0x53544f524dULL;
    hipLaunchKernelGGL(k_fill_synthetic, dim3(8192), dim3(256), 0, 0, d, L, n, 0ULL, seed);
    CK(hipDeviceSynchronize());

    // host reference for the first K blocks
    const uint64_t K = std::min<uint64_t>(n, 2048);
    std::vector<uint8_t> hb(K * L);
    CK(hipMemcpy(hb.data(), d, K * L, hipMemcpyDeviceToHost));
    std::vector<uint64_t> ref(K);
    for (uint64_t i = 0; i < K; ++i) ref[i] = host_xxh64(hb.data() + i * L, L);
    std::vector<uint64_t> got(K);
    auto check = [&](const char* name) {
        CK(hipMemcpy(got.data(), out, K * 8, hipMemcpyDeviceToHost));
        uint64_t bad = 0; for (uint64_t i = 0; i < K; ++i) bad += got[i] != ref[i];
        if (bad) printf("  !! %s: %llu / %llu mismatches\n", name, (unsigned long long)bad, (unsigned long long)K);
        CK(hipMemset(out, 0, K * 8));
    };

    // Interleaved A/B over rounds (guide §5.4 rule 24): every variant once per round.
    const int rounds = argc > 3 ? atoi(argv[3]) : 3;
    const dim3 gq((unsigned)((n * 4 + 255) / 256));
    const dim3 gg((unsigned)((n + 63) / 64));
    struct V { std::string name; std::function<void()> f; bool hash; };
    std::vector<V> vs;
    vs.push_back({"readpeak nt grid=16384", [&] { hipLaunchKernelGGL(k_readpeak<true>, dim3(16384), dim3(256), 0, 0, (const u64x2*)d, bytes / 16, sink); }, false});
    vs.push_back({"quad U=16", [&] { hipLaunchKernelGGL((k_xxh64_quad<16, false, false, false, false>), gq, dim3(256), 0, 0, d, L, nullptr, (uint32_t)L, nullptr, n, out, nullptr, nullptr, nullptr); }, true});
    // glds<T, R, nt> with W waves per workgroup (16 blocks per wave); S = barrier-synchronised
    // ring, N = per-wave ring (each wave waits only for its own pieces)
#define GW(W, T, R, SY)                                                                                       \
    vs.push_back({std::string("glds " #W "w T=" #T " R=" #R) + (SY ? " sync" : " nosync"), [&] {                              \
        hipLaunchKernelGGL((k_xxh64_glds<T, R, 2, true, false, W, SY>), dim3((unsigned)((n + 16 * W - 1) / (16 * W))), \
                           dim3(64 * W), 0, 0, d, L, (uint32_t)L, n, out, nullptr, nullptr, nullptr); }, true})
    GW(8, 16, 2, true);
    // cache-policy bits of the LDS-DMA loads (aux: 1 = sc0, 2 = nt, 16 = sc1) and the XCD remap
#define GA(AUXV, XC)                                                                                           \
    vs.push_back({std::string("glds 8w T=16 R=2 aux=" #AUXV) + (XC ? " xcd" : ""), [&] {                       \
        hipLaunchKernelGGL((k_xxh64_glds<16, 2, AUXV, true, false, 8, true, XC>), dim3((unsigned)((n + 127) / 128)), \
                           dim3(512), 0, 0, d, L, (uint32_t)L, n, out, nullptr, nullptr, nullptr); }, true})

    const dim3 g8((unsigned)((n + 127) / 128));
    vs.push_back({"wave-per-block (4 waves/WG)", [&] { hipLaunchKernelGGL((k_xxh64_wave<4>), dim3((unsigned)((n + 3) / 4)), dim3(256), 0, 0, d, L, (uint32_t)L, n, out); }, true});
    vs.push_back({"wg-per-block (k_xxh64_wide)", [&] { hipLaunchKernelGGL((k_xxh64_wide<false, false, false>), dim3((unsigned)n), dim3(256), 0, 0, d, L, nullptr, (uint32_t)L, nullptr, n, out, nullptr, nullptr, nullptr); }, true});
    // persistent form: one workgroup per CU, the tile stream runs across group boundaries
    const dim3 gp((unsigned)std::min<uint64_t>((n + 127) / 128, (uint64_t)prop.multiProcessorCount));
    vs.push_back({"persist 8w T=16", [&] { hipLaunchKernelGGL((k_xxh64_glds_p<16, 2, true, false, 8>), gp, dim3(512), 0, 0, d, L, (uint32_t)L, n, out, nullptr, nullptr, nullptr); }, true});
    vs.push_back({"persist 8w T=20", [&] { hipLaunchKernelGGL((k_xxh64_glds_p<20, 2, true, false, 8>), gp, dim3(512), 0, 0, d, L, (uint32_t)L, n, out, nullptr, nullptr, nullptr); }, true});
    vs.push_back({"persist 8w T=16 noHash", [&] { hipLaunchKernelGGL((k_xxh64_glds_p<16, 2, false, false, 8>), gp, dim3(512), 0, 0, d, L, (uint32_t)L, n, out, nullptr, nullptr, nullptr); }, false});
    vs.push_back({"glds8w T=16 R=2 noHash", [&] { hipLaunchKernelGGL((k_xxh64_glds<16, 2, 2, false, false, 8>), g8, dim3(512), 0, 0, d, L, (uint32_t)L, n, out, nullptr, nullptr, nullptr); }, false});
    std::vector<std::vector<double>> gbs(vs.size());
    for (int r = 0; r < rounds; ++r) {
        for (size_t v = 0; v < vs.size(); ++v) {
            Timer t;
            vs[v].f();
            CK(hipDeviceSynchronize());
            if (r == 0 && vs[v].hash) check(vs[v].name.c_str());
            for (int k = 0; k < g_reps; ++k) {
                t.start(); vs[v].f(); float ms = t.stop();
                gbs[v].push_back(bytes / (ms * 1e-3) / 1e9);
            }
        }
    }
    for (size_t v = 0; v < vs.size(); ++v) {
        auto g = gbs[v]; std::sort(g.begin(), g.end());
        printf("%-28s max %7.1f  median %7.1f  min %7.1f GB/s  (median %.3f of 8 TB/s)\n", vs[v].name.c_str(), g.back(), g[g.size() / 2], g[0], g[g.size() / 2] / 8000.0);
    }
    fflush(stdout);

    // 3. compute-only ceiling (byte-equivalent: 8 B per lane per round)
    {
        const uint32_t nst = 1024; const unsigned grid = 256 * 32;
        double eq = (double)grid * 256 * nst * 8.0;
        bench("compute-only (byte-equivalent)", eq, [&] { hipLaunchKernelGGL(k_compute_only, dim3(grid), dim3(256), 0, 0, nst, sink); });
    }
    // 4. multiply rate: report Gop/s per CU-cycle via "bytes" = ops
    {
        const uint32_t it = 1 << 16; const unsigned grid = 256 * 16;
        double ops = (double)grid * 256 * it * 8.0;
        printf("(rates below: 'GB/s' column = G lane-ops/s; full-rate ceiling = 256 CU x 128 lanes x clk)\n");
        bench("mul_lo_u32", ops, [&] { hipLaunchKernelGGL(k_mulrate<0>, dim3(grid), dim3(256), 0, 0, it, (uint32_t*)sink); });
        bench("add_u32", ops, [&] { hipLaunchKernelGGL(k_mulrate<1>, dim3(grid), dim3(256), 0, 0, it, (uint32_t*)sink); });
        bench("mad_u64_u32 (x4 per 8 ops)", ops, [&] { hipLaunchKernelGGL(k_mulrate<2>, dim3(grid), dim3(256), 0, 0, it, (uint32_t*)sink); });
    }
    CK(hipFree(d)); CK(hipFree(out)); CK(hipFree(sink));
    printf("done\n");
    return 0;
}
