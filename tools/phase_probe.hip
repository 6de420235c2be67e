// Does skewing the intra-block offsets that are read at the same moment make the
// streaming kernel faster, or less dependent on where its arena lands in HBM?
// (DESIGN_LOG.md §5: the shipped kernel's rate follows the arena's physical placement,
// 0.86-0.89 of peak, because every workgroup reads the same 512-byte offset of its
// 128 blocks at once and XXH64 fixes each block's stripe order.)
//
// k_xxh64_glds_ps is the persistent streaming kernel with a per-wave start delay:
// wave v of workgroup w starts its tile stream PH tiles late, so a workgroup's rows
// sit at up to 8 different offsets of their blocks. MODE 0: no delay; 1: by wave;
// 2: by workgroup; 3: by wave and workgroup. A wave only reads the LDS rows it loaded
// (its own 16 blocks), so the delays need no extra synchronisation.
// Usage: phase_probe [GiB=128] [reps=5] [rounds=3]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <functional>
#include <string>
#include <vector>
#include "../storm_amd/csrc/kernels.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1);} } while (0)

namespace stormck {
template <int T, int AUX, int MODE, int SKEW = 0, int WAVES = 8>
__global__ __launch_bounds__(64 * WAVES) void k_xxh64_glds_ps(const uint8_t* __restrict__ base, uint64_t stride,
                                                              uint32_t len, uint64_t n, uint64_t* __restrict__ out) {
    constexpr int BPW = 16 * WAVES;
    constexpr int ROW = 32 * T;
    constexpr int TILE = BPW * ROW;
    constexpr int INSTR = TILE / 1024;
    constexpr int PER_WAVE = INSTR / WAVES;
    static_assert(INSTR % WAVES == 0 && T % 2 == 0, "a wave's pieces are its own block rows");
    __shared__ __attribute__((aligned(16))) uint8_t lds[2 * TILE];

    const uint32_t tid = threadIdx.x;
    const uint32_t wave = tid >> 6, lane = tid & 63;
    const uint64_t ngroups = (n + BPW - 1) / BPW;
    const uint64_t G = gridDim.x;
    const uint64_t g0 = blockIdx.x;
    if (g0 >= ngroups) return;
    const uint32_t nst = len >> 5, ntiles = nst / T;
    const uint64_t total = ((ngroups - g0 + G - 1) / G) * ntiles;
    const uint32_t step = SKEW > 0 ? SKEW : ntiles / WAVES;  // tiles between consecutive phases
    const uint32_t ph_idx = MODE == 1 ? wave : (MODE == 2 ? blockIdx.x % WAVES : (MODE == 3 ? (wave + blockIdx.x) % WAVES : 0));
    const uint64_t ph = static_cast<uint64_t>(ph_idx) * step;
    const uint64_t phmax = MODE == 0 ? 0 : static_cast<uint64_t>(WAVES - 1) * step;

    uint32_t prow[PER_WAVE], pofs[PER_WAVE];
#pragma unroll
    for (int k = 0; k < PER_WAVE; ++k) {
        const uint32_t off = (wave * PER_WAVE + k) * 1024 + lane * 16;
        const uint32_t b = off / ROW, q = (off % ROW) / 16;
        prow[k] = b;
        pofs[k] = ((q + glds_rot<T>(b)) % (2 * T)) * 16;
    }
    const uint8_t* src[PER_WAVE];
    uint64_t ig = g0, hg = g0, ic = 0, hc = 0;
    uint32_t it = 0, ht = 0;
    auto issue = [&](uint32_t slot) {
        if (it == 0) {
#pragma unroll
            for (int k = 0; k < PER_WAVE; ++k) {
                uint64_t gb = ig * BPW + prow[k];
                if (gb >= n) gb = n - 1;
                src[k] = base + gb * stride + pofs[k];
            }
        }
        STORMCK_GLDS_ISSUE(src, lds + slot * TILE + wave * PER_WAVE * 1024, it, PER_WAVE, ROW, AUX);
        if (++it == ntiles) {
            it = 0;
            ig += G;
        }
        ++ic;
    };
    const uint32_t b = tid >> 2, j = tid & 3;
    const uint32_t rot = glds_rot<T>(b);
    uint64_t acc = acc_seed(j);
    if (ph == 0 && total > 0) issue(0);
    for (uint64_t u = 0; u < total + phmax; ++u) {
        wait_vmcnt<0>();
        __builtin_amdgcn_s_barrier();
        if (u + 1 >= ph && ic < total) issue((u + 1) & 1);
        if (u >= ph && hc < total) {
            const uint8_t* row = lds + (u & 1) * TILE + b * ROW + (j & 1) * 8;
#pragma unroll
            for (int s = 0; s < T; ++s) {
                const uint32_t q = (2 * s + (j >> 1) + 2 * T - rot) % (2 * T);
                acc = round(acc, *reinterpret_cast<const uint64_t*>(row + q * 16));
            }
            if (++ht == ntiles) {
                const uint64_t gbk = hg * BPW + b;
                const uint64_t gb = gbk < n ? gbk : n - 1;
                const uint8_t* blk_src = base + gb * stride;
                for (uint32_t s = ntiles * T; s < nst; ++s)
                    acc = round(acc, reinterpret_cast<const uint64_t*>(blk_src)[4 * s + j]);
                const uint64_t v1 = quad_bcast<0>(acc), v2 = quad_bcast<1>(acc), v3 = quad_bcast<2>(acc),
                               v4 = quad_bcast<3>(acc);
                if (j == 0 && gbk < n)
                    out[gbk] = finish_fast(converge(v1, v2, v3, v4), len, blk_src + 32 * static_cast<uint64_t>(nst),
                                           len & 31);
                acc = acc_seed(j);
                ht = 0;
                hg += G;
            }
            ++hc;
        }
    }
}
// plain grid-stride dwordx4 read (no LDS): does the arena's placement slow every
// access pattern, or only the block-strided one?
__global__ __launch_bounds__(256) void k_readpeak_nt(const u64x2* __restrict__ p, uint64_t n16, uint64_t* out) {
    u64x2 acc = {0, 0};
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    for (; i + 3 * stride < n16; i += 4 * stride) {
        u64x2 a = ldg<true>(p + i), b = ldg<true>(p + i + stride), c = ldg<true>(p + i + 2 * stride), d = ldg<true>(p + i + 3 * stride);
        acc ^= a ^ b ^ c ^ d;
    }
    for (; i < n16; i += stride) acc ^= ldg<true>(p + i);
    if ((acc.x ^ acc.y) == 0x1234567) out[0] = acc.x;
}
}  // namespace stormck

using namespace stormck;

int main(int argc, char** argv) {
    const double gib = argc > 1 ? atof(argv[1]) : 128.0;
    const int reps = argc > 2 ? atoi(argv[2]) : 5;
    const int rounds = argc > 3 ? atoi(argv[3]) : 3;
    const uint64_t L = 32768, n = (uint64_t)(gib * 1073741824.0) / L, bytes = n * L;
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const unsigned cus = (unsigned)prop.multiProcessorCount;
    uint64_t *ref, *out;
    CK(hipMalloc(&ref, n * 8));
    CK(hipMalloc(&out, n * 8));
    std::vector<uint64_t> h_ref(n), h_out(n);
    hipEvent_t ea, eb;
    CK(hipEventCreate(&ea));
    CK(hipEventCreate(&eb));
    // two arenas at once: their placements differ (alloc_probe: 19.36 vs 19.74 ms)
    uint8_t* arena[2];
    for (auto& a : arena) {
        CK(hipMalloc(&a, bytes));
        hipLaunchKernelGGL(k_fill_synthetic, dim3(8192), dim3(256), 0, 0, a, L, n, 0ULL, 0x53544f524dULL);
    }
    CK(hipDeviceSynchronize());
    const unsigned gp = (unsigned)std::min<uint64_t>((n + 127) / 128, cus);
    struct V {
        std::string name;
        std::function<void(uint8_t*, uint64_t*)> f;
    };
    std::vector<V> vs = {
        {"shipped glds 8w T=16", [&](uint8_t* d, uint64_t* o) { hipLaunchKernelGGL((k_xxh64_glds<16, 2, 2, true, false, 8>), dim3((unsigned)((n + 127) / 128)), dim3(512), 0, 0, d, L, (uint32_t)L, n, o, nullptr, nullptr, nullptr); }},
        {"persistent, no skew", [&](uint8_t* d, uint64_t* o) { hipLaunchKernelGGL((k_xxh64_glds_ps<16, 2, 0>), dim3(gp), dim3(512), 0, 0, d, L, (uint32_t)L, n, o); }},
        {"grid-stride read nt (no hash)", [&](uint8_t* d, uint64_t* o) { hipLaunchKernelGGL(k_readpeak_nt, dim3(16384), dim3(256), 0, 0, (const u64x2*)d, bytes / 16, o); }},
        {"wave skew 16 tiles (8 KiB)", [&](uint8_t* d, uint64_t* o) { hipLaunchKernelGGL((k_xxh64_glds_ps<16, 2, 1, 16>), dim3(gp), dim3(512), 0, 0, d, L, (uint32_t)L, n, o); }},
        {"wave+wg skew 8 tiles", [&](uint8_t* d, uint64_t* o) { hipLaunchKernelGGL((k_xxh64_glds_ps<16, 2, 3, 8>), dim3(gp), dim3(512), 0, 0, d, L, (uint32_t)L, n, o); }},
        {"wave skew 8 tiles (4 KiB)", [&](uint8_t* d, uint64_t* o) { hipLaunchKernelGGL((k_xxh64_glds_ps<16, 2, 1, 8>), dim3(gp), dim3(512), 0, 0, d, L, (uint32_t)L, n, o); }},
    };
    std::vector<std::vector<float>> ms(vs.size() * 2);
    for (int a = 0; a < 2; ++a) {
        vs[0].f(arena[a], ref);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(h_ref.data(), ref, n * 8, hipMemcpyDeviceToHost));
        for (size_t v = 1; v < vs.size(); ++v) {
            if (vs[v].name.find("no hash") != std::string::npos) continue;
            CK(hipMemset(out, 0, n * 8));
            vs[v].f(arena[a], out);
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(h_out.data(), out, n * 8, hipMemcpyDeviceToHost));
            uint64_t bad = 0;
            for (uint64_t i = 0; i < n; ++i) bad += h_out[i] != h_ref[i];
            if (bad) printf("!! %s arena %d: %llu mismatches\n", vs[v].name.c_str(), a, (unsigned long long)bad);
        }
    }
    for (int r = 0; r < rounds; ++r)
        for (int a = 0; a < 2; ++a)
            for (size_t v = 0; v < vs.size(); ++v)
                for (int k = 0; k < reps; ++k) {
                    CK(hipEventRecord(ea, 0));
                    vs[v].f(arena[a], out);
                    CK(hipEventRecord(eb, 0));
                    CK(hipEventSynchronize(eb));
                    float t;
                    CK(hipEventElapsedTime(&t, ea, eb));
                    ms[v * 2 + a].push_back(t);
                }
    for (size_t v = 0; v < vs.size(); ++v)
        for (int a = 0; a < 2; ++a) {
            auto m = ms[v * 2 + a];
            std::sort(m.begin(), m.end());
            const double med = m[m.size() / 2];
            printf("%-32s arena %c  median %.3f ms  %.1f GB/s (%.3f)  min %.3f max %.3f\n", vs[v].name.c_str(), 'A' + a, med,
                   n * (L + 8) / med / 1e6, n * (L + 8) / med / 1e6 / 8000.0, m.front(), m.back());
        }
    printf("done\n");
    return 0;
}
