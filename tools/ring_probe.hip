// Does the streaming kernel run faster with more bytes in flight per CU?
//
// The shipped k_xxh64_glds_skew keeps a 2-slot ring of 64 KiB tiles (T = 16 stripes of
// 128 blocks): while one tile hashes, ONE tile is in flight, 64 KiB per CU, 16 MiB
// over the chip. At 7.2 TB/s that is 2.3 us of memory latency covered (Little's law),
// which may be all the latency there is under load -- or the limit. A ring of R slots
// of smaller tiles keeps R-1 tiles in flight in the same LDS: T = 8, R = 4 holds 96 KiB
// in flight, T = 8, R = 5 holds 128 KiB (160 KiB of LDS), T = 4, R = 8 holds 112 KiB.
//
// k_xxh64_glds_rs<T, R, SKEW> is the shipped kernel with an R-slot ring: a wave waits
// for its tile w with R-2 newer tiles still in flight, then issues tile w+R-1 into the
// slot it hashed last step. Waves start SKEW tiles apart (4 KiB for every T here), as
// shipped. Every variant is checked bit-exact against the shipped kernel, then timed
// on two arenas (their HBM placements differ), interleaved.
// Usage: ring_probe [GiB=128] [reps=5] [rounds=3]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <functional>
#include <string>
#include <vector>

#include "../storm_amd/csrc/kernels.h"

#define CK(x)                                                                                          \
    do {                                                                                               \
        hipError_t e = (x);                                                                            \
        if (e != hipSuccess) {                                                                         \
            fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__);            \
            exit(1);                                                                                   \
        }                                                                                              \
    } while (0)

namespace stormck {
// PERM 1: wave v hashes the group's blocks v, v+8, v+16, ... instead of 16v..16v+15.
// PHASE k: wave v starts (k*v mod WAVES)*SKEW tiles late (k = 1: shipped order).
template <int T, int R, int SKEW, int WAVES = 8, int PERM = 0, int PHASE = 1>
__global__ __launch_bounds__(64 * WAVES) void k_xxh64_glds_rs(const uint8_t* __restrict__ base, uint64_t stride,
                                                              uint32_t len, uint64_t n, uint64_t* __restrict__ out) {
    constexpr int BPW = 16 * WAVES;
    constexpr int ROW = 32 * T;
    constexpr int TILE = BPW * ROW;
    constexpr int INSTR = TILE / 1024;
    constexpr int PER_WAVE = INSTR / WAVES;
    static_assert(INSTR % WAVES == 0 && T % 2 == 0 && R >= 2, "a wave's pieces are its own block rows");
    __shared__ __attribute__((aligned(16))) uint8_t lds[R * TILE];

    const uint32_t tid = threadIdx.x;
    const uint32_t wave = tid >> 6, lane = tid & 63;
    const uint64_t ngroups = (n + BPW - 1) / BPW;
    const uint64_t G = gridDim.x;
    if (blockIdx.x >= ngroups) return;
    const uint32_t nst = len >> 5, ntiles = nst / T;
    const uint64_t total = ((ngroups - blockIdx.x + G - 1) / G) * ntiles;
    const int64_t ph = static_cast<int64_t>((PHASE * wave) % WAVES) * SKEW;
    auto perm = [](uint32_t bb) -> uint32_t { return PERM ? (bb % 16) * WAVES + bb / 16 : bb; };
    const uint64_t steps = total + static_cast<uint64_t>(WAVES - 1) * SKEW;

    uint32_t prow[PER_WAVE], pofs[PER_WAVE];
#pragma unroll
    for (int k = 0; k < PER_WAVE; ++k) {
        const uint32_t off = (wave * PER_WAVE + k) * 1024 + lane * 16;
        const uint32_t b = off / ROW, q = (off % ROW) / 16;
        prow[k] = b;
        pofs[k] = ((q + glds_rot<T>(b)) % (2 * T)) * 16;
    }
    const uint8_t* src[PER_WAVE];
    uint64_t ig = blockIdx.x, hg = blockIdx.x, ic = 0, hc = 0;
    uint32_t it = 0, ht = 0;
    auto issue = [&](uint32_t slot) {
        if (it == 0) {
#pragma unroll
            for (int k = 0; k < PER_WAVE; ++k) {
                uint64_t gb = ig * BPW + perm(prow[k]);
                if (gb >= n) gb = n - 1;
                src[k] = base + gb * stride + pofs[k];
            }
        }
        STORMCK_GLDS_ISSUE(src, lds + slot * TILE + wave * PER_WAVE * 1024, it, PER_WAVE, ROW, 2);
        if (++it == ntiles) {
            it = 0;
            ig += G;
        }
        ++ic;
    };
    const uint32_t b = tid >> 2, j = tid & 3;
    const uint32_t rot = glds_rot<T>(b);
    uint64_t acc = acc_seed(j);
    if (ph == 0)
        for (int k = 0; k < R - 1; ++k)
            if (ic < total) issue(k);
    for (uint64_t u = 0; u < steps; ++u) {
        const int64_t w = static_cast<int64_t>(u) - ph;  // this wave's tile to hash at this step
        if (w >= 0 && hc < total) {
            if (ic >= static_cast<uint64_t>(w) + R - 1) wait_vmcnt<PER_WAVE * (R - 2)>();
            else wait_vmcnt<0>();
        }
        __builtin_amdgcn_s_barrier();
        if (w + R - 1 >= 0 && ic < total) issue(static_cast<uint32_t>((w + R - 1) % R));
        if (w >= 0 && hc < total) {
            const uint8_t* row = lds + (w % R) * TILE + b * ROW + (j & 1) * 8;
#pragma unroll
            for (int s = 0; s < T; ++s) {
                const uint32_t q = (2 * s + (j >> 1) + 2 * T - rot) % (2 * T);
                acc = round(acc, *reinterpret_cast<const uint64_t*>(row + q * 16));
            }
            if (++ht == ntiles) {
                const uint64_t gbk = hg * BPW + perm(b);
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
// Per-block phases (round 2, placement): every block of a wave also starts E(b) tiles
// late, E(b) in [0, 8), on top of the wave's 8-tile skew, so the 128 blocks of a
// workgroup read 64 different 512 B rows at any moment and concurrent addresses differ
// in bits 9..14 too, not only in the bits the page mapping decides. Addresses are
// computed per step from (step - phase): no per-lane counters. MODE 1: E = b mod 8
// (the two blocks of one DMA instruction differ); MODE 2: E = (b mod 16) / 2 (they
// share a phase).
template <int MODE>
__global__ __launch_bounds__(512) void k_xxh64_glds_qs(const uint8_t* __restrict__ base, uint64_t stride,
                                                       uint32_t len, uint64_t n, uint64_t* __restrict__ out) {
    constexpr int T = 16, WAVES = 8, BPW = 128, ROW = 32 * T, TILE = BPW * ROW, PER_WAVE = TILE / 1024 / WAVES;
    constexpr int SKEW = 8;
    __shared__ __attribute__((aligned(16))) uint8_t lds[2 * TILE];
    const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const uint64_t ngroups = (n + BPW - 1) / BPW, G = gridDim.x;
    if (blockIdx.x >= ngroups) return;
    const uint32_t nst = len >> 5;
    constexpr uint32_t NT = 64;  // 32 KiB blocks only (probe): divisions by NT are shifts
    if (nst / T != NT) return;
    const int64_t tiles = static_cast<int64_t>((ngroups - blockIdx.x + G - 1) / G) * NT;  // per block
    auto phase = [&](uint32_t b) -> int64_t {
        const uint32_t e = MODE == 1 ? (b % 8) : ((b % 16) / 2);
        return static_cast<int64_t>((b / 16) * SKEW + e);
    };
    const int64_t steps = tiles + 7 * SKEW + 7;
    uint32_t prow[PER_WAVE], pofs[PER_WAVE];
    int64_t pph[PER_WAVE];
#pragma unroll
    for (int k = 0; k < PER_WAVE; ++k) {
        const uint32_t off = (wave * PER_WAVE + k) * 1024 + lane * 16;
        const uint32_t b = off / ROW, q = (off % ROW) / 16;
        prow[k] = b;
        pofs[k] = ((q + glds_rot<T>(b)) % (2 * T)) * 16;
        pph[k] = phase(b);
    }
    // per piece: the source of its next row, advanced one row per issue and moved to
    // the block's next group after its last row (no per-step address arithmetic)
    const uint8_t* src[PER_WAVE];
    uint64_t gbk[PER_WAVE];
#pragma unroll
    for (int k = 0; k < PER_WAVE; ++k) {
        gbk[k] = blockIdx.x * BPW + prow[k];
        src[k] = base + (gbk[k] < n ? gbk[k] : n - 1) * stride + pofs[k];
    }
    auto issue = [&](int64_t v) {  // the pieces of virtual step v into slot v & 1
        uint8_t* dst = lds + (v & 1) * TILE + wave * PER_WAVE * 1024;
#pragma unroll
        for (int k = 0; k < PER_WAVE; ++k) {
            const int64_t r = v - pph[k];
            if (r >= 0 && r < tiles) {
                __builtin_amdgcn_global_load_lds(src[k], dst + k * 1024, 16, 0, 2);
                if ((r & (NT - 1)) == NT - 1) {
                    gbk[k] += G * BPW;
                    src[k] = base + (gbk[k] < n ? gbk[k] : n - 1) * stride + pofs[k];
                } else {
                    src[k] += ROW;
                }
            }
        }
    };
    const uint32_t b = tid >> 2, j = tid & 3;
    const uint32_t rot = glds_rot<T>(b);
    const int64_t ph = phase(b);
    uint64_t acc = acc_seed(j);
    issue(0);
    for (int64_t u = 0; u < steps; ++u) {
        wait_vmcnt<0>();
        __builtin_amdgcn_s_barrier();
        if (u + 1 < steps) issue(u + 1);
        const int64_t r = u - ph;
        if (r >= 0 && r < tiles) {
            const uint8_t* row = lds + (u & 1) * TILE + b * ROW + (j & 1) * 8;
#pragma unroll
            for (int s = 0; s < T; ++s) {
                const uint32_t q = (2 * s + (j >> 1) + 2 * T - rot) % (2 * T);
                acc = round(acc, *reinterpret_cast<const uint64_t*>(row + q * 16));
            }
            if (static_cast<uint64_t>(r) % NT == NT - 1) {
                const uint64_t grp = static_cast<uint64_t>(r) / NT;
                const uint64_t gbk = (blockIdx.x + grp * G) * BPW + b;
                const uint64_t gb = gbk < n ? gbk : n - 1;
                const uint8_t* blk_src = base + gb * stride;
                for (uint32_t s = NT * T; s < nst; ++s) acc = round(acc, reinterpret_cast<const uint64_t*>(blk_src)[4 * s + j]);
                const uint64_t v1 = quad_bcast<0>(acc), v2 = quad_bcast<1>(acc), v3 = quad_bcast<2>(acc),
                               v4 = quad_bcast<3>(acc);
                if (j == 0 && gbk < n)
                    out[gbk] = finish_fast(converge(v1, v2, v3, v4), len, blk_src + 32 * static_cast<uint64_t>(nst),
                                           len & 31);
                acc = acc_seed(j);
            }
        }
    }
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
    uint8_t* arena[2];
    for (auto& a : arena) {
        CK(hipMalloc(&a, bytes));
        hipLaunchKernelGGL(k_fill_synthetic, dim3(8192), dim3(256), 0, 0, a, L, n, 0ULL, 0x53544f524dULL);
    }
    CK(hipDeviceSynchronize());
    struct V {
        std::string name;
        std::function<void(uint8_t*, uint64_t*)> f;
    };
    const dim3 g(cus), blk(512);
    std::vector<V> vs = {
        {"shipped skew 8w T=16 R=2", [&](uint8_t* d, uint64_t* o) { hipLaunchKernelGGL((k_xxh64_glds_skew<16, 2, false, 8, 8, true>), g, blk, 0, 0, d, L, (uint32_t)L, n, o, nullptr, nullptr, nullptr); }},
        {"block phases b mod 8", [&](uint8_t* d, uint64_t* o) { hipLaunchKernelGGL((k_xxh64_glds_qs<1>), g, blk, 0, 0, d, L, (uint32_t)L, n, o); }},
        {"block phases (b mod 16)/2", [&](uint8_t* d, uint64_t* o) { hipLaunchKernelGGL((k_xxh64_glds_qs<2>), g, blk, 0, 0, d, L, (uint32_t)L, n, o); }},
        {"shipped again", [&](uint8_t* d, uint64_t* o) { hipLaunchKernelGGL((k_xxh64_glds_skew<16, 2, false, 8, 8, true>), g, blk, 0, 0, d, L, (uint32_t)L, n, o, nullptr, nullptr, nullptr); }},
    };
    std::vector<std::vector<float>> ms(vs.size() * 2);
    for (int a = 0; a < 2; ++a) {
        vs[0].f(arena[a], ref);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(h_ref.data(), ref, n * 8, hipMemcpyDeviceToHost));
        for (size_t v = 1; v < vs.size(); ++v) {
            CK(hipMemset(out, 0, n * 8));
            vs[v].f(arena[a], out);
            CK(hipGetLastError());
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(h_out.data(), out, n * 8, hipMemcpyDeviceToHost));
            uint64_t bad = 0;
            for (uint64_t i = 0; i < n; ++i) bad += h_out[i] != h_ref[i];
            printf("%-32s arena %c: %s (%llu mismatches)\n", vs[v].name.c_str(), 'A' + a, bad ? "MISMATCH" : "bit-exact",
                   (unsigned long long)bad);
            fflush(stdout);
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
            printf("%-32s arena %c  median %.3f ms  %.1f GB/s (%.3f)  min %.3f max %.3f\n", vs[v].name.c_str(), 'A' + a,
                   med, n * (L + 8) / med / 1e6, n * (L + 8) / med / 1e6 / 8000.0, m.front(), m.back());
        }
    printf("done\n");
    return 0;
}
