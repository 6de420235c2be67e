// What clock does the shader run at while the c3 kernel streams, and does rocprofv3
// change it? (DESIGN_LOG.md §5: the process under `rocprofv3 --kernel-trace` times the
// shipped kernel 2-5 % slower than the plain bench, and there the hash falls below
// its own hash-free control.)
//
// One process, one 128 GiB arena (4M x 32 KiB blocks). Stream A runs, R rounds of:
//   hash  the shipped k_xxh64_glds_skew<16,2,false,8,8,true>
//   xor   the same data movement with the hash replaced by xor (bench's read peak)
// each launch bracketed by 1-thread marker kernels that store s_memrealtime (100 MHz
// constant clock). Stream B runs one 64-thread sampler workgroup beside them: lane 0
// stores (s_memtime, s_memrealtime) pairs every ~200 us, s_sleep in between. s_memtime
// counts shader clocks, so the shader clock over an interval is
// d(memtime) / d(realtime) x 100 MHz. Per launch: duration from its markers, the rate
// as a fraction of 8 TB/s, and the mean shader clock of the samples inside it.
// With fill=1 each launch pair is preceded by the on-device regeneration of the arena
// (k_fill_synthetic, as bench.py does per pass); its interval is reported as "fill".
// Usage: clock_probe [rounds=4] [fill=0]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

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
__global__ void k_mark(uint64_t* marks, int i) {
    if (threadIdx.x == 0) marks[i] = __builtin_amdgcn_s_memrealtime();
}

// Samples until `ticks` of the 100 MHz clock have passed or `max_samples` are taken:
// every wave of the grid reaches the exit.
__global__ void k_sampler(uint64_t* samples, uint32_t max_samples, uint64_t ticks, uint64_t period) {
    if (threadIdx.x != 0) return;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    uint64_t next = t0;
    for (uint32_t k = 0; k < max_samples;) {
        const uint64_t rt = __builtin_amdgcn_s_memrealtime();
        if (rt - t0 > ticks) break;
        if (rt >= next) {
            const uint64_t mt = __builtin_amdgcn_s_memtime();
            const uint64_t rt2 = __builtin_amdgcn_s_memrealtime();
            samples[2 * k] = mt;
            samples[2 * k + 1] = (rt + rt2) / 2;
            ++k;
            next = rt + period;
        }
        __builtin_amdgcn_s_sleep(32);
    }
}
}  // namespace stormck

using namespace stormck;

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 4;
    const bool fill = argc > 2 && atoi(argv[2]) != 0;
    const uint64_t L = 32768, n = 4194304;
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const unsigned cus = (unsigned)prop.multiProcessorCount;
    uint8_t* A;
    uint64_t *out, *marks, *samples;
    const uint32_t max_samples = 1 << 16;
    CK(hipMalloc(&A, n * L));
    CK(hipMalloc(&out, n * 8));
    CK(hipMalloc(&marks, 4096 * 8));
    CK(hipMalloc(&samples, 2ULL * max_samples * 8));
    CK(hipMemset(samples, 0, 2ULL * max_samples * 8));
    hipLaunchKernelGGL(k_fill_synthetic, dim3(8192), dim3(256), 0, 0, A, L, n, 0ULL, 0x53544f524dULL);
    CK(hipDeviceSynchronize());
    hipStream_t sa, sb;
    CK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
    // warm-up launches (clock ramp), untimed
    for (int w = 0; w < 3; ++w)
        hipLaunchKernelGGL((k_xxh64_glds_skew<16, 2, false, 8, 8, true>), dim3(cus), dim3(512), 0, sa, A, L, 32768u, n,
                           out, nullptr, nullptr, nullptr);
    CK(hipStreamSynchronize(sa));
    // sampler for the whole sequence (~45 ms per launch pair and round, plus margin)
    const uint64_t ticks = (uint64_t)(rounds * (fill ? 4 : 2) * 30 + 200) * 100000ULL;  // 100 MHz ticks
    hipLaunchKernelGGL(k_sampler, dim3(1), dim3(64), 0, sb, samples, max_samples, ticks, 20000ULL);
    CK(hipGetLastError());
    int m = 0;
    hipLaunchKernelGGL(k_mark, dim3(1), dim3(64), 0, sa, marks, m++);
    std::vector<int> kind;  // 1 hash, 0 xor, 2 fill
    for (int r = 0; r < rounds; ++r) {
        if (fill) {
            hipLaunchKernelGGL(k_fill_synthetic, dim3(8192), dim3(256), 0, sa, A, L, n, (uint64_t)r * n, 0x53544f524dULL);
            hipLaunchKernelGGL(k_mark, dim3(1), dim3(64), 0, sa, marks, m++);
            kind.push_back(2);
        }
        hipLaunchKernelGGL((k_xxh64_glds_skew<16, 2, false, 8, 8, true>), dim3(cus), dim3(512), 0, sa, A, L, 32768u, n,
                           out, nullptr, nullptr, nullptr);
        hipLaunchKernelGGL(k_mark, dim3(1), dim3(64), 0, sa, marks, m++);
        kind.push_back(1);
        if (fill) {
            hipLaunchKernelGGL(k_fill_synthetic, dim3(8192), dim3(256), 0, sa, A, L, n, (uint64_t)r * n, 0x53544f524dULL);
            hipLaunchKernelGGL(k_mark, dim3(1), dim3(64), 0, sa, marks, m++);
            kind.push_back(2);
        }
        hipLaunchKernelGGL((k_xxh64_glds_skew<16, 2, false, 8, 8, false>), dim3(cus), dim3(512), 0, sa, A, L, 32768u,
                           n, out, nullptr, nullptr, nullptr);
        hipLaunchKernelGGL(k_mark, dim3(1), dim3(64), 0, sa, marks, m++);
        kind.push_back(0);
    }
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    std::vector<uint64_t> mk(m), sm(2ULL * max_samples);
    CK(hipMemcpy(mk.data(), marks, m * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(sm.data(), samples, sm.size() * 8, hipMemcpyDeviceToHost));
    uint32_t ns = 0;
    while (ns < max_samples && sm[2 * ns + 1] != 0) ++ns;
    const double bytes = (double)n * (L + 8);
    printf("samples %u, idle-or-busy clock over the whole sampler run: %.0f MHz\n", ns,
           ns > 1 ? (double)(sm[2 * (ns - 1)] - sm[0]) / (double)(sm[2 * (ns - 1) + 1] - sm[1]) * 100.0 : 0.0);
    double fr[3] = {0, 0, 0}, mhz[3] = {0, 0, 0};
    int cnt[3] = {0, 0, 0};
    const char* kname[3] = {"xor", "hash", "fill"};
    for (int i = 0; i + 1 < m; ++i) {
        const uint64_t a = mk[i], b = mk[i + 1];
        const double ms = (double)(b - a) / 1e5;
        // clock from the first and last sample strictly inside [a, b]
        int first = -1, last = -1;
        for (uint32_t k = 0; k < ns; ++k) {
            const uint64_t rt = sm[2 * k + 1];
            if (rt > a && rt < b) {
                if (first < 0) first = (int)k;
                last = (int)k;
            }
        }
        double clk = 0;
        if (first >= 0 && last > first)
            clk = (double)(sm[2 * last] - sm[2 * first]) / (double)(sm[2 * last + 1] - sm[2 * first + 1]) * 100.0;
        const double frac = bytes / (ms * 1e-3) / 8e12;
        printf("%-4s %2d  %.3f ms  frac %.4f  sclk %.0f MHz (%d samples)\n", kname[kind[i]], i / (fill ? 4 : 2), ms, frac,
               clk, last >= first && first >= 0 ? last - first + 1 : 0);
        fr[kind[i]] += frac;
        mhz[kind[i]] += clk;
        cnt[kind[i]]++;
    }
    for (int k = 1; k >= 0; --k)
        printf("mean %-4s frac %.4f  sclk %.0f MHz\n", kname[k], fr[k] / cnt[k], mhz[k] / cnt[k]);
    if (cnt[2]) printf("mean fill sclk %.0f MHz\n", mhz[2] / cnt[2]);
    return 0;
}
