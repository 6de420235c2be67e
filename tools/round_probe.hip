// Cycles per XXH64 round for one wave, operands in registers (no memory), timed
// in-kernel with s_memtime. Which form of the round sets the latency floor of a
// one-block-per-quad chain (small batches, DESIGN_LOG.md §4)?
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/round_probe tools/round_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "../storm_amd/csrc/xxh64_dev.h"

using namespace stormck;

#define CK(x)                                                                                \
    do {                                                                                     \
        hipError_t e = (x);                                                                  \
        if (e != hipSuccess) {                                                               \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
            exit(1);                                                                         \
        }                                                                                    \
    } while (0)

constexpr uint64_t inv_odd(uint64_t a) {
    uint64_t x = a;
    for (int i = 0; i < 5; ++i) x *= 2 - a * x;
    return x;
}

__device__ __forceinline__ uint64_t step_t(uint64_t x, uint64_t t) {
    const uint32_t xl = static_cast<uint32_t>(x), xh = static_cast<uint32_t>(x >> 32);
    const uint32_t rh = __builtin_amdgcn_alignbit(xh, xl, 1);
    const uint32_t rl = __builtin_amdgcn_alignbit(xl, xh, 1);
    uint64_t prod, carry;
    asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(prod), "=s"(carry) : "v"(rl), "s"(static_cast<uint32_t>(kP1)), "v"(t));
    const uint32_t hi = static_cast<uint32_t>(prod >> 32) + rl * static_cast<uint32_t>(kP1 >> 32) + rh * static_cast<uint32_t>(kP1);
    return (static_cast<uint64_t>(hi) << 32) | static_cast<uint32_t>(prod);
}

// MODE 0: classic round(acc, w); 1: folded step with t = w*P2 in the loop;
// 2: folded step with t given (no w*P2); 3: two independent classic chains;
// 4: add + rotate only (no multiply); 5: one 64-bit multiply by P1 per round only
template <int MODE>
__global__ void k_rounds(const uint64_t* __restrict__ in, uint64_t* __restrict__ out, uint32_t rounds,
                         long long* __restrict__ cycles) {
    uint64_t w[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) w[u] = in[threadIdx.x * 16 + u];
    uint64_t a = in[1024 + threadIdx.x], b = a ^ 0x1234;
    __builtin_amdgcn_s_waitcnt(0);
    const long long t0 = clock64();
    for (uint32_t r = 0; r < rounds; r += 16) {
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            if constexpr (MODE == 0) a = round(a, w[u]);
            else if constexpr (MODE == 1) a = step_t(a, w[u] * kP2);
            else if constexpr (MODE == 2) a = step_t(a, w[u]);
            else if constexpr (MODE == 3) { a = round(a, w[u]); b = round(b, w[u]); }
            else if constexpr (MODE == 4) a = rotl<31>(a + w[u]);
            else a = a * kP1 + w[u];
        }
    }
    const long long t1 = clock64();
    out[threadIdx.x] = a ^ b;
    if (threadIdx.x == 0) cycles[blockIdx.x] = t1 - t0;
}

int main() {
    uint64_t *in, *out; long long* cyc;
    CK(hipMalloc(&in, 4096 * 8)); CK(hipMalloc(&out, 4096 * 8)); CK(hipMalloc(&cyc, 1024 * 8));
    CK(hipMemset(in, 0x5a, 4096 * 8));
    const uint32_t rounds = 16384;
    const char* names[] = {"classic round(acc,w)", "folded, t=w*P2 in loop", "folded, t given", "2 classic chains",
                           "add+rotl only", "mul P1 + add only"};
    // s_memtime counts at a fixed 100 MHz on gfx9 (not the shader clock): also time with events
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (int pass = 0; pass < 2; ++pass) {
        for (int m = 0; m < 6; ++m) {
            auto launch = [&](unsigned grid) {
                switch (m) {
                    case 0: hipLaunchKernelGGL(k_rounds<0>, dim3(grid), dim3(64), 0, 0, in, out, rounds, cyc); break;
                    case 1: hipLaunchKernelGGL(k_rounds<1>, dim3(grid), dim3(64), 0, 0, in, out, rounds, cyc); break;
                    case 2: hipLaunchKernelGGL(k_rounds<2>, dim3(grid), dim3(64), 0, 0, in, out, rounds, cyc); break;
                    case 3: hipLaunchKernelGGL(k_rounds<3>, dim3(grid), dim3(64), 0, 0, in, out, rounds, cyc); break;
                    case 4: hipLaunchKernelGGL(k_rounds<4>, dim3(grid), dim3(64), 0, 0, in, out, rounds, cyc); break;
                    default: hipLaunchKernelGGL(k_rounds<5>, dim3(grid), dim3(64), 0, 0, in, out, rounds, cyc); break;
                }
            };
            for (int w = 0; w < 20; ++w) launch(1);
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0, 0));
            for (int w = 0; w < 20; ++w) launch(1);
            CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
            float ms; CK(hipEventElapsedTime(&ms, e0, e1));
            long long c; CK(hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost));
            if (pass) printf("%-26s  %8.2f ns/round (events)   %8.3f memtime ticks/round\n", names[m], ms * 1e6 / 20 / rounds,
                             (double)c / rounds);
        }
    }
    printf("done\n");
    return 0;
}
