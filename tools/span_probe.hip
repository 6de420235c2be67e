// Is the streaming checksum kernel's 0.85-0.90 of 8 TB/s the HBM's read ceiling, or
// the ceiling of its access pattern over a 128 GiB arena?
//
// In the key-tag probe a grid-stride non-temporal read (4 x 16 B loads in flight per
// lane) read 12.9 GB at 7.5-7.8 TB/s, above the 7.0-7.2 TB/s the checksum kernel and
// its hash-free control reach on the c3 arena. Two things differ: the span (12.9 GB
// against 137 GB) and the pattern (each workgroup of the checksum kernel walks 128
// blocks 32 KiB apart in step, so the chip has ~32K 4 KiB regions open at once; the
// grid-stride read sweeps one contiguous 64 MiB window). This probe times, on
// prefixes of one arena, interleaved:
//   hash   the shipped k_xxh64_glds_skew<16,2,false,8,8,true>
//   xor    the same data movement with the hash replaced by xor (bench's read peak)
//   gs4    grid-stride nt read, 4 x 16 B in flight per lane
//   gs8    grid-stride nt read, 8 x 16 B in flight per lane
// Round 2 of the probe adds placement: the same kernels on 12 GiB regions of the
// arena and on separate 12 GiB allocations made before and after it.
// Usage: span_probe [GiB=128] [reps=5] [rounds=3]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <string>
#include <utility>
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
template <int U>
__global__ __launch_bounds__(256) void k_read_gs(const u64x2* __restrict__ p, uint64_t n16, uint64_t* out) {
    u64x2 acc = {0, 0};
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    for (; i + (U - 1) * stride < n16; i += U * stride) {
        u64x2 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = ldg<true>(p + i + u * stride);
#pragma unroll
        for (int u = 0; u < U; ++u) acc ^= v[u];
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
    const uint64_t L = 32768, nmax = (uint64_t)(gib * 1073741824.0) / L, n12 = 393216;
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const unsigned cus = (unsigned)prop.multiProcessorCount;
    // allocation order: B (12 GiB), then the arena A, then C (12 GiB)
    uint8_t *B, *A, *C;
    uint64_t* out;
    CK(hipMalloc(&B, n12 * L));
    CK(hipMalloc(&A, nmax * L));
    CK(hipMalloc(&C, n12 * L));
    CK(hipMalloc(&out, nmax * 8));
    for (auto [p, n] : {std::pair<uint8_t*, uint64_t>{B, n12}, {A, nmax}, {C, n12}})
        hipLaunchKernelGGL(k_fill_synthetic, dim3(8192), dim3(256), 0, 0, p, L, n, 0ULL, 0x53544f524dULL);
    CK(hipDeviceSynchronize());
    printf("B %p  A %p  C %p\n", (void*)B, (void*)A, (void*)C);
    hipEvent_t ea, eb;
    CK(hipEventCreate(&ea));
    CK(hipEventCreate(&eb));
    struct R {
        std::string name;
        uint8_t* p;
        uint64_t n;
    };
    std::vector<R> regions = {{"B: own 12 GiB, allocated first", B, n12},
                              {"A: first 12 GiB of the arena", A, n12},
                              {"A: 12 GiB at 64 GiB", A + (nmax / 2) * L, n12},
                              {"A: last 12 GiB", A + (nmax - n12) * L, n12},
                              {"C: own 12 GiB, allocated last", C, n12},
                              {"A: whole arena", A, nmax}};
    const char* names[4] = {"hash", "xor", "gs4", "gs8"};
    auto run = [&](int k, uint8_t* base, uint64_t n) {
        switch (k) {
            case 0:
                hipLaunchKernelGGL((k_xxh64_glds_skew<16, 2, false, 8, 8, true>), dim3(cus), dim3(512), 0, 0, base, L,
                                   (uint32_t)L, n, out, nullptr, nullptr, nullptr);
                break;
            case 1:
                hipLaunchKernelGGL((k_xxh64_glds_skew<16, 2, false, 8, 8, false>), dim3(cus), dim3(512), 0, 0, base, L,
                                   (uint32_t)L, n, out, nullptr, nullptr, nullptr);
                break;
            case 2:
                hipLaunchKernelGGL(k_read_gs<4>, dim3(16384), dim3(256), 0, 0, (const u64x2*)base, n * L / 16, out);
                break;
            default:
                hipLaunchKernelGGL(k_read_gs<8>, dim3(8192), dim3(256), 0, 0, (const u64x2*)base, n * L / 16, out);
        }
    };
    std::vector<std::vector<float>> ms(regions.size() * 4);
    for (int r = 0; r < rounds; ++r)
        for (size_t s = 0; s < regions.size(); ++s)
            for (int k = 0; k < 4; ++k) {
                run(k, regions[s].p, regions[s].n);  // warm
                for (int i = 0; i < reps; ++i) {
                    CK(hipEventRecord(ea, 0));
                    run(k, regions[s].p, regions[s].n);
                    CK(hipEventRecord(eb, 0));
                    CK(hipEventSynchronize(eb));
                    float t;
                    CK(hipEventElapsedTime(&t, ea, eb));
                    ms[s * 4 + k].push_back(t);
                }
            }
    CK(hipGetLastError());
    for (size_t s = 0; s < regions.size(); ++s)
        for (int k = 0; k < 4; ++k) {
            auto m = ms[s * 4 + k];
            std::sort(m.begin(), m.end());
            const double med = m[m.size() / 2], bytes = regions[s].n * (double)L;
            printf("%-32s %-5s median %8.3f ms  %7.1f GB/s (%.3f of 8 TB/s)  best %.3f\n", regions[s].name.c_str(),
                   names[k], med, bytes / med / 1e6, bytes / med / 1e6 / 8000.0, bytes / m.front() / 1e6 / 8000.0);
        }
    printf("done\n");
    return 0;
}
