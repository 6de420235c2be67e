// Does the shipped streaming kernel's rate depend on WHERE its arena lands in HBM?
// Bench runs in separate processes differ by ~2% while every process is steady
// (DESIGN_LOG.md §5). One process: several 128 GiB arenas from hipMalloc and
// hipExtMallocWithFlags(hipDeviceMallocContiguous), each filled and timed.
// Times the shipped large-batch kernel (k_xxh64_glds_skew, 256 workgroups).
// Usage: alloc_probe [GiB=128] [reps=5]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>
#include "../storm_amd/csrc/kernels.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1);} } while (0)
using namespace stormck;

static double time_arena(uint8_t* d, uint64_t n, uint64_t* out, int reps) {
    const uint64_t L = 32768;
    hipLaunchKernelGGL(k_fill_synthetic, dim3(8192), dim3(256), 0, 0, d, L, n, 0ULL, 0x53544f524dULL);
    CK(hipDeviceSynchronize());
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    std::vector<float> ms;
    for (int r = 0; r < reps + 1; ++r) {
        CK(hipEventRecord(a, 0));
        hipLaunchKernelGGL((k_xxh64_glds_skew<16, 2, false, 8, 8>), dim3(256), dim3(512), 0, 0,
                           d, L, (uint32_t)L, n, out, nullptr, nullptr, nullptr);
        CK(hipEventRecord(b, 0)); CK(hipEventSynchronize(b));
        float t; CK(hipEventElapsedTime(&t, a, b));
        if (r) ms.push_back(t);
    }
    std::sort(ms.begin(), ms.end());
    return ms[ms.size() / 2];
}

int main(int argc, char** argv) {
    const double gib = argc > 1 ? atof(argv[1]) : 128.0;
    const int reps = argc > 2 ? atoi(argv[2]) : 5;
    const uint64_t L = 32768, n = (uint64_t)(gib * 1073741824.0) / L, bytes = n * L;
    uint64_t* out; CK(hipMalloc(&out, n * 8));
    auto report = [&](const char* what, uint8_t* d) {
        const double ms = time_arena(d, n, out, reps);
        printf("%-44s %p  %.3f ms  %.1f GB/s (%.3f)\n", what, (void*)d, ms, n * (L + 8) / ms / 1e6, n * (L + 8) / ms / 1e6 / 8000.0);
        fflush(stdout);
    };
    uint8_t *A = nullptr, *B = nullptr, *C = nullptr;
    CK(hipMalloc(&A, bytes));
    report("hipMalloc A", A);
    CK(hipMalloc(&B, bytes));
    report("hipMalloc B (A still held)", B);
    report("hipMalloc A again", A);
    CK(hipFree(A)); CK(hipFree(B));
    hipError_t e = hipExtMallocWithFlags((void**)&C, bytes, hipDeviceMallocContiguous);
    if (e == hipSuccess) {
        report("hipExtMallocWithFlags contiguous C", C);
        CK(hipFree(C));
    } else {
        printf("contiguous allocation of %.0f GiB failed: %s\n", gib, hipGetErrorString(e));
        (void)hipGetLastError();
    }
    // memory types: fine-grained and uncached device memory (MTYPE) instead of the default
    for (unsigned flags : {static_cast<unsigned>(hipDeviceMallocFinegrained), static_cast<unsigned>(hipDeviceMallocUncached)}) {
        uint8_t* F = nullptr;
        hipError_t ef = hipExtMallocWithFlags((void**)&F, bytes, flags);
        if (ef == hipSuccess) {
            report(flags == hipDeviceMallocFinegrained ? "hipExtMallocWithFlags fine-grained" : "hipExtMallocWithFlags uncached", F);
            CK(hipFree(F));
        } else {
            printf("flags %u allocation failed: %s\n", flags, hipGetErrorString(ef));
            (void)hipGetLastError();
        }
    }
    // eight small allocations in a row, then a big one after them
    std::vector<uint8_t*> small(8);
    for (auto& p : small) CK(hipMalloc(&p, 1ULL << 30));
    CK(hipMalloc(&A, bytes));
    report("hipMalloc after 8 x 1 GiB", A);
    CK(hipFree(A));
    for (auto p : small) CK(hipFree(p));
    CK(hipMalloc(&A, bytes + (1ULL << 30)));
    report("hipMalloc +1 GiB, arena at +0", A);
    report("same, arena at +512 MiB", A + (512ULL << 20));
    CK(hipFree(A));
    printf("done\n");
    return 0;
}
