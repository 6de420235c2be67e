// Host -> HBM gather of scattered 32 KiB blocks (storm's dirty slots of a registered
// cache.data): one hipMemcpyBatchAsync of many 32 KiB copies vs per-block
// hipMemcpyAsync vs one contiguous DMA vs a kernel reading the host pages in place.
// Decides whether f1 on a host arena should stage blocks in HBM (DESIGN_LOG.md §5).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/gather_probe tools/gather_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <numeric>
#include <random>
#include <vector>
#include <sys/mman.h>
#include "../storm_amd/csrc/kernels.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1);} } while (0)
using namespace stormck;

int main(int argc, char** argv) {
    const uint64_t L = 32768, slots = 1 << 18;  // 8 GiB host arena
    const uint64_t n = argc > 1 ? atoll(argv[1]) : 32768;  // dirty blocks (1 GiB)
    uint8_t* host = nullptr;
    CK(hipHostMalloc(reinterpret_cast<void**>(&host), slots * L, hipHostMallocDefault));
    for (uint64_t i = 0; i < slots * L; i += 4096) host[i] = static_cast<uint8_t>(i >> 12);
    uint8_t* d = nullptr;
    CK(hipMalloc(&d, n * L));
    uint64_t* out = nullptr;
    CK(hipMalloc(&out, n * 8));
    std::vector<uint64_t> pick(slots);
    std::iota(pick.begin(), pick.end(), 0);
    std::shuffle(pick.begin(), pick.end(), std::mt19937_64(7));
    pick.resize(n);
    std::vector<void*> dsts(n), srcs(n);
    std::vector<size_t> sizes(n, L);
    for (uint64_t i = 0; i < n; ++i) { dsts[i] = d + i * L; srcs[i] = host + pick[i] * L; }
    hipStream_t st; CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    auto rate = [&](const char* name, auto&& f) {
        f(); CK(hipStreamSynchronize(st));
        float best = 1e9;
        for (int r = 0; r < 3; ++r) {
            CK(hipEventRecord(a, st)); f(); CK(hipEventRecord(b, st)); CK(hipEventSynchronize(b));
            float ms; CK(hipEventElapsedTime(&ms, a, b)); best = std::min(best, ms);
        }
        printf("%-44s %8.2f ms  %6.1f GiB/s\n", name, best, n * L / (best * 1e-3) / 1073741824.0);
        fflush(stdout);
    };
    rate("contiguous DMA (same bytes)", [&] { CK(hipMemcpyAsync(d, host, n * L, hipMemcpyHostToDevice, st)); });
    size_t fail = 0;
    rate("hipMemcpyBatchAsync, scattered 32 KiB", [&] {
        CK(hipMemcpyBatchAsync(dsts.data(), srcs.data(), sizes.data(), n, nullptr, nullptr, 0, &fail, st)); });
    rate("hipMemcpyAsync per block, scattered", [&] {
        for (uint64_t i = 0; i < n; ++i) CK(hipMemcpyAsync(dsts[i], srcs[i], L, hipMemcpyHostToDevice, st)); });
    uint64_t* offs = nullptr;
    CK(hipMalloc(&offs, n * 8));
    std::vector<uint64_t> ho(n);
    for (uint64_t i = 0; i < n; ++i) ho[i] = pick[i] * L;
    CK(hipMemcpy(offs, ho.data(), n * 8, hipMemcpyHostToDevice));
    uint8_t* dhost = nullptr;
    CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&dhost), host, 0));
    rate("quad gather kernel reading host in place", [&] {
        hipLaunchKernelGGL((k_xxh64_quad<16, false, true, false>), dim3((unsigned)((n * 4 + 255) / 256)), dim3(256), 0, st,
                           dhost, 0, nullptr, (uint32_t)L, offs, n, out, nullptr, nullptr, nullptr); });
    // contiguous blocks read in place by each streaming kernel (the device entry point on a
    // registered host arena picks by batch size; which kernel reads PCIe best?)
    rate("glds streaming kernel, contiguous host blocks", [&] {
        hipLaunchKernelGGL((k_xxh64_glds<16, 2, 2, true, false, 8>), dim3((unsigned)((n + 127) / 128)), dim3(512), 0, st,
                           dhost, L, (uint32_t)L, n, out, nullptr, nullptr, nullptr); });
    rate("quad kernel, contiguous host blocks", [&] {
        hipLaunchKernelGGL((k_xxh64_quad<16, false, false, false>), dim3((unsigned)((n * 4 + 255) / 256)), dim3(256), 0, st,
                           dhost, L, nullptr, (uint32_t)L, nullptr, n, out, nullptr, nullptr, nullptr); });
    rate("glds streaming kernel, contiguous, default policy", [&] {
        hipLaunchKernelGGL((k_xxh64_glds<16, 2, 0, true, false, 8>), dim3((unsigned)((n + 127) / 128)), dim3(512), 0, st,
                           dhost, L, (uint32_t)L, n, out, nullptr, nullptr, nullptr); });
    // the same kernels on malloc'd memory page-locked with hipHostRegister (how a Go
    // caller's cache.data would be pinned) instead of hipHostMalloc
    uint8_t* reg = static_cast<uint8_t*>(aligned_alloc(1 << 21, n * L));
    for (uint64_t i = 0; i < n * L; i += 4096) reg[i] = static_cast<uint8_t>(i >> 12);
    CK(hipHostRegister(reg, n * L, hipHostRegisterMapped));
    uint8_t* dreg = nullptr;
    CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&dreg), reg, 0));
    rate("registered malloc: contiguous DMA", [&] { CK(hipMemcpyAsync(d, reg, n * L, hipMemcpyHostToDevice, st)); });
    rate("registered malloc: glds streaming kernel", [&] {
        hipLaunchKernelGGL((k_xxh64_glds<16, 2, 2, true, false, 8>), dim3((unsigned)((n + 127) / 128)), dim3(512), 0, st,
                           dreg, L, (uint32_t)L, n, out, nullptr, nullptr, nullptr); });
    rate("registered malloc: quad kernel", [&] {
        hipLaunchKernelGGL((k_xxh64_quad<16, false, false, false>), dim3((unsigned)((n * 4 + 255) / 256)), dim3(256), 0, st,
                           dreg, L, nullptr, (uint32_t)L, nullptr, n, out, nullptr, nullptr, nullptr); });
    CK(hipHostUnregister(reg));
    free(reg);
    // base alignment: the same registered buffer read from +16 and +64 bytes (a 16-byte
    // aligned allocation, as numpy's, vs a cache-line aligned one, as Go's large objects)
    {
        uint8_t* r3 = static_cast<uint8_t*>(aligned_alloc(1 << 21, n * L + 4096));
        for (uint64_t i = 0; i < n * L + 4096; i += 4096) r3[i] = 1;
        CK(hipHostRegister(r3, n * L + 4096, hipHostRegisterMapped));
        uint8_t* dr3 = nullptr;
        CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&dr3), r3, 0));
        for (uint64_t shift : {16ULL, 64ULL, 256ULL}) {
            char name[80];
            snprintf(name, sizeof name, "glds streaming kernel, base %% 4096 = %llu", (unsigned long long)shift);
            rate(name, [&] {
                hipLaunchKernelGGL((k_xxh64_glds<16, 2, 2, true, false, 8>), dim3((unsigned)((n + 127) / 128)), dim3(512), 0,
                                   st, dr3 + shift, L, (uint32_t)L, n, out, nullptr, nullptr, nullptr); });
        }
        CK(hipHostUnregister(r3));
        free(r3);
    }
    // the same with transparent huge pages refused (4 KiB pages, as most heaps get)
    for (int huge = 0; huge < 2; ++huge) {
        uint8_t* r2 = static_cast<uint8_t*>(aligned_alloc(1 << 21, n * L));
        madvise(r2, n * L, huge ? MADV_HUGEPAGE : MADV_NOHUGEPAGE);
        for (uint64_t i = 0; i < n * L; i += 4096) r2[i] = static_cast<uint8_t>(i >> 12);
        CK(hipHostRegister(r2, n * L, hipHostRegisterMapped));
        uint8_t* dr2 = nullptr;
        CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&dr2), r2, 0));
        rate(huge ? "MADV_HUGEPAGE: glds streaming kernel" : "MADV_NOHUGEPAGE: glds streaming kernel", [&] {
            hipLaunchKernelGGL((k_xxh64_glds<16, 2, 2, true, false, 8>), dim3((unsigned)((n + 127) / 128)), dim3(512), 0,
                               st, dr2, L, (uint32_t)L, n, out, nullptr, nullptr, nullptr); });
        rate(huge ? "MADV_HUGEPAGE: quad gather, scattered" : "MADV_NOHUGEPAGE: quad gather, scattered", [&] {
            hipLaunchKernelGGL((k_xxh64_quad<16, false, false, false>), dim3((unsigned)((n * 4 + 255) / 256)), dim3(256), 0,
                               st, dr2, L, nullptr, (uint32_t)L, nullptr, n, out, nullptr, nullptr, nullptr); });
        CK(hipHostUnregister(r2));
        free(r2);
    }
    printf("done\n");
    return 0;
}
