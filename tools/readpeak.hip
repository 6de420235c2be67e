// Measured read peak for bench.py (measurement only, not part of libstormck): the
// shipped large-batch kernel's data movement (k_xxh64_glds_skew, LDS-DMA ring, waves
// 4 KiB apart) with the XXH64 arithmetic replaced by xor, launched on the bench's own
// arena, so the kernel's fraction of it is measured on the same HBM placement
// (DESIGN_LOG.md §5: the rate depends on where the arena lands).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -o tools/libreadpeak.so tools/readpeak.hip
#include <hip/hip_runtime.h>

#include "../storm_amd/csrc/kernels.h"

extern "C" int readpeak_xor_skew(const void* base, uint64_t stride, uint32_t len, uint64_t n, uint64_t* out,
                                 void* stream) {
    if (!base || !out || n == 0 || (stride & 15) || len < 32u * 16) return -1;
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
        return -2;
    const uint64_t groups = (n + 127) / 128;
    const unsigned grid = static_cast<unsigned>(groups < static_cast<uint64_t>(cus) ? groups : cus);
    hipLaunchKernelGGL((stormck::k_xxh64_glds_skew<16, 2, false, 8, 8, false>), dim3(grid), dim3(512), 0,
                       static_cast<hipStream_t>(stream), static_cast<const uint8_t*>(base), stride, len, n, out,
                       nullptr, nullptr, nullptr);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
