// Probe (GPU box): where the dispatcher places the waves of a grid. Each wave records
// HW_ID (SIMD, CU, SH, SE) and XCC_ID, and stays resident ~200 us so that the whole
// grid is on the chip at once. Printed per (waves per workgroup, workgroups): CUs used,
// most workgroups on one CU, most waves on one SIMD, and how many SIMDs would hold two
// or more chain waves if the chain waves were the first C = waves/2 of each workgroup
// (k_pointer_level_pc's static roles) or ranked by SIMD (pc_role<true>).
//   hipcc --offload-arch=gfx950 -O3 -o tools/hwid_probe tools/hwid_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <map>
#include <tuple>
#include <vector>

__global__ void k_where(uint32_t* out) {
    uint32_t hwid, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    const uint64_t t0 = wall_clock64();
    while (wall_clock64() - t0 < 20000) __builtin_amdgcn_s_sleep(8);  // 100 MHz clock: 200 us
    const uint32_t w = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
    if ((threadIdx.x & 63) == 0) {
        out[2 * w] = hwid;
        out[2 * w + 1] = xcc;
    }
}

int main() {
    const int wpw[] = {2, 4, 8};
    const int grids[] = {219, 256, 437, 874};
    uint32_t* d;
    if (hipMalloc(&d, 8 * 8192) != hipSuccess) return 1;
    for (int W : wpw)
        for (int G : grids) {
            if (G * W > 8192) continue;
            hipLaunchKernelGGL(k_where, dim3(G), dim3(64 * W), 0, 0, d);
            if (hipDeviceSynchronize() != hipSuccess) return 2;
            std::vector<uint32_t> h(2 * G * W);
            if (hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost) != hipSuccess) return 3;
            using Cu = std::tuple<uint32_t, uint32_t, uint32_t, uint32_t>;  // xcc, se, sh, cu
            std::map<Cu, std::map<uint32_t, int>> wgs_on_cu;                  // cu -> wg -> waves
            std::map<std::pair<Cu, uint32_t>, int> waves_on_simd, chains_static, chains_ranked;
            for (int g = 0; g < G; ++g) {
                std::map<uint32_t, int> per_simd;  // this workgroup's waves per SIMD
                std::vector<uint32_t> simd_of(W);
                Cu cu{};
                for (int w = 0; w < W; ++w) {
                    const uint32_t hw = h[2 * (g * W + w)], xcc = h[2 * (g * W + w) + 1] & 0xf;
                    cu = Cu{xcc, (hw >> 13) & 7, (hw >> 12) & 1, (hw >> 8) & 15};
                    simd_of[w] = (hw >> 4) & 3;
                    wgs_on_cu[cu][g]++;
                    waves_on_simd[{cu, simd_of[w]}]++;
                    if (w < W / 2) chains_static[{cu, simd_of[w]}]++;
                    per_simd[simd_of[w]]++;
                }
                // pc_role<true>: rank-major order over (rank within SIMD, SIMD)
                std::map<uint32_t, int> seen;
                std::vector<std::pair<int, uint32_t>> order;
                for (int w = 0; w < W; ++w) order.push_back({seen[simd_of[w]]++, simd_of[w]});
                std::sort(order.begin(), order.end());
                for (int i = 0; i < W / 2; ++i) chains_ranked[{cu, order[i].second}]++;
            }
            int max_wg = 0, max_waves = 0, dbl_static = 0, dbl_ranked = 0;
            for (auto& kv : wgs_on_cu) max_wg = std::max<int>(max_wg, kv.second.size());
            for (auto& kv : waves_on_simd) max_waves = std::max(max_waves, kv.second);
            for (auto& kv : chains_static) dbl_static += kv.second >= 2;
            for (auto& kv : chains_ranked) dbl_ranked += kv.second >= 2;
            std::printf("waves/wg %d  wgs %4d: CUs used %3zu, max wgs/CU %d, max waves/SIMD %d, "
                        "SIMDs with >=2 chain waves: static %d, ranked %d\n",
                        W, G, wgs_on_cu.size(), max_wg, max_waves, dbl_static, dbl_ranked);
            if (W == 8 && G == 219) {  // one workgroup's placement in full
                for (int w = 0; w < W; ++w)
                    std::printf("  wg0 wave %d: simd %u cu %u se %u xcc %u\n", w, (h[2 * w] >> 4) & 3,
                                (h[2 * w] >> 8) & 15, (h[2 * w] >> 13) & 7, h[2 * w + 1] & 0xf);
            }
        }
    (void)hipFree(d);
    return 0;
}
