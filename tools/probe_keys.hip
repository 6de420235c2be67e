// A/B probe of the f4 key-tag kernels (48-byte keys, the keystore benchmark's shape,
// /root/reference/keystore/benchmark_test.go:27-32): lane kernel, per-wave double
// buffer (k_key_tags_lds) and the ring variants, interleaved over rounds, each checked
// bit-exact against a host XXH64 on the first keys.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/probe_keys tools/probe_keys.hip
//   tools/probe_keys [Mkeys=64] [reps=5] [rounds=3]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "../storm_amd/csrc/kernels.h"

using namespace stormck;

#define CK(x)                                                                     \
    do {                                                                          \
        hipError_t e = (x);                                                       \
        if (e != hipSuccess) {                                                    \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
            exit(1);                                                              \
        }                                                                         \
    } while (0)

static uint64_t rl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
static uint64_t hround(uint64_t a, uint64_t w) { return rl(a + w * kP2, 31) * kP1; }
static uint64_t hmerge(uint64_t h, uint64_t v) { return (h ^ hround(0, v)) * kP1 + kP4; }
static uint64_t rd64(const uint8_t* p) { uint64_t v; memcpy(&v, p, 8); return v; }
static uint64_t host_xxh64(const uint8_t* p, uint64_t n) {
    uint64_t h; const uint8_t* e = p + n;
    if (n >= 32) {
        uint64_t v1 = kV1, v2 = kV2, v3 = kV3, v4 = kV4;
        for (; p + 32 <= e; p += 32) { v1 = hround(v1, rd64(p)); v2 = hround(v2, rd64(p + 8)); v3 = hround(v3, rd64(p + 16)); v4 = hround(v4, rd64(p + 24)); }
        h = rl(v1, 1) + rl(v2, 7) + rl(v3, 12) + rl(v4, 18);
        h = hmerge(h, v1); h = hmerge(h, v2); h = hmerge(h, v3); h = hmerge(h, v4);
    } else h = kP5;
    h += n;
    for (; p + 8 <= e; p += 8) h = rl(h ^ hround(0, rd64(p)), 27) * kP1 + kP4;
    if (p + 4 <= e) { uint32_t w; memcpy(&w, p, 4); h = rl(h ^ (uint64_t)w * kP1, 23) * kP2 + kP3; p += 4; }
    for (; p < e; ++p) h = rl(h ^ (uint64_t)(*p) * kP5, 11) * kP1;
    h ^= h >> 33; h *= kP2; h ^= h >> 29; h *= kP3; h ^= h >> 32;
    return h;
}

namespace stormck {
// CANDIDATE: workgroup-synchronised, persistent LDS-DMA ring for fixed-stride keys (the
// streaming checksum kernel's scheme applied to keys). A tile is WAVES x BW batches of
// 64 keys, contiguous in memory (BW * 3 KiB per wave at 48-byte keys); each wave loads
// and hashes its own batches; tile t+1 is in flight while tile t hashes; one barrier per
// tile so every tile leaves as one burst. Workgroups walk tiles blockIdx.x + k*gridDim.x.
template <int P, int BW, int WAVES, int KLEN>
__global__ __launch_bounds__(64 * WAVES) void k_key_tags_wg(const uint8_t* __restrict__ keys, uint64_t batches,
                                                            uint64_t* __restrict__ out) {
    constexpr uint32_t kStride = 16 * P, kRegion = 64 * kStride;   // one batch
    constexpr uint32_t kWaveBytes = BW * kRegion, kTile = WAVES * kWaveBytes;
    __shared__ __attribute__((aligned(16))) uint8_t lds[2 * kTile];
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint64_t bpt = static_cast<uint64_t>(WAVES) * BW;        // batches per tile
    const uint64_t ntile = batches / bpt;                          // whole tiles only (host handles the rest)
    const uint64_t G = gridDim.x;
    if (blockIdx.x >= ntile) return;
    const uint64_t steps = (ntile - blockIdx.x + G - 1) / G;
    auto issue = [&](uint64_t tile, uint32_t slot) {
        const uint8_t* s_ = keys + (tile * bpt + static_cast<uint64_t>(wave) * BW) * kRegion + lane * 16;
        uint8_t* d_ = lds + slot * kTile + wave * kWaveBytes;
#pragma unroll
        for (int p_ = 0; p_ < static_cast<int>(BW * P); ++p_)
            __builtin_amdgcn_global_load_lds(s_ + p_ * 1024, d_ + p_ * 1024, 16, 0, 2);
    };
    issue(blockIdx.x, 0);
    for (uint64_t u = 0; u < steps; ++u) {
        wait_vmcnt<0>();
        __builtin_amdgcn_s_barrier();
        const uint64_t tile = blockIdx.x + u * G;
        if (u + 1 < steps) issue(tile + G, (u + 1) & 1);
#pragma unroll
        for (int bb = 0; bb < BW; ++bb) {
            const uint8_t* k = lds + (u & 1) * kTile + wave * kWaveBytes + bb * kRegion + lane * kStride;
            uint64_t v1 = kV1, v2 = kV2, v3 = kV3, v4 = kV4;
#pragma unroll
            for (uint32_t s = 0; s < KLEN / 32; ++s) {
                const u64x2 x = *reinterpret_cast<const u64x2*>(k + 32 * s);
                const u64x2 y = *reinterpret_cast<const u64x2*>(k + 32 * s + 16);
                v1 = round(v1, x.x);
                v2 = round(v2, x.y);
                v3 = round(v3, y.x);
                v4 = round(v4, y.y);
            }
            const uint64_t h = finish_lds16(KLEN >= 32 ? converge(v1, v2, v3, v4) : kP5, KLEN, k + 32 * (KLEN / 32),
                                            KLEN & 31);
            out[(tile * bpt + static_cast<uint64_t>(wave) * BW + bb) * 64 + lane] = h;
        }
    }
}
__global__ __launch_bounds__(256) void k_read_nt(const u64x2* __restrict__ p, uint64_t n16, uint64_t* out) {
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
// The traffic of the key-tag pass without its hash: each lane reads one 48-byte key
// (3 x 16 B, non-temporal) and writes one 8-byte word, grid-stride. Its rate is the
// ceiling of a read-48 / write-8 stream on this HBM, the bound f4 is measured against.
template <bool NTS>
__global__ __launch_bounds__(256) void k_copy_fold(const u64x2* __restrict__ p, uint64_t n, uint64_t* __restrict__ out) {
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
        const u64x2 a = ldg<true>(p + 3 * i), b = ldg<true>(p + 3 * i + 1), c = ldg<true>(p + 3 * i + 2);
        const u64x2 f = a ^ b ^ c;
        if (NTS) __builtin_nontemporal_store(f.x ^ f.y, out + i);
        else out[i] = f.x ^ f.y;
    }
}
// The same traffic fully coalesced: a wave reads a batch's 3 KiB as 3 contiguous
// 1 KiB loads (16 B per lane) and writes 512 B (8 B per lane), grid-stride over
// batches, U batches per wave-iteration in flight. No hash; the values are not tags.
template <int U>
__global__ __launch_bounds__(256) void k_stream_rw(const u64x2* __restrict__ p, uint64_t batches, uint64_t* __restrict__ out) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t waves = (uint64_t)gridDim.x * 4;
    uint64_t w = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    for (; w + (U - 1) * waves < batches; w += U * waves) {
        u64x2 v[U][3];
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int k = 0; k < 3; ++k) v[u][k] = ldg<true>(p + (w + u * waves) * 192 + k * 64 + lane);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const u64x2 f = v[u][0] ^ v[u][1] ^ v[u][2];
            __builtin_nontemporal_store(f.x ^ f.y, out + (w + u * waves) * 64 + lane);
        }
    }
    for (; w < batches; w += waves) {
        const u64x2 f = ldg<true>(p + w * 192 + lane) ^ ldg<true>(p + w * 192 + 64 + lane) ^ ldg<true>(p + w * 192 + 128 + lane);
        __builtin_nontemporal_store(f.x ^ f.y, out + w * 64 + lane);
    }
}
}  // namespace stormck

struct Timer {
    hipEvent_t a, b;
    Timer() { CK(hipEventCreate(&a)); CK(hipEventCreate(&b)); }
    void start() { CK(hipEventRecord(a, 0)); }
    float stop() { CK(hipEventRecord(b, 0)); CK(hipEventSynchronize(b)); float ms; CK(hipEventElapsedTime(&ms, a, b)); return ms; }
};

int main(int argc, char** argv) {
    const uint64_t n = (uint64_t)((argc > 1 ? atof(argv[1]) : 64.0) * (1 << 20)) / 64 * 64;
    const int reps = argc > 2 ? atoi(argv[2]) : 5, rounds = argc > 3 ? atoi(argv[3]) : 3;
    constexpr uint32_t klen = 48;
    uint8_t* keys; CK(hipMalloc(&keys, n * klen));
    uint64_t* out; CK(hipMalloc(&out, n * 8));
    hipLaunchKernelGGL(k_fill_synthetic, dim3(8192), dim3(256), 0, 0, keys, 48ULL * 1024, n * klen / (48 * 1024), 0ULL, 0x53544f524dULL);
    CK(hipDeviceSynchronize());
    const uint64_t K = std::min<uint64_t>(n, 1 << 16);
    std::vector<uint8_t> hk(K * klen);
    CK(hipMemcpy(hk.data(), keys, K * klen, hipMemcpyDeviceToHost));
    std::vector<uint64_t> ref(K), got(K);
    for (uint64_t i = 0; i < K; ++i) ref[i] = host_xxh64(hk.data() + i * klen, klen);
    // also check the LAST keys (grid tail)
    std::vector<uint8_t> hk2(K * klen);
    CK(hipMemcpy(hk2.data(), keys + (n - K) * klen, K * klen, hipMemcpyDeviceToHost));
    std::vector<uint64_t> ref2(K), got2(K);
    for (uint64_t i = 0; i < K; ++i) ref2[i] = host_xxh64(hk2.data() + i * klen, klen);

    const uint64_t batches = n / 64;
    struct V { std::string name; std::function<void()> f; };
    std::vector<V> vs;
    vs.push_back({"lane k_key_tags", [&] {
        hipLaunchKernelGGL((k_key_tags<false, false>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, keys, (uint64_t)klen,
                           nullptr, nullptr, klen, n, out); }});
    vs.push_back({"lds double buffer pw8", [&] {
        const uint64_t waves = (batches + 7) / 8;
        hipLaunchKernelGGL(k_key_tags_lds<2>, dim3((unsigned)((waves + 3) / 4)), dim3(256), 4 * 2 * 64 * klen, 0, keys, klen, klen,
                           batches, 8u, out); }});
#define RV(RING, PW)                                                                                       \
    vs.push_back({"ring R=" #RING " PW=" #PW, [&] {                                                        \
        const uint64_t waves = (batches + PW - 1) / PW;                                                    \
        hipLaunchKernelGGL((k_key_tags_ring<2, 3, RING, PW>), dim3((unsigned)((waves + 3) / 4)), dim3(256), \
                           4 * RING * 64 * klen, 0, keys, klen, batches, out); }})
    RV(4, 8);
#define SMV(SM, NAME)                                                                                        \
    vs.push_back({NAME, [&] {                                                                                \
        const uint64_t waves = (batches + 7) / 8;                                                            \
        hipLaunchKernelGGL((k_key_tags_ring<2, 3, 4, 8, 48, SM>), dim3((unsigned)((waves + 3) / 4)), dim3(256), \
                           4 * 4 * 64 * klen, 0, keys, klen, batches, out); }})
    SMV(0, "ring klen=48 (shipped)");
    SMV(1, "ring klen=48, nt stores");
    SMV(2, "ring klen=48, no stores");
    SMV(3, "ring klen=48, LDS-staged x4");
    SMV(4, "ring klen=48, LDS-staged x4 nt");
    vs.push_back({"grid-stride read nt, no hash", [&] {
        hipLaunchKernelGGL(k_read_nt, dim3(16384), dim3(256), 0, 0, (const u64x2*)keys, n * klen / 16, out); }});
    vs.push_back({"read 48 / write 8, no hash", [&] {
        hipLaunchKernelGGL(k_copy_fold<false>, dim3(16384), dim3(256), 0, 0, (const u64x2*)keys, n, out); }});
    vs.push_back({"read 48 / write 8 nt, no hash", [&] {
        hipLaunchKernelGGL(k_copy_fold<true>, dim3(16384), dim3(256), 0, 0, (const u64x2*)keys, n, out); }});
    vs.push_back({"r48/w8 nt, no hash, 64K WGs", [&] {
        hipLaunchKernelGGL(k_copy_fold<true>, dim3(65536), dim3(256), 0, 0, (const u64x2*)keys, n, out); }});
    vs.push_back({"coalesced r3K/w512 U=1, no hash", [&] {
        hipLaunchKernelGGL(k_stream_rw<1>, dim3(16384), dim3(256), 0, 0, (const u64x2*)keys, batches, out); }});
    vs.push_back({"coalesced r3K/w512 U=2, no hash", [&] {
        hipLaunchKernelGGL(k_stream_rw<2>, dim3(8192), dim3(256), 0, 0, (const u64x2*)keys, batches, out); }});
    vs.push_back({"coalesced r3K/w512 U=4, no hash", [&] {
        hipLaunchKernelGGL(k_stream_rw<4>, dim3(4096), dim3(256), 0, 0, (const u64x2*)keys, batches, out); }});
    vs.push_back({"coalesced r3K/w512 U=4, 1K WGs", [&] {
        hipLaunchKernelGGL(k_stream_rw<4>, dim3(1024), dim3(256), 0, 0, (const u64x2*)keys, batches, out); }});
    hipDeviceProp_t prop; CK(hipGetDeviceProperties(&prop, 0));
    const unsigned cus = (unsigned)prop.multiProcessorCount;
#define WG(BW, MULT)                                                                                        \
    vs.push_back({"wg ring BW=" #BW " grid=" #MULT "xCU", [&] {                                            \
        hipLaunchKernelGGL((k_key_tags_wg<3, BW, 8, 48>), dim3(cus * MULT), dim3(512), 0, 0, keys, batches, out); }})
    WG(1, 1); WG(2, 1); WG(3, 1); WG(1, 2); WG(1, 3);
    std::vector<std::vector<double>> gks(vs.size());
    for (int r = 0; r < rounds; ++r)
        for (size_t v = 0; v < vs.size(); ++v) {
            CK(hipMemset(out, 0, n * 8));
            vs[v].f();
            CK(hipDeviceSynchronize());
            if (r == 0) {
                CK(hipMemcpy(got.data(), out, K * 8, hipMemcpyDeviceToHost));
                CK(hipMemcpy(got2.data(), out + (n - K), K * 8, hipMemcpyDeviceToHost));
                uint64_t bad = 0;
                for (uint64_t i = 0; i < K; ++i) bad += (got[i] != ref[i]) + (got2[i] != ref2[i]);
                if (bad && vs[v].name.find("no ") == std::string::npos)
                    printf("  !! %s: %llu mismatches\n", vs[v].name.c_str(), (unsigned long long)bad);
            }
            Timer t;
            for (int k = 0; k < reps; ++k) { t.start(); vs[v].f(); gks[v].push_back(n / (t.stop() * 1e-3) / 1e9); }
        }
    printf("keys %llu x %u B (%.2f GB + %.2f GB out)\n", (unsigned long long)n, klen, n * klen / 1e9, n * 8 / 1e9);
    printf("GB/s counts %u B per key (key read + tag written); the read-only variants move %u B\n", klen + 8, klen);
    for (size_t v = 0; v < vs.size(); ++v) {
        auto g = gks[v]; std::sort(g.begin(), g.end());
        const double med = g[g.size() / 2];
        printf("%-26s max %7.2f  median %7.2f Gkeys/s  = %7.1f GB/s (%.3f of 8 TB/s)\n", vs[v].name.c_str(), g.back(), med,
               med * (klen + 8), med * (klen + 8) / 8000.0);
    }
    printf("done\n");
    return 0;
}
