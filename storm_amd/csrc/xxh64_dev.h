// XXH64 (seed 0) building blocks for gfx950 device code.
//
// The hashed function is storm's blocks.Checksum = xxhash.Sum64
// (/root/reference/blocks/checksum.go:15-17; github.com/cespare/xxhash/v2 v2.2.0,
// /root/reference/go.mod:6). Algorithm: SURVEY.md Appendix A.
//
// CDNA4 notes:
//  - a 64x64->64 multiply by a constant lowers to v_mad_u64_u32 + 2 v_mul_lo_u32 +
//    v_add3_u32; acc + w*P2 folds the add into the v_mad_u64_u32 accumulator.
//  - 64-bit rotates are two v_alignbit_b32 (full rate) instead of the
//    v_lshlrev_b64 + v_lshrrev + v_or sequence the compiler picks for (x<<r)|(x>>64-r).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace stormck {

constexpr uint64_t kP1 = 0x9E3779B185EBCA87ULL;
constexpr uint64_t kP2 = 0xC2B2AE3D27D4EB4FULL;
constexpr uint64_t kP3 = 0x165667B19E3779F9ULL;
constexpr uint64_t kP4 = 0x85EBCA77C2B2AE63ULL;
constexpr uint64_t kP5 = 0x27D4EB2F165667C5ULL;

// Seeds of the four stripe accumulators for seed 0.
constexpr uint64_t kV1 = kP1 + kP2;
constexpr uint64_t kV2 = kP2;
constexpr uint64_t kV3 = 0;
constexpr uint64_t kV4 = 0ULL - kP1;

// rotl for 0 < R < 32 with two alignbit ops.
template <int R>
__device__ __forceinline__ uint64_t rotl(uint64_t x) {
    static_assert(R > 0 && R < 32, "rotl via alignbit covers 1..31");
    const uint32_t lo = static_cast<uint32_t>(x);
    const uint32_t hi = static_cast<uint32_t>(x >> 32);
    const uint32_t nhi = __builtin_amdgcn_alignbit(hi, lo, 32 - R);
    const uint32_t nlo = __builtin_amdgcn_alignbit(lo, hi, 32 - R);
    return (static_cast<uint64_t>(nhi) << 32) | nlo;
}

__device__ __forceinline__ uint64_t round(uint64_t acc, uint64_t w) {
    acc += w * kP2;
    acc = rotl<31>(acc);
    return acc * kP1;
}

// round() on a word already multiplied by P2 (pw = w * P2). The latency kernels stage a
// block in LDS and have all 256 threads premultiply its stripe words there, so the one
// quad that walks the serial chain issues the add, the rotate and the P1 multiply only:
// a lone wave is issue-bound, and the P2 multiply is 4 of its ~11 instructions a round.
__device__ __forceinline__ uint64_t round_pm(uint64_t acc, uint64_t pw) {
    acc += pw;
    acc = rotl<31>(acc);
    return acc * kP1;
}

__device__ __forceinline__ uint64_t merge(uint64_t h, uint64_t v) {
    h ^= round(0, v);
    return h * kP1 + kP4;
}

// h from the four stripe accumulators (n >= 32 path).
__device__ __forceinline__ uint64_t converge(uint64_t v1, uint64_t v2, uint64_t v3, uint64_t v4) {
    uint64_t h = rotl<1>(v1) + rotl<7>(v2) + rotl<12>(v3) + rotl<18>(v4);
    h = merge(h, v1);
    h = merge(h, v2);
    h = merge(h, v3);
    h = merge(h, v4);
    return h;
}

__device__ __forceinline__ uint64_t avalanche(uint64_t h) {
    h ^= h >> 33;
    h *= kP2;
    h ^= h >> 29;
    h *= kP3;
    h ^= h >> 32;
    return h;
}

__device__ __forceinline__ uint64_t ld64_unaligned(const uint8_t* p) {
    uint64_t v = 0;
#pragma unroll
    for (int i = 7; i >= 0; --i) v = (v << 8) | p[i];
    return v;
}
__device__ __forceinline__ uint32_t ld32_unaligned(const uint8_t* p) {
    return static_cast<uint32_t>(p[0]) | (static_cast<uint32_t>(p[1]) << 8) |
           (static_cast<uint32_t>(p[2]) << 16) | (static_cast<uint32_t>(p[3]) << 24);
}

// Tail (< 32 bytes at p, `rem` of them) + avalanche, given h after the stripe
// phase (or P5 for n < 32) and the total length n. Byte loads: the tail is at most
// 31 bytes per block, so its cost is negligible next to the stripe loop.
__device__ __forceinline__ uint64_t finish(uint64_t h, uint64_t n, const uint8_t* p, uint32_t rem) {
    h += n;
    while (rem >= 8) {
        h ^= round(0, ld64_unaligned(p));
        h = rotl<27>(h) * kP1 + kP4;
        p += 8;
        rem -= 8;
    }
    if (rem >= 4) {
        h ^= static_cast<uint64_t>(ld32_unaligned(p)) * kP1;
        h = rotl<23>(h) * kP2 + kP3;
        p += 4;
        rem -= 4;
    }
    while (rem > 0) {
        h ^= static_cast<uint64_t>(*p) * kP5;
        h = rotl<11>(h) * kP1;
        ++p;
        --rem;
    }
    return avalanche(h);
}

// splitmix64: the synthetic-block generator of SURVEY.md §8d.
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

}  // namespace stormck
