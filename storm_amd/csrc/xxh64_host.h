// XXH64 (seed 0) on one host core: the latency leg of a single blocks.Checksum call.
//
// storm calls blocks.Checksum one block at a time from its commit callbacks and cold
// reads (cache/trace.go:282,307, cache/cache.go:73,160, persistence/init.go:44). One
// XXH64 is four serial accumulator chains, so one buffer can use at most 4 GPU lanes:
// a single call costs a launch, a sync and a ~1.3 GB/s chain on the device (35 us for
// 32 KiB), against ~1.3 us on one host core. Single calls therefore hash
// here ("single calls stay on the C++ CPU path"); every batch, where
// the blocks are independent, goes to the gfx950 kernels. This is not a fallback for a
// missing device: batched entry points still fail with STORMCK_ENODEV without one.
//
// Algorithm: SURVEY.md Appendix A (= github.com/cespare/xxhash/v2 v2.2.0 Sum64,
// /root/reference/go.mod:6, called at /root/reference/blocks/checksum.go:16).
#pragma once
#include <stddef.h>
#include <stdint.h>
#include <string.h>

namespace stormck::host {

inline constexpr uint64_t P1 = 0x9E3779B185EBCA87ULL;
inline constexpr uint64_t P2 = 0xC2B2AE3D27D4EB4FULL;
inline constexpr uint64_t P3 = 0x165667B19E3779F9ULL;
inline constexpr uint64_t P4 = 0x85EBCA77C2B2AE63ULL;
inline constexpr uint64_t P5 = 0x27D4EB2F165667C5ULL;

inline uint64_t rotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }

// little-endian loads (x86-64 / aarch64 hosts are little-endian, as storm's amd64 is)
inline uint64_t le64(const unsigned char* p) {
    uint64_t v;
    memcpy(&v, p, 8);
    return v;
}
inline uint32_t le32(const unsigned char* p) {
    uint32_t v;
    memcpy(&v, p, 4);
    return v;
}

inline uint64_t lane(uint64_t acc, uint64_t w) { return rotl(acc + w * P2, 31) * P1; }

inline uint64_t fold(uint64_t h, uint64_t acc) { return (h ^ lane(0, acc)) * P1 + P4; }

inline uint64_t xxh64(const void* data, size_t n) {
    const unsigned char* p = static_cast<const unsigned char*>(data);
    const unsigned char* const end = p + n;
    uint64_t h;
    if (n >= 32) {
        uint64_t a = P1 + P2, b = P2, c = 0, d = 0 - P1;
        // two stripes per iteration: the four chains stay independent, the loop
        // overhead halves
        for (; end - p >= 64; p += 64) {
            a = lane(a, le64(p));
            b = lane(b, le64(p + 8));
            c = lane(c, le64(p + 16));
            d = lane(d, le64(p + 24));
            a = lane(a, le64(p + 32));
            b = lane(b, le64(p + 40));
            c = lane(c, le64(p + 48));
            d = lane(d, le64(p + 56));
        }
        if (end - p >= 32) {
            a = lane(a, le64(p));
            b = lane(b, le64(p + 8));
            c = lane(c, le64(p + 16));
            d = lane(d, le64(p + 24));
            p += 32;
        }
        h = rotl(a, 1) + rotl(b, 7) + rotl(c, 12) + rotl(d, 18);
        h = fold(fold(fold(fold(h, a), b), c), d);
    } else {
        h = P5;
    }
    h += static_cast<uint64_t>(n);
    for (; end - p >= 8; p += 8) h = rotl(h ^ lane(0, le64(p)), 27) * P1 + P4;
    if (end - p >= 4) {
        h = rotl(h ^ (static_cast<uint64_t>(le32(p)) * P1), 23) * P2 + P3;
        p += 4;
    }
    for (; p < end; ++p) h = rotl(h ^ (*p * P5), 11) * P1;
    h ^= h >> 33;
    h *= P2;
    h ^= h >> 29;
    h *= P3;
    return h ^ (h >> 32);
}

}  // namespace stormck::host
