// XXH64 (seed 0) on one host core: the latency leg of a single blocks.Checksum call.
//
// storm calls blocks.Checksum one block at a time from its commit callbacks and cold
// reads (cache/trace.go:282,307, cache/cache.go:73,160, persistence/init.go:44). One
// XXH64 is four serial accumulator chains, so one buffer can use at most 4 GPU lanes:
// a single call costs a launch, a sync and a ~1.3 GB/s chain on the device (35 us for
// 32 KiB, DESIGN_LOG.md §5), against ~1.3 us on one host core. Single calls therefore hash
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
#if defined(__x86_64__) && !defined(__HIP_DEVICE_COMPILE__)
#define STORMCK_HOST_X4 1
#include <immintrin.h>
#endif

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

// Several buffers at once (the f1 host leg hashes a height's blocks this way). One XXH64
// is four serial chains whose rounds each cost two 64-bit multiplies; a scalar core runs
// them one imul at a time. With AVX-512 (F, VL, DQ) one 256-bit vpmullq does a round of
// all four accumulators of a buffer, and four buffers' chains interleave: the rounds of
// the stripes every buffer has run vectorised, each buffer then finishes its own stripes,
// merge and tail on the scalar path. Results are bit-identical to xxh64().
inline uint64_t xxh64_finish(uint64_t h, const unsigned char* p, size_t rem, size_t n) {
    const unsigned char* const end = p + rem;
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

#ifdef STORMCK_HOST_X4
__attribute__((target("avx512f,avx512vl,avx512dq"))) inline void xxh64_x4_avx512(const unsigned char* const* p,
                                                                                    const size_t* n, uint64_t* out) {
    const __m256i p1 = _mm256_set1_epi64x(static_cast<long long>(P1));
    const __m256i p2 = _mm256_set1_epi64x(static_cast<long long>(P2));
    const __m256i seed = _mm256_set_epi64x(static_cast<long long>(0 - P1), 0, static_cast<long long>(P2),
                                           static_cast<long long>(P1 + P2));
    __m256i acc[4] = {seed, seed, seed, seed};
    size_t common = SIZE_MAX;
    for (int k = 0; k < 4; ++k) common = n[k] < common ? n[k] : common;
    common /= 32;
    for (size_t s = 0; s < common; ++s) {
        for (int k = 0; k < 4; ++k) {
            const __m256i w = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(p[k] + 32 * s));
            acc[k] = _mm256_mullo_epi64(_mm256_rol_epi64(_mm256_add_epi64(acc[k], _mm256_mullo_epi64(w, p2)), 31), p1);
        }
    }
    for (int k = 0; k < 4; ++k) {
        if (n[k] < 32) {
            out[k] = xxh64_finish(P5, p[k], n[k], n[k]);
            continue;
        }
        alignas(32) uint64_t a[4];
        _mm256_store_si256(reinterpret_cast<__m256i*>(a), acc[k]);
        const size_t ns = n[k] / 32;
        for (size_t s = common; s < ns; ++s) {
            const unsigned char* q = p[k] + 32 * s;
            a[0] = lane(a[0], le64(q));
            a[1] = lane(a[1], le64(q + 8));
            a[2] = lane(a[2], le64(q + 16));
            a[3] = lane(a[3], le64(q + 24));
        }
        uint64_t h = rotl(a[0], 1) + rotl(a[1], 7) + rotl(a[2], 12) + rotl(a[3], 18);
        h = fold(fold(fold(fold(h, a[0]), a[1]), a[2]), a[3]);
        out[k] = xxh64_finish(h, p[k] + 32 * ns, n[k] - 32 * ns, n[k]);
    }
}
#endif

// Whether xxh64_x4_avx512 can run on this CPU (checked once).
inline bool has_x4() {
#ifdef STORMCK_HOST_X4
    static const bool ok = __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512vl") &&
                           __builtin_cpu_supports("avx512dq");
    return ok;
#else
    return false;
#endif
}

// out[k] = xxh64(p[k], n[k]) for k < 4.
inline void xxh64_x4(const unsigned char* const* p, const size_t* n, uint64_t* out) {
#ifdef STORMCK_HOST_X4
    if (has_x4()) {
        xxh64_x4_avx512(p, n, out);
        return;
    }
#endif
    for (int k = 0; k < 4; ++k) out[k] = xxh64(p[k], n[k]);
}

}  // namespace stormck::host
