// Host XXH64 throughput probe (round 4): is the commit host leg's per-thread rate bound by
// the 64-bit multiplier (scalar imul) and would AVX-512 vpmullq over several blocks at once
// lift it? Variants over 32 KiB blocks from a 256 MiB buffer (past the LLC), one thread:
//   scalar1   the library's host leg (xxh64_host.h), one block at a time
//   scalar4   four blocks' chains interleaved by hand, scalar
//   ymm1      one block, its four accumulators in one 256-bit register (vpmullq ymm)
//   ymmK      K blocks interleaved, one ymm register each (K = 2, 4, 8)
//   zmm2x     two blocks per zmm register, 2 / 4 registers (4 / 8 blocks)
// Every variant's checksums are compared with scalar1's. Not part of the library.
#include <immintrin.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../storm_amd/csrc/xxh64_host.h"

using namespace stormck::host;

static uint64_t finish_tail(uint64_t h, const unsigned char* p, size_t rem, size_t n) {
    h += n;
    const unsigned char* end = p + rem;
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

static uint64_t merge4(uint64_t a, uint64_t b, uint64_t c, uint64_t d) {
    uint64_t h = rotl(a, 1) + rotl(b, 7) + rotl(c, 12) + rotl(d, 18);
    return fold(fold(fold(fold(h, a), b), c), d);
}

// K blocks of n bytes (n >= 32), one ymm of accumulators each
template <int K>
__attribute__((target("avx512f,avx512vl,avx512dq"))) static void ymm_k(const unsigned char* const* p, size_t n,
                                                                          uint64_t* out) {
    const __m256i p1 = _mm256_set1_epi64x(static_cast<long long>(P1));
    const __m256i p2 = _mm256_set1_epi64x(static_cast<long long>(P2));
    __m256i acc[K];
    for (int k = 0; k < K; ++k)
        acc[k] = _mm256_set_epi64x(static_cast<long long>(0 - P1), 0, static_cast<long long>(P2),
                                   static_cast<long long>(P1 + P2));
    const size_t ns = n / 32;
    for (size_t s = 0; s < ns; ++s) {
#pragma GCC unroll 8
        for (int k = 0; k < K; ++k) {
            const __m256i w = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(p[k] + 32 * s));
            acc[k] = _mm256_mullo_epi64(_mm256_rol_epi64(_mm256_add_epi64(acc[k], _mm256_mullo_epi64(w, p2)), 31), p1);
        }
    }
    for (int k = 0; k < K; ++k) {
        alignas(32) uint64_t a[4];
        _mm256_store_si256(reinterpret_cast<__m256i*>(a), acc[k]);
        out[k] = finish_tail(merge4(a[0], a[1], a[2], a[3]), p[k] + 32 * ns, n - 32 * ns, n);
    }
}

// 2R blocks, two per zmm register (R registers)
template <int R>
__attribute__((target("avx512f,avx512dq"))) static void zmm2(const unsigned char* const* p, size_t n, uint64_t* out) {
    const __m512i p1 = _mm512_set1_epi64(static_cast<long long>(P1));
    const __m512i p2 = _mm512_set1_epi64(static_cast<long long>(P2));
    __m512i acc[R];
    const __m512i seed = _mm512_set_epi64(static_cast<long long>(0 - P1), 0, static_cast<long long>(P2),
                                          static_cast<long long>(P1 + P2), static_cast<long long>(0 - P1), 0,
                                          static_cast<long long>(P2), static_cast<long long>(P1 + P2));
    for (int r = 0; r < R; ++r) acc[r] = seed;
    const size_t ns = n / 32;
    for (size_t s = 0; s < ns; ++s) {
#pragma GCC unroll 4
        for (int r = 0; r < R; ++r) {
            const __m256i lo = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(p[2 * r] + 32 * s));
            const __m256i hi = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(p[2 * r + 1] + 32 * s));
            const __m512i w = _mm512_inserti64x4(_mm512_castsi256_si512(lo), hi, 1);
            acc[r] = _mm512_mullo_epi64(_mm512_rol_epi64(_mm512_add_epi64(acc[r], _mm512_mullo_epi64(w, p2)), 31), p1);
        }
    }
    for (int r = 0; r < R; ++r) {
        alignas(64) uint64_t a[8];
        _mm512_store_si512(reinterpret_cast<__m512i*>(a), acc[r]);
        for (int h = 0; h < 2; ++h)
            out[2 * r + h] = finish_tail(merge4(a[4 * h], a[4 * h + 1], a[4 * h + 2], a[4 * h + 3]),
                                         p[2 * r + h] + 32 * ns, n - 32 * ns, n);
    }
}

static void scalar4(const unsigned char* const* p, size_t n, uint64_t* out) {
    uint64_t v[4][4];
    for (int k = 0; k < 4; ++k) {
        v[k][0] = P1 + P2;
        v[k][1] = P2;
        v[k][2] = 0;
        v[k][3] = 0 - P1;
    }
    const size_t ns = n / 32;
    for (size_t s = 0; s < ns; ++s)
        for (int k = 0; k < 4; ++k)
            for (int j = 0; j < 4; ++j) v[k][j] = lane(v[k][j], le64(p[k] + 32 * s + 8 * j));
    for (int k = 0; k < 4; ++k)
        out[k] = finish_tail(merge4(v[k][0], v[k][1], v[k][2], v[k][3]), p[k] + 32 * ns, n - 32 * ns, n);
}

int main(int argc, char** argv) {
    const size_t B = 32768, N = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 8192;  // 256 MiB
    std::vector<unsigned char> buf(N * B);
    uint64_t x = 0x9E3779B97F4A7C15ULL;
    for (size_t i = 0; i < buf.size(); i += 8) {
        x ^= x << 13;
        x ^= x >> 7;
        x ^= x << 17;
        std::memcpy(&buf[i], &x, 8);
    }
    std::vector<uint64_t> want(N), got(N);
    for (size_t i = 0; i < N; ++i) want[i] = xxh64(&buf[i * B], B);
    const bool avx = __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512dq") &&
                     __builtin_cpu_supports("avx512vl");
    auto run = [&](const char* name, int group, auto fn) {
        double best = 1e30;
        for (int rep = 0; rep < 5; ++rep) {
            const auto t0 = std::chrono::steady_clock::now();
            for (size_t i = 0; i < N; i += group) {
                const unsigned char* ps[8];
                for (int k = 0; k < group; ++k) ps[k] = &buf[(i + k) * B];
                fn(ps, B, &got[i]);
            }
            best = std::min(best, std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
        }
        const bool ok = got == want;
        std::printf("%-10s %7.2f GiB/s  %s\n", name, N * B / best / (1 << 30), ok ? "ok" : "MISMATCH");
        std::fill(got.begin(), got.end(), 0);
    };
    run("scalar1", 1, [](const unsigned char* const* p, size_t n, uint64_t* o) { o[0] = xxh64(p[0], n); });
    run("scalar4", 4, scalar4);
    if (!avx) {
        std::printf("no AVX-512 (f, dq, vl): SIMD variants skipped\n");
        return 0;
    }
    run("ymm1", 1, ymm_k<1>);
    run("ymm2", 2, ymm_k<2>);
    run("ymm4", 4, ymm_k<4>);
    run("ymm8", 8, ymm_k<8>);
    run("zmm2x2", 4, zmm2<2>);
    run("zmm2x4", 8, zmm2<4>);
    return 0;
}
