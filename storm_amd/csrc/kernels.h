// gfx950 kernels of the storm block-checksum engine.
//
// Hot path: XXH64(seed 0) of every block of a batch = storm's blocks.Checksum /
// blocks.BlockChecksum (/root/reference/blocks/checksum.go:10-17) applied to many
// independent blocks at once.
//
// Why not "one wavefront per block": XXH64 carries four serial accumulator
// recurrences over a block's stripes (acc = rotl(acc + w*P2, 31) * P1 per 8-byte word),
// and the recurrence is not associative, so at most FOUR lanes can work on one block.
// Mapping: a quad of lanes per block (lane j owns accumulator j and reads word j of
// each 32-byte stripe), 16 blocks per wave64; the 4 accumulators meet through DPP quad
// permutes for the merge; lane 0 of the quad does tail + avalanche. Kernels:
//   * k_xxh64_glds   : uniform-length batches, stripes staged HBM -> LDS by LDS-DMA
//   * k_xxh64_glds_skew: the same for large batches, persistent, waves' streams 4 KiB apart
//   * k_xxh64_quad   : any shape (per-block lengths, offsets, alignment), register loads
//   * k_xxh64_single : one slice <= 64 KiB read from pinned host memory (latency path)
//   * k_xxh64_wide   : small batches, one workgroup per block staged whole into LDS
//   * k_commit_level*: f1 commit levels; k_pointer_level / _node: Merkle nodes
//   * k_key_tags*    : f4, one lane per short key
// (A lane-per-block mapping was measured and rejected: 0.59-0.66 of HBM peak,
// profiles/r01_probe*.txt; DESIGN_LOG.md §4. Its kernel left the library in round 2.)
// The per-block sizes (stride / explicit offsets) and lengths (uniform / per-block)
// cover storm's block types: 72, 28808, 30000, 31808, 32768 bytes.
#pragma once
#include "../../include/stormck.h"
#include "xxh64_dev.h"

namespace stormck {

typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));

#ifdef STORMCK_DEBUG_QUAD
// Debug build (tools/libstormck_debug.so): quad merges that ran with part of their quad
// inactive. update_dpp with bound_ctrl = false returns `old` (0) for a source lane that
// is not in exec, so such a merge silently reads zeros (DESIGN_LOG.md §4, "Quad merges").
__device__ unsigned long long g_partial_quads;
#endif

// Broadcast lane k of each quad (DPP quad_perm) for a 64-bit value. Every lane of the
// quad must be active: a source lane outside exec reads as 0 (bound_ctrl = false, old =
// 0). The debug build counts every merge that breaks this (g_partial_quads).
template <int K>
__device__ __forceinline__ uint64_t quad_bcast(uint64_t v) {
#ifdef STORMCK_DEBUG_QUAD
    {
        const uint64_t exec = __builtin_amdgcn_read_exec();
        const uint32_t quad = __lane_id() & ~3u;
        if (((exec >> quad) & 0xFull) != 0xFull) atomicAdd(&g_partial_quads, 1ull);
    }
#endif
    constexpr int ctrl = K | (K << 2) | (K << 4) | (K << 6);
    const int lo = __builtin_amdgcn_update_dpp(0, static_cast<int>(static_cast<uint32_t>(v)), ctrl, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, static_cast<int>(static_cast<uint32_t>(v >> 32)), ctrl, 0xF, 0xF, false);
    return (static_cast<uint64_t>(static_cast<uint32_t>(hi)) << 32) | static_cast<uint32_t>(lo);
}

__device__ __forceinline__ uint64_t acc_seed(uint32_t j) {
    return j == 0 ? kV1 : (j == 1 ? kV2 : (j == 2 ? kV3 : kV4));
}

// Streaming load; NT selects the non-temporal cache policy (data is read once).
template <bool NT, typename T>
__device__ __forceinline__ T ldg(const T* p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}

// s_waitcnt vmcnt(N) only (expcnt / lgkmcnt left at their "don't wait" maxima).
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
    static_assert(N >= 0 && N < 64, "vmcnt range");
#if defined(__HIP_DEVICE_COMPILE__)
    constexpr int imm = (N & 0xF) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8);
    __builtin_amdgcn_s_waitcnt(imm);
#endif
}

// Wait for this wave's outstanding LDS reads (lgkmcnt(0)), vmcnt/expcnt untouched.
__device__ __forceinline__ void wait_lgkm0() {
#if defined(__HIP_DEVICE_COMPILE__)
    __builtin_amdgcn_s_waitcnt(0xF | (0x3 << 14) | (0x7 << 4));
#endif
}

// Stripe loop of one accumulator over nst stripes, 8-byte-aligned source.
// p points at word j of stripe 0; word j of stripe s is p[4*s].
// Software-pipelined in groups of U loads: group g+1 is in flight while group g hashes.
// PM: the words are premultiplied by P2 (round_pm).
template <int U, bool NT = false, bool PM = false>
__device__ __forceinline__ uint64_t quad_stripes_aligned(const uint64_t* __restrict__ p, uint32_t nst, uint64_t acc) {
    auto rnd = [](uint64_t a, uint64_t w) { return PM ? round_pm(a, w) : round(a, w); };
    const uint32_t ngroups = nst / U;
    uint32_t s = 0;
    if (ngroups > 0) {
        uint64_t wa[U], wb[U];
#pragma unroll
        for (int u = 0; u < U; ++u) wa[u] = ldg<NT>(p + 4 * u);
        uint32_t g = 1;
        for (; g + 1 < ngroups; g += 2) {
            const uint64_t* q = p + 4 * U * g;
#pragma unroll
            for (int u = 0; u < U; ++u) wb[u] = ldg<NT>(q + 4 * u);
#pragma unroll
            for (int u = 0; u < U; ++u) acc = rnd(acc, wa[u]);
            q += 4 * U;
#pragma unroll
            for (int u = 0; u < U; ++u) wa[u] = ldg<NT>(q + 4 * u);
#pragma unroll
            for (int u = 0; u < U; ++u) acc = rnd(acc, wb[u]);
        }
        if (g < ngroups) {
            const uint64_t* q = p + 4 * U * g;
#pragma unroll
            for (int u = 0; u < U; ++u) wb[u] = ldg<NT>(q + 4 * u);
#pragma unroll
            for (int u = 0; u < U; ++u) acc = rnd(acc, wa[u]);
#pragma unroll
            for (int u = 0; u < U; ++u) acc = rnd(acc, wb[u]);
        } else {
#pragma unroll
            for (int u = 0; u < U; ++u) acc = rnd(acc, wa[u]);
        }
        s = ngroups * U;
    }
    for (; s < nst; ++s) acc = rnd(acc, p[4 * s]);
    return acc;
}

// quad_stripes_aligned with D groups of U loads in flight (D - 1 ahead of the one being
// hashed), rotated through registers. Loads of groups past the last are clamped to it, so
// no load sits under a branch; the last D - 1 groups hash from registers.
template <int U, int D>
__device__ __forceinline__ uint64_t quad_stripes_deep(const uint64_t* __restrict__ p, uint32_t nst, uint64_t acc) {
    static_assert(D >= 2, "at least one group ahead");
    // the scheduler would interleave the groups' loads, and the counted vmcnt wait for
    // one group would then drain the others: sched barriers keep each group's loads
    // together and in order
    auto fence = []() __attribute__((always_inline)) {
#if defined(__HIP_DEVICE_COMPILE__)
        __builtin_amdgcn_sched_barrier(0);
#endif
    };
    const uint32_t G = nst / U;
    if (G > 0) {
        uint64_t w[D][U];
        const uint32_t last = G - 1;
#pragma unroll
        for (int d = 0; d < D - 1; ++d) {
            const uint64_t* q = p + 4 * U * min(static_cast<uint32_t>(d), last);
#pragma unroll
            for (int u = 0; u < U; ++u) w[d][u] = q[4 * u];
            fence();
        }
        uint32_t g = 0;
        for (; g + D <= G; g += D) {
#pragma unroll
            for (int d = 0; d < D; ++d) {
                const uint64_t* q = p + 4 * U * min(g + d + D - 1, last);
#pragma unroll
                for (int u = 0; u < U; ++u) w[(d + D - 1) % D][u] = q[4 * u];
                fence();
#pragma unroll
                for (int u = 0; u < U; ++u) acc = round(acc, w[d][u]);
                fence();
            }
        }
#pragma unroll
        for (int d = 0; d < D - 1; ++d)
            if (static_cast<uint32_t>(d) < G - g) {
#pragma unroll
                for (int u = 0; u < U; ++u) acc = round(acc, w[d][u]);
            }
    }
    for (uint32_t s = G * U; s < nst; ++s) acc = round(acc, p[4 * s]);
    return acc;
}

// Byte-granular stripe loop for blocks whose start is not 8-byte aligned.
__device__ __forceinline__ uint64_t quad_stripes_unaligned(const uint8_t* p, uint32_t nst, uint64_t acc) {
    for (uint32_t s = 0; s < nst; ++s) acc = round(acc, ld64_unaligned(p + 32 * s));
    return acc;
}

// Tail + avalanche with word loads when the tail start is 8-byte aligned.
__device__ __forceinline__ uint64_t finish_fast(uint64_t h, uint64_t n, const uint8_t* p, uint32_t rem) {
    if ((reinterpret_cast<uintptr_t>(p) & 7) != 0) return finish(h, n, p, rem);
    h += n;
    const uint64_t* w = reinterpret_cast<const uint64_t*>(p);
    while (rem >= 8) {
        h ^= round(0, *w++);
        h = rotl<27>(h) * kP1 + kP4;
        rem -= 8;
    }
    const uint8_t* b = reinterpret_cast<const uint8_t*>(w);
    if (rem >= 4) {
        h ^= static_cast<uint64_t>(*reinterpret_cast<const uint32_t*>(b)) * kP1;
        h = rotl<23>(h) * kP2 + kP3;
        b += 4;
        rem -= 4;
    }
    while (rem > 0) {
        h ^= static_cast<uint64_t>(*b) * kP5;
        h = rotl<11>(h) * kP1;
        ++b;
        --rem;
    }
    return avalanche(h);
}

// Tail + avalanche for a 16-byte-aligned tail in LDS, read with ds_read_b128 only
// (at most roundup16(rem) bytes, so never past a 16-byte-padded key). The compiler
// guards narrower LDS reads behind in-flight LDS-DMA with a full vmcnt(0) wait, which
// would drain a key kernel's whole prefetch ring at every key's tail.
// Tail + avalanche of the rem < 32 tail bytes held little-endian in w[0..3].
__device__ __forceinline__ uint64_t finish_regs(uint64_t h, uint64_t n, const uint64_t (&w)[4], uint32_t rem) {
    h += n;
#pragma unroll
    for (int q = 0; q < 3; ++q) {
        if (rem >= 8u * (q + 1)) {
            h ^= round(0, w[q]);
            h = rotl<27>(h) * kP1 + kP4;
        }
    }
    const uint32_t nw = rem >> 3;
    uint64_t x = nw == 0 ? w[0] : (nw == 1 ? w[1] : (nw == 2 ? w[2] : w[3]));
    uint32_t r = rem & 7;
    if (r >= 4) {
        h ^= (x & 0xffffffffULL) * kP1;
        h = rotl<23>(h) * kP2 + kP3;
        x >>= 32;
        r -= 4;
    }
    for (; r > 0; --r) {
        h ^= (x & 0xff) * kP5;
        h = rotl<11>(h) * kP1;
        x >>= 8;
    }
    return avalanche(h);
}

__device__ __forceinline__ uint64_t finish_lds16(uint64_t h, uint64_t n, const uint8_t* p, uint32_t rem) {
    u64x2 a = {0, 0}, b = {0, 0};
    if (rem > 0) a = *reinterpret_cast<const u64x2*>(p);
    if (rem > 16) b = *reinterpret_cast<const u64x2*>(p + 16);
    const uint64_t w[4] = {a.x, a.y, b.x, b.y};
    return finish_regs(h, n, w, rem);
}

// ---------------------------------------------------------------------------
// Quad kernel: 4 lanes per block. Block i starts at base + (OFFS ? offs[i] : i*stride)
// and is LENS ? lens[i] : len bytes long. 256-thread workgroups = 64 blocks.
// VERIFY: instead of writing the checksum, compare with expected[i]; on mismatch
// atomically lower *first_bad to i and count into *n_bad.
// ---------------------------------------------------------------------------
template <int U, bool LENS, bool OFFS, bool VERIFY, bool NT = false, int D = 0, int TH = 256>
__global__ __launch_bounds__(TH) void k_xxh64_quad(const uint8_t* __restrict__ base, uint64_t stride,
                                                      const uint32_t* __restrict__ lens, uint32_t len,
                                                      const uint64_t* __restrict__ offs, uint64_t n,
                                                      uint64_t* __restrict__ out,
                                                      const uint64_t* __restrict__ expected,
                                                      unsigned long long* __restrict__ first_bad,
                                                      unsigned long long* __restrict__ n_bad) {
    const uint64_t gtid = static_cast<uint64_t>(blockIdx.x) * TH + threadIdx.x;
    const uint64_t blk_raw = gtid >> 2;
    const uint32_t j = threadIdx.x & 3;
    const bool live = blk_raw < n;
    const uint64_t blk = live ? blk_raw : n - 1;  // dead quads shadow the last block; never store
    const uint8_t* src = base + (OFFS ? offs[blk] : blk * stride);
    const uint32_t L = LENS ? lens[blk] : len;
    const uint32_t nst = L >> 5;

    uint64_t acc = acc_seed(j);
    const bool aligned = (reinterpret_cast<uintptr_t>(src) & 7) == 0;
    if (aligned) {
        if constexpr (D >= 2)
            acc = quad_stripes_deep<U, D>(reinterpret_cast<const uint64_t*>(src) + j, nst, acc);
        else
            acc = quad_stripes_aligned<U, NT>(reinterpret_cast<const uint64_t*>(src) + j, nst, acc);
    } else {
        acc = quad_stripes_unaligned(src + 8 * j, nst, acc);
    }
    const uint64_t v1 = quad_bcast<0>(acc);
    const uint64_t v2 = quad_bcast<1>(acc);
    const uint64_t v3 = quad_bcast<2>(acc);
    const uint64_t v4 = quad_bcast<3>(acc);
    if (j == 0 && live) {
        const uint64_t h0 = (L >= 32) ? converge(v1, v2, v3, v4) : kP5;
        const uint64_t h = finish_fast(h0, L, src + 32 * static_cast<uint64_t>(nst), L & 31);
        if (VERIFY) {
            if (h != expected[blk]) {
                atomicMin(first_bad, static_cast<unsigned long long>(blk));
                atomicAdd(n_bad, 1ULL);
            }
        } else {
            out[blk] = h;
        }
    }
}

// ---------------------------------------------------------------------------
// Single-slice latency kernel (stormck_checksum = one blocks.Checksum call). One
// 256-thread workgroup copies the slice from pinned host memory into LDS (every
// thread issues all of its 16-byte reads before storing any: one PCIe round trip per
// 64 KiB), quad 0 hashes it from LDS, and lane 0 stores the checksum straight into
// pinned host memory, so a call is one launch and one stream sync, with no DMA
// commands. src is 16-byte aligned and readable up to the next 16-byte boundary.
// ---------------------------------------------------------------------------
constexpr uint32_t kSingleMax = 64 * 1024;

// K rounds of 16-byte loads per thread, all issued before the first LDS store. Indices
// past the end clamp to the last word (a duplicate load and an identical store), so
// there is no per-load branch and no wait between loads.
template <int K>
__device__ __forceinline__ void single_stage(const uint4* __restrict__ src, uint4* buf, uint32_t words) {
    uint4 r[K];
#pragma unroll
    for (int k = 0; k < K; ++k) r[k] = src[min(threadIdx.x + 256u * k, words - 1)];
#pragma unroll
    for (int k = 0; k < K; ++k) buf[min(threadIdx.x + 256u * k, words - 1)] = r[k];
}

// single_stage, with the block's stripe words premultiplied by P2 on their way into LDS
// (round_pm). The block starts `shift8` 8-byte words into the staged cover (0 or 1:
// only 8-byte-aligned starts take this path) and its first `nw` words are stripe words.
template <int K>
__device__ __forceinline__ void single_stage_pm(const uint4* __restrict__ src, uint4* buf, uint32_t words,
                                                uint32_t shift8, uint32_t nw) {
    uint4 r[K];
#pragma unroll
    for (int k = 0; k < K; ++k) r[k] = src[min(threadIdx.x + 256u * k, words - 1)];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint32_t idx = min(threadIdx.x + 256u * k, words - 1);
        uint64_t a = (static_cast<uint64_t>(r[k].y) << 32) | r[k].x;
        uint64_t b = (static_cast<uint64_t>(r[k].w) << 32) | r[k].z;
        const uint32_t wa = 2 * idx - shift8;  // block word index of a (wraps below 0)
        if (wa < nw) a *= kP2;
        if (wa + 1 < nw) b *= kP2;
        buf[idx] = make_uint4(static_cast<uint32_t>(a), static_cast<uint32_t>(a >> 32), static_cast<uint32_t>(b),
                              static_cast<uint32_t>(b >> 32));
    }
}

template <int KMAX>
__device__ __forceinline__ void stage_pm_switch(const uint4* __restrict__ src, uint4* buf, uint32_t words,
                                                uint32_t shift8, uint32_t nw) {
    switch ((words + 255) / 256) {
        case 0: break;
        case 1: single_stage_pm<1>(src, buf, words, shift8, nw); break;
        case 2: single_stage_pm<2>(src, buf, words, shift8, nw); break;
        case 3: single_stage_pm<3>(src, buf, words, shift8, nw); break;
        case 4: single_stage_pm<4>(src, buf, words, shift8, nw); break;
        case 5: single_stage_pm<5>(src, buf, words, shift8, nw); break;
        case 6: single_stage_pm<6>(src, buf, words, shift8, nw); break;
        case 7: single_stage_pm<7>(src, buf, words, shift8, nw); break;
        case 8: single_stage_pm<8>(src, buf, words, shift8, nw); break;
        default:
            if constexpr (KMAX > 8) {
                switch ((words + 255) / 256) {
                    case 9: single_stage_pm<9>(src, buf, words, shift8, nw); break;
                    case 10: single_stage_pm<10>(src, buf, words, shift8, nw); break;
                    case 11: single_stage_pm<11>(src, buf, words, shift8, nw); break;
                    case 12: single_stage_pm<12>(src, buf, words, shift8, nw); break;
                    case 13: single_stage_pm<13>(src, buf, words, shift8, nw); break;
                    case 14: single_stage_pm<14>(src, buf, words, shift8, nw); break;
                    case 15: single_stage_pm<15>(src, buf, words, shift8, nw); break;
                    default: single_stage_pm<16>(src, buf, words, shift8, nw); break;
                }
            } else {
                single_stage_pm<8>(src, buf, words, shift8, nw);
            }
            break;
    }
}

__global__ __launch_bounds__(256) void k_xxh64_single(const uint8_t* __restrict__ src, uint32_t n,
                                                        uint64_t* __restrict__ out) {
    __shared__ uint4 buf[kSingleMax / 16];
    const uint32_t words = (n + 15) / 16;
    const uint4* s16 = reinterpret_cast<const uint4*>(src);
    const uint32_t nst = n >> 5;
    stage_pm_switch<16>(s16, buf, words, 0, 4 * nst);
    __syncthreads();
    if (threadIdx.x >= 4) return;
    const uint32_t j = threadIdx.x;
    const uint8_t* s = reinterpret_cast<const uint8_t*>(buf);
    const uint64_t acc = quad_stripes_aligned<16, false, true>(reinterpret_cast<const uint64_t*>(s) + j, nst, acc_seed(j));
    const uint64_t v1 = quad_bcast<0>(acc), v2 = quad_bcast<1>(acc), v3 = quad_bcast<2>(acc), v4 = quad_bcast<3>(acc);
    if (j == 0) {
        const uint64_t h0 = (n >= 32) ? converge(v1, v2, v3, v4) : kP5;
        *out = finish_fast(h0, n, s + 32 * nst, n & 31);
    }
}

// ---------------------------------------------------------------------------
// Small-batch kernel ("wide"): one 256-thread workgroup per block. The block (its
// 16-byte-aligned cover, <= 32 KiB) moves HBM -> registers -> LDS in ONE memory round
// trip (every thread issues all its loads before storing any), then quad 0 hashes it
// from LDS. Per-block latency = one round trip + the serial XXH64 chain, where the
// streaming kernels pay a round trip per tile and put 128 blocks on one CU; the host
// picks it for batches too small to fill the chip (launch_checksum). A block whose
// cover exceeds 32 KiB (per-block lengths only) is hashed straight from memory.
// ---------------------------------------------------------------------------
constexpr uint32_t kWideMax = 32 * 1024;

// One block of a staged kernel: its first byte and its length.
struct BlockRef {
    const uint8_t* p;
    uint32_t len;
};

// Pipelined staging (multi_stage_hash_pipe, below): 4 KiB chunks (256 16-byte pieces)
// of each block through a ring of kRingSlots LDS slots per block, an LDS counter per
// chunk, 3 stager waves. A slot holds 2 pieces of pre-pad (the previous chunk's last
// 32 bytes) and the chunk, so a stripe or tail that starts in one chunk and ends in
// the next reads contiguous bytes from the later chunk's slot. Blocks are
// ring_block_pieces(RS) = 2 (mod 16) pieces apart, so the 5 chains of a wave read distinct
// LDS banks (as kMultiPieces below).
// The chunk is a template parameter (CP pieces): 4 KiB up to 8 blocks per workgroup;
// 2 KiB at 16 blocks per workgroup, whose 4-slot rings must fit the same LDS.
constexpr uint32_t kChunkPieces = 256;
constexpr uint32_t kPipeMaxPieces = 4096;  // staged covers up to 64 KiB
constexpr uint32_t pipe_max_chunks(uint32_t cp) { return kPipeMaxPieces / cp; }
constexpr uint32_t kPipeMaxChunks = pipe_max_chunks(kChunkPieces);
constexpr uint32_t kPipeStagers = 3;     // waves 1..3 of a 256-thread workgroup
constexpr uint32_t kRingSlots = 4;  // shipped ring depth (7 measured slower, profiles/r02_pipe/)
constexpr uint32_t kSlotPieces = 2 + kChunkPieces;
// pieces between two blocks' rings: >= RS slots of 2 + CP pieces, = 2 (mod 16)
constexpr uint32_t ring_block_pieces(uint32_t rs, uint32_t cp = kChunkPieces) {
    return (rs * (2 + cp) + 13) / 16 * 16 + 2;
}
constexpr uint32_t kRingSlackPieces = 2;  // a 32-byte tail read past the last slot stays inside
static_assert(ring_block_pieces(4) == 1042 && ring_block_pieces(7) == 1810 && ring_block_pieces(4, 128) == 530,
              "ring layout");

// Quad 0's part of k_xxh64_wide. Inlined once per branch, so the words are read with
// ds_read from the staged copy and with global loads otherwise: through one generic
// pointer both would be flat loads, which the compiler can only wait for all at once
// (s_waitcnt vmcnt(0) lgkmcnt(0) per group, no prefetch overlap).
template <bool VERIFY, bool PM = false>
__device__ __forceinline__ void wide_hash(const uint8_t* s, uint32_t L, uint64_t blk, uint64_t* __restrict__ out,
                                          const uint64_t* __restrict__ expected,
                                          unsigned long long* __restrict__ first_bad,
                                          unsigned long long* __restrict__ n_bad) {
    const uint32_t j = threadIdx.x;
    const uint32_t nst = L >> 5;
    uint64_t acc = acc_seed(j);
    if constexpr (PM) {  // staged with premultiplied stripe words, 8-byte aligned
        acc = quad_stripes_aligned<16, false, true>(reinterpret_cast<const uint64_t*>(s) + j, nst, acc);
    } else if ((reinterpret_cast<uintptr_t>(s) & 7) == 0) {
        acc = quad_stripes_aligned<16>(reinterpret_cast<const uint64_t*>(s) + j, nst, acc);
    } else {
        acc = quad_stripes_unaligned(s + 8 * j, nst, acc);
    }
    const uint64_t v1 = quad_bcast<0>(acc), v2 = quad_bcast<1>(acc), v3 = quad_bcast<2>(acc), v4 = quad_bcast<3>(acc);
    if (j == 0) {
        const uint64_t h0 = (L >= 32) ? converge(v1, v2, v3, v4) : kP5;
        const uint64_t h = finish_fast(h0, L, s + 32 * static_cast<uint64_t>(nst), L & 31);
        if (VERIFY) {
            if (h != expected[blk]) {
                atomicMin(first_bad, static_cast<unsigned long long>(blk));
                atomicAdd(n_bad, 1ULL);
            }
        } else {
            out[blk] = h;
        }
    }
}

template <bool LENS, bool OFFS, bool VERIFY>
__global__ __launch_bounds__(256) void k_xxh64_wide(const uint8_t* __restrict__ base, uint64_t stride,
                                                      const uint32_t* __restrict__ lens, uint32_t len,
                                                      const uint64_t* __restrict__ offs, uint64_t n,
                                                      uint64_t* __restrict__ out,
                                                      const uint64_t* __restrict__ expected,
                                                      unsigned long long* __restrict__ first_bad,
                                                      unsigned long long* __restrict__ n_bad) {
    __shared__ uint4 buf[kWideMax / 16];
    const uint64_t blk = blockIdx.x;
    const uint8_t* src = base + (OFFS ? offs[blk] : blk * stride);
    const uint32_t L = LENS ? lens[blk] : len;
    const uint32_t shift = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(src) & 15);
    const uint32_t words = (shift + L + 15) / 16;
    if (words <= kWideMax / 16) {
        // a 16-byte window holding a byte of the block lies in that byte's page
        const uint4* cover = reinterpret_cast<const uint4*>(src - shift);
        if ((shift & 7) == 0) {  // 8-byte-aligned start: stripe words premultiplied on the way in
            stage_pm_switch<8>(cover, buf, words, shift / 8, 4 * (L >> 5));
            __syncthreads();
            if (threadIdx.x >= 4) return;
            wide_hash<VERIFY, true>(reinterpret_cast<const uint8_t*>(buf) + shift, L, blk, out, expected, first_bad,
                                    n_bad);
            return;
        }
        switch ((words + 255) / 256) {
            case 0: break;
            case 1: single_stage<1>(cover, buf, words); break;
            case 2: single_stage<2>(cover, buf, words); break;
            case 3: single_stage<3>(cover, buf, words); break;
            case 4: single_stage<4>(cover, buf, words); break;
            case 5: single_stage<5>(cover, buf, words); break;
            case 6: single_stage<6>(cover, buf, words); break;
            case 7: single_stage<7>(cover, buf, words); break;
            default: single_stage<8>(cover, buf, words); break;
        }
        __syncthreads();
        if (threadIdx.x >= 4) return;
        wide_hash<VERIFY>(reinterpret_cast<const uint8_t*>(buf) + shift, L, blk, out, expected, first_bad, n_bad);
        return;
    }
    if (threadIdx.x >= 4) return;
    wide_hash<VERIFY>(src, L, blk, out, expected, first_bad, n_bad);
}

// ---------------------------------------------------------------------------
// Batches that fit one workgroup per CU at BPW blocks each ("wide multi"): a 256-thread
// workgroup stages BPW blocks (covers <= 32 KiB, 8-byte-aligned starts) into LDS in one
// memory round trip, stripe words premultiplied by P2, then wave 0's lanes 4b..4b+3
// walk block b's chain. The chain wave is issue-bound, so BPW blocks cost about what
// one costs; at BPW = 5 a storm commit batch (~1,200 blocks) is one workgroup per CU.
// Blocks that cannot be staged (other starts, larger covers) hash from memory in the
// same lanes. multi_stage_hash is the body; k_xxh64_wide_multi (batches) and
// k_commit_level_multi (f1 levels) differ only in where a block is and what happens to
// its checksum.
// ---------------------------------------------------------------------------
// Block slots are kMultiPieces 16-byte pieces apart: 2034 = 2 (mod 16), so slot b starts
// 32 * b bytes into the 256-byte bank period and the chain's ds_read_b64 of the BPW
// blocks (4 lanes x 8 B each) hit distinct banks (a 32 KiB stride would put them all on
// the same 8 banks). 5 slots of 32,544 B fit the CU's 160 KiB.
constexpr uint32_t kMultiPieces = 2034;

// buf: BPW * kMultiPieces LDS pieces. src_of(b) -> BlockRef of block b < nlive (called by
// every thread; nlive >= 1). emit(b, h) runs on lane 0 of quad b for b < nlive.
template <int BPW, class Src, class Emit>
__device__ __forceinline__ void multi_stage_hash(uint4* buf, uint32_t nlive, Src src_of, Emit emit) {
    const uint4* cover[BPW];
    uint32_t words[BPW], shift8[BPW], nw[BPW];
#pragma unroll
    for (int b = 0; b < BPW; ++b) {
        words[b] = 0;
        cover[b] = nullptr;
        shift8[b] = 0;
        nw[b] = 0;
        if (static_cast<uint32_t>(b) < nlive) {
            const BlockRef r = src_of(static_cast<uint32_t>(b));
            const uint32_t shift = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(r.p) & 15);
            const uint32_t w = (shift + r.len + 15) / 16;
            if ((shift & 7) == 0 && w <= kMultiPieces) {
                words[b] = w;
                cover[b] = reinterpret_cast<const uint4*>(r.p - shift);
                shift8[b] = shift / 8;
                nw[b] = 4 * (r.len >> 5);
            }
        }
    }
    // every thread issues all of its loads (<= 8 pieces per block) before storing any.
    // The loads are unconditional (index clamped, blocks that are not staged read a
    // staged block's cover): a load under a branch gets its own vmcnt(0) wait, which
    // would make the 8 * BPW loads 8 * BPW round trips.
    const uint4* safe = nullptr;
#pragma unroll
    for (int b = 0; b < BPW; ++b)
        if (!safe && words[b]) safe = cover[b];
    if (safe) {  // uniform over the workgroup
        const uint4* cv[BPW];
        uint32_t lim[BPW];
#pragma unroll
        for (int b = 0; b < BPW; ++b) {
            cv[b] = words[b] ? cover[b] : safe;
            lim[b] = words[b] ? words[b] - 1 : 0;
        }
        uint4 r[BPW * 8];
#pragma unroll
        for (int k = 0; k < BPW * 8; ++k) {
            const int b = k >> 3;
            r[k] = cv[b][min(threadIdx.x + 256u * (k & 7), lim[b])];
        }
#pragma unroll
        for (int k = 0; k < BPW * 8; ++k) {
            const int b = k >> 3;
            const uint32_t idx = threadIdx.x + 256u * (k & 7);
            if (idx < words[b]) {
                uint64_t a = (static_cast<uint64_t>(r[k].y) << 32) | r[k].x;
                uint64_t c = (static_cast<uint64_t>(r[k].w) << 32) | r[k].z;
                const uint32_t wa = 2 * idx - shift8[b];
                if (wa < nw[b]) a *= kP2;
                if (wa + 1 < nw[b]) c *= kP2;
                buf[b * kMultiPieces + idx] = make_uint4(static_cast<uint32_t>(a), static_cast<uint32_t>(a >> 32),
                                                         static_cast<uint32_t>(c), static_cast<uint32_t>(c >> 32));
            }
        }
    }
    __syncthreads();
    if (threadIdx.x >= 4 * BPW) return;
    const uint32_t b = threadIdx.x >> 2, j = threadIdx.x & 3;
    const bool live = b < nlive;
    const BlockRef r = src_of(live ? b : nlive - 1);
    const uint8_t* src = r.p;
    const uint32_t L = r.len;
    const uint32_t nst = L >> 5;
    const uint32_t shift = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(src) & 15);
    const bool staged = (shift & 7) == 0 && (shift + L + 15) / 16 <= kMultiPieces;
    const uint8_t* s = staged ? reinterpret_cast<const uint8_t*>(buf + b * kMultiPieces) + shift : src;
    uint64_t acc = acc_seed(j);
    if (staged)
        acc = quad_stripes_aligned<16, false, true>(reinterpret_cast<const uint64_t*>(s) + j, nst, acc);
    else if ((reinterpret_cast<uintptr_t>(src) & 7) == 0)
        acc = quad_stripes_aligned<16>(reinterpret_cast<const uint64_t*>(src) + j, nst, acc);
    else
        acc = quad_stripes_unaligned(src + 8 * j, nst, acc);
    const uint64_t v1 = quad_bcast<0>(acc), v2 = quad_bcast<1>(acc), v3 = quad_bcast<2>(acc), v4 = quad_bcast<3>(acc);
    if (j == 0 && live) {
        const uint64_t h0 = (L >= 32) ? converge(v1, v2, v3, v4) : kP5;
        emit(b, finish_fast(h0, L, s + 32 * static_cast<uint64_t>(nst), L & 31));
    }
}

// Pipelined form of multi_stage_hash. The whole-block staging above costs one full
// round trip of BPW x 32 KiB per CU before the first chain round, and a 32 KiB block
// (cover 2,048 or 2,049 pieces) does not fit its 2,034-piece slot at all. Here the
// workgroup stages the first 4 KiB chunk of every block together; then wave 0 walks
// the chains while waves 1-3 stage chunks 1.. in order through a 4-slot ring per
// block (layout above). Per chunk, each stager wave adds 1 to the chunk's LDS counter
// and the chain waits for 3 before reading it; the chain publishes how many chunks it
// has finished, and a stager overwrites a slot only after the chain finished the chunk
// that held it. A chain consumes a chunk in ~3 us, the stagers fill one in about one
// memory round trip, so neither side waits long. Each lane keeps its block's tail
// (< 32 bytes) in registers when it passes the tail's chunk, before the slot can be
// reused. Blocks with 8-byte-aligned starts and covers up to 64 KiB are staged; others
// hash from memory in the same lanes.
// ring: BPW * ring_block_pieces(RS) + kRingSlackPieces pieces; ready: kPipeMaxChunks words;
// done: one word. Same contract as multi_stage_hash otherwise.

// Liveness and integrity of the ring. Every wait is bounded (~0.1 s of polling): a
// chunk that never completes (a staging/chain disagreement would be a bug) must not
// leave a wave that never exits. An expired wait is an ERROR, never a value: the
// waiting wave sets the workgroup's abort word (every other wait of the workgroup then
// returns at once), the chain emits no checksum for any of its blocks (a verify counts
// them as mismatches), stagers stop writing slots, and the kernel stores its fault code
// into the fault slot of the stream it runs on (pinned host memory, one per stream),
// which the host-synchronous entry points check after their sync and
// stormck_device_status(stream) reports for the async ones.
// fault codes: kernel id | side
constexpr uint32_t kFaultWideMulti = 1u, kFaultCommitMulti = 2u;
constexpr uint32_t kFaultChain = 0x100u, kFaultStager = 0x200u;
constexpr uint32_t kPipeSpin = 1u << 22;

// Pipe control shared by one workgroup's chain and stager waves (LDS), plus the
// kernel's fault word and its debug stall (STORMCK_DEBUG_STALL_CHUNK: stager wave 1 of
// workgroup 0 never reports chunk `stall`, so the chain's wait for it expires).
struct PipeCtl {
    uint32_t* ready;   // pipe_max_chunks(CP) LDS counters
    uint32_t* done;    // LDS: chunks the chain has finished
    uint32_t* abort;   // LDS: set by the first expired wait
    uint32_t* fault;   // pinned host fault slot of the launch's stream, or null
    uint32_t kernel;   // kFault* id
    uint32_t stall;    // 0 = off
};

// The ring's signals are LDS words between the waves of one workgroup. LDS executes a
// wave's operations in order, so a counter bump issued after a wave's slot writes is seen
// only after them, and reads issued after a counter was seen come after the writes it
// counts: relaxed atomics plus compiler-only fences suffice. (An acquire / release fence
// would also wait for the wave's outstanding global loads, vmcnt(0), which serialises
// a stager's double-buffered loads.)
__device__ __forceinline__ void lds_signal_fence() { __atomic_signal_fence(__ATOMIC_SEQ_CST); }

// Wait until *word >= at_least. false: the wait expired (this call set the abort word)
// or another wave of the workgroup aborted.
__device__ __forceinline__ bool pipe_wait(const PipeCtl& pc, const uint32_t* word, uint32_t at_least,
                                          uint32_t side) {
    lds_signal_fence();
    for (uint32_t spin = 0; __hip_atomic_load(word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < at_least;
         ++spin) {
        if (__hip_atomic_load(pc.abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) return false;
        if (spin >= kPipeSpin) {
            __hip_atomic_store(pc.abort, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (pc.fault) __hip_atomic_store(pc.fault, pc.kernel | side, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            return false;
        }
        __builtin_amdgcn_s_sleep(1);
    }
    lds_signal_fence();  // the caller's LDS reads / writes stay after the wait
    return true;
}

// DBL: each stager keeps two chunks in flight (loads of chunk c+1 issued before chunk c
// is stored): with 2 KiB chunks one chunk per memory round trip is less than the chains
// consume.
// Void(b): block b of a stalled workgroup gets no checksum; a verify counts it as a
// mismatch there (fails closed), a checksum or commit launch leaves it unwritten.
template <int BPW, uint32_t RS, uint32_t CP, bool DBL, class Src, class Emit, class Void>
__device__ __forceinline__ void multi_stage_hash_pipe(uint4* ring, const PipeCtl& pc, uint32_t nlive, Src src_of,
                                                      Emit emit, Void void_block) {
    static_assert(BPW <= 16 && CP <= 256 && kPipeMaxPieces % CP == 0, "one chain wave, chunks of <= 256 pieces");
    uint32_t* ready = pc.ready;
    uint32_t* done = pc.done;
    constexpr uint32_t kMaxPieces = kPipeMaxPieces;
    constexpr uint32_t kSlot = 2 + CP;                   // pieces per ring slot
    constexpr uint32_t kPasses = (kSlot + 191) / 192;    // stager loads per block per chunk
    constexpr uint32_t kRingBlockPieces = ring_block_pieces(RS, CP);
    const uint4* cover[BPW];
    uint32_t words[BPW], shift8[BPW], nw[BPW];
    uint32_t nch = 0;  // chunks of the longest staged block (uniform over the workgroup)
#pragma unroll
    for (int b = 0; b < BPW; ++b) {
        words[b] = 0;
        cover[b] = nullptr;
        shift8[b] = 0;
        nw[b] = 0;
        if (static_cast<uint32_t>(b) < nlive) {
            const BlockRef r = src_of(static_cast<uint32_t>(b));
            const uint32_t shift = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(r.p) & 15);
            const uint32_t w = (shift + r.len + 15) / 16;
            if ((shift & 7) == 0 && w > 0 && w <= kMaxPieces) {
                words[b] = w;
                cover[b] = reinterpret_cast<const uint4*>(r.p - shift);
                shift8[b] = shift / 8;
                nw[b] = 4 * (r.len >> 5);
                nch = max(nch, (w + CP - 1) / CP);
            }
        }
    }
    const uint4* safe = nullptr;
#pragma unroll
    for (int b = 0; b < BPW; ++b)
        if (!safe && words[b]) safe = cover[b];
    const uint4* cv[BPW];
    uint32_t lim[BPW];
#pragma unroll
    for (int b = 0; b < BPW; ++b) {
        cv[b] = words[b] ? cover[b] : safe;
        lim[b] = words[b] ? words[b] - 1 : 0;
    }
    // cover piece idx of block b, premultiplied, into ring position pos of the block
    auto put = [&](int b, uint32_t pos, uint32_t idx, const uint4& v) {
        uint64_t a = (static_cast<uint64_t>(v.y) << 32) | v.x;
        uint64_t c = (static_cast<uint64_t>(v.w) << 32) | v.z;
        const uint32_t wa = 2 * idx - shift8[b];
        if (wa < nw[b]) a *= kP2;
        if (wa + 1 < nw[b]) c *= kP2;
        ring[b * kRingBlockPieces + pos] = make_uint4(static_cast<uint32_t>(a), static_cast<uint32_t>(a >> 32),
                                                      static_cast<uint32_t>(c), static_cast<uint32_t>(c >> 32));
    };
    if (threadIdx.x < pipe_max_chunks(CP)) ready[threadIdx.x] = 0;
    if (threadIdx.x == 0) {
        *done = 0;
        *pc.abort = 0;
    }
    if (safe) {  // chunk 0 into slot 0, threads < CP one piece of each block
        uint4 r[BPW];
#pragma unroll
        for (int b = 0; b < BPW; ++b) r[b] = cv[b][min(threadIdx.x, lim[b])];
#pragma unroll
        for (int b = 0; b < BPW; ++b)
            if (threadIdx.x < CP && threadIdx.x < words[b]) put(b, 2 + threadIdx.x, threadIdx.x, r[b]);
    }
    __syncthreads();
    if (threadIdx.x >= 64) {
        // stagers: slot position k < CP + 2 of chunk c holds cover piece CP*c - 2 + k; over
        // 192 threads as k = t, t + 192, ... (a load past the slot repeats a clamped
        // address and is not stored)
        const uint32_t t = threadIdx.x - 64;
        auto load = [&](uint32_t c, uint4 (&r)[BPW][kPasses]) __attribute__((always_inline)) {
#pragma unroll
            for (int b = 0; b < BPW; ++b)
#pragma unroll
                for (int q = 0; q < static_cast<int>(kPasses); ++q)
                    r[b][q] = cv[b][min(c * CP - 2 + min(t + 192u * q, kSlot - 1), lim[b])];
        };
        // chunk c into its slot, then count this wave in; false: stop (expired wait / abort)
        auto store = [&](uint32_t c, const uint4 (&r)[BPW][kPasses]) __attribute__((always_inline)) -> bool {
            // the slot's old chunk is finished; on an expired wait (or an abort) stop
            // writing: the chain may still be reading the slot
            if (c >= RS && !pipe_wait(pc, done, c - RS + 1, kFaultStager)) return false;
            const uint32_t slot = (c % RS) * kSlot;
#pragma unroll
            for (int b = 0; b < BPW; ++b)
#pragma unroll
                for (int q = 0; q < static_cast<int>(kPasses); ++q) {
                    const uint32_t k = t + 192u * q, idx = c * CP - 2 + k;
                    if (k < kSlot && idx < words[b]) put(b, slot + k, idx, r[b][q]);
                }
            // the slot writes are performed before the count (LDS order; see pipe_wait)
            wait_lgkm0();
            lds_signal_fence();
            const bool stalled = pc.stall == c && blockIdx.x == 0 && threadIdx.x < 128;  // debug knob only
            if ((threadIdx.x & 63) == 0 && !stalled)
                __hip_atomic_fetch_add(ready + c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            return true;
        };
        if constexpr (DBL) {
            // two buffers, fully unrolled (no loop back-edge, across which the compiler
            // would wait for every load): each store waits for exactly the older buffer
            uint4 ra[BPW][kPasses], rb[BPW][kPasses];
            if (nch > 1) load(1, ra);
#pragma unroll
            for (uint32_t p = 0; p < pipe_max_chunks(CP) / 2; ++p) {
                const uint32_t c = 1 + 2 * p;
                if (c >= nch) break;
                if (c + 1 < nch) load(c + 1, rb);
                if (!store(c, ra)) return;
                if (c + 1 >= nch) break;
                if (c + 2 < nch) load(c + 2, ra);
                if (!store(c + 1, rb)) return;
            }
        } else {
            for (uint32_t c = 1; c < nch; ++c) {
                uint4 r[BPW][kPasses];
                load(c, r);
                if (!store(c, r)) return;
            }
        }
        return;
    }
    if (threadIdx.x >= 4 * BPW) return;
    const uint32_t b = threadIdx.x >> 2, j = threadIdx.x & 3;
    const bool live = b < nlive;
    const BlockRef r = src_of(live ? b : nlive - 1);
    const uint8_t* src = r.p;
    const uint32_t L = r.len;
    const uint32_t nst = L >> 5;
    const uint32_t shift = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(src) & 15);
    // exactly the staging condition above
    const uint32_t w = (shift + L + 15) / 16;
    const bool staged = safe && (shift & 7) == 0 && w > 0 && w <= kMaxPieces;
    const uint8_t* blk_ring = reinterpret_cast<const uint8_t*>(ring + b * kRingBlockPieces);
    const uint32_t tail_chunk = (shift + L - (L > 0 ? 1 : 0)) / (16 * CP);
    uint64_t acc = acc_seed(j);
    uint64_t tail[4] = {0, 0, 0, 0};
    uint32_t s_done = 0;
    bool ok = true;
    // every chain lane runs the chunk loop (lane 0 publishes progress for the wave)
    for (uint32_t c = 0; c < nch; ++c) {
        if (c > 0 && !pipe_wait(pc, ready + c, kPipeStagers, kFaultChain)) {
            ok = false;  // the chunk never arrived: no checksum from this workgroup
            break;
        }
        if (staged) {
            // slot byte of cover byte x of this chunk: 32 + x - 16*CP*c
            const uint8_t* slot = blk_ring + (c % RS) * kSlot * 16 + 32;
            const int64_t base = static_cast<int64_t>(shift) - static_cast<int64_t>(16 * CP) * c;
            const uint32_t end = min(nst, (16 * CP * (c + 1) - shift) / 32);
            if (end > s_done) {
                acc = quad_stripes_aligned<16, false, true>(
                    reinterpret_cast<const uint64_t*>(slot + base + 32 * static_cast<int64_t>(s_done)) + j, end - s_done,
                    acc);
                s_done = end;
            }
            if (c == tail_chunk) {  // the tail's last byte is in this chunk, its first at most 31 before
                const uint64_t* tp = reinterpret_cast<const uint64_t*>(slot + base + 32 * static_cast<int64_t>(nst));
#pragma unroll
                for (int q = 0; q < 4; ++q) tail[q] = tp[q];
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        if (threadIdx.x == 0) __hip_atomic_store(done, c + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    if (!staged) {
        if ((reinterpret_cast<uintptr_t>(src) & 7) == 0)
            acc = quad_stripes_aligned<16>(reinterpret_cast<const uint64_t*>(src) + j, nst, acc);
        else
            acc = quad_stripes_unaligned(src + 8 * j, nst, acc);
    }
    // a stager that gave up (its wait for `done` expired) also voids the workgroup:
    // it may have left a slot unwritten that the chain already passed
    if (__hip_atomic_load(pc.abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) ok = false;
    if (!ok) {
        if (j == 0 && live) void_block(b);
        return;
    }
    const uint64_t v1 = quad_bcast<0>(acc), v2 = quad_bcast<1>(acc), v3 = quad_bcast<2>(acc), v4 = quad_bcast<3>(acc);
    if (j == 0 && live) {
        const uint64_t h0 = (L >= 32) ? converge(v1, v2, v3, v4) : kP5;
        emit(b, staged ? finish_regs(h0, L, tail, L & 31)
                       : finish_fast(h0, L, src + 32 * static_cast<uint64_t>(nst), L & 31));
    }
}

// RING: ring slots of the pipelined body (multi_stage_hash_pipe); 0 stages whole blocks first.
template <bool LENS, bool OFFS, bool VERIFY, int BPW, uint32_t RING = kRingSlots, uint32_t CP = kChunkPieces,
          bool DBL = false>
__global__ __launch_bounds__(256) void k_xxh64_wide_multi(const uint8_t* __restrict__ base, uint64_t stride,
                                                            const uint32_t* __restrict__ lens, uint32_t len,
                                                            const uint64_t* __restrict__ offs, uint64_t n,
                                                            uint64_t* __restrict__ out,
                                                            const uint64_t* __restrict__ expected,
                                                            unsigned long long* __restrict__ first_bad,
                                                            unsigned long long* __restrict__ n_bad,
                                                            uint32_t* __restrict__ fault, uint32_t stall) {
    static_assert(RING > 0 ? (BPW * ring_block_pieces(RING, CP) + kRingSlackPieces) * 16 <= 150 * 1024
                           : BPW * kMultiPieces * 16 <= 160 * 1024,
                  "LDS");
    const uint64_t first = static_cast<uint64_t>(blockIdx.x) * BPW;
    const uint32_t nlive = static_cast<uint32_t>(min<uint64_t>(BPW, n - first));
    auto src_of = [&](uint32_t b) {
        const uint64_t blk = first + b;
        return BlockRef{base + (OFFS ? offs[blk] : blk * stride), LENS ? lens[blk] : len};
    };
    auto emit = [&](uint32_t b, uint64_t h) {
        const uint64_t blk = first + b;
        if (VERIFY) {
            if (h != expected[blk]) {
                atomicMin(first_bad, static_cast<unsigned long long>(blk));
                atomicAdd(n_bad, 1ULL);
            }
        } else {
            out[blk] = h;
        }
    };
    if constexpr (RING > 0) {
        __shared__ uint4 ring[BPW * ring_block_pieces(RING, CP) + kRingSlackPieces];
        __shared__ uint32_t ready[pipe_max_chunks(CP)], done[1], abort_w[1];
        const PipeCtl pc{ready, done, abort_w, fault, kFaultWideMulti, stall};
        auto void_block = [&](uint32_t b) {
            if (VERIFY) {  // fail closed: an unhashed block is a mismatch
                atomicMin(first_bad, static_cast<unsigned long long>(first + b));
                atomicAdd(n_bad, 1ULL);
            }
        };
        multi_stage_hash_pipe<BPW, RING, CP, DBL>(ring, pc, nlive, src_of, emit, void_block);
    } else {
        __shared__ uint4 buf[BPW * kMultiPieces];
        multi_stage_hash<BPW>(buf, nlive, src_of, emit);
    }
}

// ---------------------------------------------------------------------------
// LDS-staged quad kernel ("glds"): uniform length, 16-byte aligned base/stride.
// A 256-thread workgroup owns 64 consecutive blocks. Tiles of T stripes (32*T bytes)
// of all 64 blocks stream HBM -> LDS with global_load_lds_dwordx4 (each wave-
// instruction moves 1 KiB: 64 lanes x 16 B, 16 B contiguous per lane; the LDS
// destination is lane-linear, so the layout is set by the per-lane SOURCE address)
// into a ring of R tile slots, R-1 tiles ahead of the hashing. Lane (b, j) of the
// quad for block b then reads word j of each stripe with ds_read_b64.
// Bank-conflict-free reads: within block b's row, 16-byte piece q holds source piece
// (q + rot(b)) mod 2T, so the 8 blocks read by one 32-lane ds_read_b64 group hit 32
// distinct 8-byte bank pairs.
// ---------------------------------------------------------------------------
template <int T>
__device__ __forceinline__ uint32_t glds_rot(uint32_t b) {
    constexpr uint32_t pieces = 2 * T;
    if constexpr (T >= 8) return (2 * b) % pieces;
    else return (2 * (b / (8 / T))) % pieces;
}

// One tile's worth of this wave's LDS-DMA pieces: instruction k moves 64 x 16 B from
// the lanes' sources (advanced by t tiles) to dst + k*1024 (lane-linear). A macro:
// the builtin's size/aux operands must stay literal constants.
#if defined(__HIP_DEVICE_COMPILE__)  // target builtin: device pass only (host pass only emits the stub)
#define STORMCK_GLDS_ISSUE(SRC, DST, T_, NK, ROW_, AUX_)                                              \
    do {                                                                                           \
        _Pragma("unroll") for (int k_ = 0; k_ < (NK); ++k_)                                        \
            __builtin_amdgcn_global_load_lds((SRC)[k_] + static_cast<uint64_t>(T_) * (ROW_),       \
                                             (DST) + k_ * 1024, 16, 0, (AUX_));                    \
    } while (0)
#else
#define STORMCK_GLDS_ISSUE(SRC, DST, T_, NK, ROW_, AUX_) do { } while (0)
#endif

template <int T, int R, int AUX, bool HASH = true, bool VERIFY = false, int WAVES = 4, bool SYNC = true, bool XCD = false>
__global__ __launch_bounds__(64 * WAVES) void k_xxh64_glds(const uint8_t* __restrict__ base, uint64_t stride, uint32_t len,
                                                     uint64_t n, uint64_t* __restrict__ out,
                                                     const uint64_t* __restrict__ expected = nullptr,
                                                     unsigned long long* __restrict__ first_bad = nullptr,
                                                     unsigned long long* __restrict__ n_bad = nullptr) {
    constexpr int BPW = 16 * WAVES;         // blocks per workgroup (a quad of lanes per block)
    constexpr int ROW = 32 * T;             // bytes per block per tile
    constexpr int TILE = BPW * ROW;         // bytes per tile
    constexpr int INSTR = TILE / 1024;      // glds wave-instructions per tile (whole workgroup)
    constexpr int PER_WAVE = INSTR / WAVES; // ... per wave
    static_assert(INSTR % WAVES == 0, "tile must split evenly over the waves");
    static_assert(R >= 2, "ring needs >= 2 slots");
    static_assert(SYNC || T % 2 == 0, "without SYNC a wave's pieces must be its own block rows");
    __shared__ __attribute__((aligned(16))) uint8_t lds[R * TILE];

    const uint32_t tid = threadIdx.x;
    const uint32_t wave = tid >> 6, lane = tid & 63;
    uint32_t wg = blockIdx.x;
    if constexpr (XCD) {
        // workgroups are dealt round-robin to the 8 XCDs: give XCD x a contiguous range
        if ((gridDim.x & 7) == 0) wg = (wg & 7) * (gridDim.x >> 3) + (wg >> 3);
    }
    const uint64_t blk0 = static_cast<uint64_t>(wg) * BPW;
    const uint32_t nst = len >> 5;
    const uint32_t ntiles = nst / T;

    // Per-lane source pointers of this wave's PER_WAVE instructions (tile 0).
    const uint8_t* src[PER_WAVE];
#pragma unroll
    for (int k = 0; k < PER_WAVE; ++k) {
        const uint32_t ii = wave * PER_WAVE + k;            // instruction index within the tile
        const uint32_t off = ii * 1024 + lane * 16;          // byte offset in the tile image
        const uint32_t b = off / ROW, q = (off % ROW) / 16;  // block row, LDS piece
        const uint32_t p = (q + glds_rot<T>(b)) % (2 * T);  // source piece
        uint64_t gb = blk0 + b;
        if (gb >= n) gb = n - 1;                             // shadow the last block; never stored
        src[k] = base + gb * stride + p * 16;
    }

    const uint32_t b = tid >> 2, j = tid & 3;
    const uint32_t rot = glds_rot<T>(b);
    uint64_t acc = acc_seed(j);

    // prologue: R-1 tiles in flight
#pragma unroll
    for (int t = 0; t < R - 1; ++t)
        if (t < static_cast<int>(ntiles))
            STORMCK_GLDS_ISSUE(src, lds + (t % R) * TILE + wave * PER_WAVE * 1024, t, PER_WAVE, ROW, AUX);

    for (uint32_t t = 0; t < ntiles; ++t) {
        // tile t landed (this wave's pieces), then every wave's pieces
        if (t + R - 2 < ntiles) wait_vmcnt<PER_WAVE * (R - 2)>();
        else wait_vmcnt<0>();
        // A wave's pieces are exactly the rows of its own 16 blocks, so a wave only
        // reads what it loaded. SYNC keeps the waves in step with a barrier; without
        // it each wave only retires its own reads of tile t-1 before refilling.
        if constexpr (SYNC) __builtin_amdgcn_s_barrier();
        else wait_lgkm0();
        // all waves finished reading tile t-1: refill its slot with tile t+R-1
        if (t + R - 1 < ntiles)
            STORMCK_GLDS_ISSUE(src, lds + ((t + R - 1) % R) * TILE + wave * PER_WAVE * 1024, t + R - 1, PER_WAVE, ROW, AUX);
        const uint8_t* row = lds + (t % R) * TILE + b * ROW + (j & 1) * 8;
#pragma unroll
        for (int s = 0; s < T; ++s) {
            const uint32_t q = (2 * s + (j >> 1) + 2 * T - rot) % (2 * T);
            const uint64_t w = *reinterpret_cast<const uint64_t*>(row + q * 16);
            if constexpr (HASH) acc = round(acc, w);
            else acc ^= w;  // measurement control: same data movement, no hash arithmetic
        }
    }
    // remainder stripes + tail straight from global memory (none for 32 KiB blocks)
    const uint64_t gbk = blk0 + b;
    const uint64_t gb = gbk < n ? gbk : n - 1;
    const uint8_t* blk_src = base + gb * stride;
    for (uint32_t s = ntiles * T; s < nst; ++s)
        acc = round(acc, reinterpret_cast<const uint64_t*>(blk_src)[4 * s + j]);
    const uint64_t v1 = quad_bcast<0>(acc), v2 = quad_bcast<1>(acc), v3 = quad_bcast<2>(acc), v4 = quad_bcast<3>(acc);
    if (j == 0 && gbk < n) {
        const uint64_t h0 = (len >= 32) ? converge(v1, v2, v3, v4) : kP5;
        const uint64_t h = finish_fast(h0, len, blk_src + 32 * static_cast<uint64_t>(nst), len & 31);
        if constexpr (VERIFY) {
            if (h != expected[gbk]) {
                atomicMin(first_bad, static_cast<unsigned long long>(gbk));
                atomicAdd(n_bad, 1ULL);
            }
        } else {
            out[gbk] = h;
        }
    }
}

// ---------------------------------------------------------------------------
// Large uniform batches: the same LDS-DMA ring, persistent and with the waves' streams
// skewed by 4 KiB. One workgroup per CU walks groups g = blockIdx.x, + gridDim.x, ...
// of 16*WAVES blocks, and the tile stream runs on across group boundaries. Wave v
// starts its stream v*SKEW tiles late, so at any moment a workgroup reads its blocks
// at WAVES different offsets, SKEW*32*T bytes apart, instead of all at one offset.
// Measured (profiles/r01_probe_phase_skew.txt): 4 KiB apart, 0.897 -> 0.912 of peak
// on a well-placed arena and no change on a badly placed one; 512 B, 1 KiB and 2 KiB
// apart all lose. The first and last (WAVES-1)*SKEW steps leave some waves idle, so
// the host uses this kernel only when each workgroup has thousands of steps.
// A wave only reads the LDS rows it loaded itself (its own 16 blocks: T even), so the
// skew needs no synchronisation beyond the ring's per-step barrier.
// ---------------------------------------------------------------------------
// HASH = false: the same data movement with the hash replaced by xor (the measured
// read peak bench.py reports beside the kernel, tools/readpeak.hip).
template <int T, int AUX, bool VERIFY, int WAVES, int SKEW, bool HASH = true>
__global__ __launch_bounds__(64 * WAVES) void k_xxh64_glds_skew(const uint8_t* __restrict__ base, uint64_t stride,
                                                                uint32_t len, uint64_t n, uint64_t* __restrict__ out,
                                                                const uint64_t* __restrict__ expected,
                                                                unsigned long long* __restrict__ first_bad,
                                                                unsigned long long* __restrict__ n_bad) {
    constexpr int BPW = 16 * WAVES;
    constexpr int ROW = 32 * T;
    constexpr int TILE = BPW * ROW;
    constexpr int INSTR = TILE / 1024;
    constexpr int PER_WAVE = INSTR / WAVES;
    static_assert(INSTR % WAVES == 0 && T % 2 == 0, "a wave's pieces must be its own block rows");
    __shared__ __attribute__((aligned(16))) uint8_t lds[2 * TILE];

    const uint32_t tid = threadIdx.x;
    const uint32_t wave = tid >> 6, lane = tid & 63;
    const uint64_t ngroups = (n + BPW - 1) / BPW;
    const uint64_t G = gridDim.x;
    if (blockIdx.x >= ngroups) return;
    const uint32_t nst = len >> 5, ntiles = nst / T;
    const uint64_t total = ((ngroups - blockIdx.x + G - 1) / G) * ntiles;  // this workgroup's tile steps
    const uint64_t ph = static_cast<uint64_t>(wave) * SKEW;                  // this wave's start delay
    const uint64_t steps = total + static_cast<uint64_t>(WAVES - 1) * SKEW;   // the same for every wave

    // piece geometry (the same in every group): block row and source byte offset
    uint32_t prow[PER_WAVE], pofs[PER_WAVE];
#pragma unroll
    for (int k = 0; k < PER_WAVE; ++k) {
        const uint32_t off = (wave * PER_WAVE + k) * 1024 + lane * 16;
        const uint32_t b = off / ROW, q = (off % ROW) / 16;
        prow[k] = b;
        pofs[k] = ((q + glds_rot<T>(b)) % (2 * T)) * 16;
    }
    const uint8_t* src[PER_WAVE];
    uint64_t ig = blockIdx.x, hg = blockIdx.x, ic = 0, hc = 0;  // issue / hash: group, tiles done
    uint32_t it = 0, ht = 0;                                    // issue / hash: tile within the group
    auto issue = [&](uint32_t slot) {
        if (it == 0) {
#pragma unroll
            for (int k = 0; k < PER_WAVE; ++k) {
                uint64_t gb = ig * BPW + prow[k];
                if (gb >= n) gb = n - 1;  // shadow the last block; never stored
                src[k] = base + gb * stride + pofs[k];
            }
        }
        STORMCK_GLDS_ISSUE(src, lds + slot * TILE + wave * PER_WAVE * 1024, it, PER_WAVE, ROW, AUX);
        if (++it == ntiles) {
            it = 0;
            ig += G;
        }
        ++ic;
    };
    const uint32_t b = tid >> 2, j = tid & 3;
    const uint32_t rot = glds_rot<T>(b);
    uint64_t acc = acc_seed(j);
    if (ph == 0 && total > 0) issue(0);
    for (uint64_t u = 0; u < steps; ++u) {
        wait_vmcnt<0>();
        __builtin_amdgcn_s_barrier();
        if (u + 1 >= ph && ic < total) issue((u + 1) & 1);  // this wave's step u+1 into the other slot
        if (u >= ph && hc < total) {
            const uint8_t* row = lds + (u & 1) * TILE + b * ROW + (j & 1) * 8;
#pragma unroll
            for (int s = 0; s < T; ++s) {
                const uint32_t q = (2 * s + (j >> 1) + 2 * T - rot) % (2 * T);
                const uint64_t w = *reinterpret_cast<const uint64_t*>(row + q * 16);
                if constexpr (HASH) acc = round(acc, w);
                else acc ^= w;
            }
            if (++ht == ntiles) {
                // the group's blocks are complete: remainder stripes and tail from global
                // memory (none for 32 KiB blocks), then the checksum
                const uint64_t gbk = hg * BPW + b;
                const uint64_t gb = gbk < n ? gbk : n - 1;
                const uint8_t* blk_src = base + gb * stride;
                for (uint32_t s = ntiles * T; s < nst; ++s)
                    acc = round(acc, reinterpret_cast<const uint64_t*>(blk_src)[4 * s + j]);
                const uint64_t v1 = quad_bcast<0>(acc), v2 = quad_bcast<1>(acc), v3 = quad_bcast<2>(acc),
                               v4 = quad_bcast<3>(acc);
                if (j == 0 && gbk < n) {
                    const uint64_t h = finish_fast(converge(v1, v2, v3, v4), len,
                                                   blk_src + 32 * static_cast<uint64_t>(nst), len & 31);
                    if constexpr (VERIFY) {
                        if (h != expected[gbk]) {
                            atomicMin(first_bad, static_cast<unsigned long long>(gbk));
                            atomicAdd(n_bad, 1ULL);
                        }
                    } else {
                        out[gbk] = h;
                    }
                }
                acc = acc_seed(j);
                ht = 0;
                hg += G;
            }
            ++hc;
        }
    }
}

// ---------------------------------------------------------------------------
// Per-block lengths and/or gathered offsets through the LDS-DMA ring: the batch shape
// storm produces (dirty slots of cache.data, cache/cache.go:36-40, with mixed
// Sizeof(T), blocks/objectlist/block.go:29-40, blocks/blob/block.go:25-29). The
// k_xxh64_glds_skew scheme (workgroups of 16*WAVES blocks, 512-byte rows, 2-slot ring,
// persistent with the waves SKEW tiles apart) with three changes:
//  * each wave streams its own number of tiles per group: the longest of its 16
//    blocks, the last tile partial. LDS-DMA lanes of pieces past a block's last stripe
//    are switched off (exec mask) and the quads predicate the rounds of a partial tile,
//    so every stripe of a staged block comes through LDS; the tail (< 32 B) is read
//    from global memory when the group ends;
//  * a block whose start is not 16-byte aligned is not staged: its quad hashes it from
//    global memory when its group ends (any alignment is correct; storm's slots are
//    32 KiB aligned, so this is the exception, and the host sends base+stride batches
//    with unaligned rows to k_xxh64_quad);
//  * the waves' streams differ in length, so a step runs while any wave of the
//    workgroup still has work: each wave posts a flag before the step's barrier.
// The starts and lengths of group g+G are loaded while group g streams, so a group
// change waits for no memory.
// ---------------------------------------------------------------------------
// Locality order of a large gather. A workgroup's 128 blocks are read in lock step, a
// 512-byte row of each per tile. Gathered from random slots of a large arena (storm's
// dirty slots), the rows of one step land on the HBM channels at random, unevenly, and
// the step waits for the busiest channel: 0.76-0.78 of 8 TB/s on 4M shuffled 32 KiB slots
// against 0.85-0.87 in slot order on the same arenas (profiles/r03d/, r03f/). Bucketing by
// 32 MiB region alone (TLB locality) changed nothing (r03f); the blocks of a group must
// be in address order. So: a counting sort by 32 MiB region of the offset (4,096
// buckets, wrapping every 128 GiB): k_order_count (a histogram per part of the input in
// LDS, added to the bucket totals), k_order_scan_buckets (their exclusive scan),
// k_order_place (each part reserves a range of every bucket it uses with one global
// atomic and places its elements there, ranked with LDS atomics); then k_order_sort
// sorts each bucket of up to kOrderSortMax blocks by offset in LDS. Every checksum is
// still written at its own index. Round 4 rebuilt the order this way (512 parts instead
// of a 128-part count matrix, a counting pass instead of a bitonic network in the sort):
// 0.31 ms per 4M-block gather before (profiles/r03b/gather_kernel_stats.csv).
constexpr uint32_t kOrderShift = 25, kOrderBuckets = 4096, kOrderParts = 512;
// k_order_place's parts. Fewer, longer parts put a part's elements of one bucket side by
// side (~8 per bucket at 4M blocks rather than ~2), but 128 of them measured slower than
// 512: 133.7 against 122-123 us per 4M blocks (profiles/r04_check3/), so the same as the
// count's
constexpr uint32_t kOrderPlaceParts = kOrderParts;

__device__ __forceinline__ uint32_t order_bucket(uint64_t off) {
    return static_cast<uint32_t>(off >> kOrderShift) & (kOrderBuckets - 1);
}

// The elements split into P contiguous parts, one workgroup each.
template <uint32_t P = kOrderParts>
__device__ __forceinline__ void order_part(uint64_t n, uint32_t w, uint64_t* lo, uint64_t* hi) {
    *lo = n * w / P;
    *hi = n * (w + 1) / P;
}

// Bucket totals: each part counts its elements per bucket in LDS, then adds its nonzero
// counts to totals[b] (zeroed by the caller): one global atomic per (part, bucket) used.
__global__ __launch_bounds__(256) void k_order_count(const uint64_t* __restrict__ offs, uint64_t n,
                                                     uint32_t* __restrict__ totals) {
    __shared__ uint32_t h[kOrderBuckets];
    for (uint32_t i = threadIdx.x; i < kOrderBuckets; i += 256) h[i] = 0;
    __syncthreads();
    uint64_t lo, hi;
    order_part(n, blockIdx.x, &lo, &hi);
    for (uint64_t i = lo + threadIdx.x; i < hi; i += 256) atomicAdd(&h[order_bucket(offs[i])], 1u);
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < kOrderBuckets; i += 256)
        if (h[i]) atomicAdd(&totals[i], h[i]);
}

// One workgroup of 1024 threads: bucket totals (bounds[B + b]) -> bounds[b] / bounds[B + b]
// = bucket b's first / one-past-last position, and cursor[b] = its first position (the
// next free place k_order_place reserves from).
__global__ __launch_bounds__(1024) void k_order_scan_buckets(uint32_t* __restrict__ bounds,
                                                             uint32_t* __restrict__ cursor) {
    constexpr uint32_t PER = kOrderBuckets / 1024;
    __shared__ uint32_t part[1024];
    uint32_t c[PER], sum = 0;
    for (uint32_t k = 0; k < PER; ++k) sum += c[k] = bounds[kOrderBuckets + threadIdx.x * PER + k];
    part[threadIdx.x] = sum;
    __syncthreads();
    for (uint32_t d = 1; d < 1024; d <<= 1) {  // inclusive Hillis-Steele scan of the thread sums
        const uint32_t add = threadIdx.x >= d ? part[threadIdx.x - d] : 0;
        __syncthreads();
        part[threadIdx.x] += add;
        __syncthreads();
    }
    uint32_t run = part[threadIdx.x] - sum;
    for (uint32_t k = 0; k < PER; ++k) {
        const uint32_t b = threadIdx.x * PER + k;
        bounds[b] = run;
        cursor[b] = run;
        run += c[k];
        bounds[kOrderBuckets + b] = run;
    }
}

// Each of kOrderPlaceParts parts counts its elements per bucket (its offsets then stay in L2),
// reserves a range of each bucket it uses with one global atomic, and places its elements
// there (rank inside the part by LDS atomics). The order inside a bucket is the
// reservations' arrival order; k_order_sort then orders each bucket by offset.
// IDX: place the indices only; k_order_sort<true> then reads each block's offset through
// its index (half the scattered placement stores, a gathered read in the sort instead).
template <bool IDX = false>
__global__ __launch_bounds__(256) void k_order_place(const uint64_t* __restrict__ offs, uint64_t n,
                                                     uint32_t* __restrict__ cursor, uint32_t* __restrict__ order,
                                                     uint64_t* __restrict__ s_offs) {
    __shared__ uint32_t pos[kOrderBuckets];
    for (uint32_t i = threadIdx.x; i < kOrderBuckets; i += 256) pos[i] = 0;
    __syncthreads();
    uint64_t lo, hi;
    order_part<kOrderPlaceParts>(n, blockIdx.x, &lo, &hi);
    for (uint64_t i = lo + threadIdx.x; i < hi; i += 256) atomicAdd(&pos[order_bucket(offs[i])], 1u);
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < kOrderBuckets; i += 256)
        if (pos[i]) pos[i] = atomicAdd(&cursor[i], pos[i]);
    __syncthreads();
    for (uint64_t i = lo + threadIdx.x; i < hi; i += 256) {
        const uint64_t o = offs[i];
        const uint32_t at = atomicAdd(&pos[order_bucket(o)], 1u);
        order[at] = static_cast<uint32_t>(i);
        if constexpr (!IDX) s_offs[at] = o;  // with the index: k_order_sort reads both in bucket order
    }
}

constexpr uint32_t kOrderSortMax = 2048;
// k_order_sort's counting pass: 1,024 sub-buckets of 32 KiB per 32 MiB region (storm's
// slots: one block each), runs of up to kOrderRunMax entries finished by insertion sort
constexpr uint32_t kOrderSub = 1024, kOrderSubShift = kOrderShift - 10, kOrderRunMax = 16;

// one workgroup per bucket: its entries order[start[b] .. end[b]) sorted by offset (larger
// buckets stay in placement order)
// Sort key: [offset inside the 32 MiB region] [the entry's index in the bucket]. A counting
// pass by 32 KiB sub-bucket orders the entries in a few barriers (a bitonic network over
// 1,024 entries takes 55); the entries of one sub-bucket (one per 32 KiB slot in storm's
// cache.data) are then put in key order by insertion, one thread per sub-bucket. A bucket
// with a sub-bucket of more than kOrderRunMax entries (blocks packed below 2 KiB apart)
// takes the bitonic network instead, one 64-bit compare-exchange per pair per pass. The
// index finds the block's number and offset, kept in LDS. The bucket's offsets (placed
// beside the indices by k_order_place) and lengths are written in the new order too
// (s_offs, s_lens), so the hash kernel reads them sequentially; only the checksum store
// goes through order. Grouping a region's blocks by tile count first (fewer masked rows
// in a wave) measured worse: 0.78 against 0.85 of 8 TB/s on the shuffled storm-length
// gather (profiles/r03k/), address order wins.
template <bool IDX = false>
__global__ __launch_bounds__(256) void k_order_sort(const uint32_t* __restrict__ lens, const uint32_t* __restrict__ bounds,
                                                    uint32_t* __restrict__ order, uint64_t* __restrict__ s_offs,
                                                    uint32_t* __restrict__ s_lens, const uint64_t* __restrict__ offs) {
    static_assert(kOrderSortMax <= 2048 && kOrderShift + 11 <= 64, "key fields");
    static_assert(kOrderSub == 4 * 256, "four sub-buckets per thread");
    __shared__ uint64_t key[kOrderSortMax];
    __shared__ uint64_t off[kOrderSortMax];
    __shared__ uint32_t val[kOrderSortMax];
    __shared__ uint32_t hist[kOrderSub];
    __shared__ uint32_t first[kOrderSub];
    __shared__ uint16_t at[kOrderSortMax];
    __shared__ uint32_t wsum[4], longest;
    const uint32_t tid = threadIdx.x;
    const uint32_t lo = bounds[blockIdx.x], cnt = bounds[kOrderBuckets + blockIdx.x] - lo;
    if (cnt > kOrderSortMax) {  // left in placement order
        if (lens || IDX)
            for (uint32_t i = tid; i < cnt; i += 256) {
                const uint32_t v = order[lo + i];
                if (lens) s_lens[lo + i] = lens[v];
                if constexpr (IDX) s_offs[lo + i] = offs[v];
            }
        return;
    }
    constexpr uint64_t kRegion = (uint64_t{1} << kOrderShift) - 1;
    for (uint32_t i = tid; i < kOrderSub; i += 256) hist[i] = 0;
    if (tid == 0) longest = 0;
    __syncthreads();
    for (uint32_t i = tid; i < cnt; i += 256) {
        const uint32_t v = order[lo + i];
        const uint64_t o = IDX ? offs[v] : s_offs[lo + i];
        val[i] = v;
        off[i] = o;
        key[i] = ((o & kRegion) << 11) | i;
        atomicAdd(&hist[static_cast<uint32_t>((o & kRegion) >> kOrderSubShift)], 1u);
    }
    __syncthreads();  // (every thread's reads of s_offs and order are done before the writes below)
    // exclusive scan of the sub-bucket counts, four per thread, and the longest run
    uint32_t c[4], mine = 0, run = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        c[k] = hist[4 * tid + k];
        mine += c[k];
        run = max(run, c[k]);
    }
    const uint32_t lane = tid & 63, w = tid >> 6;
    uint32_t inc = mine;
    for (uint32_t d = 1; d < 64; d <<= 1) {
        const uint32_t up = static_cast<uint32_t>(__shfl_up(static_cast<int>(inc), d));
        if (lane >= d) inc += up;
    }
    if (lane == 63) wsum[w] = inc;
    atomicMax(&longest, run);
    __syncthreads();
    if (longest <= kOrderRunMax) {
        uint32_t base = inc - mine;
        for (uint32_t v = 0; v < w; ++v) base += wsum[v];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            first[4 * tid + k] = base;
            hist[4 * tid + k] = base;  // the sub-bucket's next place
            base += c[k];
        }
        __syncthreads();
        for (uint32_t i = tid; i < cnt; i += 256)
            at[atomicAdd(&hist[static_cast<uint32_t>((off[i] & kRegion) >> kOrderSubShift)], 1u)] =
                static_cast<uint16_t>(i);
        __syncthreads();
        // each sub-bucket's entries [first, hist) in key order (insertion; at most kOrderRunMax)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t s0 = first[4 * tid + k], s1 = hist[4 * tid + k];
            for (uint32_t a = s0 + 1; a < s1; ++a) {
                const uint16_t e = at[a];
                const uint64_t ke = key[e];
                uint32_t b = a;
                for (; b > s0 && key[at[b - 1]] > ke; --b) at[b] = at[b - 1];
                at[b] = e;
            }
        }
        __syncthreads();
        for (uint32_t i = tid; i < cnt; i += 256) {
            const uint32_t e = at[i];
            const uint32_t v = val[e];
            order[lo + i] = v;
            s_offs[lo + i] = off[e];
            if (lens) s_lens[lo + i] = lens[v];
        }
        return;
    }
    // bitonic network over the keys (padded to a power of two with the largest key)
    uint32_t m = 2;
    while (m < cnt) m <<= 1;
    for (uint32_t i = cnt + tid; i < m; i += 256) key[i] = ~uint64_t{0};
    __syncthreads();
    for (uint32_t k = 2; k <= m; k <<= 1) {
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t t = tid; t < m / 2; t += 256) {
                const uint32_t i = 2 * j * (t / j) + t % j, p = i + j;
                const uint64_t a = key[i], cc = key[p];
                if ((a > cc) == ((i & k) == 0)) {
                    key[i] = cc;
                    key[p] = a;
                }
            }
            __syncthreads();
        }
    }
    for (uint32_t i = tid; i < cnt; i += 256) {
        const uint32_t e = static_cast<uint32_t>(key[i]) & 2047;
        const uint32_t v = val[e];
        order[lo + i] = v;
        s_offs[lo + i] = off[e];
        if (lens) s_lens[lo + i] = lens[v];
    }
}

// The checksums of a locality-ordered gather hashed into their sorted positions, then
// moved to the caller's indices in one pass: out[order[k]] = s_out[k].
__global__ __launch_bounds__(256) void k_order_scatter(const uint32_t* __restrict__ order,
                                                       const uint64_t* __restrict__ s_out, uint64_t* __restrict__ out,
                                                       uint64_t n) {
    for (uint64_t k = blockIdx.x * 256ull + threadIdx.x; k < n; k += gridDim.x * 256ull) out[order[k]] = s_out[k];
}

// Rows of a group by length, rotated per workgroup step (round 4; probe build only: it
// measured 0.794 against 0.848 of 8 TB/s for address order, profiles/r04_gather_rank/).
// A wave streams as many
// tiles as the longest of its 16 blocks, so with storm's four leaf lengths mixed at random
// nearly every wave runs 64 tiles while its blocks average 60.75. Here the 128 blocks of a
// group stay the same set (the group's address window is unchanged): they are only
// re-dealt to rows so that each wave gets 16 blocks of adjacent length ranks, and the
// rank slice a wave gets rotates with the workgroup's group counter k = g / G (the
// persistent kernel's groups g, g + G, ...), so over 8 groups every wave gets every
// slice once and the waves of a workgroup stay together. Within a slice, ties keep the
// address order. Full groups only; the last partial group is left as it is. One
// workgroup of 128 threads per group.
#ifdef STORMCK_PROBES
__global__ __launch_bounds__(128) void k_order_rank(uint32_t* __restrict__ order, uint64_t* __restrict__ s_offs,
                                                    uint32_t* __restrict__ s_lens, uint64_t G) {
    __shared__ uint32_t len[128], ord[128];
    __shared__ uint64_t off[128];
    const uint32_t t = threadIdx.x;
    const uint64_t g = blockIdx.x, at = g * 128 + t;
    len[t] = s_lens[at];
    ord[t] = order[at];
    off[t] = s_offs[at];
    __syncthreads();
    const uint32_t mine = len[t];
    uint32_t rank = 0;
    for (uint32_t u = 0; u < 128; ++u) {
        const uint32_t l = len[u];
        rank += (l < mine) || (l == mine && u < t);
    }
    const uint32_t k = static_cast<uint32_t>((g / G) & 7);
    const uint32_t wave = ((rank >> 4) + 8 - k) & 7;
    const uint64_t to = g * 128 + wave * 16 + (rank & 15);
    order[to] = ord[t];
    s_offs[to] = off[t];
    s_lens[to] = mine;
}
#endif

// The stripes of a block that k_xxh64_glds_var did not stage (a start that is not 16-byte
// aligned), straight from global memory. Out of line: the kernel's hot loop stays compact.
__device__ __noinline__ uint64_t var_stripes_from_global(const uint8_t* p, uint32_t nst, uint32_t j, uint64_t acc) {
    if ((reinterpret_cast<uintptr_t>(p) & 7) == 0)
        return quad_stripes_aligned<16>(reinterpret_cast<const uint64_t*>(p) + j, nst, acc);
    return quad_stripes_unaligned(p + 8 * j, nst, acc);
}

// ORD: offs and lens are in a locality order of a large gather (k_order_*, s_offs /
// s_lens), and order[i] is the index of the i-th block: its checksum's slot.
// CONTIG (probe build): a persistent workgroup takes a contiguous run of groups instead of
// every G-th group.
template <int T, int AUX, bool VERIFY, int WAVES, int SKEW, bool LENS, bool OFFS, bool ORD = false, bool CONTIG = false>
__global__ __launch_bounds__(64 * WAVES) void k_xxh64_glds_var(const uint8_t* __restrict__ base, uint64_t stride,
                                                               const uint32_t* __restrict__ lens, uint32_t len,
                                                               const uint64_t* __restrict__ offs, uint64_t n,
                                                               uint64_t* __restrict__ out,
                                                               const uint64_t* __restrict__ expected,
                                                               unsigned long long* __restrict__ first_bad,
                                                               unsigned long long* __restrict__ n_bad,
                                                               const uint32_t* __restrict__ order = nullptr) {
    constexpr int BPW = 16 * WAVES;
    constexpr int ROW = 32 * T;
    constexpr int TILE = BPW * ROW;
    constexpr int INSTR = TILE / 1024;
    constexpr int PER_WAVE = INSTR / WAVES;
    static_assert(INSTR % WAVES == 0 && T % 2 == 0 && WAVES <= 8, "a wave's pieces must be its own block rows");
    // the ring, then the count of waves whose stream has ended (in the same array: a
    // second __shared__ array makes hipcc guard ds_reads after an LDS-DMA with vmcnt(0),
    // k_commit_level_glds)
    __shared__ __attribute__((aligned(16))) uint8_t lds[2 * TILE + 16];
    uint32_t* n_finished = reinterpret_cast<uint32_t*>(lds + 2 * TILE);

    const uint32_t tid = threadIdx.x;
    const uint32_t wave = tid >> 6, lane = tid & 63;
    const uint64_t ngroups = (n + BPW - 1) / BPW;
    const uint64_t G = gridDim.x;
    // this workgroup's groups: g_first, g_step(g_first), ... below g_end
    const uint64_t g_per = CONTIG ? (ngroups + G - 1) / G : 0;
    const uint64_t g_first = CONTIG ? blockIdx.x * g_per : blockIdx.x;
    const uint64_t g_end = CONTIG ? min(ngroups, g_first + g_per) : ngroups;
    auto g_step = [&](uint64_t g) { return CONTIG ? g + 1 : g + G; };
    if (g_first >= g_end) return;
    const uint64_t ph = static_cast<uint64_t>(wave) * SKEW;  // this wave's start delay
    if (tid == 0) *n_finished = 0;
    __syncthreads();  // before any wave can finish

    auto block_ptr = [&](uint64_t gb) -> const uint8_t* { return base + (OFFS ? offs[gb] : gb * stride); };
    auto staged_bytes = [](const uint8_t* p, uint32_t L) -> uint32_t {  // stripe bytes through LDS, 0 = none
        return (reinterpret_cast<uintptr_t>(p) & 15) == 0 ? (L >> 5) * 32 : 0;
    };
    auto wave_max = [](uint32_t v) {
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) v = max(v, static_cast<uint32_t>(__shfl_xor(static_cast<int>(v), m)));
        return v;
    };

    // ---- issue side: piece k of this lane is row prow[k] of the group, source byte pofs[k]
    uint32_t prow[PER_WAVE], pofs[PER_WAVE];
#pragma unroll
    for (int k = 0; k < PER_WAVE; ++k) {
        const uint32_t off = (wave * PER_WAVE + k) * 1024 + lane * 16;
        const uint32_t b = off / ROW, q = (off % ROW) / 16;
        prow[k] = b;
        pofs[k] = ((q + glds_rot<T>(b)) % (2 * T)) * 16;
    }
    const uint8_t* i_src[PER_WAVE];
    uint32_t i_lim[PER_WAVE];
    const uint8_t* i_np[PER_WAVE];  // next group, prefetched
    uint32_t i_nl[PER_WAVE];
    auto i_fetch = [&](uint64_t g) __attribute__((always_inline)) {
#pragma unroll
        for (int k = 0; k < PER_WAVE; ++k) {
            const uint64_t gb = g * BPW + prow[k];
            const bool live = g < g_end && gb < n;
            const uint64_t gc = live ? gb : 0;
            // unconditional loads (clamped index): a load under a branch gets its own
            // vmcnt(0) wait, which would serialise the 2 * PER_WAVE loads
            const uint32_t l = LENS ? lens[gc] : len;
            i_np[k] = block_ptr(gc);
            i_nl[k] = live ? l : 0;
        }
    };
    uint64_t ig = g_first;
    [[maybe_unused]] uint32_t it = 0;  // tile of group ig to issue next (used by the device pass)
    uint32_t i_ntl = 0;
    [[maybe_unused]] uint32_t i_full = 0;  // whole-tile stripe bytes of every block (device pass)
    bool i_done = false;
    auto i_switch = [&]() __attribute__((always_inline)) {  // make the prefetched group current, prefetch the one after
        uint32_t tiles = 0, lim_min = 0xffffffffu;
#pragma unroll
        for (int k = 0; k < PER_WAVE; ++k) {
            i_src[k] = i_np[k] + pofs[k];
            i_lim[k] = staged_bytes(i_np[k], i_nl[k]);
            tiles = max(tiles, (i_lim[k] + ROW - 1) / ROW);
            lim_min = min(lim_min, i_lim[k]);
        }
        i_ntl = wave_max(tiles);
        // stripe bytes every block of the wave has, in whole tiles: tiles below it are full
        i_full = ~wave_max(~lim_min) / ROW * ROW;
        i_fetch(g_step(ig));
    };
    auto i_next_group = [&]() __attribute__((always_inline)) {  // the next group with tiles for this wave
        for (;;) {
            ig = g_step(ig);
            if (ig >= g_end) {
                i_done = true;
                return;
            }
            i_switch();
            if (i_ntl > 0) return;
        }
    };
    i_fetch(ig);
    i_switch();
    if (i_ntl == 0) i_next_group();
#if defined(__HIP_DEVICE_COMPILE__)
    // a tile every piece of the wave has (all its blocks still have >= a whole tile left)
    // issues unmasked, as k_xxh64_glds_skew; a block's partial last tile masks by piece
#define STORMCK_GLDS_VAR_ISSUE(SLOT)                                                                   \
    do {                                                                                               \
        uint8_t* dst_ = lds + (SLOT) * TILE + wave * PER_WAVE * 1024;                                  \
        const uint32_t t0_ = it * ROW;                                                                 \
        if (__builtin_expect(t0_ + ROW <= i_full, 1)) {                                                \
            _Pragma("unroll") for (int k_ = 0; k_ < PER_WAVE; ++k_)                                    \
                __builtin_amdgcn_global_load_lds(i_src[k_] + t0_, dst_ + k_ * 1024, 16, 0, AUX);      \
        } else {                                                                                       \
            _Pragma("unroll") for (int k_ = 0; k_ < PER_WAVE; ++k_) if (t0_ + pofs[k_] < i_lim[k_])    \
                __builtin_amdgcn_global_load_lds(i_src[k_] + t0_, dst_ + k_ * 1024, 16, 0, AUX);      \
        }                                                                                              \
        ++it;                                                                                          \
    } while (0)
#else
#define STORMCK_GLDS_VAR_ISSUE(SLOT) do { } while (0)
#endif

    // ---- hash side: quad (b, j) hashes row b of each group
    const uint32_t b = tid >> 2, j = tid & 3;
    const uint32_t rot = glds_rot<T>(b);
    const uint8_t* h_np = nullptr;  // next group, prefetched
    uint32_t h_nl = 0;
    uint64_t h_nidx = 0;  // the block's index (its checksum's slot)
    bool h_nlive = false;
    auto h_fetch = [&](uint64_t g) __attribute__((always_inline)) {
        const uint64_t gb = g * BPW + b;
        h_nlive = g < g_end && gb < n;
        const uint64_t gc = h_nlive ? gb : 0;
        const uint32_t l = LENS ? lens[gc] : len;  // unconditional, as i_fetch
        h_np = block_ptr(gc);
        h_nl = h_nlive ? l : 0;
        h_nidx = ORD ? order[gc] : gc;
    };
    uint64_t hg = g_first;
    uint32_t ht = 0, h_ntl = 0, h_L = 0, h_nst = 0, h_sst = 0;
    uint64_t h_idx = 0;
    const uint8_t* h_p = nullptr;
    bool h_live = false, h_done = false;
    uint64_t acc = acc_seed(j);
    // the tail (< 32 bytes after the last stripe) of a staged block, loaded when its group
    // starts: 8-byte-aligned words that hold a tail byte (never past the page of the
    // block's last byte); the other addresses read a word of out / expected, unused
    uint64_t tail[4] = {0, 0, 0, 0};
    const uint8_t* safe = VERIFY ? reinterpret_cast<const uint8_t*>(expected) : reinterpret_cast<const uint8_t*>(out);
    auto h_switch = [&]() __attribute__((always_inline)) {
        h_p = h_np;
        h_L = h_nl;
        h_live = h_nlive;
        h_idx = h_nidx;
        h_nst = h_L >> 5;
        const uint32_t sb = staged_bytes(h_p, h_L);
        h_sst = sb >> 5;  // stripes through LDS (h_nst, or 0 if not staged)
        h_ntl = wave_max((sb + ROW - 1) / ROW);
        acc = acc_seed(j);
        const uint32_t rem = h_L & 31;
        const uint8_t* t = h_p + 32 * static_cast<uint64_t>(h_nst);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const bool use = j == 0 && sb > 0 && 8u * q < rem;  // (sb > 0: 16-byte aligned start)
            tail[q] = *reinterpret_cast<const uint64_t*>(use ? t + 8 * q : safe);
        }
        h_fetch(g_step(hg));
    };
    auto h_finish = [&]() __attribute__((always_inline)) {  // the group's blocks are complete: unstaged stripes, tail, checksum
        if (__builtin_expect(h_sst < h_nst, 0)) acc = var_stripes_from_global(h_p, h_nst, j, acc);
        const uint64_t v1 = quad_bcast<0>(acc), v2 = quad_bcast<1>(acc), v3 = quad_bcast<2>(acc), v4 = quad_bcast<3>(acc);
        if (j == 0 && h_live) {
            const uint64_t gbk = h_idx;
            const uint64_t h0 = (h_L >= 32) ? converge(v1, v2, v3, v4) : kP5;
            const uint64_t h = h_sst == h_nst && h_L >= 32 ? finish_regs(h0, h_L, tail, h_L & 31)
                                                           : finish_fast(h0, h_L, h_p + 32 * static_cast<uint64_t>(h_nst), h_L & 31);
            if constexpr (VERIFY) {
                if (h != expected[gbk]) {
                    atomicMin(first_bad, static_cast<unsigned long long>(gbk));
                    atomicAdd(n_bad, 1ULL);
                }
            } else {
                out[gbk] = h;
            }
        }
    };
    auto h_next_group = [&]() __attribute__((always_inline)) {  // finish groups without tiles on the way
        for (;;) {
            hg = g_step(hg);
            if (hg >= g_end) {
                h_done = true;
                // count this wave out; the add lands before the next barrier, after which
                // every wave reads the count
                if (lane == 0) __hip_atomic_fetch_add(n_finished, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                wait_lgkm0();
                return;
            }
            h_switch();
            if (h_ntl > 0) return;
            h_finish();
        }
    };
    h_fetch(hg);
    h_switch();
    if (h_ntl == 0) {
        h_finish();
        h_next_group();
    }

    // Each step: wait for this wave's tile, barrier, read the finished-wave count (used at
    // the step's end: every wave read it after the same barrier, so all leave together);
    // then group changes (their loads were prefetched and have landed: the step's
    // vmcnt(0) covered them, where after this step's LDS-DMA issue a use of them would
    // wait for the new tile too), the issue of the next tile into the other slot, and
    // the rounds of this one.
    if (ph == 0 && !i_done) STORMCK_GLDS_VAR_ISSUE(0u);
    bool h_fin = false;  // the current group's last tile is hashed: finish it next step
    for (uint64_t u = 0;; ++u) {
        wait_vmcnt<0>();
        __builtin_amdgcn_s_barrier();
        const uint32_t finished = __hip_atomic_load(n_finished, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (__builtin_expect(h_fin, 0)) {
            h_fin = false;
            h_finish();
            h_next_group();
        }
        if (u + 1 >= ph && !i_done) {
            if (__builtin_expect(it == i_ntl, 0)) {
                it = 0;
                i_next_group();
            }
            if (!i_done) STORMCK_GLDS_VAR_ISSUE((u + 1) & 1);
        }
        if (u >= ph && !h_done) {
            const uint8_t* row = lds + (u & 1) * TILE + b * ROW + (j & 1) * 8;
            const uint32_t s0 = ht * T;
            // all T words read first (the reads stay batched); a full tile takes the plain
            // rounds, the block's last partial tile selects: a predicate on each round
            // would put each LDS read in its own branch and wait for it there
            uint64_t w[T];
#pragma unroll
            for (int s = 0; s < T; ++s) {
                const uint32_t q = (2 * s + (j >> 1) + 2 * T - rot) % (2 * T);
                w[s] = *reinterpret_cast<const uint64_t*>(row + q * 16);
            }
            if (__builtin_expect(s0 + T <= h_sst, 1)) {
#pragma unroll
                for (int s = 0; s < T; ++s) acc = round(acc, w[s]);
            } else {
#pragma unroll
                for (int s = 0; s < T; ++s) {
                    const uint64_t r = round(acc, w[s]);
                    acc = s0 + s < h_sst ? r : acc;
                }
            }
            if (++ht == h_ntl) {
                ht = 0;
                h_fin = true;
            }
        }
        if (finished == WAVES) break;  // every wave's stream had ended before this step's barrier
    }
#undef STORMCK_GLDS_VAR_ISSUE
}

// ---------------------------------------------------------------------------
// Merkle pointer tree: storm pointer.Block nodes (blocks/pointer/block.go:10-13).
// Node bytes: fanout x {Checksum, Address, BirthRevision} (24 B each, LE) then fanout
// BlockType bytes, zero-padded to a multiple of 8 (Go struct size). Words are
// synthesised on the fly from the children; the node never exists in memory.
// ---------------------------------------------------------------------------
__host__ __device__ inline uint32_t pointer_block_size(uint32_t fanout) { return (fanout * 25u + 7u) & ~7u; }

// Children {cs[lo+i], addr_base+lo+i, rev} of one type, i < cnt.
struct LevelWords {
    const uint64_t* cs;
    uint64_t lo, addr_base, rev;
    uint32_t cnt, fanout;
    uint8_t type;
    __device__ __forceinline__ uint64_t operator()(uint32_t k) const {
        const uint32_t pw = 3 * fanout;
        if (k < pw) {
            const uint32_t i = k / 3, f = k - 3 * i;
            if (i >= cnt) return 0;
            return f == 0 ? cs[lo + i] : (f == 1 ? addr_base + lo + i : rev);
        }
        const uint32_t pos = 8 * (k - pw);
        if (pos >= cnt) return 0;
        const uint32_t nb = (cnt - pos) >= 8 ? 8 : (cnt - pos);
        const uint64_t rep = 0x0101010101010101ULL * type;
        return nb == 8 ? rep : (rep & ((1ULL << (8 * nb)) - 1));
    }
};

// Explicit entries (AoS Pointer + type byte), i < cnt.
struct EntryWords {
    const uint64_t* entries;  // 3 u64 per entry
    const uint8_t* types;
    uint32_t cnt, fanout;
    __device__ __forceinline__ uint64_t operator()(uint32_t k) const {
        const uint32_t pw = 3 * fanout;
        if (k < pw) {
            const uint32_t i = k / 3;
            return i < cnt ? entries[k] : 0;
        }
        const uint32_t pos = 8 * (k - pw);
        uint64_t w = 0;
        for (uint32_t b = 0; b < 8; ++b)
            if (pos + b < cnt) w |= static_cast<uint64_t>(types[pos + b]) << (8 * b);
        return w;
    }
};

// XXH64 of a synthesised node by one quad (lane j = accumulator j). Every lane of
// the quad returns the hash. size is a multiple of 8 (no 4-/1-byte tail). Words are
// fetched U stripes ahead (group g+1's child loads in flight while group g hashes):
// fetched one at a time, each round waited for its load, which made a 1,200-way
// level of 14K nodes take 240 us instead of the ~30 us serial XXH64 chain.
// PM: stripe words (k < 4 * nst) come premultiplied by P2; the tail words do not.
template <class W, int U = 16, bool PM = false>
__device__ __forceinline__ uint64_t hash_words_quad(const W& word, uint32_t size, uint32_t j) {
    auto rnd = [](uint64_t a, uint64_t w) { return PM ? round_pm(a, w) : round(a, w); };
    const uint32_t nst = size >> 5;
    uint64_t acc = acc_seed(j);
    const uint32_t ngroups = nst / U;
    uint32_t s = 0;
    if (ngroups > 0) {
        uint64_t wa[U], wb[U];
#pragma unroll
        for (int u = 0; u < U; ++u) wa[u] = word(4 * u + j);
        for (uint32_t g = 1; g < ngroups; ++g) {
#pragma unroll
            for (int u = 0; u < U; ++u) wb[u] = word(4 * (g * U + u) + j);
#pragma unroll
            for (int u = 0; u < U; ++u) acc = rnd(acc, wa[u]);
#pragma unroll
            for (int u = 0; u < U; ++u) wa[u] = wb[u];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc = rnd(acc, wa[u]);
        s = ngroups * U;
    }
    for (; s < nst; ++s) acc = rnd(acc, word(4 * s + j));
    const uint64_t v1 = quad_bcast<0>(acc), v2 = quad_bcast<1>(acc), v3 = quad_bcast<2>(acc), v4 = quad_bcast<3>(acc);
    uint64_t h = (size >= 32) ? converge(v1, v2, v3, v4) : kP5;
    h += size;
    for (uint32_t k = 4 * nst; k < size / 8; ++k) {
        h ^= round(0, word(k));
        h = rotl<27>(h) * kP1 + kP4;
    }
    return avalanche(h);
}

__global__ __launch_bounds__(256) void k_pointer_level(const uint64_t* __restrict__ cs, uint64_t m,
                                                        uint64_t addr_base, uint64_t rev, uint8_t type,
                                                        uint32_t fanout, uint64_t* __restrict__ parent_cs) {
    const uint64_t gtid = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x;
    const uint64_t pj = gtid >> 2;
    const uint64_t pm = (m + fanout - 1) / fanout;
    const uint32_t j = threadIdx.x & 3;
    const uint64_t node = pj < pm ? pj : pm - 1;
    LevelWords w;
    w.cs = cs; w.lo = node * fanout; w.addr_base = addr_base; w.rev = rev; w.fanout = fanout; w.type = type;
    w.cnt = static_cast<uint32_t>((m - w.lo) < fanout ? (m - w.lo) : fanout);
    const uint64_t h = hash_words_quad(w, pointer_block_size(fanout), j);
    if (j == 0 && pj < pm) parent_cs[pj] = h;
}

// Wide levels at a fan-out F that tiles evenly (storm's F = 1200, 30,000 B nodes):
// one wave per 16 nodes, a quad per node, and the node words staged in LDS already
// multiplied by P2, so the chain lanes issue only add, rotate and the P1 multiply.
//
// k_pointer_level above makes every lane synthesise its own word per round: the index
// arithmetic, a field select, an 8-byte child load and the P2 multiply sit in the
// chain's instruction stream (~25 instructions a round, 148 us for the 13,981 nodes
// over 16M leaves). Here the wave instead works tile by tile. A tile is 15 stripes of
// every node = 20 child slots (60 words); the pointer region is F/20 tiles. For each
// tile:
//   * produce: lane l owns 5 (node, slot) items. Their child checksums arrive
//     D tiles ahead in registers (coalesced 8-byte loads: the wave's 16 nodes are
//     contiguous children), and the lane writes {cs*P2, (addr_base+i)*P2, rev*P2}
//     into the tile's LDS ring slot. Address words are linear in i, so each item's
//     premultiplied address advances by 20*P2 per tile (one 64-bit add);
//   * consume: the quads walk the previous tile's 15 rounds from LDS. A node's tile
//     row is 15 stripes (odd), so the 8 quads of a 32-lane ds_read_b64 group hit 8
//     distinct 32-byte bank groups.
// One wave owns its LDS (15 KiB), so no barrier: LDS operations of one wave execute in
// order. The type bytes (37 stripes + the 16-byte tail at F = 1200) are the constant
// type byte for full nodes; only the level's last node can be partial, and the one
// wave that holds it takes the masked variant (FULL = false) of the same code.
// A tile is TS stripes of every node = TS·4/3 child slots. A node's row in LDS is an
// odd number of stripes (TS, or TS+1 for even TS), so the 8 quads of a 32-lane
// ds_read_b64 group hit 8 distinct 32-byte bank groups.
template <uint32_t TS>
struct RingShape {
    static_assert(TS % 3 == 0, "whole child slots per tile");
    static constexpr uint32_t SL = TS * 4 / 3;        // child slots per tile
    static constexpr uint32_t RS = (TS | 1u) * 4;     // words per node row in LDS
};

// The producer side of one wave's 16 nodes: lane `lane` owns IT (node, slot) items of
// every tile, loads their child checksums and writes the premultiplied words.
template <uint32_t F, uint32_t TS_, bool FULL, uint32_t NODES = 16>
struct RingProducer {
    static constexpr uint32_t TS = TS_, SL = RingShape<TS_>::SL, RS = RingShape<TS_>::RS, NT = F / SL,
                              IT = NODES * SL / 64;
    static_assert(F % SL == 0 && IT * 64 == NODES * SL, "tile shape");
    uint32_t pq[IT], pu[IT], cnt_i[IT];
    const uint64_t* gp[IT];
    uint64_t addr_pm[IT];
    uint64_t rev_pm, step_pm;

    __device__ __forceinline__ RingProducer(const uint64_t* __restrict__ cs, uint64_t m, uint64_t pm, uint64_t node0,
                                            uint64_t addr_base, uint64_t rev, uint32_t lane) {
        rev_pm = rev * kP2;
        step_pm = static_cast<uint64_t>(SL) * kP2;
#pragma unroll
        for (uint32_t r = 0; r < IT; ++r) {
            const uint32_t item = lane + 64 * r;
            pq[r] = item / SL;
            pu[r] = item % SL;
            uint64_t node = node0 + pq[r];
            if (!FULL) {
                if (node >= pm) node = pm - 1;  // idle quads of the last wave: hash a copy, store nothing
                const uint64_t left = m - node * F;
                cnt_i[r] = static_cast<uint32_t>(left < F ? left : F);
            }
            const uint64_t g = node * F + pu[r];
            gp[r] = cs + g;
            addr_pm[r] = (addr_base + g) * kP2;
        }
    }
    __device__ __forceinline__ void load(uint32_t t, uint64_t* dst) const {
#pragma unroll
        for (uint32_t r = 0; r < IT; ++r) {
            if (FULL) {
                dst[r] = gp[r][t * SL];
            } else {
                const uint32_t slot = t * SL + pu[r];
                dst[r] = slot < cnt_i[r] ? gp[r][t * SL] : 0;
            }
        }
    }
    __device__ __forceinline__ void produce(uint32_t t, const uint64_t* src, uint64_t (*tile)[RS]) const {
#pragma unroll
        for (uint32_t r = 0; r < IT; ++r) {
            uint64_t* w = &tile[pq[r]][3 * pu[r]];
            const uint64_t a = addr_pm[r] + t * step_pm;
            if (FULL) {
                w[0] = src[r] * kP2;
                w[1] = a;
                w[2] = rev_pm;
            } else {
                const bool valid = t * SL + pu[r] < cnt_i[r];
                w[0] = src[r] * kP2;  // src is 0 for a missing child
                w[1] = valid ? a : 0;
                w[2] = valid ? rev_pm : 0;
            }
        }
    }
};

// After the pointer tiles: the type bytes (stripes 3F/4 .. nst-1, then the tail
// words), the merge and the avalanche; lane 0 of the quad stores the node's checksum.
template <uint32_t F, bool FULL>
__device__ __forceinline__ void ring_finish(uint64_t acc, uint32_t j, uint64_t node, uint64_t pm, uint64_t m,
                                            uint8_t type, uint64_t* __restrict__ parent_cs) {
    constexpr uint32_t kSize = (F * 25u + 7u) & ~7u, kWords = kSize / 8, kNst = kSize / 32;
    constexpr uint32_t kPtrStripes = 3 * F / 4;
    const uint64_t rep = 0x0101010101010101ULL * type;
    uint32_t cnt = F;
    if (!FULL) {
        const uint64_t nn = node < pm ? node : pm - 1;
        const uint64_t left = m - nn * F;
        cnt = static_cast<uint32_t>(left < F ? left : F);
    }
    auto type_word = [&](uint32_t k) -> uint64_t {  // k: word index within the type region
        if (FULL) return rep;
        const uint32_t pos = 8 * k;
        if (pos >= cnt) return 0;
        const uint32_t nb = (cnt - pos) >= 8 ? 8 : (cnt - pos);
        return nb == 8 ? rep : (rep & ((1ULL << (8 * nb)) - 1));
    };
    if (FULL) {
        const uint64_t rep_pm = rep * kP2;
        for (uint32_t s = kPtrStripes; s < kNst; ++s) acc = round_pm(acc, rep_pm);
    } else {
        for (uint32_t s = kPtrStripes; s < kNst; ++s) acc = round(acc, type_word(4 * (s - kPtrStripes) + j));
    }
    const uint64_t v1 = quad_bcast<0>(acc), v2 = quad_bcast<1>(acc), v3 = quad_bcast<2>(acc), v4 = quad_bcast<3>(acc);
    uint64_t h = converge(v1, v2, v3, v4) + kSize;
    for (uint32_t k = 4 * kNst; k < kWords; ++k) {
        h ^= round(0, type_word(k - 3 * F));
        h = rotl<27>(h) * kP1 + kP4;
    }
    h = avalanche(h);
    if (j == 0 && node < pm) parent_cs[node] = h;
}

// Producer / consumer waves (k_pointer_level_pc): C chain waves and C producer waves
// per workgroup; producer wave C+i writes the premultiplied tiles of chain wave i's
// 16 nodes, and the quads of the chain waves walk them, so a chain wave's instruction
// stream holds only the LDS reads and the add / rotate / P1 multiply. One barrier per
// tile: tile t+1 is written (slot (t+1)&1) while tile t is read (slot t&1); the
// barrier after both orders the next reuse of each slot.
template <uint32_t F, uint32_t TS_, int D, int C, bool FULL>
__device__ __forceinline__ void pointer_level_pc_body(const uint64_t* __restrict__ cs, uint64_t m, uint64_t pm,
                                                      uint64_t node0, uint64_t addr_base, uint64_t rev, uint8_t type,
                                                      uint64_t* __restrict__ parent_cs,
                                                      uint64_t (*ring)[16 * C][RingShape<TS_>::RS], uint32_t wave) {
    using P = RingProducer<F, TS_, FULL>;
    constexpr uint32_t TS = P::TS, NT = P::NT, IT = P::IT;
    static_assert(NT % D == 0 && D % 2 == 0, "tile shape / static ring slots");
    const uint32_t lane = threadIdx.x & 63;
    if (wave >= C) {  // producer wave for chain wave (wave - C)
        const uint32_t pair = wave - C;
        const P prod(cs, m, pm, node0 + 16 * pair, addr_base, rev, lane);
        uint64_t raw[D][IT];
        auto tile = [&](int slot) { return reinterpret_cast<uint64_t(*)[P::RS]>(&ring[slot][16 * pair][0]); };
#pragma unroll
        for (int d = 0; d < D; ++d) prod.load(d, raw[d]);
        prod.produce(0, raw[0], tile(0));
        prod.load(D, raw[0]);
        __syncthreads();
        for (uint32_t t0 = 0; t0 < NT; t0 += D) {
#pragma unroll
            for (int d = 0; d < D; ++d) {
                const uint32_t t = t0 + d;
                const int nb = (d + 1) % D;
                if (t + 1 < NT) {
                    prod.produce(t + 1, raw[nb], tile((d + 1) & 1));
                    if (t + 1 + D < NT) prod.load(t + 1 + D, raw[nb]);
                }
                __syncthreads();
            }
        }
    } else {  // chain wave
        const uint32_t q = wave * 16 + (lane >> 2), j = lane & 3;
        uint64_t acc = acc_seed(j);
        __syncthreads();
        for (uint32_t t0 = 0; t0 < NT; t0 += D) {
#pragma unroll
            for (int d = 0; d < D; ++d) {
                const uint64_t* row = &ring[d & 1][q][j];
#pragma unroll
                for (uint32_t s = 0; s < TS; ++s) acc = round_pm(acc, row[4 * s]);
                __syncthreads();
            }
        }
        ring_finish<F, FULL>(acc, j, node0 + q, pm, m, type, parent_cs);
    }
}

// Role of a wave in a workgroup of 2C waves: chain waves must not share a SIMD with each
// other, since a chain is bounded by its wave's VALU issue (DESIGN_LOG.md §5, "Merkle tree
// per step"). With SIMD roles, every wave reads the SIMD it was placed on (HW_ID bits
// 5:4) and takes a rank among the workgroup's waves on that SIMD; the waves are then
// ordered by (rank, SIMD) and the first C of that order are the chain waves. So the
// chains land on C distinct SIMDs whenever the dispatcher spreads the workgroup's
// waves over at least C of them, whatever order it placed them in. Without SIMD roles
// the role is the wave index (chain waves first).
template <bool SIMDROLE>
__device__ __forceinline__ uint32_t pc_role(uint32_t* simd_cnt) {
    const uint32_t wave = threadIdx.x >> 6;
    if (!SIMDROLE) return wave;
    if (threadIdx.x < 4) simd_cnt[threadIdx.x] = 0;
    __syncthreads();
    uint32_t hwid;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));
    const uint32_t simd = (hwid >> 4) & 3;
    uint32_t rank = 0;
    if ((threadIdx.x & 63) == 0) rank = atomicAdd(&simd_cnt[simd], 1u);
    rank = __builtin_amdgcn_readfirstlane(rank);
    __syncthreads();
    uint32_t pos = 0;
#pragma unroll
    for (uint32_t s = 0; s < 4; ++s) {
        const uint32_t c = simd_cnt[s];
        pos += (c < rank ? c : rank) + ((s < simd && c > rank) ? 1u : 0u);
    }
    return pos;
}

template <uint32_t F, uint32_t TS, int D, int C, bool SIMDROLE = false>
__global__ __launch_bounds__(128 * C) void k_pointer_level_pc(const uint64_t* __restrict__ cs, uint64_t m,
                                                              uint64_t addr_base, uint64_t rev, uint8_t type,
                                                              uint64_t* __restrict__ parent_cs) {
    __shared__ uint64_t ring[2][16 * C][RingShape<TS>::RS];  // two tiles per chain wave
    __shared__ uint32_t simd_cnt[4];
    const uint32_t role = pc_role<SIMDROLE>(simd_cnt);
    const uint64_t pm = (m + F - 1) / F;
    const uint64_t node0 = static_cast<uint64_t>(blockIdx.x) * 16 * C;
    if (node0 + 16 * C <= m / F)  // workgroup-uniform
        pointer_level_pc_body<F, TS, D, C, true>(cs, m, pm, node0, addr_base, rev, type, parent_cs, ring, role);
    else
        pointer_level_pc_body<F, TS, D, C, false>(cs, m, pm, node0, addr_base, rev, type, parent_cs, ring, role);
}

// Small levels (a handful of nodes, e.g. the top of a shard tree): one workgroup per
// node. All 256 threads synthesise the node's words into LDS at once, then quad 0
// hashes from LDS. A quad synthesising its own words issues ~25 instructions per
// round where hashing alone needs ~11, and a lone wave is issue-bound: 75 us per
// 30,000 B node against ~26 us for the bare XXH64 chain. Nodes up to kNodeLds bytes.
constexpr uint32_t kNodeLds = 32768;
struct LdsWords {
    const uint64_t* p;
    __device__ __forceinline__ uint64_t operator()(uint32_t k) const { return p[k]; }
};

template <class W>
__device__ __forceinline__ void hash_node_wide(const W& w, uint32_t size, uint64_t* __restrict__ out) {
    __shared__ uint64_t node[kNodeLds / 8];
    const uint32_t words = size / 8, nw = 4 * (size >> 5);
    for (uint32_t k = threadIdx.x; k < words; k += blockDim.x) node[k] = k < nw ? w(k) * kP2 : w(k);
    __syncthreads();
    if (threadIdx.x < 4) {
        const uint64_t h = hash_words_quad<LdsWords, 16, true>(LdsWords{node}, size, threadIdx.x);
        if (threadIdx.x == 0) *out = h;
    }
}

__global__ __launch_bounds__(256) void k_pointer_level_wide(const uint64_t* __restrict__ cs, uint64_t m,
                                                             uint64_t addr_base, uint64_t rev, uint8_t type,
                                                             uint32_t fanout, uint64_t* __restrict__ parent_cs) {
    LevelWords w;
    w.cs = cs; w.lo = static_cast<uint64_t>(blockIdx.x) * fanout; w.addr_base = addr_base; w.rev = rev;
    w.fanout = fanout; w.type = type;
    w.cnt = static_cast<uint32_t>((m - w.lo) < fanout ? (m - w.lo) : fanout);
    hash_node_wide(w, pointer_block_size(fanout), parent_cs + blockIdx.x);
}

__global__ __launch_bounds__(256) void k_pointer_node(const uint64_t* __restrict__ entries,
                                                       const uint8_t* __restrict__ types, uint32_t cnt,
                                                       uint32_t fanout, uint64_t* __restrict__ out_cs) {
    EntryWords w{entries, types, cnt, fanout};
    const uint32_t size = pointer_block_size(fanout);
    if (size <= kNodeLds) {
        hash_node_wide(w, size, out_cs);
    } else if (threadIdx.x < 4) {
        const uint64_t h = hash_words_quad(w, size, threadIdx.x);
        if (threadIdx.x == 0) *out_cs = h;
    }
}

__global__ __launch_bounds__(256) void k_pack_pointer_blocks(const uint64_t* __restrict__ cs, uint64_t m,
                                                              uint64_t addr_base, uint64_t rev, uint8_t type,
                                                              uint32_t fanout, uint8_t* __restrict__ dst,
                                                              uint64_t dst_stride) {
    const uint32_t words = pointer_block_size(fanout) / 8;
    const uint64_t pm = (m + fanout - 1) / fanout;
    const uint64_t total = pm * words;
    for (uint64_t t = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x; t < total;
         t += static_cast<uint64_t>(gridDim.x) * 256) {
        const uint64_t node = t / words;
        const uint32_t k = static_cast<uint32_t>(t - node * words);
        LevelWords w;
        w.cs = cs; w.lo = node * fanout; w.addr_base = addr_base; w.rev = rev; w.fanout = fanout; w.type = type;
        w.cnt = static_cast<uint32_t>((m - w.lo) < fanout ? (m - w.lo) : fanout);
        reinterpret_cast<uint64_t*>(dst + node * dst_stride)[k] = w(k);
    }
}

// root = {cs ? cs[0] : 0, addr, rev} of `type` (1-entry level, or the empty tree).
__global__ void k_set_root(const uint64_t* __restrict__ cs, uint64_t addr, uint64_t rev, uint8_t type,
                           uint64_t* __restrict__ root, uint8_t* __restrict__ root_type) {
    if (threadIdx.x == 0) {
        root[0] = cs ? cs[0] : 0;
        root[1] = addr;
        root[2] = rev;
        *root_type = type;
    }
}

// Multi-GPU combine (stormck_merkle_root_multi): after the gather, shard s's root row
// {cs, addr, rev, type} is table row map[s]; the combining node's entries are those rows in
// shard order (what k_pointer_node hashes).
__global__ void k_gather_root_rows(const uint64_t* __restrict__ table, const uint32_t* __restrict__ map,
                                   uint32_t count, uint64_t* __restrict__ entries, uint8_t* __restrict__ types) {
    for (uint32_t s = threadIdx.x; s < count; s += blockDim.x) {
        const uint64_t* row = table + 4ull * map[s];
        entries[3ull * s] = row[0];
        entries[3ull * s + 1] = row[1];
        entries[3ull * s + 2] = row[2];
        types[s] = static_cast<uint8_t>(row[3]);
    }
}

// ---------------------------------------------------------------------------
// f1: one level of a level-synchronous commit. blocks[lo, lo + cnt) are this level's
// dirty records in commit order (the host lays them out so; they may sit in pinned
// host memory, read over PCIe). Quad per dirty block: hash the block's bytes (gather
// by data_offset, per-block length), then lane 0 performs storm's PostCommitFunc
// (cache/trace.go:274-320): Pointer{cs, address, birth_revision} into the parent's
// origin slot and the block type into the origin type byte. Origins belong to blocks
// of later levels (parents), which this launch never reads. out_cs[lo + k] = checksum.
// ---------------------------------------------------------------------------
// Small f1 levels (the pointer blocks above the leaves, the root, a short commit): one
// workgroup per dirty block, as k_xxh64_wide. The block is staged into LDS in one round
// trip with its stripe words premultiplied by P2 (8-byte-aligned starts; others and
// blocks over 32 KiB hash from memory), then quad 0 walks the chain and lane 0 performs
// the PostCommitFunc store, as k_commit_level.
__global__ __launch_bounds__(256) void k_commit_level_wide(uint8_t* __restrict__ arena,
                                                            const stormck_dirty_block* __restrict__ blocks,
                                                            uint64_t lo, uint64_t* __restrict__ out_cs) {
    __shared__ uint4 buf[kWideMax / 16];
    const uint64_t k = lo + blockIdx.x;
    const stormck_dirty_block b = blocks[k];
    const uint8_t* src = arena + b.data_offset;
    const uint32_t L = b.length;
    const uint32_t nst = L >> 5;
    const uint32_t shift = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(src) & 15);
    const uint32_t words = (shift + L + 15) / 16;
    const uint32_t j = threadIdx.x;
    uint64_t acc = acc_seed(j & 3);
    const uint8_t* s;
    if ((shift & 7) == 0 && words <= kWideMax / 16) {  // uniform over the workgroup
        stage_pm_switch<8>(reinterpret_cast<const uint4*>(src - shift), buf, words, shift / 8, 4 * nst);
        __syncthreads();
        if (j >= 4) return;
        s = reinterpret_cast<const uint8_t*>(buf) + shift;
        acc = quad_stripes_aligned<16, false, true>(reinterpret_cast<const uint64_t*>(s) + j, nst, acc);
    } else {
        if (j >= 4) return;
        s = src;
        if ((reinterpret_cast<uintptr_t>(s) & 7) == 0)
            acc = quad_stripes_aligned<16>(reinterpret_cast<const uint64_t*>(s) + j, nst, acc);
        else
            acc = quad_stripes_unaligned(s + 8 * j, nst, acc);
    }
    const uint64_t v1 = quad_bcast<0>(acc), v2 = quad_bcast<1>(acc), v3 = quad_bcast<2>(acc), v4 = quad_bcast<3>(acc);
    if (j == 0) {
        const uint64_t h0 = (L >= 32) ? converge(v1, v2, v3, v4) : kP5;
        const uint64_t h = finish_fast(h0, L, s + 32 * static_cast<uint64_t>(nst), L & 31);
        out_cs[k] = h;
        if (b.origin_pointer != STORMCK_NO_ORIGIN) {
            uint64_t* p = reinterpret_cast<uint64_t*>(arena + b.origin_pointer);
            p[0] = h;
            p[1] = b.address;
            p[2] = b.birth_revision;
            arena[b.origin_type] = b.type;
        }
    }
}

// Mid-size f1 levels (a storm commit's ~1,200 leaves): the wide-multi scheme, BPW dirty
// blocks per workgroup staged premultiplied in one round trip, one chain wave. The
// workgroup's BPW records (56 B each, possibly in pinned host memory) cross the bus
// once, into LDS, before any block address is known.
template <int BPW, uint32_t RING = kRingSlots, uint32_t CP = kChunkPieces, bool DBL = false>
__global__ __launch_bounds__(256) void k_commit_level_multi(uint8_t* __restrict__ arena,
                                                             const stormck_dirty_block* __restrict__ blocks,
                                                             uint64_t lo, uint64_t cnt,
                                                             uint64_t* __restrict__ out_cs,
                                                             uint32_t* __restrict__ fault, uint32_t stall) {
    constexpr uint32_t RW = sizeof(stormck_dirty_block) / 8;  // 7 words per record
    static_assert(RING > 0 ? (BPW * ring_block_pieces(RING, CP) + kRingSlackPieces) * 16 + BPW * RW * 8 <= 150 * 1024
                           : BPW * kMultiPieces * 16 + BPW * RW * 8 <= 160 * 1024,
                  "LDS");
    static_assert(BPW * RW <= 256, "one record word per thread");
    __shared__ uint64_t rec_w[BPW * RW];
    const uint64_t first = static_cast<uint64_t>(blockIdx.x) * BPW;
    const uint32_t nlive = static_cast<uint32_t>(min<uint64_t>(BPW, cnt - first));
    if (threadIdx.x < nlive * RW)
        rec_w[threadIdx.x] = reinterpret_cast<const uint64_t*>(blocks + lo + first)[threadIdx.x];
    __syncthreads();
    const stormck_dirty_block* rec = reinterpret_cast<const stormck_dirty_block*>(rec_w);
    auto src_of = [&](uint32_t b) { return BlockRef{arena + rec[b].data_offset, rec[b].length}; };
    auto emit = [&](uint32_t b, uint64_t h) {
        const stormck_dirty_block& r = rec[b];
        out_cs[lo + first + b] = h;
        if (r.origin_pointer != STORMCK_NO_ORIGIN) {
            uint64_t* p = reinterpret_cast<uint64_t*>(arena + r.origin_pointer);
            p[0] = h;
            p[1] = r.address;
            p[2] = r.birth_revision;
            arena[r.origin_type] = r.type;
        }
    };
    if constexpr (RING > 0) {
        __shared__ uint4 ring[BPW * ring_block_pieces(RING, CP) + kRingSlackPieces];
        __shared__ uint32_t ready[pipe_max_chunks(CP)], done[1], abort_w[1];
        const PipeCtl pc{ready, done, abort_w, fault, kFaultCommitMulti, stall};
        multi_stage_hash_pipe<BPW, RING, CP, DBL>(ring, pc, nlive, src_of, emit, [](uint32_t) {});
    } else {
        __shared__ uint4 buf[BPW * kMultiPieces];
        multi_stage_hash<BPW>(buf, nlive, src_of, emit);
    }
}

template <int U>
__global__ __launch_bounds__(256) void k_commit_level(uint8_t* __restrict__ arena,
                                                       const stormck_dirty_block* __restrict__ blocks, uint64_t lo,
                                                       uint64_t cnt, uint64_t* __restrict__ out_cs) {
    const uint64_t gtid = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x;
    const uint64_t k = gtid >> 2;
    const uint32_t j = threadIdx.x & 3;
    const bool live = k < cnt;
    const uint64_t kk = live ? k : cnt - 1;
    const stormck_dirty_block b = blocks[lo + kk];
    const uint8_t* src = arena + b.data_offset;
    const uint32_t L = b.length;
    const uint32_t nst = L >> 5;
    uint64_t acc = acc_seed(j);
    if ((reinterpret_cast<uintptr_t>(src) & 7) == 0)
        acc = quad_stripes_aligned<U>(reinterpret_cast<const uint64_t*>(src) + j, nst, acc);
    else
        acc = quad_stripes_unaligned(src + 8 * j, nst, acc);
    const uint64_t v1 = quad_bcast<0>(acc), v2 = quad_bcast<1>(acc), v3 = quad_bcast<2>(acc), v4 = quad_bcast<3>(acc);
    if (j == 0 && live) {
        const uint64_t h0 = (L >= 32) ? converge(v1, v2, v3, v4) : kP5;
        const uint64_t h = finish_fast(h0, L, src + 32 * static_cast<uint64_t>(nst), L & 31);
        out_cs[lo + kk] = h;
        if (b.origin_pointer != STORMCK_NO_ORIGIN) {
            uint64_t* p = reinterpret_cast<uint64_t*>(arena + b.origin_pointer);
            p[0] = h;
            p[1] = b.address;
            p[2] = b.birth_revision;
            arena[b.origin_type] = b.type;
        }
    }
}

// ---------------------------------------------------------------------------
// f1 fast path: one commit level through the LDS-DMA ring (the k_xxh64_glds scheme
// with a ring of 2 tiles) for arenas whose block offsets are 16-byte aligned. The
// workgroup's 128 records (7 KiB, possibly in host memory) are first copied into LDS
// with 8-byte loads spread over all threads, so each record crosses the bus once. Blocks
// of a workgroup may differ in length: block b streams floor(nst_b / T) whole tiles,
// the workgroup runs the longest block's tile count, and LDS-DMA lanes of blocks that
// have run out of tiles are switched off (exec mask). With a 2-slot ring every tile
// is waited for with vmcnt(0), so a wave that issued fewer pieces cannot mis-count.
// Remainder stripes and the tail come from global memory; lane 0 of each quad then
// performs the PostCommitFunc store (see k_commit_level).
// ---------------------------------------------------------------------------
template <int T, int AUX, int WAVES>
__global__ __launch_bounds__(64 * WAVES) void k_commit_level_glds(uint8_t* __restrict__ arena,
                                                                   const stormck_dirty_block* __restrict__ blocks,
                                                                   uint64_t lo, uint64_t cnt,
                                                                   uint64_t* __restrict__ out_cs) {
    constexpr int R = 2;
    constexpr int BPW = 16 * WAVES;
    constexpr int ROW = 32 * T;
    constexpr int TILE = BPW * ROW;
    constexpr int INSTR = TILE / 1024;
    constexpr int PER_WAVE = INSTR / WAVES;
    constexpr int RW = sizeof(stormck_dirty_block) / 8;  // 7 words per record
    static_assert(INSTR % WAVES == 0, "tile must split evenly over the waves");
    __shared__ __attribute__((aligned(16))) uint8_t lds[R * TILE];
    // the records sit in ring slot 1 until the first tile is issued into it. (A second
    // __shared__ array makes hipcc guard every ds_read after an LDS-DMA with vmcnt(0),
    // which serialises the ring: 12% slower, measured.)
    uint64_t* rec_lds = reinterpret_cast<uint64_t*>(lds + TILE);
    static_assert(BPW * RW * 8 <= TILE, "records fit in one ring slot");

    const uint32_t tid = threadIdx.x;
    const uint32_t wave = tid >> 6, lane = tid & 63;
    const uint64_t k0 = static_cast<uint64_t>(blockIdx.x) * BPW;  // first level-local block of this workgroup
    const uint32_t nrec = static_cast<uint32_t>(min<uint64_t>(BPW, cnt - k0));
    {
        const uint64_t* src = reinterpret_cast<const uint64_t*>(blocks + lo + k0);
        uint64_t w[(BPW * RW + 64 * WAVES - 1) / (64 * WAVES)];
#pragma unroll
        for (int m = 0; m < (BPW * RW + 64 * WAVES - 1) / (64 * WAVES); ++m) {
            const uint32_t q = tid + m * 64 * WAVES;
            w[m] = q < nrec * RW ? src[q] : 0;
        }
#pragma unroll
        for (int m = 0; m < (BPW * RW + 64 * WAVES - 1) / (64 * WAVES); ++m) {
            const uint32_t q = tid + m * 64 * WAVES;
            if (q < BPW * RW) rec_lds[q] = w[m];
        }
    }
    __syncthreads();
    const stormck_dirty_block* recs = reinterpret_cast<const stormck_dirty_block*>(rec_lds);

    // per-lane LDS-DMA sources: block of each of this wave's PER_WAVE pieces
    const uint8_t* src[PER_WAVE];
    uint32_t ntl[PER_WAVE];
#pragma unroll
    for (int k = 0; k < PER_WAVE; ++k) {
        const uint32_t ii = wave * PER_WAVE + k;
        const uint32_t off = ii * 1024 + lane * 16;
        const uint32_t bb = off / ROW, q = (off % ROW) / 16;
        const uint32_t piece = (q + glds_rot<T>(bb)) % (2 * T);
        const bool plive = bb < nrec;
        const stormck_dirty_block& r = recs[plive ? bb : 0];
        src[k] = arena + r.data_offset + piece * 16;
        ntl[k] = plive ? (r.length >> 5) / T : 0;
    }
    // this lane's hash block (quad) and the workgroup's tile count
    const uint32_t b = tid >> 2, j = tid & 3;
    const uint64_t kb = k0 + b;
    const bool live = b < nrec;
    const stormck_dirty_block rec = recs[live ? b : 0];
    const uint32_t L = rec.length, nst = L >> 5;
    const uint32_t my_tiles = live ? nst / T : 0;
    uint32_t wg_tiles = my_tiles;
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) wg_tiles = max(wg_tiles, static_cast<uint32_t>(__shfl_xor(static_cast<int>(wg_tiles), m)));
    uint32_t* red = reinterpret_cast<uint32_t*>(lds);
    if (lane == 0) red[wave] = wg_tiles;
    __syncthreads();
    wg_tiles = 0;
    for (int w = 0; w < WAVES; ++w) wg_tiles = max(wg_tiles, red[w]);
    __syncthreads();  // the reduction slots are reused by the ring

    const uint32_t rot = glds_rot<T>(b);
    uint64_t acc = acc_seed(j);
#if defined(__HIP_DEVICE_COMPILE__)
#define STORMCK_GLDS_ISSUE_MASKED(T_, SLOT)                                                              \
    do {                                                                                              \
        uint8_t* dst_ = lds + (SLOT) * TILE + wave * PER_WAVE * 1024;                                \
        _Pragma("unroll") for (int k_ = 0; k_ < PER_WAVE; ++k_) if ((T_) < ntl[k_])                   \
            __builtin_amdgcn_global_load_lds(src[k_] + static_cast<uint64_t>(T_) * ROW, dst_ + k_ * 1024, \
                                             16, 0, AUX);                                             \
    } while (0)
#else
#define STORMCK_GLDS_ISSUE_MASKED(T_, SLOT) do { } while (0)
#endif
    if (wg_tiles > 0) STORMCK_GLDS_ISSUE_MASKED(0u, 0);
    for (uint32_t t = 0; t < wg_tiles; ++t) {
        wait_vmcnt<0>();
        __builtin_amdgcn_s_barrier();
        if (t + 1 < wg_tiles) STORMCK_GLDS_ISSUE_MASKED(t + 1, (t + 1) & 1);
        if (t < my_tiles) {
            const uint8_t* row = lds + (t & 1) * TILE + b * ROW + (j & 1) * 8;
#pragma unroll
            for (int s = 0; s < T; ++s) {
                const uint32_t q = (2 * s + (j >> 1) + 2 * T - rot) % (2 * T);
                acc = round(acc, *reinterpret_cast<const uint64_t*>(row + q * 16));
            }
        }
    }
#undef STORMCK_GLDS_ISSUE_MASKED
    const uint8_t* bsrc = arena + rec.data_offset;
    for (uint32_t s = my_tiles * T; s < nst; ++s) acc = round(acc, reinterpret_cast<const uint64_t*>(bsrc)[4 * s + j]);
    const uint64_t v1 = quad_bcast<0>(acc), v2 = quad_bcast<1>(acc), v3 = quad_bcast<2>(acc), v4 = quad_bcast<3>(acc);
    if (j == 0 && live) {
        const uint64_t h0 = (L >= 32) ? converge(v1, v2, v3, v4) : kP5;
        const uint64_t h = finish_fast(h0, L, bsrc + 32 * static_cast<uint64_t>(nst), L & 31);
        out_cs[lo + kb] = h;
        if (rec.origin_pointer != STORMCK_NO_ORIGIN) {
            uint64_t* p = reinterpret_cast<uint64_t*>(arena + rec.origin_pointer);
            p[0] = h;
            p[1] = rec.address;
            p[2] = rec.birth_revision;
            arena[rec.origin_type] = rec.type;
        }
    }
}

// ---------------------------------------------------------------------------
// f4: key tags — xxhash.Sum64(key) for short keys (keystore/keystore.go:33,66;
// keys are 1..256 bytes, objectlist.MaxKeyComponentLength). One lane per key (all
// four accumulators in the lane): for inputs of a few stripes the merge and tail
// dominate, and a quad would leave three lanes idle through them. Key i is at
// keys + (OFFS ? offs[i] : i*stride), LENS ? lens[i] : len bytes; 8-byte loads when
// the key is 8-byte aligned, byte loads otherwise.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t ld64_any(const uint8_t* p, bool aligned) {
    return aligned ? *reinterpret_cast<const uint64_t*>(p) : ld64_unaligned(p);
}

template <bool OFFS, bool LENS>
__global__ __launch_bounds__(256) void k_key_tags(const uint8_t* __restrict__ keys, uint64_t stride,
                                                   const uint64_t* __restrict__ offs, const uint32_t* __restrict__ lens,
                                                   uint32_t len, uint64_t n, uint64_t* __restrict__ out) {
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x;
    if (i >= n) return;
    const uint8_t* p = keys + (OFFS ? offs[i] : i * stride);
    const uint32_t L = LENS ? lens[i] : len;
    const bool al = (reinterpret_cast<uintptr_t>(p) & 7) == 0;
    const uint32_t nst = L >> 5;
    uint64_t h;
    if (L >= 32) {
        uint64_t v1 = kV1, v2 = kV2, v3 = kV3, v4 = kV4;
        for (uint32_t s = 0; s < nst; ++s) {
            const uint8_t* q = p + 32 * s;
            v1 = round(v1, ld64_any(q, al));
            v2 = round(v2, ld64_any(q + 8, al));
            v3 = round(v3, ld64_any(q + 16, al));
            v4 = round(v4, ld64_any(q + 24, al));
        }
        h = converge(v1, v2, v3, v4);
    } else {
        h = kP5;
    }
    out[i] = finish_fast(h, L, p + 32 * nst, L & 31);
}

// f4 fast path for fixed-stride keys (stride % 16 == 0, stride <= 256, 16-byte aligned
// base): each wave owns runs of 64 consecutive keys = one contiguous 64*stride-byte
// region, streamed HBM -> LDS by LDS-DMA (stride/16 wave-instructions, fully
// coalesced) into a per-wave double buffer; the next batch is in flight while the
// lanes hash the current one from LDS (lane l: its key at l*stride). Only whole
// batches of 64 keys; the caller hashes the remainder with k_key_tags. Waits are per
// wave (vmcnt + the wave's own LDS), so no workgroup barrier is needed.
// f4 ring variant for a compile-time stride of 16*P bytes: each wave owns PW
// consecutive batches of 64 keys, keeps RING-1 batches in flight through a RING-slot
// LDS ring, and holds its PW tags in registers until the end, so the loop issues no
// stores and a counted vmcnt wait ((RING-2)*P LDS-DMA ops younger than the batch being
// hashed) is exact. A wave with fewer than PW batches (the grid's last) waits vmcnt(0).
// KLEN > 0: every key is KLEN bytes (a compile-time constant, e.g. storm's 48-byte keys
// at stride 48), so the stripe count and the tail fold into straight-line code; the
// kernel is VALU-bound (about 28 64-bit multiplies per 48-byte key) and the generic tail
// costs about a third of its instructions. KLEN = 0: the runtime `len`.
// SM (how the tags reach HBM): 0 = one 8-byte store per lane per batch; 1 = the same,
// non-temporal; 2 = none (read-only probe); 3 = staged in the wave's LDS, then 16-byte
// stores (4 KiB contiguous per wave); 4 = 3, non-temporal.
template <int AUX, int P, int RING, int PW, int KLEN = 0, int SM = 0>
__global__ __launch_bounds__(256) void k_key_tags_ring(const uint8_t* __restrict__ keys, uint32_t len_rt,
                                                        uint64_t batches, uint64_t* __restrict__ out) {
    static_assert(RING >= 2 && PW >= RING, "ring");
    static_assert(KLEN >= 0 && KLEN <= 16 * P, "key length within the stride");
    const uint32_t len = KLEN > 0 ? static_cast<uint32_t>(KLEN) : len_rt;
    constexpr uint32_t kStride = 16 * P, kRegion = 64 * kStride;
    extern __shared__ __attribute__((aligned(16))) uint8_t dyn_lds[];
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    uint8_t* buf = dyn_lds + wave * RING * kRegion;
    const uint64_t b0 = (static_cast<uint64_t>(blockIdx.x) * 4 + wave) * PW;
    if (b0 >= batches) return;
    const uint32_t nb = static_cast<uint32_t>(batches - b0 < PW ? batches - b0 : PW);
    const uint32_t nst = len >> 5, rem = len & 31;
#if defined(__HIP_DEVICE_COMPILE__)
#define STORMCK_RING_ISSUE(I)                                                                              \
    do {                                                                                                  \
        const uint8_t* s_ = keys + (b0 + (I)) * kRegion + lane * 16;                                      \
        uint8_t* d_ = buf + ((I) % RING) * kRegion;                                                       \
        _Pragma("unroll") for (int p_ = 0; p_ < P; ++p_)                                                  \
            __builtin_amdgcn_global_load_lds(s_ + p_ * 1024, d_ + p_ * 1024, 16, 0, AUX);                  \
    } while (0)
#else
#define STORMCK_RING_ISSUE(I) do { } while (0)
#endif
    auto hash_slot = [&](uint32_t i) -> uint64_t {
        const uint8_t* k = buf + (i % RING) * kRegion + lane * kStride;
        uint64_t hh;
        if (len >= 32) {
            uint64_t v1 = kV1, v2 = kV2, v3 = kV3, v4 = kV4;
            for (uint32_t s = 0; s < nst; ++s) {
                const u64x2 x = *reinterpret_cast<const u64x2*>(k + 32 * s);
                const u64x2 y = *reinterpret_cast<const u64x2*>(k + 32 * s + 16);
                v1 = round(v1, x.x);
                v2 = round(v2, x.y);
                v3 = round(v3, y.x);
                v4 = round(v4, y.y);
            }
            hh = converge(v1, v2, v3, v4);
        } else {
            hh = kP5;
        }
        return finish_lds16(hh, len, k + 32 * nst, rem);
    };
    uint64_t h[PW];
    if (nb == PW) {
#pragma unroll
        for (int i = 0; i < RING - 1; ++i) STORMCK_RING_ISSUE(i);
#pragma unroll
        for (int i = 0; i < PW; ++i) {
            // batches i+1 .. min(i+RING-2, PW-1) were issued after batch i
            constexpr int kYoungest = RING - 2;
            if (i + kYoungest <= PW - 1) wait_vmcnt<kYoungest * P>();
            else wait_vmcnt<0>();
            // slot (i+RING-1) % RING was last read by batch i-1: its LDS reads retire first
            if (i + RING - 1 < PW) {
                wait_lgkm0();
                STORMCK_RING_ISSUE(i + RING - 1);
            }
            h[i] = hash_slot(i);
        }
    } else {
        for (uint32_t i = 0; i < nb; ++i) {
            STORMCK_RING_ISSUE(i);
            wait_vmcnt<0>();
            h[0] = hash_slot(i);
            out[(b0 + i) * 64 + lane] = h[0];
        }
        return;
    }
    if constexpr (SM == 3 || SM == 4) {
        static_assert(PW % 2 == 0 && PW * 64 * 8 <= RING * kRegion, "tags fit in the wave's ring");
        wait_lgkm0();  // the last batch's LDS reads are done: the ring is free
        uint64_t* tl = reinterpret_cast<uint64_t*>(buf);
#pragma unroll
        for (int i = 0; i < PW; ++i) tl[i * 64 + lane] = h[i];
        u64x2* dst = reinterpret_cast<u64x2*>(out + b0 * 64);
#pragma unroll
        for (int k = 0; k < PW / 2; ++k) {
            const u64x2 v = reinterpret_cast<const u64x2*>(tl)[k * 64 + lane];
            if constexpr (SM == 4) __builtin_nontemporal_store(v, dst + k * 64 + lane);
            else dst[k * 64 + lane] = v;
        }
    } else if constexpr (SM != 2) {
#pragma unroll
        for (int i = 0; i < PW; ++i) {
            if constexpr (SM == 1) __builtin_nontemporal_store(h[i], out + (b0 + i) * 64 + lane);
            else out[(b0 + i) * 64 + lane] = h[i];
        }
    } else {
#pragma unroll
        for (int i = 0; i < PW; ++i)
            if (h[i] == 0x5354524d5354524dULL) out[(b0 + i) * 64 + lane] = h[i];  // keeps the hash live
    }
#undef STORMCK_RING_ISSUE
}

template <int AUX>
__global__ __launch_bounds__(256) void k_key_tags_lds(const uint8_t* __restrict__ keys, uint32_t stride, uint32_t len,
                                                       uint64_t batches, uint32_t per_wave,
                                                       uint64_t* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) uint8_t dyn_lds[];
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t region = 64 * stride;       // bytes per batch
    [[maybe_unused]] const uint32_t pieces = region / 1024;  // LDS-DMA wave-instructions per batch
    uint8_t* buf = dyn_lds + wave * 2 * region;
    const uint64_t wid = static_cast<uint64_t>(blockIdx.x) * 4 + wave;
    const uint64_t b0 = wid * per_wave;
    if (b0 >= batches) return;
    const uint64_t b1 = (b0 + per_wave < batches) ? b0 + per_wave : batches;
    const uint32_t nst = len >> 5, rem = len & 31;
#if defined(__HIP_DEVICE_COMPILE__)
#define STORMCK_KEYS_ISSUE(B, SLOT)                                                                      \
    do {                                                                                               \
        const uint8_t* s_ = keys + (B) * region + lane * 16;                                           \
        uint8_t* d_ = buf + (SLOT) * region;                                                           \
        for (uint32_t p_ = 0; p_ < pieces; ++p_)                                                       \
            __builtin_amdgcn_global_load_lds(s_ + p_ * 1024, d_ + p_ * 1024, 16, 0, AUX);              \
    } while (0)
#else
#define STORMCK_KEYS_ISSUE(B, SLOT) do { } while (0)
#endif
    STORMCK_KEYS_ISSUE(b0, 0u);
    for (uint64_t b = b0; b < b1; ++b) {
        const uint32_t slot = static_cast<uint32_t>(b - b0) & 1;
        wait_vmcnt<0>();  // batch b landed (this wave's own pieces)
        if (b + 1 < b1) STORMCK_KEYS_ISSUE(b + 1, slot ^ 1u);
        const uint8_t* k = buf + slot * region + lane * stride;
        uint64_t h;
        if (len >= 32) {
            uint64_t v1 = kV1, v2 = kV2, v3 = kV3, v4 = kV4;
            for (uint32_t s = 0; s < nst; ++s) {
                const u64x2 x = *reinterpret_cast<const u64x2*>(k + 32 * s);
                const u64x2 y = *reinterpret_cast<const u64x2*>(k + 32 * s + 16);
                v1 = round(v1, x.x);
                v2 = round(v2, x.y);
                v3 = round(v3, y.x);
                v4 = round(v4, y.y);
            }
            h = converge(v1, v2, v3, v4);
        } else {
            h = kP5;
        }
        out[b * 64 + lane] = finish_lds16(h, len, k + 32 * nst, rem);
        // the slot is refilled two batches later, after this wave's reads retired
        // (the compiler waits lgkmcnt before the hash consumes them)
    }
#undef STORMCK_KEYS_ISSUE
}

// ---------------------------------------------------------------------------
// Synthetic block generator: word w of logical block (first + i)
// = splitmix64(seed ^ ((first + i) << 20 + w)). One 16-byte store per lane,
// grid-stride over the whole [n x stride] region (stride % 16 == 0).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_fill_synthetic(uint8_t* __restrict__ dst, uint64_t stride, uint64_t n,
                                                         uint64_t first, uint64_t seed) {
    const uint64_t pairs_per_block = stride / 16;
    const uint64_t total = pairs_per_block * n;
    for (uint64_t t = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x; t < total;
         t += static_cast<uint64_t>(gridDim.x) * 256) {
        const uint64_t i = t / pairs_per_block;
        const uint64_t w = (t - i * pairs_per_block) * 2;
        const uint64_t key = seed ^ (((first + i) << 20) + w);
        const uint64_t key2 = seed ^ (((first + i) << 20) + w + 1);
        ulonglong2 v;
        v.x = splitmix64(key);
        v.y = splitmix64(key2);
        reinterpret_cast<ulonglong2*>(dst + i * stride)[w / 2] = v;
    }
}

}  // namespace stormck
