// Host-side sanitizer driver for libstormck (ASan + UBSan, or TSan).
//
// Built by tests/sanitize/build.sh against a copy of libstormck whose HOST code is
// instrumented (hipcc -Xarch_host -fsanitize=...; device code is untouched, GPU
// sanitizers are not used). It drives the library's host orchestration through the
// C ABI:
//   * the single-call leg stormck_xxh64 / stormck_checksum on every length 0..4100 at
//     every start offset mod 8, against the oracle (out-of-bounds reads show up here);
//   * argument validation of every entry point (EINVAL before any device work);
//   * the batch host leg (stormck_checksum_host_leg / _verify_host_leg) from several
//     caller threads at once, and the routed batch with a device;
//   * f1 commit planning: validation, the threaded height walk-up (ForkJoin pool),
//     cycle / range / alignment errors, on shuffled forests up to 300K records;
//   * with a gfx950 device (GPU box): the same commits run to completion on a device
//     arena and are compared with the oracle's serial commit; the host pipeline
//     (pageable and registered sources, parallel staging copies, both stages), the
//     batched verify and the file read-verify reader threads, and four host threads
//     calling the library at once; the split leg (host threads and the device worker
//     on one call, fixed and balanced, checksum, verify and commit) from two callers; the
//     one-process multi-GPU root (stormck_merkle_root_multi, in-process RCCL) from two.
// Exit status 0 = every check passed and the sanitizer reported nothing (sanitizer
// reports abort the process: halt_on_error / -fno-sanitize-recover).
#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include <hip/hip_runtime_api.h>

#include "stormck.h"

extern "C" {
uint64_t oracle_xxh64(const void* data, size_t n);
void oracle_fill_synthetic(void* dst, size_t stride, size_t n, uint64_t first, uint64_t seed);
size_t oracle_pointer_block_size(uint32_t fanout);
void oracle_pack_pointer_block(uint8_t* dst, uint32_t fanout, const uint64_t* cs, const uint64_t* addr,
                               const uint64_t* rev, const uint8_t* types, uint32_t m);
size_t oracle_merkle_root(const uint64_t* leaf_cs, size_t n, uint64_t leaf_addr_base, uint64_t node_addr_base,
                          uint64_t rev, uint32_t fanout, uint64_t root[3], uint8_t* root_type);
int oracle_commit(uint8_t* arena, stormck_dirty_block* blocks, size_t n, uint64_t revision, uint64_t* last_allocated,
                  uint64_t* out_cs);
}

static std::atomic<int> g_fail{0};
#define CHECK(cond)                                                                                  \
    do {                                                                                             \
        if (!(cond)) {                                                                               \
            std::fprintf(stderr, "FAIL %s:%d: %s (%s)\n", __FILE__, __LINE__, #cond, stormck_last_error()); \
            ++g_fail;                                                                                \
        }                                                                                            \
    } while (0)

static void single_calls() {
    std::mt19937_64 rng(7);
    std::vector<uint8_t> buf(4100 + 16);
    for (auto& c : buf) c = static_cast<uint8_t>(rng());
    for (size_t n = 0; n <= 4100; ++n) {
        for (size_t off = 0; off < 8; ++off) {
            // an exact-size heap copy, so a read past the end is a heap overflow
            std::vector<uint8_t> exact(buf.begin() + off, buf.begin() + off + n);
            const uint64_t want = oracle_xxh64(n ? exact.data() : buf.data(), n);
            CHECK(stormck_xxh64(exact.data(), n) == want);
            uint64_t out = 0;
            CHECK(stormck_checksum(n ? exact.data() : nullptr, n, &out) == STORMCK_OK && out == want);
        }
    }
    CHECK(stormck_xxh64(nullptr, 0) == 0xEF46DB3751D8E999ULL);
}

static void argument_errors() {
    uint64_t out = 0, fb = 0, nb = 0;
    uint8_t small[64] = {};
    CHECK(stormck_checksum("abc", 3, nullptr) == STORMCK_EINVAL);
    CHECK(stormck_checksum(nullptr, 3, &out) == STORMCK_EINVAL);
    CHECK(stormck_checksum_gpu("abc", 3, nullptr) == STORMCK_EINVAL);
    CHECK(stormck_checksum_gpu(small, (256ULL << 20) + 1, &out) == STORMCK_EINVAL);
    CHECK(stormck_checksum_device(reinterpret_cast<void*>(1 << 20), 16, nullptr, 32, 2, &out, nullptr) == STORMCK_EINVAL);
    CHECK(stormck_checksum_device(nullptr, 32, nullptr, 32, 2, &out, nullptr) == STORMCK_EINVAL);
    CHECK(stormck_checksum_gather_device(small, nullptr, nullptr, 32, 2, &out, nullptr) == STORMCK_EINVAL);
    CHECK(stormck_verify_device(small, 32, nullptr, 32, 2, &out, nullptr, nullptr) == STORMCK_EINVAL);
    CHECK(stormck_pointer_level_device(&out, 5, 0, 1, 2, 0, &out, nullptr) == STORMCK_EINVAL);
    CHECK(stormck_pointer_node_device(reinterpret_cast<stormck_pointer*>(small), small, 11, 10, &out, nullptr) ==
          STORMCK_EINVAL);
    CHECK(stormck_pack_pointer_blocks_device(&out, 5, 0, 1, 2, 10, small, 200, nullptr) == STORMCK_EINVAL);
    CHECK(stormck_merkle_root_device(&out, 5000, 0, 5000, 1, 10, small, 8, reinterpret_cast<stormck_pointer*>(small),
                                     small, nullptr) == STORMCK_EINVAL);
    CHECK(stormck_fill_synthetic_device(small, 24, 4, 0, 1, nullptr) == STORMCK_EINVAL);
    CHECK(stormck_host_register(nullptr, 0) == STORMCK_EINVAL);
    CHECK(stormck_host_device_pointer(nullptr, nullptr) == STORMCK_EINVAL);
    CHECK(stormck_key_tags_device(nullptr, 48, nullptr, nullptr, 48, 10, &out, nullptr) == STORMCK_EINVAL);
    CHECK(stormck_checksum_host(nullptr, 32, nullptr, 32, 4, &out) == STORMCK_EINVAL);
    CHECK(stormck_checksum_host_multi(small, 32, nullptr, 32, 2, &out, nullptr, 0) == STORMCK_EINVAL);
    stormck_shard sh[2] = {};
    stormck_pointer pr{};
    uint8_t pt = 0;
    const int dev0 = 0;
    CHECK(stormck_shard_plan(10, 0, &dev0, 1, sh, nullptr) == STORMCK_EINVAL);
    CHECK(stormck_shard_plan(10, 2, nullptr, 0, sh, nullptr) == STORMCK_EINVAL);
    CHECK(stormck_merkle_root_multi(sh, 2, 1, 20, 1200, nullptr, &pt, nullptr, nullptr) == STORMCK_EINVAL);
    CHECK(stormck_merkle_root_multi(sh, 0, 1, 20, 1200, &pr, &pt, nullptr, nullptr) == STORMCK_EINVAL);
    CHECK(stormck_merkle_root_multi(sh, 2, 1, 20, 1, &pr, &pt, nullptr, nullptr) == STORMCK_EINVAL);
    const uint64_t addr_big[1] = {1ULL << 60}, addr0[1] = {0};
    const uint32_t len100[1] = {100};
    const uint64_t exp0[1] = {0};
    const int devnull = open("/dev/null", O_RDONLY);
    CHECK(stormck_read_verify_fd(devnull, addr_big, len100, 1, 32768, small, 64, exp0, 0, &fb, &nb) == STORMCK_EINVAL);
    CHECK(stormck_read_verify_fd(devnull, addr0, len100, 1, 32768, small, 64, exp0, STORMCK_READ_FULL_BLOCK, &fb,
                                 &nb) == STORMCK_EINVAL);
    CHECK(stormck_read_verify_fd(devnull, addr0, len100, 1, 0, small, 64, exp0, 0, &fb, &nb) == STORMCK_EINVAL);
    close(devnull);
}

// storm's dirty forest (storm_amd.commit.pointer_forest): leaves in slots 1..n, pointer
// blocks level by level after them, the top block hanging off the singularity (slot 0).
struct Forest {
    std::vector<stormck_dirty_block> b;
    uint64_t arena_bytes = 0, last = 0;
};

static Forest make_forest(uint64_t n_leaves, uint32_t fanout, uint64_t slot, uint64_t revision, std::mt19937_64& rng,
                          bool shuffle) {
    Forest f;
    const uint32_t pbs = (fanout * 25u + 7u) & ~7u;
    std::vector<uint64_t> levels;
    for (uint64_t m = n_leaves; m > 1;) levels.push_back(m = (m + fanout - 1) / fanout);
    const uint64_t total = n_leaves + std::accumulate(levels.begin(), levels.end(), uint64_t{0});
    f.b.resize(total);
    for (uint64_t i = 0; i < total; ++i) {
        auto& r = f.b[i];
        std::memset(&r, 0, sizeof r);
        r.data_offset = (i + 1) * slot;
        r.length = i < n_leaves ? static_cast<uint32_t>(std::min<uint64_t>(slot, 72 + rng() % slot)) : pbs;
        r.type = i < n_leaves ? STORMCK_LEAF_BLOCK : STORMCK_POINTER_BLOCK;
        r.address = i + 1;
        r.birth_revision = rng() % 3 == 0 ? revision : revision + 1;  // a third relocate
    }
    uint64_t start = 0, count = n_leaves;
    for (uint64_t lv : levels) {
        const uint64_t ps = start + count;
        for (uint64_t c = 0; c < count; ++c) {
            const uint64_t p = ps + c / fanout, k = c % fanout;
            f.b[start + c].parent = static_cast<int64_t>(p);
            f.b[start + c].origin_pointer = f.b[p].data_offset + 24 * k;
            f.b[start + c].origin_type = f.b[p].data_offset + 24ULL * fanout + k;
        }
        start = ps;
        count = lv;
    }
    f.b[start].parent = STORMCK_NO_PARENT;
    f.b[start].origin_pointer = 32;  // singularity SpacePointer / SpaceBlockType
    f.b[start].origin_type = 56;
    f.last = total;
    f.arena_bytes = (total + 1) * slot;
    if (shuffle) {  // parents before children in the caller's array
        std::vector<uint64_t> perm(total), inv(total);
        std::iota(perm.begin(), perm.end(), 0);
        std::shuffle(perm.begin(), perm.end(), rng);
        for (uint64_t i = 0; i < total; ++i) inv[perm[i]] = i;
        std::vector<stormck_dirty_block> nb(total);
        for (uint64_t i = 0; i < total; ++i) {
            nb[i] = f.b[perm[i]];
            if (nb[i].parent >= 0) nb[i].parent = static_cast<int64_t>(inv[nb[i].parent]);
        }
        f.b.swap(nb);
    }
    return f;
}

static bool has_device() {
    int c = 0;
    return stormck_device_count(&c) == STORMCK_OK && c > 0;
}

static void commit_planning(bool device) {
    std::mt19937_64 rng(11);
    const uint64_t sizes[] = {1, 2, 137, 5000, 70000, 300000};
    for (uint64_t nl : sizes) {
        for (bool shuffle : {false, true}) {
            // big forests: fan-out 100 (2,504 B pointer blocks) in 4 KiB slots keeps the
            // host copy small while level 0 still runs in several chunks
            const uint32_t fanout = nl > 10000 ? 100 : 10;
            const uint64_t slot = nl > 10000 ? 4096 : 1024;
            Forest f = make_forest(nl, fanout, slot, 5, rng, shuffle);
            const uint64_t n = f.b.size();
            std::vector<uint64_t> cs(n, 0);
            uint64_t last = f.last;
            if (!device) {
                const auto before = f.b;
                const int rc = stormck_commit_device(reinterpret_cast<void*>(1 << 20), f.b.data(), n, 5, &last,
                                                     cs.data(), nullptr);
                CHECK(rc == STORMCK_ENODEV);
                CHECK(last == f.last && std::memcmp(before.data(), f.b.data(), n * sizeof(stormck_dirty_block)) == 0);
                continue;
            }
            if (f.arena_bytes > (2ULL << 30)) continue;  // keep the host copy small
            std::vector<uint8_t> host(f.arena_bytes, 0);
            for (uint64_t i = 0; i < n; ++i)
                if (f.b[i].type == STORMCK_LEAF_BLOCK)
                    for (uint32_t k = 0; k < f.b[i].length; k += 8) host[f.b[i].data_offset + k] = static_cast<uint8_t>(rng());
            void* d_arena = nullptr;
            CHECK(hipMalloc(&d_arena, f.arena_bytes) == hipSuccess);
            CHECK(hipMemcpy(d_arena, host.data(), f.arena_bytes, hipMemcpyHostToDevice) == hipSuccess);
            auto ref = f.b;
            uint64_t ref_last = f.last;
            std::vector<uint64_t> ref_cs(n, 0);
            CHECK(oracle_commit(host.data(), ref.data(), n, 5, &ref_last, ref_cs.data()) == 0);
            CHECK(stormck_commit_device(d_arena, f.b.data(), n, 5, &last, cs.data(), nullptr) == STORMCK_OK);
            CHECK(last == ref_last && cs == ref_cs);
            CHECK(std::memcmp(ref.data(), f.b.data(), n * sizeof(stormck_dirty_block)) == 0);
            std::vector<uint8_t> back(f.arena_bytes);
            CHECK(hipMemcpy(back.data(), d_arena, f.arena_bytes, hipMemcpyDeviceToHost) == hipSuccess);
            CHECK(back == host);
            CHECK(hipFree(d_arena) == hipSuccess);
            std::printf("commit %llu leaves%s: ok\n", static_cast<unsigned long long>(nl), shuffle ? " (shuffled)" : "");
        }
    }
    // planning errors, with or without a device: parent range, origin alignment, cycle
    Forest f = make_forest(25, 10, 1024, 1, rng, false);
    std::vector<uint64_t> cs(f.b.size());
    uint64_t last = f.last;
    auto bad = f.b;
    bad[3].parent = 1000000;
    CHECK(stormck_commit_device(reinterpret_cast<void*>(1 << 20), bad.data(), bad.size(), 1, &last, cs.data(), nullptr) ==
          STORMCK_EINVAL);
    bad = f.b;
    bad[3].origin_pointer += 4;
    CHECK(stormck_commit_device(reinterpret_cast<void*>(1 << 20), bad.data(), bad.size(), 1, &last, cs.data(), nullptr) ==
          STORMCK_EINVAL);
    bad = f.b;
    bad[bad.size() - 1].parent = 0;  // root -> leaf 0 -> ... -> root
    CHECK(stormck_commit_device(reinterpret_cast<void*>(1 << 20), bad.data(), bad.size(), 1, &last, cs.data(), nullptr) ==
          STORMCK_EINVAL);
}

// f1's host leg (no device needed): stormck_commit_host on 1 thread and on the pool,
// against the oracle's serial commit, from several caller threads at once (each height
// fans out over the shared ForkJoin pool); with a device, the routed stormck_commit on
// a pageable arena (the host leg by construction).
static void commit_host_leg(bool device) {
    auto one = [&](uint64_t nl, bool shuffle, uint32_t threads, uint64_t seed) {
        std::mt19937_64 rng(seed);
        const uint32_t fanout = nl > 10000 ? 100 : 10;
        const uint64_t slot = nl > 10000 ? 4096 : 1024;
        Forest f = make_forest(nl, fanout, slot, 5, rng, shuffle);
        const uint64_t n = f.b.size();
        std::vector<uint8_t> host(f.arena_bytes, 0);
        for (uint64_t i = 0; i < n; ++i)
            if (f.b[i].type == STORMCK_LEAF_BLOCK)
                for (uint32_t k = 0; k < f.b[i].length; k += 8) host[f.b[i].data_offset + k] = static_cast<uint8_t>(rng());
        auto ref_arena = host;
        auto ref = f.b;
        uint64_t ref_last = f.last, last = f.last;
        std::vector<uint64_t> ref_cs(n, 0), cs(n, 0);
        CHECK(oracle_commit(ref_arena.data(), ref.data(), n, 5, &ref_last, ref_cs.data()) == 0);
        if (device && threads == 7) {  // the routed entry on pageable memory
            uint32_t leg = 0;
            CHECK(stormck_commit(host.data(), f.b.data(), n, 5, &last, cs.data(), nullptr, 0, &leg) == STORMCK_OK &&
                  leg == STORMCK_LEG_HOST);
        } else {
            CHECK(stormck_commit_host(host.data(), f.b.data(), n, 5, &last, cs.data(), threads) == STORMCK_OK);
        }
        CHECK(last == ref_last && cs == ref_cs && host == ref_arena);
        CHECK(std::memcmp(ref.data(), f.b.data(), n * sizeof(stormck_dirty_block)) == 0);
    };
    for (uint64_t nl : {uint64_t{1}, uint64_t{2}, uint64_t{137}, uint64_t{5000}, uint64_t{70000}})
        for (bool shuffle : {false, true})
            for (uint32_t threads : {1u, 0u}) one(nl, shuffle, threads, 21 + nl);
    std::vector<std::thread> th;
    for (int t = 0; t < 4; ++t)
        th.emplace_back([&, t] {
            for (int it = 0; it < 3; ++it) one(3000 + 977 * t, t & 1, (it == 2) ? 7u : 0u, 50 + 10 * t + it);
        });
    for (auto& x : th) x.join();
}

// The batch host leg (no device needed): stormck_checksum_host_leg / _verify_host_leg on
// exact-size heap copies (a read past a block shows up), per-block lengths 0..stride,
// unaligned starts, 1 thread and the pool, from several caller threads at once; with a
// device, the routed stormck_checksum_batch on both host-thread settings.
static void batch_host_leg(bool device) {
    auto one = [&](uint64_t n, uint64_t stride, uint64_t off, uint32_t threads, uint64_t seed) {
        std::mt19937_64 rng(seed);
        std::vector<uint8_t> buf(n * stride + off);
        for (auto& c : buf) c = static_cast<uint8_t>(rng());
        std::vector<uint32_t> lens(n);
        for (auto& l : lens) l = static_cast<uint32_t>(rng() % (stride + 1));
        if (n) lens[n - 1] = static_cast<uint32_t>(stride);  // the last block ends at the buffer's end
        std::vector<uint8_t> exact(buf.begin() + off, buf.end());
        std::vector<uint64_t> want(n), got(n, 0);
        for (uint64_t i = 0; i < n; ++i) want[i] = oracle_xxh64(exact.data() + i * stride, lens[i]);
        CHECK(stormck_checksum_host_leg(exact.data(), stride, lens.data(), 0, n, got.data(), threads) == STORMCK_OK &&
              got == want);
        uint64_t fb = 0, nb = 0;
        auto bad = want;
        if (n > 2) bad[n / 2] ^= 1;
        const int rc = stormck_verify_host_leg(exact.data(), stride, lens.data(), 0, n, bad.data(), &fb, &nb, threads);
        CHECK(n > 2 ? (rc == STORMCK_EMISMATCH && fb == n / 2 && nb == 1) : (rc == STORMCK_OK && nb == 0));
        if (device) {
            uint32_t leg = 0;
            std::fill(got.begin(), got.end(), 0);
            CHECK(stormck_checksum_batch(exact.data(), stride, lens.data(), 0, n, got.data(), threads, &leg) ==
                      STORMCK_OK &&
                  got == want && (n == 0 || leg == STORMCK_LEG_HOST || leg == STORMCK_LEG_DEVICE));
        }
    };
    for (uint64_t n : {uint64_t{0}, uint64_t{1}, uint64_t{3}, uint64_t{4}, uint64_t{7}, uint64_t{1000}})
        for (uint64_t off : {uint64_t{0}, uint64_t{5}})
            for (uint32_t threads : {1u, 0u}) one(n, n > 100 ? 4096 : 200, off, threads, 31 + n + off);
    std::vector<std::thread> th;
    for (int t = 0; t < 4; ++t)
        th.emplace_back([&, t] {
            for (int it = 0; it < 3; ++it) one(700 + 131 * t, 8192, t & 1, it == 2 ? 1u : 0u, 60 + 10 * t + it);
        });
    for (auto& x : th) x.join();
}

static void host_pipeline_paths() {
    std::mt19937_64 rng(3);
    const uint64_t n = 12000, stride = 32768;  // 375 MiB: two 256 MiB pipeline chunks
    std::vector<uint8_t> buf(n * stride);
    for (size_t i = 0; i < buf.size(); i += 8) buf[i] = static_cast<uint8_t>(rng());
    std::vector<uint32_t> lens(n);
    for (auto& l : lens) l = static_cast<uint32_t>(rng() % (stride + 1));
    std::vector<uint64_t> want(n), got(n);
    for (uint64_t i = 0; i < n; ++i) want[i] = oracle_xxh64(buf.data() + i * stride, lens[i]);
    CHECK(stormck_checksum_host(buf.data(), stride, lens.data(), 0, n, got.data()) == STORMCK_OK && got == want);
    uint64_t fb = 0, nb = 0;
    CHECK(stormck_verify_host(buf.data(), stride, lens.data(), 0, n, want.data(), &fb, &nb) == STORMCK_OK && nb == 0);
    auto bad = want;
    bad[7777] ^= 1;
    CHECK(stormck_verify_host(buf.data(), stride, lens.data(), 0, n, bad.data(), &fb, &nb) == STORMCK_EMISMATCH &&
          fb == 7777 && nb == 1);
    CHECK(stormck_host_register(buf.data(), buf.size()) == STORMCK_OK);
    std::fill(got.begin(), got.end(), 0);
    CHECK(stormck_checksum_host(buf.data(), stride, lens.data(), 0, n, got.data()) == STORMCK_OK && got == want);
    // one batch over several devices from one process (worker thread per listed device;
    // the box has one GPU, so device 0 is listed three times): ranges, offsets, merge
    const int devs[3] = {0, 0, 0};
    std::fill(got.begin(), got.end(), 0);
    CHECK(stormck_checksum_host_multi(buf.data(), stride, lens.data(), 0, n, got.data(), devs, 3) == STORMCK_OK &&
          got == want);
    bad[11111] ^= 1;
    CHECK(stormck_verify_host_multi(buf.data(), stride, lens.data(), 0, n, bad.data(), &fb, &nb, devs, 3) ==
              STORMCK_EMISMATCH &&
          fb == 7777 && nb == 2);
    bad[11111] ^= 1;
    CHECK(stormck_host_unregister(buf.data()) == STORMCK_OK);
    uint64_t one = 0;
    CHECK(stormck_checksum_gpu(buf.data() + 3, 70000, &one) == STORMCK_OK && one == oracle_xxh64(buf.data() + 3, 70000));
    // file read-verify: reader threads, pipelined verify
    char path[] = "/tmp/stormck_sanitize_XXXXXX";
    const int fd = mkstemp(path);
    CHECK(fd >= 0);
    CHECK(write(fd, buf.data(), 4096 * stride) == static_cast<ssize_t>(4096 * stride));
    std::vector<uint64_t> addrs(3000), exp(3000);
    std::vector<uint32_t> l2(3000);
    for (uint64_t i = 0; i < 3000; ++i) {
        addrs[i] = rng() % 4096;
        l2[i] = lens[addrs[i]];
        exp[i] = want[addrs[i]];
    }
    std::vector<uint8_t> slots(3000 * stride);
    CHECK(stormck_read_verify_fd(fd, addrs.data(), l2.data(), 3000, stride, slots.data(), stride, exp.data(), 0, &fb,
                                 &nb) == STORMCK_OK && nb == 0);
    // many small super-chunks: the reader pool runs ahead of the verifier across them;
    // then a mismatch and a read past the end of the file, both in a later super-chunk
    setenv("STORMCK_READ_SUPER_BYTES", "200000", 1);
    CHECK(stormck_read_verify_fd(fd, addrs.data(), l2.data(), 3000, stride, slots.data(), stride, exp.data(), 0, &fb,
                                 &nb) == STORMCK_OK && nb == 0);
    exp[2500] ^= 1;
    CHECK(stormck_read_verify_fd(fd, addrs.data(), l2.data(), 3000, stride, slots.data(), stride, exp.data(), 0, &fb,
                                 &nb) == STORMCK_EMISMATCH && fb == 2500 && nb == 1);
    exp[2500] ^= 1;
    addrs[2600] = 5000;  // beyond the 4096 blocks written
    l2[2600] = 64;
    CHECK(stormck_read_verify_fd(fd, addrs.data(), l2.data(), 3000, stride, slots.data(), stride, exp.data(), 0, &fb,
                                 &nb) == STORMCK_EINVAL &&
          std::string(stormck_last_error()).find("block index 2600") != std::string::npos);
    unsetenv("STORMCK_READ_SUPER_BYTES");
    close(fd);
    unlink(path);
}

// The split leg: one call's blocks on the host threads (from the front) and the device
// worker thread (from the back) at once, with fixed boundaries and balanced, checksum and
// verify, from two caller threads (one call owns the device worker at a time; a balanced
// call that finds it busy runs without it), then the split commit on a registered arena.
static void split_paths() {
    const uint64_t n = 3000, stride = 32768;
    std::mt19937_64 rng(17);
    std::vector<uint8_t> buf(n * stride);
    for (size_t i = 0; i < buf.size(); i += 8) buf[i] = static_cast<uint8_t>(rng());
    std::vector<uint32_t> lens(n);
    for (auto& l : lens) l = static_cast<uint32_t>(rng() % (stride + 1));
    std::vector<uint64_t> want(n);
    for (uint64_t i = 0; i < n; ++i) want[i] = oracle_xxh64(buf.data() + i * stride, lens[i]);
    CHECK(stormck_host_register(buf.data(), buf.size()) == STORMCK_OK);
    stormck_route_rates slow_host;
    std::memset(&slow_host, 0, sizeof slow_host);
    slow_host.host_thread = 2000.0;
    slow_host.host_memory = slow_host.host_cached = 8000.0;
    slow_host.link_pinned = 55000.0;
    slow_host.link_pageable = slow_host.link_inplace = 50000.0;
    CHECK(stormck_route_set_rates(&slow_host, STORMCK_RATES_FREEZE) == STORMCK_OK);
    auto run = [&](int t) {
        std::vector<uint64_t> got(n);
        for (uint64_t d : {uint64_t{0}, uint64_t{1}, n / 2, n, STORMCK_SPLIT_BALANCED}) {
            uint64_t done = 0, fb = 0, nb = 0;
            std::fill(got.begin(), got.end(), 0);
            CHECK(stormck_checksum_split(buf.data(), stride, lens.data(), 0, n, got.data(), nullptr, 0, 0, d, &done) ==
                      STORMCK_OK &&
                  got == want && (d == STORMCK_SPLIT_BALANCED ? done <= n : done == d));
            auto bad = want;
            bad[n / 2 - 1 + t] ^= 1;
            CHECK(stormck_verify_split(buf.data(), stride, lens.data(), 0, n, bad.data(), &fb, &nb, nullptr, 0, 0, d,
                                       &done) == STORMCK_EMISMATCH &&
                  fb == n / 2 - 1 + t && nb == 1);
        }
        uint32_t leg = 0;
        std::fill(got.begin(), got.end(), 0);
        CHECK(stormck_checksum_batch(buf.data(), stride, lens.data(), 0, n, got.data(), 0, &leg) == STORMCK_OK &&
              got == want);
    };
    std::vector<std::thread> th;
    for (int t = 0; t < 2; ++t) th.emplace_back(run, t);
    for (auto& x : th) x.join();
    CHECK(stormck_host_unregister(buf.data()) == STORMCK_OK);
    for (uint64_t dl : {uint64_t{0}, uint64_t{1}, uint64_t{700}, STORMCK_SPLIT_BALANCED}) {
        Forest f = make_forest(2000, 100, 4096, 5, rng, true);
        const uint64_t nb = f.b.size();
        std::vector<uint8_t> host(f.arena_bytes, 0);
        for (uint64_t i = 0; i < nb; ++i)
            if (f.b[i].type == STORMCK_LEAF_BLOCK)
                for (uint32_t k = 0; k < f.b[i].length; k += 8) host[f.b[i].data_offset + k] = static_cast<uint8_t>(rng());
        auto ref_arena = host;
        auto ref = f.b;
        uint64_t ref_last = f.last, last = f.last, done = 0;
        std::vector<uint64_t> ref_cs(nb, 0), cs(nb, 0);
        CHECK(oracle_commit(ref_arena.data(), ref.data(), nb, 5, &ref_last, ref_cs.data()) == 0);
        CHECK(stormck_host_register(host.data(), host.size()) == STORMCK_OK);
        CHECK(stormck_commit_split(host.data(), f.b.data(), nb, 5, &last, cs.data(), nullptr, 0, 0, dl, &done) ==
                  STORMCK_OK &&
              (dl == STORMCK_SPLIT_BALANCED || done == dl));
        CHECK(last == ref_last && cs == ref_cs && host == ref_arena);
        CHECK(std::memcmp(ref.data(), f.b.data(), nb * sizeof(stormck_dirty_block)) == 0);
        CHECK(stormck_host_unregister(host.data()) == STORMCK_OK);
    }
    CHECK(stormck_route_set_rates(nullptr, STORMCK_RATES_LEARN) == STORMCK_OK);
}

// Several host threads on one device at once, as cgo callers on many goroutines would
// be (stormck.h: the library is safe for concurrent callers; host pipelines sharing a
// device are serialised inside). Each thread hashes and verifies its own batch, makes
// single calls on both legs, and provokes an error whose thread-local message must be
// its own.
static void concurrent_callers() {
    constexpr int kThreads = 4;
    constexpr uint64_t n = 600, stride = 32768;
    std::vector<std::vector<uint8_t>> bufs(kThreads);
    std::vector<std::vector<uint32_t>> lens(kThreads);
    std::vector<std::vector<uint64_t>> want(kThreads);
    for (int t = 0; t < kThreads; ++t) {
        std::mt19937_64 rng(100 + t);
        bufs[t].resize(n * stride);
        for (size_t i = 0; i < bufs[t].size(); i += 8) bufs[t][i] = static_cast<uint8_t>(rng());
        lens[t].resize(n);
        for (auto& l : lens[t]) l = static_cast<uint32_t>(rng() % (stride + 1));
        want[t].resize(n);
        for (uint64_t i = 0; i < n; ++i) want[t][i] = oracle_xxh64(bufs[t].data() + i * stride, lens[t][i]);
    }
    const int devnull = open("/dev/null", O_RDONLY);
    CHECK(devnull >= 0);
    std::vector<std::thread> th;
    for (int t = 0; t < kThreads; ++t)
        th.emplace_back([&, t] {
            CHECK(stormck_init(0) == STORMCK_OK);
            const uint8_t* b = bufs[t].data();
            std::vector<uint64_t> got(n), bad = want[t];
            bad[(t + 1) * 100] ^= 1;
            for (int it = 0; it < 5; ++it) {
                std::fill(got.begin(), got.end(), 0);
                CHECK(stormck_checksum_host(b, stride, lens[t].data(), 0, n, got.data()) == STORMCK_OK &&
                      got == want[t]);
                uint64_t fb = 0, nb = 0;
                CHECK(stormck_verify_host(b, stride, lens[t].data(), 0, n, bad.data(), &fb, &nb) == STORMCK_EMISMATCH &&
                      fb == static_cast<uint64_t>((t + 1) * 100) && nb == 1);
                uint64_t one = 0;
                CHECK(stormck_checksum_gpu(b + 8 * t, 5000 + t, &one) == STORMCK_OK &&
                      one == oracle_xxh64(b + 8 * t, 5000 + t));
                CHECK(stormck_xxh64(b + it * stride, lens[t][it]) == want[t][it]);
                // an argument error naming this thread's own block index
                std::vector<uint64_t> addr(t + 1, 0), exp(t + 1, 0);
                std::vector<uint32_t> l(t + 1, 64);
                addr[t] = UINT64_MAX;
                std::vector<uint8_t> slots((t + 1) * 64);
                CHECK(stormck_read_verify_fd(devnull, addr.data(), l.data(), t + 1, 32768, slots.data(), 64, exp.data(),
                                             0, &fb, &nb) == STORMCK_EINVAL &&
                      std::string(stormck_last_error()).find("of block index " + std::to_string(t) + " ") !=
                          std::string::npos);
            }
        });
    for (auto& x : th) x.join();
    close(devnull);
}

// The one-process multi-GPU root (stormck_merkle_root_multi) on device 0, from two callers
// at once (the library serialises the calls): five planned shards whose blocks the library
// hashes, their trees, the one-rank RCCL gather and the combine, against the oracle's shard
// trees and combining node.
static void multi_root_paths() {
    constexpr uint64_t n_total = 5003, stride = 4096, kShards = 5;
    constexpr uint64_t seed = 0x53544F524DULL;
    const int dev0 = 0;
    std::vector<stormck_shard> plan(kShards);
    uint64_t root_addr = 0;
    CHECK(stormck_shard_plan(n_total, kShards, &dev0, 1, plan.data(), &root_addr) == STORMCK_OK &&
          root_addr == 2 * n_total);
    std::vector<uint8_t> host(n_total * stride);
    oracle_fill_synthetic(host.data(), stride, n_total, 0, seed);
    std::vector<uint64_t> cs(n_total);
    for (uint64_t i = 0; i < n_total; ++i) cs[i] = oracle_xxh64(host.data() + i * stride, stride);
    uint64_t rc[kShards], ra[kShards], rr[kShards];
    uint8_t rt[kShards];
    for (uint64_t s = 0; s < kShards; ++s) {
        uint64_t root[3];
        oracle_merkle_root(cs.data() + plan[s].leaf_addr_base, plan[s].n, plan[s].leaf_addr_base, plan[s].node_addr_base,
                           1, STORMCK_POINTERS_PER_BLOCK, root, &rt[s]);
        rc[s] = root[0];
        ra[s] = root[1];
        rr[s] = root[2];
    }
    std::vector<uint8_t> node(oracle_pointer_block_size(STORMCK_POINTERS_PER_BLOCK));
    oracle_pack_pointer_block(node.data(), STORMCK_POINTERS_PER_BLOCK, rc, ra, rr, rt, kShards);
    const uint64_t want = oracle_xxh64(node.data(), node.size());
    void* d_blocks = nullptr;
    CHECK(stormck_device_alloc(n_total * stride, &d_blocks) == STORMCK_OK);
    CHECK(stormck_fill_synthetic_device(d_blocks, stride, n_total, 0, seed, nullptr) == STORMCK_OK);
    CHECK(stormck_device_status(nullptr) == STORMCK_OK);
    auto run = [&](int t) {
        CHECK(stormck_init(0) == STORMCK_OK);
        void* d_cs = nullptr;
        CHECK(stormck_device_alloc(n_total * 8, &d_cs) == STORMCK_OK);
        std::vector<stormck_shard> shards = plan;
        for (stormck_shard& sh : shards) {
            sh.d_blocks = static_cast<uint8_t*>(d_blocks) + sh.leaf_addr_base * stride;
            sh.stride = stride;
            sh.len = static_cast<uint32_t>(stride - 8 * t);  // the callers hash different lengths
            sh.d_checksums = static_cast<uint64_t*>(d_cs) + sh.leaf_addr_base;
        }
        for (int it = 0; it < 3; ++it) {
            stormck_pointer root{};
            uint8_t type = 0;
            std::vector<stormck_pointer> srows(kShards);
            std::vector<uint8_t> stypes(kShards);
            CHECK(stormck_merkle_root_multi(shards.data(), kShards, 1, root_addr, STORMCK_POINTERS_PER_BLOCK, &root, &type,
                                            srows.data(), stypes.data()) == STORMCK_OK);
            if (t == 0) {
                CHECK(root.checksum == want && root.address == root_addr && root.birth_revision == 1 &&
                      type == STORMCK_POINTER_BLOCK);
                for (uint64_t s = 0; s < kShards; ++s)
                    CHECK(srows[s].checksum == rc[s] && srows[s].address == ra[s] && stypes[s] == rt[s]);
            } else {
                CHECK(root.address == root_addr && type == STORMCK_POINTER_BLOCK && root.checksum != want);
            }
        }
        CHECK(stormck_device_free(d_cs) == STORMCK_OK);
    };
    std::vector<std::thread> th;
    for (int t = 0; t < 2; ++t) th.emplace_back(run, t);
    for (auto& x : th) x.join();
    CHECK(stormck_device_free(d_blocks) == STORMCK_OK);
}

int main() {
    std::setvbuf(stdout, nullptr, _IONBF, 0);  // progress lines reach a log file at once
    single_calls();
    std::printf("single calls: done\n");
    argument_errors();
    const bool device = has_device();
    std::printf("device: %s\n", device ? "yes" : "no (planning up to the device check)");
    if (device) CHECK(stormck_init(0) == STORMCK_OK);
    commit_planning(device);
    std::printf("commit planning: done\n");
    commit_host_leg(device);
    std::printf("commit host leg: done\n");
    batch_host_leg(device);
    std::printf("batch host leg: done\n");
    if (device) host_pipeline_paths();
    if (device) concurrent_callers();
    if (device) std::printf("concurrent callers: done\n");
    if (device) split_paths();
    if (device) std::printf("split leg: done\n");
    if (device) multi_root_paths();
    if (device) std::printf("multi-GPU root: done\n");
    stormck_shutdown();
    std::printf("%s: %d failure(s)\n", g_fail.load() ? "FAILED" : "ok", g_fail.load());
    return g_fail ? 1 : 0;
}
