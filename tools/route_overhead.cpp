// Probe (GPU box): the fixed cost the routed entry points add to storm's smallest calls,
// in C, without Python: the primitives a routed call runs before it hashes (pointer
// classification, the host-readability check, the stream query) and the routed call
// against its host leg on three 32 KiB blocks, pageable and registered; then two callers
// at once on the halves of a c5-size batch.
//   hipcc -O2 -std=c++17 -Iinclude tools/route_overhead.cpp -Lstorm_amd/lib -lstormck \
//       -Wl,-rpath,'$ORIGIN/../storm_amd/lib' -pthread -o tools/route_overhead
#include <hip/hip_runtime.h>
#include <sys/uio.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "stormck.h"

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// median over 9 rounds of the mean of `reps` calls, in microseconds
template <class F>
static double per_call(F f, int reps = 2000) {
    std::vector<double> r;
    for (int k = 0; k < 9; ++k) {
        const double t0 = now_us();
        for (int i = 0; i < reps; ++i) f();
        r.push_back((now_us() - t0) / reps);
    }
    std::sort(r.begin(), r.end());
    return r[4];
}

int main(int argc, char** argv) {
    const bool only_c5 = argc > 1 && std::strcmp(argv[1], "c5") == 0;  // the c5-size A/B alone (traceable)
    if (stormck_init(0) != STORMCK_OK) {
        std::fprintf(stderr, "init: %s\n", stormck_last_error());
        return 1;
    }
    const uint64_t blk = 32768, n = 3;
    void* pg = std::aligned_alloc(4096, 1 << 20);
    void* rg = std::aligned_alloc(4096, 1 << 20);
    std::fill_n(static_cast<unsigned char*>(pg), 1 << 20, 7);
    std::fill_n(static_cast<unsigned char*>(rg), 1 << 20, 7);
    if (stormck_host_register(rg, 1 << 20) != STORMCK_OK) {
        std::fprintf(stderr, "register: %s\n", stormck_last_error());
        return 1;
    }
    hipStream_t st;
    (void)hipStreamCreate(&st);
    hipPointerAttribute_t a;
    uint32_t leg = 0;
    if (!only_c5) {
    std::printf("hipPointerGetAttributes registered %.3f us\n", per_call([&] { (void)hipPointerGetAttributes(&a, rg); }));
    std::printf("hipPointerGetAttributes pageable   %.3f us\n", per_call([&] {
                    if (hipPointerGetAttributes(&a, pg) != hipSuccess) (void)hipGetLastError();
                }));
    std::printf("process_vm_readv 2 bytes           %.3f us\n", per_call([&] {
                    unsigned char got[2];
                    iovec l = {got, 2};
                    iovec r[2] = {{pg, 1}, {static_cast<unsigned char*>(pg) + 3 * blk - 1, 1}};
                    (void)process_vm_readv(getpid(), &l, 1, r, 2, 0);
                }));
    std::printf("hipStreamQuery null stream         %.3f us\n", per_call([&] { (void)hipStreamQuery(nullptr); }));
    std::printf("hipStreamQuery created stream      %.3f us\n", per_call([&] { (void)hipStreamQuery(st); }));

    uint64_t out[n];
    for (void* base : {pg, rg}) {
        const char* what = base == pg ? "pageable  " : "registered";
        const double h = per_call([&] { (void)stormck_checksum_host_leg(base, blk, nullptr, blk, n, out, 1); });
        const double r = per_call([&] { (void)stormck_checksum_batch(base, blk, nullptr, blk, n, out, 0, &leg); });
        std::printf("batch %s 3 x 32 KiB: host leg %.3f us  routed %.3f us (leg %u)  +%.3f us\n", what, h, r, leg, r - h);
    }
    stormck_dirty_block b[n] = {};
    for (uint64_t i = 0; i < n; ++i) {
        b[i].data_offset = i * blk;
        b[i].origin_pointer = STORMCK_NO_ORIGIN;
        b[i].parent = STORMCK_NO_PARENT;
        b[i].address = i + 1;
        b[i].birth_revision = 5;
        b[i].length = static_cast<uint32_t>(blk);
        b[i].type = STORMCK_LEAF_BLOCK;
    }
    for (void* base : {pg, rg}) {
        const char* what = base == pg ? "pageable  " : "registered";
        uint64_t last = 100;
        const double h = per_call([&] { (void)stormck_commit_host(base, b, n, 9, &last, out, 1); });
        const double r = per_call([&] { (void)stormck_commit(base, b, n, 9, &last, out, nullptr, 0, &leg); });
        const double rs = per_call([&] { (void)stormck_commit(base, b, n, 9, &last, out, st, 0, &leg); });
        std::printf("commit %s 3 x 32 KiB: host %.3f us  routed %.3f us  routed on a stream %.3f us (leg %u)  +%.3f us\n",
                    what, h, r, rs, leg, r - h);
    }
    }  // !only_c5
    // two callers at once on the halves of a registered c5-size batch (1,202 x 32 KiB
    // slots), against one call on the whole: threads started beforehand and released
    // together, so only the library's handling of the second caller is timed
    {
        const uint64_t nb = 1202, half = nb / 2;
        const uint64_t bytes = nb * blk;
        void* c5 = std::aligned_alloc(4096, bytes);
        std::fill_n(static_cast<unsigned char*>(c5), bytes, 5);
        stormck_host_register(c5, bytes);
        std::vector<uint64_t> o(nb);
        const double one = per_call([&] { (void)stormck_checksum_batch(c5, blk, nullptr, 31808, nb, o.data(), 0, &leg); }, 50);
        std::printf("c5-size batch, one caller: %.1f us (leg %u)\n", one, leg);
        // the routed batch against the host leg it takes, alternating call by call (registered
        // and pageable copies of the same slots): what routing costs at storm's commit size
        {
            void* c5p = std::aligned_alloc(4096, bytes);
            std::memcpy(c5p, c5, bytes);
            for (void* base : {c5, c5p}) {
                std::vector<double> th, tr;
                int seen[4] = {0, 0, 0, 0};  // legs the routed calls took
                for (int rep = 0; rep < 201; ++rep) {
                    double h = 0, r = 0;
                    for (int k = 0; k < 2; ++k) {  // which goes first alternates: each follows the other
                        const double t0 = now_us();
                        if ((k ^ rep) & 1) {
                            (void)stormck_checksum_batch(base, blk, nullptr, 31808, nb, o.data(), 0, &leg);
                            r = now_us() - t0;
                            ++seen[leg & 3];
                        } else {
                            (void)stormck_checksum_host_leg(base, blk, nullptr, 31808, nb, o.data(), 0);
                            h = now_us() - t0;
                        }
                    }
                    if (rep) {
                        th.push_back(h);
                        tr.push_back(r);
                    }
                }
                std::sort(th.begin(), th.end());
                std::sort(tr.begin(), tr.end());
                std::printf("c5-size batch %s, alternating: host leg (pool) %.1f us  routed %.1f us  x%.3f  "
                            "(routed legs: host %d, device %d, split %d)\n",
                            base == c5 ? "registered" : "pageable  ", th[100], tr[100], tr[100] / th[100], seen[1],
                            seen[2], seen[3]);
            }
            std::free(c5p);
        }
        // the same on the registered slots, five forms in rotation (each follows every other):
        // which part of the routed call costs what at this size
        {
            const char* names[5] = {"host_leg(0)", "batch(0)", "host_leg(16)", "batch(16)", "batch(1)"};
            std::vector<double> t[5];
            for (int rep = 0; rep < 101; ++rep)
                for (int j = 0; j < 5; ++j) {
                    const int k = (j + rep) % 5;
                    const double t0 = now_us();
                    switch (k) {
                        case 0: (void)stormck_checksum_host_leg(c5, blk, nullptr, 31808, nb, o.data(), 0); break;
                        case 1: (void)stormck_checksum_batch(c5, blk, nullptr, 31808, nb, o.data(), 0, &leg); break;
                        case 2: (void)stormck_checksum_host_leg(c5, blk, nullptr, 31808, nb, o.data(), 16); break;
                        case 3: (void)stormck_checksum_batch(c5, blk, nullptr, 31808, nb, o.data(), 16, &leg); break;
                        default: (void)stormck_checksum_batch(c5, blk, nullptr, 31808, nb, o.data(), 1, &leg); break;
                    }
                    if (rep) t[k].push_back(now_us() - t0);
                }
            std::printf("c5-size batch registered, rotating medians:");
            for (int k = 0; k < 5; ++k) {
                std::sort(t[k].begin(), t[k].end());
                std::printf(" %s %.1f", names[k], t[k][t[k].size() / 2]);
            }
            std::printf(" us\n");
        }
        for (int round = 0; round < 3; ++round) {
            std::atomic<int> go{0}, ready{0};
            double t_done[2] = {0, 0};
            uint32_t legs[2] = {0, 0};
            auto body = [&](int k) {
                ready.fetch_add(1);
                while (go.load(std::memory_order_acquire) == 0) {
                }
                const uint64_t lo = k ? half : 0, cnt = k ? nb - half : half;
                (void)stormck_checksum_batch(static_cast<unsigned char*>(c5) + lo * blk, blk, nullptr, 31808, cnt,
                                             o.data() + lo, 0, &legs[k]);
                t_done[k] = now_us();
            };
            std::vector<double> walls;
            for (int rep = 0; rep < 20; ++rep) {
                ready = 0;
                go = 0;
                std::thread a(body, 0), b(body, 1);
                while (ready.load() < 2) {
                }
                const double t0 = now_us();
                go.store(1, std::memory_order_release);
                a.join();
                b.join();
                walls.push_back(std::max(t_done[0], t_done[1]) - t0);
            }
            std::sort(walls.begin(), walls.end());
            std::printf("c5-size batch, two callers on halves: median %.1f us, min %.1f, max %.1f (legs %u %u)\n",
                        walls[walls.size() / 2], walls.front(), walls.back(), legs[0], legs[1]);
        }
        // the same slots as one height of a commit with one host thread: the routed commit
        // (which picks the split) against the split called directly, alternating
        std::vector<stormck_dirty_block> fb(nb);
        for (uint64_t i = 0; i < nb; ++i) {
            fb[i] = {};
            fb[i].data_offset = i * blk;
            fb[i].origin_pointer = STORMCK_NO_ORIGIN;
            fb[i].parent = STORMCK_NO_PARENT;
            fb[i].address = i + 1;
            fb[i].birth_revision = 5;
            fb[i].length = 31808;
            fb[i].type = STORMCK_LEAF_BLOCK;
        }
        std::vector<double> t_routed, t_split;
        uint64_t last = 1u << 20, done = 0;
        auto show = [&](const char* when) {
            stormck_route_rates rr;
            stormck_route_get_rates(&rr);
            uint32_t pleg = 0;
            double us[3];
            stormck_route_plan_commit(fb.data(), nb, STORMCK_MEM_PINNED, 1, 1, &pleg, us);
            std::printf("%s: rates thread %.0f memory %.0f cached %.0f inplace %.0f latency %.1f; plan leg %u: "
                        "host %.1f device %.1f split %.1f us\n",
                        when, rr.host_thread, rr.host_memory, rr.host_cached, rr.link_inplace, rr.device_latency,
                        pleg, us[0], us[1], us[2]);
        };
        show("before");
        for (int rep = 0; rep < 61; ++rep) {
            double t0 = now_us();
            (void)stormck_commit(c5, fb.data(), nb, 9, &last, o.data(), nullptr, 1, &leg);
            const double r = now_us() - t0;
            t0 = now_us();
            (void)stormck_commit_split(c5, fb.data(), nb, 9, &last, o.data(), nullptr, 0, 1, STORMCK_SPLIT_BALANCED,
                                       &done);
            const double s = now_us() - t0;
            if (rep) {
                t_routed.push_back(r);
                t_split.push_back(s);
            }
            if (rep < 3) {
                std::printf("rep %d: routed %.1f us (leg %u), split %.1f us (device %llu leaves)\n", rep, r, leg, s,
                            static_cast<unsigned long long>(done));
                show("after");
            }
        }
        std::sort(t_routed.begin(), t_routed.end());
        std::sort(t_split.begin(), t_split.end());
        std::printf("c5-size commit, 1 host thread: routed %.1f us (leg %u)  split %.1f us (device %llu leaves)\n",
                    t_routed[30], leg, t_split[30], static_cast<unsigned long long>(done));
        stormck_host_unregister(c5);
        std::free(c5);
    }
    (void)hipStreamDestroy(st);
    stormck_host_unregister(rg);
    std::free(pg);
    std::free(rg);
    stormck_shutdown();
    return 0;
}
