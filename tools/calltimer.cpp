// Measurement helper (not product): times storm-sized calls of libstormck in a C loop, so
// bench.py's end-to-end tables compare the legs of a few-microsecond call by what the calls
// cost, not by what Python's ctypes adds per argument (the routed calls take two arguments
// more than their host legs). storm calls the library through cgo, whose cost per call does
// not depend on the argument count. Built by storm_amd/build.py build_calltimer:
//   g++ -O2 -std=c++17 -shared -fPIC -Iinclude tools/calltimer.cpp -Lstorm_amd/lib -lstormck
#include <chrono>
#include <cstdint>
#include <vector>

#include "stormck.h"

namespace {
double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
}  // namespace

extern "C" {

// Legs of a commit (bench.py commit_e2e): 0 stormck_commit_device on `arena` (a device
// pointer), 1 stormck_commit_host, 2 stormck_commit_split (balanced), 3 stormck_commit
// (routed). The records are copied from `tmpl` once and committed `reps` times back to back
// (relocation happens in the first; hashing and the stores repeat in every one). Returns
// microseconds per call; *rc the last status, *leg the routed leg, *done the split's device
// leaves, *last_out the last allocated block.
double calltimer_commit(int leg, void* arena, const stormck_dirty_block* tmpl, uint64_t n, uint64_t revision,
                        uint64_t last, uint64_t* out, uint32_t threads, int reps, int* rc, uint32_t* leg_used,
                        uint64_t* done, uint64_t* last_out) {
    std::vector<stormck_dirty_block> b(tmpl, tmpl + n);
    uint64_t la = last;
    int r = STORMCK_OK;
    const double t0 = now_us();
    for (int k = 0; k < reps; ++k) {
        switch (leg) {
            case 0: r = stormck_commit_device(arena, b.data(), n, revision, &la, out, nullptr); break;
            case 1: r = stormck_commit_host(arena, b.data(), n, revision, &la, out, threads); break;
            case 2:
                r = stormck_commit_split(arena, b.data(), n, revision, &la, out, nullptr, 0, threads,
                                         STORMCK_SPLIT_BALANCED, done);
                break;
            default: r = stormck_commit(arena, b.data(), n, revision, &la, out, nullptr, threads, leg_used); break;
        }
    }
    const double us = (now_us() - t0) / reps;
    *rc = r;
    *last_out = la;
    return us;
}

// Legs of a host-memory batch (bench.py batch_e2e): 0 stormck_checksum_host (the device
// pipeline), 1 stormck_checksum_host_leg, 2 stormck_checksum_split (balanced), 3
// stormck_checksum_batch (routed). Microseconds per call over `reps` back-to-back calls.
double calltimer_batch(int leg, const void* base, uint64_t stride, const uint32_t* lens, uint32_t len, uint64_t n,
                       uint64_t* out, uint32_t threads, int reps, int* rc, uint32_t* leg_used, uint64_t* done) {
    int r = STORMCK_OK;
    const double t0 = now_us();
    for (int k = 0; k < reps; ++k) {
        switch (leg) {
            case 0: r = stormck_checksum_host(base, stride, lens, len, n, out); break;
            case 1: r = stormck_checksum_host_leg(base, stride, lens, len, n, out, threads); break;
            case 2:
                r = stormck_checksum_split(base, stride, lens, len, n, out, nullptr, 0, threads, STORMCK_SPLIT_BALANCED,
                                           done);
                break;
            default: r = stormck_checksum_batch(base, stride, lens, len, n, out, threads, leg_used); break;
        }
    }
    const double us = (now_us() - t0) / reps;
    *rc = r;
    return us;
}

}  // extern "C"
