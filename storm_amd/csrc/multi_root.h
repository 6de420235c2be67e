// Multi-GPU in one process (include/stormck.h "multi-GPU, one process"; SURVEY.md §7 step 7,
// §8e): every shard's checksums and tree on its own device, the shard roots gathered over
// xGMI by in-process RCCL, the combining pointer block hashed on every device.
//
// Included by stormck.hip inside its anonymous namespace, after the dispatch it calls
// (launch through stormck_checksum_device, stormck_merkle_root_device,
// stormck_pointer_node_device) and the fault slots (take_fault).
//
// One call on D distinct devices holding S shards:
//   A. a host thread per device enqueues, on each shard's stream, the shard's checksums (when
//      it has blocks) and its tree, whose root row {cs, addr, rev, type} lands in that device's
//      send rows; the device's gather stream waits for its shards;
//   B. one ncclAllGather of R rows per device (R = most shards on one device; rows a device
//      does not fill stay zero) over the communicator of the D devices, in one group from the
//      calling thread (ncclCommInitAll's single-thread, multi-device pattern);
//   C. on every device: the rows in shard order (k_gather_root_rows), the combining node
//      (k_pointer_node), its root row copied to pinned host memory; the devices must agree.
// The only bytes on xGMI are the D x R x 32-byte root rows: latency-bound by design.

// RCCL, loaded at the first multi-device call rather than linked: it is a 573 MB library that
// single-GPU users never need. A process that already holds one (torch's, soname
// librccl.so.1) shares it.
struct Rccl {
    decltype(&ncclCommInitAll) init_all = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclAllGather) all_gather = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
    decltype(&ncclGetVersion) get_version = nullptr;
    int version = 0;
    std::string error;  // why it is not usable ("" when it is)
};

const Rccl& rccl() {
    static const Rccl r = [] {
        Rccl x;
        void* h = nullptr;
        std::string why;
        for (const char* name : {"librccl.so.1", "/opt/rocm/lib/librccl.so.1"}) {
            h = dlopen(name, RTLD_NOW | RTLD_LOCAL);
            if (h) break;
            if (const char* e = dlerror()) why += std::string(e) + "; ";
        }
        if (!h) {
            x.error = "RCCL (librccl.so.1) cannot be loaded: " + why;
            return x;
        }
        bool ok = true;
        auto bind = [&](auto& fn, const char* name) {
            fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
            if (!fn) {
                ok = false;
                x.error += std::string(x.error.empty() ? "RCCL lacks " : ", ") + name;
            }
        };
        bind(x.init_all, "ncclCommInitAll");
        bind(x.destroy, "ncclCommDestroy");
        bind(x.all_gather, "ncclAllGather");
        bind(x.group_start, "ncclGroupStart");
        bind(x.group_end, "ncclGroupEnd");
        bind(x.error_string, "ncclGetErrorString");
        bind(x.get_version, "ncclGetVersion");
        if (ok && x.get_version(&x.version) != ncclSuccess) x.version = 0;
        return x;
    }();
    return r;
}

#define NCCL_TRY(expr)                                                                             \
    do {                                                                                           \
        const ncclResult_t r_ = (expr);                                                            \
        if (r_ != ncclSuccess)                                                                     \
            return fail(STORMCK_EHIP, std::string(#expr) + ": " + rccl().error_string(r_));        \
    } while (0)

// Per-device state of the multi calls, guarded by g_multi_mu (calls are serialised: a
// communicator runs one collective at a time).
struct MultiDev {
    int device = -1;
    hipStream_t stream = nullptr;  // the gather and the combine, and shards passed without a stream
    uint64_t* d_buf = nullptr;     // send / recv rows, map, entries, types, node checksum, trees
    uint64_t d_words = 0;
    uint64_t* h_row = nullptr;     // pinned: this device's combined root row
    uint64_t* h_table = nullptr;   // pinned: the gathered rows (read from the first device)
    uint64_t h_words = 0;
};

std::mutex g_multi_mu;
std::vector<std::unique_ptr<MultiDev>> g_multi_dev;                    // by device index
std::vector<std::pair<std::vector<int>, std::vector<ncclComm_t>>> g_comms;  // per device set

// The communicators of `devs` (in this order: rank k = devs[k]), created once per device set.
int comms_for(const std::vector<int>& devs, std::vector<ncclComm_t>** out) {
    for (auto& e : g_comms)
        if (e.first == devs) {
            *out = &e.second;
            return STORMCK_OK;
        }
    const Rccl& R = rccl();
    if (!R.error.empty()) return fail(STORMCK_EHIP, R.error);
    std::vector<ncclComm_t> comms(devs.size(), nullptr);
    NCCL_TRY(R.init_all(comms.data(), static_cast<int>(devs.size()), devs.data()));
    g_comms.emplace_back(devs, std::move(comms));
    *out = &g_comms.back().second;
    return STORMCK_OK;
}

// The calling thread's current device is `dev`; g_multi_dev already has its entry.
int multi_dev(int dev, uint64_t words, uint64_t h_words, MultiDev** out) {
    if (!g_multi_dev[dev]) {
        std::unique_ptr<MultiDev> m(new MultiDev());
        m->device = dev;
        HIP_TRY(hipStreamCreateWithFlags(&m->stream, hipStreamNonBlocking));
        HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&m->h_row), 4 * sizeof(uint64_t), hipHostMallocDefault));
        g_multi_dev[dev] = std::move(m);
    }
    MultiDev* m = g_multi_dev[dev].get();
    if (m->d_words < words) {  // every earlier call has finished with it (calls synchronise)
        if (m->d_buf) HIP_TRY(hipFree(m->d_buf));
        m->d_buf = nullptr;
        m->d_words = 0;
        HIP_TRY(hipMalloc(&m->d_buf, words * sizeof(uint64_t)));
        m->d_words = words;
    }
    if (m->h_words < h_words) {
        if (m->h_table) HIP_TRY(hipHostFree(m->h_table));
        m->h_table = nullptr;
        m->h_words = 0;
        HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&m->h_table), h_words * sizeof(uint64_t), hipHostMallocDefault));
        m->h_words = h_words;
    }
    *out = m;
    return STORMCK_OK;
}

// stormck_shutdown: the communicators and the per-device buffers.
void multi_release() {
    std::lock_guard<std::mutex> g(g_multi_mu);
    if (g_comms.empty() && g_multi_dev.empty()) return;  // never used: no HIP call at all
    if (!g_comms.empty() && rccl().error.empty())
        for (auto& e : g_comms)
            for (ncclComm_t c : e.second)
                if (c) (void)rccl().destroy(c);
    g_comms.clear();
    int prev = 0;
    (void)hipGetDevice(&prev);
    for (auto& m : g_multi_dev) {
        if (!m) continue;
        (void)hipSetDevice(m->device);
        if (m->stream) (void)hipStreamSynchronize(m->stream);
        (void)hipFree(m->d_buf);
        (void)hipHostFree(m->h_row);
        (void)hipHostFree(m->h_table);
        if (m->stream) (void)hipStreamDestroy(m->stream);
    }
    g_multi_dev.clear();
    (void)hipSetDevice(prev);
    (void)hipGetLastError();
}

int shard_plan(uint64_t n_total, uint32_t n_shards, const int* devices, int n_devices, stormck_shard* shards,
               uint64_t* root_addr) {
    if (!shards || n_shards == 0) return fail(STORMCK_EINVAL, "shards: at least one");
    if (!devices || n_devices <= 0 || n_devices > 64) return fail(STORMCK_EINVAL, "devices: 1..64 entries");
    if (n_total > (UINT64_MAX >> 2)) return fail(STORMCK_EINVAL, "n_total too large for the address convention");
    const uint64_t q = n_total / n_shards, r = n_total % n_shards;
    for (uint32_t s = 0; s < n_shards; ++s) {
        const uint64_t lo = s * q + std::min<uint64_t>(s, r);
        stormck_shard& sh = shards[s];
        std::memset(&sh, 0, sizeof sh);
        sh.n = q + (s < r ? 1 : 0);
        sh.leaf_addr_base = lo;
        sh.node_addr_base = n_total + lo;
        sh.device = devices[static_cast<uint64_t>(s) * static_cast<uint64_t>(n_devices) / n_shards];
    }
    if (root_addr) *root_addr = 2 * n_total;
    return STORMCK_OK;
}

// The gather layout of shards[0..S): the distinct devices in order of first appearance (the
// communicator's ranks), shard s -> (device slot, its row among that device's shards), R =
// the most shards on one device, and map[s] = slot * R + row, shard s's row of the gathered
// D x R table. Needs no device (stormck_multi_layout exposes it to the CPU tests).
struct MultiLayout {
    std::vector<int> devs;
    std::vector<uint32_t> slot, row, per_dev, map;
    uint64_t R = 0;
};

int multi_layout(const stormck_shard* shards, uint32_t S, MultiLayout* L) {
    L->devs.clear();
    L->per_dev.clear();
    L->slot.assign(S, 0);
    L->row.assign(S, 0);
    L->map.assign(S, 0);
    for (uint32_t s = 0; s < S; ++s) {
        const int dev = shards[s].device;
        if (dev < 0) return fail(STORMCK_EINVAL, "shards[" + std::to_string(s) + "].device is negative");
        const auto it = std::find(L->devs.begin(), L->devs.end(), dev);
        L->slot[s] = static_cast<uint32_t>(it - L->devs.begin());
        if (it == L->devs.end()) {
            if (L->devs.size() == 64) return fail(STORMCK_EINVAL, "more than 64 devices");
            L->devs.push_back(dev);
            L->per_dev.push_back(0);
        }
        L->row[s] = L->per_dev[L->slot[s]]++;
    }
    L->R = S ? *std::max_element(L->per_dev.begin(), L->per_dev.end()) : 0;
    for (uint32_t s = 0; s < S; ++s) L->map[s] = static_cast<uint32_t>(L->slot[s] * L->R + L->row[s]);
    return STORMCK_OK;
}

int merkle_root_multi(const stormck_shard* shards, uint32_t S, uint64_t rev, uint64_t root_addr, uint32_t fanout,
                      stormck_pointer* root, uint8_t* root_type, stormck_pointer* shard_roots, uint8_t* shard_types) {
    if (!root || !root_type) return fail(STORMCK_EINVAL, "null root pointer");
    if (fanout < 2 || fanout > kMaxFanout) return fail(STORMCK_EINVAL, "fanout out of range");
    if (!shards || S == 0 || S > fanout) return fail(STORMCK_EINVAL, "n_shards: 1..fanout shards");
    int rc = device_check();
    if (rc) return rc;
    int count = 0;
    HIP_TRY(hipGetDeviceCount(&count));
    for (uint32_t s = 0; s < S; ++s) {
        const stormck_shard& sh = shards[s];
        const std::string who = "shards[" + std::to_string(s) + "]";
        if (sh.device < 0 || sh.device >= count)
            return fail(STORMCK_EINVAL, who + ".device = " + std::to_string(sh.device) + " is not a visible device");
        if (sh.n > 0 && !sh.d_checksums) return fail(STORMCK_EINVAL, who + ".d_checksums is null");
        if (sh.d_blocks && sh.n > 1 && sh.stride < sh.len)
            return fail(STORMCK_EINVAL, who + ": stride smaller than len (blocks overlap)");
        if (sh.stream) {  // work enqueued on another device's stream would run there
            hipDevice_t sd = -1;
            HIP_TRY(hipStreamGetDevice(static_cast<hipStream_t>(sh.stream), &sd));
            if (sd != sh.device)
                return fail(STORMCK_EINVAL, who + ".stream belongs to device " + std::to_string(sd) + ", not " +
                                                std::to_string(sh.device));
        }
    }
    MultiLayout lay;
    rc = multi_layout(shards, S, &lay);
    if (rc) return rc;
    for (const int dev : lay.devs) {
        hipDeviceProp_t prop;
        HIP_TRY(hipGetDeviceProperties(&prop, dev));
        if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
            return fail(STORMCK_ENODEV, "device " + std::to_string(dev) + " is not gfx950: " + prop.gcnArchName);
    }
    const std::vector<int>& devs = lay.devs;
    const std::vector<uint32_t>&slot = lay.slot, &row = lay.row, &map = lay.map;
    const uint64_t D = devs.size();
    const uint64_t R = lay.R;
    // device buffer layout, in u64 words: send [R*4] | recv [D*R*4] | map [S u32] | entries [S*3]
    // | types [S bytes] | node checksum [1] | root row [4] | the device's shard trees
    const uint64_t o_send = 0, o_recv = R * 4, o_map = o_recv + D * R * 4, o_ent = o_map + (S + 1) / 2,
                   o_types = o_ent + 3ull * S, o_cs = o_types + (S + 7) / 8, o_row = o_cs + 1, o_ws = o_row + 4;
    std::vector<uint64_t> ws_off(S), ws_words(S), dev_words(D, o_ws);
    for (uint32_t s = 0; s < S; ++s) {
        ws_words[s] = (stormck_merkle_workspace_bytes(shards[s].n, fanout) + 7) / 8;
        ws_off[s] = dev_words[slot[s]];
        dev_words[slot[s]] += ws_words[s];
    }

    std::lock_guard<std::mutex> serial(g_multi_mu);
    // sized here, so the per-device threads below each touch only their own entry
    const int top = *std::max_element(devs.begin(), devs.end());
    if (g_multi_dev.size() <= static_cast<size_t>(top)) g_multi_dev.resize(top + 1);
    int prev = 0;
    HIP_TRY(hipGetDevice(&prev));
    struct Part {
        MultiDev* m = nullptr;
        std::vector<hipEvent_t> events;
        int rc = STORMCK_OK;
        std::string err;
    };
    std::vector<Part> part(D);
    // A: each device's shards, from a host thread per device (the calling thread takes the first)
    auto enqueue = [&](uint64_t d) -> int {
        Part& P = part[d];
        HIP_TRY(hipSetDevice(devs[d]));
        int r = multi_dev(devs[d], dev_words[d], d == 0 ? D * R * 4 : 0, &P.m);
        if (r) return r;
        uint64_t* buf = P.m->d_buf;
        HIP_TRY(hipMemsetAsync(buf + o_send, 0, R * 4 * sizeof(uint64_t), P.m->stream));
        hipEvent_t zeroed = nullptr;
        HIP_TRY(hipEventCreateWithFlags(&zeroed, hipEventDisableTiming));
        P.events.push_back(zeroed);
        HIP_TRY(hipEventRecord(zeroed, P.m->stream));
        for (uint32_t s = 0; s < S; ++s) {
            if (slot[s] != d) continue;
            const stormck_shard& sh = shards[s];
            hipStream_t st = sh.stream ? static_cast<hipStream_t>(sh.stream) : P.m->stream;
            if (st != P.m->stream) HIP_TRY(hipStreamWaitEvent(st, zeroed, 0));
            if (sh.d_blocks && sh.n) {
                r = stormck_checksum_device(sh.d_blocks, sh.stride, nullptr, sh.len, sh.n, sh.d_checksums, st);
                if (r) return r;
            }
            uint64_t* rw = buf + o_send + 4ull * row[s];
            r = stormck_merkle_root_device(sh.d_checksums, sh.n, sh.leaf_addr_base, sh.node_addr_base, rev, fanout,
                                           buf + o_ws + ws_off[s], ws_words[s] * 8,
                                           reinterpret_cast<stormck_pointer*>(rw), reinterpret_cast<uint8_t*>(rw + 3),
                                           st);
            if (r) return r;
            if (st != P.m->stream) {
                hipEvent_t done = nullptr;
                HIP_TRY(hipEventCreateWithFlags(&done, hipEventDisableTiming));
                P.events.push_back(done);
                HIP_TRY(hipEventRecord(done, st));
                HIP_TRY(hipStreamWaitEvent(P.m->stream, done, 0));
            }
        }
        return STORMCK_OK;
    };
    auto work = [&](uint64_t d) {
        part[d].rc = enqueue(d);
        if (part[d].rc) part[d].err = g_last_error;  // this thread's message
    };
    {
        std::vector<std::thread> threads;
        uint64_t spawned = 1;
        try {
            for (; spawned < D; ++spawned) threads.emplace_back(work, spawned);
        } catch (const std::system_error&) {
            // no more threads: the calling thread enqueues the devices that have none
        }
        for (uint64_t d = 0; d < D; ++d)
            if (d == 0 || d >= spawned) work(d);
        for (std::thread& t : threads) t.join();
    }
    auto cleanup = [&] {
        for (uint64_t d = 0; d < D; ++d) {
            if (part[d].m) {
                (void)hipSetDevice(devs[d]);
                (void)hipStreamSynchronize(part[d].m->stream);
            }
            for (hipEvent_t e : part[d].events) (void)hipEventDestroy(e);
        }
        (void)hipSetDevice(prev);
    };
    for (uint64_t d = 0; d < D; ++d)
        if (part[d].rc) {
            const int code = part[d].rc;
            const std::string msg = "device " + std::to_string(devs[d]) + ": " + part[d].err;
            cleanup();
            return fail(code, msg);
        }
    // B + C: the gather, then the combine on every device
    auto gather_combine = [&]() -> int {
        std::vector<ncclComm_t>* comms = nullptr;
        int r = comms_for(devs, &comms);
        if (r) return r;
        const Rccl& RC = rccl();
        NCCL_TRY(RC.group_start());
        for (uint64_t d = 0; d < D; ++d) {
            uint64_t* buf = part[d].m->d_buf;
            const ncclResult_t e =
                RC.all_gather(buf + o_send, buf + o_recv, R * 4, ncclUint64, (*comms)[d], part[d].m->stream);
            if (e != ncclSuccess) {
                (void)RC.group_end();
                return fail(STORMCK_EHIP, "ncclAllGather on device " + std::to_string(devs[d]) + ": " +
                                              RC.error_string(e));
            }
        }
        NCCL_TRY(RC.group_end());
        for (uint64_t d = 0; d < D; ++d) {
            MultiDev* m = part[d].m;
            uint64_t* buf = m->d_buf;
            HIP_TRY(hipSetDevice(devs[d]));
            HIP_TRY(hipMemcpyAsync(buf + o_map, map.data(), S * sizeof(uint32_t), hipMemcpyHostToDevice, m->stream));
            hipLaunchKernelGGL(k_gather_root_rows, dim3(1), dim3(256), 0, m->stream, buf + o_recv,
                               reinterpret_cast<const uint32_t*>(buf + o_map), S, buf + o_ent,
                               reinterpret_cast<uint8_t*>(buf + o_types));
            HIP_TRY(hipGetLastError());
            r = stormck_pointer_node_device(reinterpret_cast<const stormck_pointer*>(buf + o_ent),
                                            reinterpret_cast<const uint8_t*>(buf + o_types), S, fanout, buf + o_cs,
                                            m->stream);
            if (r) return r;
            HIP_TRY(hipMemsetAsync(buf + o_row, 0, 4 * sizeof(uint64_t), m->stream));
            hipLaunchKernelGGL(k_set_root, dim3(1), dim3(64), 0, m->stream, buf + o_cs, root_addr, rev,
                               static_cast<uint8_t>(STORMCK_POINTER_BLOCK), buf + o_row,
                               reinterpret_cast<uint8_t*>(buf + o_row + 3));
            HIP_TRY(hipGetLastError());
            HIP_TRY(hipMemcpyAsync(m->h_row, buf + o_row, 4 * sizeof(uint64_t), hipMemcpyDeviceToHost, m->stream));
            if (d == 0)
                HIP_TRY(hipMemcpyAsync(m->h_table, buf + o_recv, D * R * 4 * sizeof(uint64_t), hipMemcpyDeviceToHost,
                                       m->stream));
        }
        for (uint64_t d = 0; d < D; ++d) HIP_TRY(hipStreamSynchronize(part[d].m->stream));
        // a ring kernel that faulted on a shard's stream wrote no checksums for some blocks
        for (uint32_t s = 0; s < S; ++s) {
            if (!shards[s].d_blocks || !shards[s].n) continue;
            hipStream_t st = shards[s].stream ? static_cast<hipStream_t>(shards[s].stream) : part[slot[s]].m->stream;
            r = take_fault(devs[slot[s]], st);
            if (r) return r;
        }
        return STORMCK_OK;
    };
    rc = gather_combine();
    const std::string msg = g_last_error;
    cleanup();
    g_last_error = msg;
    if (rc) return rc;
    const uint64_t* r0 = part[0].m->h_row;
    for (uint64_t d = 1; d < D; ++d)
        if (std::memcmp(part[d].m->h_row, r0, 4 * sizeof(uint64_t)) != 0)
            return fail(STORMCK_EHIP, "devices " + std::to_string(devs[0]) + " and " + std::to_string(devs[d]) +
                                          " disagree on the global root");
    root->checksum = r0[0];
    root->address = r0[1];
    root->birth_revision = r0[2];
    *root_type = static_cast<uint8_t>(r0[3]);
    const uint64_t* table = part[0].m->h_table;
    for (uint32_t s = 0; s < S; ++s) {
        const uint64_t* t = table + 4ull * map[s];
        if (shard_roots) shard_roots[s] = stormck_pointer{t[0], t[1], t[2]};
        if (shard_types) shard_types[s] = static_cast<uint8_t>(t[3]);
    }
    return STORMCK_OK;
}
