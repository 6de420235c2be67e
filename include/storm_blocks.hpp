// storm_blocks.hpp — C++ mirror of storm's Go package `blocks` over libstormck.
//
// Same names, argument meaning and error behaviour as the reference:
//   Hash, BlockAddress, BlockSize, BlockType, Pointer      blocks/types.go:4-39
//   Checksum(b)                                            blocks/checksum.go:15-17
//   BlockChecksum(&block)                                  blocks/checksum.go:10-12
//   VerifyChecksum(address, p, expected) -> error or nil   blocks/checksum.go:20-27
// plus ChecksumBatch / VerifyChecksumBatch, the entry points the GPU path exists for.
// Block layouts (Go amd64, padding included) mirror blocks/{pointer,blob,objectlist,
// spacelist,singularity}/block.go; the `test` build-tag fan-outs are template args.
//
// Single calls (Checksum, BlockChecksum, VerifyChecksum) hash on the calling thread
// through stormck_xxh64, the library's single-call leg: one buffer is four serial
// XXH64 chains, which one host core walks faster than the GPU (DESIGN_LOG.md §5), and like
// Go's Checksum it cannot fail. Batches run on the gfx950 device, or on the library's
// host leg when its cost model predicts the PCIe link makes the device slower for a
// host-memory batch; they need a device either way, and a failure throws
// storm::blocks::DeviceError. ChecksumGPU / ChecksumBatchGPU are the device legs alone.
#pragma once

#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <new>
#include <optional>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <utility>
#include <vector>

#include "stormck.h"

namespace storm::blocks {

using Hash = uint64_t;
using BlockAddress = uint64_t;
using ObjectID = uint64_t;
using SpaceID = uint64_t;

inline constexpr int64_t BlockSize = 32 * 1024;

enum BlockType : uint8_t { FreeBlockType = 0, PointerBlockType = 1, LeafBlockType = 2 };

struct Pointer {
    Hash Checksum;
    BlockAddress Address;
    uint64_t BirthRevision;
};
static_assert(sizeof(Pointer) == 24 && sizeof(Pointer) == sizeof(stormck_pointer));

class DeviceError : public std::runtime_error {
public:
    explicit DeviceError(int code)
        : std::runtime_error("stormck error " + std::to_string(code) + ": " + stormck_last_error()), code_(code) {}
    int code() const { return code_; }

private:
    int code_;
};

// The value VerifyChecksum returns on mismatch (pkg/errors.Errorf in the reference).
class Error {
public:
    explicit Error(std::string msg) : msg_(std::move(msg)) {}
    const std::string& message() const { return msg_; }  // Go: err.Error()

private:
    std::string msg_;
};

namespace detail {
inline void check(int rc) {
    if (rc != STORMCK_OK) throw DeviceError(rc);
}
// Go's %#v of an unsigned integer: 0x-prefixed lowercase hex without padding.
inline std::string go_hex(uint64_t v) {
    char buf[24];
    std::snprintf(buf, sizeof buf, "0x%llx", static_cast<unsigned long long>(v));
    return buf;
}
}  // namespace detail

// Checksum computes checksum of bytes.
inline Hash Checksum(const void* b, size_t n) { return stormck_xxh64(b, n); }

// The same single call on the device (k_xxh64_single), up to 256 MiB.
inline Hash ChecksumGPU(const void* b, size_t n) {
    uint64_t out = 0;
    detail::check(stormck_checksum_gpu(b, n, &out));
    return out;
}
inline Hash Checksum(const std::vector<uint8_t>& b) { return Checksum(b.data(), b.size()); }

// BlockChecksum computes checksum of the block: all sizeof(T) bytes of the live
// object, padding included (photon.NewFromValue(b).B in the reference).
template <class T>
inline Hash BlockChecksum(const T* b) {
    static_assert(std::is_trivially_copyable_v<T>, "blocks are plain structs");
    return Checksum(b, sizeof(T));
}

// VerifyChecksum verifies that checksum of provided data matches the expected one.
// Returns std::nullopt (Go: nil) on match.
inline std::optional<Error> VerifyChecksum(BlockAddress address, const void* p, size_t n, Hash expectedChecksum) {
    const Hash checksum = Checksum(p, n);
    if (checksum == expectedChecksum) return std::nullopt;
    return Error("checksum mismatch for block " + std::to_string(address) + ", computed: " + detail::go_hex(checksum) +
                 ", expected: " + detail::go_hex(expectedChecksum));
}

// Batched checksums of n host blocks at base + i*stride (length bytes each, or lens[i]),
// routed by the library's cost model (stormck_checksum_batch): its host leg on
// host_threads threads (0 = the pool), the device over PCIe, or both at once on disjoint
// blocks (the split leg, for registered memory), whichever it predicts is fastest.
inline std::vector<Hash> ChecksumBatch(const void* base, size_t n, size_t stride, uint32_t length,
                                       const uint32_t* lens = nullptr, uint32_t host_threads = 0) {
    std::vector<Hash> out(n);
    if (n) detail::check(stormck_checksum_batch(base, stride, lens, length, n, out.data(), host_threads, nullptr));
    return out;
}

enum class Leg : uint32_t { None = STORMCK_LEG_NONE, Host = STORMCK_LEG_HOST, Device = STORMCK_LEG_DEVICE,
                            Split = STORMCK_LEG_SPLIT };

// ChecksumBatch, also reporting the leg the library took.
inline std::vector<Hash> ChecksumBatchLeg(const void* base, size_t n, size_t stride, uint32_t length, Leg* leg,
                                          const uint32_t* lens = nullptr, uint32_t host_threads = 0) {
    std::vector<Hash> out(n);
    uint32_t used = STORMCK_LEG_NONE;
    if (n) detail::check(stormck_checksum_batch(base, stride, lens, length, n, out.data(), host_threads, &used));
    if (leg) *leg = static_cast<Leg>(used);
    return out;
}

// The split leg alone (stormck_checksum_split) on pinned or registered memory: the host
// threads from the front, the route devices from the back. device_blocks:
// STORMCK_SPLIT_BALANCED (sized from the measured rates) or exactly the last
// device_blocks blocks on the devices. *device_done: the blocks the devices hashed.
inline std::vector<Hash> ChecksumBatchSplit(const void* base, size_t n, size_t stride, uint32_t length,
                                            const uint32_t* lens = nullptr, uint32_t host_threads = 0,
                                            uint64_t device_blocks = STORMCK_SPLIT_BALANCED,
                                            uint64_t* device_done = nullptr) {
    std::vector<Hash> out(n);
    if (n)
        detail::check(stormck_checksum_split(base, stride, lens, length, n, out.data(), nullptr, 0, host_threads,
                                             device_blocks, device_done));
    return out;
}

// storm's cache.data registered with the library for its lifetime (the Go binding's
// NewHostArena): page-locked and mapped, so the device and split legs read it in place.
class HostArena {
public:
    explicit HostArena(size_t bytes) : bytes_(bytes), p_(std::aligned_alloc(4096, (bytes + 4095) / 4096 * 4096)) {
        if (!p_) throw std::bad_alloc();
        const int rc = stormck_host_register(p_, bytes_);
        if (rc != STORMCK_OK) {
            std::free(p_);
            throw DeviceError(rc);
        }
    }
    ~HostArena() {
        (void)stormck_host_unregister(p_);
        std::free(p_);
    }
    HostArena(const HostArena&) = delete;
    HostArena& operator=(const HostArena&) = delete;
    uint8_t* data() { return static_cast<uint8_t*>(p_); }
    size_t size() const { return bytes_; }

private:
    size_t bytes_;
    void* p_;
};

// Cache.Commit's data phase as the Go binding's CommitBatch runs it (stormck_commit): the
// dirty forest in `arena` (cache.data; registered: any leg, unregistered: the host leg),
// children first, relocation, each block's Pointer and type stored into its parent.
// `dirty` gets the relocated addresses and birth revisions, as storm's blockMetadata.
struct CommitResult {
    std::vector<Hash> checksums;  // per dirty block, in the caller's order
    BlockAddress last_allocated;
    Leg leg;
};
inline CommitResult CommitBatch(void* arena, std::vector<stormck_dirty_block>& dirty, uint64_t revision,
                                BlockAddress last_allocated, uint32_t host_threads = 0, void* stream = nullptr) {
    CommitResult r{std::vector<Hash>(dirty.size()), last_allocated, Leg::None};
    uint64_t la = last_allocated;
    uint32_t used = STORMCK_LEG_NONE;
    if (!dirty.empty())
        detail::check(stormck_commit(arena, dirty.data(), dirty.size(), revision, &la, r.checksums.data(), stream,
                                     host_threads, &used));
    r.last_allocated = la;
    r.leg = static_cast<Leg>(used);
    return r;
}

// The routing model's rates (bytes/us) as measured so far, and the devices routed calls use.
inline stormck_route_rates RouteRates() {
    stormck_route_rates r{};
    detail::check(stormck_route_get_rates(&r));
    return r;
}
inline void RouteDevices(const std::vector<int>& devices) {
    detail::check(stormck_route_devices(devices.empty() ? nullptr : devices.data(), static_cast<int>(devices.size())));
}

// One process, several GPUs (stormck_shard_plan / stormck_merkle_root_multi): n_total leaves
// dealt into n_shards contiguous shards over `devices`; the caller fills each shard's device
// buffers (d_blocks / stride / len / d_checksums / stream). Returns the shards and the
// combining node's address.
inline std::pair<std::vector<stormck_shard>, BlockAddress> PlanShards(uint64_t n_total, uint32_t n_shards,
                                                                      const std::vector<int>& devices) {
    std::vector<stormck_shard> shards(n_shards);
    uint64_t root_addr = 0;
    detail::check(stormck_shard_plan(n_total, n_shards, devices.data(), static_cast<int>(devices.size()),
                                     shards.data(), &root_addr));
    return {shards, root_addr};
}

// Every shard's checksums (when d_blocks is set) and tree on its device, the shard roots
// gathered over xGMI by in-process RCCL, the combining pointer block hashed on every device.
struct MultiRoot {
    Pointer root;  // {checksum, root_addr, revision}, of type Pointer
    std::vector<Pointer> shard_roots;
    std::vector<BlockType> shard_types;
};
inline MultiRoot MerkleRootDevices(const std::vector<stormck_shard>& shards, uint64_t revision, BlockAddress root_addr,
                                   uint32_t fanout = STORMCK_POINTERS_PER_BLOCK) {
    MultiRoot r{{}, std::vector<Pointer>(shards.size()), std::vector<BlockType>(shards.size())};
    uint8_t type = 0;
    detail::check(stormck_merkle_root_multi(shards.data(), static_cast<uint32_t>(shards.size()), revision, root_addr,
                                            fanout, reinterpret_cast<stormck_pointer*>(&r.root), &type,
                                            reinterpret_cast<stormck_pointer*>(r.shard_roots.data()),
                                            reinterpret_cast<uint8_t*>(r.shard_types.data())));
    return r;
}

// The layout MerkleRootDevices gathers with (stormck_multi_layout; needs no GPU): the shards'
// distinct devices in order of first appearance (the RCCL ranks), the root rows each device
// sends, and each shard's row of the gathered table.
struct GatherLayout {
    std::vector<int32_t> devices;
    uint32_t rows = 0;
    std::vector<uint32_t> table_row;
};
inline GatherLayout MultiLayout(const std::vector<stormck_shard>& shards) {
    GatherLayout g;
    g.devices.resize(64);
    g.table_row.resize(shards.size());
    uint32_t nd = 0;
    detail::check(stormck_multi_layout(shards.data(), static_cast<uint32_t>(shards.size()), g.devices.data(), &nd,
                                       &g.rows, g.table_row.data()));
    g.devices.resize(nd);
    return g;
}

// The device leg alone (stormck_checksum_host: H2D, kernel, D2H pipelined).
inline std::vector<Hash> ChecksumBatchGPU(const void* base, size_t n, size_t stride, uint32_t length,
                                          const uint32_t* lens = nullptr) {
    std::vector<Hash> out(n);
    if (n) detail::check(stormck_checksum_host(base, stride, lens, length, n, out.data()));
    return out;
}

struct VerifyResult {
    uint64_t first_bad;  // n when every block matches
    uint64_t n_bad;
};

// Routed as ChecksumBatch (stormck_verify_batch).
inline VerifyResult VerifyChecksumBatch(const void* base, size_t n, size_t stride, uint32_t length,
                                        const Hash* expected, const uint32_t* lens = nullptr,
                                        uint32_t host_threads = 0) {
    VerifyResult r{n, 0};
    if (!n) return r;
    const int rc =
        stormck_verify_batch(base, stride, lens, length, n, expected, &r.first_bad, &r.n_bad, host_threads, nullptr);
    if (rc != STORMCK_OK && rc != STORMCK_EMISMATCH) throw DeviceError(rc);
    return r;
}

// ---- block layouts -------------------------------------------------------------

// pointer.Block (blocks/pointer/block.go:10-13); PointersPerBlock = 1200 (params.go:6),
// 10 under the `test` tag (params_testing.go:6).
template <size_t PointersPerBlock = 1200>
struct PointerBlock {
    Pointer Pointers[PointersPerBlock];
    BlockType PointedBlockTypes[PointersPerBlock];
};

// blob.Block (blocks/blob/block.go:25-29)
struct BlobBlock {
    uint8_t Data[BlockSize - 8];
    uint64_t NUsedSlots;
};

// objectlist.Block (blocks/objectlist/block.go:29-40); ChunksPerBlock = 600 / 10.
template <size_t ChunksPerBlock = 600>
struct ObjectListBlock {
    uint8_t Blob[ChunksPerBlock * 32];
    uint64_t KeyTagReminders[ChunksPerBlock];
    ObjectID ObjectLinks[ChunksPerBlock];
    uint16_t ChunkPointers[ChunksPerBlock];
    uint16_t NextChunkPointers[ChunksPerBlock];
    uint8_t ChunkPointerStates[ChunksPerBlock];
    uint16_t NUsedChunks;
    uint16_t FreeChunkIndex;
};

// spacelist.Space / Block (blocks/spacelist/block.go:21-36); SpacesPerBlock = 400 / 10.
struct Space {
    uint64_t SpaceIDTagReminder;
    ObjectID NextObjectID;
    Pointer KeyStorePointer;
    Pointer ObjectStorePointer;
    BlockType KeyStoreBlockType;
    BlockType ObjectStoreBlockType;
    uint8_t State;
};
template <size_t SpacesPerBlock = 400>
struct SpaceListBlock {
    Space Spaces[SpacesPerBlock];
    uint16_t NUsedSpaces;
};

// singularity.Block (blocks/singularity/block.go:8-19)
struct SingularityBlock {
    Hash Checksum;
    uint64_t StormID;
    uint64_t Revision;
    uint64_t NBlocks;
    Pointer SpacePointer;
    BlockType SpaceBlockType;
    BlockAddress LastAllocatedBlock;
};

// Go amd64 sizes (unsafe.Sizeof) — what BlockChecksum hashes.
static_assert(sizeof(SingularityBlock) == 72);
static_assert(sizeof(PointerBlock<>) == 30000 && sizeof(PointerBlock<10>) == 256);
static_assert(sizeof(BlobBlock) == 32768);
static_assert(sizeof(ObjectListBlock<>) == 31808 && sizeof(ObjectListBlock<10>) == 536);
static_assert(sizeof(Space) == 72);
static_assert(sizeof(SpaceListBlock<>) == 28808 && sizeof(SpaceListBlock<10>) == 728);
static_assert(sizeof(PointerBlock<>) <= BlockSize && sizeof(ObjectListBlock<>) <= BlockSize &&
              sizeof(SpaceListBlock<>) <= BlockSize);  // blocks/types_test.go:18-32

}  // namespace storm::blocks
