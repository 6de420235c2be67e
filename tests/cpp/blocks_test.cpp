// C++ mirror of storm's blocks tests, run against libstormck (batches and ChecksumGPU on
// the GPU, single calls on the library's host leg), plus the routed legs on a registered
// arena (HostArena, the split leg).
// Each TEST mirrors a reference test (file:line in its comment). Relations are
// asserted here; absolute values are printed as one JSON object for
// tests/test_cpp_mirror.py to compare with tests/golden/layouts.json.
#include <cstddef>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "storm_blocks.hpp"

using namespace storm::blocks;

static int g_fail = 0;
#define EXPECT(cond)                                                               \
    do {                                                                           \
        if (!(cond)) {                                                             \
            std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond);   \
            ++g_fail;                                                              \
        }                                                                          \
    } while (0)

static std::string hex(uint64_t v) {
    char b[24];
    std::snprintf(b, sizeof b, "\"0x%016llx\"", static_cast<unsigned long long>(v));
    return b;
}

// blocks/pointer/block_test.go:11-35
static std::string TestPointerChecksum() {
    auto b = std::make_unique<PointerBlock<>>();
    std::memset(b.get(), 0, sizeof(*b));
    std::vector<Hash> seq;
    seq.push_back(BlockChecksum(b.get()));
    b->Pointers[0].Checksum = 2;
    seq.push_back(BlockChecksum(b.get()));
    b->PointedBlockTypes[0] = LeafBlockType;
    seq.push_back(BlockChecksum(b.get()));
    b->PointedBlockTypes[1] = LeafBlockType;
    seq.push_back(BlockChecksum(b.get()));
    b->Pointers[1].Address = 2;
    seq.push_back(BlockChecksum(b.get()));
    b->Pointers[2].Checksum = 4;
    seq.push_back(BlockChecksum(b.get()));
    for (size_t i = 1; i < seq.size(); ++i) EXPECT(seq[i] != seq[i - 1]);
    EXPECT(ChecksumGPU(b.get(), sizeof(*b)) == seq.back());  // the device single call agrees
    std::string out = "[";
    for (size_t i = 0; i < seq.size(); ++i) out += (i ? "," : "") + hex(seq[i]);
    return out + "]";
}

// blocks/blob/block_test.go:13-49: four Object[item]{tag, {f1, f2}, state} in Data
struct Item {
    uint64_t Field1;
    uint8_t Field2;
};
struct Object {
    uint64_t ObjectIDTagReminder;
    Item Obj;
    uint8_t State;
};
static std::string TestMappingBlobToSlice() {
    auto block = std::make_unique<BlobBlock>();
    std::memset(block.get(), 0, sizeof(*block));
    const Hash before = BlockChecksum(block.get());
    Object items[4] = {{1, {2, 3}, 1}, {4, {5, 6}, 2}, {7, {8, 9}, 0}, {10, {11, 12}, 1}};
    static_assert(sizeof(Object) == 32, "Go layout of Object[item]");
    for (int k = 0; k < 4; ++k) {
        Object o{};
        std::memset(&o, 0, sizeof o);  // padding zeroed, as newBlock does (cache/cache.go:282-284)
        o.ObjectIDTagReminder = items[k].ObjectIDTagReminder;
        o.Obj.Field1 = items[k].Obj.Field1;
        o.Obj.Field2 = items[k].Obj.Field2;
        o.State = items[k].State;
        std::memcpy(block->Data + 32 * k, &o, sizeof o);
    }
    const uint8_t want_rows[4][4] = {{1, 2, 3, 1}, {4, 5, 6, 2}, {7, 8, 9, 0}, {10, 11, 12, 1}};
    for (int k = 0; k < 4; ++k)
        for (int q = 0; q < 4; ++q) {
            EXPECT(block->Data[32 * k + 8 * q] == want_rows[k][q]);
            for (int z = 1; z < 8; ++z) EXPECT(block->Data[32 * k + 8 * q + z] == 0);
        }
    const Hash after = BlockChecksum(block.get());
    EXPECT(after != before);
    return hex(after);
}

// cache/cache_test.go:23-42 + persistence/store_test.go:26-48: singularity checksum
// over the block with Checksum = 0; a corrupted checksum must fail verification.
static std::string TestSingularity() {
    SingularityBlock s;
    std::memset(&s, 0, sizeof s);
    s.StormID = 0x73746F726D;
    s.Revision = 3;
    s.NBlocks = 1 << 20;
    s.SpacePointer = Pointer{0x1122334455667788ULL, 42, 2};
    s.SpaceBlockType = LeafBlockType;
    s.LastAllocatedBlock = 777;
    s.Checksum = 0;
    const Hash cs = BlockChecksum(&s);
    s.Checksum = cs;
    SingularityBlock copy = s;
    copy.Checksum = 0;
    EXPECT(!VerifyChecksum(0, &copy, sizeof copy, cs).has_value());
    auto err = VerifyChecksum(0, &copy, sizeof copy, 0);
    EXPECT(err.has_value());
    if (err) EXPECT(err->message() == "checksum mismatch for block 0, computed: " + detail::go_hex(cs) + ", expected: 0x0");
    return hex(cs);
}

// cache/cache_test.go:260-300 (TestNewBlocksProduceConsistentResult): a struct with
// padding, created twice in randomised memory with the same field values. newBlock
// zeroes the slot first (cache/cache.go:282-284), so the two images, padding
// included, and their checksums are identical; without the zeroing they differ.
struct paddedStruct {
    uint64_t Field1;
    uint8_t Field2;
    uint64_t Field3;
};
static_assert(sizeof(paddedStruct) == 24, "Go layout: 7 padding bytes after Field2");
static void TestNewBlocksProduceConsistentResult() {
    uint8_t slot1[sizeof(paddedStruct)], slot2[sizeof(paddedStruct)];
    uint64_t x = 0x243F6A8885A308D3ULL;
    for (size_t i = 0; i < sizeof slot1; ++i) {  // randomizeCache
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        slot1[i] = static_cast<uint8_t>(x);
        slot2[i] = static_cast<uint8_t>(x >> 8);
    }
    auto fill = [](uint8_t* slot, bool zero) {
        if (zero) std::memset(slot, 0, sizeof(paddedStruct));  // newBlock
        paddedStruct v;
        std::memcpy(&v, slot, sizeof v);
        v.Field1 = 1;
        v.Field2 = 0x02;
        v.Field3 = 3;
        std::memcpy(slot, &v, sizeof v);
    };
    fill(slot1, true);
    fill(slot2, true);
    EXPECT(std::memcmp(slot1, slot2, sizeof slot1) == 0);
    EXPECT(Checksum(slot1, sizeof slot1) == Checksum(slot2, sizeof slot2));
    uint8_t dirty1[sizeof slot1], dirty2[sizeof slot2];
    std::memset(dirty1, 0xAB, sizeof dirty1);
    std::memset(dirty2, 0xCD, sizeof dirty2);
    fill(dirty1, false);
    fill(dirty2, false);
    EXPECT(Checksum(dirty1, sizeof dirty1) != Checksum(dirty2, sizeof dirty2));  // padding is hashed
}

// blocks.Checksum on "abc" and the empty slice (public XXH64 answers)
static void TestKnownAnswers() {
    EXPECT(Checksum("abc", 3) == 0x44BC2CF5AD770999ULL);
    EXPECT(Checksum(nullptr, 0) == 0xEF46DB3751D8E999ULL);
    EXPECT(ChecksumGPU("abc", 3) == 0x44BC2CF5AD770999ULL);
    EXPECT(ChecksumGPU(nullptr, 0) == 0xEF46DB3751D8E999ULL);
    auto err = VerifyChecksum(42, "abc", 3, 0);
    EXPECT(err && err->message() == "checksum mismatch for block 42, computed: 0x44bc2cf5ad770999, expected: 0x0");
}

// batch == per-block single calls, and verify finds a corrupted block
static void TestBatch() {
    const size_t n = 300, stride = 32768;
    std::vector<uint8_t> buf(n * stride);
    uint64_t x = 0x9E3779B97F4A7C15ULL;
    for (auto& c : buf) {
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        c = static_cast<uint8_t>(x);
    }
    auto cs = ChecksumBatch(buf.data(), n, stride, stride);
    for (size_t i = 0; i < n; i += 37) EXPECT(cs[i] == Checksum(buf.data() + i * stride, stride));
    EXPECT(ChecksumBatchGPU(buf.data(), n, stride, stride) == cs);  // the device leg alone
    EXPECT(ChecksumBatch(buf.data(), n, stride, stride, nullptr, 1) == cs);
    auto ok = VerifyChecksumBatch(buf.data(), n, stride, stride, cs.data());
    EXPECT(ok.first_bad == n && ok.n_bad == 0);
    buf[123 * stride + 7] ^= 1;
    auto bad = VerifyChecksumBatch(buf.data(), n, stride, stride, cs.data());
    EXPECT(bad.first_bad == 123 && bad.n_bad == 1);
}

// The routed legs on storm's configuration: cache.data registered (HostArena), the routed
// batch, the split leg with fixed and balanced shares, verify across the boundary.
static void TestRoutedLegs() {
    const size_t n = 2000, stride = 32768;
    HostArena arena(n * stride);
    uint64_t x = 0x2545F4914F6CDD1DULL;
    for (size_t i = 0; i < arena.size(); ++i) {
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        arena.data()[i] = static_cast<uint8_t>(x);
    }
    std::vector<uint32_t> lens(n);
    const uint32_t storm[] = {72, 28808, 30000, 31808, 32768};
    for (size_t i = 0; i < n; ++i) lens[i] = storm[(i * 7) % 5];
    std::vector<Hash> want(n);
    for (size_t i = 0; i < n; ++i) want[i] = Checksum(arena.data() + i * stride, lens[i]);
    Leg leg = Leg::None;
    EXPECT(ChecksumBatchLeg(arena.data(), n, stride, 0, &leg, lens.data()) == want);
    EXPECT(leg == Leg::Host || leg == Leg::Device || leg == Leg::Split);
    for (uint64_t d : {uint64_t{0}, uint64_t{1}, uint64_t{n / 2}, uint64_t{n}}) {
        uint64_t done = ~0ULL;
        EXPECT(ChecksumBatchSplit(arena.data(), n, stride, 0, lens.data(), 0, d, &done) == want);
        EXPECT(done == d);
    }
    EXPECT(ChecksumBatchSplit(arena.data(), n, stride, 0, lens.data(), 1) == want);  // balanced, one host thread
    std::vector<Hash> bad = want;
    bad[n / 2 - 1] ^= 1;
    bad[n / 2] ^= 1;
    uint64_t fb = 0, nb = 0, dd = 0;
    const int rc = stormck_verify_split(arena.data(), stride, lens.data(), 0, n, bad.data(), &fb, &nb, nullptr, 0, 0,
                                        n / 2, &dd);
    EXPECT(rc == STORMCK_EMISMATCH && fb == n / 2 - 1 && nb == 2 && dd == n / 2);
    EXPECT(RouteRates().host_thread > 0);
    RouteDevices({});
}

// Cache.Commit's data phase (cache/cache.go:87-137, trace.go:274-320) through CommitBatch:
// three objectlist leaves under one pointer block in a registered arena. Leaves first,
// relocated in order, their Pointers and types stored into the pointer block, whose
// checksum then covers them.
static void TestCommitBatch() {
    const size_t slot = 32768;
    HostArena arena(4 * slot);
    std::memset(arena.data(), 0, arena.size());
    for (size_t i = slot; i < arena.size(); ++i) arena.data()[i] = static_cast<uint8_t>(i * 2654435761u >> 13);
    std::vector<stormck_dirty_block> dirty(4);
    for (int i = 0; i < 3; ++i) {
        dirty[i] = {};
        dirty[i].data_offset = (i + 1) * slot;
        dirty[i].origin_pointer = i * sizeof(Pointer);
        dirty[i].origin_type = offsetof(PointerBlock<>, PointedBlockTypes) + i;
        dirty[i].parent = 3;
        dirty[i].address = 10 + i;
        dirty[i].birth_revision = 1;
        dirty[i].length = sizeof(ObjectListBlock<>);
        dirty[i].type = LeafBlockType;
    }
    dirty[3] = {};
    dirty[3].data_offset = 0;
    dirty[3].origin_pointer = STORMCK_NO_ORIGIN;
    dirty[3].parent = STORMCK_NO_PARENT;
    dirty[3].address = 50;
    dirty[3].birth_revision = 1;
    dirty[3].length = sizeof(PointerBlock<>);
    dirty[3].type = PointerBlockType;
    std::vector<Hash> leaves(3);
    for (int i = 0; i < 3; ++i) leaves[i] = Checksum(arena.data() + (i + 1) * slot, sizeof(ObjectListBlock<>));
    const CommitResult r = CommitBatch(arena.data(), dirty, 5, 100);
    EXPECT(r.leg == Leg::Host || r.leg == Leg::Device || r.leg == Leg::Split);
    EXPECT(r.last_allocated == 104);
    const auto* pb = reinterpret_cast<const PointerBlock<>*>(arena.data());
    for (int i = 0; i < 3; ++i) {
        EXPECT(r.checksums[i] == leaves[i]);
        EXPECT(dirty[i].address == 101u + i && dirty[i].birth_revision == 6);
        EXPECT(pb->Pointers[i].Checksum == leaves[i] && pb->Pointers[i].Address == 101u + i &&
               pb->Pointers[i].BirthRevision == 6 && pb->PointedBlockTypes[i] == LeafBlockType);
    }
    EXPECT(dirty[3].address == 104 && r.checksums[3] == BlockChecksum(pb));
}

// zero blocks of every type (prod sizes and `test`-tag sizes)
template <class T>
static std::string zero_cs() {
    auto b = std::make_unique<T>();
    std::memset(b.get(), 0, sizeof(T));
    return hex(BlockChecksum(b.get()));
}

// The one-process multi-GPU root through the mirror: 4 shards of 5,000 synthetic 4 KiB blocks
// (logical blocks 0..19,999, stormck_fill_synthetic_device) on device 0, hashed, treed,
// gathered through a one-rank RCCL communicator and combined; tests/test_cpp_mirror.py checks
// the roots against the oracle.
static std::string TestMerkleRootDevices() {
    const uint64_t n_total = 20000, stride = 4096;
    auto [shards, root_addr] = PlanShards(n_total, 4, {0});
    EXPECT(root_addr == 2 * n_total && shards.size() == 4);
    // the gather layout: one device sends all four rows; interleaved over three devices, ranks
    // by first appearance and R = 2 rows each
    const GatherLayout one = MultiLayout(shards);
    EXPECT(one.devices == std::vector<int32_t>{0} && one.rows == 4 &&
           one.table_row == std::vector<uint32_t>({0, 1, 2, 3}));
    std::vector<stormck_shard> mixed = shards;
    const int32_t on[4] = {3, 1, 3, 2};
    for (int k = 0; k < 4; ++k) mixed[k].device = on[k];
    const GatherLayout three = MultiLayout(mixed);
    EXPECT(three.devices == std::vector<int32_t>({3, 1, 2}) && three.rows == 2 &&
           three.table_row == std::vector<uint32_t>({0, 2, 1, 4}));
    void* blocks = nullptr;
    void* cs = nullptr;
    detail::check(stormck_device_alloc(n_total * stride, &blocks));
    detail::check(stormck_device_alloc(n_total * 8, &cs));
    detail::check(stormck_fill_synthetic_device(blocks, stride, n_total, 0, 0x53544F524DULL, nullptr));
    detail::check(stormck_device_status(nullptr));  // the fill (null stream) has landed
    for (stormck_shard& sh : shards) {
        sh.d_blocks = static_cast<uint8_t*>(blocks) + sh.leaf_addr_base * stride;
        sh.stride = stride;
        sh.len = static_cast<uint32_t>(stride);
        sh.d_checksums = static_cast<uint64_t*>(cs) + sh.leaf_addr_base;
    }
    const MultiRoot r = MerkleRootDevices(shards, 1, root_addr);
    EXPECT(r.root.Address == root_addr && r.root.BirthRevision == 1);
    std::string out = "{\"root\": " + hex(r.root.Checksum) + ", \"shard_roots\": [";
    for (size_t k = 0; k < r.shard_roots.size(); ++k) {
        EXPECT(r.shard_types[k] == LeafBlockType || r.shard_types[k] == PointerBlockType);
        out += (k ? ", [" : "[") + hex(r.shard_roots[k].Checksum) + ", " + std::to_string(r.shard_roots[k].Address) +
               ", " + std::to_string(static_cast<int>(r.shard_types[k])) + "]";
    }
    detail::check(stormck_device_free(blocks));
    detail::check(stormck_device_free(cs));
    return out + "]}";
}

int main() {
    std::string ptr = TestPointerChecksum();
    std::string blob = TestMappingBlobToSlice();
    std::string sing = TestSingularity();
    TestKnownAnswers();
    TestBatch();
    TestRoutedLegs();
    TestCommitBatch();
    TestNewBlocksProduceConsistentResult();
    std::string multi = TestMerkleRootDevices();
    std::printf("{\"multi\": %s, \"pointer_block_test_sequence\": %s, \"blob_test_block\": %s, \"singularity\": %s, "
                "\"zero\": {\"prod\": {\"pointer\": %s, \"objectlist\": %s, \"spacelist\": %s, \"blob\": %s, "
                "\"singularity\": %s}, \"test\": {\"pointer\": %s, \"objectlist\": %s, \"spacelist\": %s}}, "
                "\"failures\": %d}\n",
                multi.c_str(), ptr.c_str(), blob.c_str(), sing.c_str(), zero_cs<PointerBlock<>>().c_str(),
                zero_cs<ObjectListBlock<>>().c_str(), zero_cs<SpaceListBlock<>>().c_str(), zero_cs<BlobBlock>().c_str(),
                zero_cs<SingularityBlock>().c_str(), zero_cs<PointerBlock<10>>().c_str(),
                zero_cs<ObjectListBlock<10>>().c_str(), zero_cs<SpaceListBlock<10>>().c_str(), g_fail);
    return g_fail ? 1 : 0;
}
