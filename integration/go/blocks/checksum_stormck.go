//go:build stormck

// Package blocks — GPU-backed checksum for storm (drop-in for blocks/checksum.go).
//
// A storm maintainer adds this file to github.com/outofforest/storm/blocks and
// puts `//go:build !stormck` on the existing blocks/checksum.go. `go build
// -tags stormck` then routes block checksums through libstormck; without the tag
// storm is unchanged. Signatures of Checksum, BlockChecksum and VerifyChecksum are
// identical to blocks/checksum.go:10-27. Those single calls (one block, from
// cache/trace.go:282,307, cache/cache.go:73,160, persistence/init.go:44) take the
// library's host leg, stormck_xxh64: one buffer is four serial XXH64 chains, which
// one core walks faster than a GPU launch (DESIGN_LOG.md §5), so unchanged callers pay
// what xxhash.Sum64 costs them today, and like Sum64 the call cannot fail.
// ChecksumBatch / VerifyChecksumBatch / ReadVerifyBatch / CommitBatch are additions
// for batched callers (level-synchronous commit, batched cold-read verify). A batch or
// commit in host memory (storm's cache.data) runs on the leg the library's cost model
// predicts is fastest: the MI355X (gfx950) over PCIe, the library's host threads, or both
// at once on one call (the split leg, for the registered cache.data): the host threads
// take blocks from the front and the GPUs from the back (ChecksumBatch, CommitBatch).
// Without a gfx950 device these calls return the library's error (STORMCK_ENODEV), even
// where the host leg would have been chosen: a stormck build needs its GPU
// (INTEGRATION.md §2).
//
// Not compiled in this repository (no Go toolchain in the build image); the C
// side it binds is exercised by tests/test_abi.py and tests/test_cpp_mirror.py.
package blocks

/*
#cgo CFLAGS: -I${SRCDIR}/../third_party/stormck/include
#cgo LDFLAGS: -L${SRCDIR}/../third_party/stormck/lib -lstormck -Wl,-rpath,${SRCDIR}/../third_party/stormck/lib
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include "stormck.h"
*/
import "C"

import (
	"os"
	"unsafe"

	"github.com/outofforest/photon"
	"github.com/pkg/errors"
)

func stormckError(rc C.int) error {
	return errors.Errorf("stormck error %d: %s", int(rc), C.GoString(C.stormck_last_error()))
}

func bytesPtr(b []byte) unsafe.Pointer {
	if len(b) == 0 {
		return nil
	}
	return unsafe.Pointer(&b[0])
}

// BlockChecksum computes checksum of the block.
func BlockChecksum[T Block](b *T) Hash {
	return Checksum(photon.NewFromValue(b).B)
}

// Checksum computes checksum of bytes (XXH64 seed 0, bit-exact with xxhash.Sum64).
// Like the reference it cannot fail: stormck_xxh64 hashes on the calling thread.
func Checksum(b []byte) Hash {
	// cgo pointer rules: b holds no Go pointers and libstormck does not retain it
	// after the (synchronous) call returns.
	return Hash(C.stormck_xxh64(bytesPtr(b), C.uint64_t(len(b))))
}

// VerifyChecksum verifies that checksum of provided data matches the expected one.
func VerifyChecksum(address BlockAddress, p []byte, expectedChecksum Hash) error {
	checksum := Checksum(p)
	if checksum == expectedChecksum {
		return nil
	}
	return errors.Errorf("checksum mismatch for block %d, computed: %#v, expected: %#v",
		address, checksum, expectedChecksum)
}

// BatchHostThreads is the number of host threads the host leg of ChecksumBatch and
// VerifyChecksumBatch may use (0 = the library's pool, up to 16). It also steers the leg
// choice: with fewer host threads the device and split legs win sooner (DESIGN.md §4.2).
var BatchHostThreads uint32

// ChecksumBatch computes checksums of n blocks at data[i*stride:], length bytes each.
// The blocks live in host memory, so libstormck routes the batch (stormck_checksum_batch)
// to whichever leg its measured cost model predicts is fastest: the GPU, through the PCIe
// link (ChecksumBatchGPU), its host leg on BatchHostThreads threads, or, when data is
// registered (RegisterHostMemory) or otherwise page-locked, both at once. All are bit-exact.
func ChecksumBatch(data []byte, n, stride, length int, out []Hash) error {
	if n == 0 {
		return nil
	}
	if len(out) < n || len(data) < (n-1)*stride+length {
		return errors.New("ChecksumBatch: buffer too small")
	}
	rc := C.stormck_checksum_batch(bytesPtr(data), C.uint64_t(stride), nil, C.uint32_t(length), C.uint64_t(n),
		(*C.uint64_t)(unsafe.Pointer(&out[0])), C.uint32_t(BatchHostThreads), nil)
	if rc != C.STORMCK_OK {
		return stormckError(rc)
	}
	return nil
}

// ChecksumBatchGPU is ChecksumBatch on the GPU leg alone (stormck_checksum_host: H2D,
// kernel and D2H pipelined on the current device).
func ChecksumBatchGPU(data []byte, n, stride, length int, out []Hash) error {
	if n == 0 {
		return nil
	}
	if len(out) < n || len(data) < (n-1)*stride+length {
		return errors.New("ChecksumBatchGPU: buffer too small")
	}
	rc := C.stormck_checksum_host(bytesPtr(data), C.uint64_t(stride), nil, C.uint32_t(length), C.uint64_t(n),
		(*C.uint64_t)(unsafe.Pointer(&out[0])))
	if rc != C.STORMCK_OK {
		return stormckError(rc)
	}
	return nil
}

// ChecksumBatchDevices is ChecksumBatch spread over several GPUs of this process
// (stormck_checksum_host_multi): contiguous ranges, one per entry of devices, each
// over its own device's PCIe link. storm is one process, so this is how one commit
// batch uses every GPU of a node.
func ChecksumBatchDevices(data []byte, n, stride, length int, out []Hash, devices []int32) error {
	if n == 0 {
		return nil
	}
	if len(out) < n || len(data) < (n-1)*stride+length || len(devices) == 0 {
		return errors.New("ChecksumBatchDevices: argument sizes")
	}
	rc := C.stormck_checksum_host_multi(bytesPtr(data), C.uint64_t(stride), nil, C.uint32_t(length), C.uint64_t(n),
		(*C.uint64_t)(unsafe.Pointer(&out[0])), (*C.int)(unsafe.Pointer(&devices[0])), C.int(len(devices)))
	if rc != C.STORMCK_OK {
		return stormckError(rc)
	}
	return nil
}

// VerifyChecksumBatch verifies n blocks; it returns the first mismatching index
// (n when all match) and the number of mismatches. Routed as ChecksumBatch
// (stormck_verify_batch).
func VerifyChecksumBatch(data []byte, n, stride, length int, expected []Hash) (firstBad, nBad int, err error) {
	if n == 0 {
		return 0, 0, nil
	}
	if len(expected) < n || len(data) < (n-1)*stride+length {
		return 0, 0, errors.New("VerifyChecksumBatch: buffer too small")
	}
	var fb, nb C.uint64_t
	rc := C.stormck_verify_batch(bytesPtr(data), C.uint64_t(stride), nil, C.uint32_t(length), C.uint64_t(n),
		(*C.uint64_t)(unsafe.Pointer(&expected[0])), &fb, &nb, C.uint32_t(BatchHostThreads), nil)
	if rc != C.STORMCK_OK && rc != C.STORMCK_EMISMATCH {
		return 0, 0, stormckError(rc)
	}
	return int(fb), int(nb), nil
}

// ReadVerifyBatch reads len(addresses) blocks from the device file f (block i:
// lens[i] bytes at addresses[i]*BlockSize, as persistence.Store.ReadBlock does) into
// dst[i*dstStride:] and verifies each against expected[i] on the GPU — a batched
// cache.fetchBlock cold read (cache/cache.go:139-167). It returns the first
// mismatching index (len(addresses) when all verify) and the mismatch count.
func ReadVerifyBatch(f *os.File, addresses []BlockAddress, lens []uint32, expected []Hash,
	dst []byte, dstStride int) (firstBad, nBad int, err error) {
	n := len(addresses)
	if n == 0 {
		return 0, 0, nil
	}
	if len(lens) != n || len(expected) != n || len(dst) < (n-1)*dstStride+int(BlockSize) {
		return 0, 0, errors.New("ReadVerifyBatch: argument sizes")
	}
	var fb, nb C.uint64_t
	rc := C.stormck_read_verify_fd(C.int(f.Fd()), (*C.uint64_t)(unsafe.Pointer(&addresses[0])),
		(*C.uint32_t)(unsafe.Pointer(&lens[0])), C.uint64_t(n), C.uint64_t(BlockSize), bytesPtr(dst),
		C.uint64_t(dstStride), (*C.uint64_t)(unsafe.Pointer(&expected[0])), 0, &fb, &nb)
	if rc != C.STORMCK_OK && rc != C.STORMCK_EMISMATCH {
		return 0, 0, stormckError(rc)
	}
	return int(fb), int(nb), nil
}

// RegisterHostMemory page-locks a long-lived buffer (e.g. cache.data, allocated once
// in cache.New, cache/cache.go:36-40) so batches DMA straight from it and CommitBatch
// can let the GPU read and write it in place. This keeps a reference to the memory
// inside the HIP runtime after the call returns, which the cgo pointer rules do not
// allow for Go-heap memory: allocate the buffer outside the Go heap (C.malloc, mmap or
// hipHostMalloc, wrapped with unsafe.Slice) and keep it registered until
// UnregisterHostMemory. See INTEGRATION.md §3.
func RegisterHostMemory(b []byte) error {
	if rc := C.stormck_host_register(bytesPtr(b), C.uint64_t(len(b))); rc != C.STORMCK_OK {
		return stormckError(rc)
	}
	return nil
}

// NewHostArena returns n zeroed bytes outside the Go heap (a 4 KiB-aligned C
// allocation), registered with RegisterHostMemory: storm's cache.data in the stormck
// build (cache/cache.go:36-40, newArena in integration/go/cache/commit_stormck.go), the
// arena CommitBatch hashes and updates in place. It lives as long as the process, as
// cache.data does.
func NewHostArena(n int) ([]byte, error) {
	if n <= 0 {
		return nil, errors.New("NewHostArena: size must be positive")
	}
	p := C.aligned_alloc(4096, C.size_t((n+4095)&^4095))
	if p == nil {
		return nil, errors.New("NewHostArena: out of host memory")
	}
	C.memset(p, 0, C.size_t(n))
	b := unsafe.Slice((*byte)(p), n)
	if err := RegisterHostMemory(b); err != nil {
		C.free(p)
		return nil, err
	}
	return b, nil
}

// DirtyBlock mirrors stormck_dirty_block (include/stormck.h): one dirty block of
// Cache.Commit's data phase, its blockMetadata plus its BlockOrigin as byte offsets into
// the arena (cache.data), and the index of its parent record.
type DirtyBlock struct {
	DataOffset    uint64       // offset of the block in the arena
	OriginPointer uint64       // offset of the parent's blocks.Pointer slot, or NoOrigin
	OriginType    uint64       // offset of the parent's BlockType byte, or NoOrigin
	Parent        int64        // index of the parent's record, or NoParent
	Address       BlockAddress // in: current address; out: after relocation
	BirthRevision uint64       // in/out, as commitBlock (cache/cache.go:114-118)
	Length        uint32       // bytes hashed: unsafe.Sizeof of the block's type
	Type          BlockType
	_             [3]byte
}

const (
	NoOrigin = ^uint64(0)
	NoParent = int64(-1)
)

// compile-time check that DirtyBlock has the C layout (56 bytes)
var _ = [1]struct{}{}[unsafe.Sizeof(DirtyBlock{})-56]

// CommitHostThreads is the number of host threads CommitBatch's host leg may use (0 = the
// library's pool, up to 16). It also steers the leg choice: with fewer host threads the
// device leg wins sooner (DESIGN_LOG.md §11 f1, "End to end from host memory").
var CommitHostThreads uint32

// CommitBatch runs Cache.Commit's data phase (cache/cache.go:87-137, trace.go:274-320)
// for every dirty block, children first, level by level, through libstormck's routed
// commit (stormck_commit): the arena is storm's cache.data, registered with
// RegisterHostMemory, and the library picks the faster leg for this forest from its
// measured cost model: the GPU reading and writing the arena in place over PCIe, one
// launch per height, or its host leg (storm's own loop, with each height's blocks spread
// over CommitHostThreads threads when there is enough to hash). Either leg stores each
// {checksum, address, birth revision} and type into the parent's origin in the arena.
// Relocations are written back into dirty; out[i] is dirty[i]'s checksum; leg reports
// the leg taken (LegHost / LegDevice / LegSplit).
func CommitBatch(arena []byte, dirty []DirtyBlock, revision uint64, lastAllocated *BlockAddress, out []Hash) (leg uint32, err error) {
	if len(dirty) == 0 {
		return LegNone, nil
	}
	if len(out) < len(dirty) {
		return LegNone, errors.New("CommitBatch: out too small")
	}
	la := C.uint64_t(*lastAllocated)
	var used C.uint32_t
	rc := C.stormck_commit(bytesPtr(arena), (*C.stormck_dirty_block)(unsafe.Pointer(&dirty[0])), C.uint64_t(len(dirty)),
		C.uint64_t(revision), &la, (*C.uint64_t)(unsafe.Pointer(&out[0])), nil, C.uint32_t(CommitHostThreads), &used)
	// the library reports the relocations it applied to dirty, also on a failure part-way
	*lastAllocated = BlockAddress(la)
	if rc != C.STORMCK_OK {
		return uint32(used), stormckError(rc)
	}
	return uint32(used), nil
}

// Legs of CommitBatch and the routed batches (STORMCK_LEG_*).
const (
	LegNone   = uint32(C.STORMCK_LEG_NONE)
	LegHost   = uint32(C.STORMCK_LEG_HOST)
	LegDevice = uint32(C.STORMCK_LEG_DEVICE)
	LegSplit  = uint32(C.STORMCK_LEG_SPLIT)
)

// SetBatchDevices lists the GPUs the routed calls (ChecksumBatch, VerifyChecksumBatch,
// CommitBatch) may use; each brings its own PCIe link to a split. nil: the calling
// thread's current device (the default). storm is one process, so this is how one commit
// uses every GPU of a node (stormck_route_devices).
func SetBatchDevices(devices []int32) error {
	var p *C.int
	if len(devices) > 0 {
		p = (*C.int)(unsafe.Pointer(&devices[0]))
	}
	if rc := C.stormck_route_devices(p, C.int(len(devices))); rc != C.STORMCK_OK {
		return stormckError(rc)
	}
	return nil
}

// UnregisterHostMemory undoes RegisterHostMemory.
func UnregisterHostMemory(b []byte) error {
	if rc := C.stormck_host_unregister(bytesPtr(b)); rc != C.STORMCK_OK {
		return stormckError(rc)
	}
	return nil
}

// Shard mirrors stormck_shard (include/stormck.h): one device-resident shard of a batch on an
// 8-GPU node, driven from storm's one process. Blocks and Checksums are device addresses on
// Device (e.g. from a HIP allocation the caller owns); they are not Go pointers, so the cgo
// pointer rules do not apply to them.
type Shard struct {
	Blocks       uintptr // block i at Blocks + i*Stride, Len bytes; 0: Checksums already holds the leaf checksums
	Stride       uint64
	N            uint64       // leaves of the shard
	Checksums    uintptr      // N uint64 checksums on Device: written when Blocks is set, read otherwise
	LeafAddrBase BlockAddress // leaf i is addressed LeafAddrBase + i
	NodeAddrBase BlockAddress // the shard tree's interior nodes from here, level by level
	Stream       uintptr      // a HIP stream of Device the shard's work follows (0: the library's own)
	Device       int32
	Len          uint32
}

// compile-time checks that Shard and Pointer have the C layouts (64 and 24 bytes)
var (
	_ = [1]struct{}{}[unsafe.Sizeof(Shard{})-64]
	_ = [1]struct{}{}[unsafe.Sizeof(Pointer{})-24]
)

// PlanShards deals nTotal leaves into nShards contiguous shards over devices
// (stormck_shard_plan: consecutive shards per device, leaf and node addresses disjoint,
// SURVEY.md §8e) and returns them with the combining node's address. The caller fills each
// shard's Blocks / Stride / Len / Checksums / Stream. Needs no GPU.
func PlanShards(nTotal uint64, nShards int, devices []int32) ([]Shard, BlockAddress, error) {
	if nShards <= 0 || len(devices) == 0 {
		return nil, 0, errors.New("PlanShards: need shards and devices")
	}
	shards := make([]Shard, nShards)
	var rootAddr C.uint64_t
	rc := C.stormck_shard_plan(C.uint64_t(nTotal), C.uint32_t(nShards), (*C.int)(unsafe.Pointer(&devices[0])),
		C.int(len(devices)), (*C.stormck_shard)(unsafe.Pointer(&shards[0])), &rootAddr)
	if rc != C.STORMCK_OK {
		return nil, 0, stormckError(rc)
	}
	return shards, BlockAddress(rootAddr), nil
}

// MerkleRootDevices computes the global Merkle root of device-resident shards from this one
// process (stormck_merkle_root_multi): each shard's checksums (when Blocks is set) and its
// pointer-block tree on its own GPU, the shard roots all-gathered over xGMI by in-process
// RCCL, and the combining pointer.Block (blocks/pointer/block.go:10-13) hashed on every GPU.
// It returns the root Pointer (type Pointer) and every shard's root. Synchronous.
func MerkleRootDevices(shards []Shard, revision uint64, rootAddr BlockAddress) (Pointer, []Pointer, []BlockType, error) {
	n := len(shards)
	if n == 0 {
		return Pointer{}, nil, nil, errors.New("MerkleRootDevices: no shards")
	}
	var root Pointer
	var rootType C.uint8_t
	shardRoots := make([]Pointer, n)
	shardTypes := make([]BlockType, n)
	rc := C.stormck_merkle_root_multi((*C.stormck_shard)(unsafe.Pointer(&shards[0])), C.uint32_t(n),
		C.uint64_t(revision), C.uint64_t(rootAddr), C.STORMCK_POINTERS_PER_BLOCK,
		(*C.stormck_pointer)(unsafe.Pointer(&root)), &rootType,
		(*C.stormck_pointer)(unsafe.Pointer(&shardRoots[0])), (*C.uint8_t)(unsafe.Pointer(&shardTypes[0])))
	if rc != C.STORMCK_OK {
		return Pointer{}, nil, nil, stormckError(rc)
	}
	if BlockType(rootType) != PointerBlockType {
		return Pointer{}, nil, nil, errors.Errorf("MerkleRootDevices: root of type %d", rootType)
	}
	return root, shardRoots, shardTypes, nil
}

// GatherLayout returns the layout MerkleRootDevices gathers the shard roots with
// (stormck_multi_layout): the shards' distinct devices in order of first appearance (the
// RCCL ranks), the root rows each device sends, and each shard's row of the gathered table.
// Needs no GPU.
func GatherLayout(shards []Shard) ([]int32, int, []uint32, error) {
	n := len(shards)
	if n == 0 {
		return nil, 0, nil, errors.New("GatherLayout: no shards")
	}
	devices := make([]int32, 64)
	tableRow := make([]uint32, n)
	var nDev, rows C.uint32_t
	rc := C.stormck_multi_layout((*C.stormck_shard)(unsafe.Pointer(&shards[0])), C.uint32_t(n),
		(*C.int32_t)(unsafe.Pointer(&devices[0])), &nDev, &rows, (*C.uint32_t)(unsafe.Pointer(&tableRow[0])))
	if rc != C.STORMCK_OK {
		return nil, 0, nil, stormckError(rc)
	}
	return devices[:nDev], int(rows), tableRow, nil
}
