/*
 * stormck — MI355X-native block-checksum engine for storm (C ABI).
 *
 * Drop-in boundary for storm's per-block content hash (Go package `blocks`):
 *
 *   func Checksum(b []byte) Hash                         /root/reference/blocks/checksum.go:15-17
 *   func BlockChecksum[T Block](b *T) Hash               /root/reference/blocks/checksum.go:10-12
 *   func VerifyChecksum(address, p, expected) error      /root/reference/blocks/checksum.go:20-27
 *   type Pointer struct{Checksum, Address, BirthRevision} /root/reference/blocks/types.go:35-39
 *
 * The hash is XXH64 with seed 0 (github.com/cespare/xxhash/v2 v2.2.0 Sum64,
 * /root/reference/go.mod:6), bit-exact. All entry points are plain C: pointers and
 * sizes only. Every function returns 0 on success or a negative STORMCK_E* code;
 * stormck_last_error() then holds a thread-local message.
 *
 * "_device" entry points take device pointers (HBM) and a hipStream_t passed as
 * void* (NULL = the null stream of the calling thread's current device); they are
 * asynchronous with respect to the host, like any kernel launch on that stream.
 * "_host" entry points take host memory and return when the results are in host
 * memory (H2D -> kernel -> D2H, pipelined).
 *
 * There is no CPU fallback: without a usable gfx950 device every batched, device,
 * routed and Merkle entry point returns STORMCK_ENODEV. Host computation is a measured leg,
 * never a substitute for a missing device:
 *  - the latency leg of a SINGLE call (stormck_xxh64 / stormck_checksum): one buffer is
 *    four serial XXH64 chains, which one host core walks faster than the GPU at every
 *    length, so single calls stay on the host by design;
 *  - the host legs of data that lives in HOST memory (stormck_commit_host,
 *    stormck_checksum_host_leg), which the routed entry points (stormck_commit,
 *    stormck_checksum_batch) run alone, or beside the devices (the split leg), when the
 *    library's cost model predicts that is faster than the PCIe-bound device leg.
 */
#ifndef STORMCK_H
#define STORMCK_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define STORMCK_ABI_VERSION 7

#define STORMCK_OK 0
#define STORMCK_EINVAL (-1)  /* bad argument (null pointer, n/len/stride out of range, ...) */
#define STORMCK_EHIP (-2)    /* HIP runtime error */
#define STORMCK_ENODEV (-3)  /* no usable gfx950 device */
#define STORMCK_ENOMEM (-4)  /* device / pinned allocation failed */
#define STORMCK_EMISMATCH (-5) /* verify: at least one checksum differs (see first_bad) */

/* storm block types, blocks/types.go:7-15 */
#define STORMCK_FREE_BLOCK 0
#define STORMCK_POINTER_BLOCK 1
#define STORMCK_LEAF_BLOCK 2

/* storm's PointersPerBlock (blocks/pointer/params.go:6; 10 under the `test` build tag,
 * blocks/pointer/params_testing.go:6). */
#define STORMCK_POINTERS_PER_BLOCK 1200

/* blocks.Pointer, 24 bytes, Go amd64 layout (blocks/types.go:35-39). */
typedef struct stormck_pointer {
    uint64_t checksum;
    uint64_t address;
    uint64_t birth_revision;
} stormck_pointer;

/* ---- library / device ---------------------------------------------------- */

int stormck_abi_version(void);
/* Provenance of this build: "sha256:<hex>" of the sources it was compiled from
 * (storm_amd/build.py SOURCES), so a prebuilt library can be matched to a tree. */
const char* stormck_build_id(void);
const char* stormck_last_error(void);
/* Number of visible gfx950 devices (0 on a machine without one). */
int stormck_device_count(int* count);
/* Select `device` for the calling thread and register its context. Pinned staging
 * for the host path is allocated lazily by the first _host call on that device. */
int stormck_init(int device);
/* Free pinned staging / device buffers of every context. */
void stormck_shutdown(void);
/* Ring-kernel faults. The small-batch kernels stage blocks through an LDS ring whose
 * waits are bounded; a wait that expires (a liveness bug, never expected) is an error,
 * not a value: the kernel writes no checksum for the blocks of the stalled workgroup (a
 * verify counts each of them as a mismatch, so it fails closed) and records the fault in
 * the slot of the STREAM it was launched on. Host-synchronous entry points (_host,
 * _host_multi, stormck_commit_device, stormck_read_verify_fd) check their own streams'
 * slots after their sync and return STORMCK_EHIP naming the kernel; their outputs are
 * then unspecified. For the asynchronous _device entry points, stormck_device_status
 * synchronises `stream` and returns STORMCK_EHIP if a ring kernel launched on that
 * stream (on the calling thread's current device) faulted since the last check (the
 * fault is then cleared), otherwise the stream's own status. Faults never cross streams:
 * concurrent callers on distinct streams see only their own (the legacy null stream is
 * one stream, shared by every thread of the device). The slots are allocated by
 * stormck_init; a first ring launch inside a stream capture without it is STORMCK_EINVAL.
 * A ring launch captured into a graph reports into the slot of the stream it was
 * captured on, so check that stream after replays (status on a stream that is being
 * captured is STORMCK_EINVAL).
 * Up to 1024 streams per device have a slot of their own at once; past that the least
 * recently launched stream with no pending fault gives its slot up. */
int stormck_device_status(void* stream);
/* Release `stream`'s fault slot on the calling thread's current device; call it before
 * destroying a stream that ring kernels were launched on. It synchronises the stream, and
 * returns STORMCK_EHIP if a fault was still pending there (which is then cleared), so a
 * stream created later with the same handle never inherits it. */
int stormck_stream_forget(void* stream);
/* Device memory for a block arena (storm's cache.data mirrored in HBM): hipMalloc on the
 * calling thread's current device, outside any caching allocator, so an arena taken first
 * in a process is placed the same way whatever else the process allocates. */
int stormck_device_alloc(uint64_t bytes, void** d_ptr);
int stormck_device_free(void* d_ptr);

/* ---- hot path: batch checksums of device-resident blocks -------------------
 * Block i starts at d_base + i*stride and is (d_lens ? d_lens[i] : len) bytes
 * long. out[i] = XXH64(block i) = blocks.Checksum(block bytes). Any alignment is
 * accepted; 8-byte-aligned blocks take the fast path. n == 0 is a no-op.
 * With d_lens, len may carry an upper bound of the lengths (0 = unknown), which the
 * library plans the launch with: batches of short blocks (storm's `-tags test` sizes)
 * take a different kernel than 32 KiB ones. Results never depend on it. The same holds
 * for the gather and verify entry points below. */
int stormck_checksum_device(const void* d_base, uint64_t stride, const uint32_t* d_lens, uint32_t len,
                            uint64_t n, uint64_t* d_out, void* stream);

/* Same, block i at d_base + d_offsets[i] (e.g. the dirty slots of storm's cache.data,
 * /root/reference/cache/cache.go:36-40). */
int stormck_checksum_gather_device(const void* d_base, const uint64_t* d_offsets, const uint32_t* d_lens,
                                   uint32_t len, uint64_t n, uint64_t* d_out, void* stream);

/* Batched blocks.VerifyChecksum. d_result[0] = index of the first block whose checksum
 * differs from d_expected (n if none), d_result[1] = number of mismatches. The result
 * is written on `stream` (no host sync); check it after synchronising. */
int stormck_verify_device(const void* d_base, uint64_t stride, const uint32_t* d_lens, uint32_t len,
                          uint64_t n, const uint64_t* d_expected, uint64_t* d_result, void* stream);

/* ---- host-memory batch (starts and ends in host memory) -------------------- */

/* out[i] = XXH64 of host block i (base + i*stride, lens ? lens[i] : len). Pipelined
 * H2D / kernel / D2H through library-owned pinned staging on the calling thread's
 * current device; memory registered with stormck_host_register is DMA'd directly. */
int stormck_checksum_host(const void* base, uint64_t stride, const uint32_t* lens, uint32_t len, uint64_t n,
                          uint64_t* out);
/* Batched verify of host blocks: *first_bad = first mismatching index (n if none),
 * *n_bad = mismatch count. Returns STORMCK_EMISMATCH if n_bad > 0. */
int stormck_verify_host(const void* base, uint64_t stride, const uint32_t* lens, uint32_t len, uint64_t n,
                        const uint64_t* expected, uint64_t* first_bad, uint64_t* n_bad);
/* The same two calls spread over several devices from one process (storm is one Go
 * process; each device has its own PCIe link): the n blocks split into n_devices
 * contiguous ranges whose sizes differ by at most one, and range k runs on
 * devices[k] in its own host thread. Results are as from the single-device calls
 * (first_bad is the lowest mismatching index of the whole batch, n_bad the total).
 * A device may be listed more than once; its ranges then run one after another.
 * Memory registered with stormck_host_register is pinned for every device. The
 * calling thread's current device is left as it was. On failure the message names
 * the device and block range of the lowest failing range. */
int stormck_checksum_host_multi(const void* base, uint64_t stride, const uint32_t* lens, uint32_t len, uint64_t n,
                                uint64_t* out, const int* devices, int n_devices);
int stormck_verify_host_multi(const void* base, uint64_t stride, const uint32_t* lens, uint32_t len, uint64_t n,
                              const uint64_t* expected, uint64_t* first_bad, uint64_t* n_bad, const int* devices,
                              int n_devices);
/* A host-memory batch routed by cost (the Go shim's ChecksumBatch / VerifyChecksumBatch).
 * Over PCIe a device moves about 52 GiB/s end to end, while host threads hash the same
 * bytes four blocks at a time (AVX-512) until host memory binds: stormck_checksum_batch runs
 * each batch on the leg the library's cost model predicts is fastest (the routing section
 * below): the host leg, the device leg (stormck_checksum_host, or _host_multi over the route
 * devices), or, for pinned or registered memory, the split leg (both at once).
 * host_threads: threads the host part may use (0 = the library pool, at most 16; 1 = keep
 * the other cores for the caller; a call that finds the pool held by another call plans
 * with its own thread only). *leg_used (optional) = STORMCK_LEG_HOST / _DEVICE / _SPLIT.
 * Same arguments, results and errors as the _host calls; device memory, or memory the host
 * cannot read, is STORMCK_EINVAL (use _device). Needs a gfx950 device like every batched
 * entry point: STORMCK_ENODEV without one, even when the model would pick the host leg
 * (a stormck build needs its GPU).
 * stormck_checksum_host_leg / stormck_verify_host_leg: the host leg alone, on `threads`
 * pool threads (0 = the pool); needs no device. */
int stormck_checksum_batch(const void* base, uint64_t stride, const uint32_t* lens, uint32_t len, uint64_t n,
                           uint64_t* out, uint32_t host_threads, uint32_t* leg_used);
int stormck_verify_batch(const void* base, uint64_t stride, const uint32_t* lens, uint32_t len, uint64_t n,
                         const uint64_t* expected, uint64_t* first_bad, uint64_t* n_bad, uint32_t host_threads,
                         uint32_t* leg_used);
int stormck_checksum_host_leg(const void* base, uint64_t stride, const uint32_t* lens, uint32_t len, uint64_t n,
                              uint64_t* out, uint32_t threads);
int stormck_verify_host_leg(const void* base, uint64_t stride, const uint32_t* lens, uint32_t len, uint64_t n,
                            const uint64_t* expected, uint64_t* first_bad, uint64_t* n_bad, uint32_t threads);
/* ---- single calls (Go blocks.Checksum / BlockChecksum / VerifyChecksum, one block)
 * stormck_xxh64: XXH64 seed 0 of p[0..n_bytes) on the calling host thread; cannot
 * fail (p may be NULL only when n_bytes == 0). What the Go shim's Checksum calls.
 * stormck_checksum: the single-call dispatch. Below the measured host/device crossover
 * (never reached: the device single call is slower at every length, DESIGN_LOG.md §5) it
 * is stormck_xxh64; any length, no device needed.
 * stormck_checksum_gpu: the same hash through the device: one k_xxh64_single launch
 * for slices up to 64 KiB, the host pipeline with a batch of one up to 256 MiB;
 * longer slices return STORMCK_EINVAL. Needs a device. */
uint64_t stormck_xxh64(const void* p, uint64_t n_bytes);
int stormck_checksum(const void* p, uint64_t n_bytes, uint64_t* out);
int stormck_checksum_gpu(const void* p, uint64_t n_bytes, uint64_t* out);
/* Page-lock and map a host range (for every device) so the device and split legs DMA it or
 * read it in place, without staging copies. Also sets up the calling thread's current
 * device's staging for those legs (once per process: 2.25 GiB of HBM and 1 GiB of pinned
 * host memory, ~0.3 s), so the first routed call that uses the device does not pay for it.
 * The library keeps the range in its own list (the routed calls recognise it without a
 * runtime query): release it with stormck_host_unregister, not hipHostUnregister directly. */
int stormck_host_register(void* p, uint64_t bytes);
int stormck_host_unregister(void* p);
/* Device-visible address of host memory registered with stormck_host_register: the
 * *_device entry points (stormck_commit_device's arena included) then read and write
 * it in place over PCIe. This runs f1 on storm's cache.data where it lives, in host
 * memory (cache/cache.go:36-40), at link rate instead of HBM rate. Block rows must be
 * 256-byte aligned for that (a 16-byte offset costs about a quarter of the rate). */
int stormck_host_device_pointer(void* p, void** d_p);

/* ---- Merkle pointer tree (storm pointer.Block nodes) -----------------------
 * One level: children are entries {cs[i], child_addr_base + i, rev}, all of type
 * child_type. Parent j packs children [j*fanout, min((j+1)*fanout, m)) into a storm
 * pointer.Block (blocks/pointer/block.go:10-13; size = 25*fanout rounded up to 8
 * bytes, unused slots zero) and d_parent_cs[j] = XXH64(that block). The node bytes
 * are never materialised: each word is synthesised from the child arrays. */
int stormck_pointer_level_device(const uint64_t* d_child_cs, uint64_t m, uint64_t child_addr_base,
                                 uint64_t rev, uint8_t child_type, uint32_t fanout, uint64_t* d_parent_cs,
                                 void* stream);
/* One node from explicit entries (d_entries[0..count), d_types[0..count)), count <=
 * fanout. Writes *d_out_cs. Used to combine per-shard roots. */
int stormck_pointer_node_device(const stormck_pointer* d_entries, const uint8_t* d_types, uint32_t count,
                                uint32_t fanout, uint64_t* d_out_cs, void* stream);
/* Materialise pointer blocks of one level (same rule as pointer_level) into
 * d_blocks (pm blocks at dst_stride bytes), e.g. to be written to storage. */
int stormck_pack_pointer_blocks_device(const uint64_t* d_child_cs, uint64_t m, uint64_t child_addr_base,
                                       uint64_t rev, uint8_t child_type, uint32_t fanout, void* d_blocks,
                                       uint64_t dst_stride, void* stream);
/* Workspace bytes stormck_merkle_root_device needs for n leaves. */
uint64_t stormck_merkle_workspace_bytes(uint64_t n, uint32_t fanout);
/* Whole shard tree (DESIGN.md "Shard Merkle tree"): leaves {d_leaf_cs[i],
 * leaf_addr_base + i, rev} of type Leaf; interior nodes get addresses
 * node_addr_base, node_addr_base+1, ... level by level, bottom-up. Writes the root
 * Pointer to *d_root and its type to *d_root_type (device memory). n == 0 -> zero root,
 * type Free; n == 1 -> the leaf's own pointer, type Leaf. */
int stormck_merkle_root_device(const uint64_t* d_leaf_cs, uint64_t n, uint64_t leaf_addr_base,
                               uint64_t node_addr_base, uint64_t rev, uint32_t fanout, void* d_workspace,
                               uint64_t workspace_bytes, stormck_pointer* d_root, uint8_t* d_root_type,
                               void* stream);

/* ---- multi-GPU, one process: device-resident shards and their global root (c4) --------
 * storm is one Go process; on an 8-GPU node it reaches every GPU from it.
 * A batch of device-resident blocks is sharded into contiguous ranges, each on its own
 * device. stormck_merkle_root_multi runs each shard's checksums (optional) and its shard
 * tree (stormck_merkle_root_device) on the shard's device, from one host thread per device,
 * gathers the shard roots over xGMI with in-process RCCL (ncclCommInitAll over the distinct
 * devices, one ncclAllGather of their root rows), and hashes the combining pointer block on
 * EVERY device; the devices must agree. The reference has no multi-device code; the tree
 * shape is this library's and the node format storm's (blocks/pointer/block.go:10-13).
 * One shard: */
typedef struct stormck_shard {
    const void* d_blocks;    /* block i at d_blocks + i*stride on `device`, `len` bytes; NULL: the
                              * leaf checksums are already in d_checksums (nothing is hashed) */
    uint64_t stride;
    uint64_t n;              /* leaves of the shard */
    uint64_t* d_checksums;   /* n u64 on `device`: written when d_blocks is set, else read */
    uint64_t leaf_addr_base; /* Address of leaf i is leaf_addr_base + i (Leaf type, rev) */
    uint64_t node_addr_base; /* interior nodes: node_addr_base, +1, ... level by level, bottom-up */
    void* stream;            /* a stream of `device` the shard's work runs on, after what is already
                              * queued there (e.g. the launches that wrote d_checksums); NULL: the
                              * library's own stream, which waits for no other stream. A stream of
                              * another device is STORMCK_EINVAL */
    int32_t device;          /* HIP device index holding the shard */
    uint32_t len;            /* bytes hashed per block (when d_blocks is set) */
} stormck_shard;

/* The build's shard convention (storm_amd/dist.py): n_total leaves in n_shards
 * contiguous ranges whose sizes differ by at most one; shard s holds leaves [lo_s, hi_s),
 * addressed lo_s..hi_s-1, its interior nodes from n_total + lo_s (disjoint from every other
 * shard's and from the leaves for fanout >= 3), and the combining node gets 2 * n_total.
 * Fills n, leaf_addr_base, node_addr_base and device (shards are dealt to devices[0..n_devices)
 * in consecutive runs: shard s on devices[s * n_devices / n_shards]) of shards[0..n_shards) and
 * zeroes the rest; the caller sets d_blocks / stride / len / d_checksums / stream, with shard
 * s's blocks being logical blocks [lo_s, hi_s) (lo_s = leaf_addr_base). *root_addr (optional)
 * = 2 * n_total. Needs no device. */
int stormck_shard_plan(uint64_t n_total, uint32_t n_shards, const int* devices, int n_devices, stormck_shard* shards,
                       uint64_t* root_addr);

/* The global root of shards[0..n_shards) (1 <= n_shards <= fanout): every shard's tree
 * (leaves of type Leaf, birth revision rev), then one pointer block holding the shard roots
 * in shard order, hashed on every device: *root = {its checksum, root_addr, rev}, *root_type =
 * Pointer. shard_roots / shard_types (optional, n_shards each) = the shard roots (a shard of
 * n == 0 has a zero root of type Free, of n == 1 its leaf's own Pointer). Synchronous: returns
 * when every shard's work and the gather have finished; the shards' streams may then be reused.
 * A device may hold several shards (the gather then carries several rows per device; with one
 * device the gather is a one-rank RCCL communicator). RCCL (librccl.so.1, from the ROCm
 * install or already in the process) is loaded at the first call and its communicators are
 * kept per device set; STORMCK_EHIP names an RCCL that cannot be loaded or fails. Calls are
 * serialised process-wide (a communicator serves one collective at a time). */
int stormck_merkle_root_multi(const stormck_shard* shards, uint32_t n_shards, uint64_t rev, uint64_t root_addr,
                              uint32_t fanout, stormck_pointer* root, uint8_t* root_type, stormck_pointer* shard_roots,
                              uint8_t* shard_types);

/* The gather layout stormck_merkle_root_multi uses for shards[0..n_shards), without a device
 * (planning only; device indices are not checked against the visible devices):
 * devices[0..*n_devices) = the shards' distinct devices in order of first appearance (the
 * communicator's ranks), *rows = R, the most shards on one device (each device sends R root
 * rows of 32 bytes; rows it does not fill stay zero), table_row[s] = the row of the gathered
 * D x R table holding shard s's root (device slot * R + the shard's place among that device's
 * shards). devices needs room for 64 entries. */
int stormck_multi_layout(const stormck_shard* shards, uint32_t n_shards, int32_t* devices, uint32_t* n_devices,
                         uint32_t* rows, uint32_t* table_row);

/* ---- f2/f3: batched cold read + verify from a file device -------------------
 * storm's cold fetch reads a block from its Dev and verifies it
 * (cache.fetchBlock: Store.ReadBlock(address, Data[:Sizeof(T)]) then
 * blocks.VerifyChecksum, /root/reference/cache/cache.go:139-167,
 * persistence/store.go:39-51; filedev = *os.File, pkg/filedev/filedev.go). This
 * does it for n blocks at once: block i (lens[i] bytes at file offset
 * addresses[i] * block_size) is read with parallel pread() into
 * dst + i*dst_stride (e.g. the cache slots), then all n are verified on the GPU
 * against expected[i]. With STORMCK_READ_FULL_BLOCK each read covers block_size
 * bytes while lens[i] bytes are still what is hashed. A descriptor opened with
 * O_DIRECT (no page cache) always reads full blocks; dst, dst_stride and block_size
 * must then be 512-byte aligned (the device's own alignment may be stricter).
 * Consecutive addresses whose slots are contiguous (dst_stride == block_size) are
 * read with one pread of up to 1 MiB. With dst registered (stormck_host_register)
 * the verify DMAs straight from the slots, with no staging copy.
 * *first_bad = first mismatching index (n if none), *n_bad = count; returns
 * STORMCK_EMISMATCH if any block fails, STORMCK_EINVAL on a short read. */
#define STORMCK_READ_FULL_BLOCK 1u
int stormck_read_verify_fd(int fd, const uint64_t* addresses, const uint32_t* lens, uint64_t n, uint64_t block_size,
                           void* dst, uint64_t dst_stride, const uint64_t* expected, uint32_t flags,
                           uint64_t* first_bad, uint64_t* n_bad);

/* ---- f4: key tags ----------------------------------------------------------
 * xxhash.Sum64(key) for a batch of short keys (keystore.GetObjectID /
 * EnsureObjectID hash each key to a tree tag: /root/reference/keystore/keystore.go:33,66;
 * keys are 1..256 bytes, objectlist.MaxKeyComponentLength). Key i is at
 * d_keys + (d_offsets ? d_offsets[i] : i*stride), (d_lens ? d_lens[i] : len) bytes;
 * any alignment. One lane per key. Same results as stormck_checksum_device, which
 * remains correct for keys of any length. */
int stormck_key_tags_device(const void* d_keys, uint64_t stride, const uint64_t* d_offsets, const uint32_t* d_lens,
                            uint32_t len, uint64_t n, uint64_t* d_out, void* stream);

/* ---- f1: level-synchronous batched commit ----------------------------------
 * storm's Cache.Commit hashes dirty blocks children-first, one at a time
 * (commitData / commitBlock, /root/reference/cache/cache.go:87-137) and each
 * block's PostCommitFunc stores {Checksum, Address, BirthRevision} and its type
 * into the parent through a BlockOrigin (/root/reference/cache/trace.go:274-320,
 * cache/types.go BlockOrigin). Blocks at the same height are independent, so the
 * library commits a whole dirty forest one LEVEL per launch: hash every block of
 * the level (gather), then scatter its Pointer and type into its origin.
 *
 * One entry per dirty block (blockMetadata + BlockOrigin), offsets relative to the
 * device arena (storm's cache.data): */
#define STORMCK_NO_ORIGIN UINT64_MAX
#define STORMCK_NO_PARENT (-1)
typedef struct stormck_dirty_block {
    uint64_t data_offset;    /* block bytes: d_arena + data_offset (blockMetadata.Data) */
    uint64_t origin_pointer; /* arena offset of the blocks.Pointer the parent keeps for this block
                              * (BlockOrigin.Pointer; 8-byte aligned), or STORMCK_NO_ORIGIN */
    uint64_t origin_type;    /* arena offset of the parent's BlockType byte (BlockOrigin.BlockType) */
    int64_t parent;          /* index of the dirty block that holds the origin, or STORMCK_NO_PARENT
                              * (origin outside the batch, e.g. the singularity) */
    uint64_t address;        /* in/out: blockMetadata.Address */
    uint64_t birth_revision; /* in/out: blockMetadata.BirthRevision */
    uint32_t length;         /* bytes hashed = unsafe.Sizeof(T) */
    uint8_t type;            /* STORMCK_LEAF_BLOCK / STORMCK_POINTER_BLOCK, stored at origin_type */
    uint8_t reserved[3];
} stormck_dirty_block;

/* Commit the dirty forest blocks[0..n) held in d_arena:
 *  - order: children before parents (by height), index order within a height;
 *  - relocation, in that order (cache/cache.go:114-118): if birth_revision <=
 *    revision then address = ++*last_allocated_block, birth_revision = revision + 1;
 *  - per block: cs = XXH64(arena + data_offset, length); if origin_pointer is set,
 *    arena[origin_pointer] = Pointer{cs, address, birth_revision} and
 *    arena[origin_type] = type.
 * Writes out_checksums[i] (host) and updates blocks[i].address / birth_revision.
 * Synchronous on `stream`. Any children-first order is a valid storm commit order
 * (storm's own order follows Go map iteration); this one is deterministic.
 * Argument errors (parent range, origin alignment, cycles) and a missing device are
 * reported before anything is changed. A HIP failure part-way leaves the commit
 * partly applied, as storm's own loop does on a write error; *last_allocated_block
 * then still matches the relocations already written into blocks. */
int stormck_commit_device(void* d_arena, stormck_dirty_block* blocks, uint64_t n, uint64_t revision,
                          uint64_t* last_allocated_block, uint64_t* out_checksums, void* stream);

/* The same commit on host threads (the "host leg"): identical rules, order, relocation,
 * stores, outputs and errors as stormck_commit_device, with `arena` a HOST pointer
 * (storm's cache.data) and the blocks of one height hashed on `threads` library pool
 * threads (0 = all of the pool, at most 16; 1 = storm's serial loop). Needs no device:
 * it is the leg stormck_commit picks for forests too small to repay a launch per height
 * and the link (DESIGN_LOG.md §11 f1). */
int stormck_commit_host(void* arena, stormck_dirty_block* blocks, uint64_t n, uint64_t revision,
                        uint64_t* last_allocated_block, uint64_t* out_checksums, uint32_t threads);
/* Cache.Commit's data phase as storm's cache calls it (the Go binding's CommitBatch):
 * `arena` is cache.data. An HBM arena (stormck_device_alloc) is committed by
 * stormck_commit_device. A host arena registered with stormck_host_register is committed
 * on the leg the library's cost model (routing section below) predicts is fastest: the
 * device leg in place over the link, the host leg on host_threads threads (0 = the pool),
 * or the split (stormck_commit_split: the leaves on both at once). An unregistered host
 * arena is out of the devices' reach and takes the host leg. Before a host or split leg
 * reads a registered arena, a non-NULL `stream` is synchronised (device writes the caller
 * queued on it land first). With `stream` NULL those legs wait for nothing: storm writes
 * cache.data on the host only (the Go binding passes nil), and the query would be most of
 * the routed call's cost on its smallest commits; a caller whose null-stream work writes the
 * arena synchronises it first (the device leg itself launches on the null stream then).
 * *leg_used (optional) = STORMCK_LEG_HOST / _DEVICE / _SPLIT. Needs a gfx950 device
 * like every batched entry point (STORMCK_ENODEV without one). */
#define STORMCK_LEG_NONE 0u
#define STORMCK_LEG_HOST 1u
#define STORMCK_LEG_DEVICE 2u
#define STORMCK_LEG_SPLIT 3u
int stormck_commit(void* arena, stormck_dirty_block* blocks, uint64_t n, uint64_t revision,
                   uint64_t* last_allocated_block, uint64_t* out_checksums, void* stream, uint32_t host_threads,
                   uint32_t* leg_used);

/* ---- routing of host-memory work: the split leg and the measured rates -----------
 * Host-memory work (stormck_checksum_batch / _verify_batch, stormck_commit) runs on one of
 * three legs:
 *   STORMCK_LEG_HOST    the library's host threads alone;
 *   STORMCK_LEG_DEVICE  the device(s) alone, over PCIe;
 *   STORMCK_LEG_SPLIT   both at once on disjoint blocks of the one call: the host threads
 *                       take blocks from the front, each device takes chunks from the back,
 *                       each chunk sized from the rates so that the device finishes when the
 *                       host does, until they meet. The devices DMA (batch) or read in place
 *                       (commit) pinned or registered memory, with no host copy.
 * The choice is the smallest time a cost model predicts. Its rates (bytes per microsecond)
 * and the devices' start latency start at priors measured on an MI355X box and are measured
 * again by the calls themselves: every host, device or split leg large enough to time
 * updates its rate (EWMA). */
typedef struct stormck_route_rates {
    double host_thread;    /* one host thread (four blocks at once where the CPU has AVX-512) */
    double host_memory;    /* the host pool's cap on passes that stream from host memory */
    double host_cached;    /* the same on passes of at most 64 MiB, which can run from the host's
                            * caches (a commit hashes blocks its caller has just written) */
    double link_pinned;    /* one device's pipeline from pinned or registered host memory */
    double link_pageable;  /* one device's pipeline from pageable memory (through pinned staging) */
    double link_inplace;   /* one device's kernels reading registered host memory in place */
    double device_latency; /* microseconds from a split's start until a device's first chunk is
                            * back, beyond that chunk's bytes over the link (wake, launch, sync) */
    uint64_t observations; /* calls that updated the rates since the priors or the last set */
} stormck_route_rates;
int stormck_route_get_rates(stormck_route_rates* rates);
/* Replace the rates (rates == NULL: back to the priors). flags: STORMCK_RATES_FREEZE stops
 * the calls from updating them (tests, A/B); STORMCK_RATES_LEARN lets them. */
#define STORMCK_RATES_LEARN 0u
#define STORMCK_RATES_FREEZE 1u
int stormck_route_set_rates(const stormck_route_rates* rates, uint32_t flags);
/* The devices the routed entry points may use, process-wide (storm is one process; each
 * device brings its own PCIe link). n_devices == 0: the calling thread's current device
 * (the default). Listing a device twice lists it once. */
int stormck_route_devices(const int* devices, int n_devices);
/* The decision alone, from the model: no device and no data needed. memory:
 * STORMCK_MEM_PAGEABLE or STORMCK_MEM_PINNED (page-locked; for a commit, registered);
 * n_devices: devices the call could use (0: host leg only). *leg = the leg the routed call
 * would take (STORMCK_LEG_NONE for n == 0); predicted_us (optional, 3 doubles): host,
 * device and split time, INFINITY where the leg cannot run or the split gains nothing. */
#define STORMCK_MEM_PAGEABLE 0u
#define STORMCK_MEM_PINNED 1u
int stormck_route_plan_batch(uint64_t stride, const uint32_t* lens, uint32_t len, uint64_t n, uint32_t memory,
                             uint32_t host_threads, uint32_t n_devices, uint32_t* leg, double* predicted_us);
int stormck_route_plan_commit(const stormck_dirty_block* blocks, uint64_t n, uint32_t memory, uint32_t host_threads,
                              uint32_t n_devices, uint32_t* leg, double* predicted_us);
/* The split leg alone. base: pinned or registered host memory (pageable is STORMCK_EINVAL:
 * the devices would need host threads to copy it, which hash faster than they copy).
 * devices / n_devices: the devices that take part (NULL / 0: the route devices);
 * host_threads: 0 = the pool. device_blocks: STORMCK_SPLIT_BALANCED to size the devices'
 * chunks from the rates as they run; otherwise exactly the last device_blocks blocks go to
 * the devices and the others to the host threads (tests, A/B). *device_done (optional):
 * blocks the devices hashed. Results and errors as stormck_checksum_host / _verify_host
 * (first_bad is the lowest mismatching index over both sides, n_bad their sum). */
#define STORMCK_SPLIT_BALANCED UINT64_MAX
int stormck_checksum_split(const void* base, uint64_t stride, const uint32_t* lens, uint32_t len, uint64_t n,
                           uint64_t* out, const int* devices, int n_devices, uint32_t host_threads,
                           uint64_t device_blocks, uint64_t* device_done);
int stormck_verify_split(const void* base, uint64_t stride, const uint32_t* lens, uint32_t len, uint64_t n,
                         const uint64_t* expected, uint64_t* first_bad, uint64_t* n_bad, const int* devices,
                         int n_devices, uint32_t host_threads, uint64_t device_blocks, uint64_t* device_done);
/* A commit with its leaves (height 0) split: the same rules, order, relocation, stores,
 * outputs and errors as stormck_commit_host, with `arena` registered host memory; the
 * devices hash leaves from the back of the leaf height in place and the host threads store
 * every Pointer (cache/trace.go:274-320); the upper heights (a few pointer blocks) run on
 * the host threads. device_leaves: STORMCK_SPLIT_BALANCED or the exact number of leaves, the
 * last ones of the commit order, the devices hash; *device_done (optional): leaves they
 * hashed. */
int stormck_commit_split(void* arena, stormck_dirty_block* blocks, uint64_t n, uint64_t revision,
                         uint64_t* last_allocated_block, uint64_t* out_checksums, const int* devices, int n_devices,
                         uint32_t host_threads, uint64_t device_leaves, uint64_t* device_done);

/* ---- synthetic data (benchmarks / tests) -----------------------------------
 * Word w of block i = splitmix64(seed ^ (((first + i) << 20) + w)), w < stride/8,
 * little-endian. stride % 16 == 0, d_dst 16-byte aligned. */
int stormck_fill_synthetic_device(void* d_dst, uint64_t stride, uint64_t n, uint64_t first, uint64_t seed,
                                  void* stream);

#ifdef __cplusplus
}
#endif

#endif /* STORMCK_H */
