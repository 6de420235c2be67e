/*
 * ORACLE — TEST INFRASTRUCTURE ONLY. Never linked into or called by the product
 * (storm_amd/, libstormck.so). Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load the library built from this file.
 *
 * Plain-C restatement of storm's per-block content hash and of the data it is
 * applied to:
 *
 *   blocks.Checksum(b)      = Hash(xxhash.Sum64(b))        /root/reference/blocks/checksum.go:15-17
 *   blocks.BlockChecksum(&T)= Checksum(bytes of *T)        /root/reference/blocks/checksum.go:10-12
 *   blocks.VerifyChecksum   = compare + formatted error     /root/reference/blocks/checksum.go:20-27
 *
 * xxhash.Sum64 lives in the un-vendored third-party module
 * github.com/cespare/xxhash/v2 v2.2.0 (/root/reference/go.mod:6, go.sum:1-2),
 * which is absent from this container. It implements the published XXH64
 * algorithm with seed 0; this file restates that published algorithm
 * (SURVEY.md Appendix A). Parity of this restatement is pinned by
 * tests/test_oracle.py against (1) the public XXH64 known-answer vectors and
 * (2) golden fixtures produced by libxxhash 0.8.2 (python-xxhash 3.8.1) with
 * oracle/gen_golden.py — see DESIGN.md "Oracle and parity pinning".
 *
 * Also restated here (build-defined, reference node format):
 *   - the deterministic synthetic block generator,
 *   - storm pointer-block (Merkle node) packing, pointer.Block layout
 *     /root/reference/blocks/pointer/block.go:10-13, Pointer
 *     /root/reference/blocks/types.go:35-39, and the shard tree of DESIGN.md.
 */
#include <stdint.h>
#include <stddef.h>
#include <string.h>
#include <stdlib.h>
#include <pthread.h>

#define P1 0x9E3779B185EBCA87ULL
#define P2 0xC2B2AE3D27D4EB4FULL
#define P3 0x165667B19E3779F9ULL
#define P4 0x85EBCA77C2B2AE63ULL
#define P5 0x27D4EB2F165667C5ULL

static inline uint64_t rotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }

static inline uint64_t rd64(const uint8_t* p) {
    uint64_t v = 0;
    for (int i = 7; i >= 0; --i) v = (v << 8) | p[i];  /* little-endian, as Go's binary.LittleEndian */
    return v;
}
static inline uint32_t rd32(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

static inline uint64_t xround(uint64_t acc, uint64_t w) {
    acc += w * P2;
    acc = rotl(acc, 31);
    return acc * P1;
}
static inline uint64_t xmerge(uint64_t h, uint64_t v) {
    h ^= xround(0, v);
    return h * P1 + P4;
}

/* XXH64(p, n, seed = 0): the function blocks.Checksum delegates to (checksum.go:16). */
uint64_t oracle_xxh64(const void* data, size_t n) {
    const uint8_t* p = (const uint8_t*)data;
    const uint8_t* end = p + n;
    uint64_t h;
    if (n >= 32) {
        uint64_t v1 = P1 + P2, v2 = P2, v3 = 0, v4 = (uint64_t)0 - P1;
        const uint8_t* lim = end - 32;
        do {
            v1 = xround(v1, rd64(p));
            v2 = xround(v2, rd64(p + 8));
            v3 = xround(v3, rd64(p + 16));
            v4 = xround(v4, rd64(p + 24));
            p += 32;
        } while (p <= lim);
        h = rotl(v1, 1) + rotl(v2, 7) + rotl(v3, 12) + rotl(v4, 18);
        h = xmerge(h, v1);
        h = xmerge(h, v2);
        h = xmerge(h, v3);
        h = xmerge(h, v4);
    } else {
        h = P5;
    }
    h += (uint64_t)n;
    while (p + 8 <= end) {
        h ^= xround(0, rd64(p));
        h = rotl(h, 27) * P1 + P4;
        p += 8;
    }
    if (p + 4 <= end) {
        h ^= (uint64_t)rd32(p) * P1;
        h = rotl(h, 23) * P2 + P3;
        p += 4;
    }
    while (p < end) {
        h ^= (uint64_t)(*p) * P5;
        h = rotl(h, 11) * P1;
        p++;
    }
    h ^= h >> 33;
    h *= P2;
    h ^= h >> 29;
    h *= P3;
    h ^= h >> 32;
    return h;
}

/* Batch over blocks at base + i*stride, length lens ? lens[i] : len. */
void oracle_checksum_batch(const void* base, size_t stride, const uint32_t* lens, uint32_t len,
                           size_t n, uint64_t* out) {
    const uint8_t* b = (const uint8_t*)base;
    for (size_t i = 0; i < n; ++i) out[i] = oracle_xxh64(b + i * stride, lens ? lens[i] : len);
}

/* ---- multi-threaded batch (CPU baseline "all cores" leg) ---- */
typedef struct {
    const uint8_t* base; size_t stride; const uint64_t* offs; const uint32_t* lens; uint32_t len;
    size_t lo, hi; uint64_t* out;
} mt_arg;
static void* mt_body(void* a_) {
    mt_arg* a = (mt_arg*)a_;
    for (size_t i = a->lo; i < a->hi; ++i)
        a->out[i] = oracle_xxh64(a->base + (a->offs ? a->offs[i] : i * a->stride), a->lens ? a->lens[i] : a->len);
    return NULL;
}
static void mt_run(const void* base, size_t stride, const uint64_t* offs, const uint32_t* lens, uint32_t len,
                   size_t n, uint64_t* out, int threads) {
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t th[256];
    mt_arg args[256];
    for (int t = 0; t < threads; ++t) {
        args[t].base = (const uint8_t*)base; args[t].stride = stride; args[t].offs = offs; args[t].lens = lens;
        args[t].len = len; args[t].out = out;
        args[t].lo = n * (size_t)t / (size_t)threads;
        args[t].hi = n * (size_t)(t + 1) / (size_t)threads;
        pthread_create(&th[t], NULL, mt_body, &args[t]);
    }
    for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
}
void oracle_checksum_batch_mt(const void* base, size_t stride, const uint32_t* lens, uint32_t len,
                              size_t n, uint64_t* out, int threads) {
    mt_run(base, stride, NULL, lens, len, n, out, threads);
}
/* Gathered blocks: block i at base + offs[i] (stormck_checksum_gather_device's shape). */
void oracle_checksum_gather_mt(const void* base, const uint64_t* offs, const uint32_t* lens, uint32_t len,
                               size_t n, uint64_t* out, int threads) {
    mt_run(base, 0, offs, lens, len, n, out, threads);
}

/* ---- synthetic blocks ----
 * word w (8 bytes, little-endian) of block i = splitmix64(seed ^ (i * 2^20 + w)),
 * for w in [0, stride/8). */
static inline uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
uint64_t oracle_synth_word(uint64_t seed, uint64_t block, uint64_t word) {
    return splitmix64(seed ^ ((block << 20) + word));
}
/* Fill n blocks of `stride` bytes (multiple of 8) for logical indices first..first+n-1. */
void oracle_fill_synthetic(void* dst, size_t stride, size_t n, uint64_t first, uint64_t seed) {
    uint8_t* d = (uint8_t*)dst;
    size_t words = stride / 8;
    for (size_t i = 0; i < n; ++i) {
        for (size_t w = 0; w < words; ++w) {
            uint64_t v = oracle_synth_word(seed, first + i, w);
            memcpy(d + i * stride + w * 8, &v, 8);  /* host is little-endian (x86-64) */
        }
    }
}

/* ---- storm pointer block (Merkle node) ----
 * pointer.Block{Pointers [F]blocks.Pointer; PointedBlockTypes [F]blocks.BlockType}
 * (blocks/pointer/block.go:10-13): F*24 bytes of {Checksum, Address, BirthRevision}
 * u64 LE, then F type bytes; Sizeof = 25*F (30000 for F=1200, 250 for the test tag
 * F=10... Go pads the struct to 8-byte alignment: 25*F rounded up to a multiple of 8,
 * i.e. 30000 for F=1200 and 256 for F=10, matching SURVEY.md §2). Unused slots are 0. */
size_t oracle_pointer_block_size(uint32_t fanout) {
    size_t raw = (size_t)fanout * 25;
    return (raw + 7) & ~(size_t)7;
}
void oracle_pack_pointer_block(uint8_t* dst, uint32_t fanout, const uint64_t* cs,
                               const uint64_t* addr, const uint64_t* rev, const uint8_t* types,
                               uint32_t m) {
    size_t sz = oracle_pointer_block_size(fanout);
    memset(dst, 0, sz);
    for (uint32_t k = 0; k < m; ++k) {
        memcpy(dst + 24 * (size_t)k, &cs[k], 8);
        memcpy(dst + 24 * (size_t)k + 8, &addr[k], 8);
        memcpy(dst + 24 * (size_t)k + 16, &rev[k], 8);
        dst[24 * (size_t)fanout + k] = types[k];
    }
}

/* Shard Merkle tree (DESIGN.md "Shard Merkle tree"):
 *   level 0: entries {cs[i], leaf_addr_base + i, rev}, type Leaf (2)
 *   level L+1: consecutive groups of `fanout` level-L entries packed into one pointer
 *     block; its entry is {xxh64(node bytes), node address, rev}, type Pointer (1).
 *     Node addresses are allocated sequentially from node_addr_base, level by level,
 *     bottom-up (storm allocates ++LastAllocatedBlock in commit order, children first:
 *     /root/reference/cache/cache.go:114-118).
 *   The single entry of the first level with one entry is the root.
 *   n == 0 -> root = {0,0,0}, type Free (0).
 * Returns the number of interior nodes allocated. */
size_t oracle_merkle_root(const uint64_t* leaf_cs, size_t n, uint64_t leaf_addr_base,
                          uint64_t node_addr_base, uint64_t rev, uint32_t fanout,
                          uint64_t root[3], uint8_t* root_type) {
    if (n == 0) {
        root[0] = root[1] = root[2] = 0;
        *root_type = 0;
        return 0;
    }
    size_t m = n;
    uint64_t* cs = (uint64_t*)malloc(m * 8);
    uint64_t* ad = (uint64_t*)malloc(m * 8);
    memcpy(cs, leaf_cs, m * 8);
    for (size_t i = 0; i < m; ++i) ad[i] = leaf_addr_base + i;
    uint8_t type = 2;
    uint64_t next_addr = node_addr_base;
    size_t nodes = 0;
    size_t bsz = oracle_pointer_block_size(fanout);
    uint8_t* blk = (uint8_t*)malloc(bsz);
    uint64_t* revs = (uint64_t*)malloc((size_t)fanout * 8);
    uint8_t* types = (uint8_t*)malloc(fanout);
    for (uint32_t k = 0; k < fanout; ++k) revs[k] = rev;
    while (m > 1) {
        size_t pm = (m + fanout - 1) / fanout;
        memset(types, type, fanout);
        for (size_t j = 0; j < pm; ++j) {
            size_t lo = j * fanout;
            uint32_t cnt = (uint32_t)((m - lo) < fanout ? (m - lo) : fanout);
            oracle_pack_pointer_block(blk, fanout, cs + lo, ad + lo, revs, types, cnt);
            cs[j] = oracle_xxh64(blk, bsz);
            ad[j] = next_addr + j;
        }
        next_addr += pm;
        nodes += pm;
        m = pm;
        type = 1;
    }
    root[0] = cs[0];
    root[1] = ad[0];
    root[2] = rev;
    *root_type = type;
    free(cs); free(ad); free(blk); free(revs); free(types);
    return nodes;
}

/* ---- storm commit (f1 checker) ----
 * Serial restatement of Cache.Commit's data phase (/root/reference/cache/cache.go:87-137)
 * with the post-commit pointer write of newPointerBlockPostCommitFunc /
 * newLeafBlockPostCommitFunc (/root/reference/cache/trace.go:274-320):
 *   repeat: for meta in dirty (iteration order below): if it still has uncommitted
 *   dirty children (NReferences > 0) skip; else commitBlock: relocate if
 *   BirthRevision <= Revision (LastAllocatedBlock++), hash the block, store
 *   {Checksum, Address, BirthRevision} + type at its BlockOrigin, release the parent.
 * storm iterates a Go map (unspecified order); the checker iterates by (height,
 * index), the order libstormck documents, so addresses are comparable. Heights are
 * computed here by fixpoint relaxation (independent of the library's walk-up). */
typedef struct {
    uint64_t data_offset, origin_pointer, origin_type;
    int64_t parent;
    uint64_t address, birth_revision;
    uint32_t length;
    uint8_t type, reserved[3];
} oracle_dirty_block;

static _Thread_local const oracle_dirty_block* g_sort_blocks;  /* per thread: callers may run concurrently */
static _Thread_local const uint32_t* g_sort_height;
static int cmp_order(const void* a, const void* b) {
    size_t x = *(const size_t*)a, y = *(const size_t*)b;
    if (g_sort_height[x] != g_sort_height[y]) return g_sort_height[x] < g_sort_height[y] ? -1 : 1;
    return x < y ? -1 : (x > y);
}

int oracle_commit(uint8_t* arena, oracle_dirty_block* blocks, size_t n, uint64_t revision,
                  uint64_t* last_allocated, uint64_t* out_cs) {
    uint32_t* height = (uint32_t*)calloc(n ? n : 1, sizeof(uint32_t));
    uint64_t* pending = (uint64_t*)calloc(n ? n : 1, sizeof(uint64_t));
    uint8_t* done = (uint8_t*)calloc(n ? n : 1, 1);
    size_t* order = (size_t*)malloc((n ? n : 1) * sizeof(size_t));
    for (int changed = 1, rounds = 0; changed; ++rounds) {
        if (rounds > (int)n + 1) { free(height); free(pending); free(done); free(order); return -1; }
        changed = 0;
        for (size_t i = 0; i < n; ++i) {
            int64_t p = blocks[i].parent;
            if (p >= 0 && height[p] < height[i] + 1) { height[p] = height[i] + 1; changed = 1; }
        }
    }
    for (size_t i = 0; i < n; ++i) {
        order[i] = i;
        if (blocks[i].parent >= 0) pending[blocks[i].parent]++;
    }
    g_sort_blocks = blocks;
    g_sort_height = height;
    qsort(order, n, sizeof(size_t), cmp_order);
    size_t remaining = n;
    while (remaining > 0) {
        size_t progressed = 0;
        for (size_t k = 0; k < n; ++k) {
            size_t i = order[k];
            if (done[i] || pending[i] > 0) continue;
            oracle_dirty_block* b = &blocks[i];
            if (b->birth_revision <= revision) {          /* cache.go:114-118 */
                *last_allocated += 1;
                b->address = *last_allocated;
                b->birth_revision = revision + 1;
            }
            uint64_t cs = oracle_xxh64(arena + b->data_offset, b->length);  /* BlockChecksum */
            out_cs[i] = cs;
            if (b->origin_pointer != UINT64_MAX) {       /* *origin.Pointer = ...; *origin.BlockType = ... */
                memcpy(arena + b->origin_pointer, &cs, 8);
                memcpy(arena + b->origin_pointer + 8, &b->address, 8);
                memcpy(arena + b->origin_pointer + 16, &b->birth_revision, 8);
                arena[b->origin_type] = b->type;
            }
            if (b->parent >= 0) pending[b->parent]--;    /* parent.NReferences -= NCommits */
            done[i] = 1;
            remaining--;
            progressed++;
        }
        if (!progressed) { free(height); free(pending); free(done); free(order); return -1; }
    }
    free(height); free(pending); free(done); free(order);
    return 0;
}
