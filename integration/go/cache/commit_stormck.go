//go:build stormck

package cache

// Cache.Commit's data phase through libstormck. storm commits dirty blocks one at a time,
// children first (cache/cache.go:87-137): each commitBlock relocates, writes the block,
// and runs its PostCommitFunc, which hashes it (blocks.BlockChecksum) and stores
// {Checksum, Address, BirthRevision} and the type into the parent through the
// BlockOrigin (cache/trace.go:261-308). Blocks at the same height are independent, so
// commitDirty hands the whole dirty forest to blocks.CommitBatch (libstormck's routed
// stormck_commit), which commits it height by height on the leg its measured cost model
// picks: the GPU (one launch per height, reading cache.data in place over PCIe: it is
// registered host memory, newArena) or the library's host leg (storm's own loop, each
// height spread over host threads). For storm's per-revision commits the host leg wins
// on the measured box (DESIGN_LOG.md §11 f1, "End to end from host memory"), so the stormck
// build is never slower than storm's loop. The host then finishes what storm's loop
// leaves behind. The same steps, in the same order, are mirrored in Python by
// storm_amd/commit.py commit_cache and checked there against a restatement of storm's
// own loop (tests/test_cache_commit.py).
//
// Differences from storm's loop, none visible in the committed state:
//   - order: storm follows Go map iteration; this commits by height, then record order
//     (any children-first order is a storm order);
//   - a dirty block that stays referenced (NReferences > 0 once its dirty children are
//     counted) makes storm's loop spin forever (cache.go:88-90); here Commit fails
//     before anything changes;
//   - WriteBlock of every block comes after all hashing, then the relocation swaps
//     (storm interleaves them per block; the written bytes are the same, since a
//     block's bytes are final once its children have stored their pointers).

import (
	"sort"
	"unsafe"

	"github.com/pkg/errors"

	"github.com/outofforest/storm/blocks"
)

// newArena: cache.data outside the Go heap, registered for in-place device access
// (the HIP runtime keeps a reference to it, which the cgo rules forbid for Go memory).
func newArena(n uint64) ([]byte, error) {
	return blocks.NewHostArena(int(n))
}

// offsetIn returns p's byte offset in cache.data, or false when p lies outside it (the
// singularity block, cache.go:30).
func (c *Cache) offsetIn(p unsafe.Pointer) (uint64, bool) {
	if len(c.data) == 0 {
		return 0, false
	}
	base := uintptr(unsafe.Pointer(&c.data[0]))
	x := uintptr(p)
	if x < base || x >= base+uintptr(len(c.data)) {
		return 0, false
	}
	return uint64(x - base), true
}

// collectDirty lists the dirty forest as records: the dirty set, then every ancestor
// reached through a recorded parent (storm adds those to the dirty set only when a
// child's PostCommitFunc runs, trace.go:278-281,302-305). external lists the records
// whose origin is outside cache.data (the root's SpacePointer in the singularity).
func (c *Cache) collectDirty() (metas []*blockMetadata, dirty []blocks.DirtyBlock, external []int, err error) {
	index := make(map[*blockMetadata]int, len(c.dirtyBlocks))
	for meta := range c.dirtyBlocks {
		index[meta] = len(metas)
		metas = append(metas, meta)
	}
	for k := 0; k < len(metas); k++ {
		m := metas[k]
		if m.PostCommitFunc == nil || m.commit.parent == nil {
			continue
		}
		if _, ok := index[m.commit.parent]; !ok {
			index[m.commit.parent] = len(metas)
			metas = append(metas, m.commit.parent)
		}
	}
	dirty = make([]blocks.DirtyBlock, len(metas))
	for i, m := range metas {
		d := &dirty[i]
		off, ok := c.offsetIn(unsafe.Pointer(&m.Data[0]))
		if !ok {
			return nil, nil, nil, errors.Errorf("block %d: data outside cache.data", m.Address)
		}
		d.DataOffset = off
		d.Address = m.Address
		d.BirthRevision = m.BirthRevision
		d.OriginPointer = blocks.NoOrigin
		d.OriginType = blocks.NoOrigin
		d.Parent = blocks.NoParent
		if m.PostCommitFunc == nil { // committed and written, nothing stored anywhere
			continue
		}
		d.Length = m.commit.size
		d.Type = m.commit.typ
		po, okP := c.offsetIn(unsafe.Pointer(m.commit.origin.Pointer))
		to, okT := c.offsetIn(unsafe.Pointer(m.commit.origin.BlockType))
		switch {
		case okP && okT:
			d.OriginPointer, d.OriginType = po, to
		case !okP && !okT:
			external = append(external, i)
		default:
			return nil, nil, nil, errors.Errorf("block %d: origin straddles cache.data", m.Address)
		}
		if m.commit.parent != nil {
			d.Parent = int64(index[m.commit.parent])
		}
	}
	return metas, dirty, external, nil
}

// commitHeights: each record's height above the blocks with no dirty child, the level
// stormck_commit_device commits it in.
func commitHeights(dirty []blocks.DirtyBlock) ([]int, error) {
	h := make([]int, len(dirty))
	for i := range dirty {
		cur, d := i, 0
		for dirty[cur].Parent != blocks.NoParent {
			cur = int(dirty[cur].Parent)
			d++
			if d > len(dirty) {
				return nil, errors.New("commit: parent links form a cycle")
			}
			if h[cur] >= d {
				break
			}
			h[cur] = d
		}
	}
	return h, nil
}

// commitOrder: by height, then record order (stormck_commit_device's order).
func commitOrder(h []int) []int {
	order := make([]int, len(h))
	for i := range order {
		order[i] = i
	}
	sort.SliceStable(order, func(a, b int) bool { return h[order[a]] < h[order[b]] })
	return order
}

// checkReferences replays storm's reference accounting children first: a child's
// PostCommitFunc lowers its parent's NReferences by the child's NCommits and adds them
// to the parent's NCommits (trace.go:278-281), and a block commits only at
// NReferences == 0 (cache.go:88-90).
func checkReferences(metas []*blockMetadata, dirty []blocks.DirtyBlock, order []int) error {
	refs := make([]uint64, len(metas))
	commits := make([]uint64, len(metas))
	for i, m := range metas {
		refs[i], commits[i] = m.NReferences, m.NCommits
	}
	for _, i := range order {
		if refs[i] != 0 {
			return errors.Errorf("commit: dirty block %d is still referenced (%d)", metas[i].Address, refs[i])
		}
		if p := dirty[i].Parent; p != blocks.NoParent {
			refs[p] -= commits[i]
			commits[p] += commits[i]
		}
	}
	return nil
}

func (c *Cache) commitDirty() error {
	if len(c.dirtyBlocks) == 0 {
		return nil
	}
	metas, dirty, external, err := c.collectDirty()
	if err != nil {
		return err
	}
	h, err := commitHeights(dirty)
	if err != nil {
		return err
	}
	order := commitOrder(h)
	if err := checkReferences(metas, dirty, order); err != nil {
		return err
	}
	before := make([]blocks.BlockAddress, len(dirty))
	for i := range dirty {
		before[i] = dirty[i].Address
	}
	out := make([]blocks.Hash, len(dirty))
	sb := c.singularityBlock.V
	last := sb.LastAllocatedBlock
	_, err = blocks.CommitBatch(c.data, dirty, sb.Revision, &last, out)
	// relocations the library applied (commitBlock, cache.go:114-118), also on a failure
	sb.LastAllocatedBlock = last
	for i, m := range metas {
		m.Address, m.BirthRevision = dirty[i].Address, dirty[i].BirthRevision
	}
	if err != nil {
		return err
	}
	// the PostCommitFunc stores whose origin is not in cache.data
	for _, i := range external {
		o := metas[i].commit.origin
		*o.Pointer = blocks.Pointer{Checksum: out[i], Address: dirty[i].Address, BirthRevision: dirty[i].BirthRevision}
		*o.BlockType = dirty[i].Type
	}
	// commitBlock's write and bookkeeping (cache.go:119-136); the accounting above
	// leaves every NReferences and NCommits of the forest at zero
	for _, i := range order {
		m := metas[i]
		if err := c.store.WriteBlock(m.Address, m.Data); err != nil {
			return err
		}
		delete(c.dirtyBlocks, m)
		m.PostCommitFunc = nil
		m.NCommits = 0
		m.NReferences = 0
	}
	// a relocated block moves into the slot of its new address (cache.go:97-107)
	for _, i := range order {
		m := metas[i]
		if m.Address == before[i] {
			continue
		}
		m.State = invalidBlockState
		m2, err := c.findCachedBlock(m.Address, m.BirthRevision)
		if err != nil {
			return err
		}
		m2.State = usedBlockState
		m2.Data, m.Data = m.Data, m2.Data
	}
	return nil
}
