// Package cache — what the stormck commit needs from storm's cache, in every build.
//
// A storm maintainer adds this file to github.com/outofforest/storm/cache and applies
// trace_types.patch (beside this file). The patch adds one field to blockMetadata and
// one call in each PostCommitFunc constructor, so the values the closure captures are
// also kept as data; routes Commit through commitDirty; and takes cache.data from
// newArena. Without the stormck tag, commitDirty is storm's own commitData and newArena
// is make([]byte, n) (commit_default.go): storm is unchanged.
package cache

import (
	"github.com/outofforest/storm/blocks"
)

// commitRecord is what a PostCommitFunc closure captured (cache/trace.go:261-308): the
// origin it stores the block's Pointer and type into, the parent whose NReferences it
// lowers, the bytes BlockChecksum hashes (unsafe.Sizeof of the block type) and the type
// it stores. Valid while PostCommitFunc is non-nil; each constructor sets both together.
type commitRecord struct {
	origin BlockOrigin
	parent *blockMetadata
	size   uint32
	typ    blocks.BlockType
}

func (m *blockMetadata) recordCommit(origin BlockOrigin, parent *blockMetadata, size uintptr,
	typ blocks.BlockType) {
	m.commit = commitRecord{origin: origin, parent: parent, size: uint32(size), typ: typ}
}
