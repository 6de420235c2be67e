//go:build !stormck

package keystore

import "github.com/cespare/xxhash/v2"

// keyTag is the tree tag of a key: storm's own xxhash.Sum64 (keystore/keystore.go:33,66).
func keyTag(key []byte) uint64 {
	return xxhash.Sum64(key)
}
