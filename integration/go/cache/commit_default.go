//go:build !stormck

package cache

// Without the stormck tag Commit runs storm's own sequential commitData
// (cache/cache.go:87-111) and cache.data is an ordinary Go slice.

func (c *Cache) commitDirty() error {
	return c.commitData()
}

func newArena(n uint64) ([]byte, error) {
	return make([]byte, n), nil
}
