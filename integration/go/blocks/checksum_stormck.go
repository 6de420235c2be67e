//go:build stormck

// Package blocks — GPU-backed checksum for storm (drop-in for blocks/checksum.go).
//
// A storm maintainer adds this file to github.com/outofforest/storm/blocks and
// puts `//go:build !stormck` on the existing blocks/checksum.go. `go build
// -tags stormck` then routes every block checksum through libstormck (MI355X,
// gfx950); without the tag storm is unchanged. Signatures of Checksum,
// BlockChecksum and VerifyChecksum are identical to blocks/checksum.go:10-27;
// ChecksumBatch / VerifyChecksumBatch / RegisterHostMemory are additions for
// batched callers (level-synchronous commit, batched cold-read verify).
//
// Not compiled in this repository (no Go toolchain in the build image); the C
// side it binds is exercised by tests/test_abi.py and tests/test_cpp_mirror.py.
package blocks

/*
#cgo CFLAGS: -I${SRCDIR}/../third_party/stormck/include
#cgo LDFLAGS: -L${SRCDIR}/../third_party/stormck/lib -lstormck -Wl,-rpath,${SRCDIR}/../third_party/stormck/lib
#include <stdint.h>
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
// The reference cannot fail; a device failure here is unrecoverable and panics.
func Checksum(b []byte) Hash {
	var out C.uint64_t
	// cgo pointer rules: b holds no Go pointers and libstormck does not retain it
	// after the (synchronous) call returns.
	if rc := C.stormck_checksum(bytesPtr(b), C.uint64_t(len(b)), &out); rc != C.STORMCK_OK {
		panic(stormckError(rc))
	}
	return Hash(out)
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

// ChecksumBatch computes checksums of n blocks at data[i*stride:], length bytes each.
func ChecksumBatch(data []byte, n, stride, length int, out []Hash) error {
	if n == 0 {
		return nil
	}
	if len(out) < n || len(data) < (n-1)*stride+length {
		return errors.New("ChecksumBatch: buffer too small")
	}
	rc := C.stormck_checksum_host(bytesPtr(data), C.uint64_t(stride), nil, C.uint32_t(length), C.uint64_t(n),
		(*C.uint64_t)(unsafe.Pointer(&out[0])))
	if rc != C.STORMCK_OK {
		return stormckError(rc)
	}
	return nil
}

// VerifyChecksumBatch verifies n blocks; it returns the first mismatching index
// (n when all match) and the number of mismatches.
func VerifyChecksumBatch(data []byte, n, stride, length int, expected []Hash) (firstBad, nBad int, err error) {
	if n == 0 {
		return 0, 0, nil
	}
	var fb, nb C.uint64_t
	rc := C.stormck_verify_host(bytesPtr(data), C.uint64_t(stride), nil, C.uint32_t(length), C.uint64_t(n),
		(*C.uint64_t)(unsafe.Pointer(&expected[0])), &fb, &nb)
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
// in cache.New, cache/cache.go:36-40) so batches DMA straight from it. The Go heap
// does not move large allocations; the caller keeps the slice alive until
// UnregisterHostMemory.
func RegisterHostMemory(b []byte) error {
	if rc := C.stormck_host_register(bytesPtr(b), C.uint64_t(len(b))); rc != C.STORMCK_OK {
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
