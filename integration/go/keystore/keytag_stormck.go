//go:build stormck

// Package keystore: tree tags through libstormck (f4).
//
// keystore.GetObjectID and EnsureObjectID hash each key to its tree tag with
// xxhash.Sum64(key) (keystore/keystore.go:33,66). A storm maintainer adds this file
// and keytag_default.go to github.com/outofforest/storm/keystore and changes those
// two calls to keyTag(key). Without the stormck tag, keyTag is xxhash.Sum64 and
// storm is unchanged.
//
// One tag is a hash of at most objectlist.MaxKeyComponentLength (256) bytes. It takes
// the library's host leg, stormck_xxh64, on the calling thread: a few nanoseconds,
// and like Sum64 it cannot fail. KeyTagsDevice is the batch addition for keys that
// are resident in HBM (bench.py --workload keytags: 64M x 48 B keys at about 105 G
// keys/s on one MI355X).
//
// Not compiled in this repository (no Go toolchain in the build image). The C side it
// binds is exercised by tests/test_abi.py and tests/test_gpu_parity.py.
package keystore

/*
#cgo CFLAGS: -I${SRCDIR}/../third_party/stormck/include
#cgo LDFLAGS: -L${SRCDIR}/../third_party/stormck/lib -lstormck -Wl,-rpath,${SRCDIR}/../third_party/stormck/lib
#include <stdint.h>
#include "stormck.h"
*/
import "C"

import (
	"unsafe"

	"github.com/pkg/errors"
)

// keyTag is xxhash.Sum64(key), bit-exact.
func keyTag(key []byte) uint64 {
	if len(key) == 0 {
		return uint64(C.stormck_xxh64(nil, 0))
	}
	return uint64(C.stormck_xxh64(unsafe.Pointer(&key[0]), C.uint64_t(len(key))))
}

// KeyTagsDevice writes xxhash.Sum64 of n keys in device memory to dOut[i]. Key i is
// at dKeys + i*stride and holds length bytes. The call is asynchronous on stream (a
// hipStream_t, nil for the default stream); the pointers are HIP device allocations,
// not Go memory.
func KeyTagsDevice(dKeys unsafe.Pointer, stride uint64, length uint32, n uint64, dOut unsafe.Pointer,
	stream unsafe.Pointer) error {
	if rc := C.stormck_key_tags_device(dKeys, C.uint64_t(stride), nil, nil, C.uint32_t(length), C.uint64_t(n),
		(*C.uint64_t)(dOut), stream); rc != 0 {
		return errors.Errorf("stormck error %d: %s", int(rc), C.GoString(C.stormck_last_error()))
	}
	return nil
}
