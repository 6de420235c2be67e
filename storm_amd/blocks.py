"""Host mirror of storm's Go package ``blocks`` over libstormck.

Same names, argument meaning and error behaviour as the reference:

=====================  ===========================================================
``Checksum(b)``        ``func Checksum(b []byte) Hash``  blocks/checksum.go:15-17
``BlockChecksum(b)``   ``func BlockChecksum[T Block](b *T) Hash``  checksum.go:10-12
``VerifyChecksum``     ``func VerifyChecksum(address, p, expected) error``  :20-27
``Pointer``            ``type Pointer struct{...}``  blocks/types.go:35-39
``BlockType``          Free / Pointer / Leaf  blocks/types.go:7-15
``BLOCK_SIZE``         ``const BlockSize = 32 * 1024``  blocks/types.go:4
=====================  ===========================================================

plus the batch entry points the GPU path exists for (``ChecksumBatch``,
``VerifyChecksumBatch``, ``ReadVerifyBatch``; f1's batched commit is in
``storm_amd.commit``). Batches fail loudly without a device. A batch in host memory
is routed by the library's measured cost model, as the commit is: the gfx950 kernels
over PCIe (``ChecksumBatchGPU``), host threads (``ChecksumBatchHost``), or both at once on
pinned or registered memory (``ChecksumBatchSplit``), whichever it predicts is fastest
(DESIGN.md §4.2). A single ``Checksum`` is one buffer, four serial XXH64
chains: libstormck hashes it on the calling host thread (stormck_checksum, the
latency leg SURVEY.md §8b specifies; measured faster than the device single call at
every length, DESIGN_LOG.md §5). ``ChecksumGPU`` is the same call through the device
(k_xxh64_single), for tests and A/B.
"""
from __future__ import annotations

import ctypes
import os
from enum import IntEnum
from typing import Optional, Sequence, Tuple

import numpy as np

from . import _lib
from ._lib import PointerStruct as Pointer  # noqa: F401  (re-export: blocks.Pointer)

BLOCK_SIZE = 32 * 1024

Hash = int
BlockAddress = int


class BlockType(IntEnum):
    """blocks.BlockType (/root/reference/blocks/types.go:7-15)."""

    FREE = 0
    POINTER = 1
    LEAF = 2


FreeBlockType = BlockType.FREE
PointerBlockType = BlockType.POINTER
LeafBlockType = BlockType.LEAF


class ChecksumMismatchError(Exception):
    """The error VerifyChecksum returns (reference: pkg/errors.Errorf, checksum.go:25-26)."""

    def __init__(self, address: int, computed: int, expected: int):
        super().__init__(
            f"checksum mismatch for block {address}, computed: {_go_hex(computed)}, expected: {_go_hex(expected)}")
        self.address = address
        self.computed = computed
        self.expected = expected


def _go_hex(v: int) -> str:
    # Go's %#v of an unsigned integer type: 0x-prefixed lowercase hex, no padding.
    return "0x%x" % v


def _as_u8(b) -> np.ndarray:
    """Zero-copy uint8 view of any buffer-protocol object (bytes, bytearray,
    memoryview, numpy array, ctypes structure)."""
    if isinstance(b, np.ndarray):
        return np.ascontiguousarray(b).view(np.uint8).reshape(-1)
    return np.frombuffer(b, dtype=np.uint8)


def Checksum(b) -> Hash:
    """XXH64 (seed 0) of the bytes of ``b`` (stormck_checksum: the single-call leg)."""
    a = _as_u8(b)
    out = ctypes.c_uint64(0)
    _lib.check(_lib.lib.stormck_checksum(a.ctypes.data if a.size else None, a.size, ctypes.byref(out)))
    return out.value


def ChecksumGPU(b) -> Hash:
    """The same hash through the device (stormck_checksum_gpu): k_xxh64_single for up
    to 64 KiB, a batch of one through the host pipeline up to 256 MiB."""
    a = _as_u8(b)
    out = ctypes.c_uint64(0)
    _lib.check(_lib.lib.stormck_checksum_gpu(a.ctypes.data if a.size else None, a.size, ctypes.byref(out)))
    return out.value


def BlockChecksum(block) -> Hash:
    """Checksum of the full in-memory image of a block struct (``ctypes.sizeof``
    bytes, padding included — what photon.NewFromValue(b).B exposes)."""
    return Checksum(memoryview(block).cast("B"))


def VerifyChecksum(address: BlockAddress, p, expected_checksum: Hash) -> Optional[ChecksumMismatchError]:
    """Returns None when Checksum(p) == expected, else the mismatch error (Go returns
    an error value; callers raise it when they need to)."""
    checksum = Checksum(p)
    if checksum == expected_checksum:
        return None
    return ChecksumMismatchError(address, checksum, expected_checksum)


def _lens_arg(n: int, length: Optional[int], lens: Optional[Sequence[int]]):
    if lens is not None:
        la = np.ascontiguousarray(np.asarray(lens, dtype=np.uint32))
        if la.size != n:
            raise ValueError("lens must have one entry per block")
        return la, 0
    if length is None:
        raise ValueError("length or lens required")
    return None, int(length)


def _devices_arg(devices: Optional[Sequence[int]]):
    if devices is None:
        return None
    d = (ctypes.c_int * len(devices))(*[int(x) for x in devices])
    return d


def _batch_args(buf, n: int, stride: int, length, lens):
    a = _as_u8(buf)
    la, ln = _lens_arg(n, length, lens)
    if n and a.size < (n - 1) * stride + (int(la.max()) if la is not None else ln):
        raise ValueError("buffer too small for n blocks")
    return a, la, ln, (la.ctypes.data if la is not None else None)


def _expected_arg(n: int, expected) -> np.ndarray:
    exp = np.ascontiguousarray(np.asarray(expected, dtype=np.uint64))
    if exp.size != n:
        raise ValueError("expected must have one entry per block")
    return exp


def ChecksumBatchLeg(buf, n: int, stride: int, length: Optional[int] = None,
                     lens: Optional[Sequence[int]] = None, host_threads: int = 0) -> Tuple[np.ndarray, int]:
    """ChecksumBatch, also returning the leg the library took (_lib.LEG_HOST /
    LEG_DEVICE / LEG_SPLIT; LEG_NONE for an empty batch)."""
    a, la, ln, lp = _batch_args(buf, n, stride, length, lens)
    out = np.zeros(n, dtype=np.uint64)
    leg = ctypes.c_uint32(_lib.LEG_NONE)
    if n == 0:
        return out, leg.value
    _lib.check(_lib.lib.stormck_checksum_batch(a.ctypes.data, stride, lp, ln, n, out.ctypes.data, host_threads,
                                               ctypes.byref(leg)))
    return out, leg.value


def ChecksumBatch(buf, n: int, stride: int, length: Optional[int] = None,
                  lens: Optional[Sequence[int]] = None, devices: Optional[Sequence[int]] = None,
                  host_threads: int = 0) -> np.ndarray:
    """Checksums of ``n`` host blocks at ``buf + i*stride`` (``length`` bytes each or
    ``lens[i]``). Returns uint64[n]. The library routes the batch (stormck_checksum_batch):
    the device leg over PCIe (ChecksumBatchGPU), the host leg on ``host_threads`` threads
    (ChecksumBatchHost; 0 = the library pool) or, for pinned or registered memory, both at
    once (ChecksumBatchSplit), whichever its measured cost model predicts is fastest. ``devices``: hash on these devices in contiguous ranges, one host
    thread each (stormck_checksum_host_multi) instead of routing."""
    if devices is not None:
        return ChecksumBatchGPU(buf, n, stride, length, lens, devices)
    return ChecksumBatchLeg(buf, n, stride, length, lens, host_threads)[0]


def ChecksumBatchGPU(buf, n: int, stride: int, length: Optional[int] = None,
                     lens: Optional[Sequence[int]] = None, devices: Optional[Sequence[int]] = None) -> np.ndarray:
    """The device leg of ChecksumBatch: H2D -> gfx950 kernel -> D2H, pipelined
    (stormck_checksum_host); ``devices``: spread over these devices
    (stormck_checksum_host_multi); default: the current device."""
    a, la, ln, lp = _batch_args(buf, n, stride, length, lens)
    out = np.zeros(n, dtype=np.uint64)
    if n == 0:
        return out
    d = _devices_arg(devices)
    if d is None:
        _lib.check(_lib.lib.stormck_checksum_host(a.ctypes.data, stride, lp, ln, n, out.ctypes.data))
    else:
        _lib.check(_lib.lib.stormck_checksum_host_multi(a.ctypes.data, stride, lp, ln, n, out.ctypes.data, d, len(d)))
    return out


def ChecksumBatchHost(buf, n: int, stride: int, length: Optional[int] = None,
                      lens: Optional[Sequence[int]] = None, threads: int = 0) -> np.ndarray:
    """The host leg of ChecksumBatch (stormck_checksum_host_leg): the blocks hashed on
    ``threads`` library pool threads (0 = the pool), four at a time with AVX-512; needs
    no device."""
    a, la, ln, lp = _batch_args(buf, n, stride, length, lens)
    out = np.zeros(n, dtype=np.uint64)
    if n:
        _lib.check(_lib.lib.stormck_checksum_host_leg(a.ctypes.data, stride, lp, ln, n, out.ctypes.data, threads))
    return out


def _verify_rc(rc: int, fb, nb) -> Tuple[int, int]:
    if rc != _lib.EMISMATCH:
        _lib.check(rc)
    return fb.value, nb.value


def VerifyChecksumBatchLeg(buf, n: int, stride: int, expected: Sequence[int], length: Optional[int] = None,
                           lens: Optional[Sequence[int]] = None, host_threads: int = 0) -> Tuple[int, int, int]:
    """VerifyChecksumBatch, also returning the leg taken: (first_bad, n_bad, leg)."""
    a, la, ln, lp = _batch_args(buf, n, stride, length, lens)
    exp = _expected_arg(n, expected)
    if n == 0:
        return 0, 0, _lib.LEG_NONE
    fb, nb, leg = ctypes.c_uint64(0), ctypes.c_uint64(0), ctypes.c_uint32(_lib.LEG_NONE)
    rc = _lib.lib.stormck_verify_batch(a.ctypes.data, stride, lp, ln, n, exp.ctypes.data, ctypes.byref(fb),
                                       ctypes.byref(nb), host_threads, ctypes.byref(leg))
    return _verify_rc(rc, fb, nb) + (leg.value,)


def VerifyChecksumBatch(buf, n: int, stride: int, expected: Sequence[int], length: Optional[int] = None,
                        lens: Optional[Sequence[int]] = None,
                        devices: Optional[Sequence[int]] = None, host_threads: int = 0) -> Tuple[int, int]:
    """Batched VerifyChecksum. Returns (first_bad, n_bad); first_bad == n when all match.
    Routed as ChecksumBatch (stormck_verify_batch); ``devices`` as in ChecksumBatch."""
    if devices is not None:
        return VerifyChecksumBatchGPU(buf, n, stride, expected, length, lens, devices)
    return VerifyChecksumBatchLeg(buf, n, stride, expected, length, lens, host_threads)[:2]


def VerifyChecksumBatchGPU(buf, n: int, stride: int, expected: Sequence[int], length: Optional[int] = None,
                           lens: Optional[Sequence[int]] = None,
                           devices: Optional[Sequence[int]] = None) -> Tuple[int, int]:
    """The device leg of VerifyChecksumBatch (stormck_verify_host / _host_multi)."""
    a, la, ln, lp = _batch_args(buf, n, stride, length, lens)
    exp = _expected_arg(n, expected)
    if n == 0:
        return 0, 0
    fb, nb = ctypes.c_uint64(0), ctypes.c_uint64(0)
    d = _devices_arg(devices)
    if d is None:
        rc = _lib.lib.stormck_verify_host(a.ctypes.data, stride, lp, ln, n, exp.ctypes.data, ctypes.byref(fb),
                                          ctypes.byref(nb))
    else:
        rc = _lib.lib.stormck_verify_host_multi(a.ctypes.data, stride, lp, ln, n, exp.ctypes.data, ctypes.byref(fb),
                                                ctypes.byref(nb), d, len(d))
    return _verify_rc(rc, fb, nb)


def VerifyChecksumBatchHost(buf, n: int, stride: int, expected: Sequence[int], length: Optional[int] = None,
                            lens: Optional[Sequence[int]] = None, threads: int = 0) -> Tuple[int, int]:
    """The host leg of VerifyChecksumBatch (stormck_verify_host_leg); needs no device."""
    a, la, ln, lp = _batch_args(buf, n, stride, length, lens)
    exp = _expected_arg(n, expected)
    if n == 0:
        return 0, 0
    fb, nb = ctypes.c_uint64(0), ctypes.c_uint64(0)
    rc = _lib.lib.stormck_verify_host_leg(a.ctypes.data, stride, lp, ln, n, exp.ctypes.data, ctypes.byref(fb),
                                          ctypes.byref(nb), threads)
    return _verify_rc(rc, fb, nb)


def ChecksumBatchSplit(buf, n: int, stride: int, length: Optional[int] = None,
                       lens: Optional[Sequence[int]] = None, devices: Optional[Sequence[int]] = None,
                       host_threads: int = 0, device_blocks: Optional[int] = None) -> Tuple[np.ndarray, int]:
    """The split leg of ChecksumBatch (stormck_checksum_split): host threads hash from the
    front, the devices (``devices``, default the route devices) from the back, at once.
    ``buf`` must be pinned or registered (RegisterHostMemory). ``device_blocks``: None =
    balanced by the library's rates; else exactly the last ``device_blocks`` blocks go to
    the devices. Returns (checksums, blocks the devices hashed)."""
    a, la, ln, lp = _batch_args(buf, n, stride, length, lens)
    out = np.zeros(n, dtype=np.uint64)
    if n == 0:
        return out, 0
    d = _devices_arg(devices)
    done = ctypes.c_uint64(0)
    _lib.check(_lib.lib.stormck_checksum_split(a.ctypes.data, stride, lp, ln, n, out.ctypes.data, d,
                                               len(d) if d is not None else 0, host_threads,
                                               _lib.SPLIT_BALANCED if device_blocks is None else device_blocks,
                                               ctypes.byref(done)))
    return out, done.value


def VerifyChecksumBatchSplit(buf, n: int, stride: int, expected: Sequence[int], length: Optional[int] = None,
                             lens: Optional[Sequence[int]] = None, devices: Optional[Sequence[int]] = None,
                             host_threads: int = 0, device_blocks: Optional[int] = None) -> Tuple[int, int, int]:
    """The split leg of VerifyChecksumBatch: (first_bad, n_bad, blocks the devices hashed)."""
    a, la, ln, lp = _batch_args(buf, n, stride, length, lens)
    exp = _expected_arg(n, expected)
    if n == 0:
        return 0, 0, 0
    d = _devices_arg(devices)
    fb, nb, done = ctypes.c_uint64(0), ctypes.c_uint64(0), ctypes.c_uint64(0)
    rc = _lib.lib.stormck_verify_split(a.ctypes.data, stride, lp, ln, n, exp.ctypes.data, ctypes.byref(fb),
                                       ctypes.byref(nb), d, len(d) if d is not None else 0, host_threads,
                                       _lib.SPLIT_BALANCED if device_blocks is None else device_blocks,
                                       ctypes.byref(done))
    return _verify_rc(rc, fb, nb) + (done.value,)


def RouteDevices(devices: Optional[Sequence[int]] = None) -> None:
    """The devices the routed calls may use (stormck_route_devices); None: the calling
    thread's current device."""
    d = _devices_arg(devices) if devices else None
    _lib.check(_lib.lib.stormck_route_devices(d, len(d) if d is not None else 0))


def RouteRates() -> dict:
    """The routing model's current rates (bytes/us) and how many calls refined them."""
    r = _lib.RouteRates()
    _lib.check(_lib.lib.stormck_route_get_rates(ctypes.byref(r)))
    return r.as_dict()


def SetRouteRates(rates: Optional[dict] = None, freeze: bool = False) -> None:
    """Replace the routing rates (None: back to the priors); ``freeze`` stops the calls
    from updating them."""
    r = None
    if rates is not None:
        r = _lib.RouteRates(**{k: v for k, v in rates.items() if k != "observations"})
    _lib.check(_lib.lib.stormck_route_set_rates(ctypes.byref(r) if r is not None else None,
                                                _lib.RATES_FREEZE if freeze else _lib.RATES_LEARN))


def PlanBatch(n: int, stride: int, length: Optional[int] = None, lens: Optional[Sequence[int]] = None,
              pinned: bool = False, host_threads: int = 0, n_devices: int = 1) -> Tuple[int, Tuple[float, ...]]:
    """The routed batch's decision alone (stormck_route_plan_batch; no device needed):
    (leg, (host_us, device_us, split_us))."""
    la, ln = _lens_arg(n, length, lens)
    leg, us = ctypes.c_uint32(0), (ctypes.c_double * 3)()
    _lib.check(_lib.lib.stormck_route_plan_batch(stride, la.ctypes.data if la is not None else None, ln, n,
                                                 _lib.MEM_PINNED if pinned else _lib.MEM_PAGEABLE, host_threads,
                                                 n_devices, ctypes.byref(leg), us))
    return leg.value, tuple(us)


READ_FULL_BLOCK = 1  # STORMCK_READ_FULL_BLOCK


def ReadVerifyBatch(fd: int, addresses, lens, expected, dst, dst_stride: int, block_size: int = BLOCK_SIZE,
                    full_block: bool = False) -> Tuple[int, int]:
    """Batched cold read + verify (cache.fetchBlock for many blocks: Store.ReadBlock,
    persistence/store.go:39-51, then VerifyChecksum): reads block i from file `fd` at
    addresses[i] * block_size into dst + i*dst_stride and verifies it on the GPU.
    Returns (first_bad, n_bad); first_bad == n when every block verifies. A descriptor
    opened with O_DIRECT reads whole blocks into 512-byte aligned slots (stormck.h)."""
    ad = np.ascontiguousarray(np.asarray(addresses, dtype=np.uint64))
    la = np.ascontiguousarray(np.asarray(lens, dtype=np.uint32))
    ex = np.ascontiguousarray(np.asarray(expected, dtype=np.uint64))
    if isinstance(dst, np.ndarray) and not dst.flags.c_contiguous:
        raise ValueError("dst must be C-contiguous (a strided view would be read into a temporary copy)")
    d = _as_u8(dst)
    if not d.flags.writeable:
        raise ValueError("dst must be writable (the blocks are read into it)")
    n = ad.size
    if la.size != n or ex.size != n:
        raise ValueError("addresses, lens and expected need one entry per block")
    import fcntl
    full_block = full_block or bool(fcntl.fcntl(fd, fcntl.F_GETFL) & os.O_DIRECT)  # O_DIRECT reads whole blocks
    if n and d.size < (n - 1) * dst_stride + (block_size if full_block else int(la.max())):
        raise ValueError("dst too small")
    if n == 0:
        return 0, 0
    fb, nb = ctypes.c_uint64(0), ctypes.c_uint64(0)
    rc = _lib.lib.stormck_read_verify_fd(fd, ad.ctypes.data, la.ctypes.data, n, block_size, d.ctypes.data, dst_stride,
                                         ex.ctypes.data, READ_FULL_BLOCK if full_block else 0, ctypes.byref(fb),
                                         ctypes.byref(nb))
    if rc != _lib.EMISMATCH:
        _lib.check(rc)
    return fb.value, nb.value


def RegisterHostMemory(buf) -> None:
    """Page-lock a long-lived host buffer (storm's cache.data, allocated once in
    cache.New, cache/cache.go:36-40): host batches then DMA straight from it, and
    HostDevicePointer gives kernels in-place access to it. Kernels reading it in place
    run at the PCIe link rate only from 256-byte aligned rows (DESIGN_LOG.md §5); a
    misaligned buffer works, more slowly, and draws a warning."""
    a = _as_u8(buf)
    if a.ctypes.data % 256:
        import warnings
        warnings.warn(f"host buffer at {a.ctypes.data:#x} is not 256-byte aligned: in-place device reads of it "
                      "run at about 70% of the PCIe link rate", RuntimeWarning, stacklevel=2)
    _lib.check(_lib.lib.stormck_host_register(a.ctypes.data, a.nbytes))


def UnregisterHostMemory(buf) -> None:
    _lib.check(_lib.lib.stormck_host_unregister(_as_u8(buf).ctypes.data))


def HostDevicePointer(buf) -> int:
    """Device address of a registered host buffer (for the *_device entry points,
    e.g. commit.commit_device on a host-resident arena)."""
    d = ctypes.c_void_p()
    _lib.check(_lib.lib.stormck_host_device_pointer(_as_u8(buf).ctypes.data, ctypes.byref(d)))
    return int(d.value or 0)
