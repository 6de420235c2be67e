"""Seeded random batches across the batch-size dispatch of launch_checksum
(storm_amd/csrc/stormck.hip): one workgroup per block (<= 128), five staged blocks per
workgroup (<= 5 per CU), 8 and 16 ring-staged blocks per workgroup (<= 16 per CU),
register quad, LDS-staged streaming in 2- and 8-wave workgroups (uniform lengths:
k_xxh64_glds; per-block lengths and gathered offsets: k_xxh64_glds_var); uniform lengths, per-block lengths and gathered offsets; 16-byte, 8-byte and
odd base alignments and strides; checksum and verify (first bad index, count). Every
block is compared with the C oracle (XXH64 seed 0 = blocks.Checksum,
/root/reference/blocks/checksum.go:15-17). The named tests in test_gpu_parity.py pin
each class's edges; this one covers the cross product at random points."""
import numpy as np
import pytest

from oracle import oracle as o

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

CLASSES = [(1, 128), (129, 1280), (1281, 2048), (2049, 4096), (4097, 10239), (10240, 24575), (24576, 40000)]
BUDGET = 48 << 20  # bytes of block data per case


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def _case(seed):
    rng = np.random.default_rng(seed)
    lo, hi = CLASSES[seed % len(CLASSES)]
    n = int(rng.integers(lo, hi + 1))
    mode = ("uniform", "lens", "gather")[int(rng.integers(0, 3))]
    aligned = bool(rng.integers(0, 2))  # 16-byte base and stride: the streaming kernels' condition
    maxlen = max(1, min(33000, BUDGET // n - 64))
    if aligned and mode == "uniform" and rng.integers(0, 2):
        length = int(rng.integers(512, maxlen + 1)) if maxlen >= 512 else int(rng.integers(0, maxlen + 1))
    else:
        length = int(rng.integers(0, maxlen + 1))
    lens = rng.integers(0, length + 1, size=n).astype(np.uint32) if mode != "uniform" else None
    stride = length + int(rng.integers(0, 64))
    shift = 0
    if aligned:
        stride = (stride + 15) // 16 * 16
    else:
        shift = int(rng.choice([8, int(rng.integers(1, 16))]))
    stride = max(stride, 1)
    return rng, n, mode, length, lens, stride, shift


@pytest.mark.parametrize("seed", range(49))
def test_dispatch_fuzz(dev, seed):
    from storm_amd import engine
    rng, n, mode, length, lens, stride, shift = _case(seed)
    size = shift + n * stride + 64
    host = rng.integers(0, 256, size=size, dtype=np.uint8)
    d = torch.from_numpy(host).to(dev)
    base = d.data_ptr() + shift
    out = torch.empty(n, dtype=torch.int64, device=dev)
    d_lens = torch.from_numpy(lens.view(np.int32)).to(dev) if lens is not None else None
    lp = d_lens.data_ptr() if d_lens is not None else 0
    if mode == "gather":
        offs = (np.arange(n, dtype=np.uint64) * stride + shift
                + rng.integers(0, max(1, stride - int(lens.max()) + 1), size=n).astype(np.uint64))
        d_offs = torch.from_numpy(offs.view(np.int64)).to(dev)
        engine.checksum_gather_device(d.data_ptr(), d_offs.data_ptr(), n, out.data_ptr(), 0, lp)
        want = np.array([o.xxh64(host[int(offs[i]):int(offs[i]) + int(lens[i])]) for i in range(n)],
                        dtype=np.uint64)
    else:
        engine.checksum_device(base, stride, n, out.data_ptr(), length, lp)
        want = o.checksum_batch(host[shift:], n, stride, length, lens=lens, threads=8)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint64)
    bad_blocks = np.nonzero(got != want)[0]
    assert len(bad_blocks) == 0, (seed, n, mode, length, stride, shift, bad_blocks[:8])
    if mode == "gather":
        return
    # verify through the same dispatch: k corrupted expectations
    k = int(rng.integers(0, min(n, 5) + 1))
    idx = np.sort(rng.choice(n, size=k, replace=False)) if k else np.array([], dtype=np.int64)
    exp = want.copy()
    exp[idx] ^= np.uint64(1)
    res = torch.zeros(2, dtype=torch.int64, device=dev)
    engine.verify_device(base, stride, n, torch.from_numpy(exp.view(np.int64)).to(dev).data_ptr(), res.data_ptr(),
                         length, lp)
    torch.cuda.synchronize()
    first = int(idx[0]) if k else n
    assert res.cpu().numpy().view(np.uint64).tolist() == [first, k], (seed, n, mode, length, stride, shift)
