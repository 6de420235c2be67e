"""Rate drift within one process: one 128 GiB arena, the bench's hash launch timed in
blocks of 4 launches, with and without idle gaps between blocks (bench variance study,
DESIGN_LOG.md §5). Usage: python tools/drift.py [rounds]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from storm_amd import engine  # noqa: E402

BLOCK, N = 32768, 4 << 20


def main(rounds: int):
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    arena = torch.empty((N, BLOCK), dtype=torch.uint8, device=dev)
    engine.fill_synthetic_device(arena.data_ptr(), BLOCK, N, 0, 0x53544F524D)
    cs = torch.empty(N, dtype=torch.int64, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    torch.cuda.synchronize()

    def block(k=4):
        e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        e[0].record()
        for _ in range(k):
            engine.checksum_device(arena.data_ptr(), BLOCK, N, cs.data_ptr(), BLOCK, 0, st)
        e[1].record()
        torch.cuda.synchronize()
        return e[0].elapsed_time(e[1]) / k

    t0 = time.perf_counter()
    for r in range(rounds):
        gap = 0.0 if r % 3 else 5.0
        if gap:
            time.sleep(gap)
        ms = block()
        print("t=%6.1fs gap=%.0fs  %.3f ms/launch  %.1f GB/s" % (time.perf_counter() - t0, gap, ms,
                                                                  N * (BLOCK + 8) / ms / 1e6), flush=True)
    # sustained: 10 s of back-to-back launches, reported per second
    t1 = time.perf_counter()
    while time.perf_counter() - t1 < 10:
        ms = block(12)
        print("sustained t=%6.1fs  %.3f ms/launch" % (time.perf_counter() - t0, ms), flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 12)
