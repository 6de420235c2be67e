"""Probe (GPU box): which filesystems under the box's writable paths take O_DIRECT,
and what a 2 GiB sequential O_DIRECT write and read of 32 KiB blocks runs at there."""
import mmap
import os
import subprocess
import time

paths = [os.getcwd(), "/tmp", os.path.expanduser("~"), "/dev/shm", os.environ.get("TMPDIR", "/tmp")]
print(subprocess.run(["df", "-hT"] + paths, capture_output=True, text=True).stdout)
for p in dict.fromkeys(paths):
    f = os.path.join(p, f".odirect_probe_{os.getpid()}")
    try:
        fd = os.open(f, os.O_RDWR | os.O_CREAT | os.O_DIRECT, 0o600)
    except OSError as e:
        print(p, "O_DIRECT open failed:", e)
        continue
    try:
        buf = mmap.mmap(-1, 1 << 20)
        buf.write(os.urandom(1 << 20))
        n = 2048
        t0 = time.perf_counter()
        for i in range(n):
            os.pwrite(fd, buf, i << 20)
        os.fsync(fd)
        tw = time.perf_counter() - t0
        t0 = time.perf_counter()
        for i in range(n):
            os.preadv(fd, [buf], i << 20)
        tr = time.perf_counter() - t0
        print(p, f"O_DIRECT ok: write {n / tw / 1024:.2f} GiB/s, read {n / tr / 1024:.2f} GiB/s (1 MiB, QD1)")
    except OSError as e:
        print(p, "O_DIRECT I/O failed:", e)
    finally:
        os.close(fd)
        os.unlink(f)
