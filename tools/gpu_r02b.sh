# r02b: c4 / c3 root tests, the skewed-kernel test (every block vs the oracle), the
# bench at N = 1 (c3 root check) and a self-spawned 2-rank c4 rehearsal on one GPU (gloo)
set -o pipefail
out=gpurun_out/r02b
mkdir -p $out
nproc > $out/host.txt; cat /sys/fs/cgroup/cpu.max >> $out/host.txt 2>&1; grep -m1 "model name" /proc/cpuinfo >> $out/host.txt
python -c "import os; print('affinity', len(os.sched_getaffinity(0)))" >> $out/host.txt
timeout -k 10 300 python -u -m pytest tests/test_c4_gpu.py "tests/test_gpu_parity.py::test_large_batch_skewed_kernel" -x -v --timeout 250 --timeout-method thread > $out/tests.log 2>&1 && echo tests-ok &&
timeout -k 10 300 python bench.py > $out/bench.log 2>&1 && echo bench-ok && tail -1 $out/bench.log &&
timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --arena 2097152 --no-cpu --steps 2 --warmup 1 > $out/bench_spawn2.log 2>&1 && echo spawn-ok && tail -1 $out/bench_spawn2.log
