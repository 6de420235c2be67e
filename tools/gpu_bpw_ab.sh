# Blocks per workgroup of the ring-staged wide-multi kernels: 8 (STORMCK_MULTI_BPW default
# under test) vs 5, alternating on one box: parity tests under both, c5 objectlist batch +
# commit forest, BenchmarkStorm's blob mix, uniform batches of 1,200-2,560 blocks.
set -o pipefail
out=gpurun_out/${1:-bpw_ab}
mkdir -p $out
export TMPDIR=/tmp
for b in 8 5; do
  STORMCK_MULTI_BPW=$b timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_dispatch_fuzz.py tests/test_commit.py tests/test_full_size_gpu.py -k "ring or c5 or fuzz or commit" -m gpu -x -q --timeout 100 --timeout-method thread > $out/tests$b.log 2>&1 && echo "tests bpw $b ok: $(tail -1 $out/tests$b.log)" || { echo tests$b-failed; tail -20 $out/tests$b.log; exit 1; }
done
for i in 1 2; do
  for b in 8 5; do
    STORMCK_MULTI_BPW=$b timeout -k 10 120 python bench.py --workload c5 --steps 300 --warmup 10 --no-cpu > $out/ol_b$b.$i.log 2>&1 || exit 1
    STORMCK_MULTI_BPW=$b timeout -k 10 120 python bench.py --workload c5 --c5-mix storm --steps 300 --warmup 10 --no-cpu > $out/st_b$b.$i.log 2>&1 || exit 1
    STORMCK_MULTI_BPW=$b timeout -k 10 120 python tools/small_batch_probe.py 1200 1280 1600 2048 2560 > $out/sz_b$b.$i.txt 2>&1 || exit 1
    echo "bpw $b run $i: objectlist $(grep -o '"batch_us": [0-9.]*' $out/ol_b$b.$i.log) $(grep -o '"commit_forest_us": [0-9.]*' $out/ol_b$b.$i.log) | storm $(grep -o '"batch_us": [0-9.]*' $out/st_b$b.$i.log) $(grep -o '"commit_forest_us": [0-9.]*' $out/st_b$b.$i.log) | $(grep -h '^n=' $out/sz_b$b.$i.txt | tr '\n' ' ') | mismatches $(cat $out/ol_b$b.$i.log $out/st_b$b.$i.log | grep -c MISMATCH)"
  done
done
