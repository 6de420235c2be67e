# Ring depth of the pipelined wide-multi staging: 4 slots (shipped) vs 6 (STORMCK_RING_SLOTS=6),
# alternating on one box: c5 objectlist batch + commit forest and BenchmarkStorm's blob mix;
# parity tests that reach the kernels under the 6-slot ring first.
set -o pipefail
out=gpurun_out/${1:-ring_ab}
mkdir -p $out
export TMPDIR=/tmp
STORMCK_RING_SLOTS=6 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_dispatch_fuzz.py tests/test_commit.py -k "ring or c5 or fuzz or commit" -m gpu -x -q --timeout 100 --timeout-method thread > $out/tests6.log 2>&1 && echo tests6-ok && tail -1 $out/tests6.log || { echo tests6-failed; tail -20 $out/tests6.log; exit 1; }
for i in 1 2 3; do
  for r in 4 6; do
    STORMCK_RING_SLOTS=$r timeout -k 10 120 python bench.py --workload c5 --steps 300 --warmup 10 --no-cpu > $out/ol_r$r.$i.log 2>&1 || exit 1
    STORMCK_RING_SLOTS=$r timeout -k 10 120 python bench.py --workload c5 --c5-mix storm --steps 300 --warmup 10 --no-cpu > $out/st_r$r.$i.log 2>&1 || exit 1
    echo "ring $r run $i: objectlist $(grep -o '"batch_us": [0-9.]*' $out/ol_r$r.$i.log) $(grep -o '"commit_forest_us": [0-9.]*' $out/ol_r$r.$i.log) | storm $(grep -o '"batch_us": [0-9.]*' $out/st_r$r.$i.log) $(grep -o '"commit_forest_us": [0-9.]*' $out/st_r$r.$i.log) $(grep -c MISMATCH $out/ol_r$r.$i.log $out/st_r$r.$i.log | tr '\n' ' ')"
  done
done
