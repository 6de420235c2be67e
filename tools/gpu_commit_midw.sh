# Mid-size commit levels: LDS-DMA commit kernel in 3-/1-wave workgroups (default) against
# the launches before (STORMCK_COMMIT_MIDW=0); commit parity first.
set -o pipefail
out=gpurun_out/${1:-commit_midw}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "commit" > $out/tests.log 2>&1; rc=$?
grep -E "passed|failed|error" $out/tests.log | tail -3; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for k in 1 0; do
    for n in 12288 20000 36864; do
      STORMCK_COMMIT_MIDW=$k timeout -k 10 200 python bench.py --workload commit --commit-leaves $n --steps 20 --warmup 3 > $out/c${k}_${n}_$i.log 2>&1 || exit 1
      python -c "import json; d=json.loads(open('$out/c${k}_${n}_$i.log').read().strip().splitlines()[-1]); print('midw=$k n=$n run $i', d['ms_per_step'], 'ms')"
    done
  done
done
