# Round 4, first GPU session (repo root on the GPU box): the whole -m gpu suite, then the
# arena-placement experiment the round-3 verdict asked for: fresh c3 bench processes
# alternating plain hipMalloc / VMM (one physical allocation) / VMM (1 GiB allocations),
# 4 per mode, then one per mode under rocprofv3 --kernel-trace --stats.
# Usage: bash tools/gpu_r04_first.sh <tag> [runs]
set -o pipefail
tag=${1:-r04_first}
runs=${2:-4}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1; rc=$?
grep -E "passed|failed|error" $out/tests.log | tail -3
# plain test failures (1) leave the GPU fine; anything else (timeout, crash) ends the call
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for i in $(seq 1 $runs); do
  for mode in plain vmm vmm1g; do
    timeout -k 10 200 python bench.py --no-cpu --steps 5 --warmup 1 --alloc $mode > $out/plain_${mode}_$i.log 2>&1 || exit 1
    python tools/placement_summary.py $out/plain_${mode}_$i.log | tee -a $out/placement.jsonl || exit 1
  done
done
for mode in plain vmm vmm1g; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
      -d $R/$out/prof_$mode -o trace -- python3 $R/bench.py --no-cpu --steps 5 --warmup 1 --alloc $mode \
      > $R/$out/prof_$mode.log 2>&1) || exit 1
  python tools/placement_summary.py $out/prof_$mode.log $out/prof_$mode | tee -a $out/placement.jsonl || exit 1
done
exit $rc
