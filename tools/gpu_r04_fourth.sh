# Round 4, fourth GPU session: the -m gpu suite, the f1 end-to-end table again (routed
# legs with the refit host rate), and the gather A/B of k_order_rank (rows of a group
# dealt by length rank; probe build, STORMCK_GATHER_RANK=1 = by rank), 3 fresh
# processes per side, alternating.
# Usage: bash tools/gpu_r04_fourth.sh <tag>
set -o pipefail
out=gpurun_out/${1:-r04_fourth}
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1; rc=$?
grep -E "passed|failed|error" $out/tests.log | tail -3
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python bench.py --workload commit_e2e --steps 9 > $out/commit_e2e.log 2>&1 || exit 1
for i in 1 2 3; do
  for r in 0 1; do
    STORMCK_LIBRARY=tools/libstormck_probes.so STORMCK_GATHER_RANK=$r timeout -k 10 200 python bench.py \
        --workload gather --steps 5 --warmup 1 > $out/gather_rank${r}_$i.log 2>&1 || exit 1
    python3 -c "
import json,sys
d=json.loads([l for l in open('$out/gather_rank${r}_$i.log') if l.startswith('{')][-1]); r=d['roofline']
print('rank=$r run $i', r['frac'], r['avg_launch_ms'], r['uniform_same_arena']['frac'], d['digest'])"
  done
done
exit $rc
