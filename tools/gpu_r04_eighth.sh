# Round 4, eighth GPU session: the -m gpu suite (routed host batches included), smoke,
# the default c3 bench line, the host-memory batch E2E table by leg (batch_e2e), then a
# gather A/B: storm's mixed lengths vs one 32 KiB length through the same gathered,
# locality-ordered path (2 fresh processes each, alternating).
# Usage: bash tools/gpu_r04_eighth.sh <tag>
set -o pipefail
out=gpurun_out/${1:-r04_eighth}
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1; rc=$?
grep -E "passed|failed|error" $out/tests.log | tail -3; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 && tail -1 $out/smoke.log &&
timeout -k 10 300 python bench.py > $out/bench.log 2>&1 && tail -c 600 $out/bench.log &&
timeout -k 10 400 python bench.py --workload batch_e2e --steps 7 > $out/batch_e2e.log 2>&1 && tail -c 300 $out/batch_e2e.log || exit 1
for i in 1 2; do
  for L in 0 32768; do
    timeout -k 10 200 python bench.py --workload gather --steps 5 --warmup 1 --gather-lens $L > $out/gather_L${L}_$i.log 2>&1 || exit 1
    python3 -c "
import json
d=json.loads([l for l in open('$out/gather_L${L}_$i.log') if l.startswith('{')][-1]); r=d['roofline']
print('lens=$L run $i', r['frac'], r['avg_launch_ms'], r['uniform_same_arena']['frac'])"
  done
done
