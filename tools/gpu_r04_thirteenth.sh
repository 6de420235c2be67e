# Round 4, thirteenth GPU session: check of the final tree (all GPU tests, smoke, the
# default c3 bench line), then a rocprofv3 kernel trace of the gather workload (the order
# kernels with the 128-part placement) and two gather lines beside the uniform kernel.
# Usage: bash tools/gpu_r04_thirteenth.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/${1:-r04_thirteenth}
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1; rc=$?
grep -E "passed|failed|error" $out/tests.log | tail -3; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 && tail -1 $out/smoke.log &&
timeout -k 10 300 python bench.py > $out/bench.log 2>&1 && tail -c 400 $out/bench.log || exit 1
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/gather_trace" -o trace -- \
    python3 "$R/bench.py" --workload gather --steps 5 --warmup 1 > "$out/gather_trace.log" 2>&1) || exit 1
for i in 1 2; do
  timeout -k 10 200 python bench.py --workload gather --steps 5 --warmup 1 > $out/gather_$i.log 2>&1 || exit 1
  python3 -c "
import json
d=json.loads([l for l in open('$out/gather_$i.log') if l.startswith('{')][-1]); r=d['roofline']
print('gather $i', r['frac'], r['avg_launch_ms'], r['uniform_same_arena']['frac'], round(r['frac']/r['uniform_same_arena']['frac'],4), d['digest'])"
done
