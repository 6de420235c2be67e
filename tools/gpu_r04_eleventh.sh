# Round 4, eleventh GPU session: the rebuilt locality order (k_order_*): the -m gpu suite,
# a rocprofv3 kernel trace of the gather workload (the order kernels' own times), then
# the gathered-form A/B again (32 KiB and storm's lengths; strided / sorted offsets /
# shuffled offsets), 2 fresh processes each, alternating.
# Usage: bash tools/gpu_r04_eleventh.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/${1:-r04_eleventh}
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1; rc=$?
grep -E "passed|failed|error" $out/tests.log | tail -3; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/gather_trace" -o trace -- \
    python3 "$R/bench.py" --workload gather --steps 5 --warmup 1 > "$out/gather_trace.log" 2>&1) || exit 1
run() {  # name, env..., -- bench args
  local name=$1; shift
  timeout -k 10 200 env "$@" > $out/$name.log 2>&1 || return 1
  python3 -c "
import json
d=json.loads([l for l in open('$out/$name.log') if l.startswith('{')][-1]); r=d['roofline']
print('$name', r['frac'], r['avg_launch_ms'], r['uniform_same_arena']['frac'], round(r['frac']/r['uniform_same_arena']['frac'],4), d['digest'])"
}
B="python bench.py --workload gather --steps 5 --warmup 1"
for i in 1 2; do
  for L in 32768 0; do
    run strided_L${L}_$i X=1 $B --gather-lens $L --gather-order strided || exit 1
    run seq_order_L${L}_$i X=1 $B --gather-lens $L --gather-order sequential || exit 1
    run shuffled_L${L}_$i X=1 $B --gather-lens $L --gather-order shuffled || exit 1
  done
done
