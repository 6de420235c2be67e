# Round 4, twelfth GPU session: deferred scatter of a locality-ordered gather's checksums
# (probe build, STORMCK_GATHER_DEFER=1: coalesced stores into the sorted positions, then
# k_order_scatter) against the in-kernel scattered stores: parity of the gather tests
# through the deferred form, a kernel trace of it, then shuffled gathers (storm's lengths
# and 32 KiB) alternating, 2 fresh processes each.
# Usage: bash tools/gpu_r04_twelfth.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/${1:-r04_twelfth}
mkdir -p $out
P="STORMCK_LIBRARY=tools/libstormck_probes.so"
timeout -k 10 600 env $P STORMCK_GATHER_DEFER=1 python -u -m pytest tests/test_glds_var.py -x -v --timeout 300 \
    --timeout-method thread > $out/tests_defer.log 2>&1; rc=$?
grep -E "passed|failed|error" $out/tests_defer.log | tail -3; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 env STORMCK_LIBRARY=$R/tools/libstormck_probes.so STORMCK_GATHER_DEFER=1 \
    rocprofv3 --kernel-trace --stats --output-format csv -d "$out/defer_trace" -o trace -- \
    python3 "$R/bench.py" --workload gather --steps 5 --warmup 1 > "$out/defer_trace.log" 2>&1) || exit 1
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
  for L in 0 32768; do
    for D in 0 1; do
      run defer${D}_L${L}_$i $P STORMCK_GATHER_DEFER=$D $B --gather-lens $L || exit 1
    done
  done
done
