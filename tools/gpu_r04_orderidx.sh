# Round 4: index-only placement (probe build, STORMCK_ORDER_IDX=1) against the shipped
# order pass: gather parity through it, kernel traces of both (the order kernels' times),
# 2 gather lines each, alternating.
# Usage: bash tools/gpu_r04_orderidx.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/${1:-r04_orderidx}
mkdir -p $out
P="STORMCK_LIBRARY=$R/tools/libstormck_probes.so"
timeout -k 10 600 env $P STORMCK_ORDER_IDX=1 python -u -m pytest tests/test_glds_var.py -x -v --timeout 300 \
    --timeout-method thread > $out/tests_idx.log 2>&1; rc=$?
grep -E "passed|failed|error" $out/tests_idx.log | tail -3; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
for X in 0 1; do
  (cd /tmp && timeout -k 10 300 env $P STORMCK_ORDER_IDX=$X rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$out/trace_idx$X" -o trace -- python3 "$R/bench.py" --workload gather --steps 5 --warmup 1 \
      > "$out/trace_idx$X.log" 2>&1) || exit 1
  python3 - <<PY
import csv
for row in csv.reader(open("$out/trace_idx$X/trace_kernel_stats.csv")):
    if row[0].startswith("stormck::k_order") or "k_order" in row[0]:
        print("idx=$X", row[0].split("(")[0], round(float(row[3]) / 1000, 1), "us")
PY
done
for i in 1 2; do
  for X in 0 1; do
    timeout -k 10 200 env $P STORMCK_ORDER_IDX=$X python bench.py --workload gather --steps 5 --warmup 1 > $out/idx${X}_$i.log 2>&1 || exit 1
    python3 -c "
import json
d=json.loads([l for l in open('$out/idx${X}_$i.log') if l.startswith('{')][-1]); r=d['roofline']
print('idx=$X run $i', r['frac'], r['avg_launch_ms'], r['uniform_same_arena']['frac'], round(r['frac']/r['uniform_same_arena']['frac'],4), d['digest'])"
  done
done
