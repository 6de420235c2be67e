# k_xxh64_wide_multi: GPU tests, then c5 and small-batch latencies with it off/on (GPU box).
set -o pipefail
out=gpurun_out/multi
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for m in 0 1; do
  STORMCK_WIDE_MULTI=$m timeout -k 10 120 python -u bench.py --workload c5 --steps 200 --no-cpu > $out/c5_$m.log 2>&1 || exit 1
  echo "multi=$m c5: $(tail -1 $out/c5_$m.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("batch_us", d["batch_us"], "commit_forest_us", d["commit_forest_us"])')"
done
for m in 0 1; do
  STORMCK_WIDE_MULTI=$m timeout -k 10 120 python -u bench.py --workload commit --steps 10 --no-cpu > $out/commit_$m.log 2>&1 || exit 1
  echo "multi=$m commit 1M: $(tail -1 $out/commit_$m.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("ms", d["ms_per_step"])')"
done
