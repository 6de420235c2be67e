# f1 small-level kernel: GPU tests, then c5 (commit of one storm batch) and the 1M-leaf
# commit with k_commit_level_wide off (0) and at 256 / 1024 blocks (GPU box, repo root).
set -o pipefail
out=gpurun_out/cw
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for w in 0 256 1024; do
  STORMCK_COMMIT_WIDE=$w timeout -k 10 120 python -u bench.py --workload c5 --steps 200 --no-cpu > $out/c5_$w.log 2>&1 || exit 1
  echo "wide<=$w c5: $(tail -1 $out/c5_$w.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("batch_us", d["batch_us"], "commit_forest_us", d["commit_forest_us"])')"
  STORMCK_COMMIT_WIDE=$w timeout -k 10 120 python -u bench.py --workload commit --steps 10 --no-cpu > $out/commit_$w.log 2>&1 || exit 1
  echo "wide<=$w commit 1M: $(tail -1 $out/commit_$w.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("ms", d["ms_per_step"], "GiB/s", d["value"])')"
done
