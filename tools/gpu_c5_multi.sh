# c5 commit forest: k_commit_level_multi (leaf level) A/B against the register-quad level
# kernel (STORMCK_COMMIT_MULTI=0), commit + parity tests, kernel trace of the shipped path.
set -o pipefail
out=gpurun_out/${1:-c5m}
mkdir -p $out
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 300 python -u -m pytest tests/test_commit.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1 && echo tests-ok && tail -1 $out/tests.log &&
for i in 1 2; do
  STORMCK_COMMIT_MULTI=0 timeout -k 10 120 python bench.py --workload c5 --steps 200 --warmup 10 --no-cpu > $out/quad$i.log 2>&1 || exit 1
  echo "quad  $i: $(grep -o '"commit_forest_us": [0-9.]*' $out/quad$i.log)"
  timeout -k 10 120 python bench.py --workload c5 --steps 200 --warmup 10 --no-cpu > $out/multi$i.log 2>&1 || exit 1
  echo "multi $i: $(grep -o '"commit_forest_us": [0-9.]*' $out/multi$i.log)"
done &&
STORMCK_TRACE=1 timeout -k 10 120 python bench.py --workload c5 --steps 20 --warmup 2 --settle 0 --no-cpu > $out/trace.log 2>&1 &&
(cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$out/prof" -o c5 -- \
   python3 "$R/bench.py" --workload c5 --steps 200 --warmup 10 --no-cpu > "$R/$out/prof.log" 2>&1) && echo prof-ok
