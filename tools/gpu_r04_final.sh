# Round 4, final GPU check of the tree: all GPU tests, smoke, the default c3 bench line,
# one gather line (storm's batch shape) and one batch_e2e table.
# Usage: bash tools/gpu_r04_final.sh <tag>
set -o pipefail
out=gpurun_out/${1:-r04_final}
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1; rc=$?
grep -E "passed|failed|error" $out/tests.log | tail -3; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 && tail -1 $out/smoke.log &&
timeout -k 10 300 python bench.py > $out/bench.log 2>&1 && tail -c 300 $out/bench.log &&
timeout -k 10 200 python bench.py --workload gather --steps 5 --warmup 1 > $out/gather.log 2>&1 && tail -c 200 $out/gather.log &&
timeout -k 10 400 python bench.py --workload batch_e2e --steps 7 > $out/batch_e2e.log 2>&1 && tail -c 200 $out/batch_e2e.log
