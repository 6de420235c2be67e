# Round 4, fourth GPU session: the -m gpu suite on the refit cost model, and the f1
# end-to-end table again (routed legs with the refit host rate).
# Usage: bash tools/gpu_r04_fourth.sh <tag>
set -o pipefail
out=gpurun_out/${1:-r04_fourth}
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1; rc=$?
grep -E "passed|failed|error" $out/tests.log | tail -3
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python bench.py --workload commit_e2e --steps 9 > $out/commit_e2e.log 2>&1 || exit 1
exit $rc
