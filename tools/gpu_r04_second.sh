# Round 4, second GPU session: the whole -m gpu suite, then the f1 end-to-end table from
# registered host memory (bench.py --workload commit_e2e).
# Usage: bash tools/gpu_r04_second.sh <tag>
set -o pipefail
out=gpurun_out/${1:-r04_second}
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1; rc=$?
grep -E "passed|failed|error" $out/tests.log | tail -3
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python bench.py --workload commit_e2e --steps 9 > $out/commit_e2e.log 2>&1 || exit 1
tail -c 3000 $out/commit_e2e.log
exit $rc
