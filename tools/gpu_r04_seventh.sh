# Round 4, seventh GPU session: check of HEAD after the re-entry (all GPU tests, smoke,
# the default c3 bench line).
# Usage: bash tools/gpu_r04_seventh.sh <tag>
set -o pipefail
out=gpurun_out/${1:-r04_seventh}
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1; rc=$?
grep -E "passed|failed|error" $out/tests.log | tail -3; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 && tail -1 $out/smoke.log &&
timeout -k 10 300 python bench.py > $out/bench.log 2>&1 && tail -c 600 $out/bench.log
