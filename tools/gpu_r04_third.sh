# Round 4, third GPU session: the -m gpu suite, smoke, the f1 end-to-end table after the
# cost-model refit, and the default c3 bench line.
# Usage: bash tools/gpu_r04_third.sh <tag>
set -o pipefail
out=gpurun_out/${1:-r04_third}
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1; rc=$?
grep -E "passed|failed|error" $out/tests.log | tail -3
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 && tail -1 $out/smoke.log || exit 1
timeout -k 10 400 python bench.py --workload commit_e2e --steps 9 > $out/commit_e2e.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > $out/bench.log 2>&1 || exit 1
tail -c 600 $out/bench.log
# host XXH64 rates of the box's CPU (no GPU use): scalar vs AVX-512 multi-block
timeout -k 10 120 ./tools/host_xxh64_probe > $out/host_xxh64.txt 2>&1 && cat $out/host_xxh64.txt
exit $rc
