# Round 4, second GPU session: the whole -m gpu suite, the f1 end-to-end table from
# registered host memory (bench.py --workload commit_e2e), and a parity run of the
# kernel-family tests through the debug build, which counts quad merges made with a
# partially active quad (STORMCK_CHECK_PARTIAL_QUADS, tests/conftest.py).
# Usage: bash tools/gpu_r04_second.sh <tag>
set -o pipefail
out=gpurun_out/${1:-r04_second}
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1; rc=$?
grep -E "passed|failed|error" $out/tests.log | tail -3
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python bench.py --workload commit_e2e --steps 9 > $out/commit_e2e.log 2>&1 || exit 1
tail -c 1500 $out/commit_e2e.log
STORMCK_LIBRARY=tools/libstormck_debug.so STORMCK_CHECK_PARTIAL_QUADS=1 timeout -k 10 600 python -u -m pytest \
    tests/test_dispatch_fuzz.py tests/test_glds_var.py tests/test_commit.py tests/test_gpu_parity.py \
    -m gpu -x -v --timeout 300 --timeout-method thread > $out/debug_quads.log 2>&1 || exit 1
tail -4 $out/debug_quads.log
exit $rc
