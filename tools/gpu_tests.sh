# All GPU tests, then the Merkle level probe of the default kernel
set -o pipefail
out=gpurun_out/${1:-tests}
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $out/tests.log 2>&1; rc=$?
grep -E "passed|failed|error" $out/tests.log | tail -3
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/merkle_probe.py > $out/merkle.txt 2>&1 && grep "level of" $out/merkle.txt
