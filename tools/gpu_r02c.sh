# r02c: all GPU tests, the Merkle level probe (ring vs register-quad kernel), and the
# single-call probe (host leg vs device single call)
set -o pipefail
out=gpurun_out/r02c
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 250 --timeout-method thread > $out/tests.log 2>&1; rc=$?
tail -3 $out/tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 120 python tools/merkle_probe.py > $out/merkle_ring.txt 2>&1 && cat $out/merkle_ring.txt &&
STORMCK_POINTER_RING=0 timeout -k 10 120 python tools/merkle_probe.py > $out/merkle_quad.txt 2>&1 && cat $out/merkle_quad.txt &&
timeout -k 10 200 ./tools/single_call_probe > $out/single_call.txt 2>&1 && cat $out/single_call.txt
