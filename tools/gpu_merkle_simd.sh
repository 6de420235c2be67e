# Merkle level: SIMD-ranked roles and C per level (A/B against static roles / C = 1),
# the dispatcher's wave placement, and the pointer-level parity tests.
set -o pipefail
out=gpurun_out/${1:-merkle_simd}
mkdir -p $out
timeout -k 10 60 ./tools/hwid_probe > $out/hwid.txt 2>&1 && cat $out/hwid.txt &&
timeout -k 10 200 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "pointer or merkle or c4 or root" > $out/tests.log 2>&1; rc=$?
tail -2 $out/tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 120 python tools/merkle_probe.py > $out/auto_$i.txt 2>&1 && grep "level of" $out/auto_$i.txt | head -3 &&
STORMCK_POINTER_SIMD=0 timeout -k 10 120 python tools/merkle_probe.py > $out/static_$i.txt 2>&1 && grep "level of" $out/static_$i.txt | head -3 | sed 's/^/static /' &&
STORMCK_POINTER_C=1 timeout -k 10 120 python tools/merkle_probe.py > $out/c1_$i.txt 2>&1 && grep "level of" $out/c1_$i.txt | head -3 | sed 's/^/c1 /' || exit 1
done
