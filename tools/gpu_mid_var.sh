# Mid-size per-block-length batches (storm's mixed sizes): var kernel in 3-/1-wave
# workgroups (default) against 2-wave ones (STORMCK_MID_WAVES=5); parity first.
set -o pipefail
out=gpurun_out/${1:-mid_var}
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "var or fuzz or gather or lens or verify" > $out/tests.log 2>&1; rc=$?
grep -E "passed|failed|error" $out/tests.log | tail -3; [ $rc -eq 0 ] || exit $rc
S="10240 12288 16384 20000 24575"
for i in 1 2; do
  for w in 0 5; do
    PROBE_LENS=1 STORMCK_MID_WAVES=$w timeout -k 10 120 python tools/small_batch_probe.py $S > $out/var_w${w}_$i.txt 2>&1 || exit 1
    echo "knob $w run $i: $(grep n= $out/var_w${w}_$i.txt | tr '\n' ' ')"
  done
done
