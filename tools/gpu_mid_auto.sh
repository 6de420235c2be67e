# Mid-size uniform batches after the balanced W-wave dispatch: parity of the uniform
# paths and the dispatch fuzz, then us per launch, default against the kernels before
# (STORMCK_MID_WAVES=5), alternating in one session.
set -o pipefail
out=gpurun_out/${1:-mid_auto}
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "uniform_fast_path or fuzz or verify_device or large_batch" > $out/tests.log 2>&1; rc=$?
grep -E "passed|failed|error" $out/tests.log | tail -3; [ $rc -eq 0 ] || exit $rc
S="8192 9216 9728 9984 10240 12288 16384 20000 24575"
for i in 1 2; do
  for w in 0 5; do
    STORMCK_MID_WAVES=$w timeout -k 10 120 python tools/small_batch_probe.py $S > $out/auto_w${w}_$i.txt 2>&1 || exit 1
    echo "knob $w run $i: $(grep n= $out/auto_w${w}_$i.txt | tr '\n' ' ')"
  done
done
