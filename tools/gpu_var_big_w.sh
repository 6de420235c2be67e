# Per-block-length batches of 24K-128K blocks: 3-wave workgroups where they balance
# better (default) against 8-wave ones (STORMCK_BIG_W=0); parity first.
set -o pipefail
out=gpurun_out/${1:-var_big_w}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "var or gather or fuzz or lens" > $out/tests.log 2>&1; rc=$?
grep -E "passed|failed|error" $out/tests.log | tail -3; [ $rc -eq 0 ] || exit $rc
S="24641 32768 36864 40000 45000 49152"
for i in 1 2; do
  for k in 1 0; do
    PROBE_LENS=1 STORMCK_BIG_W=$k timeout -k 10 120 python tools/small_batch_probe.py $S > $out/varbigw${k}_$i.txt 2>&1 || exit 1
    echo "big_w=$k run $i: $(grep n= $out/varbigw${k}_$i.txt | tr '\n' ' ')"
  done
done
