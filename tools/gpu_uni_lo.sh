set -o pipefail
out=gpurun_out/uni_lo
mkdir -p $out
S="7168 8192 8704 9216 9728"
for i in 1 2; do
  for k in 0 3 1; do
    STORMCK_MID_WAVES=$k timeout -k 10 120 python tools/small_batch_probe.py $S > $out/unilo_${k}_$i.txt 2>&1 || exit 1
    echo "mid_waves=$k run $i: $(grep n= $out/unilo_${k}_$i.txt | tr '\n' ' ')"
  done
done
