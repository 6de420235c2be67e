# Per-block-length batches of 10K-50K blocks: var kernel (default) against the register
# quad kernel (STORMCK_GLDS_VAR=0).
set -o pipefail
out=gpurun_out/${1:-var_hi}
mkdir -p $out
S="10240 12288 16384 20000 24575 36864 49152"
for i in 1 2; do
  for k in 1 0; do
    PROBE_LENS=1 STORMCK_GLDS_VAR=$k timeout -k 10 120 python tools/small_batch_probe.py $S > $out/varhi_${k}_$i.txt 2>&1 || exit 1
    echo "glds_var=$k run $i: $(grep n= $out/varhi_${k}_$i.txt | tr '\n' ' ')"
  done
done
