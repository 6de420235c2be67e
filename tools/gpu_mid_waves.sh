# Mid-size uniform batches: the LDS-DMA kernel in W-wave workgroups (STORMCK_MID_WAVES)
# against the shipped dispatch (quad kernels below 10,240 blocks, 2-wave LDS-DMA above).
set -o pipefail
out=gpurun_out/${1:-mid_waves}
mkdir -p $out
S="6144 8192 10000 10240 12288 16384 20000 24575"
for i in 1 2; do
  for w in 0 1 2 3 4; do
    STORMCK_MID_WAVES=$w timeout -k 10 120 python tools/small_batch_probe.py $S > $out/w${w}_$i.txt 2>&1 || exit 1
    echo "W=$w run $i: $(grep n= $out/w${w}_$i.txt | tr '\n' ' ')"
  done
done
