# Merkle level probe, A/B of the in-tree library against a variant build given as $2
# (both in one box session, alternating): bash tools/gpu_merkle_ab.sh <out> <variant.so>
set -o pipefail
out=gpurun_out/${1:-merkle_ab}
mkdir -p $out
for r in 1 2; do
  timeout -k 10 120 python tools/merkle_probe.py > $out/base$r.txt 2>&1 || exit 1
  MERKLE_PROBE_LIB=$2 timeout -k 10 120 python tools/merkle_probe.py > $out/variant$r.txt 2>&1 || exit 1
  grep "level of" $out/base$r.txt $out/variant$r.txt
done
