# Merkle level probe over the STORMCK_POINTER_RING modes given as arguments
set -o pipefail
out=gpurun_out/${1:-merkle_modes}; shift
mkdir -p $out
for mode in "$@"; do
  STORMCK_POINTER_RING=$mode timeout -k 10 120 python tools/merkle_probe.py > $out/mode$mode.txt 2>&1 || exit 1
  grep "level of" $out/mode$mode.txt
done
