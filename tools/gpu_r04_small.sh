# Round 4: per-block-length batches of storm's `-tags test` sizes (256 / 536 / 728 B in
# 1 KiB slots, storm_test.go:131-138): the shipped dispatch (k_xxh64_glds_var from 44
# blocks per CU, its tile estimate assuming 32 KiB blocks) against the register quad kernel
# (probe build, STORMCK_GLDS_VAR=0), strided and shuffled, 1M and 4M blocks.
# Usage: bash tools/gpu_r04_small.sh <tag>
set -o pipefail
out=gpurun_out/${1:-r04_small}
mkdir -p $out
run() {  # name, env..., -- bench args
  local name=$1; shift
  timeout -k 10 200 env "$@" > $out/$name.log 2>&1 || return 1
  python3 -c "
import json
d=json.loads([l for l in open('$out/$name.log') if l.startswith('{')][-1]); r=d['roofline']
print('$name', d['G_blocks_per_s'], 'Gblk/s', r['frac'], r['avg_launch_ms'], d['digest'])"
}
P="STORMCK_LIBRARY=tools/libstormck_probes.so"
for n in 1048576 4194304; do
  for mode in strided shuffled; do
    B="python bench.py --workload gather --steps 5 --warmup 1 --gather-blocks $n --gather-slot 1024 --gather-lens-set 256,536,728 --gather-order $mode"
    for i in 1 2; do
      run var_${mode}_${n}_$i X=1 $B || exit 1
      run quad_${mode}_${n}_$i $P STORMCK_GLDS_VAR=0 $B || exit 1
    done
  done
done
