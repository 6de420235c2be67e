# Round 4 (after the -m gpu suite): where per-block-length batches should switch from the register quad kernel to
# k_xxh64_glds_var: 4M blocks (2M from 8 KiB) of one length L in L-byte slots, strided,
# lengths passed per block; shipped dispatch (var) against STORMCK_GLDS_VAR=0 (quad).
# Usage: bash tools/gpu_r04_small2.sh <tag>
set -o pipefail
out=gpurun_out/${1:-r04_small2}
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1; rc=$?
grep -E "passed|failed|error" $out/tests.log | tail -3; [ $rc -eq 0 ] || exit $rc
run() {  # name, env..., -- bench args
  local name=$1; shift
  timeout -k 10 200 env "$@" > $out/$name.log 2>&1 || return 1
  python3 -c "
import json
d=json.loads([l for l in open('$out/$name.log') if l.startswith('{')][-1]); r=d['roofline']
print('$name', d['G_blocks_per_s'], 'Gblk/s', r['frac'], r['avg_launch_ms'], d['digest'])"
}
P="STORMCK_LIBRARY=tools/libstormck_probes.so"
for L in 1024 2048 4096 8192 16384; do  # var forced by STORMCK_VAR_MIN_LEN=0
  n=4194304; [ $L -ge 8192 ] && n=2097152
  B="python bench.py --workload gather --steps 5 --warmup 1 --gather-blocks $n --gather-slot $L --gather-lens-set $L --gather-order strided"
  run var_L${L} $P STORMCK_VAR_MIN_LEN=0 $B || exit 1
  run quad_L${L} $P STORMCK_GLDS_VAR=0 $B || exit 1
done
# the shipped dispatch with the length bound, on the `-tags test` mix (quad expected)
for mode in strided shuffled; do
  run product_${mode} X=1 python bench.py --workload gather --steps 5 --warmup 1 --gather-blocks 1048576 \
      --gather-slot 1024 --gather-lens-set 256,536,728 --gather-order $mode || exit 1
done
