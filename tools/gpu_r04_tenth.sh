# Round 4, tenth GPU session: which part of the gathered form costs the 4-6 % (every
# block 32 KiB, 2 fresh processes each, alternating):
#   strided          no offsets (stormck_checksum_device with lens)
#   seq_noorder      sorted offsets, no locality-order pass (probe build, STORMCK_GATHER_ORDER=0)
#   seq_order        sorted offsets through the order pass (order = identity: writes in order)
#   shuffled         shuffled offsets through the order pass (scattered checksum writes)
# Usage: bash tools/gpu_r04_tenth.sh <tag>
set -o pipefail
out=gpurun_out/${1:-r04_tenth}
mkdir -p $out
run() {  # name, env..., -- bench args
  local name=$1; shift
  timeout -k 10 200 env "$@" > $out/$name.log 2>&1 || return 1
  python3 -c "
import json
d=json.loads([l for l in open('$out/$name.log') if l.startswith('{')][-1]); r=d['roofline']
print('$name', r['frac'], r['avg_launch_ms'], r['uniform_same_arena']['frac'], round(r['frac']/r['uniform_same_arena']['frac'],4), d['digest'])"
}
B="python bench.py --workload gather --steps 5 --warmup 1 --gather-lens 32768"
for i in 1 2; do
  run strided_$i X=1 $B --gather-order strided || exit 1
  run seq_noorder_$i STORMCK_LIBRARY=tools/libstormck_probes.so STORMCK_GATHER_ORDER=0 $B --gather-order sequential || exit 1
  run seq_order_$i X=1 $B --gather-order sequential || exit 1
  run shuffled_$i X=1 $B --gather-order shuffled || exit 1
done
