# Round 4, ninth GPU session: the batch E2E table with the refit cost model, then where
# the gather path's per-byte loss comes from: the var kernel on storm's lengths and on one
# 32 KiB length, gathered (locality-ordered) and strided (no offsets), 2 fresh processes
# each, every line beside the uniform kernel on its own arena.
# Usage: bash tools/gpu_r04_ninth.sh <tag>
set -o pipefail
out=gpurun_out/${1:-r04_ninth}
mkdir -p $out
timeout -k 10 400 python bench.py --workload batch_e2e --steps 7 > $out/batch_e2e.log 2>&1 && tail -c 300 $out/batch_e2e.log || exit 1
for i in 1 2; do
  for mode in shuffled strided; do
    for L in 0 32768; do
      timeout -k 10 200 python bench.py --workload gather --steps 5 --warmup 1 --gather-order $mode --gather-lens $L \
          > $out/gather_${mode}_L${L}_$i.log 2>&1 || exit 1
      python3 -c "
import json
d=json.loads([l for l in open('$out/gather_${mode}_L${L}_$i.log') if l.startswith('{')][-1]); r=d['roofline']
print('$mode lens=$L run $i', r['frac'], r['avg_launch_ms'], r['uniform_same_arena']['frac'], d['digest'])"
    done
  done
done
