# Round 4, sixth GPU session: gather A/B of contiguous group runs per persistent workgroup
# (probe build, STORMCK_GATHER_CONTIG=1) against every G-th group (shipped), 3 fresh
# processes per side, alternating; digests must match.
# Usage: bash tools/gpu_r04_sixth.sh <tag>
set -o pipefail
out=gpurun_out/${1:-r04_sixth}
mkdir -p $out
for i in 1 2 3; do
  for c in 0 1; do
    STORMCK_LIBRARY=tools/libstormck_probes.so STORMCK_GATHER_CONTIG=$c timeout -k 10 200 python bench.py \
        --workload gather --steps 5 --warmup 1 > $out/gather_contig${c}_$i.log 2>&1 || exit 1
    python3 -c "
import json
d=json.loads([l for l in open('$out/gather_contig${c}_$i.log') if l.startswith('{')][-1]); r=d['roofline']
print('contig=$c run $i', r['frac'], r['avg_launch_ms'], r['uniform_same_arena']['frac'], d['digest'])"
  done
done
