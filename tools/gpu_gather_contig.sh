# gather: shuffled slots on a default vs a physically contiguous arena (TLB reach)
set -o pipefail
out=gpurun_out/${1:-gather_contig}
mkdir -p $out
for c in 0 1 0 1; do
  STORMCK_ALLOC_CONTIGUOUS=$c timeout -k 10 300 python bench.py --workload gather --steps 5 --warmup 1 > $out/g_c$c.log 2>&1 || exit 1
  python -c "import json; d=json.loads(open('$out/g_c$c.log').read().strip().splitlines()[-1]); print('contiguous=$c', d['value'], d['roofline']['frac'], d['roofline']['avg_launch_ms'], 'uniform', d['roofline']['uniform_same_arena']['frac'], d['config']['arena'])"
done
