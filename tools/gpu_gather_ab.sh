# gather workload A/B: slot order x length mix (what costs the var kernel its rate)
set -o pipefail
out=gpurun_out/${1:-gather_ab}
mkdir -p $out
for cfg in "shuffled 0" "sequential 0" "shuffled 32768" "sequential 32768"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --workload gather --gather-order $1 --gather-lens $2 --steps 5 --warmup 1 > $out/g_$1_$2.log 2>&1 || exit 1
  python -c "import json; d=json.loads(open('$out/g_$1_$2.log').read().strip().splitlines()[-1]); print('$1 $2', d['value'], d['roofline']['frac'], d['roofline']['avg_launch_ms'], 'uniform on this arena', d['roofline']['uniform_same_arena']['frac'])"
done
STORMCK_GATHER_ORDER=0 timeout -k 10 300 python bench.py --workload gather --steps 5 --warmup 1 > $out/g_noorder.log 2>&1 || exit 1
python -c "import json; d=json.loads(open('$out/g_noorder.log').read().strip().splitlines()[-1]); print('shuffled mix, no locality order', d['value'], d['roofline']['frac'], d['roofline']['avg_launch_ms'])"
STORMCK_GLDS_VAR=0 timeout -k 10 300 python bench.py --workload gather --steps 3 --warmup 1 > $out/g_quad.log 2>&1 || exit 1
python -c "import json; d=json.loads(open('$out/g_quad.log').read().strip().splitlines()[-1]); print('quad shuffled mix', d['value'], d['roofline']['frac'], d['roofline']['avg_launch_ms'])"
