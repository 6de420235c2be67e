# c3 bench line in several fresh processes on one box: the spread from the arena's
# HBM placement (each process allocates its own 128 GiB arena)
set -o pipefail
out=gpurun_out/${1:-spread}
mkdir -p $out
for i in 1 2 3 4 5; do
  timeout -k 10 200 python bench.py --no-cpu > $out/bench_$i.log 2>&1 || exit 1
  python -c "import json,sys; d=json.loads(open('$out/bench_$i.log').read().strip().splitlines()[-1]); r=d['roofline']; print($i, d['value'], r['frac'], r['avg_launch_ms'], r['measured_read_peak']['frac'] if r['measured_read_peak'] else None, d['root_check'])"
done
