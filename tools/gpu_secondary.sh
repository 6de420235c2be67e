# The secondary workloads' bench lines (f1 commit, c5 mixed batch, f4 key tags)
set -o pipefail
out=gpurun_out/${1:-secondary}
mkdir -p $out
for w in commit c5 keytags; do
  timeout -k 10 240 python bench.py --workload $w > $out/bench_$w.log 2>&1 || exit 1
  tail -1 $out/bench_$w.log
done
