# Kernel durations of the c5 batch with and without k_xxh64_wide_multi (GPU box).
set -o pipefail
out=gpurun_out/multiprof
mkdir -p $out
export TMPDIR=/tmp
R=$(pwd)
cd /tmp
for m in 0 1; do
  STORMCK_WIDE_MULTI=$m timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$out/m$m -o t -- python3 $R/bench.py --workload c5 --steps 50 --no-cpu > $R/$out/m$m.log 2>&1 || exit 1
done
for m in 0 1; do echo "multi=$m"; cut -c1-200 $R/$out/m$m/t_kernel_stats.csv | head -6; done
