# Placement A/B (round 3): fresh bench.py processes on one box, alternating the shipped
# skew shape (0) and the placement-robust shape (1: blocks v+8k, phases 3v), each with
# its arena as the process's first device allocation (hipMalloc via the library); then
# the same under rocprofv3 --kernel-trace. Usage: bash tools/gpu_placement.sh <tag> [runs]
set -o pipefail
tag=${1:-placement}
runs=${2:-4}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
R=$(pwd)
for i in $(seq 1 $runs); do
  for shape in 0 1; do
    STORMCK_SKEW_SHAPE=$shape timeout -k 10 200 python bench.py --no-cpu --steps 5 --warmup 1 > $out/plain_s${shape}_$i.log 2>&1 || exit 1
    python tools/placement_summary.py $out/plain_s${shape}_$i.log || exit 1
  done
done
for i in 1 2; do
  for shape in 0 1; do
    (cd /tmp && STORMCK_SKEW_SHAPE=$shape timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
        -d $R/$out/prof_s${shape}_$i -o trace -- python3 $R/bench.py --no-cpu --steps 5 --warmup 1 \
        > $R/$out/prof_s${shape}_$i.log 2>&1) || exit 1
    python tools/placement_summary.py $out/prof_s${shape}_$i.log $out/prof_s${shape}_$i || exit 1
  done
done
