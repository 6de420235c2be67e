# var-kernel iteration: parity + gather A/B (usage: bash tools/gpu_r03d.sh <tag>)
set -o pipefail
tag=${1:-r03d}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_glds_var.py tests/test_dispatch_fuzz.py -x -q --timeout 500 --timeout-method thread -m gpu > $out/tests.log 2>&1; rc=$?
echo tests-rc=$rc; tail -2 $out/tests.log; [ $rc -eq 0 ] || exit 1
bash tools/gpu_gather_ab.sh $tag/gather_ab || exit 1
export TMPDIR=/tmp
R=$(pwd)
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$out/prof_gather -o trace -- \
    python3 $R/bench.py --workload gather --steps 5 --warmup 1 > $R/$out/prof_gather.log 2>&1) || exit 1
echo prof-done
