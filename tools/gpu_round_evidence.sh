# Tests, bench, and the rocprofv3 evidence for the dominant kernel (GPU box, repo root):
# kernel trace + stats of the bench command, FETCH_SIZE / WRITE_SIZE passes, calibration.
set -o pipefail
tag=${1:-r01d}
out=gpurun_out/ev_$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1 && echo tests-ok && tail -1 $out/tests.log &&
timeout -k 10 300 python bench.py > $out/bench.log 2>&1 && echo bench-ok && tail -1 $out/bench.log &&
bash tools/profile.sh $tag > $out/profile.log 2>&1 && echo profile-ok
