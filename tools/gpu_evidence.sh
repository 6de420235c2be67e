# Round evidence on the GPU box: all GPU tests, smoke, bench, the rocprofv3 session
# (kernel trace + stats of the bench, FETCH_SIZE / WRITE_SIZE passes, calibration),
# and the filesystem probe. Usage: bash tools/gpu_evidence.sh <tag>
set -o pipefail
tag=${1:-r02}
out=gpurun_out/ev_$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 60 python tools/fs_probe.py > $out/fs_probe.txt 2>&1; cat $out/fs_probe.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread > $out/tests.log 2>&1 && echo tests-ok && tail -1 $out/tests.log &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 && echo smoke-ok && tail -1 $out/smoke.log &&
timeout -k 10 300 python bench.py > $out/bench.log 2>&1 && echo bench-ok && tail -1 $out/bench.log &&
bash tools/profile.sh $tag > $out/profile.log 2>&1 && echo profile-ok
