# Round-end rehearsal on the GPU box: what the driver runs (pytest -m gpu, smoke, bench)
set -o pipefail
out=gpurun_out/${1:-final}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $out/tests.log 2>&1 && echo tests-ok && tail -1 $out/tests.log &&
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 && echo smoke-ok && tail -1 $out/smoke.log &&
timeout -k 10 300 python bench.py > $out/bench.log 2>&1 && echo bench-ok && tail -1 $out/bench.log
