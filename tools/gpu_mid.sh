# 2-wave mid-batch dispatch: GPU tests, smoke, small-batch probe, bench
set -o pipefail
out=gpurun_out/${1:-mid}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $out/tests.log 2>&1 && echo tests-ok && tail -1 $out/tests.log &&
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 && echo smoke-ok && tail -1 $out/smoke.log &&
timeout -k 10 120 ./tools/probe_small 20 > $out/probe_small.txt 2>&1 && echo probe-ok &&
timeout -k 10 300 python bench.py > $out/bench.log 2>&1 && echo bench-ok && tail -1 $out/bench.log
