# GPU tests + bench + E2E host-path rates (GPU box, repo root)
set -o pipefail
out=gpurun_out/${1:-chk}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $out/tests.log 2>&1 && echo tests-ok && tail -1 $out/tests.log &&
timeout -k 10 300 python bench.py > $out/bench.log 2>&1 && echo bench-ok && tail -1 $out/bench.log &&
timeout -k 10 400 python tools/e2e_bench.py > $out/e2e.log 2>&1 && echo e2e-ok && tail -1 $out/e2e.log
