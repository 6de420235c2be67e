set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/t_gpu.log 2>&1 && echo tests-ok &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && echo smoke-ok &&
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 && echo bench-ok && tail -1 gpurun_out/bench.log
