# f4 key tags: parity tests + bench + kernel stats (run on the GPU box from the repo root)
set -o pipefail
mkdir -p gpurun_out/keys
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "key" --timeout 120 --timeout-method thread > gpurun_out/keys/tests.log 2>&1 && echo tests-ok && tail -1 gpurun_out/keys/tests.log &&
timeout -k 10 200 python bench.py --workload keytags --no-cpu > gpurun_out/keys/bench.log 2>&1 && echo bench-ok && tail -1 gpurun_out/keys/bench.log &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/keys/prof -o run --output-format csv -- python3 bench.py --workload keytags --no-cpu > gpurun_out/keys/prof.log 2>&1 && echo prof-ok
