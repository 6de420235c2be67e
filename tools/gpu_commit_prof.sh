# f1 commit: parity tests, phase trace, kernel trace (run on the GPU box from the repo root)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_commit.py tests/test_abi.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/commit_tests.log 2>&1 && echo tests-ok &&
STORMCK_TRACE=1 timeout -k 10 300 python bench.py --workload commit --no-cpu --steps 5 > gpurun_out/commit_trace.log 2>&1 && echo trace-ok && tail -1 gpurun_out/commit_trace.log &&
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/commit_prof -o run -- python3 bench.py --workload commit --no-cpu --steps 5 > gpurun_out/commit_prof.log 2>&1 && echo prof-ok
