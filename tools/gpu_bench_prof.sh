# GPU tests + c3 bench + rocprofv3 kernel stats of the same bench command (GPU box, repo root)
set -o pipefail
out=gpurun_out/${1:-bp}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1 && echo tests-ok && tail -1 $out/tests.log &&
timeout -k 10 300 python bench.py > $out/bench.log 2>&1 && echo bench-ok && tail -1 $out/bench.log &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv -- python3 bench.py --no-cpu > $out/bench_under_rocprof.log 2>&1 && echo prof-ok
