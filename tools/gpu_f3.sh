# f3: the O_DIRECT read-verify test, then the E2E host-path tool (8 GiB)
set -o pipefail
out=gpurun_out/${1:-f3}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "read_verify" -x -v --timeout 250 --timeout-method thread > $out/tests.log 2>&1 && tail -3 $out/tests.log &&
timeout -k 10 400 python tools/e2e_bench.py --gib 8 > $out/e2e.txt 2>&1 && cat $out/e2e.txt
