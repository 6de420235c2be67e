set -o pipefail
out=gpurun_out/wide1; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 120 ./tools/probe_small_old 20 > $out/probe_old.txt 2>&1 && echo old-ok &&
timeout -k 10 120 ./tools/probe_small 20 > $out/probe_new.txt 2>&1 && echo new-ok &&
timeout -k 10 120 ./tools/probe_small_old 20 > $out/probe_old2.txt 2>&1 && echo old2-ok &&
timeout -k 10 120 ./tools/probe_small 20 > $out/probe_new2.txt 2>&1 && echo new2-ok &&
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $out/tests.log 2>&1 && echo tests-ok && tail -1 $out/tests.log
