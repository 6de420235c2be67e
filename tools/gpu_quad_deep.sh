# mid-size batches: the one-wave, 4-deep quad workgroups (default up to 16 blocks per CU)
# against 256-thread workgroups (STORMCK_QUAD_SPREAD=0); parity first, then a rocprofv3
# kernel trace of the probe at 2,049 / 3,072 / 4,096 / 8,192 blocks.
set -o pipefail
out=gpurun_out/${1:-quad_deep}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_dispatch_fuzz.py tests/test_gpu_parity.py -m gpu -x -q --timeout 150 --timeout-method thread > $out/tests.log 2>&1 && echo "tests ok: $(tail -1 $out/tests.log)" || { echo tests-failed; tail -20 $out/tests.log; exit 1; }
S="1024 2048 2049 3072 4096 5120 8192"
for i in 1 2; do
  timeout -k 10 120 python tools/small_batch_probe.py $S > $out/spread.$i.txt 2>&1 || exit 1
  STORMCK_QUAD_SPREAD=0 timeout -k 10 120 python tools/small_batch_probe.py $S > $out/quad256.$i.txt 2>&1 || exit 1
  echo "run $i spread: $(grep '^n=' $out/spread.$i.txt | tr '\n' ' ') | 256-thread: $(grep '^n=' $out/quad256.$i.txt | tr '\n' ' ')"
done
R=$(pwd)
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$out/prof -o trace -- \
    python3 $R/tools/small_batch_probe.py 2049 3072 4096 8192 > $R/$out/prof.log 2>&1) || exit 1
echo prof-done
