# 16 blocks per workgroup through a 2-slot ring (batches of 8-16 per CU) vs the quad kernel
# (STORMCK_NO_BPW16=1): parity tests, then uniform batches of 2,048-4,096 blocks alternating.
set -o pipefail
out=gpurun_out/${1:-bpw16}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_dispatch_fuzz.py tests/test_commit.py tests/test_full_size_gpu.py -k "ring or c5 or fuzz or commit" -m gpu -x -q --timeout 150 --timeout-method thread > $out/tests.log 2>&1 && echo "tests ok: $(tail -1 $out/tests.log)" || { echo tests-failed; tail -20 $out/tests.log; exit 1; }
for i in 1 2; do
  timeout -k 10 120 python tools/small_batch_probe.py 2048 2560 3072 4096 > $out/b16.$i.txt 2>&1 || exit 1
  STORMCK_NO_BPW16=1 timeout -k 10 120 python tools/small_batch_probe.py 2048 2560 3072 4096 > $out/quad.$i.txt 2>&1 || exit 1
  echo "run $i 16/wg: $(grep '^n=' $out/b16.$i.txt | tr '\n' ' ') | quad: $(grep '^n=' $out/quad.$i.txt | tr '\n' ' ')"
done
