# round 3: the gathered / per-block-length LDS-DMA kernel (parity, fuzz, bench + rocprof),
# and the storm-side commit binding on the GPU. Usage: bash tools/gpu_r03b.sh <tag>
set -o pipefail
tag=${1:-r03b}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 900 python -u -m pytest tests/test_glds_var.py tests/test_dispatch_fuzz.py tests/test_cache_commit.py tests/test_gpu_parity.py tests/test_ring_fault.py tests/test_commit.py tests/test_multi_device.py tests/test_sanitize.py \
    -x -v -s --timeout 600 --timeout-method thread -m gpu > $out/tests.log 2>&1; rc=$?
echo tests-rc=$rc; tail -3 $out/tests.log; [ $rc -eq 0 ] || exit 1
bash tools/gpu_gather_ab.sh $tag/gather_ab || exit 1
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$out/prof_gather -o trace -- \
    python3 $R/bench.py --workload gather --steps 5 --warmup 1 > $R/$out/prof_gather.log 2>&1) || exit 1
echo done
# small batches (31,808 B in 32 KiB slots): the 16-block ring against the quad kernel
timeout -k 10 120 python tools/small_batch_probe.py 1200 2048 2049 3072 4096 4097 6144 8192 > $out/small_wide16.txt 2>&1 || exit 1
cat $out/small_wide16.txt
STORMCK_WIDE16=0 timeout -k 10 120 python tools/small_batch_probe.py 2049 3072 4096 > $out/small_quad.txt 2>&1 || exit 1
cat $out/small_quad.txt
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$out/prof_small -o trace -- \
    python3 $R/tools/small_batch_probe.py 2049 4096 8192 > $R/$out/prof_small.log 2>&1) || exit 1
echo small-done
# TSan with the narrow suppressions (called_from_lib only): does the driver stay clean?
TSAN_OPTIONS="halt_on_error=0:second_deadlock_stack=1:suppressions=$R/tests/sanitize/tsan.supp" \
    timeout -k 10 600 tests/sanitize/build/host_paths_tsan > $out/tsan_narrow.txt 2>&1; echo tsan-narrow-rc=$?
grep -c "WARNING: ThreadSanitizer" $out/tsan_narrow.txt || true
