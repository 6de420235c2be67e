# Round 4, fifth GPU session: VMM arena diagnostics (fresh processes: 2 MiB chunks alone,
# then after a one-allocation VMM arena was freed), then the -m gpu suite.
# Usage: bash tools/gpu_r04_fifth.sh <tag>
set -o pipefail
out=gpurun_out/${1:-r04_fifth}
mkdir -p $out
timeout -k 10 120 python tools/vmm_probe.py 1:2097152 1:2097152 > $out/vmm_a.txt 2>&1; echo "vmm_a rc $?"; cat $out/vmm_a.txt
timeout -k 10 120 python tools/vmm_probe.py 1:0 1:2097152 1:1073741824 0:0 1:2097152 > $out/vmm_b.txt 2>&1; echo "vmm_b rc $?"; cat $out/vmm_b.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1; rc=$?
grep -E "passed|failed|error" $out/tests.log | tail -3
exit $rc
