set -o pipefail
out=gpurun_out/r03b_tsan
mkdir -p $out
R=$(pwd)
TSAN_OPTIONS="halt_on_error=1:second_deadlock_stack=1:suppressions=$R/tests/sanitize/tsan.supp" timeout -k 10 600 tests/sanitize/build/host_paths_tsan > $out/tsan_full.txt 2>&1; echo rc=$?
