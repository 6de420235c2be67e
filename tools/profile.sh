#!/bin/bash
# rocprofv3 evidence for the dominant kernel (run on the GPU box via gpurun).
#   1. kernel trace + stats of the bench command (average duration of the dominant kernel)
#   2. separate PMC passes: FETCH_SIZE, WRITE_SIZE (one bench step of one 2M-block arena pass)
#   3. FETCH_SIZE calibration on the probe (read-peak kernel with a known byte count)
# Usage: tools/profile.sh <tag>
set -u
TAG=${1:-r01}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
# fresh plain processes first (the placement spread the line is drawn from), then the
# profiled one
for i in 1 2 3; do
  timeout -k 10 300 python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu > "$OUT/plain_$i.log" 2>&1 || { echo "plain $i failed rc=$?"; exit 1; }
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o trace -- \
    python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu > "$OUT/trace.log" 2>&1 || { echo "trace failed rc=$?"; exit 1; }
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o fetch -- \
    python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu --blocks 2097152 > "$OUT/fetch.log" 2>&1 || { echo "fetch failed rc=$?"; exit 1; }
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o write -- \
    python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu --blocks 2097152 > "$OUT/write.log" 2>&1 || { echo "write failed rc=$?"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/calib" -o calib -- \
    "$R/tools/probe" 8 1 > "$OUT/calib.log" 2>&1 || { echo "calib failed rc=$?"; exit 1; }
# the gather workload (storm's dirty slots: 4M storm-length blocks, shuffled slots):
# kernel trace, FETCH_SIZE / WRITE_SIZE of one step
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/gather_trace" -o trace -- \
    python3 "$R/bench.py" --workload gather --steps 5 --warmup 1 > "$OUT/gather_trace.log" 2>&1 || { echo "gather trace failed rc=$?"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/gather_fetch" -o fetch -- \
    python3 "$R/bench.py" --workload gather --steps 1 --warmup 0 > "$OUT/gather_fetch.log" 2>&1 || { echo "gather fetch failed rc=$?"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/gather_write" -o write -- \
    python3 "$R/bench.py" --workload gather --steps 1 --warmup 0 > "$OUT/gather_write.log" 2>&1 || { echo "gather write failed rc=$?"; exit 1; }
echo "profile done"
# then, in the build container: python tools/collect_profile.py <tag>
