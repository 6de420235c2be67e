#!/bin/bash
# SQ / LDS counter passes for the dominant kernel (one bench step, one arena pass).
# Each pass runs alone (rocprofv3 --pmc only; no trace domains). Usage: tools/profile_sq.sh <tag>
set -u
TAG=${1:-r01}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/sq_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
run() {  # name, counters...
    local name=$1; shift
    timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o "$name" -- \
        python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu --blocks 4194304 > "$OUT/$name.log" 2>&1
}
run waves SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU || { echo "waves pass failed rc=$?"; exit 1; }
run insts SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL GRBM_GUI_ACTIVE || { echo "insts pass failed rc=$?"; exit 1; }
echo "sq profile done"
