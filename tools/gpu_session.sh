#!/bin/bash
# One GPU session on the MI355X box (the one runner; it replaces the per-session scripts of
# rounds 1-4, whose logs stay under profiles/):
#
#   gpurun -- 'bash tools/gpu_session.sh <tag> <step> [<step> ...]'
#
# Output goes to gpurun_out/<tag>/. Each step runs under its own time limit, and the
# session stops at the first step that fails (a fault, an abort or a timeout ends it: no
# retries). Steps:
#   tests                  every -m gpu test
#   tests:<file>[,<file>]  the -m gpu tests of those files
#   smoke                  __graft_entry__.smoke()
#   bench                  the default bench line (c3, BASELINE metric)
#   batch_e2e commit_e2e gather c5 commit keytags
#                          bench.py --workload <step> --steps 7
#   inproc                 bench.py --in-process at N = 1 on c4 (all 64M blocks, one device):
#                          the strong-scaling N = 1 point, through stormck_merkle_root_multi
#   overhead               tools/route_overhead: the routed calls' fixed cost in C
#   placement              8 fresh plain c3 processes (bench.py --steps 5 --no-cpu): the spread
#                          of the line's frac with where each arena lands in HBM
#   prof                   tools/profile.sh <tag>: fresh plain c3 processes, the bench under
#                          rocprofv3 --kernel-trace --stats, separate FETCH_SIZE / WRITE_SIZE
#                          passes and their calibration, the gather workload likewise
#                          (then, in the build container: python tools/collect_profile.py <tag>)
set -o pipefail
tag=${1:?usage: gpu_session.sh <tag> <step>...}
shift
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
PYTEST=(python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread)
for step in "$@"; do
    echo "== $step $(date +%T)"
    case $step in
        tests)
            timeout -k 10 1500 "${PYTEST[@]}" tests > "$out/tests.log" 2>&1; rc=$?
            grep -E "passed|failed|error" "$out/tests.log" | tail -3 ;;
        tests:*)
            files=${step#tests:}
            name=$(echo "$files" | tr ',/' '__')
            timeout -k 10 900 "${PYTEST[@]}" ${files//,/ } > "$out/tests_$name.log" 2>&1; rc=$?
            grep -E "passed|failed|error" "$out/tests_$name.log" | tail -3 ;;
        smoke)
            timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1; rc=$?
            tail -1 "$out/smoke.log" ;;
        bench)
            timeout -k 10 400 python bench.py > "$out/bench.log" 2>&1; rc=$?
            tail -c 400 "$out/bench.log"; echo ;;
        batch_e2e|commit_e2e|gather|c5|commit|keytags)
            timeout -k 10 900 python bench.py --workload "$step" --steps 7 > "$out/$step.log" 2>&1; rc=$?
            tail -c 300 "$out/$step.log"; echo ;;
        inproc)
            timeout -k 10 600 python bench.py --in-process --gpus 1 --total-blocks 67108864 --steps 3 --warmup 1 \
                --no-cpu > "$out/inproc.log" 2>&1; rc=$?
            tail -c 400 "$out/inproc.log"; echo ;;
        overhead)
            timeout -k 10 300 ./tools/route_overhead > "$out/route_overhead.log" 2>&1; rc=$?
            grep -E "commit|batch" "$out/route_overhead.log" | head -6 ;;
        placement)
            rc=0
            for i in 1 2 3 4 5 6 7 8; do
                timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu > "$out/placement_$i.log" 2>&1 || { rc=$?; break; }
                python tools/placement_summary.py "$out/placement_$i.log" | tee -a "$out/placement.jsonl"
            done ;;
        prof)
            timeout -k 10 1100 bash tools/profile.sh "$tag" > "$out/prof.log" 2>&1; rc=$?
            tail -3 "$out/prof.log" ;;
        *)
            echo "unknown step $step"; rc=2 ;;
    esac
    if [ "$rc" -ne 0 ]; then
        echo "step $step failed: $rc"
        exit "$rc"
    fi
done
echo "== done $(date +%T)"
