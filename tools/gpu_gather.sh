# Gathered per-block-length batches: parity (var/gather/fuzz tests), then the gather
# workload twice (storm's mixed lengths from shuffled slots; in slot order). The A/B of
# round 3 (profiles/r03_gather_rows/) also ran a row-stream kernel and a per-group length
# ranking; both lost and were removed.
set -o pipefail
out=gpurun_out/${1:-gather}
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "var or gather or fuzz or lens or mixed or c5 or verify" > $out/tests.log 2>&1; rc=$?
grep -E "passed|failed|error" $out/tests.log | tail -3; [ $rc -eq 0 ] || exit $rc
summ() { python -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; print('$2', d['value'], r['frac'], r['avg_launch_ms'], 'uniform same arena', r['uniform_same_arena']['frac'])"; }
timeout -k 10 300 python bench.py --workload gather --steps 5 --warmup 1 > $out/shuffled.log 2>&1 && summ $out/shuffled.log "mix shuffled" &&
timeout -k 10 300 python bench.py --workload gather --gather-order sequential --steps 5 --warmup 1 > $out/sequential.log 2>&1 && summ $out/sequential.log "mix sequential"
