# Round-end rehearsal plus the wide-multi size sweep: pytest -m gpu, smoke, bench,
# c5 (objectlist, blob mix), uniform batches of 1,200-2,560 blocks.
set -o pipefail
out=gpurun_out/${1:-final2}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $out/tests.log 2>&1 && echo tests-ok && tail -1 $out/tests.log &&
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 && echo smoke-ok && tail -1 $out/smoke.log &&
timeout -k 10 300 python bench.py > $out/bench.log 2>&1 && echo bench-ok && grep -o '"value": [0-9.]*\|"frac": [0-9.]*\|"root_check": "[^"]*' $out/bench.log | head -4 | tr '\n' ' ' && echo &&
timeout -k 10 120 python bench.py --workload c5 --steps 300 --warmup 10 --no-cpu > $out/c5.log 2>&1 &&
timeout -k 10 120 python bench.py --workload c5 --c5-mix storm --steps 300 --warmup 10 --no-cpu > $out/c5_storm.log 2>&1 &&
timeout -k 10 120 python tools/small_batch_probe.py 1200 1280 1600 2048 2560 > $out/sizes.txt 2>&1 &&
echo "c5 $(grep -o '"batch_us": [0-9.]*\|"commit_forest_us": [0-9.]*\|"root_check": "[^"]*' $out/c5.log | tr '\n' ' ') | storm $(grep -o '"batch_us": [0-9.]*\|"commit_forest_us": [0-9.]*' $out/c5_storm.log | tr '\n' ' ') | $(grep '^n=' $out/sizes.txt | tr '\n' ' ')"
