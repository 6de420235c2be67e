# Pipelined staging in the wide-multi kernels (kernels.h multi_stage_hash_pipe): all GPU
# tests, then A/B against whole-block staging (STORMCK_STAGE_PIPE=0): c5 batch + commit
# forest, the 1M-leaf commit, and kernel stats of the c5 runs.
set -o pipefail
out=gpurun_out/${1:-pipe}
mkdir -p $out
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1 && echo tests-ok && tail -1 $out/tests.log || { echo tests-failed; tail -30 $out/tests.log; exit 1; }
for i in 1 2; do
  STORMCK_STAGE_PIPE=0 timeout -k 10 120 python bench.py --workload c5 --steps 300 --warmup 10 --no-cpu > $out/whole$i.log 2>&1 || exit 1
  echo "whole $i: $(grep -o '"batch_us": [0-9.]*' $out/whole$i.log) $(grep -o '"commit_forest_us": [0-9.]*' $out/whole$i.log) $(grep -o '"root_check": "[^"]*' $out/whole$i.log)"
  timeout -k 10 120 python bench.py --workload c5 --steps 300 --warmup 10 --no-cpu > $out/pipe$i.log 2>&1 || exit 1
  echo "pipe  $i: $(grep -o '"batch_us": [0-9.]*' $out/pipe$i.log) $(grep -o '"commit_forest_us": [0-9.]*' $out/pipe$i.log) $(grep -o '"root_check": "[^"]*' $out/pipe$i.log)"
done
timeout -k 10 120 python bench.py --workload c5 --c5-mix storm --steps 300 --warmup 10 --no-cpu > $out/pipe_storm.log 2>&1 && echo "storm mix: $(grep -o '"batch_us": [0-9.]*' $out/pipe_storm.log) $(grep -o '"commit_forest_us": [0-9.]*' $out/pipe_storm.log) $(grep -o '"root_check": "[^"]*' $out/pipe_storm.log)" &&
timeout -k 10 200 python bench.py --workload commit --steps 30 --warmup 2 --no-cpu > $out/commit.log 2>&1 && echo "commit 1M: $(grep -o '"ms_per_step": [0-9.]*' $out/commit.log) $(grep -o '"root_check": "[^"]*' $out/commit.log)" &&
(cd /tmp && STORMCK_STAGE_PIPE=0 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$out/prof_whole" -o w -- \
   python3 "$R/bench.py" --workload c5 --steps 200 --warmup 10 --no-cpu > "$R/$out/prof_whole.log" 2>&1) &&
(cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$out/prof_pipe" -o p -- \
   python3 "$R/bench.py" --workload c5 --steps 200 --warmup 10 --no-cpu > "$R/$out/prof_pipe.log" 2>&1) && echo prof-ok
