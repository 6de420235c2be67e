# 1M-leaf f1 commit (bench --workload commit): k_commit_level_multi for its 875-block
# pointer level vs the register-quad level kernel (STORMCK_COMMIT_MULTI=0): whole-step
# times alternating, then the level kernels' own durations under rocprofv3.
set -o pipefail
out=gpurun_out/${1:-commit_ab}
mkdir -p $out
R=$(pwd)
export TMPDIR=/tmp
for i in 1 2 3; do
  STORMCK_COMMIT_MULTI=0 timeout -k 10 200 python bench.py --workload commit --steps 30 --warmup 2 --no-cpu > $out/quad$i.log 2>&1 || exit 1
  echo "quad  $i: $(grep -o '"ms_per_step": [0-9.]*' $out/quad$i.log) $(grep -o '"root_check": "[a-z]*' $out/quad$i.log)"
  timeout -k 10 200 python bench.py --workload commit --steps 30 --warmup 2 --no-cpu > $out/multi$i.log 2>&1 || exit 1
  echo "multi $i: $(grep -o '"ms_per_step": [0-9.]*' $out/multi$i.log) $(grep -o '"root_check": "[a-z]*' $out/multi$i.log)"
done &&
(cd /tmp && STORMCK_COMMIT_MULTI=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$out/prof_quad" -o q -- \
   python3 "$R/bench.py" --workload commit --steps 10 --warmup 2 --no-cpu > "$R/$out/prof_quad.log" 2>&1) &&
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$out/prof_multi" -o m -- \
   python3 "$R/bench.py" --workload commit --steps 10 --warmup 2 --no-cpu > "$R/$out/prof_multi.log" 2>&1) && echo prof-ok
