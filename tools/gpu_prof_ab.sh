# Is the bench under rocprofv3 slower because of the profiler or because it runs later?
# bench, bench under --kernel-trace, bench, bench under --kernel-trace, bench: one box.
set -o pipefail
out=gpurun_out/prof_ab
mkdir -p $out
export TMPDIR=/tmp
R=$(pwd)
for i in 1 2 3 4 5; do
  if [ $((i % 2)) -eq 0 ]; then
    (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$out/trace$i" -o t -- \
      python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu > "$R/$out/run$i.log" 2>&1) || exit 1
    echo "run $i (rocprofv3): $(grep -o '"frac": [0-9.]*' $out/run$i.log | head -1)"
  else
    timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu > $out/run$i.log 2>&1 || exit 1
    echo "run $i (plain):     $(grep -o '"frac": [0-9.]*' $out/run$i.log | head -1)"
  fi
done
