# Shader clock during the c3 kernel and its hash-free control (tools/clock_probe.hip):
# without and with the bench's per-pass regeneration, plain and under
# rocprofv3 --kernel-trace, alternating; then bench.py plain / traced / plain.
set -o pipefail
out=gpurun_out/${1:-clock}
mkdir -p $out
R=$(pwd)
export TMPDIR=/tmp
for i in 1 2 3 4 5; do
  if [ $((i % 2)) -eq 0 ]; then
    (cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$out/trace$i" -o t -- \
       "$R/tools/clock_probe" 4 1 > "$R/$out/run$i.txt" 2>&1) || exit 1
    echo "run $i traced: $(grep -h mean $out/run$i.txt | tr '\n' ' ')"
  else
    timeout -k 10 120 tools/clock_probe 4 1 > $out/run$i.txt 2>&1 || exit 1
    echo "run $i plain:  $(grep -h mean $out/run$i.txt | tr '\n' ' ')"
  fi
done
for i in 6 7 8; do
  if [ $i -eq 7 ]; then
    (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$out/trace$i" -o t -- \
      python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu > "$R/$out/bench$i.log" 2>&1) || exit 1
    echo "bench $i traced: $(grep -o '"frac": [0-9.]*' $out/bench$i.log | head -1) peak $(grep -o '"measured_read_peak": {"GB/s": [0-9.]*' $out/bench$i.log)"
  else
    timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu > $out/bench$i.log 2>&1 || exit 1
    echo "bench $i plain:  $(grep -o '"frac": [0-9.]*' $out/bench$i.log | head -1) peak $(grep -o '"measured_read_peak": {"GB/s": [0-9.]*' $out/bench$i.log)"
  fi
done
