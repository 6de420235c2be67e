set -o pipefail
mkdir -p gpurun_out/var
for i in 1 2 3; do timeout -k 10 200 python bench.py --no-cpu > gpurun_out/var/b$i.log 2>&1 || exit 1; done
timeout -k 10 200 python bench.py --no-cpu --settle 5 > gpurun_out/var/s5.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --no-cpu --steps 20 > gpurun_out/var/k20.log 2>&1 || exit 1
sleep 20
timeout -k 10 200 python bench.py --no-cpu > gpurun_out/var/after_sleep.log 2>&1 || exit 1
rocm-smi --showtemp --showpower --showclocks > gpurun_out/var/smi.txt 2>&1 || true
echo done
