# secondary workloads (c5, f4 key tags) + kernel stats (run on the GPU box from the repo root)
set -o pipefail
mkdir -p gpurun_out/sec
export TMPDIR=/tmp
timeout -k 10 200 python bench.py --workload c5 --steps 50 > gpurun_out/sec/c5.log 2>&1 && echo c5-ok && tail -1 gpurun_out/sec/c5.log &&
timeout -k 10 200 python bench.py --workload keytags --no-cpu > gpurun_out/sec/keytags.log 2>&1 && echo keytags-ok && tail -1 gpurun_out/sec/keytags.log &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/sec/c5prof -o run -- python3 bench.py --workload c5 --steps 20 --no-cpu > gpurun_out/sec/c5prof.log 2>&1 && echo prof-ok
