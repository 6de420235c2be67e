# Two gloo ranks sharing one GPU, with Python stacks dumped every 30 s (GPU box, repo root).
set -o pipefail
mkdir -p gpurun_out/dist
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 tools/trace_run.py bench.py --gpus 2 --dist-backend gloo --blocks 2097152 --arena 1048576 --steps 3 --warmup 1 > gpurun_out/dist/gloo_diag.log 2>&1; rc=$?; tail -c 6000 gpurun_out/dist/gloo_diag.log; exit $rc
