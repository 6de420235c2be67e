# N>1 code path rehearsed on one GPU (GPU box, repo root): RCCL at world size 1, and two
# ranks sharing the GPU over gloo. The 8-GPU RCCL run is the driver's.
set -o pipefail
mkdir -p gpurun_out/dist
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --force-dist --no-cpu > gpurun_out/dist/nccl_world1.log 2>&1 && echo nccl1-ok && tail -1 gpurun_out/dist/nccl_world1.log &&
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --dist-backend gloo --blocks 2097152 --arena 1048576 --steps 3 --warmup 1 > gpurun_out/dist/gloo_n2.log 2>&1 && echo gloo2-ok && tail -1 gpurun_out/dist/gloo_n2.log
