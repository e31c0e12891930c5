#!/bin/bash
# GPU box: bench.py's distributed path with 2 ranks on the one GPU (gloo for the
# barrier / max-over-ranks collectives: two RCCL ranks cannot share a device), then RCCL with 1 rank.
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
LDPC_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/dist2.log 2>&1
rc=$?; echo "gloo x2 rc=$rc"; grep -o '"value": [0-9.]*\|"n_gpus": [0-9]*\|"ms_per_step": [0-9.]*' gpurun_out/dist2.log; [ $rc -ne 0 ] && { tail -20 gpurun_out/dist2.log; exit $rc; }
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29542 bench.py --gpus 1 --steps 3 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/dist1.log 2>&1
rc=$?; echo "rccl x1 rc=$rc"; grep -o '"value": [0-9.]*\|"n_gpus": [0-9]*' gpurun_out/dist1.log; exit $rc
