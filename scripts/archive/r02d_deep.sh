#!/bin/bash
# GPU box: configs[3] deep FER point on one GPU (ring code n=20000, SPA 100 it, early stop),
# checkpointed every round under gpurun_out/ck_cfg4 (a rerun resumes).
set -u
mkdir -p gpurun_out/ck_cfg4
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 ${DEEP_SECONDS_LIMIT:-1140} python scripts/fer_sweep.py cfg4 --points ${POINT:-0.80} --trials 4000000000 \
  --seconds ${DEEP_SECONDS:-1050} --stop-errors 50 --batch 65536 --checkpoint-dir gpurun_out/ck_cfg4 > gpurun_out/deep.jsonl 2> gpurun_out/deep.err
rc=$?; echo "rc=$rc"; cat gpurun_out/deep.jsonl; tail -3 gpurun_out/deep.err; exit $rc
