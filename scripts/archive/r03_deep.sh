#!/bin/bash
# GPU box: configs[3] deep FER point (ring code n=20000, SPA 100 it, early stop, sigma 0.80) to the
# reference's 200 frame errors (parallel_simulator.py:198), resumed from the checkpoint in ck_in/
# (round 2's 50-error run, its trial range ended at the first uncounted trial), checkpointed
# every round under gpurun_out/ck_cfg4.
set -u
mkdir -p gpurun_out/ck_cfg4
[ -f gpurun_out/ck_cfg4/cfg4_p=0.8_seed=11_B=65536.json ] || cp ck_in/cfg4_p=0.8_seed=11_B=65536.json gpurun_out/ck_cfg4/
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 ${DEEP_SECONDS_LIMIT:-1130} python scripts/fer_sweep.py cfg4 --points 0.80 --trials 8000000000 \
  --seconds ${DEEP_SECONDS:-1020} --stop-errors 200 --batch 65536 --checkpoint-dir gpurun_out/ck_cfg4 > gpurun_out/deep_r03.jsonl 2> gpurun_out/deep_r03.err
rc=$?; echo "rc=$rc"; cat gpurun_out/deep_r03.jsonl; tail -3 gpurun_out/deep_r03.err; exit $rc
