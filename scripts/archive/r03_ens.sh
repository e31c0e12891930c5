#!/bin/bash
# GPU box: configs[4] expurgated-ensemble FER points (a fresh device-sampled (3,6) n = 64,800
# graph per trial, BEC, 200 iterations, expurgation X = 3; parallel_simulator_expurgated.py) to
# the reference's 200 frame errors, checkpointed every round under gpurun_out/ck_ens (copied
# from ck_in/ens when present, so a cut-off run resumes).
set -u
mkdir -p gpurun_out/ck_ens
[ -d ck_in/ens ] && cp -n ck_in/ens/*.json gpurun_out/ck_ens/ 2>/dev/null
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 ${ENS_LIMIT:-1100} python scripts/fer_sweep.py ens --points ${ENS_POINTS:-0.425,0.42} --trials 4000000000 \
  --seconds ${ENS_SECONDS:-900} --stop-errors 200 --batch 65536 --checkpoint-dir gpurun_out/ck_ens > gpurun_out/ens_r03.jsonl 2> gpurun_out/ens_r03.err
rc=$?; echo "rc=$rc"; cat gpurun_out/ens_r03.jsonl; tail -3 gpurun_out/ens_r03.err; exit $rc
