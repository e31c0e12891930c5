#!/bin/bash
# GPU box: one FER campaign point (scripts/fer_sweep.py) to STOP frame errors (the reference's
# stop rule, parallel_simulator.py:198) or SECONDS, checkpointed every round under
# gpurun_out/ck_<TAG> (seeded from ck_in/<TAG> when present, so a cut-off run resumes).
#   scripts/fer_campaign.sh <cfg3|cfg4|ens> <point> <seed> <stop> <seconds> <tag>
set -u
CFG=$1; PT=$2; SEED=$3; STOP=$4; SECS=$5; TAG=$6
mkdir -p gpurun_out/ck_$TAG
[ -d ck_in/$TAG ] && cp -n ck_in/$TAG/*.json gpurun_out/ck_$TAG/ 2>/dev/null
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 $((SECS + 150)) python scripts/fer_sweep.py $CFG --points $PT --seed $SEED --trials 100000000000 \
  --seconds $SECS --stop-errors $STOP --batch 65536 --checkpoint-dir gpurun_out/ck_$TAG >> gpurun_out/fer_$TAG.jsonl 2> gpurun_out/fer_$TAG.err
rc=$?; echo "rc=$rc"; tail -1 gpurun_out/fer_$TAG.jsonl; tail -3 gpurun_out/fer_$TAG.err; exit $rc
