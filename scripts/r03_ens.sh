#!/bin/bash
# GPU box: sampler phase ablation (60 fixed attempts per graph, 2 graphs per CU) then the
# configs[4] expurgated-ensemble FER points (n=64800 (3,6) BEC, 200 it, X=3), checkpointed
# under gpurun_out/ck_ens.
set -u
mkdir -p gpurun_out/ck_ens
export HSA_ENABLE_IPC_MODE_LEGACY=0
for v in fa l1 l1c sb1 nofy; do
  echo -n "$v: "; LDPC_LIB_PATH=build_variants/$v.so timeout -k 10 120 python scripts/diag/sampler_launch.py 64800 512 2 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
done
timeout -k 10 ${ENS_LIMIT:-1100} python scripts/fer_sweep.py ens --points ${ENS_POINTS:-0.425,0.42} --trials 4000000000 \
  --seconds ${ENS_SECONDS:-840} --stop-errors 200 --batch 16384 --checkpoint-dir gpurun_out/ck_ens > gpurun_out/ens_r03.jsonl 2> gpurun_out/ens_r03.err
rc=$?; echo "rc=$rc"; cat gpurun_out/ens_r03.jsonl; tail -3 gpurun_out/ens_r03.err; exit $rc
