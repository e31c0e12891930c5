#!/bin/bash
# GPU box: round-end sequence at HEAD (tests, smoke, bench, torchrun bench) then sampler timing
# at n = 10^4 / 64,800 with the lowered sequential threshold.
set -u
bash scripts/gpu_round.sh || exit $?
export HSA_ENABLE_IPC_MODE_LEGACY=0
for spec in "10000 16384" "64800 16384"; do
  set -- $spec
  timeout -k 10 200 python scripts/diag/sampler_launch.py $1 $2 2 2>&1 | grep -v amdgpu.ids || exit 1
done
bash scripts/r03k_samp_prof.sh
