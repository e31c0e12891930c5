#!/bin/bash
# Phase ablation of the (3,6) n=1e4 decode, SPA and min-sum, fixed 50 iterations and early stop
# (hard decisions only), across build_variants/*.so (v0 = baseline, p1 = no check phase,
# p2 = no variable phase).
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for cfg in "ALGO=0 ET=0" "ALGO=1 ET=0" "ALGO=0 ET=1" "ALGO=1 ET=1"; do
  echo "== $cfg"
  env $cfg timeout -k 10 200 python scripts/kbench36.py build_variants/*.so || exit $?
done > gpurun_out/r03b_ablate.log 2>&1
rc=$?; cat gpurun_out/r03b_ablate.log; exit $rc
