#!/bin/bash
# GPU box: sequential-draw sampler vs the one-level Rao-Sandelius kernel below 65,536 sockets
# (LDPC_SEQ_MIN_E override of build_variants/seqenv.so; timing only).
set -u
export HSA_ENABLE_IPC_MODE_LEGACY=0
for spec in "1000 65536" "4000 32768" "10000 16384" "20000 16384"; do
  set -- $spec
  for m in 65536 1024; do
    echo -n "seq_min=$m "
    LDPC_SEQ_MIN_E=$m LDPC_LIB_PATH=build_variants/seqenv.so timeout -k 10 200 python scripts/diag/sampler_launch.py $1 $2 2 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
  done
done
