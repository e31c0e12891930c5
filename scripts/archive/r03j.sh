#!/bin/bash
# GPU box: sequential-draw sampler after the wave-level round sync -- bit-exact sampler /
# ensemble tests, then sampler and ensemble-MC timing at configs[4]'s n = 64,800.
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -k "sample or ensemble or cfg5" > gpurun_out/r03j_samp_tests.log 2>&1
rc=$?; echo "sampler pytest rc=$rc"; tail -3 gpurun_out/r03j_samp_tests.log; grep -E "^FAILED|Error" gpurun_out/r03j_samp_tests.log | head -5; [ $rc -ne 0 ] && exit $rc
for G in 4096 16384; do
  timeout -k 10 200 python scripts/diag/sampler_launch.py 64800 $G 2 2>&1 | grep -v amdgpu.ids || exit 1
done
timeout -k 10 200 python scripts/diag/sampler_launch.py 30000 16384 2 2>&1 | grep -v amdgpu.ids || exit 1
for B in 16384 65536; do
  timeout -k 10 300 python scripts/diag/ens_time.py 0.42 $B 2>&1 | grep -v amdgpu.ids || exit 1
done
