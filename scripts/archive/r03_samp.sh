#!/bin/bash
# Sampler profile at n = 64,800: timing, kernel trace, PMC passes (one launch of 256 graphs).
set -u
mkdir -p gpurun_out/samp
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 120 python scripts/diag/sampler_launch.py 64800 256 3 2>&1 | grep -v amdgpu.ids
timeout -k 10 120 python scripts/diag/sampler_launch.py 10000 4096 2 2>&1 | grep -v amdgpu.ids
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex sample -f csv -d gpurun_out/samp/pmc$i -o run -- python3 scripts/diag/sampler_launch.py 64800 256 1 > gpurun_out/samp/pmc$i.log 2>&1
  rc=$?; echo "pmc pass $i rc=$rc"; [ $rc -ne 0 ] && { tail -3 gpurun_out/samp/pmc$i.log; exit $rc; }
done <<GROUPS
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS
GRBM_GUI_ACTIVE GRBM_COUNT
FETCH_SIZE
WRITE_SIZE
GROUPS
python3 scripts/pmc_summary.py gpurun_out/samp 256 2>&1 | tail -30
