#!/bin/bash
# GPU box: kernel trace + PMC passes of one sample_seq_kernel launch ((3,6) n = 64,800, 16,384 graphs).
set -u
mkdir -p gpurun_out/prof_samp
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
OUT=gpurun_out/prof_samp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- python3 scripts/diag/sampler_launch.py 64800 16384 1 > $OUT/trace.log 2>&1 || exit $?
echo trace ok; grep graphs $OUT/trace.log
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex sample_seq -f csv -d $OUT/pmc$i -o run -- python3 scripts/diag/sampler_launch.py 64800 16384 1 > $OUT/pmc$i.log 2>&1
  rc=$?; echo "pmc pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -3 $OUT/pmc$i.log; exit $rc; fi
done <<GROUPS
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU
SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_BRANCH GRBM_GUI_ACTIVE
GROUPS
find $OUT -name "*counter_collection.csv" | head
