#!/bin/bash
# GPU box: kernel trace + PMC passes of one sampler launch ((3,6), n = N, G graphs).
#   TAG=r04s N=64800 G=4096 ./scripts/prof_sampler.sh
set -u
TAG=${TAG:-samp}; N=${N:-64800}; G=${G:-4096}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- python3 scripts/diag/sampler_launch.py $N $G 2 > $OUT/trace.log 2>&1 || exit $?
echo "trace ok"; tail -2 $OUT/trace.log
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "sample_" -f csv -d $OUT/pmc$i -o run -- python3 scripts/diag/sampler_launch.py $N $G 1 > $OUT/pmc$i.log 2>&1
  rc=$?
  echo "pmc pass $i ($grp) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/pmc$i.log; [ $rc -ge 124 ] && exit $rc; fi
done <<GROUPS
${PMC_GROUPS:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA
SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_SALU SQ_IFETCH SQ_INSTS_GDS}
GROUPS
python3 scripts/pmc_kernels.py $OUT
exit 0
