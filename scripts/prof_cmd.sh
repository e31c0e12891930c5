#!/bin/bash
# GPU box: kernel trace + PMC passes of one command, per-kernel summary.
#   TAG=r04x KREGEX=bp_loc ./scripts/prof_cmd.sh python3 scripts/kbench_mc.py cfg3 0.07
# (the command must be the program itself: python3 ..., never a shell or env wrapper)
set -u
TAG=${TAG:-x}; KREGEX=${KREGEX:-.}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- "$@" > $OUT/trace.log 2>&1 || { echo "trace rc=$?"; tail -5 $OUT/trace.log; exit 1; }
echo "trace ok"; tail -3 $OUT/trace.log
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $grp --kernel-include-regex "$KREGEX" -f csv -d $OUT/pmc$i -o run -- "$@" > $OUT/pmc$i.log 2>&1
  rc=$?
  echo "pmc pass $i ($grp) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/pmc$i.log; [ $rc -ge 124 ] && exit $rc; fi
done <<GROUPS
${PMC_GROUPS:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA}
GROUPS
python3 scripts/pmc_kernels.py $OUT > $OUT/pmc_kernels.txt 2>&1; cat $OUT/pmc_kernels.txt
find $OUT/trace -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \; 2>/dev/null
cut -c1-150 $OUT/kernel_stats.csv 2>/dev/null | head -8
exit 0
