#!/bin/bash
# GPU box: kernel-trace stats of the bench command + PMC passes (one counter group per pass).
#   TAG=r01 ./scripts/profile.sh
set -u
TAG=${TAG:-r01}
echo "${GIT_SHA:-unknown}" > gpurun_out/prof_$TAG.sha 2>/dev/null || true
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
BENCH="bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- python3 $BENCH > $OUT/trace_bench.log 2>&1 || exit $?
echo "trace ok"; tail -1 $OUT/trace_bench.log
PMC_BATCH=${PMC_BATCH:-65536}
PMCB="bench.py --steps 1 --warmup 0 --batch $PMC_BATCH --no-cpu-baseline --no-extras"
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "${KREGEX:-bp_lds}" -f csv -d $OUT/pmc$i -o run -- python3 $PMCB > $OUT/pmc$i.log 2>&1
  rc=$?
  echo "pmc pass $i ($grp) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/pmc$i.log; [ $rc -ge 124 ] && exit $rc; fi
done <<GROUPS
${PMC_GROUPS:-FETCH_SIZE
WRITE_SIZE
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS
SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE GRBM_COUNT
SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_INSTS_SALU}
GROUPS
python3 scripts/pmc_summary.py $OUT $PMC_BATCH > $OUT/pmc_summary.txt 2>&1; cat $OUT/pmc_summary.txt
exit 0
