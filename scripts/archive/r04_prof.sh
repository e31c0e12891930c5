#!/bin/bash
# Round-4 profiles on one MI355X: (1) the bench line + headline trace and PMC passes
# (scripts/profile.sh, bp_loc_kernel fixed-count SPA); (2) trace + PMC passes of one launch each
# of the early-stop decodes (SPA hard decisions, min-sum hard decisions) and of configs[2]'s
# fused BSC min-sum Monte-Carlo (scripts/diag/decode_launch.py).
#   TAG=r04a ./scripts/r04_prof.sh [bench|decode|all]
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG=${TAG:-r04a}
WHAT=${1:-all}
if [ "$WHAT" != decode ]; then
  timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.log 2>&1
  rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_$TAG.log; [ $rc -ne 0 ] && exit $rc
  TAG=$TAG KREGEX=bp_loc ./scripts/profile.sh > gpurun_out/profile_$TAG.log 2>&1 || exit $?
  echo "headline profile ok"
fi
[ "$WHAT" = bench ] && exit 0
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for spec in "et:--algo spa --et 1 --post 0" "mset:--algo minsum --et 1 --post 0" "mc:--mc-bsc 0.07"; do
  name=${spec%%:*}; args=${spec#*:}
  OUT=gpurun_out/prof_${TAG}_$name; mkdir -p $OUT
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- python3 scripts/diag/decode_launch.py $args --warmup 2 --reps 3 --out $OUT/trace_stats.json > $OUT/trace.log 2>&1 || exit $?
  echo "$name trace ok"
  timeout -k 10 100 python3 scripts/diag/decode_launch.py $args --out $OUT/launch_stats.json > $OUT/launch.log 2>&1 || exit $?
  i=0
  while read -r grp; do
    [ -z "$grp" ] && continue
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex bp_loc -f csv -d $OUT/pmc$i -o run -- python3 scripts/diag/decode_launch.py $args > $OUT/pmc$i.log 2>&1
    rc=$?; echo "$name pmc pass $i rc=$rc"
    if [ $rc -ne 0 ]; then tail -3 $OUT/pmc$i.log; exit $rc; fi
  done <<GROUPS
FETCH_SIZE
WRITE_SIZE
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS
SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE GRBM_COUNT
SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_INSTS_SALU
SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_WAIT_INST_ANY SQ_INSTS_SALU
GROUPS
  python3 scripts/pmc_summary.py $OUT 65536 > $OUT/pmc_summary.txt 2>&1
done
echo done
