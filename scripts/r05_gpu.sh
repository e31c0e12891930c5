#!/bin/bash
# Round-5 GPU-box steps; every GPU step under its own time limit, chained so that the first
# failure ends the call.
#   scripts/r05_gpu.sh <step> [<step> ...]
#   steps: parity   the new parity tests (peel overflow branch, ring code frames that never stop)
#          gputests the whole -m gpu suite
#          valu     scripts/diag/valu_rate (prebuilt in build_diag/) -> gpurun_out/valu_rate.jsonl
#          ldsidx   one bench launch under rocprofv3 --pmc SQ_LDS_IDX_ACTIVE (+ conflicts, clock)
#          bench    python bench.py (default flags) -> gpurun_out/bench_r05.log
#          prof     TAG=$TAG scripts/profile.sh on bp_loc (trace + PMC passes)
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG=${TAG:-r05a}
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
for step in "$@"; do
  case $step in
    parity)
      timeout -k 10 900 $PYT tests/test_gpu_peel.py "tests/test_gpu_fullsize.py::test_ring_cfg3_early_stop_posteriors_100it_vs_oracle" \
        > gpurun_out/parity_$TAG.log 2>&1 || { tail -40 gpurun_out/parity_$TAG.log; exit 1; }
      grep -E "passed|failed" gpurun_out/parity_$TAG.log | tail -3 ;;
    gputests)
      timeout -k 10 1000 $PYT -m gpu tests > gpurun_out/gputests_$TAG.log 2>&1 || { tail -40 gpurun_out/gputests_$TAG.log; exit 1; }
      tail -3 gpurun_out/gputests_$TAG.log ;;
    valu)
      timeout -k 10 120 ./build_diag/valu_rate > gpurun_out/valu_rate_$TAG.jsonl 2>&1 || { tail gpurun_out/valu_rate_$TAG.jsonl; exit 1; }
      cat gpurun_out/valu_rate_$TAG.jsonl ;;
    ldsidx)
      cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
      OUT=gpurun_out/prof_${TAG}_ldsidx
      mkdir -p $OUT
      timeout -s KILL 150 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
        --kernel-include-regex bp_loc -f csv -d $OUT/pmc1 -o run -- \
        python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-extras > $OUT/pmc1.log 2>&1 || { tail -5 $OUT/pmc1.log; exit 1; }
      python3 scripts/pmc_summary.py $OUT 65536 > $OUT/pmc_summary.txt 2>&1; cat $OUT/pmc_summary.txt ;;
    bench)
      timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_$TAG.log; exit 1; }
      tail -1 gpurun_out/bench_$TAG.log ;;
    prof)
      PMC_GROUPS="FETCH_SIZE
WRITE_SIZE
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS
SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE GRBM_COUNT
SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_INSTS_SALU
SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_BRANCH" \
        TAG=$TAG KREGEX=bp_loc ./scripts/profile.sh > gpurun_out/profile_$TAG.log 2>&1 || { tail -20 gpurun_out/profile_$TAG.log; exit 1; }
      tail -30 gpurun_out/profile_$TAG.log ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
  echo "step $step ok"
done
