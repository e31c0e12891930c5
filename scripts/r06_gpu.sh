#!/bin/bash
# GPU box, round 6: one call = a list of named steps, each under its own time limit; stops at the
# first step that crashes, faults or times out (a test failure, rc 1, does not stop the list).
#   scripts/r06_gpu.sh <step> [<step> ...]
# steps:
#   samp_tests   sampler parity tests (device == oracle, ensemble MC, peel)
#   samp_time    sampler timing, this build against $LIBS (default build_variants/r05.so, the round-5 build)
#   samp_stats   search-pass counters of a -DLDPC_SEQ_STATS=1 build (build_variants/stats.so)
#   samp_prof    rocprofv3 kernel trace + PMC passes of one sampler launch (scripts/prof_sampler.sh)
#   dropin       drop-in message_passing tests + per-call rates (bench.dropin_*_rates)
#   hprof        headline decode: rocprofv3 trace of the bench command + PMC passes (scripts/profile.sh)
#   valu         VALU issue-price probe (build_diag/valu_rate, scripts/diag/valu_rate.hip)
#   gputests     the whole -m gpu suite
#   bench        bench.py (default arguments)
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
ROOT=$(pwd)
run() {  # run <seconds> <log> <cmd...>
    local t=$1 log=$2; shift 2
    timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1
    local rc=$?
    echo "[$log] rc=$rc"; tail -${TAIL:-12} "gpurun_out/$log"
    return $rc
}
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
for s in "$@"; do
    case $s in
    samp_tests)
        run 900 r06_samp_tests.log $PYT tests/test_gpu_parity.py::test_device_sampler_matches_oracle \
            tests/test_gpu_parity.py::test_device_irregular_sampler_matches_oracle \
            tests/test_gpu_parity.py::test_ensemble_mc_matches_oracle tests/test_gpu_peel.py \
            tests/test_gpu_fullsize.py::test_cfg5_ensemble_mc_n64800_vs_oracle
        rc=$? ;;
    samp_time)
        run 600 r06_samp_time.log python scripts/diag/sampler_time.py --sizes ${SIZES:-64800:4096,64800:16384} \
            iib_project_ldpc_codes_amd/libldpc_mi355x.so ${LIBS:-build_variants/r05.so}
        rc=$? ;;
    samp_stats)
        LDPC_LIB_PATH=build_variants/stats.so run 300 r06_samp_stats.log python scripts/diag/seq_stats.py ${N:-64800} ${G:-4096}
        rc=$? ;;
    samp_stats16k)
        LDPC_LIB_PATH=build_variants/stats.so run 300 r06_samp_stats16k.log python scripts/diag/seq_stats.py 64800 16384
        rc=$? ;;
    ens_time)
        run 600 r06_ens_time.log bash -c "python scripts/diag/ens_time.py 0.42 16384 && python scripts/diag/ens_time.py 0.42 65536"
        rc=$? ;;
    samp_prof)
        TAG=${TAG:-r06s} N=${N:-64800} G=${G:-4096} run 900 r06_samp_prof.log bash scripts/prof_sampler.sh
        rc=$? ;;
    dropin)
        run 600 r06_dropin.log $PYT tests/test_gpu_parity.py -k dropin
        rc=$?
        if [ $rc -eq 0 ]; then
            run 300 r06_dropin_time.log python -c "import json, bench; print(json.dumps({'gpu': bench.dropin_gpu_rates(2.0), 'ref': bench.dropin_reference_rates(2.0)}, indent=1))"
            rc=$?
        fi ;;
    hprof)
        PMC_GROUPS="FETCH_SIZE
WRITE_SIZE
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS
SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE GRBM_COUNT
SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_INSTS_SALU
SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_BRANCH" \
        TAG=${HTAG:-r06h} KREGEX=bp_loc run 900 r06_hprof.log bash scripts/profile.sh
        rc=$? ;;
    valu)
        run 300 r06_valu_rate.jsonl ./build_diag/valu_rate
        rc=$? ;;
    gputests)
        run 1500 r06_gputests.log $PYT tests -m gpu
        rc=$? ;;
    bench)
        run 600 r06_bench.log python bench.py ${BENCH_ARGS:-}
        rc=$? ;;
    *) echo "unknown step $s"; exit 2 ;;
    esac
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $s (rc=$rc)"; exit $rc; fi
done
