#!/bin/bash
# GPU box, round 6: one call = a list of named steps, each under its own time limit; stops at the
# first step that crashes, faults or times out (a test failure, rc 1, does not stop the list).
#   scripts/r06_gpu.sh <step> [<step> ...]
# steps:
#   samp_tests   sampler parity tests (device == oracle, ensemble MC, peel)
#   samp_time    sampler timing, this build against build_variants/r5tree (round-5 build)
#   ens4185      finish the configs[4] eps=0.4185 point from the round-5 tree (its stream)
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
        run 600 r06_samp_time.log python scripts/diag/sampler_time.py --sizes ${SIZES:-10000:4096,64800:4096,64800:16384} \
            iib_project_ldpc_codes_amd/libldpc_mi355x.so build_variants/r5tree/iib_project_ldpc_codes_amd/libldpc_mi355x.so
        rc=$? ;;
    ens4185)
        (cd build_variants/r5tree && bash scripts/fer_campaign.sh ens 0.4185 21 200 ${ENS_SECS:-600} ens4185)
        rc=$?
        cp -r build_variants/r5tree/gpurun_out/. gpurun_out/r5tree/ 2>/dev/null
        echo "[ens4185] rc=$rc" ;;
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
