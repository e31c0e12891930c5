#!/bin/bash
# CPU-only sanitizer run: the oracle restatement and the C ABI's host code (graph validation,
# lane / irregular layout builders, the host-only debug entry points) built with
# -fsanitize=address,undefined, driven by the CPU test suites.  No GPU is touched (no HIP device
# here: the device entry points return LDPC_ENODEV before any device work).
#   ./scripts/sanitize.sh [pytest args]     -> log in results/sanitize_<date>.log
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
make -s -C "$ROOT/iib_project_ldpc_codes_amd/csrc" all asan
make -s -C "$ROOT/oracle" all asan
ASAN_RT=$(gcc -print-file-name=libasan.so)
UBSAN_RT=$(gcc -print-file-name=libubsan.so)
export LDPC_LIB_PATH="$ROOT/iib_project_ldpc_codes_amd/csrc/build/asan/libldpc_mi355x_asan.so"
export ORACLE_LIB_PATH="$ROOT/oracle/_build/asan/liboracle.so"
# leaks: the CPython interpreter and torch hold allocations until exit; every other error aborts
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:halt_on_error=1:detect_odr_violation=0
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
cd "$ROOT"
LD_PRELOAD="$ASAN_RT $UBSAN_RT" python -m pytest -q -p no:cacheprovider -m "not gpu" \
  tests/test_host.py tests/test_oracle_golden.py tests/test_ml_oracle.py tests/test_ensembles.py \
  tests/test_mc_plan.py tests/test_loc_layout.py "$@"
