#!/bin/bash
# A variant library that differs from the product build only in csrc/ldpc_kernels.hip's flags:
#   scripts/build_kernel_variant.sh <name> [-DFLAG=...]  -> build_variants/<name>.so
# (links the product objects of the other translation units: run `make` first)
set -e
cd "$(dirname "$0")/.."
name=$1; shift
C=iib_project_ldpc_codes_amd/csrc
mkdir -p build_variants
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Iinclude -I$C "$@" \
  -c $C/ldpc_kernels.hip -o build_variants/kern_$name.o
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC build_variants/kern_$name.o $C/build/sampler.o $C/build/peel.o \
  $C/build/capi.o $C/build/mc_run.o $C/build/loc_layout.o -Wl,--version-script=$C/exports.map -Wl,-Bsymbolic -ldl \
  -o build_variants/$name.so
ls -la build_variants/$name.so
