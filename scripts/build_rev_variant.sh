#!/bin/bash
# A variant library whose csrc/sampler.hip is taken from git revision REV (the other translation
# units are this tree's product objects: run `make` first):
#   scripts/build_rev_variant.sh <rev> <name> [-DFLAG=...]  -> build_variants/<name>.so
set -e
cd "$(dirname "$0")/.."
rev=$1; name=$2; shift 2
C=iib_project_ldpc_codes_amd/csrc
mkdir -p build_variants
git show "$rev:$C/sampler.hip" > $C/sampler_rev_$name.hip
trap 'rm -f $C/sampler_rev_$name.hip' EXIT
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Iinclude -I$C "$@" \
  -c $C/sampler_rev_$name.hip -o build_variants/sampler_$name.o
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC $C/build/ldpc_kernels.o build_variants/sampler_$name.o $C/build/peel.o \
  $C/build/capi.o $C/build/mc_run.o $C/build/loc_layout.o -Wl,--version-script=$C/exports.map -Wl,-Bsymbolic -ldl \
  -o build_variants/$name.so
ls -la build_variants/$name.so
