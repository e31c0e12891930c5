#!/bin/bash
# Build experimental variants of libldpc_mi355x.so into build_variants/<name>.so
set -e
cd "$(dirname "$0")/.."
mkdir -p build_variants
build() {
  name=$1; shift
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Iinclude -Iiib_project_ldpc_codes_amd/csrc "$@" \
    -shared iib_project_ldpc_codes_amd/csrc/ldpc_kernels.hip iib_project_ldpc_codes_amd/csrc/sampler.hip iib_project_ldpc_codes_amd/csrc/peel.hip iib_project_ldpc_codes_amd/csrc/capi.cpp iib_project_ldpc_codes_amd/csrc/mc_run.cpp iib_project_ldpc_codes_amd/csrc/loc_layout.cpp -ldl \
    -Wl,--version-script=iib_project_ldpc_codes_amd/csrc/exports.map -Wl,-Bsymbolic -o build_variants/$name.so &
}
build v0
for spec in ${VARIANTS:-}; do name=${spec%%:*}; flags=${spec#*:}; build $name ${flags//,/ }; done
wait
ls -la build_variants
