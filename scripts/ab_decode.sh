#!/bin/bash
# GPU box: A/B timing of the early-stop and Monte-Carlo decode launches across library builds.
#   ./scripts/ab_decode.sh build_variants/x.so ...   (the in-tree library first)
set -u
mkdir -p gpurun_out
for lib in iib_project_ldpc_codes_amd/libldpc_mi355x.so "$@"; do
  for spec in "fixed:--algo spa --et 0 --post 1" "et:--algo spa --et 1 --post 0" "msfixed:--algo minsum --et 0 --post 1" "mset:--algo minsum --et 1 --post 0" "mc:--mc-bsc 0.07"; do
    name=${spec%%:*}; args=${spec#*:}
    out=$(LDPC_LIB_PATH=$lib timeout -k 10 120 python3 scripts/diag/decode_launch.py $args --warmup 2 --reps 5) || { echo "$lib $name failed"; exit 1; }
    python3 - "$lib" "$name" "$out" <<'PY'
import json, sys
lib, name, d = sys.argv[1], sys.argv[2], json.loads(sys.argv[3].strip().split("\n")[-1])
ms = min(d["ms"])
its = d.get("mean_its", d.get("iters"))
print(f"{lib.split('/')[-1]:22s} {name:8s} {ms:8.2f} ms  mean_its {its:6.2f}  {d['batch'] / ms * 1e3 / 1e6:6.3f} M cw/s  "
      f"{d['batch'] * its / ms * 1e3 / 1e6:7.1f} M cw-it/s", flush=True)
PY
  done
done
