#!/bin/bash
# GPU box: kernel-trace + PMC passes of the irregular (config-4 shape) generic kernel.
set -u
OUT=gpurun_out/prof_irr
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
CMD="scripts/kbench_irr.py iib_project_ldpc_codes_amd/libldpc_mi355x.so"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- python3 $CMD > $OUT/trace.log 2>&1 || exit $?
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $grp --kernel-include-regex bp_irr -f csv -d $OUT/pmc$i -o run -- python3 $CMD > $OUT/pmc$i.log 2>&1
  rc=$?; echo "pass $i ($grp) rc=$rc"; [ $rc -ge 124 ] && exit $rc
done <<GROUPS
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU
SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_FLAT SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU GRBM_GUI_ACTIVE
TCC_HIT_sum TCC_MISS_sum
FETCH_SIZE
GROUPS
python3 - <<PY
import csv, glob, collections
tot = collections.defaultdict(float); cnt = collections.Counter()
for f in glob.glob("$OUT/pmc*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        tot[r["Counter_Name"]] += float(r["Counter_Value"]); cnt[(r["Counter_Name"], r.get("Dispatch_Id", ""))] += 1
nd = {}
for (k, d) in cnt: nd[k] = nd.get(k, 0) + 1
for k in sorted(tot): print(f"{k:28s} {tot[k] / max(nd[k], 1):18.1f} per dispatch ({nd[k]} dispatches)")
PY
exit 0
