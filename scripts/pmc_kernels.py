"""Per-kernel summary of rocprofv3 --pmc passes (every pmc*/ directory under <dir>).
usage: python scripts/pmc_kernels.py <prof_dir>   -> <prof_dir>/pmc_kernels.json"""
import csv
import glob
import json
import sys

d = sys.argv[1]
out = {}
for f in sorted(glob.glob(f"{d}/pmc*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        e = out.setdefault(k, {"counters": {}, "dispatches": {}})
        disp = r.get("Dispatch_Id", "0")
        e["dispatches"][disp] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        c = r["Counter_Name"]
        e["counters"][c] = e["counters"].get(c, 0.0) + float(r["Counter_Value"])
for k, e in out.items():
    print(k)
    for c, v in sorted(e["counters"].items()):
        print(f"   {c:26s} {v:20.1f}")
json.dump(out, open(f"{d}/pmc_kernels.json", "w"), indent=1)
