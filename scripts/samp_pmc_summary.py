"""Summarise the sampler profile of scripts/archive/r03k_samp_prof.sh (gpurun_out/prof_samp): kernel time
from the trace, PMC counters of the sample_seq_kernel launch, per graph and per attempt.
    python scripts/samp_pmc_summary.py gpurun_out/prof_samp G > profiles/<tag>_sampler_pmc.json"""
import collections
import csv
import glob
import json
import os
import sys

d = sys.argv[1]
G = int(sys.argv[2])
out = {"graphs_per_launch": G}
for f in glob.glob(os.path.join(d, "trace", "*kernel_stats.csv")):
    for r in csv.DictReader(open(f)):
        if "sample_seq" in r["Name"]:
            out["kernel"] = r["Name"]
            out["avg_ms"] = float(r["AverageNs"]) / 1e6
            out["calls"] = int(r["Calls"])
acc = collections.defaultdict(float)
for f in sorted(glob.glob(os.path.join(d, "pmc*", "*counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        if "sample_seq" in r.get("Kernel_Name", "sample_seq"):
            acc[r["Counter_Name"]] += float(r["Counter_Value"])
out["counters"] = dict(acc)
out["per_graph"] = {k: v / G for k, v in acc.items() if k.startswith("SQ_INSTS")}
if "avg_ms" in out:
    out["graphs_per_s"] = G / (out["avg_ms"] / 1e3)
print(json.dumps(out, indent=1))
