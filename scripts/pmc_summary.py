"""Summarise rocprofv3 --pmc CSVs: one value per counter for the decode kernel dispatches."""
import csv, glob, json, sys
d = sys.argv[1]
vals = {}
dur = {}
for f in sorted(glob.glob(f"{d}/pmc*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Counter_Name"]
        vals[k] = vals.get(k, 0.0) + float(r["Counter_Value"])
        dur[k] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for k in sorted(vals):
    print(f"{k:28s} {vals[k]:20.1f}   dispatch_ns={dur[k]}")
json.dump(vals, open(f"{d}/pmc_summary.json", "w"), indent=1)
