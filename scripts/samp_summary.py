"""Sampler profile summary -> profiles/<tag>_sampler_summary.json: kernel times (rocprofv3 trace),
PMC counters of the three sampler kernels of one launch (scripts/prof_sampler.sh), divided by the
search pass's round count from a -DLDPC_SEQ_STATS=1 build of the same stream
(scripts/diag/seq_stats.py output, same n / G / seed: the stream does not depend on the schedule,
so the round count of the stats build holds for the product build up to the schedule's waste).
    python scripts/samp_summary.py <prof_dir> <seq_stats.log> <G> <git> > profiles/<tag>_sampler_summary.json"""
import csv
import glob
import json
import os
import re
import sys

d, stats_log, G, git = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
times = {}
for f in glob.glob(os.path.join(d, "trace", "*kernel_stats.csv")):
    for r in csv.DictReader(open(f)):
        for k in ("sample_search_kernel", "sample_seq_kernel", "sample_var_side_kernel"):
            if k in r["Name"]:
                times[k] = float(r["AverageNs"]) / 1e6
pm = json.load(open(os.path.join(d, "pmc_kernels.json")))
c = next(iter(pm.values()))["counters"]
st = {}
for line in open(stats_log):
    m = re.match(r"\s+(\w+)\s+(\d+)$", line)
    if m:
        st[m.group(1)] = int(m.group(2))
R = st["rounds"]
xcd_cycles = c["GRBM_GUI_ACTIVE"] / 8  # GRBM_GUI_ACTIVE sums the 8 XCDs
out = {
    "what": f"sample_search_kernel + sample_seq_kernel + sample_var_side_kernel of one launch, (3,6) n = 64,800, "
            f"G = {G} graphs; PMC passes by scripts/prof_sampler.sh, rounds from the stats build (seq_stats.py)",
    "git": git,
    "kernel_avg_ms_trace": times,
    "graphs_per_s_search_trace": G / (times["sample_search_kernel"] / 1e3) if "sample_search_kernel" in times else None,
    "pmc_totals_1_launch": c,
    "stats_build": st,
    "rounds": R,
    "rounds_per_graph": R / G,
    "kept_slots_per_round": st["kept"] / R,
    "attempts_per_graph_search": st["attempts"] / G,
    "per_round": {k: c[f"SQ_INSTS_{k.upper()}"] / R for k in ("valu", "salu", "branch", "lds")},
    "valu_active_fraction": c["SQ_ACTIVE_INST_VALU"] * 4 / (1024 * xcd_cycles),
    "issue_active_any_fraction_per_simd": c["SQ_ACTIVE_INST_ANY"] * 4 / (1024 * xcd_cycles),
    "wait_any_fraction_of_wave_cycles": c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"],
    "waves_per_cu": 12.0,
    "waves_per_cu_note": "six attempts per CU (26.7 KB of LDS each: the 24.3 KB socket bitmap + ring, retry lists, "
                         "sync words), two waves per attempt",
    "formula": "VALU-active = SQ_ACTIVE_INST_VALU x 4 / 1024 SIMDs / (GRBM_GUI_ACTIVE / 8 XCDs); per_round = SQ_INSTS_* "
               "of the launch / search rounds (both waves of a round together)",
}
print(json.dumps(out, indent=1))
