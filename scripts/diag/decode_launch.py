"""One soft decode launch (or a few) of the bench code ((3,6) n = 10,000, seed 1) for profiling a
bp_loc_kernel instantiation under rocprofv3: fixed-count / early stop, with / without posteriors,
sum-product / min-sum; or (--mc-bsc P) one batch of configs[2]'s fused Monte-Carlo (BSC channel,
normalized min-sum alpha 0.75, early stop: scripts/fer_sweep.py cfg3).  Writes the launch's
iteration statistics for the issue model.
    python scripts/diag/decode_launch.py --algo spa --et 1 --post 0 [--batch 65536 --iters 50
        --sigma 0.85 --warmup 0 --reps 1 --out stats.json]
    python scripts/diag/decode_launch.py --mc-bsc 0.07 [--batch 65536 ...]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.getcwd())
import numpy as np
import torch

from iib_project_ldpc_codes_amd import decoder
from iib_project_ldpc_codes_amd.graph import TannerGraph

ap = argparse.ArgumentParser()
ap.add_argument("--algo", default="spa")
ap.add_argument("--et", type=int, default=0)
ap.add_argument("--post", type=int, default=1)
ap.add_argument("--batch", type=int, default=65536)
ap.add_argument("--iters", type=int, default=50)
ap.add_argument("--sigma", type=float, default=0.85)
ap.add_argument("--warmup", type=int, default=0)
ap.add_argument("--reps", type=int, default=1)
ap.add_argument("--out", default=None)
ap.add_argument("--mc-bsc", type=float, default=None)
a = ap.parse_args()
if a.mc_bsc is not None:
    from iib_project_ldpc_codes_amd.montecarlo import MonteCarlo
    g = TannerGraph.random_regular(10000, 3, 6, seed=1, distinct_columns=True)
    mc = MonteCarlo(g, "bsc", a.mc_bsc, a.iters, algo="minsum", alpha=0.75, early_stop=True, seed=11,
                    batch=a.batch)
    ts = []
    for r in range(a.warmup + a.reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        mc.run_batch(r * a.batch, a.batch)
        e1.record()
        torch.cuda.synchronize()
        if r >= a.warmup:
            ts.append(e0.elapsed_time(e1))
    c = mc.counters.cpu().numpy().astype(np.int64)
    out = {"mode": "mc_bsc_minsum_early_stop", "p": a.mc_bsc, "batch": a.batch, "iters": a.iters, "ms": ts,
           "kernel": g.kernel_name(), "trials": int(c[0]), "frame_errors": int(c[1]),
           "mean_its": float(c[3] / c[0]), "trials_per_s": a.batch / min(ts) * 1e3,
           "cw_it_per_s": a.batch * float(c[3] / c[0]) / min(ts) * 1e3}
    print(json.dumps(out), flush=True)
    if a.out:
        json.dump(out, open(a.out, "w"), indent=1)
    sys.exit(0)
g = TannerGraph.random_regular(10000, 3, 6, seed=1)
llr = decoder.channel_dev("awgn", a.sigma, 2026, 0, g.n, a.batch)
s = torch.cuda.current_stream()
alpha = 0.75 if a.algo == "minsum" else 1.0
ts = []
for r in range(a.warmup + a.reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    post, hard, its = decoder.bp_decode_dev(g, llr, a.iters, a.algo, alpha, bool(a.et), stream=s,
                                            want_post=bool(a.post))
    e1.record(s)
    torch.cuda.synchronize()
    if r >= a.warmup:
        ts.append(e0.elapsed_time(e1))
it = its.cpu().numpy().astype(np.int64)
stopped = it < a.iters if a.et else np.zeros_like(it, bool)
out = {"algo": a.algo, "early_stop": bool(a.et), "posteriors": bool(a.post), "batch": a.batch, "iters": a.iters,
       "sigma": a.sigma, "ms": ts, "kernel": g.kernel_name(early_stop=bool(a.et), hard_only=not a.post),
       "sum_its": int(it.sum()), "mean_its": float(it.mean()), "frac_stopped": float(stopped.mean()),
       # check phases run: stopped frames its + 1 (the last finds every check satisfied), others its;
       # variable phases: stopped frames its, others its - 1 (the last iteration forms posteriors)
       "check_phases": int((it + stopped).sum()), "variable_phases": int((it - (~stopped)).sum())}
print(json.dumps(out), flush=True)
if a.out:
    json.dump(out, open(a.out, "w"), indent=1)
