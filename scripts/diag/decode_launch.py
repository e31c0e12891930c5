"""One soft decode launch (or a few) of the bench code ((3,6) n = 10,000, seed 1) for profiling a
bp_loc_kernel instantiation under rocprofv3: fixed-count / early stop, with / without posteriors,
sum-product / min-sum.  Writes the launch's iteration statistics for the issue model.
    python scripts/diag/decode_launch.py --algo spa --et 1 --post 0 [--batch 65536 --iters 50
        --sigma 0.85 --warmup 0 --reps 1 --out stats.json]"""
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
a = ap.parse_args()
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
