"""Headline code ((3,6) n = 10,000, 65,536 frames): launch time against the fixed iteration count
(intercept = per-codeword staging / epilogue, slope = one flooding iteration), and the early-stop
decode's time and iteration distribution, to split the early-stop path's cost.
    python scripts/diag/et_cost.py  ->  one JSON line per measurement"""
import json
import os
import sys

sys.path.insert(0, os.getcwd())
import numpy as np
import torch

from iib_project_ldpc_codes_amd import decoder
from iib_project_ldpc_codes_amd.graph import TannerGraph

g = TannerGraph.random_regular(10000, 3, 6, seed=1)
B = 65536
s = torch.cuda.current_stream()


def timed(llr, iters, algo, es, want_post=True):
    ts = []
    for _ in range(3):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        post, hard, its = decoder.bp_decode_dev(g, llr, iters, algo, 0.75 if algo == "minsum" else 1.0, es, stream=s,
                                                want_post=want_post)
        b.record(s)
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return min(ts), its


for sigma in (0.85, 0.70):
    llr = decoder.channel_dev("awgn", sigma, 2026, 0, g.n, B)
    for algo in ("spa", "minsum"):
        for iters in (1, 2, 5, 10, 20, 50):
            ms, _ = timed(llr, iters, algo, False)
            print(json.dumps({"sigma": sigma, "algo": algo, "es": False, "iters": iters, "ms": round(ms, 3),
                              "kernel": g.kernel_name() if hasattr(g, "kernel_name") else None}), flush=True)
        ms, its = timed(llr, 50, algo, True)
        it = its.cpu().numpy()
        print(json.dumps({"sigma": sigma, "algo": algo, "es": True, "iters": 50, "ms": round(ms, 3),
                          "mean_its": float(it.mean()), "p50": float(np.percentile(it, 50)),
                          "p99": float(np.percentile(it, 99)), "frac_50": float((it == 50).mean()),
                          # frames dealt round-robin to 512 / 256 persistent workgroups
                          "wg512_max_over_mean": float(it.reshape(-1, 512).sum(0).max() / it.reshape(-1, 512).sum(0).mean()),
                          "wg256_max_over_mean": float(it.reshape(-1, 256).sum(0).max() / it.reshape(-1, 256).sum(0).mean())}),
              flush=True)
        ms, its = timed(llr, 50, algo, True, want_post=False)
        print(json.dumps({"sigma": sigma, "algo": algo, "es": "hard_only", "iters": 50, "ms": round(ms, 3),
                          "mean_its": float(its.float().mean().item()),
                          "kernel": g.kernel_name(early_stop=True, hard_only=True)}), flush=True)
