"""ML ("optimal") erasure decoding throughput on one MI355X, with
the CPU oracle (C restatement, one core) timed on the host beside it.

usage: python scripts/bench_ml.py [--cpu-seconds S]   (one JSON line per workload)
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from iib_project_ldpc_codes_amd import decoder  # noqa: E402
from iib_project_ldpc_codes_amd.graph import TannerGraph  # noqa: E402
from iib_project_ldpc_codes_amd.montecarlo import MonteCarlo  # noqa: E402

WORKLOADS = [  # n, eps, batch
    (100, 0.40, 65536),
    (1000, 0.40, 32768),
    (1000, 0.45, 32768),
    (2000, 0.45, 8192),
]


def cpu_rate(g, words, seconds):
    from oracle import oracle
    cptr, cvar, _, _ = g.to_csr()
    done, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        oracle.lib().oracle_ml_decode(g.n, g.m, oracle._p(cptr), oracle._p(cvar),
                                      oracle._p(np.ascontiguousarray(words[done % len(words)])),
                                      oracle._p(np.zeros(g.n, np.uint8)))
        done += 1
    el = time.perf_counter() - t0
    return {"value": done / el, "unit": "words/s", "cores": 1, "kind": "port",
            "sample": f"{done} words, oracle_ml_decode (gcc -O2) 1 core, {el:.1f} s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cpu-seconds", type=float, default=3.0)
    args = ap.parse_args()
    s = torch.cuda.current_stream()
    for n, eps, B in WORKLOADS:
        g = TannerGraph.random_regular(n, 3, 6, seed=1)
        words = decoder.channel_dev("bec", eps, 5, 0, n, B)
        out, uns = decoder.ml_decode_dev(g, words)
        torch.cuda.synchronize()
        times = []
        for _ in range(3):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            decoder.ml_decode_dev(g, words, out=out, unsolved=uns)
            b.record(s)
            torch.cuda.synchronize()
            times.append(a.elapsed_time(b))
        ms = min(times)
        u = uns.cpu().numpy()
        # fused Monte-Carlo (channel + BP + ML + counters), modes 2/5
        mc = MonteCarlo(g, "bec", eps, 50, seed=9, batch=B, optimal=True, message_passing=True)
        mc.run_batch(0, B)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        mc.run_batch(B, B)
        b.record(s)
        torch.cuda.synchronize()
        print(json.dumps({"workload": f"ML decode (3,6) n={n} eps={eps}", "batch": B,
                          "words_per_s": B / ms * 1e3, "ms": ms,
                          "mc_both_trials_per_s": B / a.elapsed_time(b) * 1e3,
                          "ml_fer": float((u > 0).mean()), "ml_ber": float(u.sum() / (B * n)),
                          "cpu_baseline": cpu_rate(g, words[:256].cpu().numpy(), args.cpu_seconds)}), flush=True)


if __name__ == "__main__":
    main()
