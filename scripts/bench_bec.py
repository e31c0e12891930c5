"""BEC erasure-decoding throughput (message_passing.c semantics) on one MI355X,
with the reference's own C (oracle/_ref/message_passing.so, compiled from the
reference sources) timed on the host as the baseline.

usage: python scripts/bench_bec.py [--cpu-seconds S] | --mc | --ensemble
(LDPC_LIB_PATH=<other build>.so times another build of the library)
Prints one JSON line per workload.
"""
import argparse
import ctypes as ct
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

WORKLOADS = [
    # name, n, eps, iters, batch
    ("cfg1 (3,6) n=1000 eps=0.4 50 it", 1000, 0.40, 50, 65536),
    ("cfg5 (3,6) n=64800 eps=0.40 200 it", 64800, 0.40, 200, 4096),
    ("cfg5 (3,6) n=64800 eps=0.42 200 it", 64800, 0.42, 200, 4096),
]


def ref_cpu(g, words, iters, seconds):
    """Reference C message_passing, one call per word, as parallel_simulator.py:131-166."""
    from oracle import oracle
    if not oracle.ref_available():
        return None
    lib = ct.CDLL(os.path.join(oracle.REF_DIR, "message_passing.so"))
    v2c = np.ascontiguousarray(g.variable_lookup, np.int32)
    c2v = np.ascontiguousarray(g.check_lookup, np.int32)
    done, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        w = np.array(words[done % words.shape[0]], dtype=np.int32)
        err = np.zeros(iters, np.int32)
        lib.message_passing(w.ctypes.data_as(ct.POINTER(ct.c_int)), ct.c_int(iters),
                            v2c.ctypes.data_as(ct.POINTER(ct.c_int)), c2v.ctypes.data_as(ct.POINTER(ct.c_int)),
                            err.ctypes.data_as(ct.POINTER(ct.c_int)), ct.c_int(g.n), ct.c_int(g.k), ct.c_int(3),
                            ct.c_int(6))
        done += 1
    el = time.perf_counter() - t0
    return {"value": done / el, "unit": "codewords/s", "cores": 1, "kind": "reference",
            "sample": f"{done} words, reference message_passing.c (oracle/_ref, gcc -O2) 1 core, {el:.1f} s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cpu-seconds", type=float, default=5.0)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    s = torch.cuda.current_stream()
    for name, n, eps, iters, B in WORKLOADS:
        g = TannerGraph.random_regular(n, 3, 6, seed=1)
        words0 = decoder.channel_dev("bec", eps, 5, 0, n, B)
        times = []
        for r in range(args.reps + 1):
            words = words0.clone()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            _, err, its = decoder.bec_decode_dev(g, words, iters)
            b.record(s)
            torch.cuda.synchronize()
            if r:
                times.append(a.elapsed_time(b))
        ms = min(times)
        mean_its = float(its.float().mean().item())
        fer = float((err[:, -1] > 0).float().mean().item())
        # fused MC batch (channel + decode + statistics)
        mc = MonteCarlo(g, "bec", eps, iters, seed=9, batch=B)
        mc.run_batch(0, B)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        mc.run_batch(B, B)
        b.record(s)
        torch.cuda.synchronize()
        mc_ms = a.elapsed_time(b)
        cpu = ref_cpu(g, words0[:64].cpu().numpy(), iters, args.cpu_seconds)
        print(json.dumps({"workload": name, "batch": B, "decode_codewords_per_s": B / ms * 1e3,
                          "decode_ms": ms, "mc_codewords_per_s": B / mc_ms * 1e3, "mean_iterations": mean_its,
                          "fer": fer, "edge_visits_per_s": B / ms * 1e3 * mean_its * 2 * 3 * n,
                          "cpu_baseline": cpu, "kernel": "bec_dec_bits_kernel"}), flush=True)


def mc_fixed(reps=3):
    """Fixed-code Monte-Carlo (run_simulation_fixed_ldpc's device engine): channel + decode +
    statistics in one fused batch; bit-sliced kernel where the erasure planes fit LDS."""
    s = torch.cuda.current_stream()
    for n, eps, iters, B in ((1000, 0.40, 50, 65536), (1000, 0.40, 50, 262144), (10000, 0.40, 50, 65536),
                             (64800, 0.40, 200, 4096)):
        g = TannerGraph.random_regular(n, 3, 6, seed=1)
        mc = MonteCarlo(g, "bec", eps, iters, seed=9, batch=B)
        mc.run_batch(0, B)
        torch.cuda.synchronize()
        ts = []
        for r in range(reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            mc.run_batch((r + 1) * B, B)
            b.record(s)
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b))
        c = mc.counters.cpu().numpy()
        print(json.dumps({"workload": f"fixed-code MC (3,6) n={n} eps={eps} {iters} it", "batch": B,
                          "trials_per_s": B / min(ts) * 1e3, "ms": min(ts),
                          "fer": float(c[1] / c[0]), "mean_iterations": float(c[3] / c[0])}), flush=True)


def ensemble(reps=2):
    """Ensemble mode: a fresh (3,6) graph per trial drawn on the device + decode."""
    s = torch.cuda.current_stream()
    for n, eps, iters, B in ((1000, 0.40, 50, 16384), (10000, 0.40, 50, 4096), (64800, 0.40, 200, 1024)):
        mc = MonteCarlo.ensemble(n, 3, 6, "bec", eps, iters, seed=3, batch=B)
        mc.run_batch(0, min(B, 256))
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        mc.run_batch(B, B)
        b.record(s)
        torch.cuda.synchronize()
        ms = a.elapsed_time(b)
        print(json.dumps({"workload": f"ensemble (3,6) n={n} eps={eps} {iters} it (graph sampled per trial)",
                          "batch": B, "trials_per_s": B / ms * 1e3, "ms": ms}), flush=True)


if __name__ == "__main__":
    if "--mc" in sys.argv:
        mc_fixed()
        sys.exit(0)
    if "--ensemble" in sys.argv:
        ensemble()
        sys.exit(0)
    main()
