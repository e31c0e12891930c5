"""configs[3] error floor: decode BI-AWGN frames of the RSU n = 20000 code (--deg2 placement) (sum-product,
100 iterations, bp_loc_kernel) at sigmas in the floor region and dump every failing frame's
structure: residual error weight, degrees of the wrong variables, unsatisfied checks (0 = the
decoder converged to another codeword), and for small patterns the induced subgraph's
check degrees (a trapping set (a, b): a wrong variables, b odd-degree checks).

    python scripts/diag/floor_dump.py [--sigmas 0.78,0.80] [--frames 2000000] [--deg2 path|zigzag]
"""
import argparse, json, os, sys, time
sys.path.insert(0, os.getcwd())
import numpy as np
import torch
from iib_project_ldpc_codes_amd import decoder, ensembles

ap = argparse.ArgumentParser()
ap.add_argument("--sigmas", default="0.78,0.80")
ap.add_argument("--frames", type=int, default=2_000_000)
ap.add_argument("--fails", type=int, default=60)
ap.add_argument("--deg2", default="path")
ap.add_argument("--n", type=int, default=20000)
ap.add_argument("--seed", type=int, default=1)
ap.add_argument("--out", default="gpurun_out/floor_dump.json")
args = ap.parse_args()
g = ensembles.sample_irregular(ensembles.RSU_DL4, args.n, seed=args.seed, deg2=args.deg2)
cptr, cvar, vptr, vslot = [np.asarray(a) for a in g.to_csr()]
vdeg = np.diff(vptr)
chk_of_slot = np.repeat(np.arange(g.m), np.diff(cptr))
vchecks = [chk_of_slot[vslot[vptr[v]:vptr[v + 1]]] for v in range(g.n)]
print("kernel", g.kernel_name(), "n", g.n, "m", g.m, "E", g.num_edges, flush=True)
B = 65536
report = {"n": g.n, "deg2": args.deg2, "points": []}
for sigma in [float(x) for x in args.sigmas.split(",")]:
    fails, frames, t0 = [], 0, time.time()
    while frames < args.frames and len(fails) < args.fails:
        llr = decoder.channel_dev("awgn", sigma, 77, frames, g.n, B)
        _, hard, _ = decoder.bp_decode_dev(g, llr, 100, "spa", early_stop=False, want_post=False)
        bad = torch.nonzero(hard.any(dim=1)).flatten()
        for b in bad.tolist():
            h = hard[b].cpu().numpy().astype(np.int64)
            wrong = np.nonzero(h)[0]
            syn = np.zeros(g.m, np.int64)
            np.add.at(syn, chk_of_slot, h[cvar])
            unsat = int((syn % 2).sum())
            rec = {"frame": frames + b, "weight": int(len(wrong)), "unsat_checks": unsat,
                   "deg_hist": {int(d): int(c) for d, c in zip(*np.unique(vdeg[wrong], return_counts=True))}}
            if len(wrong) <= 40:
                cs = np.concatenate([vchecks[v] for v in wrong])
                u, c = np.unique(cs, return_counts=True)
                rec["odd_checks"] = int((c % 2 == 1).sum())
                rec["checks_touched"] = int(len(u))
                rec["wrong_vars"] = wrong.tolist()
            fails.append(rec)
        frames += B
        print(f"sigma {sigma}: {frames} frames, {len(fails)} failures, {time.time() - t0:.0f} s", flush=True)
    w = np.array([f["weight"] for f in fails]) if fails else np.zeros(0)
    cwd = sum(1 for f in fails if f["unsat_checks"] == 0)
    point = {"sigma": sigma, "frames": frames, "failures": len(fails), "fer": len(fails) / frames,
             "codeword_failures": cwd, "weights": sorted(w.tolist()), "fails": fails[:200]}
    report["points"].append(point)
    print(json.dumps({k: v for k, v in point.items() if k != "fails"}), flush=True)
os.makedirs(os.path.dirname(args.out), exist_ok=True)
json.dump(report, open(args.out, "w"))
