"""Config-4 shape: RSU rate-1/2 irregular ensemble, n = 20000, BI-AWGN, 100 iterations."""
import json, os, sys
sys.path.insert(0, os.getcwd())
import torch
from iib_project_ldpc_codes_amd import decoder, ensembles
from iib_project_ldpc_codes_amd.montecarlo import MonteCarlo
g = ensembles.sample_irregular(ensembles.RSU_DL4, 20000, seed=1, deg2=os.environ.get("DEG2", "path"))
s = torch.cuda.current_stream()
for sigma in (0.85, 0.80):
    B = int(os.environ.get("B", "8192"))
    llr = decoder.channel_dev("awgn", sigma, 7, 0, g.n, B)
    for et in (False, True):
        decoder.bp_decode_dev(g, llr, 100, "spa", early_stop=et, want_post=False)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        _, hard, its = decoder.bp_decode_dev(g, llr, 100, "spa", early_stop=et, want_post=False)
        b.record(s)
        torch.cuda.synchronize()
        ms = a.elapsed_time(b)
        print(json.dumps({"workload": "RSU_DL4 n=20000 BI-AWGN SPA 100 it", "sigma": sigma, "early_stop": et,
                          "kernel": g.kernel_name(et), "codewords_per_s": B / ms * 1e3,
                          "mean_iterations": float(its.float().mean()), "fer": float(hard.any(1).float().mean())}),
              flush=True)
    mc = MonteCarlo(g, "awgn", sigma, 100, algo="spa", early_stop=True, seed=3, batch=B)
    mc.run_batch(0, B)
    torch.cuda.synchronize()
    a.record(s)
    mc.run_batch(B, B)
    b.record(s)
    torch.cuda.synchronize()
    print(json.dumps({"mc_codewords_per_s": B / a.elapsed_time(b) * 1e3, "sigma": sigma}), flush=True)
