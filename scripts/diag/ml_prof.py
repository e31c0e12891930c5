"""One ML decode launch per workload (for rocprofv3 PMC runs)."""
import os, sys
sys.path.insert(0, os.getcwd())
import torch
from iib_project_ldpc_codes_amd import decoder
from iib_project_ldpc_codes_amd.graph import TannerGraph
for n, eps, B in ((1000, 0.40, 32768), (2000, 0.45, 8192), (2000, 0.20, 8192)):
    g = TannerGraph.random_regular(n, 3, 6, seed=1)
    w = decoder.channel_dev("bec", eps, 5, 0, n, B)
    out, uns = decoder.ml_decode_dev(g, w)
    torch.cuda.synchronize()
    print(n, eps, B, float(uns.float().mean()), flush=True)
