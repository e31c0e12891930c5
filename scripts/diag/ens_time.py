"""Ensemble BEC Monte-Carlo throughput (fresh device-sampled (3,6) graph per trial), configs[4]
shape: n = 64,800, 200 iterations, expurgation X = 3.  LDPC_LIB_PATH selects the build.
    python scripts/diag/ens_time.py [eps] [batch]"""
import os
import sys
import time

sys.path.insert(0, os.getcwd())
import torch

from iib_project_ldpc_codes_amd import _native
from iib_project_ldpc_codes_amd.montecarlo import MonteCarlo

eps = float(sys.argv[1]) if len(sys.argv) > 1 else 0.42
B = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
mc = MonteCarlo.ensemble(64800, 3, 6, "bec", eps, 200, seed=7, batch=B, expurgation=3)
mc.run_batch(0, 256)
torch.cuda.synchronize()
t0 = time.time()
mc.run_batch(256, B)
torch.cuda.synchronize()
el = time.time() - t0
c = mc.counters.cpu().numpy()
print(f"{os.path.basename(_native.LIB_PATH)} eps={eps} B={B} {B / el:.0f} trials/s ({el:.2f} s) "
      f"frame_errors={int(c[1])} trials={int(c[0])}", flush=True)
