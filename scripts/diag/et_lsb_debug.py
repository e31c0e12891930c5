"""Hard-decision early stop on bp_loc_kernel vs the oracle: iteration counts and frame
agreement, for the in-tree library and (LDPC_LIB_PATH) another build.
    python scripts/diag/et_lsb_debug.py"""
import os
import sys

sys.path.insert(0, os.getcwd())
import numpy as np
import torch

from iib_project_ldpc_codes_amd import decoder, _native
from iib_project_ldpc_codes_amd.graph import TannerGraph
from oracle import oracle

print("lib", _native.LIB_PATH, flush=True)
g = TannerGraph.random_regular(10000, 3, 6, seed=41, distinct_columns=True)
csr = [np.ascontiguousarray(a, np.int32) for a in g.to_csr()]
llr = oracle.channel(oracle.CH_AWGN, 0.85, 17, 0, g.n, 64)
t = torch.from_numpy(llr).cuda()
for es, wp in ((True, False), (False, False), (True, True)):
    post, hard, its = decoder.bp_decode_dev(g, t, 50, "spa", 1.0, es, want_post=wp)
    torch.cuda.synchronize()
    h, i = hard.cpu().numpy(), its.cpu().numpy()
    _, oh, oi = oracle.bp_decode_batch(csr, llr, 50, 0, 1.0, es)
    print(f"es={es} want_post={wp} kernel={g.kernel_name(early_stop=es, hard_only=not wp)} its[:12]={i[:12].tolist()} "
          f"oracle its[:12]={oi[:12].tolist()} frames equal={np.mean(np.all(h == oh, axis=1)):.3f} "
          f"its equal={np.mean(i == oi):.3f} bit errs={int(h.sum())} oracle bit errs={int(oh.sum())}", flush=True)
