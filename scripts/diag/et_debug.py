"""Debug: early-stop decode on the LDS kernel vs the oracle (iterations, posteriors)."""
import sys, os
sys.path.insert(0, os.getcwd())
import numpy as np
import torch  # noqa: F401
from iib_project_ldpc_codes_amd import decoder
from iib_project_ldpc_codes_amd.graph import TannerGraph
from oracle import oracle
for n in (1000, 10000):
    g = TannerGraph.random_regular(n, 3, 6, seed=13)
    csr = oracle.csr_from_lists(g.variable_lookup, g.check_lookup, n, g.m, 3, 6)
    llr = oracle.channel(oracle.CH_AWGN, 0.80, 13, 0, n, 16)
    for algo, a in (("minsum", 1), ("spa", 0)):
        for et in (False, True):
            post, hard, its = decoder.bp_decode(g, llr, 30, algo, alpha=0.75, early_stop=et)
            opost, ohard, oits = oracle.bp_decode_batch(csr, llr, 30, a, alpha=0.75, early_stop=et)
            print(n, algo, "ET" if et else "  ", "its gpu", its[:8], "oracle", oits[:8],
                  "maxdiff", float(np.abs(post - opost).max()), "hard mism", int((hard != ohard).sum()), flush=True)
