"""Debug the irregular kernel against the oracle: first iteration with a mismatch."""
import sys, os
sys.path.insert(0, os.getcwd())
import numpy as np
import torch  # noqa: F401
from iib_project_ldpc_codes_amd import decoder, ensembles
from oracle import oracle
n = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
g = ensembles.sample_irregular_device(ensembles.RSU_DL4, n, seed=8, graph_id=50)
print("kernel", g.kernel_name(), flush=True)
llr = oracle.channel(oracle.CH_AWGN, 0.8, 3, 0, n, 8)
csr = g.to_csr()
for it in (1, 2, 3, 5, 10, 20):
    post, hard, its = decoder.bp_decode(g, llr, it, "minsum", alpha=0.75)
    opost, ohard, _ = oracle.bp_decode_batch(csr, llr, it, 1, alpha=0.75)
    bad = np.nonzero(post != opost)
    print(it, "mismatch", len(bad[0]), "frames", np.unique(bad[0])[:8], "vars", bad[1][:8],
          "maxdiff", float(np.abs(post - opost).max()), flush=True)
    if len(bad[0]):
        v = bad[1][0]
        print("  var", v, "deg", csr[2][v + 1] - csr[2][v], "gpu", post[bad[0][0], v], "oracle", opost[bad[0][0], v])
# repeatability
p1, _, _ = decoder.bp_decode(g, llr, 20, "minsum", alpha=0.75)
p2, _, _ = decoder.bp_decode(g, llr, 20, "minsum", alpha=0.75)
print("repeatable", bool(np.array_equal(p1, p2)))
