import sys, os
sys.path.insert(0, os.getcwd())
import numpy as np, torch
from iib_project_ldpc_codes_amd import decoder
from iib_project_ldpc_codes_amd.graph import TannerGraph
from oracle import oracle
g = TannerGraph.random_regular(10000, 3, 6, seed=1)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
llr = decoder.channel_dev("awgn", 0.70, 3, 0, g.n, B)
post, hard, its = decoder.bp_decode_dev(g, llr, 50, "spa")
torch.cuda.synchronize()
errs = hard.sum(dim=1).cpu().numpy()
bad = np.nonzero(errs)[0]
print("B", B, "bad frames", bad.size, "first", bad[:20], "errs", errs[bad[:20]])
csr = oracle.csr_from_lists(g.variable_lookup, g.check_lookup, g.n, g.m, 3, 6)
for b in bad[:3]:
    l = llr[b:b+1].cpu().numpy()
    op, oh, oi = oracle.bp_decode_batch(csr, l, 50, 0)
    h = hard[b].cpu().numpy()
    wrong = np.nonzero(h)[0]
    print("frame", b, "gpu errs", h.sum(), "oracle errs", oh.sum(), "wrong idx sample", wrong[:12], "mod1024", np.unique(wrong % 1024)[:10])
    # try same frame alone on gpu
    p1, h1, _ = decoder.bp_decode(g, l, 50, "spa")
    print("   alone gpu errs", h1.sum())
# determinism
post2, hard2, _ = decoder.bp_decode_dev(g, llr, 50, "spa")
torch.cuda.synchronize()
print("deterministic", bool(torch.equal(hard, hard2)), "post equal", bool(torch.equal(post, post2)))
