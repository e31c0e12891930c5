"""Compare a library build's headline SPA decode with the oracle (and with build 0) on frames of the
bench batch.  usage: python scripts/diag/variant_compare.py lib0.so lib1.so ... [FRAMES=512 ITERS=50]"""
import ctypes as ct, os, sys
sys.path.insert(0, os.getcwd())
import numpy as np
import torch
from iib_project_ldpc_codes_amd.graph import TannerGraph
from iib_project_ldpc_codes_amd import decoder
from oracle import oracle

F = int(os.environ.get("FRAMES", "512")); IT = int(os.environ.get("ITERS", "50")); SIG = float(os.environ.get("SIGMA", "0.85"))
g = TannerGraph.random_regular(10000, 3, 6, seed=1)
B = 65536
llr = decoder.channel_dev("awgn", SIG, 2026, 0, g.n, B)
pick = torch.arange(0, B, B // F, device="cuda")
sub = llr[pick].contiguous()
csr = oracle.csr_from_lists(g.variable_lookup, g.check_lookup, g.n, g.m, 3, 6)
op, oh, _ = oracle.bp_decode_batch(csr, sub.cpu().numpy(), IT, 0)
ofer = oh.any(axis=1).mean()
for p in sys.argv[1:]:
    L = ct.CDLL(os.path.abspath(p), mode=os.RTLD_LOCAL)
    L.ldpc_graph_create.argtypes = [ct.c_void_p] * 2 + [ct.c_int] * 4 + [ct.POINTER(ct.c_void_p)]
    L.ldpc_bp_decode_batch_dev.argtypes = [ct.c_void_p, ct.c_void_p, ct.c_int, ct.c_int, ct.c_int, ct.c_float, ct.c_int,
                                           ct.c_void_p, ct.c_void_p, ct.c_void_p, ct.c_void_p]
    h = ct.c_void_p()
    assert L.ldpc_graph_create(g.variable_lookup.ctypes.data, g.check_lookup.ctypes.data, g.n, g.k, 3, 6, ct.byref(h)) == 0
    post = torch.empty_like(sub); hard = torch.empty(sub.shape, dtype=torch.uint8, device="cuda")
    its = torch.empty(F, dtype=torch.int32, device="cuda")
    rc = L.ldpc_bp_decode_batch_dev(h, sub.data_ptr(), F, IT, 0, ct.c_float(1.0), 0, post.data_ptr(), hard.data_ptr(),
                                    its.data_ptr(), ct.c_void_p(torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize(); assert rc == 0
    gp, gh = post.cpu().numpy(), hard.cpu().numpy()
    same = np.all(gh == oh, axis=1)
    d = np.abs(gp[same].astype(np.float64) - op[same]); ref = np.abs(op[same].astype(np.float64))
    close = (d <= 1e-3 + 1e-3 * ref).mean()
    print(f"{p:36s} identical_frames {same.mean():.4f} fer {gh.any(axis=1).mean():.4f} (oracle {ofer:.4f}) "
          f"post_close {close:.5f} max_abs {d.max():.3g} bad_vals {(d > 2e-2 + 1e-2 * ref).sum()}")
