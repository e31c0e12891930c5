"""Time the headline SPA decode with several builds of the library (interleaved rounds).
usage: python scripts/kbench.py build_variants/*.so"""
import ctypes as ct, os, sys, time, json
sys.path.insert(0, os.getcwd())
import torch
import numpy as np
libs = sys.argv[1:]
algo = int(os.environ.get("ALGO", "0")); et = int(os.environ.get("ET", "0"))
B = int(os.environ.get("B", "65536")); N = int(os.environ.get("N", "10000"))
from iib_project_ldpc_codes_amd import _native
from iib_project_ldpc_codes_amd.graph import TannerGraph
from iib_project_ldpc_codes_amd import decoder
g = TannerGraph.random_regular(N, 3, 6, seed=1)
llr = decoder.channel_dev("awgn", 0.85, 2026, 0, g.n, B)
post = torch.empty_like(llr); hard = torch.empty(llr.shape, dtype=torch.uint8, device="cuda"); its = torch.empty(B, dtype=torch.int32, device="cuda")
handles = []
for p in libs:
    L = ct.CDLL(os.path.abspath(p), mode=os.RTLD_LOCAL)
    L.ldpc_graph_create.argtypes = [ct.c_void_p]*2 + [ct.c_int]*4 + [ct.POINTER(ct.c_void_p)]
    L.ldpc_bp_decode_batch_dev.argtypes = [ct.c_void_p, ct.c_void_p, ct.c_int, ct.c_int, ct.c_int, ct.c_float, ct.c_int, ct.c_void_p, ct.c_void_p, ct.c_void_p, ct.c_void_p]
    h = ct.c_void_p()
    assert L.ldpc_graph_create(g.variable_lookup.ctypes.data, g.check_lookup.ctypes.data, g.n, g.k, 3, 6, ct.byref(h)) == 0
    handles.append((p, L, h))
s = torch.cuda.current_stream()
res = {p: [] for p in libs}
ref = None
for rnd in range(4):
    for p, L, h in handles:
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        rc = L.ldpc_bp_decode_batch_dev(h, llr.data_ptr(), B, 50, algo, ct.c_float(0.75), et, post.data_ptr(), hard.data_ptr(), its.data_ptr(), ct.c_void_p(s.cuda_stream))
        b.record(s); torch.cuda.synchronize()
        assert rc == 0
        if rnd > 0: res[p].append(a.elapsed_time(b))
        hsum = int(hard.sum().item())
        if ref is None: ref = hsum
        if hsum != ref: print("MISMATCH", p, hsum, ref)
for p in libs:
    t = min(res[p]); print(f"{p:40s} min {t:8.2f} ms  med {np.median(res[p]):8.2f} ms  {B/t*1e3/1e3:8.1f} kcw/s")
