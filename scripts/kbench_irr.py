"""Time the irregular (config-4 shape) decode across library builds."""
import ctypes as ct, os, sys
sys.path.insert(0, os.getcwd())
import numpy as np, torch
from iib_project_ldpc_codes_amd import decoder, ensembles
g = ensembles.sample_irregular(ensembles.RSU_DL4, int(os.environ.get("N", "20000")), seed=1, deg2=os.environ.get("DEG2", "path"))
print("kernel", g.kernel_name(), "E", g.num_edges, flush=True)
B = 8192; it = int(os.environ.get("ITERS", "20")); algo = int(os.environ.get("ALGO", "0"))
llr = decoder.channel_dev("awgn", 0.8, 7, 0, g.n, B)
hard = torch.empty(llr.shape, dtype=torch.uint8, device="cuda")
s = torch.cuda.current_stream()
cp, cv, vp, vs = g.csr
for p in sys.argv[1:]:
    L = ct.CDLL(os.path.abspath(p))
    L.ldpc_graph_create_csr.argtypes = [ct.c_void_p]*4 + [ct.c_int]*2 + [ct.POINTER(ct.c_void_p)]
    L.ldpc_bp_decode_batch_dev.argtypes = [ct.c_void_p, ct.c_void_p, ct.c_int, ct.c_int, ct.c_int, ct.c_float, ct.c_int, ct.c_void_p, ct.c_void_p, ct.c_void_p, ct.c_void_p]
    h = ct.c_void_p()
    assert L.ldpc_graph_create_csr(cp.ctypes.data, cv.ctypes.data, vp.ctypes.data, vs.ctypes.data, g.n, g.m, ct.byref(h)) == 0
    ts = []
    for r in range(3):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        assert L.ldpc_bp_decode_batch_dev(h, llr.data_ptr(), B, it, algo, ct.c_float(0.75 if algo else 1.0), int(os.environ.get("ET", "0")), None, hard.data_ptr(), None, ct.c_void_p(s.cuda_stream)) == 0
        b.record(s); torch.cuda.synchronize(); ts.append(a.elapsed_time(b))
    print(f"{p:36s} {min(ts):9.2f} ms  {B/min(ts)*1e3*it/100:10.1f} cw/s@100it  errs {int(hard.sum())}")
