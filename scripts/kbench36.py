"""Time the (3,6) n = 10,000 headline decode (65,536 frames, 50 iterations) across library builds.
    python scripts/kbench36.py build_variants/a.so build_variants/b.so   (env ALGO=0|1, ET=0|1, ITERS)"""
import ctypes as ct, os, sys
sys.path.insert(0, os.getcwd())
import torch
from iib_project_ldpc_codes_amd import decoder
from iib_project_ldpc_codes_amd.graph import TannerGraph
g = TannerGraph.random_regular(10000, 3, 6, seed=1)
B = 65536; it = int(os.environ.get("ITERS", "50")); algo = int(os.environ.get("ALGO", "0"))
llr = decoder.channel_dev("awgn", float(os.environ.get("SIGMA", "0.85")), 2026, 0, g.n, B)
hard = torch.empty(llr.shape, dtype=torch.uint8, device="cuda")
s = torch.cuda.current_stream()
cp, cv, vp, vs = [__import__("numpy").ascontiguousarray(x, "int32") for x in g.to_csr()]
for p in sys.argv[1:]:
    L = ct.CDLL(os.path.abspath(p))
    L.ldpc_graph_create_csr.argtypes = [ct.c_void_p]*4 + [ct.c_int]*2 + [ct.POINTER(ct.c_void_p)]
    L.ldpc_bp_decode_batch_dev.argtypes = [ct.c_void_p, ct.c_void_p, ct.c_int, ct.c_int, ct.c_int, ct.c_float, ct.c_int, ct.c_void_p, ct.c_void_p, ct.c_void_p, ct.c_void_p]
    L.ldpc_bp_kernel_name.restype = ct.c_char_p
    h = ct.c_void_p()
    assert L.ldpc_graph_create_csr(cp.ctypes.data, cv.ctypes.data, vp.ctypes.data, vs.ctypes.data, g.n, g.m, ct.byref(h)) == 0
    ts = []
    for r in range(4):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        assert L.ldpc_bp_decode_batch_dev(h, llr.data_ptr(), B, it, algo, ct.c_float(0.75 if algo else 1.0), int(os.environ.get("ET", "0")), None, hard.data_ptr(), None, ct.c_void_p(s.cuda_stream)) == 0
        b.record(s); torch.cuda.synchronize(); ts.append(a.elapsed_time(b))
    print(f"{p:36s} {L.ldpc_bp_kernel_name(h, 0).decode():24s} {min(ts):9.2f} ms  {B/min(ts)*1e3:12.1f} cw/s  errs {int(hard.sum())}", flush=True)
