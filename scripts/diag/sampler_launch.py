"""One ldpc_sample_regular_dev launch ((3,6), n given, G graphs) for profiling the sampler.
    python scripts/diag/sampler_launch.py [n] [G] [reps]"""
import ctypes as ct
import os
import sys

sys.path.insert(0, os.getcwd())
import torch

from iib_project_ldpc_codes_amd import _native

n = int(sys.argv[1]) if len(sys.argv) > 1 else 64800
G = int(sys.argv[2]) if len(sys.argv) > 2 else 256
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 1
L = _native.lib()
chk = torch.empty((G, n * 3), dtype=torch.int32, device="cuda")
var = torch.empty_like(chk)
att = torch.empty(G, dtype=torch.int32, device="cuda")
s = torch.cuda.current_stream()
for r in range(reps):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    _native.check(L.ldpc_sample_regular_dev(n, 3, 6, 5, r * G, G, chk.data_ptr(), var.data_ptr(), att.data_ptr(),
                                            s.cuda_stream), "sample")
    b.record(s)
    torch.cuda.synchronize()
    A = att.float().abs().mean().item()
    ms = a.elapsed_time(b)
    print(f"n={n} G={G} {ms:.2f} ms {G / ms * 1e3:.0f} graphs/s mean attempts {A:.1f} "
          f"us/attempt/graph {ms * 1e3 / (G * A):.3f}", flush=True)
