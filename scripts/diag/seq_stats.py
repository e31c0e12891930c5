"""Search-pass statistics of the sequential-draw sampler (a -DLDPC_SEQ_STATS=1 build):
    LDPC_LIB_PATH=build_variants/stats.so python scripts/diag/seq_stats.py [n] [G]"""
import ctypes as ct
import os
import sys

sys.path.insert(0, os.getcwd())
import torch

from iib_project_ldpc_codes_amd import _native

n = int(sys.argv[1]) if len(sys.argv) > 1 else 64800
G = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
L = _native.lib()
chk = torch.empty((G, n * 3), dtype=torch.int32, device="cuda")
var = torch.empty_like(chk)
att = torch.empty(G, dtype=torch.int32, device="cuda")
K = 8  # kStCount of csrc/sampler.hip
st = (ct.c_uint64 * (2 * K))()
s = torch.cuda.current_stream()
_native.check(L.ldpc_sample_regular_dev(n, 3, 6, 5, 0, G, chk.data_ptr(), var.data_ptr(), att.data_ptr(),
                                        s.cuda_stream), "sample")
torch.cuda.synchronize()
_native.check(L.ldpc_debug_seq_stats(st, 1), "stats")
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record(s)
_native.check(L.ldpc_sample_regular_dev(n, 3, 6, 5, G, G, chk.data_ptr(), var.data_ptr(), att.data_ptr(),
                                        s.cuda_stream), "sample")
b.record(s)
torch.cuda.synchronize()
_native.check(L.ldpc_debug_seq_stats(st, 0), "stats")
names = ["attempts", "aborted", "rounds", "kept", "lane_iters", "spread_iters", "coll_rounds", "abort_rounds"]
d = dict(zip(names, list(st)[:K]))
emit = dict(zip(names, list(st)[K:]))
ms = a.elapsed_time(b)
print(f"n={n} G={G} {ms:.2f} ms  {G / ms * 1e3:.0f} graphs/s  mean attempts {att.float().abs().mean().item():.1f}")
for k in names:
    print(f"  {k:14s} {d[k]:16d}")
R = max(d["rounds"], 1)
A = max(d["attempts"], 1)
print(f"  per graph: attempts {d['attempts'] / G:.1f}  rounds {d['rounds'] / G:.0f}  kept/round {d['kept'] / R:.1f}  "
      f"rounds/attempt {d['rounds'] / A:.1f}  aborted/graph {d['aborted'] / G:.1f} (rounds before the abort "
      f"{d['abort_rounds'] / max(d['aborted'], 1):.0f})")
print(f"  per round: lane iters {d['lane_iters'] / R:.3f}  spread iters {d['spread_iters'] / R:.3f}  "
      f"collision rounds {d['coll_rounds'] / R:.3f}")
print(f"  emit pass: attempts {emit['attempts']}  rounds {emit['rounds']}  kept/round {emit['kept'] / max(emit['rounds'], 1):.1f}")
