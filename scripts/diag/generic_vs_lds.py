"""Per-edge throughput of the generic CSR kernel vs the LDS-resident (3,6) kernel."""
import json, os, sys
sys.path.insert(0, os.getcwd())
import torch
from iib_project_ldpc_codes_amd import decoder, ensembles
from iib_project_ldpc_codes_amd.graph import TannerGraph
s = torch.cuda.current_stream()
cases = [
    ("regular lists n=10000", TannerGraph.random_regular(10000, 3, 6, seed=1)),
    ("regular CSR n=10000", TannerGraph.from_csr(*TannerGraph.random_regular(10000, 3, 6, seed=1).to_csr())),
    ("RSU n=10000", ensembles.sample_irregular(ensembles.RSU_DL4, 10000, seed=1, deg2="zigzag")),
    ("RSU n=20000", ensembles.sample_irregular(ensembles.RSU_DL4, 20000, seed=1, deg2="zigzag")),
]
for name, g in cases:
    B = 16384
    llr = decoder.channel_dev("awgn", 0.85, 7, 0, g.n, B)
    decoder.bp_decode_dev(g, llr, 50, "spa", want_post=False)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    decoder.bp_decode_dev(g, llr, 50, "spa", want_post=False)
    b.record(s)
    torch.cuda.synchronize()
    ms = a.elapsed_time(b)
    E = g.num_edges
    print(json.dumps({"case": name, "kernel": g.kernel_name(False), "cw_per_s": B / ms * 1e3,
                      "edge_iters_per_s": B * 50 * E / ms * 1e3}), flush=True)
