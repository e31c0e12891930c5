"""Time the fused Monte-Carlo (channel + decode + counters) across library builds.
    LDPC_LIB_PATH=build_variants/x.so python scripts/kbench_mc.py cfg3 [p ...]
cfg3: (3,6) n = 10,000 BSC normalized min-sum (alpha 0.75), 50 iterations, early stop,
65,536 trials per batch (configs[2]'s shape; scripts/fer_sweep.py cfg3)."""
import os
import sys
sys.path.insert(0, os.getcwd())
import torch
from iib_project_ldpc_codes_amd.graph import TannerGraph
from iib_project_ldpc_codes_amd.montecarlo import MonteCarlo
g = TannerGraph.random_regular(10000, 3, 6, seed=1, distinct_columns=True)
B = 65536
for p in [float(x) for x in (sys.argv[2:] or ["0.075", "0.07", "0.065"])]:
    mc = MonteCarlo(g, "bsc", p, 50, algo="minsum", alpha=0.75, early_stop=True, seed=11, batch=B)
    mc.run_batch(0, B)
    torch.cuda.synchronize()
    ts = []
    for r in range(3):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        mc.run_batch((r + 1) * B, B)
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    c = mc.counters.cpu().numpy()
    print(f"{os.environ.get('LDPC_LIB_PATH', 'in-tree'):30s} {g.kernel_name():22s} p={p} {min(ts):8.2f} ms "
          f"{B / min(ts) * 1e3:12.0f} trials/s  fer {c[1] / c[0]:.2e} mean_it {c[3] / c[0]:.2f}", flush=True)
