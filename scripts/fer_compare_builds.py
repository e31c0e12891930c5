"""Same Monte-Carlo trials (same seeds, same code) decoded by the library build in
LDPC_LIB_PATH: FER / BER / mean iterations of fixed-count and early-stop sum-product
on (3,6) n=10000 BI-AWGN at a few sigma.  Run once per build and compare the lines
(used to check that the product-domain variable phase decodes like the log-domain one).
  LDPC_LIB_PATH=<build>.so python scripts/fer_compare_builds.py [--trials N]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from iib_project_ldpc_codes_amd.graph import TannerGraph  # noqa: E402
from iib_project_ldpc_codes_amd.montecarlo import MonteCarlo  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trials", type=int, default=4 * 65536)
    args = ap.parse_args()
    g = TannerGraph.random_regular(10000, 3, 6, seed=1)
    B = 65536
    for et in (False, True):
        for sigma in (0.80, 0.84, 0.88):
            mc = MonteCarlo(g, "awgn", sigma, 50, algo="spa", early_stop=et, seed=31, batch=B)
            for k in range(args.trials // B):
                mc.run_batch(k * B, B)
            torch.cuda.synchronize()
            c = mc.counters.cpu().numpy()
            print(json.dumps({"build": os.environ.get("LDPC_LIB_PATH", "default"), "sigma": sigma,
                              "early_stop": et, "trials": int(c[0]), "frame_errors": int(c[1]),
                              "fer": float(c[1] / c[0]), "bit_errors": int(c[2]),
                              "mean_iterations": float(c[3] / c[0])}), flush=True)


if __name__ == "__main__":
    main()
