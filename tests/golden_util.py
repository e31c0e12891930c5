"""Loader for tests/golden/bec_golden.npz (made by tests/golden/make_golden.py)."""
import os

import numpy as np

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_bec_golden():
    z = np.load(os.path.join(GOLD, "bec_golden.npz"))
    graphs = {}
    for gi in range(int(z["num_graphs"][0])):
        n, k, dv, dc = map(int, z[f"g{gi}_n"])
        graphs[gi] = (n, k, dv, dc, z[f"g{gi}_v2c"], z[f"g{gi}_c2v"])
    cases = []
    for ci in range(int(z["num_cases"][0])):
        gi, max_its, it, has_err = map(int, z[f"c{ci}_meta"])
        cases.append(dict(gi=gi, max_its=max_its, it=it, word=z[f"c{ci}_word"], out=z[f"c{ci}_out"],
                          errors=z[f"c{ci}_errors"], errin=z[f"c{ci}_errin"] if has_err else None))
    return graphs, cases
