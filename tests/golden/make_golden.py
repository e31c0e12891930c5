"""Generate the committed golden fixtures from the REFERENCE itself.

Run in the build container only (needs /root/reference and `make -C oracle ref`):

    python tests/golden/make_golden.py

Outputs (committed; data only -- inputs and the reference's outputs):
  bec_golden.npz   graphs drawn by the reference's random_code_generator.c
                   (10-argument call, parallel_simulator_expurgated.py:201-223)
                   plus hand-made multi-edge graphs; channel words; and the
                   outputs of the reference's message_passing.c driven with the
                   marshalling of parallel_simulator.py:131-166 (word, errors
                   with the initial erasure count prepended, return index).
                   Raw-C cases with caller-populated errors[] pin the `+=`
                   accumulation of message_passing.c:73.
  ml_golden.npz    ML-decoder system set-up: graphs (and dense H) drawn by the
                   reference's random_code_generator.c, channel words, and the
                   (target, remaining_parity_checks) buffers the reference's
                   ml_decoder.c fills, driven as parallel_simulator.py:72-88.
                   (`python tests/golden/make_golden.py ml` regenerates only this.)
  de_golden.json   BEC density evolution / threshold known answers computed by
                   the reference's tools/density_evolution.py:9-16 and
                   test_de_threshold.py:17-28, finite_length_scaling_calculation.py.
"""
import ctypes as ct
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
from oracle import oracle  # noqa: E402

REF = "/root/reference"


def reference_cases():
    assert oracle.ref_available(), "run `make -C oracle ref` first"
    rs = np.random.RandomState(20261015)
    out = {}
    graphs = []
    # reference-generated regular graphs
    for (n, dv, dc) in [(12, 3, 6), (60, 3, 6), (100, 3, 6), (1000, 3, 6), (64, 4, 8), (90, 2, 3), (10000, 3, 6)]:
        chk, var, _H = oracle.ref_generate_random_code(n, dv, dc)
        graphs.append((n, dv, dc, chk, var))
    # hand-made multi-edge graph: check 0 holds variable 1 twice (n=6, dv=2, dc=4)
    c2v_me = np.array([0, 1, 1, 2, 3, 4, 5, 0, 2, 3, 4, 5], np.int32)
    v2c_me = np.zeros(12, np.int32)
    cnt = {}
    lists = [[] for _ in range(6)]
    for c in range(3):
        for s in range(4):
            lists[c2v_me[c * 4 + s]].append(c)
    v2c_me = np.array([sorted(lst) for lst in lists], np.int32).ravel()
    graphs.append((6, 2, 4, c2v_me, v2c_me))
    del cnt

    cases = []
    for gi, (n, dv, dc, chk, var) in enumerate(graphs):
        k = int(n * (dc - dv) / dc)
        out[f"g{gi}_n"] = np.array([n, k, dv, dc], np.int32)
        out[f"g{gi}_c2v"] = np.asarray(chk, np.int32)
        out[f"g{gi}_v2c"] = np.asarray(var, np.int32)
        its_set = [1, 2, 3, 20, 50] if n <= 1000 else [50]
        eps_set = [0.3, 0.4, 0.45, 0.5] if n <= 1000 else [0.4, 0.42]
        reps = 3 if n <= 1000 else 2
        for max_its in its_set:
            for eps in eps_set:
                for _ in range(reps):
                    word = np.where(rs.rand(n) < eps, 2, 0).astype(np.float64)  # channels.py:24-26
                    cases.append((gi, word, max_its, None))
            if n <= 1000:
                for _ in range(2):  # non-codewords: pins "last known message wins"
                    word = rs.randint(0, 3, size=n).astype(np.float64)
                    cases.append((gi, word, max_its, None))
    # raw-C cases with caller-populated errors[] (message_passing.c:16-19,73)
    for gi in [1, 3]:
        n = graphs[gi][0]
        for _ in range(3):
            word = np.where(rs.rand(n) < 0.42, 2, 0).astype(np.float64)
            cases.append((gi, word, 20, rs.randint(0, 3, size=20).astype(np.int32)))

    lib_mp = ct.CDLL(os.path.join(oracle.REF_DIR, "message_passing.so"))
    for ci, (gi, word, max_its, err_in) in enumerate(cases):
        n, dv, dc, chk, var = graphs[gi]
        k = int(n * (dc - dv) / dc)
        if err_in is None:
            w_out, errs, it = oracle.ref_message_pass_decode(word, max_its, chk, var, n, k, dv, dc)
        else:
            w_out = np.array(word, dtype="int32")
            errs = err_in.copy()
            it = lib_mp.message_passing(w_out.ctypes.data_as(ct.POINTER(ct.c_int)), ct.c_int(max_its),
                                        np.asarray(var, np.int32).ctypes.data_as(ct.POINTER(ct.c_int)),
                                        np.asarray(chk, np.int32).ctypes.data_as(ct.POINTER(ct.c_int)),
                                        errs.ctypes.data_as(ct.POINTER(ct.c_int)),
                                        ct.c_int(n), ct.c_int(k), ct.c_int(dv), ct.c_int(dc))
            out[f"c{ci}_errin"] = err_in
        out[f"c{ci}_meta"] = np.array([gi, max_its, it, 0 if err_in is None else 1], np.int32)
        out[f"c{ci}_word"] = word.astype(np.int8)
        out[f"c{ci}_out"] = np.asarray(w_out, np.int8)
        out[f"c{ci}_errors"] = np.asarray(errs, np.int32)
    out["num_cases"] = np.array([len(cases)], np.int32)
    out["num_graphs"] = np.array([len(graphs)], np.int32)
    np.savez_compressed(os.path.join(HERE, "bec_golden.npz"), **out)
    print(f"bec_golden.npz: {len(graphs)} graphs, {len(cases)} cases")


def de_cases():
    sys.path.insert(0, REF)
    sys.path.insert(0, os.path.join(REF, "tools"))
    import matplotlib
    matplotlib.use("Agg")
    import density_evolution as de  # tools/density_evolution.py
    import test_de_threshold as tdt
    import finite_length_scaling_calculation as fls
    res = {
        "density_evolution_0.4_10_3_6": list(map(float, de.density_evolution(0.4, 10, 3, 6))),
        "density_evolution_0.2_10_3_6_1e-9": list(map(float, de.density_evolution(0.2, 10, 3, 6, 1e-9))),
        "density_evolution_0.45_30_3_6": list(map(float, de.density_evolution(0.45, 30, 3, 6))),
        "calc_threshold_3_6": float(tdt.calc_threshold(3, 6)),
        "alpha_3_6": float(fls.calculate_alpha(tdt.calc_threshold(3, 6), 3, 6)),
        "beta_shift_3_6": 0.616949,
    }
    with open(os.path.join(HERE, "de_golden.json"), "w") as f:
        json.dump(res, f, indent=1)
    print("de_golden.json:", {k: (v if not isinstance(v, list) else len(v)) for k, v in res.items()})


def ml_cases():
    assert oracle.ref_available(), "run `make -C oracle ref` first"
    rs = np.random.RandomState(20261016)
    out = {}
    cases = 0
    for gi, (n, dv, dc) in enumerate([(12, 3, 6), (60, 3, 6), (100, 3, 6), (64, 4, 8)]):
        chk, var, H = oracle.ref_generate_random_code(n, dv, dc)
        out[f"g{gi}_n"] = np.array([n, dv, dc], np.int32)
        out[f"g{gi}_c2v"] = np.asarray(chk, np.int32)
        out[f"g{gi}_H"] = np.asarray(H, np.uint8)
        for eps in (0.1, 0.3, 0.4, 0.45, 0.5):
            for _ in range(3):
                word = np.where(rs.rand(n) < eps, 2, 0)
                if cases % 2:  # non-codeword known values too
                    word = np.where(word == 2, 2, rs.randint(0, 2, size=n))
                target, rem = oracle.ref_ml_system(H, word, n, dv, dc)
                out[f"c{cases}_meta"] = np.array([gi], np.int32)
                out[f"c{cases}_word"] = word.astype(np.uint8)
                out[f"c{cases}_target"] = target
                out[f"c{cases}_remaining"] = rem
                cases += 1
    out["num_cases"] = np.array([cases], np.int32)
    out["num_graphs"] = np.array([4], np.int32)
    np.savez_compressed(os.path.join(HERE, "ml_golden.npz"), **out)
    print(f"ml_golden.npz: {cases} cases")


if __name__ == "__main__":
    if sys.argv[1:] == ["ml"]:
        ml_cases()
    else:
        reference_cases()
        ml_cases()
        de_cases()
