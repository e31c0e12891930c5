"""ML ("optimal") erasure decoding on the MI355X vs the CPU oracle.

Bit-exact: decoded words (2 = given up) and per-word counts, through the C ABI
(ldpc_ml_decode_batch[_dev], ldpc_ml_ensemble_decode_dev, ldpc_mc_ml_batch_dev).
The oracle itself is pinned in tests/test_ml_oracle.py.
"""
import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu


def _torch():
    import torch
    assert torch.cuda.is_available()
    return torch


def _words(rs, B, n, eps_lo, eps_hi, inconsistent_every=3):
    eps = rs.uniform(eps_lo, eps_hi, size=(B, 1))
    w = np.where(rs.rand(B, n) < eps, 2, 0).astype(np.uint8)
    for b in range(0, B, inconsistent_every):
        w[b] = np.where(w[b] == 2, 2, rs.randint(0, 2, n))
    return w


@pytest.mark.parametrize("n", [100, 256, 1000, 2000])
def test_ml_fixed_graph_matches_oracle(n):
    torch = _torch()
    from iib_project_ldpc_codes_amd import decoder
    from iib_project_ldpc_codes_amd.graph import TannerGraph
    g = TannerGraph.random_regular(n, 3, 6, seed=n)
    cptr, cvar, _, _ = g.to_csr()
    rs = np.random.RandomState(n)
    B = 512 if n <= 1000 else 96
    w = _words(rs, B, n, 0.3, 0.52)
    w[0] = 0                      # no erasure
    w[1] = 2                      # everything erased (> n-k): unchanged
    w[2] = 0
    w[2][::2] = 2                 # exactly n-k erasures
    w[3] = 0
    w[3][5] = 2                   # one erasure
    out, uns = decoder.ml_decode_dev(g, torch.from_numpy(w).cuda())
    torch.cuda.synchronize()
    ref, ref_uns = oracle.ml_decode_batch(cptr, cvar, w, n, g.m)
    np.testing.assert_array_equal(uns.cpu().numpy(), ref_uns)
    np.testing.assert_array_equal(out.cpu().numpy(), ref)
    assert (ref_uns > 0).any() and (ref_uns == 0).any()


def test_ml_host_form_and_in_place():
    torch = _torch()
    from iib_project_ldpc_codes_amd import decoder
    from iib_project_ldpc_codes_amd.graph import TannerGraph
    n = 500
    g = TannerGraph.random_regular(n, 3, 6, seed=3)
    cptr, cvar, _, _ = g.to_csr()
    w = _words(np.random.RandomState(2), 64, n, 0.35, 0.5)
    out, uns = decoder.ml_decode(g, w)
    ref, ref_uns = oracle.ml_decode_batch(cptr, cvar, w, n, g.m)
    np.testing.assert_array_equal(out, ref)
    np.testing.assert_array_equal(uns, ref_uns)
    t = torch.from_numpy(w).cuda()
    decoder.ml_decode_dev(g, t, out=t)  # d_out aliases d_words
    torch.cuda.synchronize()
    np.testing.assert_array_equal(t.cpu().numpy(), ref)


def test_ml_irregular_csr_matches_oracle():
    torch = _torch()
    from iib_project_ldpc_codes_amd import decoder, ensembles
    g = ensembles.sample_irregular(ensembles.RSU_DL4, 1000, seed=4)
    cptr, cvar, _, _ = g.to_csr()
    w = _words(np.random.RandomState(4), 256, g.n, 0.3, 0.5)
    out, uns = decoder.ml_decode_dev(g, torch.from_numpy(w).cuda())
    torch.cuda.synchronize()
    ref, ref_uns = oracle.ml_decode_batch(cptr, cvar, w, g.n, g.m)
    np.testing.assert_array_equal(out.cpu().numpy(), ref)
    np.testing.assert_array_equal(uns.cpu().numpy(), ref_uns)


def test_ml_ensemble_matches_oracle():
    torch = _torch()
    from iib_project_ldpc_codes_amd import _native, decoder
    n, dv, dc, B = 200, 3, 6, 256
    chk = torch.empty((B, n * dv), dtype=torch.int32, device="cuda")
    var = torch.empty_like(chk)
    rc = _native.lib().ldpc_sample_regular_dev(n, dv, dc, 21, 0, B, chk.data_ptr(), var.data_ptr(), None,
                                               torch.cuda.current_stream().cuda_stream)
    _native.check(rc, "ldpc_sample_regular_dev")
    w = _words(np.random.RandomState(7), B, n, 0.3, 0.5)
    out, uns = decoder.ml_ensemble_decode_dev(n, dv, dc, chk, torch.from_numpy(w).cuda())
    torch.cuda.synchronize()
    chk_h = chk.cpu().numpy()
    cptr = np.arange(n * dv // dc + 1, dtype=np.int32) * dc
    for b in range(B):
        ref, ref_uns = oracle.ml_decode_batch(cptr, chk_h[b], w[b], n, n * dv // dc)
        np.testing.assert_array_equal(out[b].cpu().numpy(), ref[0])
        assert int(uns[b]) == ref_uns[0]


def _oracle_mc(words_fn, graphs_fn, n, m, iters, stop, mp, trials):
    """Sequential reference loop (parallel_simulator.py:198-244) on oracle outputs."""
    mp_frames = mp_bits = ml_frames = ml_bits = 0
    curve = np.zeros(iters + 1, np.int64)
    i = 0
    while i < trials:
        w = words_fn(i)
        cptr, cvar, v2c = graphs_fn(i)
        if mp:
            _, err, _ = oracle.bec_decode_batch(np.where(w == 2, 2, 0)[None], iters, v2c, cvar, n, n - m, 3, 6)
            e = np.concatenate([[int((w == 2).sum())], err[0]])
            curve += e
            mp_frames += e[-1] != 0
            mp_bits += e[-1]
        _, uns = oracle.ml_decode_batch(cptr, cvar, w, n, m)
        ml_frames += uns[0] > 0
        ml_bits += uns[0]
        i += 1
        if (mp_frames if mp else ml_frames) >= stop:
            break
    return i, mp_frames, mp_bits, curve, ml_frames, ml_bits


@pytest.mark.parametrize("mp", [True, False])
def test_mc_ml_fixed_counters_match_oracle(mp):
    torch = _torch()
    from iib_project_ldpc_codes_amd.graph import TannerGraph
    from iib_project_ldpc_codes_amd.montecarlo import MonteCarlo
    n, eps, iters, B, stop = 200, 0.42, 30, 4096, 40
    g = TannerGraph.random_regular(n, 3, 6, seed=9)
    cptr, cvar, _, _ = g.to_csr()
    mc = MonteCarlo(g, "bec", eps, iters, seed=5, batch=B, optimal=True, message_passing=mp)
    mc.run_batch(0, B, stop)
    torch.cuda.synchronize()
    res = mc.results()
    words = oracle.channel(oracle.CH_BEC, eps, 5, 0, n, B).astype(np.uint8)
    i, f, bits, curve, mlf, mlb = _oracle_mc(lambda t: words[t], lambda t: (cptr, cvar, g.variable_lookup),
                                             n, g.m, iters, stop, mp, B)
    assert res["ml_num_tests"] == i
    assert res["ml_frame_errors"] == mlf and res["ml_bit_errors"] == mlb
    if mp:
        assert res["num_tests"] == i and res["frame_errors"] == f and res["bit_errors"] == bits
        np.testing.assert_array_equal(res["raw_counters"][4:], curve)
    assert (mlf if not mp else f) == stop  # the stop rule cut inside the batch


def test_mc_ml_ensemble_counters_match_oracle():
    torch = _torch()
    from iib_project_ldpc_codes_amd.montecarlo import MonteCarlo
    n, eps, iters, B = 100, 0.4, 20, 1024
    mc = MonteCarlo.ensemble(n, 3, 6, "bec", eps, iters, seed=13, batch=B, optimal=True, message_passing=True)
    mc.run_batch(0, B, 0)
    torch.cuda.synchronize()
    res = mc.results()
    words = oracle.channel(oracle.CH_BEC, eps, 13, 0, n, B).astype(np.uint8)
    cptr = np.arange(51, dtype=np.int32) * 6

    def graphs(t):
        chk, var, _ = oracle.sample_regular(n, 3, 6, 13, t)
        return cptr, chk, var
    i, f, bits, curve, mlf, mlb = _oracle_mc(lambda t: words[t], graphs, n, 50, iters, 10 ** 9, True, B)
    assert res["num_tests"] == res["ml_num_tests"] == B == i
    assert res["frame_errors"] == f and res["bit_errors"] == bits
    assert res["ml_frame_errors"] == mlf and res["ml_bit_errors"] == mlb
    assert mlf <= f  # at eps = 0.4 ML fails on fewer frames than message passing


def test_device_ensemble_ml_ber_matches_reference_plots():
    """As tests/test_ml_oracle.py, with 40x the trials on the device (per-trial counts
    come back from ldpc_ml_ensemble_decode_dev for the variance estimate)."""
    torch = _torch()
    from iib_project_ldpc_codes_amd import _native, decoder
    from tests.test_ml_oracle import PLOTTED_ML_BER_N100, ml_ber_agrees
    n, B = 100, 65536
    chk = torch.empty((B, 300), dtype=torch.int32, device="cuda")
    var = torch.empty_like(chk)
    for eps in sorted(PLOTTED_ML_BER_N100):
        counts = []
        for r in range(8):
            rc = _native.lib().ldpc_sample_regular_dev(n, 3, 6, 17, r * B, B, chk.data_ptr(), var.data_ptr(), None,
                                                       torch.cuda.current_stream().cuda_stream)
            _native.check(rc, "ldpc_sample_regular_dev")
            w = decoder.channel_dev("bec", eps, 17, r * B, n, B)
            _, uns = decoder.ml_ensemble_decode_dev(n, 3, 6, chk, w)
            counts.append(uns.cpu().numpy())
        ok, ber, ref = ml_ber_agrees(np.concatenate(counts).astype(np.float64), n, eps)
        assert ok, (eps, ber, ref)


def test_simulator_mirror_optimal_modes(tmp_path, monkeypatch):
    _torch()
    from iib_project_ldpc_codes_amd import parallel_simulator as ps
    from iib_project_ldpc_codes_amd.graph import TannerGraph
    from tests.ml_restated import optimal_decode
    monkeypatch.setattr(ps, "base_directory", str(tmp_path) + "/")
    g = TannerGraph.random_regular(100, 3, 6, seed=2)
    H = g.parity_check()
    code = ps.regular_LDPC_code(H, 100, 50, 3, 6)
    rs = np.random.RandomState(3)
    for _ in range(20):
        w = np.where(rs.rand(100) < 0.42, 2, 0)
        out = code.optimal_decode(w)
        ref, _ = optimal_decode(H, w)
        np.testing.assert_array_equal(np.asarray(out), ref)
    for mode in (1, 2, 4, 5):
        res = ps.main(["0.4", "3000", "20", "100", "3", "6", str(mode), "1"])
        assert res["ml_num_tests"] > 0
        rows = open(tmp_path / "report_data" / "simulation_data" / res["filename"]).read().splitlines()
        assert rows[-1].startswith("Optimal decoding bit-wise error")
        assert ("Message passing block-wise error" in "".join(rows)) == (mode in (2, 5))
