"""Early-stop decodes that ask for hard decisions only (post == NULL) run on bp_loc_kernel
(the stopping iteration's decisions kept in a bit per variable, csrc/ldpc_kernels.hip); the
posterior-returning early-stop decode runs on bp_loc_kernel's slab-and-replay instantiation
where the message LDS can stage the posteriors (both the (3,6) codes and the ring code here),
else on bp_lds_kernel / bp_irr_kernel.  Both must give what oracle_bp_decode (ldpc_oracle.c)
gives with early_stop = 1:

* min-sum (one check class, the (3,6) codes): hard decisions and iteration counts bit-exact;
* sum-product: iteration counts and hard decisions identical on >= 99 % of frames (the kernel's
  fp32 product form against the oracle's double-precision check rule, as test_gpu_loc.py's
  50-iteration test), and identical to the posterior-returning kernel's on >= 99 % of frames;
  every stopped frame's decisions satisfy every check (a codeword).
"""
import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available(), "GPU tests need a visible MI355X"
    return t


def _graph(kind, n):
    from iib_project_ldpc_codes_amd import ensembles
    from iib_project_ldpc_codes_amd.graph import TannerGraph
    if kind == "ring":
        g = TannerGraph.from_csr(*ensembles.sample_irregular(ensembles.RSU_DL4, n, seed=1, deg2="path").to_csr())
    else:
        g = TannerGraph.random_regular(n, 3, 6, seed=41, distinct_columns=True)
    return g, [np.ascontiguousarray(a, np.int32) for a in g.to_csr()]


def _decode(torch, g, llr, iters, algo, want_post):
    from iib_project_ldpc_codes_amd import decoder
    t = torch.from_numpy(llr).cuda()
    post, hard, its = decoder.bp_decode_dev(g, t, iters, algo, 0.75 if algo == "minsum" else 1.0, True,
                                            want_post=want_post)
    torch.cuda.synchronize()
    return hard.cpu().numpy(), its.cpu().numpy()


def _syndrome_ok(csr, hard):
    cptr, cvar = csr[0], csr[1]
    par = np.add.reduceat(hard[:, cvar].astype(np.int64), cptr[:-1], axis=1) & 1
    return ~par.any(axis=1)


@pytest.mark.parametrize("n", [1000, 10000])
def test_minsum_hard_early_stop_bit_exact(torch, n):
    g, csr = _graph("reg", n)
    assert g.kernel_name(early_stop=True, hard_only=True) == "bp_loc_kernel" or n == 1000
    llr = oracle.channel(oracle.CH_BSC, 0.07, 13, 0, g.n, 256)
    for iters in (1, 2, 7, 50):
        hard, its = _decode(torch, g, llr, iters, "minsum", False)
        _, ohard, oits = oracle.bp_decode_batch(csr, llr, iters, 1, 0.75, True)
        np.testing.assert_array_equal(its, oits)
        np.testing.assert_array_equal(hard, ohard)


@pytest.mark.parametrize("kind,n,sigma", [("reg", 10000, 0.85), ("reg", 1000, 0.80), ("ring", 20000, 0.84)])
def test_spa_hard_early_stop_vs_oracle_and_posterior_path(torch, kind, n, sigma):
    g, csr = _graph(kind, n)
    if n >= 10000:
        assert g.kernel_name(early_stop=True, hard_only=True) == "bp_loc_kernel"
    llr = oracle.channel(oracle.CH_AWGN, sigma, 17, 0, g.n, 256)
    hard, its = _decode(torch, g, llr, 50, "spa", False)
    phard, pits = _decode(torch, g, llr, 50, "spa", True)
    _, ohard, oits = oracle.bp_decode_batch(csr, llr, 50, 0, 1.0, True)
    same_o = np.all(hard == ohard, axis=1) & (its == oits)
    same_p = np.all(hard == phard, axis=1) & (its == pits)
    assert same_o.mean() >= 0.99, same_o.mean()
    assert same_p.mean() >= 0.99, same_p.mean()
    stopped = its < 50
    assert stopped.any() and np.all(_syndrome_ok(csr, hard)[stopped])
    assert np.all(its >= 1)


def test_host_form_without_posteriors_matches_device_hard_path(torch):
    """ldpc_bp_decode_batch (host pointers) with post = NULL takes the same hard-decision path."""
    from iib_project_ldpc_codes_amd import _native
    g, _ = _graph("reg", 10000)
    llr = oracle.channel(oracle.CH_AWGN, 0.85, 19, 0, g.n, 64)
    dhard, dits = _decode(torch, g, llr, 50, "spa", False)
    hard = np.zeros_like(dhard)
    its = np.zeros(64, np.int32)
    v2c = np.ascontiguousarray(g.variable_lookup, np.int32)
    c2v = np.ascontiguousarray(g.check_lookup, np.int32)
    rc = _native.lib().ldpc_bp_decode_batch(v2c.ctypes.data, c2v.ctypes.data, g.n, g.k, 3, 6, llr.ctypes.data, 64,
                                            50, 0, 1.0, 1, None, hard.ctypes.data, its.ctypes.data)
    _native.check(rc, "ldpc_bp_decode_batch")
    np.testing.assert_array_equal(hard, dhard)
    np.testing.assert_array_equal(its, dits)
