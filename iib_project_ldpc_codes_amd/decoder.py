"""Batched decoders on the MI355X (device tensors via torch, host arrays via the C ABI).

* ``bec_decode``  -- message_passing.c:7-82 over a batch of words (bit-exact).
* ``bp_decode``   -- flooding sum-product / normalized min-sum (new capability).
* ``ml_decode``   -- ML ("optimal") erasure decoding, optimal_decode of
                     parallel_simulator.py:60-129 (GF(2) elimination on the device).
* ``channel``     -- on-device BEC / BSC / BI-AWGN channel outputs (Philox).

Device forms take torch CUDA(HIP) tensors and run asynchronously on the
current torch stream; host forms take numpy arrays and block.
"""
import numpy as np

from . import _native
from ._native import ALGO_MINSUM, ALGO_SPA, CH_AWGN, CH_BEC, CH_BSC  # noqa: F401

ALGOS = {"spa": ALGO_SPA, "sum-product": ALGO_SPA, "minsum": ALGO_MINSUM, "min-sum": ALGO_MINSUM,
         ALGO_SPA: ALGO_SPA, ALGO_MINSUM: ALGO_MINSUM}
CHANNELS = {"bec": CH_BEC, "bsc": CH_BSC, "awgn": CH_AWGN, "biawgn": CH_AWGN,
            CH_BEC: CH_BEC, CH_BSC: CH_BSC, CH_AWGN: CH_AWGN}


def _torch():
    import torch
    if not torch.cuda.is_available():
        raise _native.LdpcError("device", _native.LDPC_ENODEV, "no HIP device visible to torch")
    return torch


def _stream(stream=None):
    torch = _torch()
    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream


def _ptr(t):
    return None if t is None else t.data_ptr()


# ----------------------------------------------------------------------- BEC
def bec_decode_dev(graph, words, max_iters, errors=None, its=None, stream=None):
    """words: uint8 [B, n] device tensor (0/1/2), decoded in place.
    errors: int32 [B, max_iters] (accumulated like message_passing.c:73; zeros if None).
    Returns (words, errors, its)."""
    torch = _torch()
    B = words.shape[0]
    if errors is None:
        errors = torch.zeros((B, max_iters), dtype=torch.int32, device=words.device)
    if its is None:
        its = torch.empty((B,), dtype=torch.int32, device=words.device)
    assert words.dtype == torch.uint8 and words.is_contiguous() and words.shape[1] == graph.n
    assert errors.dtype == torch.int32 and errors.is_contiguous() and tuple(errors.shape) == (B, max_iters)
    rc = _native.lib().ldpc_bec_decode_batch_dev(graph.handle(), words.data_ptr(), B, max_iters,
                                                 errors.data_ptr(), its.data_ptr(), _stream(stream))
    _native.check(rc, "ldpc_bec_decode_batch_dev")
    return words, errors, its


def bec_decode(graph, words, max_iters, errors=None):
    """Host form: words uint8/int [B, n] numpy (0/1/2).  Returns (words, errors, its)."""
    w = np.ascontiguousarray(np.atleast_2d(words), dtype=np.uint8).copy()
    B = w.shape[0]
    err = (np.zeros((B, max_iters), np.int32) if errors is None
           else np.ascontiguousarray(errors, dtype=np.int32).reshape(B, max_iters).copy())
    its = np.zeros(B, np.int32)
    if graph.csr is not None:
        torch = _torch()
        tw = torch.from_numpy(w).cuda()
        te = torch.from_numpy(err).cuda()
        _, te, ti = bec_decode_dev(graph, tw, max_iters, te)
        torch.cuda.synchronize()
        return tw.cpu().numpy(), te.cpu().numpy(), ti.cpu().numpy()
    rc = _native.lib().ldpc_bec_decode_batch(graph.variable_lookup.ctypes.data, graph.check_lookup.ctypes.data,
                                             graph.n, graph.k, graph.dv, graph.dc, w.ctypes.data, B, max_iters,
                                             err.ctypes.data, its.ctypes.data)
    _native.check(rc, "ldpc_bec_decode_batch")
    return w, err, its


# ------------------------------------------------------------------------ ML
def ml_decode_dev(graph, words, out=None, unsolved=None, stream=None):
    """words: uint8 [B, n] device tensor (0/1 known, 2 erased).  Returns (out, unsolved):
    decoded words with 2 where the reference's loop gives an unknown up, and the
    number of 2s per word (parallel_simulator.py:60-129, :235)."""
    torch = _torch()
    assert words.dtype == torch.uint8 and words.is_contiguous() and words.shape[1] == graph.n
    B = words.shape[0]
    if out is None:
        out = torch.empty_like(words)
    if unsolved is None:
        unsolved = torch.empty((B,), dtype=torch.int32, device=words.device)
    rc = _native.lib().ldpc_ml_decode_batch_dev(graph.handle(), words.data_ptr(), B, out.data_ptr(),
                                                unsolved.data_ptr(), _stream(stream))
    _native.check(rc, "ldpc_ml_decode_batch_dev")
    return out, unsolved


def ml_decode(graph, words):
    """Host form: words uint8 [B, n] numpy.  Returns (out, unsolved) numpy."""
    w = np.ascontiguousarray(np.atleast_2d(words), dtype=np.uint8)
    B = w.shape[0]
    out = np.zeros_like(w)
    uns = np.zeros(B, np.int32)
    rc = _native.lib().ldpc_ml_decode_batch(graph.handle(), w.ctypes.data, B, out.ctypes.data, uns.ctypes.data)
    _native.check(rc, "ldpc_ml_decode_batch")
    return out, uns


def ml_ensemble_decode_dev(n, dv, dc, check_lookup, words, out=None, unsolved=None, stream=None):
    """Word b decoded on graph b: check_lookup int32 [B, n*dv] device tensor
    (graph.sample_device / ldpc_sample_regular_dev layout)."""
    torch = _torch()
    B = words.shape[0]
    assert check_lookup.dtype == torch.int32 and check_lookup.is_contiguous()
    assert tuple(check_lookup.shape) == (B, n * dv) and words.dtype == torch.uint8 and words.shape[1] == n
    if out is None:
        out = torch.empty_like(words)
    if unsolved is None:
        unsolved = torch.empty((B,), dtype=torch.int32, device=words.device)
    rc = _native.lib().ldpc_ml_ensemble_decode_dev(n, dv, dc, check_lookup.data_ptr(), words.data_ptr(), B,
                                                   out.data_ptr(), unsolved.data_ptr(), _stream(stream))
    _native.check(rc, "ldpc_ml_ensemble_decode_dev")
    return out, unsolved


# ---------------------------------------------------------------------- soft
def bp_decode_dev(graph, llr, max_iters, algo="spa", alpha=1.0, early_stop=False, post=None, hard=None,
                  its=None, stream=None, want_post=True, want_hard=True):
    """llr: float32 [B, n] device tensor.  Returns (post, hard, its) device tensors."""
    torch = _torch()
    B = llr.shape[0]
    assert llr.dtype == torch.float32 and llr.is_contiguous() and llr.shape[1] == graph.n
    if post is None and want_post:
        post = torch.empty_like(llr)
    if hard is None and want_hard:
        hard = torch.empty(llr.shape, dtype=torch.uint8, device=llr.device)
    if its is None:
        its = torch.empty((B,), dtype=torch.int32, device=llr.device)
    rc = _native.lib().ldpc_bp_decode_batch_dev(graph.handle(), llr.data_ptr(), B, max_iters, ALGOS[algo],
                                                float(alpha), int(bool(early_stop)), _ptr(post), _ptr(hard),
                                                _ptr(its), _stream(stream))
    _native.check(rc, "ldpc_bp_decode_batch_dev")
    return post, hard, its


def bp_decode(graph, llr, max_iters, algo="spa", alpha=1.0, early_stop=False):
    """Host form: llr float32 [B, n] numpy.  Returns (post, hard, its) numpy."""
    torch = _torch()
    t = torch.from_numpy(np.ascontiguousarray(np.atleast_2d(llr), dtype=np.float32)).cuda()
    post, hard, its = bp_decode_dev(graph, t, max_iters, algo, alpha, early_stop)
    torch.cuda.synchronize()
    return post.cpu().numpy(), hard.cpu().numpy(), its.cpu().numpy()


# ------------------------------------------------------------------ channels
def channel_dev(kind, param, seed, first_cw, n, B, out=None, stream=None, device=None):
    """Channel outputs of the all-zero codeword for codewords first_cw..first_cw+B-1:
    BEC -> uint8 (0 / 2 erasure), BSC / AWGN -> float32 LLRs."""
    torch = _torch()
    kind = CHANNELS[kind]
    if out is None:
        dt = torch.uint8 if kind == CH_BEC else torch.float32
        out = torch.empty((B, n), dtype=dt, device=device or "cuda")
    rc = _native.lib().ldpc_channel_dev(kind, float(param), int(seed), int(first_cw), n, B, out.data_ptr(),
                                        _stream(stream))
    _native.check(rc, "ldpc_channel_dev")
    return out
