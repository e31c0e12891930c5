"""ORACLE -- test infrastructure only (see ldpc_oracle.c header).

ctypes bindings for the CPU restatement (``_build/liboracle.so``) and for the
reference's own C compiled from /root/reference into ``_ref/`` (driven with
the exact marshalling of parallel_simulator.py:131-166).  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline import this module.
"""
import ctypes as ct
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# ORACLE_LIB_PATH: the sanitizer build (scripts/sanitize.sh)
LIB_PATH = os.environ.get("ORACLE_LIB_PATH") or os.path.join(HERE, "_build", "liboracle.so")
REF_DIR = os.path.join(HERE, "_ref")

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE, "all"], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = ct.CDLL(LIB_PATH)
        P = ct.c_void_p
        i, f, u64 = ct.c_int, ct.c_float, ct.c_uint64
        _lib.oracle_message_passing.argtypes = [P, i, P, P, P, i, i, i, i]
        _lib.oracle_message_passing.restype = i
        _lib.oracle_bec_decode_batch.argtypes = [P, P, i, i, i, i, P, i, i, P, P]
        _lib.oracle_bec_decode_batch.restype = None
        _lib.oracle_build_var_slots.argtypes = [P, P, i, i, i, i, P]
        _lib.oracle_build_var_slots.restype = i
        _lib.oracle_bp_decode_batch.argtypes = [P, P, P, P, i, i, P, i, i, i, f, i, P, P, P]
        _lib.oracle_bp_decode_batch.restype = None
        _lib.oracle_philox4x32_10.argtypes = [P, P, P]
        _lib.oracle_philox4x32_10.restype = None
        _lib.oracle_channel.argtypes = [i, f, f, u64, u64, i, i, P]
        _lib.oracle_channel.restype = None
        _lib.oracle_density_evolution.argtypes = [ct.c_double, i, i, i, ct.c_double, P]
        _lib.oracle_density_evolution.restype = i
        _lib.oracle_sample_regular.argtypes = [i, i, i, u64, u64, i, P, P]
        _lib.oracle_sample_regular.restype = i
        _lib.oracle_ml_system.argtypes = [i, i, P, P, P, P, P]
        _lib.oracle_ml_system.restype = None
        _lib.oracle_ml_decode.argtypes = [i, i, P, P, P, P]
        _lib.oracle_ml_decode.restype = i
        _lib.oracle_ml_decode_batch.argtypes = [i, i, P, P, P, i, P, P]
        _lib.oracle_ml_decode_batch.restype = None
        _lib.oracle_sample_regular_batch.argtypes = [i, i, i, u64, u64, i, i, P, P, P]
        _lib.oracle_sample_regular_batch.restype = None
        _lib.oracle_sample_csr.argtypes = [i, i, P, P, u64, u64, i, P, P]
        _lib.oracle_sample_csr.restype = i
        _lib.oracle_sampler_force_seq.argtypes = [i]
        _lib.oracle_sampler_force_seq.restype = None
        _lib.oracle_check_update.argtypes = [P, i, i, f]
        _lib.oracle_check_update.restype = None
        _lib.oracle_num_threads.argtypes = []
        _lib.oracle_num_threads.restype = i
        _lib.oracle_set_num_threads.argtypes = [i]
        _lib.oracle_set_num_threads.restype = None
    return _lib


def _p(a):
    return a.ctypes.data_as(ct.c_void_p)


def message_passing(word, iterations, v2c, c2v, n, k, dv, dc, errors=None):
    """Restatement of message_passing.c:7-82.  Returns (word, errors, it)."""
    w = np.ascontiguousarray(word, dtype=np.int32).copy()
    v2c = np.ascontiguousarray(v2c, dtype=np.int32).ravel()
    c2v = np.ascontiguousarray(c2v, dtype=np.int32).ravel()
    err = np.zeros(iterations, np.int32) if errors is None else np.ascontiguousarray(errors, np.int32).copy()
    it = lib().oracle_message_passing(_p(w), iterations, _p(v2c), _p(c2v), _p(err), n, k, dv, dc)
    return w, err, it


def bec_decode_batch(words, iterations, v2c, c2v, n, k, dv, dc, errors=None):
    """errors: the caller's int32 [B, iterations] accumulators (zeros if None)."""
    words = np.ascontiguousarray(words).astype(np.int8)
    B = words.shape[0]
    v2c = np.ascontiguousarray(v2c, dtype=np.int32).ravel()
    c2v = np.ascontiguousarray(c2v, dtype=np.int32).ravel()
    err = (np.zeros((B, iterations), np.int32) if errors is None
           else np.ascontiguousarray(errors, dtype=np.int32).reshape(B, iterations).copy())
    its = np.zeros(B, np.int32)
    lib().oracle_bec_decode_batch(_p(v2c), _p(c2v), n, k, dv, dc, _p(words), B, iterations, _p(err), _p(its))
    return words, err, its


def csr_from_lists(v2c, c2v, n, m, dv, dc):
    """Regular edge lists -> (cptr, cvar, vptr, vslot) CSR slot form."""
    v2c = np.ascontiguousarray(v2c, dtype=np.int32).ravel()
    c2v = np.ascontiguousarray(c2v, dtype=np.int32).ravel()
    vslot = np.zeros(n * dv, np.int32)
    rc = lib().oracle_build_var_slots(_p(v2c), _p(c2v), n, m, dv, dc, _p(vslot))
    if rc != 0:
        raise ValueError("variable_to_check_list and check_to_variable_list disagree")
    cptr = (np.arange(m + 1, dtype=np.int32) * dc).astype(np.int32)
    vptr = (np.arange(n + 1, dtype=np.int32) * dv).astype(np.int32)
    return cptr, c2v.copy(), vptr, vslot


def bp_decode_batch(csr, llr, max_iters, algo=0, alpha=1.0, early_stop=False):
    """Soft flooding decoder (algo 0 = sum-product, 1 = normalized min-sum)."""
    cptr, cvar, vptr, vslot = [np.ascontiguousarray(a, dtype=np.int32) for a in csr]
    n = vptr.shape[0] - 1
    m = cptr.shape[0] - 1
    llr = np.ascontiguousarray(llr, dtype=np.float32)
    if llr.ndim == 1:
        llr = llr[None, :]
    B = llr.shape[0]
    post = np.zeros((B, n), np.float32)
    hard = np.zeros((B, n), np.uint8)
    its = np.zeros(B, np.int32)
    lib().oracle_bp_decode_batch(_p(cptr), _p(cvar), _p(vptr), _p(vslot), n, m, _p(llr), B, max_iters,
                                 algo, alpha, int(bool(early_stop)), _p(post), _p(hard), _p(its))
    return post, hard, its


def check_update(x, algo=0, alpha=1.0):
    """One check-node update (the decoders' rule) on a copy of the d inputs x."""
    x = np.ascontiguousarray(x, dtype=np.float32).copy()
    lib().oracle_check_update(_p(x), x.shape[0], algo, alpha)
    return x


def num_threads():
    return int(lib().oracle_num_threads())


def set_num_threads(t):
    lib().oracle_set_num_threads(int(t))


def philox(ctr, key):
    c = np.ascontiguousarray(ctr, dtype=np.uint32)
    k = np.ascontiguousarray(key, dtype=np.uint32)
    out = np.zeros(4, np.uint32)
    lib().oracle_philox4x32_10(_p(c), _p(k), _p(out))
    return out


CH_BEC, CH_BSC, CH_AWGN = 0, 1, 2


def channel_params(kind, p):
    """(p, p2) pair the channel kernels take: BSC p2 = ln((1-p)/p); AWGN p = sigma, p2 = 2/sigma^2."""
    if kind == CH_BEC:
        return float(p), 0.0
    if kind == CH_BSC:
        return float(p), float(np.float32(np.log((1.0 - p) / p)))
    return float(p), float(np.float32(2.0 / (p * p)))


def channel(kind, p, seed, first_cw, n, B):
    p, p2 = channel_params(kind, p)
    out = np.zeros((B, n), np.int8 if kind == CH_BEC else np.float32)
    lib().oracle_channel(kind, p, p2, seed, first_cw, n, B, _p(out))
    return out


def sample_regular(n, dv, dc, seed, graph, max_attempts=1 << 20):
    """Restatement of the device sampler (law of random_code_generator.c).
    Returns (check_lookup, variable_lookup, attempts)."""
    chk = np.zeros(n * dv, np.int32)
    var = np.zeros(n * dv, np.int32)
    att = lib().oracle_sample_regular(n, dv, dc, seed, graph, max_attempts, _p(chk), _p(var))
    return chk, var, att


def sample_regular_batch(n, dv, dc, seed, first_graph, G, max_attempts=1 << 20):
    """G graphs first_graph.. of the device sampler's restatement (OpenMP).
    Returns (check_lookup [G, n*dv], variable_lookup [G, n*dv], attempts [G])."""
    chk = np.zeros((G, n * dv), np.int32)
    var = np.zeros((G, n * dv), np.int32)
    att = np.zeros(G, np.int32)
    lib().oracle_sample_regular_batch(n, dv, dc, seed, first_graph, G, max_attempts, _p(chk), _p(var), _p(att))
    return chk, var, att


def sampler_force_seq(on):
    """Tests only: restate the sequential-draw sampler (sample_seq_kernel) at every graph
    size instead of the kernels' size rule."""
    lib().oracle_sampler_force_seq(1 if on else 0)


def sample_csr(var_ptr, check_ptr, seed, graph, max_attempts=1 << 20):
    """Irregular form of the device sampler.  Returns (check_var [E], var_slot [E], attempts)."""
    vp = np.ascontiguousarray(var_ptr, np.int32)
    cp = np.ascontiguousarray(check_ptr, np.int32)
    n, m, E = len(vp) - 1, len(cp) - 1, int(vp[-1])
    cv = np.zeros(E, np.int32)
    vs = np.zeros(E, np.int32)
    att = lib().oracle_sample_csr(n, m, _p(vp), _p(cp), seed, graph, max_attempts, _p(cv), _p(vs))
    return cv, vs, att


def density_evolution(eps, iterations, dv, dc, threshold=0.0):
    out = np.zeros(iterations + 1, np.float64)
    ln = lib().oracle_density_evolution(eps, iterations, dv, dc, threshold, _p(out))
    return out[:ln]


def ml_system(cptr, cvar, word, n, m):
    """ml_decoder.c:7-36 restated: (target[m], remaining[ne, m]) as uint8."""
    cptr = np.ascontiguousarray(cptr, np.int32)
    cvar = np.ascontiguousarray(cvar, np.int32)
    w = np.ascontiguousarray(word, np.uint8)
    ne = int((w == 2).sum())
    target = np.zeros(m, np.uint8)
    rem = np.zeros(max(ne, 1) * m, np.uint8)
    lib().oracle_ml_system(n, m, _p(cptr), _p(cvar), _p(w), _p(target), _p(rem))
    return target, rem[: ne * m].reshape(ne, m)


def ml_decode_batch(cptr, cvar, words, n, m):
    """optimal_decode (parallel_simulator.py:60-129) restated, per word.
    Returns (out_words uint8 [B, n] with 2 = unsolvable, unsolved int32 [B])."""
    cptr = np.ascontiguousarray(cptr, np.int32)
    cvar = np.ascontiguousarray(cvar, np.int32)
    w = np.ascontiguousarray(words, np.uint8)
    if w.ndim == 1:
        w = w[None, :]
    B = w.shape[0]
    out = np.zeros((B, n), np.uint8)
    uns = np.zeros(B, np.int32)
    lib().oracle_ml_decode_batch(n, m, _p(cptr), _p(cvar), _p(w), B, _p(out), _p(uns))
    return out, uns


# --------------------------------------------------------------------------
# Reference C (compiled from /root/reference by `make -C oracle ref`)
# --------------------------------------------------------------------------
def ref_available():
    return os.path.exists(os.path.join(REF_DIR, "message_passing.so"))


def ref_message_pass_decode(binary_sequence, max_its, check_lookup, variable_lookup, n, k, dv, dc):
    """Drive _ref/message_passing.so exactly as parallel_simulator.py:131-166 does.

    Returns (word_int32, errors_with_initial_prepended, it)."""
    check_lookup = np.array(check_lookup, dtype="int32").flatten()
    variable_lookup = np.array(variable_lookup, dtype="int32").flatten()
    errors = np.zeros(max_its, dtype="int32")
    initial = len(np.nonzero(binary_sequence == 2)[0])
    seq = np.array(binary_sequence, dtype="int32")
    c_mp = ct.CDLL(os.path.join(REF_DIR, "message_passing.so"))
    it = c_mp.message_passing(seq.ctypes.data_as(ct.POINTER(ct.c_int)), ct.c_int(max_its),
                              variable_lookup.ctypes.data_as(ct.POINTER(ct.c_int)),
                              check_lookup.ctypes.data_as(ct.POINTER(ct.c_int)),
                              errors.ctypes.data_as(ct.POINTER(ct.c_int)),
                              ct.c_int(n), ct.c_int(k), ct.c_int(dv), ct.c_int(dc))
    return seq, np.insert(errors, 0, initial), it


def ref_ml_system(parity_check, word, n, dv, dc):
    """Drive _ref/ml_decoder.so as parallel_simulator.py:72-88 does.
    Returns (target[m] uint8, remaining[ne, m] uint8) before the transpose."""
    k = int(n * (dc - dv) / dc)
    ne = int(np.count_nonzero(np.asarray(word) == 2))
    seq = np.array(word, dtype="int32")
    target = np.zeros(n - k, dtype="bool")
    rem = np.zeros(max(ne, 1) * (n - k), dtype="bool")
    H = np.ascontiguousarray(parity_check, dtype="bool")
    lib_ = ct.CDLL(os.path.join(REF_DIR, "ml_decoder.so"))
    lib_.ml_decode(seq.ctypes.data_as(ct.POINTER(ct.c_int)), target.ctypes.data_as(ct.POINTER(ct.c_bool)),
                   H.ctypes.data_as(ct.POINTER(ct.c_bool)), rem.ctypes.data_as(ct.POINTER(ct.c_bool)),
                   ct.c_int(n), ct.c_int(dv), ct.c_int(dc))
    return target.astype(np.uint8), rem[: ne * (n - k)].astype(np.uint8).reshape(ne, n - k)


def ref_srand(seed):
    """Seed glibc's rand() -- the stream the reference generator draws from (it seeds only on
    first_run, random_code_generator.c:22-25) -- so reference samples do not depend on how many
    rand() calls earlier code in the process made."""
    ct.CDLL(None).srand(ct.c_uint(seed))


def ref_generate_random_code(n, dv, dc):
    """Drive _ref/random_code_generator.so with the 10-argument call of
    parallel_simulator_expurgated.py:201-223 (first_run=False: glibc rand() stream,
    deterministic per process once ref_srand has seeded it).  Returns (check_lookup,
    variable_lookup, H)."""
    k = int(n * (dc - dv) / dc)
    lib_ = ct.CDLL(os.path.join(REF_DIR, "random_code_generator.so"))
    check_lookup = np.zeros(n * dv, dtype="int32")
    variable_lookup = np.zeros(n * dv, dtype="int32")
    parity_check = np.zeros(n * (n - k), dtype="bool")
    success = 0
    while success == 0:
        sequence = np.arange(n * dv, dtype="int32")
        parity_check[:] = False
        success = lib_.generate_random_code(
            ct.c_int(n), ct.c_int(dv), ct.c_int(dc),
            variable_lookup.ctypes.data_as(ct.POINTER(ct.c_int)),
            check_lookup.ctypes.data_as(ct.POINTER(ct.c_int)),
            sequence.ctypes.data_as(ct.POINTER(ct.c_int)),
            parity_check.ctypes.data_as(ct.POINTER(ct.c_bool)),
            ct.c_int(0), ct.c_bool(False), ct.c_int(0))
    return check_lookup, variable_lookup, parity_check.reshape(n - k, n)


def ref_bench_available():
    return os.path.exists(os.path.join(REF_DIR, "ref_bench.so"))


def ref_bench_message_passing(words, iterations, check_lookup, variable_lookup, n, k, dv, dc, threads):
    """The reference's own message_passing() (compiled unchanged into _ref/ref_bench.so) over a
    batch of words, one call per word, OpenMP over words (oracle/ref_bench.c).
    Returns (words_int32 [B, n], errors [B, iterations], its [B], threads_used)."""
    lib_ = ct.CDLL(os.path.join(REF_DIR, "ref_bench.so"))
    P, i = ct.c_void_p, ct.c_int
    lib_.ref_bench_message_passing.argtypes = [P, i, i, P, P, P, P, i, i, i, i, i]
    lib_.ref_bench_message_passing.restype = i
    w = np.ascontiguousarray(words, dtype=np.int32).copy()
    B = w.shape[0]
    v2c = np.ascontiguousarray(variable_lookup, dtype=np.int32).ravel()
    c2v = np.ascontiguousarray(check_lookup, dtype=np.int32).ravel()
    err = np.zeros((B, iterations), np.int32)
    its = np.zeros(B, np.int32)
    used = lib_.ref_bench_message_passing(_p(w), B, iterations, _p(v2c), _p(c2v), _p(err), _p(its),
                                          n, k, dv, dc, int(threads))
    return w, err, its, used


def ref_bench_timed(words, iterations, check_lookup, variable_lookup, n, k, dv, dc, threads, seconds):
    """Time ref_bench_message_passing over chunks of `words` for ~`seconds` (call in a fresh
    process: bench.py spawns one, so the OpenMP team is not confined by the parent's GPU /
    torch runtime threads).  Returns (words decoded, elapsed s, OpenMP threads used)."""
    import time
    chunk = 64 * max(int(threads), 1)
    done, i, used = 0, 0, 0
    t0 = time.perf_counter()
    while True:
        lo = (i * chunk) % words.shape[0]
        sl = words[lo:lo + chunk] if lo + chunk <= words.shape[0] else words[:chunk]
        used = ref_bench_message_passing(sl, iterations, check_lookup, variable_lookup, n, k, dv, dc, threads)[3]
        done += sl.shape[0]
        i += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            return done, el, used
