"""Second, independent restatement of the ML ("optimal") erasure decoder of
parallel_simulator.py:60-129 in numpy, used only to cross-check the C oracle
(oracle_ml_decode) on small cases.  galois is not installed here, so its
GF(2) ``row_reduce(ncols)`` is restated as well (pivot = first row at or below
the current pivot row with a 1, rows swapped, the column cleared in every other
row, stop when the pivot row runs off the bottom).  Test infrastructure only.
"""
import numpy as np


def row_reduce(M, ncols):
    M = np.array(M, dtype=np.uint8) & 1
    rows = M.shape[0]
    p = 0
    for j in range(ncols):
        if p == rows:
            break
        nz = np.nonzero(M[p:, j])[0]
        if nz.size == 0:
            continue
        i = p + int(nz[0])
        M[[p, i]] = M[[i, p]]
        others = np.nonzero(M[:, j])[0]
        others = others[others != p]
        M[others] ^= M[p]
        p += 1
    return M


def optimal_decode(H, word, cap=1000):
    """Returns (decoded word with 2 = unsolvable, number of 2s)."""
    H = np.asarray(H, np.uint8)
    word = np.asarray(word).astype(np.int64)
    m = H.shape[0]
    erased = word == 2
    ne = int(erased.sum())
    if ne == 0 or ne > m:
        return word.copy(), ne
    known = ~erased
    target = (H[:, known].astype(np.int64) @ word[known]) % 2
    A = H[:, erased]
    positions = list(np.nonzero(erased)[0])
    R = row_reduce(np.c_[A, target], ne)
    unsolvable = []
    while True:
        left = ne - len(unsolvable)
        diag = np.diagonal(R[:, :-1])
        if np.count_nonzero(diag == 1) == left or len(unsolvable) >= cap:
            break
        bad = np.nonzero(diag != 1)[0]
        f = int(bad[0]) if bad.size else diag.size  # reference raises IndexError when bad is empty
        unsolvable.append(positions.pop(f))
        drop = np.nonzero(A[:, f])[0]
        A = np.delete(np.delete(A, drop, axis=0), f, axis=1)
        target = np.delete(target, drop)
        R = row_reduce(np.c_[A, target], left - 1)
    solved = list(R[: ne - len(unsolvable), -1])
    out = word.copy()
    for v in np.nonzero(erased)[0]:
        out[v] = 2 if v in unsolvable else solved.pop(0)
    return out, int(np.count_nonzero(out == 2))
