"""The round rule of the sequential-draw sampler (csrc/sampler.hip) restated in Python and checked
against the sequential definition it must equal (oracle/ldpc_oracle.c seq_attempt): up to 256
slots (two per lane, two waves) drawn per round against the bitmap of the slots before the
round, picks marked by atomic OR in an arbitrary order, and -- when slots picked the same pool
entry -- only the slots below the cut kept: D = the lowest slot that found its bit already set;
t = D when its pick's owner (the slot that set the bit) is below it, else min(owner, the next
such slot); at least the round's first slot (undo every pick, redo the kept ones).  The word stream is a stand-in hash
(the rule, not Philox, is under test); pools compact at ceil(R/2) entries left, the last <= 64
entries are shuffled.  CPU only."""
import hashlib
import random

import pytest

FINAL = 64


def _word(att, x, k):
    return int.from_bytes(hashlib.blake2b(f"{att},{x},{k}".encode(), digest_size=4).digest(), "little")


def _draw(att, x, R, used):
    """First Lemire draw on [0, R) of slot x's stream that misses `used` (None: exhausted)."""
    kw = 0
    while True:
        if kw >= 1024:
            return None
        w = _word(att, x, kw)
        kw += 1
        mm = w * R
        lo = mm & 0xFFFFFFFF
        if lo < R:
            t = ((1 << 32) - R) % R
            while lo < t:
                if kw >= 1024:
                    return None
                w = _word(att, x, kw)
                kw += 1
                mm = w * R
                lo = mm & 0xFFFFFFFF
        i = mm >> 32
        if not used[i]:
            return i


def _final(att, arr):
    rng = random.Random(f"final{att}")
    for a in range(len(arr) - 1, 0, -1):
        j = rng.randrange(a + 1)
        arr[a], arr[j] = arr[j], arr[a]


def sequential(E, var, att):
    out, cur, R, x = [None] * E, list(var), E, 0
    while R > FINAL:
        Rn = (R + 1) // 2
        used = [0] * R
        while x < E - Rn:
            i = _draw(att, x, R, used)
            used[i] = 1
            out[x] = cur[i]
            x += 1
        cur, R = [cur[i] for i in range(R) if not used[i]], Rn
    fin = cur[:]
    _final(att, fin)
    out[x:] = fin
    return out


def rounds(E, var, att, order_rng):
    """The kernel's rounds: thread t of the workgroup owns slots base + 2t, base + 2t + 1
    (base = x0 rounded down to even; slots below x0 are done), i.e. up to 256 slots per round;
    the picks of both waves are marked by atomic ORs in an arbitrary order."""
    out, cur, R, x0, nrounds = [None] * E, list(var), E, 0, 0
    while R > FINAL:
        Rn = (R + 1) // 2
        xend = E - Rn
        bm = [0] * R
        while x0 < xend:
            nrounds += 1
            base = x0 & ~1
            slots = [s for s in range(256) if x0 <= base + s < xend]
            cand = {s: _draw(att, base + s, R, bm) for s in slots}
            order = list(slots)
            order_rng.shuffle(order)
            dup = {}
            for s in order:
                dup[s] = bm[cand[s]] == 1
                bm[cand[s]] = 1
            tend = min(256, xend - base)
            dups = sorted(s for s in slots if dup[s])
            t = min(dups[0], tend) if dups else tend
            if t < tend:
                D = dups[0]  # the lowest slot that found its bit set; its pick's owner set it
                owner = min(s for s in slots if not dup[s] and cand[s] == cand[D])
                d2 = dups[1] if len(dups) > 1 else 256
                t = D if owner < D else min(owner, d2)
                t = min(max(t, x0 - base + 1), tend)  # the round's first slot is always right
                for s in slots:
                    if not dup[s]:
                        bm[cand[s]] = 0
                for s in slots:
                    if s < t:
                        bm[cand[s]] = 1
            for s in slots:
                if s < t:
                    out[base + s] = cur[cand[s]]
            assert base + t > x0  # progress
            x0 = base + t
        cur, R = [cur[i] for i in range(R) if not bm[i]], Rn
    fin = cur[:]
    _final(att, fin)
    out[x0:] = fin
    return out, nrounds


@pytest.mark.parametrize("E", [300, 3000, 12000])
def test_round_rule_equals_sequential_draws(E):
    var = [s // 3 for s in range(E)]
    for att in range(3):
        want = sequential(E, var, att)
        for order_seed in range(2):
            got, nr = rounds(E, var, att, random.Random(1000 * att + order_seed))
            assert got == want
            assert nr >= E // 256
        assert sorted(want) == sorted(var)  # a permutation of the sockets' variables
