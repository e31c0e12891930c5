"""Test graphs that the ensembles module does not draw."""
import numpy as np


def check6_var24(m, seed=0):
    """Check-regular degree-6 rate-1/2 graph with variable degrees {2, 4}: n = 2m, variables
    0..m-1 of degree 2 on a ring (variable i joins checks i and i+1 mod m, so every check can
    take a degree-2 variable as its slot-0 local edge), variables m..2m-1 of degree 4 on
    random checks (4 sockets per check, no repeated check per variable).  Its local-edge
    layout has every check at degree 6 but DVN = 3 -- the shape that must run on the RSU
    instantiation of bp_loc_kernel, not the (3,6) one (advisor round 2)."""
    from iib_project_ldpc_codes_amd.ensembles import _csr_from_pairs
    rng = np.random.default_rng(seed)
    sock = np.repeat(np.arange(m), 4)
    rng.shuffle(sock)
    rows = sock.reshape(m, 4)
    for _ in range(1000):
        bad = [j for j in range(m) if len(set(rows[j])) < 4]
        if not bad:
            break
        for j in bad:  # swap one socket of the offending variable with a random socket
            a, b = rng.integers(4), rng.integers(m)
            c = rng.integers(4)
            rows[j, a], rows[b, c] = rows[b, c], rows[j, a]
    assert all(len(set(r)) == 4 for r in rows)
    pairs = [(i, i) for i in range(m)] + [(i, (i + 1) % m) for i in range(m)]
    pairs += [(m + j, int(c)) for j in range(m) for c in rows[j]]
    return _csr_from_pairs(2 * m, m, np.full(m, 6, np.int32), pairs)
