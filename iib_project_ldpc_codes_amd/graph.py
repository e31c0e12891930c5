"""Tanner graphs in the reference's edge-list format and their device handles.

Edge-list contract (random_code_generator.c:34-36, :53-64):
  * ``check_lookup`` (check_to_variable_list), int32[(n-k)*dc], check-major:
    the dc variables of check c at [c*dc, c*dc+dc) (socket order, unsorted);
  * ``variable_lookup`` (variable_to_check_list), int32[n*dv], variable-major:
    the dv checks of variable v in ascending order.
"""
import ctypes as ct

import numpy as np

from . import _native


class TannerGraph:
    """A regular (dv, dc) graph (or an irregular CSR graph) plus its device copy."""

    def __init__(self, variable_to_check_list, check_to_variable_list, n, k, dv, dc):
        self.n, self.k, self.dv, self.dc = int(n), int(k), int(dv), int(dc)
        self.m = self.n - self.k
        self.variable_lookup = np.ascontiguousarray(variable_to_check_list, dtype=np.int32).ravel()
        self.check_lookup = np.ascontiguousarray(check_to_variable_list, dtype=np.int32).ravel()
        if self.variable_lookup.size != self.n * self.dv or self.check_lookup.size != self.m * self.dc:
            raise ValueError("edge lists do not match (n, k, dv, dc)")
        self.csr = None
        self._handles = {}

    # ------------------------------------------------------------------ ctors
    @classmethod
    def from_csr(cls, check_ptr, check_var, var_ptr, var_slot):
        """Irregular graph in CSR slot form (ldpc_graph_create_csr)."""
        g = cls.__new__(cls)
        g.csr = tuple(np.ascontiguousarray(a, dtype=np.int32) for a in (check_ptr, check_var, var_ptr, var_slot))
        g.m = g.csr[0].size - 1
        g.n = g.csr[2].size - 1
        g.k = g.n - g.m
        g.dv = g.dc = 0
        g.variable_lookup = g.check_lookup = None
        g._handles = {}
        return g

    @classmethod
    def from_parity_check(cls, H, dv=None, dc=None):
        """Lists derived from a dense H as parallel_simulator.py:132-142 does."""
        H = np.asarray(H)
        m, n = H.shape
        check = [np.nonzero(row == 1)[0] for row in H]
        var = [np.nonzero(col == 1)[0] for col in H.T]
        dc = dc or len(check[0])
        dv = dv or len(var[0])
        return cls(np.array(var, np.int32), np.array(check, np.int32), n, n - m, dv, dc)

    @classmethod
    def random_regular(cls, n, dv, dc, seed=0, max_retries=10000, distinct_columns=False):
        """Configuration-model (dv, dc) graph with the law of random_code_generator.c:21-67:
        uniform socket permutation, check_lookup[i] = socket // dv, whole-graph redraw
        whenever a check holds a variable twice, variable_lookup in ascending check order.
        distinct_columns=True also redraws graphs with two identical columns (weight-2
        codewords), as random_code_generator_python.py:4-54 does.
        Randomness: numpy PCG64 seeded by ``seed`` (the reference uses libc rand())."""
        k = int(n * (dc - dv) / dc)
        m = n - k
        if m * dc != n * dv:
            raise ValueError("n*dv must equal (n-k)*dc for a regular graph")
        rng = np.random.default_rng(seed)
        for _ in range(max_retries + 1):
            chk = (rng.permutation(n * dv) // dv).astype(np.int32)
            rows = np.sort(chk.reshape(m, dc), axis=1)
            if dc > 1 and np.any(rows[:, 1:] == rows[:, :-1]):
                continue
            checks = np.repeat(np.arange(m, dtype=np.int32), dc)
            order = np.lexsort((checks, chk))  # by variable, then ascending check
            var = checks[order].astype(np.int32)
            if distinct_columns and np.unique(var.reshape(n, dv), axis=0).shape[0] != n:
                continue
            return cls(var, chk, n, k, dv, dc)
        raise RuntimeError("random_regular: too many redraws")

    @classmethod
    def sample_device(cls, n, dv, dc, seed=0, graph_id=0):
        """Graph `graph_id` of the on-device sampler (ldpc_sample_regular; same law as
        random_code_generator.c, counter-based so any graph can be regenerated)."""
        k = int(n * (dc - dv) / dc)
        chk = np.zeros(n * dv, np.int32)
        var = np.zeros(n * dv, np.int32)
        att = np.zeros(1, np.int32)
        rc = _native.lib().ldpc_sample_regular(n, dv, dc, int(seed), int(graph_id), 1, chk.ctypes.data,
                                               var.ctypes.data, att.ctypes.data)
        _native.check(rc, "ldpc_sample_regular")
        if att[0] <= 0:
            raise RuntimeError("sampler hit its attempt cap")
        return cls(var, chk, n, k, dv, dc)

    # ---------------------------------------------------------------- helpers
    @property
    def num_edges(self):
        return int(self.csr[0][-1]) if self.csr is not None else self.m * self.dc

    def parity_check(self):
        """Dense H (only for small graphs / tests)."""
        H = np.zeros((self.m, self.n), np.uint8)
        if self.csr is not None:
            cptr, cvar = self.csr[0], self.csr[1]
            for c in range(self.m):
                H[c, cvar[cptr[c]:cptr[c + 1]]] ^= 1
        else:
            for c in range(self.m):
                for v in self.check_lookup[c * self.dc:(c + 1) * self.dc]:
                    H[c, v] ^= 1
        return H

    def handle(self):
        """Device graph (ldpc_graph*) on the current HIP device, created once."""
        L = _native.lib()
        dev = 0
        try:
            import torch
            if torch.cuda.is_available():
                dev = torch.cuda.current_device()
        except Exception:
            pass
        h = self._handles.get(dev)
        if h is not None:
            return h
        out = ct.c_void_p()
        if self.csr is not None:
            cp, cv, vp, vs = self.csr
            rc = L.ldpc_graph_create_csr(cp.ctypes.data, cv.ctypes.data, vp.ctypes.data, vs.ctypes.data,
                                         self.n, self.m, ct.byref(out))
        else:
            rc = L.ldpc_graph_create(self.variable_lookup.ctypes.data, self.check_lookup.ctypes.data,
                                     self.n, self.k, self.dv, self.dc, ct.byref(out))
        _native.check(rc, "ldpc_graph_create")
        self._handles[dev] = out
        return out

    def kernel_name(self, early_stop=False, hard_only=False):
        """The soft kernel a decode of this graph runs (hard_only: early stop without posteriors)."""
        es = (2 if hard_only else 1) if early_stop else 0
        return _native.lib().ldpc_bp_kernel_name(self.handle(), es).decode()

    def __del__(self):
        try:
            if _native._lib is not None:
                for h in self._handles.values():
                    _native._lib.ldpc_graph_destroy(h)
        except Exception:
            pass
        self._handles = {}

    def to_csr(self):
        """(check_ptr, check_var, var_ptr, var_slot) for a regular list graph."""
        if self.csr is not None:
            return self.csr
        n, m, dv, dc = self.n, self.m, self.dv, self.dc
        vslot = np.empty(n * dv, np.int32)
        # slot of v in check c: the r-th occurrence for the r-th repeat of c in v's list
        for v in range(n):
            seen = {}
            for j in range(dv):
                c = int(self.variable_lookup[v * dv + j])
                r = seen.get(c, 0)
                seen[c] = r + 1
                hits = np.nonzero(self.check_lookup[c * dc:(c + 1) * dc] == v)[0]
                if r >= hits.size:
                    raise ValueError("edge lists disagree")
                vslot[v * dv + j] = c * dc + hits[r]
        cptr = np.arange(m + 1, dtype=np.int32) * dc
        vptr = np.arange(n + 1, dtype=np.int32) * dv
        return cptr, self.check_lookup.copy(), vptr, vslot
