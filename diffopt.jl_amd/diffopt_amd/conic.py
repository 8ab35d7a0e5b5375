"""ConicProgram back-end on the MI355X engine.

Mirrors ``DiffOpt.ConicProgram`` (reference ``src/ConicProgram/ConicProgram.jl``):

* ``ConicBatch`` — batched C-ABI handle: geometric form ``A x + b ∈ K`` in MOI
  convention (the diffcp sign flip is applied by the engine), cone table in
  ``ProductOfSets`` row order, primal ``x``, slack ``s``, dual ``y``.
* ``Model`` — single problem with the reference vocabulary:
  ``forward_differentiate`` (:257-334), ``reverse_differentiate`` (:336-394),
  ``ForwardVariablePrimal`` (:403-412), ``ReverseObjectiveFunction``
  (:396-401), ``ReverseConstraintFunction`` (``_get_dA``/``_get_db``
  :414-443), and MAX-sense handling of ``c`` (:206-208).
"""

import ctypes
import time

import numpy as np

from . import _lib
from ._arrays import Staged, colmajor, vector

ZEROS, NONNEG, NONPOS, SOC, PSD = (_lib.CONE_ZEROS, _lib.CONE_NONNEG, _lib.CONE_NONPOS,
                                   _lib.CONE_SOC, _lib.CONE_PSD_TRI)


class ConicBatch:
    def __init__(self, batch, n, cones, device=0, sparse=False):
        self.lib = _lib.load()
        self.cones = [(int(c), int(d)) for c, d in cones]
        self.batch, self.n = int(batch), int(n)
        self.m = sum(d for _, d in self.cones)
        h = ctypes.c_void_p()
        rc = self.lib.dopt_create(ctypes.byref(h), device, self.batch, self.n, self.m, 0,
                                  _lib.DOPT_KIND_CONIC)
        if rc != 0:
            raise _lib.EngineError(rc, "dopt_create failed (no HIP device?)")
        self.h = h
        self._mem = None
        self._keep = None
        # the sparse route (dopt_set_sparse): set_csc keeps A_moi sparse, LSQR matrix-free on it
        self.sparse = bool(sparse)
        if sparse:
            _lib.check(self.lib.dopt_set_sparse(self.h, 1), self.h)

    def close(self):
        if getattr(self, "h", None):
            self.lib.dopt_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def _stage(self, arrays):
        st = Staged(arrays)
        if self._mem != st.mem:
            _lib.check(self.lib.dopt_set_memory(self.h, st.mem), self.h)
            self._mem = st.mem
        if st.set_stream and st.stream != getattr(self, "_stream", -1):
            _lib.check(self.lib.dopt_set_stream(self.h, st.stream), self.h)
            self._stream = st.stream
        return st

    @property
    def N(self):
        return self.n + self.m + 1

    def set(self, A, b, c, x, s, y):
        """``A``: (B, m, n) MOI coefficients; ``c`` already sign-adjusted for MAX."""
        B, n, m = self.batch, self.n, self.m
        st = self._stage([A, b, c, x, s, y])
        args = [colmajor(A, (B, m, n)), vector(b, (B, m)), vector(c, (B, n)),
                vector(x, (B, n)), vector(s, (B, m)), vector(y, (B, m))]
        self._keep = args
        desc = np.array([v for cd in self.cones for v in cd], dtype=np.int32)
        rc = self.lib.dopt_conic_set(self.h, *[st.ptr(a) for a in args],
                                     desc.ctypes.data if desc.size else None, len(self.cones))
        _lib.check(rc, self.h)

    def set_csc(self, A, b, c, x, s, y):
        """``set`` with ``A`` (MOI coefficients, m × n) as scipy.sparse — one per
        problem or one shared — passed as Julia CSC arrays (Int64, 1-based) to
        dopt_conic_set_csc, which densifies on the device.  Host mode."""
        import scipy.sparse as sp
        B, n, m = self.batch, self.n, self.m
        mats = [A] * B if sp.issparse(A) else list(A)
        cps, rvs, nzs, off = [], [], [], 0
        for M in mats:
            M = sp.csc_matrix(M)
            if M.shape != (m, n):
                raise ValueError(f"sparse A of shape {M.shape}, expected {(m, n)}")
            cps.append(M.indptr.astype(np.int64) + off + 1)
            rvs.append(M.indices.astype(np.int64) + 1)
            nzs.append(M.data.astype(np.float64))
            off += M.nnz
        cp = np.ascontiguousarray(np.concatenate(cps))
        rv = np.ascontiguousarray(np.concatenate(rvs))
        nz = np.ascontiguousarray(np.concatenate(nzs))
        st = self._stage([b, c, x, s, y])
        if st.mem != _lib.DOPT_MEM_HOST:
            raise TypeError("set_csc takes host (numpy / scipy) arrays")
        vecs = [vector(b, (B, m)), vector(c, (B, n)), vector(x, (B, n)), vector(s, (B, m)),
                vector(y, (B, m))]
        desc = np.array([v for cd in self.cones for v in cd], dtype=np.int32)
        rc = self.lib.dopt_conic_set_csc(self.h, cp.ctypes.data, rv.ctypes.data if off else None,
                                         nz.ctypes.data if off else None, off,
                                         *[st.ptr(v) for v in vecs],
                                         desc.ctypes.data if desc.size else None, len(self.cones))
        _lib.check(rc, self.h)

    def factor(self):
        _lib.check(self.lib.dopt_conic_factor(self.h), self.h)

    def forward(self, dA=None, db=None, dc=None):
        """Returns (out (B, N) = [du | dv | dw], dx (B, n) = ForwardVariablePrimal)."""
        B, n, m = self.batch, self.n, self.m
        st = self._stage([dA, db, dc])
        dev = st.mem == _lib.DOPT_MEM_DEVICE
        args = [colmajor(dA, (B, m, n)) if dA is not None else None,
                vector(db, (B, m)) if db is not None else None,
                vector(dc, (B, n)) if dc is not None else None]
        out = Staged.empty((B, self.N), dev)
        dx = Staged.empty((B, n), dev)
        rc = self.lib.dopt_conic_forward(self.h, *[st.ptr(a) for a in args], st.ptr(out), st.ptr(dx))
        _lib.check(rc, self.h)
        return out, dx

    def reverse(self, dx, want_dA=True):
        """Returns (g (B, N), dA (B, m, n) | None, db (B, m), dc (B, n))."""
        B, n, m = self.batch, self.n, self.m
        st = self._stage([dx])
        dev = st.mem == _lib.DOPT_MEM_DEVICE
        d = vector(dx, (B, n))
        g = Staged.empty((B, self.N), dev)
        dA = Staged.empty((B, n, m), dev) if want_dA else None   # column-major (m×n)
        db = Staged.empty((B, m), dev)
        dc = Staged.empty((B, n), dev)
        rc = self.lib.dopt_conic_reverse(self.h, st.ptr(d), st.ptr(g), st.ptr(dA), st.ptr(db),
                                         st.ptr(dc))
        _lib.check(rc, self.h)
        if dA is not None:
            dA = dA.transpose(0, 2, 1) if not dev else dA.transpose(1, 2)
        return g, dA, db, dc

    def forward_reverse(self, dx, dA=None, db=None, dc=None, want_dA=True):
        """Both directions in one call, the two LSQR runs co-iterated
        (dopt_conic_forward_reverse): ((out, dx_fwd), (g, dA, db, dc)) as
        ``forward`` / ``reverse`` return them, bit-identical to those calls."""
        B, n, m = self.batch, self.n, self.m
        st = self._stage([dA, db, dc, dx])
        dev = st.mem == _lib.DOPT_MEM_DEVICE
        args = [colmajor(dA, (B, m, n)) if dA is not None else None,
                vector(db, (B, m)) if db is not None else None,
                vector(dc, (B, n)) if dc is not None else None,
                vector(dx, (B, n))]
        out = Staged.empty((B, self.N), dev)
        fdx = Staged.empty((B, n), dev)
        g = Staged.empty((B, self.N), dev)
        rA = Staged.empty((B, n, m), dev) if want_dA else None
        rb = Staged.empty((B, m), dev)
        rc_ = Staged.empty((B, n), dev)
        rc = self.lib.dopt_conic_forward_reverse(self.h, *[st.ptr(a) for a in args], st.ptr(out), st.ptr(fdx),
                                                 st.ptr(g), st.ptr(rA), st.ptr(rb), st.ptr(rc_))
        _lib.check(rc, self.h)
        if rA is not None:
            rA = rA.transpose(0, 2, 1) if not dev else rA.transpose(1, 2)
        return (out, fdx), (g, rA, rb, rc_)

    def set_maxiter(self, maxiter):
        """Cap LSQR at ``maxiter`` iterations (0: the reference's default
        max(size(M))) — dopt_conic_set_maxiter."""
        _lib.check(self.lib.dopt_conic_set_maxiter(self.h, int(maxiter)), self.h)

    def lsqr_stats(self):
        """(istop, iterations) of the last run and, after ``forward_reverse``,
        of its forward run: dict of (B,) arrays."""
        buf = np.zeros(4 * self.batch, dtype=np.int32)
        _lib.check(self.lib.dopt_conic_lsqr_stats(self.h, buf.ctypes.data), self.h)
        B = self.batch
        return {"istop": buf[:B], "iterations": buf[B:2 * B], "fwd_istop": buf[2 * B:3 * B],
                "fwd_iterations": buf[3 * B:]}

    def lsqr_norms(self):
        """LSQR's terminal estimates (rnorm, arnorm, xnorm, anorm) of the last
        run and, after ``forward_reverse``, of its forward run: dict of (B, 4)
        arrays under "last" and "fwd"."""
        buf = np.zeros(8 * self.batch, dtype=np.float64)
        _lib.check(self.lib.dopt_conic_lsqr_norms(self.h, buf.ctypes.data), self.h)
        B = self.batch
        return {"last": buf[:4 * B].reshape(B, 4), "fwd": buf[4 * B:].reshape(B, 4)}

    def info(self):
        buf = np.zeros(self.batch, dtype=np.int32)
        _lib.check(self.lib.dopt_get_info(self.h, buf.ctypes.data), self.h)
        return buf

    def iterations(self):
        buf = np.zeros(self.batch, dtype=np.int32)
        _lib.check(self.lib.dopt_get_system_size(self.h, buf.ctypes.data), self.h)
        return buf

    def set_profiling(self, on=True, phases=None):
        """Per-phase HIP-event timing on (all phases, or only the phase names
        in `phases`) or off."""
        if phases is None:
            _lib.check(self.lib.dopt_set_profiling(self.h, int(bool(on))), self.h)
        else:
            mask = _lib.phase_mask(self.lib, phases) if on else 0
            _lib.check(self.lib.dopt_set_profiling_phases(self.h, mask), self.h)

    def phase_times(self):
        return _lib.phase_times(self.lib, self.h)


class Model:
    """Single-problem ``DiffOpt.ConicProgram.Model`` on the engine."""

    def __init__(self, device=0):
        self.device = device
        self.empty()

    def empty(self):
        self.A = self.b = self.c = None
        self.cones = []
        self.max_sense = False
        self.x = self.s = self.y = None
        self._engine = None
        self.forw_grad_cache = None
        self.back_grad_cache = None
        self.diff_time = float("nan")
        self.input_dx = {}
        self.input_objective = None
        self.input_constraints = {}   # cone index -> (coeffs (dim×n), constants (dim))

    def set_problem(self, A, b, c, cones, max_sense=False):
        self.A = np.asarray(A, dtype=np.float64)
        self.b = np.asarray(b, dtype=np.float64)
        self.c = np.asarray(c, dtype=np.float64)
        self.cones = [(int(k), int(d)) for k, d in cones]
        self.max_sense = bool(max_sense)
        self._engine = None

    def rows(self, ci):
        o = sum(d for _, d in self.cones[:ci])
        return np.arange(o, o + self.cones[ci][1])

    def set_variable_primal_start(self, x):
        self.x = np.asarray(x, dtype=np.float64)
        self._engine = None

    def set_constraint_primal_start(self, s):
        self.s = np.asarray(s, dtype=np.float64)
        self._engine = None

    def set_constraint_dual_start(self, y):
        self.y = np.asarray(y, dtype=np.float64)
        self._engine = None

    def set_reverse_variable_primal(self, i, value):
        self.input_dx[int(i)] = float(value)

    def set_forward_objective_function(self, dc):
        self.input_objective = np.asarray(dc, dtype=np.float64)

    def set_forward_constraint_function(self, ci, coeffs, constants):
        self.input_constraints[int(ci)] = (np.asarray(coeffs, float), np.asarray(constants, float))

    def _ensure(self):
        m = self.A.shape[0]
        if self.y is None or np.any(np.isnan(self.y)) or len(self.y) < m:
            raise ValueError("Some constraints are missing a value for the "
                             "`ConstraintDualStart` attribute.")
        if self.s is None or np.any(np.isnan(self.s)) or len(self.s) < m:
            raise ValueError("Some constraints are missing a value for the "
                             "`ConstraintPrimalStart` attribute.")
        if self._engine is None:
            e = ConicBatch(1, self.A.shape[1], self.cones, self.device)
            c = -self.c if self.max_sense else self.c
            e.set(self.A[None], self.b[None], c[None], self.x[None], self.s[None], self.y[None])
            self._engine = e
        return self._engine

    def forward_differentiate(self):
        t0 = time.perf_counter()
        e = self._ensure()
        m, n = self.A.shape
        dA = np.zeros((m, n))
        db = np.zeros(m)
        for ci, (cf, k) in self.input_constraints.items():
            r = self.rows(ci)
            dA[r] = cf
            db[r] = k
        dc = np.zeros(n) if self.input_objective is None else self.input_objective
        out, dx = e.forward(dA[None], db[None], dc[None])
        self.forw_grad_cache = (np.asarray(out)[0], np.asarray(dx)[0])
        self.diff_time = time.perf_counter() - t0

    def reverse_differentiate(self):
        t0 = time.perf_counter()
        e = self._ensure()
        dx = np.zeros(self.A.shape[1])
        for i, v in self.input_dx.items():
            dx[i] = v
        g, dA, db, dc = e.reverse(dx[None])
        self.back_grad_cache = tuple(np.asarray(a)[0] for a in (g, dA, db, dc))
        self.diff_time = time.perf_counter() - t0

    def forward_variable_primal(self, i):
        return self.forw_grad_cache[1][i]

    def reverse_objective_function(self):
        return self.back_grad_cache[3].copy()

    def reverse_constraint_function(self, ci):
        """(dA rows, db entries) for constraint ``ci`` (``_get_dA``/``_get_db``)."""
        r = self.rows(ci)
        _, dA, db, _ = self.back_grad_cache
        return dA[r], db[r]

    def differentiate_time_sec(self):
        return self.diff_time
