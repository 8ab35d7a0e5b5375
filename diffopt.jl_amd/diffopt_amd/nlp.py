"""NonLinearProgram back-end on the MI355X engine.

Mirrors the KKT part of ``DiffOpt.NonLinearProgram`` (reference
``src/NonLinearProgram/``): the caller evaluates the model's derivatives at
the solution (the reference's MOI Nonlinear evaluator,
``_compute_optimal_hess_jac``, nlp_utilities.jl:35-92) and the engine builds
the sIpopt KKT system, factorises it with the reference's inertia correction
and solves:

* ``NLPBatch.set_structure`` / ``set`` — ``_compute_solution_and_bounds`` +
  ``_build_sensitivity_matrices`` inputs (nlp_utilities.jl:181-396);
* ``factor`` — ``_lu_with_inertia_correction`` (NonLinearProgram.jl:394-422);
* ``forward`` — ``forward_differentiate!`` (:502-528): Δp → Δx, Δdual;
* ``reverse`` — ``reverse_differentiate!`` (:530-582): Δx, Δdual → Δp;
* ``jacobian`` — ``_compute_sensitivity``'s ∂s (nlp_utilities.jl:457-500);
* ``set_kkt`` / ``kkt_solve`` — the ``NonLinearKKTJacobianFactorization``
  plug point: a given M factorised, ``K \\ N`` for many right-hand sides.

Arrays: numpy (host, copied into HBM) or torch CUDA tensors (zero-copy), with
the usual C-order shapes ``(B, rows, cols)``.
"""

import ctypes

import numpy as np

from . import _lib
from ._arrays import Staged, colmajor, vector

EQ, GEQ, LEQ = 0, 1, 2


class NLPBatch:
    """Batched NLP KKT sensitivity engine (C-ABI handle wrapper): ``n``
    primal variables, ``c`` NLP constraints, ``P`` parameters per problem."""

    def __init__(self, batch, n, c, P, device=0, deferred=False):
        self.lib = _lib.load()
        self.batch, self.n, self.c, self.P = int(batch), int(n), int(c), int(P)
        h = ctypes.c_void_p()
        rc = self.lib.dopt_create(ctypes.byref(h), device, self.batch, self.n, self.c, self.P,
                                  _lib.DOPT_KIND_NLP)
        if rc != 0:
            raise _lib.EngineError(rc, "dopt_create failed (no HIP device?)")
        self.h = h
        self._mem = None
        self._keep = None
        self._layout = None
        # opt-in: factor() returns with the LU queued (dopt_nlp_set_deferred)
        if deferred:
            _lib.check(self.lib.dopt_nlp_set_deferred(self.h, 1), self.h)

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

    # ---- structure and point ----------------------------------------------
    def set_structure(self, con_kind, has_low=None, has_up=None, sense=1):
        """con_kind[c]: 0 EqualTo, 1 GreaterThan, 2 LessThan (NLP constraint
        order); has_low / has_up[n]: variable bounds; sense +1 MIN / −1 MAX."""
        ck = np.ascontiguousarray(np.asarray(con_kind, dtype=np.int32).reshape(self.c))
        lo = np.ascontiguousarray(np.zeros(self.n, np.int8) if has_low is None else
                                  np.asarray(has_low, dtype=np.int8).reshape(self.n))
        up = np.ascontiguousarray(np.zeros(self.n, np.int8) if has_up is None else
                                  np.asarray(has_up, dtype=np.int8).reshape(self.n))
        rc = self.lib.dopt_nlp_set_structure(self.h, ck.ctypes.data, lo.ctypes.data, up.ctypes.data, int(sense))
        _lib.check(rc, self.h)
        self._layout = None

    def set(self, Hxx, Hxp, Jx, Jp, x, cval, crhs, y, xl=None, xu=None, yl=None, yu=None):
        """The point: Hessian of f − sense·yᵀc (Hxx (B,n,n), Hxp (B,n,P)),
        constraint Jacobian (Jx (B,c,n), Jp (B,c,P)), x (B,n), constraint values
        and set constants (B,c), duals y (B,c) and bound data (B,n), all in
        MOI's ConstraintDual convention."""
        B, n, c, P = self.batch, self.n, self.c, self.P
        st = self._stage([Hxx, Hxp, Jx, Jp, x, cval, crhs, y, xl, xu, yl, yu])
        args = [colmajor(Hxx, (B, n, n)), colmajor(Hxp, (B, n, P)) if P else None,
                colmajor(Jx, (B, c, n)) if c else None, colmajor(Jp, (B, c, P)) if (c and P) else None,
                vector(x, (B, n)), vector(cval, (B, c)) if c else None, vector(crhs, (B, c)) if c else None,
                vector(y, (B, c)) if c else None]
        args += [vector(a, (B, n)) if a is not None else None for a in (xl, xu, yl, yu)]
        self._keep = args
        rc = self.lib.dopt_nlp_set(self.h, *[st.ptr(a) for a in args])
        _lib.check(rc, self.h)

    def set_kkt(self, M, num_w, num_cons):
        """KKT mode: M (B, rows, rows) given; num_w / num_cons set the inertia
        correction's D (+1, −1 on rows num_w … num_w+num_cons−1)."""
        M = M if not isinstance(M, list) else np.asarray(M)
        rows = int(M.shape[-1])
        st = self._stage([M])
        Mc = colmajor(M, (self.batch, rows, rows))
        self._keep = [Mc]
        rc = self.lib.dopt_nlp_set_kkt(self.h, rows, int(num_w), int(num_cons), st.ptr(Mc))
        _lib.check(rc, self.h)
        self._layout = None

    def factor(self):
        _lib.check(self.lib.dopt_nlp_factor(self.h), self.h)

    def corrections(self):
        """Inertia corrections per problem: 0 none, k > 0, −1 failed (∂s = 0)."""
        out = np.zeros(self.batch, dtype=np.int32)
        _lib.check(self.lib.dopt_nlp_get_corrections(self.h, out.ctypes.data), self.h)
        return out

    def layout(self):
        if self._layout is None:
            v = np.zeros(7, dtype=np.int32)
            _lib.check(self.lib.dopt_nlp_get_layout(self.h, v.ctypes.data), self.h)
            keys = ("rows", "num_w", "c", "nlo", "nup", "nlow_primal", "nup_primal")
            self._layout = dict(zip(keys, (int(e) for e in v)))
        return self._layout

    @property
    def ndual(self):
        lay = self.layout()
        return self.c + lay["nlow_primal"] + lay["nup_primal"]

    def system_size(self):
        """Per-problem size of the factorised system: n + c on the reduced
        route (bounds and slacks eliminated exactly), the rows of M on the
        full one (inertia corrections, degenerate bounds, DOPT_NLP_REDUCE=0)."""
        buf = np.zeros(self.batch, dtype=np.int32)
        _lib.check(self.lib.dopt_get_system_size(self.h, buf.ctypes.data), self.h)
        return buf

    def lu_kind(self):
        """Per-problem factorisation kind (the shared blocked LU):
        _lib.LU_KIND_NOPIV / LU_KIND_PIVOT."""
        buf = np.zeros(self.batch, dtype=np.int8)
        _lib.check(self.lib.dopt_qp_get_lu_kind(self.h, buf.ctypes.data), self.h)
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
        """{phase name: (total ms, launches)} since the last call; the NLP path
        reports under the shared QP phase names (assembly, LU, solve, …)."""
        return _lib.phase_times(self.lib, self.h)

    # ---- sensitivities -----------------------------------------------------
    def forward(self, dp):
        """Δp (B, P) → (Δx (B, n), Δdual (B, c + nlow + nup))."""
        B = self.batch
        st = self._stage([dp])
        dev = st.mem == _lib.DOPT_MEM_DEVICE
        d = vector(dp, (B, self.P)) if self.P else None
        dx = Staged.empty((B, self.n), dev)
        dd = Staged.empty((B, self.ndual), dev)
        rc = self.lib.dopt_nlp_forward(self.h, st.ptr(d), st.ptr(dx), st.ptr(dd))
        _lib.check(rc, self.h)
        return dx, dd

    def reverse(self, dx=None, ddual=None):
        """Δx (B, n) and Δdual (B, c + nlow + nup) seeds (None = 0) → Δp (B, P)."""
        B = self.batch
        st = self._stage([dx, ddual])
        dev = st.mem == _lib.DOPT_MEM_DEVICE
        a = vector(dx, (B, self.n)) if dx is not None else None
        b = vector(ddual, (B, self.ndual)) if ddual is not None else None
        out = Staged.empty((B, self.P), dev)
        rc = self.lib.dopt_nlp_reverse(self.h, st.ptr(a), st.ptr(b), st.ptr(out))
        _lib.check(rc, self.h)
        return out

    def forward_reverse(self, dp, dx=None, ddual=None):
        """forward(dp) and reverse(dx, ddual) against the same factors in one
        call (dopt_nlp_forward_reverse: one pass over the factors for both
        directions) → (Δx, Δdual, Δp)."""
        B = self.batch
        st = self._stage([dp, dx, ddual])
        dev = st.mem == _lib.DOPT_MEM_DEVICE
        d = vector(dp, (B, self.P)) if self.P else None
        a = vector(dx, (B, self.n)) if dx is not None else None
        b = vector(ddual, (B, self.ndual)) if ddual is not None else None
        ox = Staged.empty((B, self.n), dev)
        od = Staged.empty((B, self.ndual), dev)
        op = Staged.empty((B, self.P), dev)
        rc = self.lib.dopt_nlp_forward_reverse(self.h, st.ptr(d), st.ptr(a), st.ptr(b), st.ptr(ox), st.ptr(od),
                                               st.ptr(op))
        _lib.check(rc, self.h)
        return ox, od, op

    def jacobian(self, device=False):
        """∂s (B, rows, P) — the reference's Δs per problem."""
        rows = self.layout()["rows"]
        out = Staged.empty((self.batch, self.P, rows), device)   # column-major rows × P
        if device and self._mem != _lib.DOPT_MEM_DEVICE:
            raise TypeError("jacobian(device=True) needs the handle in device mode (set with CUDA tensors)")
        rc = self.lib.dopt_nlp_jacobian(self.h, Staged.ptr(out))
        _lib.check(rc, self.h)
        return out.transpose(1, 2) if device else np.swapaxes(out, 1, 2)

    def kkt_solve(self, rhs):
        """KKT mode: x = K \\ rhs, rhs (k, B, rows) (or (B, rows)) → same shape."""
        squeeze = rhs.ndim == 2
        r = rhs[None] if squeeze else rhs
        k = int(r.shape[0])
        rows = int(r.shape[-1])
        st = self._stage([r])
        rr = vector(r, (k, self.batch, rows))
        out = Staged.empty((k, self.batch, rows), st.mem == _lib.DOPT_MEM_DEVICE)
        rc = self.lib.dopt_nlp_kkt_solve(self.h, k, st.ptr(rr), st.ptr(out))
        _lib.check(rc, self.h)
        return out[0] if squeeze else out
