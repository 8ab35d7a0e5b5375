"""QuadraticProgram back-end on the MI355X engine.

Mirrors ``DiffOpt.QuadraticProgram`` (reference
``src/QuadraticProgram/QuadraticProgram.jl``):

* ``QPBatch`` — the batched C-ABI handle (one KKT system per problem, all
  problems of one shape).  Accepts numpy arrays (host memory, copied into HBM)
  or torch CUDA tensors (device memory, zero-copy, inputs resident in HBM).
* ``Model`` — a single-problem model with the reference's plugin-interface
  vocabulary: ``VariablePrimalStart``/``ConstraintDualStart`` setters with the
  dual sign flip (:164-180), ``ReverseVariablePrimal`` inputs,
  ``reverse_differentiate`` (:316-351), ``forward_differentiate`` (:357-446),
  ``ForwardVariablePrimal`` (:299-305), ``ReverseObjectiveFunction``
  (:448-458), ``ReverseConstraintFunction`` (``_get_dA``/``_get_db``
  :307-314, :461-473) and ``DifferentiateTimeSec``.
"""

import ctypes

import numpy as np

from . import _lib
from ._arrays import Staged, colmajor, vector
from ._arrays import _is_torch as _is_t

LE, EQ = "LessThan", "EqualTo"


def _check_out(o, shape, device):
    """A caller-supplied output buffer must be exactly what the kernels write:
    float64, C-contiguous, `shape`, and in the memory kind of the call."""
    if _is_t(o):
        import torch
        ok = (o.dtype == torch.float64 and o.is_contiguous() and tuple(o.shape) == tuple(shape)
              and o.is_cuda == bool(device))
    else:
        ok = (not device and isinstance(o, np.ndarray) and o.dtype == np.float64
              and o.flags.c_contiguous and o.shape == tuple(shape))
    if not ok:
        raise TypeError(f"output buffer must be a C-contiguous float64 {'CUDA tensor' if device else 'numpy array'} "
                        f"of shape {tuple(shape)}")


class QPBatch:
    """Batched QP sensitivity engine (C-ABI handle wrapper)."""

    DENSE_MAX = 8192   # n + m + p of the dense route; above it the handle is sparse (dopt_set_sparse)

    def __init__(self, batch, n, m, p=0, device=0, sparse=False):
        self.lib = _lib.load()
        self.batch, self.n, self.m, self.p = int(batch), int(n), int(m), int(p)
        self.device = device
        h = ctypes.c_void_p()
        rc = self.lib.dopt_create(ctypes.byref(h), device, self.batch, self.n, self.m,
                                  self.p, _lib.DOPT_KIND_QP)
        if rc != 0:
            raise _lib.EngineError(rc, "dopt_create failed (no HIP device?)")
        self.h = h
        self._mem = None
        self._keep = None
        # the sparse route (sparse.hip): automatic above the dense cap, opt-in below
        self.sparse = bool(sparse) or self.L > self.DENSE_MAX
        if sparse:
            _lib.check(self.lib.dopt_set_sparse(self.h, 1), self.h)

    def lsqr_stats(self):
        """Sparse route: (B, 2, 2) int32 — [istop, iterations] of the last
        reverse (index 0) and forward (index 1) LSQR runs per problem."""
        out = np.zeros(4 * self.batch, dtype=np.int32)
        _lib.check(self.lib.dopt_qp_lsqr_stats(self.h, out.ctypes.data), self.h)
        return out.reshape(2, self.batch, 2).transpose(1, 0, 2)

    def close(self):
        if getattr(self, "h", None):
            self.lib.dopt_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    # ---- memory mode -------------------------------------------------------
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
    def L(self):
        return self.n + self.m + self.p

    def set(self, Q, G=None, h=None, A=None, z=None, lam=None, nu=None):
        """Problem data and primal–dual point (λ, ν in OptNet sign)."""
        B, n, m, p = self.batch, self.n, self.m, self.p
        st = self._stage([Q, G, h, A, z, lam, nu])
        Qc = colmajor(Q, (B, n, n))
        Gc = colmajor(G, (B, m, n)) if m else None
        Ac = colmajor(A, (B, p, n)) if p else None
        args = [Qc, Gc, vector(h, (B, m)) if m else None, Ac, vector(z, (B, n)),
                vector(lam, (B, m)) if m else None, vector(nu, (B, p)) if p else None]
        self._keep = args  # device mode borrows: keep the staged tensors alive
        rc = self.lib.dopt_qp_set(self.h, *[st.ptr(a) for a in args])
        _lib.check(rc, self.h)

    def set_csc(self, Q, G=None, h=None, A=None, z=None, lam=None, nu=None):
        """``set`` with Q, G, A as sparse matrices in the reference's MOI
        matrix form (scipy.sparse, one per problem or one shared by all;
        converted to Julia CSC arrays: Int64, 1-based) — dopt_qp_set_csc
        densifies them on the device.  Host mode."""
        B, n, m, p = self.batch, self.n, self.m, self.p

        def csc(mats, rows):
            import scipy.sparse as sp
            if mats is None or rows == 0:
                return None, None, None, 0
            if sp.issparse(mats):
                mats = [mats] * B
            cps, rvs, nzs, off = [], [], [], 0
            for M in mats:
                M = sp.csc_matrix(M)
                if M.shape != (rows, n):
                    raise ValueError(f"sparse matrix of shape {M.shape}, expected {(rows, n)}")
                cps.append(M.indptr.astype(np.int64) + off + 1)
                rvs.append(M.indices.astype(np.int64) + 1)
                nzs.append(M.data.astype(np.float64))
                off += M.nnz
            return (np.ascontiguousarray(np.concatenate(cps)), np.ascontiguousarray(np.concatenate(rvs)),
                    np.ascontiguousarray(np.concatenate(nzs)), off)

        st = self._stage([z, h, lam, nu])
        if st.mem != _lib.DOPT_MEM_HOST:
            raise TypeError("set_csc takes host (numpy / scipy) arrays")
        mats = [csc(Q, n), csc(G, m), csc(A, p)]
        vecs = [vector(h, (B, m)) if m else None, vector(z, (B, n)),
                vector(lam, (B, m)) if m else None, vector(nu, (B, p)) if p else None]
        args = []
        for cp, rv, nz, nnz in mats:
            args += [st.ptr(cp), st.ptr(rv if nnz else None), st.ptr(nz if nnz else None), nnz]
        args += [st.ptr(v) for v in vecs]
        self._csc_keep = (mats, vecs)   # the arrays behind `args`
        self.set_csc_args(args)
        return args

    def set_csc_args(self, args):
        """dopt_qp_set_csc on the ctypes arguments a previous ``set_csc``
        returned (arrays kept alive by this object): the ABI call alone, as the
        Julia back-end issues it with the MOI matrix form already in hand."""
        rc = self.lib.dopt_qp_set_csc(self.h, *args)
        _lib.check(rc, self.h)

    def factor(self, singular_ok=False):
        return _lib.check(self.lib.dopt_qp_factor(self.h), self.h, singular_ok)

    def _out(self, like_device):
        return Staged.empty((self.batch, self.L), like_device)

    def reverse(self, dl_dz, singular_ok=False):
        """Returns (B, n+m+p) = [dz | dλ | dν]."""
        st = self._stage([dl_dz])
        d = vector(dl_dz, (self.batch, self.n))
        out = self._out(st.mem == _lib.DOPT_MEM_DEVICE)
        rc = self.lib.dopt_qp_reverse(self.h, st.ptr(d), st.ptr(out))
        _lib.check(rc, self.h, singular_ok)
        return out

    def forward(self, dQ=None, dq=None, dG=None, dh=None, dA=None, db=None,
                singular_ok=False):
        B, n, m, p = self.batch, self.n, self.m, self.p
        st = self._stage([dQ, dq, dG, dh, dA, db])
        args = [colmajor(dQ, (B, n, n)) if dQ is not None else None,
                vector(dq, (B, n)) if dq is not None else None,
                colmajor(dG, (B, m, n)) if (dG is not None and m) else None,
                vector(dh, (B, m)) if (dh is not None and m) else None,
                colmajor(dA, (B, p, n)) if (dA is not None and p) else None,
                vector(db, (B, p)) if (db is not None and p) else None]
        out = self._out(st.mem == _lib.DOPT_MEM_DEVICE)
        rc = self.lib.dopt_qp_forward(self.h, *[st.ptr(a) for a in args], st.ptr(out))
        _lib.check(rc, self.h, singular_ok)
        return out

    def reverse_k(self, dl_dz, singular_ok=False):
        """k seeds per problem on one factorisation (dopt_qp_reverse_k):
        dl_dz (k, B, n) → (k, B, n+m+p); equal to k ``reverse`` calls to
        rounding, the blocked problems' k solves in one MFMA launch."""
        k = int(dl_dz.shape[0])
        B, n = self.batch, self.n
        st = self._stage([dl_dz])
        d = vector(dl_dz, (k, B, n))
        out = Staged.empty((k, B, self.L), st.mem == _lib.DOPT_MEM_DEVICE)
        rc = self.lib.dopt_qp_reverse_k(self.h, k, st.ptr(d), st.ptr(out))
        _lib.check(rc, self.h, singular_ok)
        return out

    def forward_k(self, dQ=None, dq=None, dG=None, dh=None, dA=None, db=None, singular_ok=False):
        """k tangents per problem (dopt_qp_forward_k): each given tangent has a
        leading seed axis (k, B, …) → (k, B, n+m+p)."""
        given = [a for a in (dQ, dq, dG, dh, dA, db) if a is not None]
        if not given:
            raise ValueError("forward_k needs at least one tangent")
        k = int(given[0].shape[0])
        B, n, m, p = self.batch, self.n, self.m, self.p
        st = self._stage([dQ, dq, dG, dh, dA, db])
        kb = k * B
        args = [colmajor(dQ, (kb, n, n)) if dQ is not None else None,
                vector(dq, (kb, n)) if dq is not None else None,
                colmajor(dG, (kb, m, n)) if (dG is not None and m) else None,
                vector(dh, (kb, m)) if (dh is not None and m) else None,
                colmajor(dA, (kb, p, n)) if (dA is not None and p) else None,
                vector(db, (kb, p)) if (db is not None and p) else None]
        out = Staged.empty((k, B, self.L), st.mem == _lib.DOPT_MEM_DEVICE)
        rc = self.lib.dopt_qp_forward_k(self.h, k, *[st.ptr(a) for a in args], st.ptr(out))
        _lib.check(rc, self.h, singular_ok)
        return out

    def forward_reverse(self, dl_dz, dQ=None, dq=None, dG=None, dh=None, dA=None,
                        db=None, out_rev=None, out_fwd=None, singular_ok=False):
        """One full sensitivity solve per problem: factor + reverse + forward."""
        B, n, m, p = self.batch, self.n, self.m, self.p
        st = self._stage([dl_dz, dQ, dq, dG, dh, dA, db])
        dev = st.mem == _lib.DOPT_MEM_DEVICE
        args = [vector(dl_dz, (B, n)),
                colmajor(dQ, (B, n, n)) if dQ is not None else None,
                vector(dq, (B, n)) if dq is not None else None,
                colmajor(dG, (B, m, n)) if (dG is not None and m) else None,
                vector(dh, (B, m)) if (dh is not None and m) else None,
                colmajor(dA, (B, p, n)) if (dA is not None and p) else None,
                vector(db, (B, p)) if (db is not None and p) else None]
        o1 = out_rev if out_rev is not None else self._out(dev)
        o2 = out_fwd if out_fwd is not None else self._out(dev)
        for o in (o1, o2):
            _check_out(o, (B, self.L), dev)
        rc = self.lib.dopt_qp_forward_reverse(self.h, *[st.ptr(a) for a in args],
                                              st.ptr(o1), st.ptr(o2))
        _lib.check(rc, self.h, singular_ok)
        return o1, o2

    # ---- parameters (ParametricOptInterface glue, reference src/parameters.jl)
    @staticmethod
    def _terms(terms):
        """terms: iterable of (param, kind, index, coef) — kinds 0 LessThan row,
        1 EqualTo row, 2 objective, 3 objective parameter×variable (index = v)."""
        t = list(terms)
        par = np.ascontiguousarray([int(x[0]) for x in t], dtype=np.int32)
        kind = np.ascontiguousarray([int(x[1]) for x in t], dtype=np.int32)
        idx = np.ascontiguousarray([int(x[2]) for x in t], dtype=np.int32)
        coef = np.ascontiguousarray([float(x[3]) for x in t], dtype=np.float64)
        return len(t), par, kind, idx, coef

    def params_reverse(self, rev, terms, nparam):
        """ReverseConstraintSet of every parameter of every problem, (B, nparam),
        from a reverse output ``rev`` (B, n+m+p) — dopt_qp_params_reverse."""
        B = self.batch
        nt, par, kind, idx, coef = self._terms(terms)
        st = self._stage([rev])
        r = vector(rev, (B, self.L))
        out = Staged.empty((B, nparam), st.mem == _lib.DOPT_MEM_DEVICE)
        p = Staged.ptr
        rc = self.lib.dopt_qp_params_reverse(self.h, st.ptr(r), nparam, nt, p(par), p(kind), p(idx), p(coef),
                                             st.ptr(out))
        _lib.check(rc, self.h)
        return out

    def params_forward(self, dp, terms):
        """Parameter tangents dp (B, nparam) → the forward tangents (dq, dh, db)
        the reference's POI glue sets (dopt_qp_params_forward), ready for
        ``forward(dq=…, dh=…, db=…)``."""
        B, n, m, p_ = self.batch, self.n, self.m, self.p
        nparam = int(dp.shape[1])
        nt, par, kind, idx, coef = self._terms(terms)
        st = self._stage([dp])
        d = vector(dp, (B, nparam))
        dev = st.mem == _lib.DOPT_MEM_DEVICE
        dq, dh, db = Staged.empty((B, n), dev), Staged.empty((B, m), dev), Staged.empty((B, p_), dev)
        pp = Staged.ptr
        rc = self.lib.dopt_qp_params_forward(self.h, st.ptr(d), nparam, nt, pp(par), pp(kind), pp(idx), pp(coef),
                                             st.ptr(dq), st.ptr(dh) if m else None, st.ptr(db) if p_ else None)
        _lib.check(rc, self.h)
        return dq, dh, db

    def reverse_grads(self, rev, dQ=True, dG=True, dA=True):
        """Materialised reverse gradients of every problem from a reverse
        output ``rev`` (B, n+m+p) — ``ReverseObjectiveFunction`` /
        ``ReverseConstraintFunction`` (QuadraticProgram.jl:448-473, :307-314):
        dict with dq (B, n), dQ (B, n, n), dG (B, m, n), g_const (B, m),
        dA (B, p, n), a_const (B, p); the gradients w.r.t. h and b are
        −g_const and −a_const.  Matrices are returned as (B, rows, cols)
        views of the column-major buffers."""
        B, n, m, p = self.batch, self.n, self.m, self.p
        st = self._stage([rev])
        dev = st.mem == _lib.DOPT_MEM_DEVICE
        r = vector(rev, (B, n + m + p))
        out = {"dq": Staged.empty((B, n), dev),
               "dQ": Staged.empty((B, n, n), dev) if dQ else None,
               "dG": Staged.empty((B, n, m), dev) if (dG and m) else None,
               "g_const": Staged.empty((B, m), dev) if m else None,
               "dA": Staged.empty((B, n, p), dev) if (dA and p) else None,
               "a_const": Staged.empty((B, p), dev) if p else None}
        rc = self.lib.dopt_qp_reverse_grads(
            self.h, st.ptr(r), *[st.ptr(out[k]) for k in ["dQ", "dq", "dG", "g_const", "dA", "a_const"]])
        _lib.check(rc, self.h)
        for k in ("dQ", "dG", "dA"):   # column-major (B, cols, rows) → (B, rows, cols) view
            if out[k] is not None:
                out[k] = out[k].transpose(1, 2) if _is_t(out[k]) else np.swapaxes(out[k], 1, 2)
        return out

    # ---- introspection -----------------------------------------------------
    def info(self):
        buf = np.zeros(self.batch, dtype=np.int32)
        _lib.check(self.lib.dopt_get_info(self.h, buf.ctypes.data), self.h)
        return buf

    def iterative(self):
        buf = np.zeros(self.batch, dtype=np.int8)
        _lib.check(self.lib.dopt_get_iterative(self.h, buf.ctypes.data), self.h)
        return buf.astype(bool)

    def system_size(self):
        buf = np.zeros(self.batch, dtype=np.int32)
        _lib.check(self.lib.dopt_get_system_size(self.h, buf.ctypes.data), self.h)
        return buf

    def last_time(self):
        return self.lib.dopt_last_time(self.h)

    def kept(self):
        """(B, m) bool mask of the inequality rows kept in the factorised
        system (False: eliminated exactly, λ_i == 0 and (Gz − h)_i != 0)."""
        buf = np.zeros((self.batch, self.m), dtype=np.int8)
        _lib.check(self.lib.dopt_qp_get_kept(self.h, buf.ctypes.data), self.h)
        return buf.astype(bool)

    def lu_kind(self):
        """Per-problem factorisation kind of the last factorisation:
        _lib.LU_KIND_LSQR / LU_KIND_NOPIV / LU_KIND_PIVOT, or LU_KIND_SMALL after a
        reverse call the one-workgroup small path served (qp_small.hip)."""
        buf = np.zeros(self.batch, dtype=np.int8)
        _lib.check(self.lib.dopt_qp_get_lu_kind(self.h, buf.ctypes.data), self.h)
        return buf

    def sym_route(self):
        """Per problem: 1 when the last factorisation took the P-symmetric
        no-pivot route (lower trailing tiles, U from L), else 0."""
        buf = np.zeros(self.batch, dtype=np.int8)
        _lib.check(self.lib.dopt_qp_get_sym(self.h, buf.ctypes.data), self.h)
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
        """{phase name: (total ms, launches)} since the last call (HIP events
        on the handle's stream)."""
        return _lib.phase_times(self.lib, self.h)

    def split(self, out):
        n, m = self.n, self.m
        return out[:, :n], out[:, n:n + m], out[:, n + m:]


class MI355XSolver:
    """The MI355X solver of the reference's ``LinearAlgebraSolver`` plug point
    (QuadraticProgram.jl:475-502; the Julia ``DiffOptMI355X.MI355XSolver``):
    ``solve_system(LHS, RHS, iterative)`` is ``iterative ? lsqr(LHS, RHS) :
    LHS \\ RHS`` on the device (dopt_lhs_solve).  The reference calls it twice
    per model (reverse with LHS, :335; forward with LHS', :438) and its
    callers loop models of one size, so the solver keeps one engine handle
    per (batch, rows) instead of creating one per call."""

    def __init__(self, device=0):
        self.device = device
        self._h = None
        self._key = None
        self._fact = None      # (memory key of the array factorised last, the array)
        self.resolves = 0      # calls served by dopt_lhs_resolve (introspection)
        self.lib = _lib.load()

    def close(self):
        if self._h is not None:
            self.lib.dopt_destroy(self._h)
            self._h = None
            self._key = None
            self._fact = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _handle(self, B, rows):
        if self._key != (B, rows):
            self.close()
            h = ctypes.c_void_p()
            rc = self.lib.dopt_create(ctypes.byref(h), self.device, B, rows, 0, 0, _lib.DOPT_KIND_NLP)
            if rc != 0:
                raise _lib.EngineError(rc, "dopt_create failed (no HIP device?)")
            self._h, self._key = h, (B, rows)
        return self._h

    def solve_system(self, LHS, RHS, iterative=False):
        """LHS (rows, rows) or a batch (B, rows, rows); RHS (rows,) / (rows, k)
        or batched (B, rows) / (B, rows, k).  A singular LHS raises
        SingularException(info), as ``\\`` does — on the engine's
        rank-revealing test |u_ii| ≤ rows·ε·max|M| (include/diffopt_mi355x.h,
        dopt_lhs_solve), which is stricter than ``\\``'s exactly-zero pivot."""
        M = np.asarray(LHS, dtype=np.float64)
        single = M.ndim == 2
        if single:
            M = M[None]
        B, rows = M.shape[0], M.shape[-1]
        if M.shape != (B, rows, rows):
            raise TypeError("LHS must be square")
        R = np.asarray(RHS, dtype=np.float64)
        if single:
            R = R[None]
        vec = R.ndim == 2
        Rk = R[..., None] if vec else R                     # (B, rows, k)
        if Rk.shape[:2] != (B, rows):
            raise TypeError("RHS does not match LHS")
        k = Rk.shape[2]
        rhs = np.ascontiguousarray(np.transpose(Rk, (2, 0, 1)))   # seed-major (k, B, rows)
        out = np.empty_like(rhs)
        h = self._handle(B, rows)
        # the reference's second call per model passes LHS' (an adjoint of the
        # LHS it just solved with: QuadraticProgram.jl:335, :438): an array
        # that is exactly the transpose of the one factorised last (same
        # memory, shape and strides reversed) AND whose contents still equal
        # the matrix factorised (a copy kept at that call: an edit in place
        # between the two calls refactorises, as `\` would) is answered from
        # those factors, once per factorisation; any other call factorises
        lhs = LHS if isinstance(LHS, np.ndarray) else None
        key = None
        if lhs is not None and lhs.ndim == 2:
            key = (lhs.__array_interface__["data"][0], lhs.shape, lhs.strides)
        reuse = (not iterative and key is not None and self._fact is not None
                 and (key[0], key[1][::-1], key[2][::-1]) == self._fact[0]
                 and np.array_equal(lhs.T, self._fact[1]))
        if reuse:
            rc = self.lib.dopt_lhs_resolve(h, k, rhs.ctypes.data, out.ctypes.data, 1)
            self.resolves += 1
            self._fact = None
        else:
            Mc = np.ascontiguousarray(np.swapaxes(M, 1, 2))        # column-major per problem
            rc = self.lib.dopt_lhs_solve(h, rows, Mc.ctypes.data, k, rhs.ctypes.data, out.ctypes.data,
                                         int(bool(iterative)))
            # (the contents factorised, for the reuse check above)
            self._fact = None if iterative or key is None else (key, np.array(lhs, copy=True))
        _lib.check(rc, h)
        X = np.transpose(out, (1, 2, 0))                           # (B, rows, k)
        if vec:
            X = X[..., 0]
        return X[0] if single else X


def solve_system(LHS, RHS, iterative=False, device=0, solver=None):
    """``QuadraticProgram.solve_system(solver, LHS, RHS, iterative)`` (see
    MI355XSolver): one call on `solver`'s cached handle, or on a temporary
    solver when none is given."""
    if solver is not None:
        return solver.solve_system(LHS, RHS, iterative)
    s = MI355XSolver(device)
    try:
        return s.solve_system(LHS, RHS, iterative)
    finally:
        s.close()


class Model:
    """Single-problem ``DiffOpt.QuadraticProgram.Model`` on the engine.

    Problem data is given in the matrix form the reference builds from MOI
    (``_gradient_cache``, :182-213): ``Q`` (symmetric Hessian), ``q``, ``G``,
    ``h`` (LessThan rows), ``A``, ``b`` (EqualTo rows).  Tangent sign handling
    of ``_fill`` (diff_opt.jl:594-656) happens in the setters below.
    """

    def __init__(self, device=0):
        self.device = device
        self.empty()

    # MOI.empty! (:126-137)
    def empty(self):
        self.Q = self.q = self.G = self.h = self.A = self.b = None
        self.x = None
        self.lam = None
        self.nu = None
        self._engine = None
        self.forw_grad_cache = None
        self.back_grad_cache = None
        self.diff_time = float("nan")
        self.input_dx = {}
        self.input_objective = None      # (dQ, dq)
        self.input_le = {}               # row -> (coeffs, constant)
        self.input_eq = {}

    def set_problem(self, Q, q, G=None, h=None, A=None, b=None):
        n = np.asarray(q).shape[0]
        self.Q = np.asarray(Q, dtype=np.float64).reshape(n, n)
        self.q = np.asarray(q, dtype=np.float64)
        self.G = np.zeros((0, n)) if G is None else np.asarray(G, float).reshape(-1, n)
        self.h = np.zeros(0) if h is None else np.asarray(h, float).ravel()
        self.A = np.zeros((0, n)) if A is None else np.asarray(A, float).reshape(-1, n)
        self.b = np.zeros(0) if b is None else np.asarray(b, float).ravel()
        self._engine = None

    @property
    def n(self):
        return self.q.shape[0]

    # ---- starts (diff_opt.jl:362-370, QuadraticProgram.jl:164-180) ---------
    def set_variable_primal_start(self, x):
        self.x = np.asarray(x, dtype=np.float64).copy()
        self._engine = None

    def set_constraint_dual_start(self, kind, duals):
        """MOI ``ConstraintDual`` values; stored with the OptNet sign flip."""
        d = -np.asarray(duals, dtype=np.float64)
        if kind == LE:
            self.lam = d
        elif kind == EQ:
            self.nu = d
        else:
            raise ValueError(kind)
        self._engine = None

    # ---- sensitivity inputs -------------------------------------------------
    def set_reverse_variable_primal(self, i, value):
        self.input_dx[int(i)] = float(value)

    def set_forward_objective_function(self, dQ=None, dq=None):
        self.input_objective = (dQ, dq)

    def set_forward_constraint_function(self, kind, row, coeffs, constant):
        """Tangent of the constraint function ``coeffsᵀx + constant`` of row
        ``row`` (``func``-in-``set``).  ``_fill``: the constant is negated for
        both EqualTo and LessThan (it is the tangent of the set constant)."""
        tgt = self.input_le if kind == LE else self.input_eq
        tgt[int(row)] = (np.asarray(coeffs, dtype=np.float64), float(constant))

    def empty_input_sensitivities(self):
        self.input_dx = {}
        self.input_objective = None
        self.input_le = {}
        self.input_eq = {}

    # ---- engine ------------------------------------------------------------
    def _ensure(self):
        n, m, p = self.n, self.G.shape[0], self.A.shape[0]
        if self.x is None or len(self.x) < n or np.any(np.isnan(self.x)):
            raise ValueError("VariablePrimalStart missing")
        lam = np.zeros(m) if self.lam is None else self.lam
        nu = np.zeros(p) if self.nu is None else self.nu
        if self._engine is None:
            e = QPBatch(1, n, m, p, self.device)
            e.set(self.Q[None], self.G[None], self.h[None], self.A[None], self.x[None],
                  lam[None], nu[None])
            self._engine = e
            self._lam, self._nu = lam, nu
        return self._engine

    def reverse_differentiate(self):
        import time
        t0 = time.perf_counter()
        e = self._ensure()
        dl = np.zeros(self.n)
        for i, v in self.input_dx.items():
            dl[i] = v
        out = np.asarray(e.reverse(dl[None]))[0]
        n, m = self.n, self.G.shape[0]
        self.back_grad_cache = (out[:n], out[n:n + m], out[n + m:])
        self.diff_time = time.perf_counter() - t0

    def forward_differentiate(self):
        import time
        t0 = time.perf_counter()
        e = self._ensure()
        n, m, p = self.n, self.G.shape[0], self.A.shape[0]
        dQ, dq = (None, None) if self.input_objective is None else self.input_objective
        dG = np.zeros((m, n))
        dh = np.zeros(m)
        for r, (c, k) in self.input_le.items():
            dG[r] = c
            dh[r] = -k
        dA = np.zeros((p, n))
        db = np.zeros(p)
        for r, (c, k) in self.input_eq.items():
            dA[r] = c
            db[r] = -k
        out = np.asarray(e.forward(
            None if dQ is None else np.asarray(dQ, float)[None],
            None if dq is None else np.asarray(dq, float)[None],
            dG[None] if m else None, dh[None] if m else None,
            dA[None] if p else None, db[None] if p else None))[0]
        self.forw_grad_cache = (out[:n], out[n:n + m], out[n + m:])
        self.diff_time = time.perf_counter() - t0

    # ---- outputs -----------------------------------------------------------
    def forward_variable_primal(self, i):
        """``ForwardVariablePrimal`` (:299-305)."""
        return self.forw_grad_cache[0][i]

    def reverse_objective_function(self):
        """``ReverseObjectiveFunction`` (:448-458): (dq, dQ) with
        ``dq = ∇z`` and ``dQ = (∇z zᵀ + z ∇zᵀ)/2`` (materialised)."""
        dz = self.back_grad_cache[0]
        z = self.x
        return dz.copy(), 0.5 * (np.outer(dz, z) + np.outer(z, dz))

    def reverse_constraint_function(self, kind, row):
        """``ReverseConstraintFunction`` (diff_opt.jl:475-481): (coefficients,
        constant) from ``_get_dA``/``_get_db`` (:307-314, :461-473)."""
        dz, dlam, dnu = self.back_grad_cache
        z = self.x
        if kind == LE:
            l = self._lam[row]
            return l * dlam[row] * z + l * dz, l * dlam[row]
        if kind == EQ:
            return dnu[row] * z + self._nu[row] * dz, dnu[row]
        raise ValueError(kind)

    def differentiate_time_sec(self):
        return self.diff_time
