"""CPU ORACLE — test infrastructure only.

This package is a CPU restatement (numpy/scipy) of the DiffOpt.jl sensitivity
algorithms on the hot path.  It is the *checker*: only
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may import it.  The product path (``diffopt.jl_amd/``) never imports, links or
calls anything in here and fails loudly when its HIP library is missing.

Parity status: pinned.  DiffOpt.jl is pure Julia and there is no Julia
toolchain in this image (absence, not a denial), so the reference itself cannot
be executed; every function below cites the reference file:line it restates and
is pinned by the reference's own known-answer tests, transcribed into
``tests/golden/*.json`` by ``tests/golden/make_golden.py`` (see
``tests/test_oracle_golden.py``).

Third-party algorithms restated here (un-vendored in the reference, no Manifest):
  * SuiteSparse UMFPACK LU via Julia SparseArrays ``\\`` (julia = "1.6") —
    restated as LAPACK getrf (dense) or SuperLU ``splu`` (sparse); both return
    the exact solution of the same linear system up to rounding.
  * IterativeSolvers.jl 0.9 ``lsqr`` — restated line by line in ``lsqr.py``
    (Paige & Saunders LSQR with atol = btol = sqrt(eps), conlim = 1/sqrt(eps),
    maxiter = max(size(A)), x0 = 0).
  * MathOptSetDistances 0.2.9 projections / projection Jacobians onto the
    dual cones — restated in ``cones.py``.
"""

from . import lsqr, cones, qp, conic  # noqa: F401
