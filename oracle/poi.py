"""CPU oracle (test infrastructure only: imported by tests/, never by the
product path) for the ParametricOptInterface glue of the QP back-end,
restating reference src/parameters.jl with its dictionary accumulation.

A term is (param, kind, index, coef); kinds as include/diffopt_mi355x.h:
0 LessThan-row parameter term, 1 EqualTo-row parameter term, 2 objective
parameter term, 3 objective parameter×variable term (index = variable).
"""
import numpy as np


def reverse(terms, nparam, lam, rev, n, m, p):
    """parameter_output_backward (parameters.jl:341-534): for every parametric
    constraint, value += coefficient · constant(ReverseConstraintFunction(ci))
    (:341-363); objective p-terms × constant(ReverseObjectiveFunction) (0.0 for
    the QP, QuadraticProgram.jl:448-458) and pv-terms × its coefficient of v
    (:505-511).  `rev` = [dz | dλ | dν] of one problem; the constants are the
    getters QuadraticProgram.jl:307-314 / 461-473 return: λ_i·dλ_i (LessThan),
    dν_i (EqualTo)."""
    dz, dl, dn = rev[:n], rev[n:n + m], rev[n + m:]
    out = {}
    for (par, kind, idx, coef) in terms:
        if kind == 0:
            s = lam[idx] * dl[idx]
        elif kind == 1:
            s = dn[idx]
        elif kind == 2:
            s = 0.0
        elif kind == 3:
            s = dz[idx]
        else:
            raise ValueError(kind)
        out[par] = out.get(par, 0.0) + coef * s          # get!(…, p, 0.0) + c·s
    res = np.zeros(nparam)
    for par, v in out.items():
        res[par] = v
    return res


def forward(terms, dp, n, m, p):
    """parameter_input_forward → ForwardConstraintFunction / ForwardObjectiveFunction
    (parameters.jl:91-270): cte(row) += dp·coef, pv terms add dp·coef to the
    objective's coefficient of v.  Returned as the QP forward tangents the
    `_fill` rules give (diff_opt.jl:616-622): dh = −cte (LessThan),
    db = −cte (EqualTo), dq_v."""
    cte_le, cte_eq, dq = np.zeros(m), np.zeros(p), np.zeros(n)
    for (par, kind, idx, coef) in terms:
        if kind == 0:
            cte_le[idx] += dp[par] * coef
        elif kind == 1:
            cte_eq[idx] += dp[par] * coef
        elif kind == 3:
            dq[idx] += dp[par] * coef
    return dq, -cte_le, -cte_eq
