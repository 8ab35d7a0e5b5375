"""The reference-shaped single-model API (diffopt_amd.qp.Model,
diffopt_amd.conic.Model) driven through every golden fixture the way the
reference's plumbing drives its back-end: MOI-sign duals in
(ConstraintDualStart, QuadraticProgram.jl:164-180), forward tangents as MOI
functions with `_fill`'s constant negation (diff_opt.jl:594-656), MAX sense
negating c but not dc (ConicProgram.jl:206-208 vs :270-278), getters out
(QuadraticProgram.jl:299-314, 448-473; ConicProgram.jl:396-443).  Expected
values are the reference tests' own (tests/golden)."""

import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _load(name):
    with open(os.path.join(HERE, "golden", name)) as f:
        return json.load(f)


QP_FX = _load("qp_fixtures.json") + _load("lp_fixtures.json")


@pytest.mark.parametrize("fx", QP_FX, ids=[f["name"] for f in QP_FX])
def test_qp_model_through_fixture(fx):
    from diffopt_amd.qp import EQ, LE, Model
    a = {k: np.array(v, dtype=float) for k, v in fx.items() if isinstance(v, list)}
    n = a["Q"].shape[0]
    G, A = a["G"].reshape(-1, n), a["A"].reshape(-1, n)
    m, p = G.shape[0], A.shape[0]
    model = Model()
    model.set_problem(a["Q"], a["q"], G, a["h"], A, a["b"])
    model.set_variable_primal_start(a["z"])
    # the solver reports MOI duals: λ = −dual(LessThan), ν = −dual(EqualTo)
    if m:
        model.set_constraint_dual_start(LE, -a["lam"])
    if p:
        model.set_constraint_dual_start(EQ, -a["nu"])
    # ---- reverse: ReverseVariablePrimal seeds → gradients
    for i, v in enumerate(a["dzb"]):
        model.set_reverse_variable_primal(i, v)
    model.reverse_differentiate()
    dq, dQ = model.reverse_objective_function()
    got = {"dqb": dq, "dQb": dQ}
    if m:
        rows = [model.reverse_constraint_function(LE, i) for i in range(m)]
        got["dGb"] = np.stack([r[0] for r in rows])
        got["dhb"] = -np.array([r[1] for r in rows])        # ∂h = −constant
    if p:
        rows = [model.reverse_constraint_function(EQ, i) for i in range(p)]
        got["dAb"] = np.stack([r[0] for r in rows])
        got["dbb"] = -np.array([r[1] for r in rows])        # ∂b = −constant
    got["grad_zb"], got["grad_lamb"], got["grad_nub"] = model.back_grad_cache
    # ---- forward: MOI function tangents; a tangent dh of h is the constant −dh
    fw = {k: np.array(v, dtype=float) for k, v in fx["fwd"].items()}
    model.set_forward_objective_function(fw.get("dQ"), fw.get("dq"))
    dG = fw.get("dG", np.zeros((m, n))).reshape(m, n)
    dh = fw.get("dh", np.zeros(m))
    for i in range(m):
        model.set_forward_constraint_function(LE, i, dG[i], -dh[i])
    dA = fw.get("dA", np.zeros((p, n))).reshape(p, n)
    db = fw.get("db", np.zeros(p))
    for i in range(p):
        model.set_forward_constraint_function(EQ, i, dA[i], -db[i])
    model.forward_differentiate()
    got["dzf"] = np.array([model.forward_variable_primal(i) for i in range(n)])
    got["z"] = a["z"]
    assert model.differentiate_time_sec() > 0
    checked = 0
    for k, v in fx["expect"].items():
        if k not in got:
            continue
        exp = np.array(v, dtype=float).reshape(np.shape(got[k]))
        np.testing.assert_allclose(got[k], exp, atol=fx["atol"], rtol=fx["rtol"], err_msg=k)
        checked += 1
    assert checked >= 1


CONIC_FX = _load("conic_fixtures.json")


@pytest.mark.parametrize("fx", CONIC_FX, ids=[f["name"] for f in CONIC_FX])
def test_conic_model_through_fixture(fx):
    from diffopt_amd.conic import Model
    A = np.array(fx["A"], dtype=float)
    m, n = A.shape
    model = Model()
    model.set_problem(A, fx["b"], fx["c"], [tuple(c) for c in fx["cones"]], fx["max_sense"])
    model.set_variable_primal_start(fx["x"])
    model.set_constraint_primal_start(fx["s"])
    model.set_constraint_dual_start(fx["y"])
    for t in fx["forward"]:
        dA = np.array(t["dA"], dtype=float)
        for ci in range(len(fx["cones"])):
            r = model.rows(ci)
            model.set_forward_constraint_function(ci, dA[r], np.array(t["db"])[r])
        model.set_forward_objective_function(t["dc"])   # not negated for MAX (:270-278)
        model.forward_differentiate()
        dx = np.array([model.forward_variable_primal(i) for i in range(n)])
        np.testing.assert_allclose(dx, t["dx"], atol=t["atol"], rtol=t["rtol"])
    for t in fx["reverse"]:
        model.input_dx = {}
        for i, v in enumerate(t["dx"]):
            model.set_reverse_variable_primal(i, v)
        model.reverse_differentiate()
        db = np.concatenate([model.reverse_constraint_function(ci)[1]
                             for ci in range(len(fx["cones"]))])
        np.testing.assert_allclose(db[t["rows"]], t["db"], atol=t["atol"], rtol=t["rtol"])
        assert model.reverse_objective_function().shape == (n,)


def test_conic_model_missing_dual_start():
    """ConicProgram.jl:186-196: a NaN (missing) dual or primal start fails."""
    from diffopt_amd.conic import Model
    fx = CONIC_FX[0]
    model = Model()
    model.set_problem(np.array(fx["A"]), fx["b"], fx["c"], [tuple(c) for c in fx["cones"]])
    model.set_variable_primal_start(fx["x"])
    model.set_constraint_primal_start(fx["s"])
    y = np.array(fx["y"], dtype=float)
    y[0] = np.nan
    model.set_constraint_dual_start(y)
    with pytest.raises(ValueError, match="ConstraintDualStart"):
        model.forward_differentiate()
