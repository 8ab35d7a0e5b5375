"""The POI oracle (oracle/poi.py) on a hand-worked case: the reference's
dictionary accumulation (parameters.jl:341-534, :91-270)."""

import numpy as np

from oracle import poi


def test_reverse_hand_worked():
    n, m, p = 2, 2, 1
    lam = np.array([2.0, 0.0])
    rev = np.array([0.5, -1.0,      # dz
                    3.0, 7.0,       # dλ
                    -4.0])          # dν
    terms = [(0, 0, 0, 1.5),        # p0 += 1.5 · λ0·dλ0 = 1.5·6 = 9
             (0, 3, 1, 2.0),        # p0 += 2 · dz1 = −2
             (1, 1, 0, -0.5),       # p1 += −0.5 · dν0 = 2
             (1, 2, 0, 9.0),        # objective constant: 0
             (1, 0, 1, 4.0)]        # λ1 = 0: 0
    np.testing.assert_allclose(poi.reverse(terms, 2, lam, rev, n, m, p), [7.0, 2.0])


def test_forward_hand_worked():
    terms = [(0, 0, 1, 2.0), (1, 0, 1, -1.0), (1, 1, 0, 3.0), (0, 3, 0, 0.5), (1, 2, 0, 100.0)]
    dq, dh, db = poi.forward(terms, np.array([1.0, 2.0]), 2, 2, 1)
    np.testing.assert_allclose(dq, [0.5, 0.0])
    np.testing.assert_allclose(dh, [0.0, -(2.0 - 2.0)])
    np.testing.assert_allclose(db, [-6.0])
