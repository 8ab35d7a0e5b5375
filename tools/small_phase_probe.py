#!/usr/bin/env python3
"""Repeated config-1 QPModel reverse calls (batch 1) for per-phase kernel
timing of qp_small_rev_kernel under rocprofv3 with the SM_EXIT variants
(tools/build_variant.sh xN qp_small -DSM_EXIT=N)."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "diffopt.jl_amd"))
from diffopt_amd.qp import QPBatch
from diffopt_amd.synthetic import QP_CONFIGS, SEED0, qp_numpy

c = QP_CONFIGS[1]
n, m, p = c["n"], c["m"], c["p"]
d = qp_numpy(1, n, m, p, c["phi"], SEED0 + 1)
e = QPBatch(1, n, m, p)
fell = 0
reps = int(os.environ.get("REPS", "20"))
for _ in range(reps):
    e.set(d["Q"], d["G"], d["h"], d["A"], d["z"], d["lam"], d["nu"])
    r = e.reverse(d["dl_dz"])
    fell += int(e.lu_kind()[0] != 3)
print("small path fell back in %d of %d calls" % (fell, reps))
if os.environ.get("STAMPS"):
    print("clock cycles %.0f  wall ticks (100 MHz) %.0f  N %.0f  -> %.0f MHz, %.2f us/step" %
          (r[0][0], r[0][1], r[0][2], r[0][0] / r[0][1] * 100, r[0][1] / 100 / r[0][2]))
    for w, o in (("t0", 4), ("t512", 7), ("t1023", 10)):
        print("  %s cycles/step: barrier %.0f  reads+update %.0f  publish %.0f" %
              ((w,) + tuple(r[0][o + i] / r[0][2] for i in range(3))))
e.close()
