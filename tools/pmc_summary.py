#!/usr/bin/env python3
"""Summarise two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE; separate runs
because they do not fit one TCC pass on gfx950) into profiles/pmc_latest.json:
HBM bytes per launch per engine kernel.

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports ½ of the
bytes of wide coalesced reads → doubled here; WRITE_SIZE is taken as is.
Calibrated per access width on this machine (tools/probe/pmc_cal.hip,
tools/pmc_calibrate.py → profiles/pmc_calibration.json): 4-, 8- and 16-byte
per-lane streaming loads and the LU's 4-row × 128-B pattern all read as 0.500
of the streamed bytes, 4-, 8- and 16-byte stores as 1.000 — one factor each.
FETCH_SIZE/WRITE_SIZE are in KB (rocprofv3 derived counters) → ×1024.

  python tools/pmc_summary.py <fetch_dir> <write_dir> <out.json> [key_suffix]   (merges into out.json;
         key_suffix, e.g. @cfg3, is appended to every kernel key — the keys bench.py looks up)
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

# rocprof kernel-name fragment → engine phase name (bench.py roofline keys)
KERNEL_PHASE = {
    "qp_fused_kernel": "qp_fused",
    "qp_factor_fast_kernel": "qp_lu",
    "qp_solve_fast_kernel": "qp_solve",
    "conic_lsqr_kernel": "conic_lsqr",     # (dense or, config 8, the sparse route's instantiation)
    "sp_lsqr_kernel": "qp_lsqr",           # the sparse QP route (config 7)
    "conic_lsqr2_kernel": "conic_lsqr",     # co-iterated forward + reverse (one launch per call)
    "conic_cone_kernel": "conic_cone",
    "conic_split_pass_kernel": "conic_split_pass",
}
# blocked QP route: one bench phase = several launches (the panel / trailing-
# update sequence of one factorisation, the two solve kernels of one step);
# summed over the dispatches and divided by the number of steps, counted by
# the per-step qp_prep_kernel dispatch
QP_GROUPS = {"qp_assemble": ("qp_prep_kernel", "qp_asm_tile_kernel", "qp_qsym_kernel"),
             "qp_lu": ("nlu_diag_kernel", "nlu_trsm_kernel", "nlu_cross_kernel", "nlu_update2_kernel",
                       "nlu_ldiag_kernel", "nlu_lcol_kernel", "blu_panel_kernel", "blu_update_kernel"),
             "qp_solve": ("blu_solve_kernel", "blu_solve_rows_kernel", "blu_solve2_kernel", "blu_sym2_kernel",
                          "blu_symsolve_kernel"),
             "qp_output": ("qp_output_kernel",)}
QP_STEP = "qp_prep_kernel"
# NLP back-end (bench config 6): the step is counted by its assembly launch
# (nlp_red_prep_kernel on the reduced route, nlp_assemble_kernel on the full
# one — the first of the two found); the LU is the left-looking no-pivot LU
# (or the partial-pivoting blocked LU), the solves the P-symmetric pair /
# single-direction sweeps (with the blocked solve kernels for pivoted problems)
NLP_GROUPS = {"qp_assemble": ("nlp_assemble_kernel", "nlp_red_prep_kernel", "qp_qsym_kernel", "nlp_pivot_check_kernel"),
              "qp_lu": ("nlu_diag_kernel", "nlu_trsm_kernel", "nlu_cross_kernel", "nlu_update2_kernel",
                        "nlu_ldiag_kernel", "nlu_lcol_kernel"),
              "qp_lu_pivot": ("blu_panel_kernel", "blu_update_kernel"),
              "qp_rhs": ("nlp_fwd_rhs_kernel", "nlp_rev_rhs_kernel", "nlp_red_rhs_kernel"),
              "qp_solve": ("blu_solve_kernel", "blu_solve_rows_kernel", "blu_symsolve_kernel", "blu_sym2_kernel"),
              "qp_output": ("nlp_fwd_out_kernel", "nlp_rev_out_kernel", "nlp_red_recover_kernel")}
NLP_STEP = ("nlp_assemble_kernel", "nlp_red_prep_kernel")
# split-path LSQR: every conic_split_* dispatch belongs to the LSQR call opened
# by the preceding conic_split_init_kernel; reported per LSQR call under the
# bench's phase name "conic_lsqr" (key "conic_lsqr_split")
SPLIT_FRAGS, SPLIT_OPEN = ("conic_split_", "conic_fsplit_"), "conic_split_init_kernel"


def per_launch(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    acc = defaultdict(lambda: defaultdict(float))   # phase → dispatch → value
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                kn = row.get("Kernel_Name", "")
                for frag, ph in KERNEL_PHASE.items():
                    if frag in kn:
                        acc[ph][row.get("Dispatch_Id")] += float(row["Counter_Value"])
    res = {ph: sum(v.values()) / len(v) for ph, v in acc.items() if v}
    tot, calls = 0.0, set()
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                kn = row.get("Kernel_Name", "")
                if any(fr in kn for fr in SPLIT_FRAGS):
                    tot += float(row["Counter_Value"])
                    if SPLIT_OPEN in kn:
                        calls.add(row.get("Dispatch_Id"))
    if calls:
        res["conic_lsqr_split"] = tot / len(calls)
    for groups, step in ((QP_GROUPS, (QP_STEP,)), (NLP_GROUPS, NLP_STEP)):
        gtot, steps = defaultdict(float), defaultdict(set)
        for f in files:
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    if row.get("Counter_Name") != counter:
                        continue
                    kn = row.get("Kernel_Name", "")
                    for st in step:
                        if st in kn:
                            steps[st].add(row.get("Dispatch_Id"))
                    for ph, frags in groups.items():
                        if any(fr in kn for fr in frags):
                            gtot[ph] += float(row["Counter_Value"])
        steps = next((steps[st] for st in step if steps[st]), None)   # the first step kernel found
        if steps:
            for ph, v in gtot.items():
                res[ph] = v / len(steps)
    return res


def main():
    fdir, wdir, out = sys.argv[1:4]
    suffix = sys.argv[4] if len(sys.argv) > 4 else ""
    fetch = per_launch(fdir, "FETCH_SIZE")
    write = per_launch(wdir, "WRITE_SIZE")
    res = {"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes",
           "correction": "FETCH_SIZE x2 (gfx950 wide-read halving), KB x1024",
           "kernels": {}}
    for ph in sorted(set(fetch) | set(write)):
        rb = fetch.get(ph, 0.0) * 2 * 1024
        wb = write.get(ph, 0.0) * 1024
        res["kernels"][ph + suffix] = {"read_bytes_per_launch": rb, "write_bytes_per_launch": wb,
                              "hbm_bytes_per_launch": rb + wb}
    if os.path.exists(out):          # merge: other configs' kernels stay
        with open(out) as f:
            old = json.load(f).get("kernels", {})
        old.update(res["kernels"])
        res["kernels"] = old
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
