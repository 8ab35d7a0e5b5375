"""ctypes binding of ``libdiffopt_mi355x.so`` (include/diffopt_mi355x.h).

The library is the product path; there is no fallback.  If it is missing the
import of any engine class raises ``EngineUnavailable`` (build it with
``make -C diffopt.jl_amd`` or ``python -c 'import __graft_entry__ as g; g.build()'``).
"""

import ctypes
import os

LIB_NAME = "libdiffopt_mi355x.so"
LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), LIB_NAME)
# A/B builds of the same engine (tools/build_variant.sh): DOPT_LIB names one
# in place of the default in-tree library (benchmarking only).  The override is
# announced on stderr and recorded in LIB_OVERRIDE, so a stale variant left in
# the environment cannot silently stand in for the in-tree build.
LIB_OVERRIDE = os.environ.get("DOPT_LIB") or None
if LIB_OVERRIDE:
    import sys
    print(f"diffopt_amd: DOPT_LIB={LIB_OVERRIDE} replaces the in-tree {LIB_PATH}", file=sys.stderr)
    LIB_PATH = LIB_OVERRIDE

DOPT_KIND_QP = 0
DOPT_KIND_CONIC = 1
DOPT_KIND_NLP = 2
DOPT_MEM_HOST = 0
DOPT_MEM_DEVICE = 1

CONE_ZEROS, CONE_NONNEG, CONE_NONPOS, CONE_SOC, CONE_PSD_TRI = 0, 1, 2, 3, 4

_c_dp = ctypes.POINTER(ctypes.c_double)
_c_ip = ctypes.POINTER(ctypes.c_int32)
_c_bp = ctypes.POINTER(ctypes.c_int8)
_h = ctypes.c_void_p

# symbol → (restype, argtypes); must match include/diffopt_mi355x.h exactly
SIGNATURES = {
    "dopt_abi_version": (ctypes.c_int, []),
    "dopt_create": (ctypes.c_int, [ctypes.POINTER(_h), ctypes.c_int, ctypes.c_int64,
                                   ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                   ctypes.c_int32]),
    "dopt_destroy": (ctypes.c_int, [_h]),
    "dopt_last_error": (ctypes.c_char_p, [_h]),
    "dopt_set_stream": (ctypes.c_int, [_h, ctypes.c_void_p]),
    "dopt_set_memory": (ctypes.c_int, [_h, ctypes.c_int32]),
    "dopt_qp_set": (ctypes.c_int, [_h] + [ctypes.c_void_p] * 7),
    "dopt_qp_factor": (ctypes.c_int, [_h]),
    "dopt_set_sparse": (ctypes.c_int, [_h, ctypes.c_int32]),
    "dopt_qp_lsqr_stats": (ctypes.c_int, [_h, ctypes.c_void_p]),
    "dopt_qp_reverse": (ctypes.c_int, [_h, ctypes.c_void_p, ctypes.c_void_p]),
    "dopt_qp_reverse_grads": (ctypes.c_int, [_h] + [ctypes.c_void_p] * 7),
    "dopt_conic_set_csc": (ctypes.c_int, [_h, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_int64] + [ctypes.c_void_p] * 6 + [ctypes.c_int32]),
    "dopt_qp_set_csc": (ctypes.c_int, [_h] + [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                              ctypes.c_int64] * 3 + [ctypes.c_void_p] * 4),
    "dopt_qp_forward": (ctypes.c_int, [_h] + [ctypes.c_void_p] * 7),
    "dopt_qp_forward_reverse": (ctypes.c_int, [_h] + [ctypes.c_void_p] * 9),
    "dopt_qp_reverse_k": (ctypes.c_int, [_h, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p]),
    "dopt_qp_forward_k": (ctypes.c_int, [_h, ctypes.c_int32] + [ctypes.c_void_p] * 7),
    "dopt_conic_forward_reverse": (ctypes.c_int, [_h] + [ctypes.c_void_p] * 10),
    "dopt_conic_lsqr_stats": (ctypes.c_int, [_h, ctypes.c_void_p]),
    "dopt_conic_set_maxiter": (ctypes.c_int, [_h, ctypes.c_int32]),
    "dopt_conic_lsqr_norms": (ctypes.c_int, [_h, ctypes.c_void_p]),
    "dopt_lhs_solve": (ctypes.c_int, [_h, ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.c_int32]),
    "dopt_lhs_resolve": (ctypes.c_int, [_h, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32]),
    "dopt_qp_params_reverse": (ctypes.c_int, [_h, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64]
                               + [ctypes.c_void_p] * 5),
    "dopt_qp_params_forward": (ctypes.c_int, [_h, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64]
                               + [ctypes.c_void_p] * 7),
    "dopt_conic_set": (ctypes.c_int, [_h] + [ctypes.c_void_p] * 6 + [ctypes.c_void_p, ctypes.c_int32]),
    "dopt_conic_factor": (ctypes.c_int, [_h]),
    "dopt_conic_forward": (ctypes.c_int, [_h] + [ctypes.c_void_p] * 5),
    "dopt_conic_reverse": (ctypes.c_int, [_h] + [ctypes.c_void_p] * 5),
    "dopt_nlp_set_structure": (ctypes.c_int, [_h, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                              ctypes.c_int32]),
    "dopt_nlp_set": (ctypes.c_int, [_h] + [ctypes.c_void_p] * 12),
    "dopt_nlp_factor": (ctypes.c_int, [_h]),
    "dopt_nlp_set_deferred": (ctypes.c_int, [_h, ctypes.c_int32]),
    "dopt_nlp_forward": (ctypes.c_int, [_h] + [ctypes.c_void_p] * 3),
    "dopt_nlp_reverse": (ctypes.c_int, [_h] + [ctypes.c_void_p] * 3),
    "dopt_nlp_forward_reverse": (ctypes.c_int, [_h] + [ctypes.c_void_p] * 6),
    "dopt_nlp_jacobian": (ctypes.c_int, [_h, ctypes.c_void_p]),
    "dopt_nlp_get_corrections": (ctypes.c_int, [_h, ctypes.c_void_p]),
    "dopt_nlp_get_layout": (ctypes.c_int, [_h, ctypes.c_void_p]),
    "dopt_nlp_set_kkt": (ctypes.c_int, [_h, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p]),
    "dopt_nlp_kkt_solve": (ctypes.c_int, [_h, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p]),
    "dopt_get_info": (ctypes.c_int, [_h, ctypes.c_void_p]),
    "dopt_get_iterative": (ctypes.c_int, [_h, ctypes.c_void_p]),
    "dopt_qp_get_kept": (ctypes.c_int, [_h, ctypes.c_void_p]),
    "dopt_qp_get_lu_kind": (ctypes.c_int, [_h, ctypes.c_void_p]),
    "dopt_qp_get_sym": (ctypes.c_int, [_h, ctypes.c_void_p]),
    "dopt_get_system_size": (ctypes.c_int, [_h, ctypes.c_void_p]),
    "dopt_last_time": (ctypes.c_double, [_h]),
    "dopt_set_profiling": (ctypes.c_int, [_h, ctypes.c_int32]),
    "dopt_set_profiling_phases": (ctypes.c_int, [_h, ctypes.c_uint32]),
    "dopt_get_phase_times": (ctypes.c_int, [_h, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32]),
    "dopt_phase_name": (ctypes.c_char_p, [ctypes.c_int32]),
}
NUM_PHASES = 11


def phase_mask(lib, names):
    """Bit mask of the phases named (dopt_phase_name), for dopt_set_profiling_phases."""
    known = {lib.dopt_phase_name(i).decode(): i for i in range(NUM_PHASES)}
    mask = 0
    for nm in names:
        if nm not in known:
            raise ValueError(f"unknown phase {nm!r}; phases: {sorted(known)}")
        mask |= 1 << known[nm]
    return mask


ABI_VERSION = 2
LU_KIND_LSQR, LU_KIND_NOPIV, LU_KIND_PIVOT, LU_KIND_SMALL = 0, 1, 2, 3


class EngineUnavailable(RuntimeError):
    pass


class EngineError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"diffopt_mi355x error {code}: {msg}")
        self.code = code


class SingularException(EngineError):
    """Mirror of Julia's ``LinearAlgebra.SingularException(info)`` raised by
    ``LHS \\ RHS`` in the reference (QuadraticProgram.jl:490)."""

    def __init__(self, info):
        super().__init__(info, f"SingularException({info})")
        self.info = info


_lib = None


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise EngineUnavailable(
            f"{LIB_PATH} not found: build the HIP engine first (make -C diffopt.jl_amd)")
    # One HIP runtime per process: PyTorch-ROCm ships its own libamdhip64
    # (soname libamdhip64.so.7).  Loading torch first makes the engine bind to
    # that same runtime, so torch device pointers, streams and RCCL work with
    # the engine; loading the system runtime first would leave torch with no
    # visible GPU (measured on the MI355X box, tools/probe/t_torch2.py).
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = ctypes.CDLL(LIB_PATH)
    if lib.dopt_abi_version() != ABI_VERSION:
        raise EngineUnavailable(f"{LIB_PATH}: ABI version {lib.dopt_abi_version()}, "
                                f"expected {ABI_VERSION} (rebuild the engine)")
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def phase_times(lib, handle):
    import numpy as np
    ms = np.zeros(NUM_PHASES, dtype=np.float64)
    cnt = np.zeros(NUM_PHASES, dtype=np.int32)
    check(lib.dopt_get_phase_times(handle, ms.ctypes.data, cnt.ctypes.data, NUM_PHASES), handle)
    return {lib.dopt_phase_name(i).decode(): (float(ms[i]), int(cnt[i]))
            for i in range(NUM_PHASES) if cnt[i]}


def check(rc, handle=None, singular_ok=False):
    if rc == 0:
        return 0
    if rc > 0:
        if singular_ok:
            return rc
        raise SingularException(rc)
    msg = load().dopt_last_error(handle).decode() if handle else ""
    raise EngineError(rc, msg)
