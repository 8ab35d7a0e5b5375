"""The C-ABI library loads and exports every symbol include/diffopt_mi355x.h
declares (CPU only: no compute calls, no device needed)."""

import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "diffopt_mi355x.h")


def header_symbols():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(dopt_[a-z_]+)\s*\(", src)))


def test_header_declares_the_boundary():
    syms = header_symbols()
    for s in ["dopt_create", "dopt_destroy", "dopt_qp_set", "dopt_qp_factor",
              "dopt_qp_reverse", "dopt_qp_forward", "dopt_conic_set",
              "dopt_conic_forward", "dopt_conic_reverse", "dopt_last_error"]:
        assert s in syms


def test_library_exports_every_header_symbol():
    from diffopt_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("library not built (run __graft_entry__.build())")
    lib = ctypes.CDLL(_lib.LIB_PATH)
    for s in header_symbols():
        assert hasattr(lib, s), f"missing export {s}"
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH],
                         capture_output=True, text=True).stdout
    exported = set(re.findall(r"\b(dopt_[a-z_]+)\b", out))
    assert set(header_symbols()) <= exported


def test_ctypes_table_matches_header():
    from diffopt_amd import _lib
    assert sorted(_lib.SIGNATURES) == header_symbols()


def test_abi_version_and_errors_without_device():
    from diffopt_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("library not built")
    lib = _lib.load()
    assert lib.dopt_abi_version() == _lib.ABI_VERSION
    # null handle paths never touch the device
    assert lib.dopt_last_error(None) == b"null handle"
    assert lib.dopt_destroy(None) == 0
    assert lib.dopt_qp_factor(None) == -1


def test_product_path_has_no_oracle_dependency():
    """The shipped package must never import the CPU oracle."""
    pkg = os.path.join(ROOT, "diffopt.jl_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".hip", ".h", ".cpp", ".jl")):
                txt = open(os.path.join(dirpath, f)).read()
                assert "import oracle" not in txt and "from oracle" not in txt, f
