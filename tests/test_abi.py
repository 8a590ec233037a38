"""The C-ABI library builds, loads and exports every symbol include/*.h declares (no GPU work)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = sorted(os.path.join(ROOT, "include", h) for h in os.listdir(os.path.join(ROOT, "include"))
                 if h.endswith(".h"))


def declared_symbols():
    names = set()
    for h in HEADERS:
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for m in re.finditer(r"\b(gsr_[a-z0-9_]+)\s*\(", src):
            names.add(m.group(1))
    return sorted(names)


def test_headers_declare_the_boundary():
    names = declared_symbols()
    for required in ("gsr_rasterize_gaussians", "gsr_rasterize_gaussians_backward",
                     "gsr_mark_visible", "gsr_last_error"):
        assert required in names


def test_library_exports_every_declared_symbol():
    from gsr_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.fail("libgsr.so is not built; run __graft_entry__.build()")
    L = _lib.load()
    for name in declared_symbols():
        assert hasattr(L, name), f"{name} declared in include/ but not exported"
        # an untyped ctypes call truncates 64-bit device pointers: every entry point is typed
        assert getattr(L, name).argtypes is not None, f"{name} has no ctypes argtypes"
    assert L.gsr_abi_version() == 1


def test_scratch_sizes_are_monotone_and_aligned():
    from gsr_amd import _lib
    L = _lib.load()
    sizes = [L.gsr_geom_buffer_bytes(p) for p in (0, 1, 1000, 100000)]
    assert sizes == sorted(sizes) and all(s % 256 == 0 for s in sizes)
    # >= 64 B record + 64 B accumulators + keys per Gaussian
    assert L.gsr_geom_buffer_bytes(100000) >= 100000 * 150
    assert L.gsr_binning_buffer_bytes(1000) >= 1000 * 16
    assert L.gsr_image_buffer_bytes(48, 64) >= 64 * 48 * 8


def test_product_package_never_imports_the_oracle():
    pkg = os.path.join(ROOT, "sdp-gs_amd")
    bad = re.compile(r"^\s*(from|import)\s+oracle|gsr_oracle|libgsr_oracle|OracleRaster", re.M)
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".hip", ".cpp", ".h", "Makefile")):
                txt = open(os.path.join(dirpath, f)).read()
                assert not bad.search(txt), f"product file {f} references the oracle"
