"""CPU: the C-ABI library loads and exports every symbol include/gpr_hip.h declares
(no compute calls: there is no GPU here)."""
import ctypes
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "gaussianprocessregression.jl_amd", "gpr_amd", "libgpr_hip.so")


def test_library_exports_every_header_symbol():
    import gpr_amd._lib as L
    names = L.header_exports()
    assert len(names) >= 25
    for n in names:
        assert hasattr(L.lib, n), f"libgpr_hip.so does not export {n}"
        assert n in L._SIGS, f"{n} declared in the header but not bound in _lib.py"
    assert set(L._SIGS) == set(names)


def test_library_is_gfx950_code_object():
    data = open(LIB, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data
    assert b"gfx942" not in data and b"gfx90a" not in data  # gfx950 only, no dual paths


def test_version_and_no_gpu_error_path():
    import gpr_amd._lib as L
    assert b"gfx950" in L.lib.gpr_version()
    assert L.lib.gpr_last_error(None) == b"null context"


def test_product_path_fails_loudly_without_library(tmp_path, monkeypatch):
    import importlib
    import sys
    monkeypatch.setenv("GPR_HIP_LIB", str(tmp_path / "missing.so"))
    sys.modules.pop("gpr_amd._lib", None)
    with pytest.raises(ImportError):
        importlib.import_module("gpr_amd._lib")
    sys.modules.pop("gpr_amd._lib", None)
    monkeypatch.delenv("GPR_HIP_LIB")
    importlib.import_module("gpr_amd._lib")


def test_product_package_never_imports_oracle():
    pkg = os.path.join(ROOT, "gaussianprocessregression.jl_amd")
    for dp, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".hip", ".hpp", ".cpp", ".jl")):
                txt = open(os.path.join(dp, f)).read()
                assert "oracle" not in txt.replace("oracle/", "").lower() or f.endswith(".md"), f
