"""CPU: the Julia shim in INTEGRATION.md binds exactly what include/gpr_hip.h declares.

Julia is not installed here, so the shim cannot run; what can drift silently is its `ccall`
type tuples.  For every `ccall((:gpr_..., lib), Ret, (T1, T2, ...), args...)` in the document
this test checks: the symbol is declared in the header and exported by libgpr_hip.so, the
return type and each argument's Julia type match the header's C type (Cint <-> int,
Float64 <-> double, Ptr{Float64} / Ref{Float64} <-> double* (const or not), Ptr{Cint} /
Ref{Cint} <-> int*, Ptr{Cvoid} <-> a handle or void*, Ref{Ptr{Cvoid}} <-> a handle*,
Cstring <-> const char*, Csize_t <-> size_t), the tuple has the header's arity, and the call
passes as many arguments as its tuple names.  It also pins that the MLL cache update binds the
fused gpr_fit_kinv (the path bench_mll.py measures), and that grad / rdiv! have device methods.
"""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DOC = os.path.join(ROOT, "INTEGRATION.md")
HEADER = os.path.join(ROOT, "include", "gpr_hip.h")


def _split_top(s):
    """Split on commas outside (), {} nesting."""
    out, depth, cur = [], 0, []
    for ch in s:
        if ch in "({[":
            depth += 1
        elif ch in ")}]":
            depth -= 1
        if ch == "," and depth == 0:
            out.append("".join(cur).strip())
            cur = []
        else:
            cur.append(ch)
    if "".join(cur).strip():
        out.append("".join(cur).strip())
    return out


def _match_paren(s, i):
    """Index of the parenthesis closing s[i] == '('."""
    depth = 0
    for j in range(i, len(s)):
        if s[j] == "(":
            depth += 1
        elif s[j] == ")":
            depth -= 1
            if depth == 0:
                return j
    raise ValueError("unbalanced")


def header_prototypes():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    txt = re.sub(r"//[^\n]*", "", txt)
    protos = {}
    for m in re.finditer(r"([A-Za-z_][\w \*]*?)\b(gpr_\w+)\s*\(([^;{]*?)\)\s*;", txt):
        ret, name, args = m.group(1).strip(), m.group(2), m.group(3)
        params = [] if args.strip() in ("", "void") else [a.strip() for a in args.split(",")]
        protos[name] = (ret, params)
    return protos


def _c_type(param):
    """'const double* dX' -> 'double*'; 'gpr_ctx_t ctx' -> 'handle'; 'gpr_ctx_t* out' ->
    'handle*'; 'void* stream' -> 'void*'."""
    p = " ".join(param.replace("*", " * ").split())
    toks = [t for t in p.split(" ") if t != "const"]
    if toks and toks[-1] != "*" and len(toks) > 1:
        toks = toks[:-1]  # drop the parameter name
    base = toks[0]
    stars = toks.count("*")
    if base in ("gpr_ctx_t", "gpr_mgpu_t"):
        return "handle" + "*" * stars
    return base + "*" * stars


_JULIA_TO_C = {
    "Cint": {"int"},
    "Float64": {"double"},
    "Csize_t": {"size_t"},
    "Cstring": {"char*"},
    "Ptr{Float64}": {"double*"},
    "Ref{Float64}": {"double*"},
    "Ptr{Cint}": {"int*"},
    "Ref{Cint}": {"int*"},
    "Ptr{Cvoid}": {"handle", "void*"},
    "Ref{Ptr{Cvoid}}": {"handle*"},
}


def shim_ccalls():
    txt = open(DOC).read()
    calls = []
    for m in re.finditer(r"ccall\(\(:(gpr_\w+),\s*lib\)", txt):
        open_ = txt.index("(", m.start())           # ccall(
        close = _match_paren(txt, open_)
        inner = txt[open_ + 1:close]
        parts = _split_top(inner)
        # parts[0] = (:name, lib), parts[1] = return type, parts[2] = (types...), rest = args
        types = _split_top(parts[2].strip()[1:-1]) if parts[2].strip().startswith("(") else []
        calls.append((m.group(1), parts[1].strip(), types, parts[3:]))
    return calls


def test_every_shim_ccall_matches_the_header():
    protos = header_prototypes()
    calls = shim_ccalls()
    assert len(calls) >= 20
    for name, ret, types, args in calls:
        assert name in protos, f"{name}: not declared in include/gpr_hip.h"
        cret, params = protos[name]
        assert _c_type(cret + " r") in _JULIA_TO_C[ret], f"{name}: returns {cret}, shim says {ret}"
        assert len(types) == len(params), \
            f"{name}: header has {len(params)} parameters, the shim's tuple {len(types)}"
        assert len(args) == len(types), \
            f"{name}: the shim passes {len(args)} arguments for {len(types)} types"
        for k, (jt, cp) in enumerate(zip(types, params)):
            assert jt in _JULIA_TO_C, f"{name} arg {k}: unmapped Julia type {jt}"
            assert _c_type(cp) in _JULIA_TO_C[jt], \
                f"{name} arg {k}: Julia {jt} vs C '{cp}'"


def test_shim_symbols_are_exported():
    import gpr_amd._lib as L
    for name, *_ in shim_ccalls():
        assert hasattr(L.lib, name), f"libgpr_hip.so does not export {name}"


def test_shim_binds_the_fused_and_device_methods():
    txt = open(DOC).read()
    body = txt[txt.index("function GPR.update_cache!(tc::HipMllGradCache"):]
    body = body[:body.index("\nend\n")]
    assert "gpr_fit_kinv" in body  # one fused call, as gpr_amd.core's MllGradCache
    for other in ("gpr_kernel,", "gpr_potrf_upper", "gpr_potrs_upper", "gpr_potri_upper"):
        assert other not in body
    assert re.search(r"function GPR\.grad\(cov::AbstractKernel, i::Integer, hp, x::ROCMat", txt)
    assert "ccall((:gpr_kernel_grad, lib)" in txt
    assert re.search(r"function LinearAlgebra\.rdiv!\(Kxp::ROCMat", txt)
    assert "ccall((:gpr_trsm_upper_trans, lib)" in txt
