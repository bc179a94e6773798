"""ctypes binding of libgpr_hip.so (include/gpr_hip.h).

The product path has no CPU fallback: if the HIP library is missing or cannot be loaded
this module raises ImportError.  ``torch`` is imported first so that the HIP runtime that
torch bundles (soname libamdhip64.so.7) is the one the library binds to -- one runtime per
process, device pointers from torch tensors are then valid in every call.
"""
from __future__ import annotations

import ctypes
import os
import re
from ctypes import POINTER, c_double, c_int, c_longlong, c_size_t, c_void_p

import torch  # noqa: F401  (load torch's HIP runtime before ours)

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GPR_HIP_LIB", os.path.join(HERE, "libgpr_hip.so"))
HEADER = os.path.join(HERE, "..", "..", "include", "gpr_hip.h")

GPR_SE = 1
GPR_WN = 2
GPR_CROSS = 0        # gpr_kernel `same`: kernel!(K, cov, hp, x, xp), x !== xp
GPR_SELF = 1         # kernel!(K, cov, hp, x): eps per SE part + noise
GPR_SAME_OBJECT = 2  # kernel!(K, cov, hp, x, x), x === xp: eps per SE part, no noise
GPR_MGPU_BROADCAST = 0  # gpr_split_predict_mgpu fit modes
GPR_MGPU_REPLICATE = 1
GPR_PREDICT_MEAN = 0
GPR_PREDICT_DIAG = 1
GPR_PREDICT_FULL = 2
GPR_COST_MSE = 1
GPR_COST_CHISQ = 2
GPR_COST_MAHALANOBIS = 3

if not os.path.exists(LIB_PATH):
    raise ImportError(f"libgpr_hip.so not found at {LIB_PATH}: build it with "
                      "`python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback)")
lib = ctypes.CDLL(LIB_PATH)

_i = c_int
_d = c_double
_p = c_void_p
_ip = POINTER(c_int)
_dp = POINTER(c_double)

_SIGS = {
    "gpr_ctx_create": (_i, [_i, _p, POINTER(c_void_p)]),
    "gpr_ctx_destroy": (_i, [_p]),
    "gpr_last_error": (ctypes.c_char_p, [_p]),
    "gpr_version": (ctypes.c_char_p, []),
    "gpr_sync": (_i, [_p]),
    "gpr_ctx_stream": (_p, [_p]),
    "gpr_malloc": (_i, [_p, c_size_t, POINTER(c_void_p)]),
    "gpr_free": (_i, [_p, _p]),
    "gpr_upload": (_i, [_p, _p, _p, c_size_t]),
    "gpr_download": (_i, [_p, _p, _p, c_size_t]),
    "gpr_set_block": (_i, [_p, _i]),
    "gpr_set_outer_block": (_i, [_p, _i]),
    "gpr_set_knob": (_i, [_p, ctypes.c_char_p, _d]),
    "gpr_get_knob": (_i, [_p, ctypes.c_char_p, _dp]),
    "gpr_timing_enable": (_i, [_p, _i]),
    "gpr_timing_get": (_i, [_p, _i, _dp, POINTER(c_longlong), _dp]),
    "gpr_timing_reset": (_i, [_p]),
    "gpr_forget_factor": (_i, [_p]),
    "gpr_kernel": (_i, [_p, _ip, _i, _dp, _i, _p, _i, _p, _i, _i, _d, _p, _i]),
    "gpr_kernel_grad": (_i, [_p, _ip, _i, _dp, _i, _p, _i, _i, _d, _p, _i]),
    "gpr_potrf_upper": (_i, [_p, _p, _i, _i, _ip]),
    "gpr_potrs_upper": (_i, [_p, _p, _i, _i, _p, _i, _i]),
    "gpr_trsm_upper_trans": (_i, [_p, _p, _i, _i, _p, _i, _i]),
    "gpr_potri_upper": (_i, [_p, _p, _i, _i, _p, _i]),
    "gpr_mll": (_i, [_p, _p, _i, _i, _p, _p, _dp]),
    "gpr_mll_grad": (_i, [_p, _ip, _i, _dp, _i, _p, _i, _p, _i, _p, _d, _i, _dp]),
    "gpr_fit": (_i, [_p, _ip, _i, _dp, _i, _p, _i, _p, _i, _i, _d, _p, _i, _p, _ip]),
    "gpr_predict": (_i, [_p, _ip, _i, _dp, _i, _p, _i, _p, _i, _p, _i, _p, _i, _i, _d, _p, _p,
                         _i, _p]),
    "gpr_fit_kinv": (_i, [_p, _ip, _i, _dp, _i, _p, _i, _p, _i, _i, _d, _p, _i, _p, _p, _i, _ip]),
    "gpr_fit_predict": (_i, [_p, _ip, _i, _dp, _i, _p, _i, _p, _i, _i, _d, _p, _i, _p, _p, _i, _i,
                             _p, _p, _i, _p, _ip]),
    "gpr_split_predict": (_i, [_p, _ip, _i, _dp, _i, _p, _i, _p, _i, _p, _p, _i, _p, _i, _i, _i,
                               _i, _i, _d, _p, _p]),
    "gpr_antideriv_se": (_i, [_p, _i, _dp, _p, _i, _dp, _dp, _p, _dp]),
    "gpr_integrate": (_i, [_p, _ip, _i, _dp, _i, _p, _i, _p, _i, _i, _dp, _dp, _d, _p, _i, _p, _dp,
                           _dp]),
    "gpr_integrate_noise": (_i, [_p, _ip, _i, _dp, _i, _p, _i, _p, _i, _i, _dp, _dp, _dp, _d, _dp,
                                 _dp]),
    "gpr_cv_batch": (_i, [_p, _ip, _i, _dp, _i, _p, _i, _p, _ip, _i, _ip, _i, _i, _i, _d, _dp]),
    "gpr_syev_apply": (_i, [_p, _p, _i, _i, _p, _i, _i, _p, _ip]),
    "gpr_sytrd_apply": (_i, [_p, _p, _i, _i, _p, _i, _i, _p, _p]),
    "gpr_split_predict_rows": (_i, [_p, _ip, _i, _dp, _i, _p, _i, _p, _i, _p, _p, _i, _p, _i, _ip,
                                    _i, _i, _i, _d, _p, _p]),
    "gpr_split_predict_shard": (_i, [_p, _ip, _i, _dp, _i, _p, _i, _p, _i, _p, _p, _i, _p, _i, _ip,
                                     _i, _i, _i, _d, _p, _i, _p]),
    "gpr_shard_pieces": (_i, [_i, _i, _i, _i, _i, _ip]),
    "gpr_packed_upper_len": (c_size_t, [_i]),
    "gpr_pack_upper": (_i, [_p, _p, _i, _i, _p]),
    "gpr_unpack_upper": (_i, [_p, _p, _i, _p, _i]),
    "gpr_mgpu_create": (_i, [_i, _ip, POINTER(c_void_p)]),
    "gpr_mgpu_destroy": (_i, [_p]),
    "gpr_mgpu_last_error": (ctypes.c_char_p, [_p]),
    "gpr_mgpu_set_knob": (_i, [_p, ctypes.c_char_p, _d]),
    "gpr_mgpu_get_knob": (_i, [_p, ctypes.c_char_p, _dp]),
    "gpr_split_predict_mgpu": (_i, [_p, _ip, _i, _dp, _i, _dp, _i, _dp, _dp, _i, _dp, _i, _i, _i, _d,
                                    _i, _dp, _dp, _ip]),
    "gpr_split_factors": (_i, [_p, _ip, _i, _dp, _i, _p, _i, _p, _i, _p, _i, _i, _p, _p, _p]),
}

for _name, (_res, _args) in _SIGS.items():
    _f = getattr(lib, _name)  # AttributeError = missing export: fail loudly
    _f.restype = _res
    _f.argtypes = _args


def header_exports(path: str = HEADER):
    """Function names declared in include/gpr_hip.h (for the export test)."""
    txt = open(path).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(gpr_[a-z0-9_]+)\s*\(", txt)))


class GprError(RuntimeError):
    pass


class PosDefException(GprError):
    """Mirror of Julia's LinearAlgebra.PosDefException(info) thrown by cholesky!."""

    def __init__(self, info: int):
        super().__init__(f"PosDefException: matrix is not positive definite; "
                         f"Cholesky factorization failed (info={info})")
        self.info = info
