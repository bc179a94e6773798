"""Host-side mirror of GaussianProcessRegression.jl's model / kernel / loss / predict API.

Every numeric step is a call into libgpr_hip.so; this module only owns device buffers
(torch tensors on one HIP stream), argument checking and the reference's dispatch logic
(which cache, which prior, LogScale or not).  Array conventions are Julia's: ``x`` is
d x N, matrices are (rows, cols) numpy arrays; on the device every matrix is stored
column-major (a torch tensor of shape (cols, rows)).
"""
from __future__ import annotations

import ctypes
import math
from typing import Optional, Sequence, Tuple

import numpy as np
import torch

from . import _lib
from ._lib import GPR_SE, GPR_WN, GprError, PosDefException, lib

F64 = torch.float64
EPS_DEFAULT = 1e-8


# =========================================================================================
# Context: one HIP stream + one libgpr_hip context per device
# =========================================================================================
class Context:
    """A libgpr_hip context bound to a dedicated torch (HIP) stream on ``device``."""

    def __init__(self, device: int = 0, nb: int = 128):
        if not torch.cuda.is_available():
            raise GprError("no HIP device visible: gpr_amd has no CPU fallback")
        self.device = torch.device("cuda", device)
        with torch.cuda.device(self.device):
            self.stream = torch.cuda.Stream(device=self.device)
        h = ctypes.c_void_p()
        rc = lib.gpr_ctx_create(device, ctypes.c_void_p(self.stream.cuda_stream), ctypes.byref(h))
        if rc != 0:
            raise GprError(f"gpr_ctx_create failed ({rc})")
        self.h = h
        if nb != 128:
            self.check(lib.gpr_set_block(self.h, nb))

    def set_knob(self, name: str, value: float) -> None:
        """gpr_set_knob: one of the library's documented switches (include/gpr_hip.h)."""
        self.check(lib.gpr_set_knob(self.h, name.encode(), float(value)), f"set_knob({name})")

    def get_knob(self, name: str) -> float:
        v = ctypes.c_double()
        self.check(lib.gpr_get_knob(self.h, name.encode(), ctypes.byref(v)), f"get_knob({name})")
        return v.value

    def check(self, rc: int, what: str = "") -> int:
        if rc < 0:
            msg = lib.gpr_last_error(self.h).decode()
            raise GprError(f"{what or 'gpr call'} failed ({rc}): {msg}")
        return rc

    def close(self):
        if getattr(self, "h", None):
            lib.gpr_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- device buffers (torch tensors allocated on this context's stream) -------------
    def empty(self, *shape) -> torch.Tensor:
        with torch.cuda.stream(self.stream):
            return torch.empty(*shape, dtype=F64, device=self.device)

    def zeros(self, *shape) -> torch.Tensor:
        with torch.cuda.stream(self.stream):
            return torch.zeros(*shape, dtype=F64, device=self.device)

    def colmajor(self, a) -> torch.Tensor:
        """Upload a Julia-indexed host array (vector or (rows, cols) matrix) column-major."""
        if isinstance(a, torch.Tensor) and a.is_cuda:
            return a
        a = np.asarray(a, dtype=np.float64)
        host = torch.from_numpy(np.ascontiguousarray(a.T))
        with torch.cuda.stream(self.stream):
            return host.to(self.device, non_blocking=False)

    def host(self, t: torch.Tensor, rows: Optional[int] = None) -> np.ndarray:
        """Download a column-major device tensor back to a Julia-indexed numpy array."""
        self.sync()
        a = t.detach().cpu().numpy()
        return a.T.copy() if a.ndim == 2 else a.copy()

    def sync(self):
        self.stream.synchronize()


_DEFAULT: Optional[Context] = None


def default_context() -> Context:
    global _DEFAULT
    if _DEFAULT is None:
        _DEFAULT = Context(0)
    return _DEFAULT


def _ptr(t: Optional[torch.Tensor]):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


# =========================================================================================
# Kernels (src/covariance.jl:15-27,60; src/compose_covar.jl:1-33)
# =========================================================================================
class AbstractKernel:
    def __add__(self, other):
        return ComposedKernel(self.parts() + other.parts())

    def parts(self):
        return (self,)

    def kinds(self):
        return [p.KIND for p in self.parts()]


class SquaredExp(AbstractKernel):
    """K(x,x') = sigma^2 exp(-|l * (x - x')|^2), hp = [sigma, l_1..l_d] (src/covariance.jl:5-15)."""
    KIND = GPR_SE

    def __eq__(self, o):
        return isinstance(o, SquaredExp)

    def __hash__(self):
        return hash("SE")

    def __repr__(self):
        return "SquaredExp()"


class WhiteNoise(AbstractKernel):
    """sigma_n^2 I on a same-object diagonal, hp = [sigma_n] (src/covariance.jl:17,60-64)."""
    KIND = GPR_WN

    def __eq__(self, o):
        return isinstance(o, WhiteNoise)

    def __hash__(self):
        return hash("WN")

    def __repr__(self):
        return "WhiteNoise()"


class ComposedKernel(AbstractKernel):
    """Sum of kernels in `+` order (src/compose_covar.jl:1-19)."""

    def __init__(self, kernels: Sequence[AbstractKernel]):
        self.kernels = tuple(kernels)

    def parts(self):
        return self.kernels

    def __repr__(self):
        return " + ".join(repr(k) for k in self.kernels)


def dim_hp(cov: AbstractKernel, dim: int) -> int:
    """src/covariance.jl:27,60; src/compose_covar.jl:26-28."""
    return sum(dim + 1 if k.KIND == GPR_SE else 1 for k in cov.parts())


class UniformScaling:
    """Julia's `λ*I`, returned by grad(::WhiteNoise) (src/deriv_covar.jl:31)."""

    def __init__(self, lam: float):
        self.lam = float(lam)

    def __repr__(self):
        return f"UniformScaling({self.lam})"


def _kinds_arr(cov: AbstractKernel):
    k = cov.kinds()
    return (ctypes.c_int * len(k))(*k), len(k)


def _hp_arr(hp):
    hp = np.ascontiguousarray(np.asarray(hp, dtype=np.float64))
    return hp, hp.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


# =========================================================================================
# Model (src/models.jl)
# =========================================================================================
class GPRModel:
    """GPRModel(covar, params, x, y; train_axis=1) (src/models.jl:17-37).

    x: d x N, y: N or N x ne.  Inputs are uploaded once and kept on the device."""

    def __init__(self, covar: AbstractKernel, params=None, x=None, y=None, train_axis: int = 1,
                 ctx: Optional[Context] = None, rng=None):
        if x is None:  # GPRModel(cov, x, y) form: random hp (src/models.jl:32-37)
            raise TypeError("x and y are required")
        x_obj = x  # the caller's object: predict(md, x) with this same object is `xp === md.x`
        x = np.asarray(x, dtype=np.float64)
        if x.ndim == 1:
            x = x[None, :]
        y = np.asarray(y, dtype=np.float64)
        d = x.shape[0]
        if params is None:
            rng = rng or np.random.default_rng()
            params = rng.random(dim_hp(covar, d))
        params = np.array(params, dtype=np.float64)
        if params.shape[0] != dim_hp(covar, d):
            raise ValueError("Parameter size mismatch.")  # src/models.jl:27
        if x.shape[-1] != y.shape[0]:
            raise ValueError("x and y size mismatch.")  # src/models.jl:28
        self.covar = covar
        self.params = params
        self.x = x
        self._x_obj = x_obj
        self.y = y
        self.train_axis = int(train_axis)
        self.ctx = ctx or default_context()
        self._dx = None
        self._dy = None

    @property
    def d(self):
        return self.x.shape[0]

    @property
    def n(self):
        return self.x.shape[1]

    def dx(self) -> torch.Tensor:
        if self._dx is None:
            self._dx = self.ctx.colmajor(self.x)
        return self._dx

    def dy(self) -> torch.Tensor:
        if self._dy is None:
            self._dy = self.ctx.colmajor(self.y)
        return self._dy

    def add_to_y(self, dy):
        """md.y .+= dy (src/update_model.jl:43); the device copy is refreshed on next use."""
        self.y = self.y + np.asarray(dy, dtype=np.float64)
        self._dy = None

    def dsample(self) -> torch.Tensor:
        """get_sample(md) on the device (src/models.jl:39-45)."""
        y = self.dy()
        return y if y.ndim == 1 else y[self.train_axis - 1]

    def __repr__(self):
        return f"GPRModel({self.covar!r}, d={self.d}, N={self.n})"


def get_sample(md: GPRModel) -> np.ndarray:
    return md.y if md.y.ndim == 1 else md.y[:, md.train_axis - 1]


# =========================================================================================
# kernel / grad (src/covariance.jl, src/compose_covar.jl, src/deriv_covar.jl)
# =========================================================================================
def kernel(cov: AbstractKernel, hp, x, xp=None, eps: float = EPS_DEFAULT,
           ctx: Optional[Context] = None, out: Optional[torch.Tensor] = None, host: bool = True):
    """kernel(cov, hp, x[, xp]) -> N x M matrix.

    ``xp is None`` is the 4-arg kernel!(K, cov, hp, x): eps per SE part plus the noise of a
    WhiteNoise part (src/compose_covar.jl:73-77).  ``xp is x`` is the 5-arg call with
    `x === xp`: eps per SE part, no noise (src/compose_covar.jl:47-61,
    src/covariance.jl:52-56).  Any other xp is a cross kernel."""
    ctx = ctx or default_context()
    dx = ctx.colmajor(x)
    n = dx.shape[0]
    d = dx.shape[1] if dx.ndim == 2 else 1
    kinds, nk = _kinds_arr(cov)
    hpa, hpp = _hp_arr(hp)
    if xp is None:
        m, dxp, same = n, None, _lib.GPR_SELF
    elif xp is x:
        m, dxp, same = n, None, _lib.GPR_SAME_OBJECT
    else:
        dxp = ctx.colmajor(xp)
        m, same = dxp.shape[0], _lib.GPR_CROSS
    K = out if out is not None else ctx.empty(m, n)
    ctx.check(lib.gpr_kernel(ctx.h, kinds, nk, hpp, d, _ptr(dx), n, _ptr(dxp), m, same, eps,
                             _ptr(K), n), "gpr_kernel")
    return ctx.host(K) if host else K


def kernel_grad(cov: AbstractKernel, i: int, hp, x, eps: float = EPS_DEFAULT,
                ctx: Optional[Context] = None):
    """grad(cov, i, hp, x) (src/deriv_covar.jl:2-32): dK/dtheta_i, i is 1-based."""
    ctx = ctx or default_context()
    hp = np.asarray(hp, dtype=np.float64)
    dim = np.asarray(x).shape[0]
    # WhiteNoise part -> UniformScaling like the reference
    off = 0
    for k in cov.parts():
        w = dim + 1 if k.KIND == GPR_SE else 1
        if off < i <= off + w and k.KIND == GPR_WN:
            return UniformScaling(2.0 * hp[off])
        off += w
    dx = ctx.colmajor(x)
    n, d = dx.shape
    kinds, nk = _kinds_arr(cov)
    hpa, hpp = _hp_arr(hp)
    DK = ctx.empty(n, n)
    ctx.check(lib.gpr_kernel_grad(ctx.h, kinds, nk, hpp, d, _ptr(dx), n, int(i), eps, _ptr(DK), n),
              "gpr_kernel_grad")
    return ctx.host(DK)


# =========================================================================================
# Losses (src/loss_grad.jl, src/cost.jl, src/caches/cost.jl)
# =========================================================================================
class MarginalLikelihood:
    """Negative log marginal likelihood (src/loss_grad.jl:5,39-52)."""


class LogScale:
    pass


class NoLogScale:
    pass


def islog(cost, md: GPRModel):
    """src/cost.jl:4-8: LogScale iff an SE part is present."""
    return LogScale() if any(k.KIND == GPR_SE for k in md.covar.parts()) else NoLogScale()


class MllLossCache:
    """Device-resident MllLossCache(hp, kchol_base, alpha) (src/caches/cost.jl:6-19)."""

    def __init__(self, md: GPRModel):
        self.ctx = md.ctx
        self.hp = md.params.copy()
        self.kchol_base = self.ctx.empty(md.n, md.n)  # column-major N x N
        self.alpha = self.ctx.empty(md.n)
        self.info = 0


class MllGradCache(MllLossCache):
    """Device-resident MllGradCache (src/caches/cost.jl:21-44): K/U, alpha, K^{-1}.

    The reference keeps per-part kernel matrices and a dK buffer; the fused gradient
    recomputes K_p and dK in registers, so only U, alpha and K^{-1} are kept."""

    def __init__(self, md: GPRModel):
        super().__init__(md)
        self.Kinv = self.ctx.empty(md.n, md.n)


def update_cache_(tc: MllLossCache, hp, md: GPRModel, eps: float = EPS_DEFAULT):
    """update_cache!(tc, hp, md) (src/cost.jl:74-111): K, in-place POTRF, alpha = K^{-1} y,
    and for MllGradCache also K^{-1}."""
    ctx = md.ctx
    tc.hp = np.array(hp, dtype=np.float64)
    kinds, nk = _kinds_arr(md.covar)
    hpa, hpp = _hp_arr(tc.hp)
    y = md.dsample()
    info = ctypes.c_int(0)
    n = md.n
    if isinstance(tc, MllGradCache):  # K, U, alpha and K^{-1} in one call (src/cost.jl:83-111)
        rc = lib.gpr_fit_kinv(ctx.h, kinds, nk, hpp, md.d, _ptr(md.dx()), n, _ptr(y), 1, n, eps,
                              _ptr(tc.kchol_base), n, _ptr(tc.alpha), _ptr(tc.Kinv), n,
                              ctypes.byref(info))
    else:
        rc = lib.gpr_fit(ctx.h, kinds, nk, hpp, md.d, _ptr(md.dx()), n, _ptr(y), 1, n, eps,
                         _ptr(tc.kchol_base), n, _ptr(tc.alpha), ctypes.byref(info))
    tc.info = info.value
    if info.value != 0:
        raise PosDefException(info.value)
    ctx.check(rc, "gpr_fit")


def _mll_value(md: GPRModel, tc: MllLossCache) -> float:
    ctx = md.ctx
    out = ctypes.c_double(0.0)
    ctx.check(lib.gpr_mll(ctx.h, _ptr(tc.kchol_base), md.n, md.n, _ptr(md.dsample()),
                          _ptr(tc.alpha), ctypes.byref(out)), "gpr_mll")
    return out.value


def _mll_grad(md: GPRModel, tc: MllGradCache, eps=EPS_DEFAULT, log_scale=False) -> np.ndarray:
    ctx = md.ctx
    kinds, nk = _kinds_arr(md.covar)
    hpa, hpp = _hp_arr(tc.hp)
    g = np.zeros(len(hpa))
    ctx.check(lib.gpr_mll_grad(ctx.h, kinds, nk, hpp, md.d, _ptr(md.dx()), md.n, _ptr(tc.Kinv),
                               md.n, _ptr(tc.alpha), eps, 1 if log_scale else 0,
                               g.ctypes.data_as(ctypes.POINTER(ctypes.c_double))), "gpr_mll_grad")
    return g


def loss(cost, hp_or_md, md: Optional[GPRModel] = None, tc: Optional[MllLossCache] = None,
         eps: float = EPS_DEFAULT) -> float:
    """loss(MLL, md) / loss(MLL, hp, md) / loss(MLL, hp, md, tc) (src/cost.jl:17-22,40-43)."""
    if md is None:
        md, hp = hp_or_md, hp_or_md.params
    else:
        hp = hp_or_md
    tc = tc or MllLossCache(md)
    update_cache_(tc, hp, md, eps)
    return _mll_value(md, tc)


def grad_(dL: np.ndarray, cost, hp, md: GPRModel, tc: Optional[MllGradCache] = None,
          eps: float = EPS_DEFAULT):
    """grad!(dL, MLL, hp, md[, tc]) (src/cost.jl:32-36,45-48,119-126)."""
    tc = tc or MllGradCache(md)
    update_cache_(tc, hp, md, eps)
    dL[:] = _mll_grad(md, tc, eps)


def grad(cost_or_cov, *args, **kw):
    """grad(MLL, md) / grad(MLL, hp, md) (src/cost.jl:24-30), or the kernel derivative
    grad(cov, i, hp, x) (src/deriv_covar.jl:2-10)."""
    if isinstance(cost_or_cov, AbstractKernel):
        return kernel_grad(cost_or_cov, *args, **kw)
    if len(args) == 1:
        md = args[0]
        hp = md.params
    else:
        hp, md = args[0], args[1]
    g = np.zeros(len(hp))
    grad_(g, cost_or_cov, hp, md, **kw)
    return g


def loss_grad_(cost, F, G, hp, md: GPRModel, tc: MllGradCache, eps: float = EPS_DEFAULT):
    """loss_grad!(cost, F, G, hp, md, tc) (src/cost.jl:50-58)."""
    update_cache_(tc, hp, md, eps)
    if G is not None:
        G[:] = _mll_grad(md, tc, eps)
    if F is not None:
        return _mll_value(md, tc)


def log_loss_grad_(cost, F, G, log_hp, md: GPRModel, tc: MllGradCache, eps: float = EPS_DEFAULT):
    """log_loss_grad!(cost, F, G, log_hp, md, tc) (src/cost.jl:60-70): hp = exp(log_hp),
    G .*= hp."""
    hp = np.exp(np.asarray(log_hp, dtype=np.float64))
    update_cache_(tc, hp, md, eps)
    if G is not None:
        G[:] = _mll_grad(md, tc, eps, log_scale=True)
    if F is not None:
        return _mll_value(md, tc)


# =========================================================================================
# Posterior (src/predict.jl, src/caches/predict.jl)
# =========================================================================================
class GPRPredictCache:
    """Device-resident GPRPredictCache(Kxx, wt, Kxp) (src/caches/predict.jl:3-31).

    Kxx holds the factor U after update_cache_; Kxp is kept transposed (N x np)."""

    def __init__(self, md: GPRModel, nxp: int = 0):
        self.ctx = md.ctx
        self.Kxx = self.ctx.empty(md.n, md.n)
        ny = 1 if md.y.ndim == 1 else md.y.shape[1]
        self.wt = self.ctx.empty(ny, md.n) if md.y.ndim == 2 else self.ctx.empty(md.n)
        self.nrhs = ny
        self.Kxp = self.ctx.empty(max(nxp, 1), md.n)


def _update_predict_cache(pc, md: GPRModel, eps=EPS_DEFAULT):
    """update_cache!(pc, md) (src/predict.jl:29-34): solves against md.y (all columns)."""
    ctx = md.ctx
    kinds, nk = _kinds_arr(md.covar)
    hpa, hpp = _hp_arr(md.params)
    info = ctypes.c_int(0)
    ctx.check(lib.gpr_fit(ctx.h, kinds, nk, hpp, md.d, _ptr(md.dx()), md.n, _ptr(md.dy()), pc.nrhs,
                          md.n, eps, _ptr(pc.Kxx), md.n, _ptr(pc.wt), ctypes.byref(info)),
              "gpr_fit")
    if info.value != 0:
        raise PosDefException(info.value)


def _dxp(md: GPRModel, xp) -> torch.Tensor:
    """Test points on the device.  ``xp is md.x`` hands the library the training inputs'
    own device buffer: pointer identity is how the C ABI sees `xp === md.x`, the
    reference's same-object branch of kernel!(Kxp, covar, hp, xp, md.x) (src/predict.jl:37,43:
    eps per SE part on Kxp's diagonal, no noise)."""
    if xp is md.x or xp is md._x_obj or (isinstance(xp, torch.Tensor) and xp is md._dx):
        return md.dx()
    return md.ctx.colmajor(xp)


def predict_(mu: Optional[torch.Tensor], Sigma: Optional[torch.Tensor], md: GPRModel, xp,
             pc: GPRPredictCache, diagonal_var: bool, mean_only: bool = False,
             eps: float = EPS_DEFAULT):
    """predict!(mu, Sigma, md, xp, pc) (src/predict.jl:36-71) on device buffers."""
    ctx = md.ctx
    kinds, nk = _kinds_arr(md.covar)
    hpa, hpp = _hp_arr(md.params)
    dxp = _dxp(md, xp)
    m = dxp.shape[0]
    if pc.Kxp.numel() < m * md.n:
        pc.Kxp = ctx.empty(m, md.n)
    mode = (_lib.GPR_PREDICT_MEAN if mean_only else
            _lib.GPR_PREDICT_DIAG if diagonal_var else _lib.GPR_PREDICT_FULL)
    ldv = m
    ctx.check(lib.gpr_predict(ctx.h, kinds, nk, hpp, md.d, _ptr(md.dx()), md.n, _ptr(pc.Kxx), md.n,
                              _ptr(pc.wt), pc.nrhs, _ptr(dxp), m, mode, eps, _ptr(mu), _ptr(Sigma),
                              ldv, _ptr(pc.Kxp)), "gpr_predict")


def predict_mean(md: GPRModel, xp, eps: float = EPS_DEFAULT) -> np.ndarray:
    """predict_mean(md, xp) (src/predict.jl:6-12)."""
    ctx = md.ctx
    m = np.asarray(xp).shape[-1]
    pc = GPRPredictCache(md, m)
    _update_predict_cache(pc, md, eps)
    mu = ctx.empty(pc.nrhs, m) if pc.nrhs > 1 else ctx.empty(m)
    predict_(mu, None, md, xp, pc, True, mean_only=True, eps=eps)
    return ctx.host(mu)


def predict(md: GPRModel, xp, diagonal_var: bool = False, eps: float = EPS_DEFAULT,
            var_range: Tuple[int, int] = (1, 3)):
    """predict(md, xp; diagonal_var) (src/predict.jl:14-25).  Returns (mu, Sigma): Sigma is
    an np x np matrix (full) or the diagonal vector.  For a Cmap grid dispatches to the split
    path (src/split_predict.jl:1), which requires diagonal_var=True."""
    if isinstance(xp, Cmap):
        return _split_predict(md, xp, eps=eps, var_range=var_range)
    ctx = md.ctx
    pc = GPRPredictCache(md, 0)
    dxp = _dxp(md, xp)
    m = dxp.shape[0]
    mu = ctx.empty(pc.nrhs, m) if pc.nrhs > 1 else ctx.empty(m)
    Sigma = ctx.empty(m) if diagonal_var else ctx.empty(m, m)
    _fit_predict(md, dxp, m, pc, mu, Sigma, diagonal_var, eps)
    return ctx.host(mu), ctx.host(Sigma)


def _fit_predict(md: GPRModel, dxp, m: int, pc: GPRPredictCache, mu, Sigma, diagonal_var: bool,
                 eps: float = EPS_DEFAULT):
    """update_cache!(pc, md) + predict!(mu, Sigma, md, xp, pc) (src/predict.jl:29-71) as ONE
    device call: the triangular solve of [K(x, xp) | y] runs inside the factorisation
    (gpr_fit_predict); pc.Kxx receives U (lower triangle keeps K), pc.wt = K^{-1} y."""
    ctx = md.ctx
    kinds, nk = _kinds_arr(md.covar)
    hpa, hpp = _hp_arr(md.params)
    mode = _lib.GPR_PREDICT_DIAG if diagonal_var else _lib.GPR_PREDICT_FULL
    info = ctypes.c_int(0)
    rc = lib.gpr_fit_predict(ctx.h, kinds, nk, hpp, md.d, _ptr(md.dx()), md.n, _ptr(md.dy()),
                             pc.nrhs, md.n, eps, _ptr(pc.Kxx), md.n, _ptr(pc.wt), _ptr(dxp), m,
                             mode, _ptr(mu), _ptr(Sigma), m, None, ctypes.byref(info))
    if info.value != 0:
        raise PosDefException(info.value)
    ctx.check(rc, "gpr_fit_predict")


# =========================================================================================
# Split kernel prediction (src/split_kernel.jl, src/split_predict.jl)
# =========================================================================================
class Cmap:
    """Cmap(op, xe, xq): virtual grid x_{e,q} = op(xe_e, xq_q) (src/split_kernel.jl:1-17).
    Only op = '+' (the only one the reference's tests and predict path use)."""

    def __init__(self, op, xe, xq):
        if op not in ("+", np.add) and op is not np.add:
            raise ValueError("Cmap supports op '+' only")
        self.op = "+"
        self.xe = np.asarray(xe, dtype=np.float64)
        self.xq = np.asarray(xq, dtype=np.float64)

    @property
    def shape(self):
        return (self.xe.shape[0], self.xe.shape[1], self.xq.shape[1])

    def points(self) -> np.ndarray:
        """xeq[:, :]: column e + (q-1) ne (src/split_kernel.jl:12-15)."""
        d, ne = self.xe.shape
        nq = self.xq.shape[1]
        return (self.xe[:, :, None] + self.xq[:, None, :]).reshape(d, ne * nq, order="F")


class GPRSplitPredictCache:
    """GPRSplitPredictCache(...; var_range=1:3) (src/caches/split_kernel.jl:1-30)."""

    def __init__(self, md: GPRModel, ne: int, nq: int, var_range: Tuple[int, int] = (1, 3)):
        self.ctx = md.ctx
        self.Kxx = self.ctx.empty(md.n, md.n)
        self.wt = self.ctx.empty(md.n)
        self.var_range = var_range  # 1-based inclusive, like Julia's UnitRange


def split_predict_(md: GPRModel, cm: Cmap, pc: GPRSplitPredictCache, mu: torch.Tensor,
                   var: torch.Tensor, e_lo: int = 0, e_hi: Optional[int] = None,
                   eps: float = EPS_DEFAULT):
    """Split-kernel mean + diagonal variance for grid rows [e_lo, e_hi) (0-based) into the
    full-layout device buffers mu (ne x nq col-major) and var (ne*nq)."""
    ctx = md.ctx
    kinds, nk = _kinds_arr(md.covar)
    hpa, hpp = _hp_arr(md.params)
    _, ne, nq = cm.shape
    e_hi = ne if e_hi is None else e_hi
    dxe = ctx.colmajor(cm.xe)
    dxq = ctx.colmajor(cm.xq)
    vlo, vhi = pc.var_range
    ctx.check(lib.gpr_split_predict(ctx.h, kinds, nk, hpp, md.d, _ptr(md.dx()), md.n, _ptr(pc.Kxx),
                                    md.n, _ptr(pc.wt), _ptr(dxe), ne, _ptr(dxq), nq, e_lo, e_hi,
                                    vlo - 1, vhi, eps, _ptr(mu), _ptr(var)), "gpr_split_predict")


def _split_predict(md: GPRModel, cm: Cmap, eps=EPS_DEFAULT, var_range=(1, 3)):
    if md.y.ndim != 1:
        raise ValueError("split prediction needs a 1-D y (Diagonal(wt), src/split_predict.jl:13)")
    ctx = md.ctx
    _, ne, nq = cm.shape
    pc = GPRSplitPredictCache(md, ne, nq, var_range)
    _update_predict_cache(pc_adapter(pc), md, eps)
    mu = ctx.empty(nq, ne)   # ne x nq column-major
    var = ctx.empty(ne * nq)
    split_predict_(md, cm, pc, mu, var, eps=eps)
    return ctx.host(mu), ctx.host(var)


class pc_adapter:
    def __init__(self, pc):
        self.Kxx, self.wt, self.nrhs = pc.Kxx, pc.wt, 1


def split_factors(cov: AbstractKernel, hp, x, cm: Cmap, part: int = 0,
                  ctx: Optional[Context] = None):
    """The SplitKernel factors A (ne x nq), B (ne x ns), C (ns x nq) of SE part `part`
    (src/split_kernel.jl:151-159), for inspection/tests."""
    ctx = ctx or default_context()
    dx, dxe, dxq = ctx.colmajor(x), ctx.colmajor(cm.xe), ctx.colmajor(cm.xq)
    ns, d = dx.shape
    _, ne, nq = cm.shape
    kinds, nk = _kinds_arr(cov)
    hpa, hpp = _hp_arr(hp)
    A, B, C = ctx.empty(nq, ne), ctx.empty(ns, ne), ctx.empty(nq, ns)
    ctx.check(lib.gpr_split_factors(ctx.h, kinds, nk, hpp, d, _ptr(dx), ns, _ptr(dxe), ne, _ptr(dxq),
                                    nq, part, _ptr(A), _ptr(B), _ptr(C)), "gpr_split_factors")
    return ctx.host(A), ctx.host(B), ctx.host(C)


# =========================================================================================
# Cache constructors and small API pieces the reference exports around the path
# =========================================================================================
def loss_cache(cost):
    """loss_cache(::MarginalLikelihood) = MllLossCache (src/cost.jl:10)."""
    if not isinstance(cost, MarginalLikelihood):
        raise TypeError(f"no loss cache for {cost!r}")
    return MllLossCache


def grad_cache(cost):
    """grad_cache / loss_grad_cache(::MarginalLikelihood) = MllGradCache (src/cost.jl:11-12)."""
    if not isinstance(cost, MarginalLikelihood):
        raise TypeError(f"no gradient cache for {cost!r}")
    return MllGradCache


loss_grad_cache = grad_cache


def predict_cache(md: GPRModel, xp):
    """predict_cache(md, xp) (src/predict.jl:1, src/split_predict.jl:1): the cache type."""
    return GPRSplitPredictCache if isinstance(xp, Cmap) else GPRPredictCache


def update_predict_cache_(pc: GPRPredictCache, md: GPRModel, eps: float = EPS_DEFAULT):
    """update_cache!(pc::GPRPredictCache, md) (src/predict.jl:29-34): K, cholesky!, wt."""
    _update_predict_cache(pc, md, eps)


def predict_mean_(mu: torch.Tensor, md: GPRModel, xp, pc: GPRPredictCache,
                  eps: float = EPS_DEFAULT):
    """predict_mean!(mu, md, xp, pc) (src/predict.jl:36-40) from an updated cache."""
    predict_(mu, None, md, xp, pc, True, mean_only=True, eps=eps)


def similar(md: GPRModel, hp, x, y) -> GPRModel:
    """similar(md, hp, x, y) (src/models.jl:47-49): same kernel, new data."""
    return GPRModel(md.covar, hp, x, y, train_axis=md.train_axis, ctx=md.ctx)


def _part_hps(cov: AbstractKernel, hp, dim: int):
    hp = np.asarray(hp, dtype=np.float64)
    out, off = [], 0
    for k in cov.parts():
        w = dim + 1 if k.KIND == GPR_SE else 1
        out.append(hp[off:off + w])
        off += w
    return out


def kernels(cov: AbstractKernel, hp, x, eps: float = EPS_DEFAULT, ctx: Optional[Context] = None):
    """kernels(K, hp, x) (src/compose_covar.jl:80-107): one N x N matrix per part of a
    composed kernel, a 1 x 1 zero for WhiteNoise (alloc_kernels :90-95); [kernel(K, hp, x)]
    for a single kernel.  Each part's matrix is built on the device."""
    x = np.asarray(x, dtype=np.float64)
    x = x[None, :] if x.ndim == 1 else x
    if not isinstance(cov, ComposedKernel):
        return [kernel(cov, hp, x, eps=eps, ctx=ctx)]
    return [np.zeros((1, 1)) if k.KIND == GPR_WN else kernel(k, h, x, eps=eps, ctx=ctx)
            for k, h in zip(cov.parts(), _part_hps(cov, hp, x.shape[0]))]


def rm_noise(cov: AbstractKernel, hps):
    """rm_noise(K::ComposedKernel, hps) (src/compose_covar.jl:30-33): the parts and per-part
    hyperparameter vectors without the WhiteNoise entries."""
    keep = [i for i, k in enumerate(cov.parts()) if k.KIND != GPR_WN]
    return [cov.parts()[i] for i in keep], [hps[i] for i in keep]
