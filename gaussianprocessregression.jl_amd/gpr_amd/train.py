"""Hyper-parameter training and model updates on device-resident caches (SURVEY.md §8(f)
ranks 1 and 4).

Mirrors src/train.jl:1-87 (``init_params``, ``train`` for zeroth/first/second-order methods,
LogScale optimisation in log space) and src/update_model.jl:1-100 (``update_sample!`` with the
``BFGSQuad`` updater, ``hessian_fd``, ``bfgs_hessian``, ``bfgs_quad``).

Every loss / gradient evaluation runs on the GPU through libgpr_hip.so (K-assembly, POTRF,
POTRS, POTRI and the fused gradient of core.update_cache_ / core._mll_grad) on ONE
MllGradCache kept resident for the whole optimisation: per iteration only the D
hyper-parameters go down and the loss and D gradient components come back.  The optimiser
itself is host control logic: the reference uses Optim.jl (not vendored, Manifest.toml), here
SciPy's ``optimize.minimize`` with the matching algorithm family stands in for it (CG for
ConjugateGradient, L-BFGS-B for LBFGS, BFGS, Nelder-Mead, and trust-exact with the
finite-difference Hessian of the gradient for NewtonTrustRegion, which is what Optim builds from
an (f, g!) pair).  Step sequences of the two libraries differ, so parity is on the optimum
(tests/test_gpu_train.py), not on the iterates.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Callable, Optional

import numpy as np

from . import core as C

# -----------------------------------------------------------------------------------------
# Optim.jl method / options stand-ins
# -----------------------------------------------------------------------------------------


class _Method:
    order = 1
    scipy = "CG"

    def __repr__(self):
        return f"{type(self).__name__}()"


class NelderMead(_Method):
    """Optim.NelderMead (ZerothOrderOptimizer)."""
    order, scipy = 0, "Nelder-Mead"


class ConjugateGradient(_Method):
    """Optim.ConjugateGradient (FirstOrderOptimizer) -- train's default (src/train.jl:10)."""
    order, scipy = 1, "CG"


class BFGS(_Method):
    order, scipy = 1, "BFGS"


class LBFGS(_Method):
    order, scipy = 1, "L-BFGS-B"


class NewtonTrustRegion(_Method):
    """Optim.NewtonTrustRegion (SecondOrderOptimizer; Hessian by finite differences of g)."""
    order, scipy = 2, "trust-exact"


@dataclass
class Options:
    """The Optim.Options fields the reference's tests use (g_tol, iterations, show_trace)."""
    g_tol: float = 1e-8
    iterations: int = 1000
    f_tol: float = 0.0
    show_trace: bool = False


@dataclass
class OptimResult:
    """What train's callers read from Optim's result (Optim.minimizer, g_converged, ...)."""
    minimizer: np.ndarray
    minimum: float
    iterations: int
    f_calls: int
    g_calls: int
    g_residual: float
    g_converged: bool
    method: str
    message: str = ""
    trace: list = field(default_factory=list)


def g_converged(res: OptimResult) -> bool:
    return res.g_converged


def minimizer(res: OptimResult) -> np.ndarray:
    return res.minimizer


def init_params(cost, md: C.GPRModel, rng=None) -> np.ndarray:
    """init_params (src/train.jl:1-7): ones for the marginal likelihood, else uniform."""
    if isinstance(cost, C.MarginalLikelihood):
        return np.ones(len(md.params))
    rng = rng or np.random.default_rng()
    return rng.random(len(md.params))


# -----------------------------------------------------------------------------------------
# train (src/train.jl:9-87)
# -----------------------------------------------------------------------------------------
class _Objective:
    """f / g / (f, g) in the optimisation variable (log hp under LogScale) over one resident
    cache; repeated points are served from the last evaluation (SciPy asks for f and g at the
    same x separately for some methods)."""

    def __init__(self, cost, md: C.GPRModel, log: bool, need_grad: bool):
        self.cost, self.md, self.log = cost, md, log
        self.tc = C.MllGradCache(md) if need_grad else C.MllLossCache(md)
        self.f_calls = self.g_calls = 0
        self._x = None
        self._f = None
        self._g = None

    def _eval(self, x, want_g: bool):
        x = np.array(x, dtype=np.float64)
        if self._x is not None and np.array_equal(x, self._x) and (self._g is not None or not want_g):
            return
        G = np.zeros(len(x)) if want_g else None
        if self.log:
            if want_g:
                f = C.log_loss_grad_(self.cost, True, G, x, self.md, self.tc)
            else:
                f = C.loss(self.cost, np.exp(x), self.md, self.tc)
        else:
            if want_g:
                f = C.loss_grad_(self.cost, True, G, x, self.md, self.tc)
            else:
                f = C.loss(self.cost, x, self.md, self.tc)
        self.f_calls += 1
        self.g_calls += int(want_g)
        self._x, self._f, self._g = x, float(f), G

    def f(self, x):
        self._eval(x, False)
        return self._f

    def fg(self, x):
        self._eval(x, True)
        return self._f, self._g.copy()

    def g(self, x):
        self._eval(x, True)
        return self._g.copy()


def train(md: C.GPRModel, cost, hp0=None, method: Optional[_Method] = None,
          options: Optional[Options] = None):
    """train(md, cost, hp0; method, options) -> (hpmin, res) (src/train.jl:9-87).

    LogScale (any SE part, src/cost.jl:4-8): the optimiser works on log(hp), the loss is taken
    at exp(x) and the gradient is log_loss_grad!'s (G .*= hp); the minimizer is returned as
    exp(x).  hp0 is used as given in both cases, as in the reference."""
    from scipy import optimize

    method = method or ConjugateGradient()
    options = options or Options()
    hp0 = init_params(cost, md) if hp0 is None else np.array(hp0, dtype=np.float64)
    log = isinstance(C.islog(cost, md), C.LogScale)
    obj = _Objective(cost, md, log, need_grad=method.order >= 1)
    x0 = hp0.copy()
    trace = []
    cb = (lambda xk, *a: trace.append(np.array(xk))) if options.show_trace else None
    if method.order == 0:
        r = optimize.minimize(obj.f, x0, method=method.scipy, callback=cb,
                              options={"maxiter": options.iterations,
                                       "fatol": options.f_tol or 1e-8})
    elif method.order == 1:
        r = optimize.minimize(obj.fg, x0, jac=True, method=method.scipy, callback=cb,
                              options={"maxiter": options.iterations, "gtol": options.g_tol})
    else:
        hess = lambda x: _sym(hessian_fd(obj.g, x))  # noqa: E731
        r = optimize.minimize(obj.f, x0, jac=obj.g, hess=hess, method=method.scipy,
                              callback=cb, options={"maxiter": options.iterations,
                                                    "gtol": options.g_tol})
    xmin = np.array(r.x, dtype=np.float64)
    gmin = obj.g(xmin) if method.order >= 1 else None
    gres = float(np.max(np.abs(gmin))) if gmin is not None else float("nan")
    res = OptimResult(minimizer=xmin, minimum=float(obj.f(xmin)), iterations=int(r.get("nit", 0)),
                      f_calls=obj.f_calls, g_calls=obj.g_calls, g_residual=gres,
                      g_converged=bool(gmin is not None and gres <= options.g_tol),
                      method=repr(method), message=str(r.get("message", "")), trace=trace)
    hpmin = np.exp(xmin) if log else xmin
    return hpmin, res


def _sym(h: np.ndarray) -> np.ndarray:
    return 0.5 * (h + h.T)


# -----------------------------------------------------------------------------------------
# update_sample! / BFGSQuad (src/update_model.jl, src/caches/update_model.jl)
# -----------------------------------------------------------------------------------------
def hessian_fd_(hess: np.ndarray, gradfn: Callable, x, eps: float = 1e-6) -> np.ndarray:
    """hessian_fd! (src/update_model.jl:94-100): forward differences of the gradient, one
    column per coordinate."""
    x = np.asarray(x, dtype=np.float64)
    g0 = np.asarray(gradfn(x), dtype=np.float64)
    for i in range(len(x)):
        xe = x.copy()
        xe[i] += eps
        hess[:, i] = (np.asarray(gradfn(xe)) - g0) / eps
    return hess


def hessian_fd(gradfn: Callable, x, eps: float = 1e-6) -> np.ndarray:
    """hessian_fd (src/update_model.jl:88-92)."""
    x = np.asarray(x, dtype=np.float64)
    return hessian_fd_(np.empty((len(x), len(x))), gradfn, x, eps)


def bfgs_hessian(Bi, s, t, rho: Optional[float] = None) -> np.ndarray:
    """bfgs_hessian (src/update_model.jl:52-56): C Bi C' + rho s s', C = I - rho s t'."""
    s = np.asarray(s, dtype=np.float64)
    t = np.asarray(t, dtype=np.float64)
    n = len(s)
    rho = 1.0 / np.dot(s, t) if rho is None else rho
    Bi = np.eye(n) * Bi if np.isscalar(Bi) else np.asarray(Bi, dtype=np.float64)
    Cm = np.eye(n) - rho * np.outer(s, t)
    B = Cm @ Bi @ Cm.T + rho * np.outer(s, s)
    return _sym(B)


def bfgs_quad_(theta: np.ndarray, JJ: np.ndarray, B: np.ndarray, gradfn: Callable, eps: float,
               max_iter: int = 100) -> int:
    """bfgs_quad! (src/update_model.jl:66-82): quasi-Newton steps theta -= B J with the BFGS
    inverse-Hessian update, until |J| <= eps; arrays updated in place, returns iterations."""
    it = 0
    while np.linalg.norm(JJ) > eps and it < max_iter:
        s = theta.copy()
        t = JJ.copy()
        theta -= B @ JJ
        JJ[:] = gradfn(theta)
        s = theta - s
        t = JJ - t
        B[:] = bfgs_hessian(B, s, t)
        it += 1
    return it


def bfgs_quad(xx, JJ, HH, gradfn: Callable, eps: float = 1e-5, max_iter: int = 100):
    """bfgs_quad (src/update_model.jl:58-64) -> (x, J, inv(B), iters); HH may be a scalar
    (Julia's I)."""
    x0 = np.array(xx, dtype=np.float64)
    J0 = np.array(JJ, dtype=np.float64)
    n = len(x0)
    H = np.eye(n) * HH if np.isscalar(HH) else np.asarray(HH, dtype=np.float64)
    B = np.linalg.inv(H)
    iters = bfgs_quad_(x0, J0, B, gradfn, eps, max_iter)
    return x0, J0, np.linalg.inv(B), iters


class BFGSQuad:
    """BFGSQuad updater (src/update_model.jl:1-4)."""


class BFGSQuadCache:
    """BFGSQuadCache(hp, J, hess_inv) (src/caches/update_model.jl:4-20)."""

    def __init__(self, md: C.GPRModel):
        D = len(md.params)
        self.hp = np.empty(D)
        self.J = np.empty(D)
        self.hess_inv = np.empty((D, D))


def updater_cache(upd):
    if isinstance(upd, BFGSQuad):
        return BFGSQuadCache
    raise TypeError(f"no cache for updater {upd!r}")


def _log_jac(cost, md: C.GPRModel, tc: C.MllGradCache):
    def jj(log_x):
        G = np.zeros(len(log_x))
        C.log_loss_grad_(cost, None, G, log_x, md, tc)
        return G
    return jj


def update_updater_cache_(uc: BFGSQuadCache, md: C.GPRModel, cost, tc: C.MllGradCache):
    """update_cache!(uc::BFGSQuadCache, md, cost, tc) (src/update_model.jl:19-32): log hp,
    its gradient and the inverse of the finite-difference Hessian (D + 1 device gradients)."""
    uc.hp[:] = np.log(md.params)
    jac = _log_jac(cost, md, tc)
    uc.J[:] = jac(uc.hp)
    uc.hess_inv[:] = np.linalg.inv(_sym(hessian_fd(jac, uc.hp)))


def update_sample_(md: C.GPRModel, dy, upd=None, cost=None, eps_J: float = 1e-3,
                   uc: Optional[BFGSQuadCache] = None, tc: Optional[C.MllGradCache] = None) -> int:
    """update_sample!(md, dy, upd, cost, eps_J) (src/update_model.jl:8-50): y += dy, then
    quasi-Newton steps on log hp from the current optimum until |J| <= eps_J; md.params is
    updated in place; returns the iteration count."""
    upd = upd or BFGSQuad()
    cost = cost or C.MarginalLikelihood()
    tc = tc or C.MllGradCache(md)
    uc = uc or updater_cache(upd)(md)
    md.add_to_y(dy)
    update_updater_cache_(uc, md, cost, tc)
    iters = bfgs_quad_(uc.hp, uc.J, uc.hess_inv, _log_jac(cost, md, tc), eps_J)
    md.params[:] = np.exp(uc.hp)
    return iters
