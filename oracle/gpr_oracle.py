"""CPU oracle: NumPy/SciPy fp64 restatement of GaussianProcessRegression.jl's dense hot path.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this module, and only as the checker / the timed CPU
baseline -- never as the thing measured or shipped.  The product path
(``gaussianprocessregression.jl_amd/gpr_amd``) never imports it and fails loudly when the
HIP library is missing.

Pinning: the reference is Julia (not installed here; its LazyTensors dependency is an
unregistered GitHub package that cannot be fetched offline), so it cannot be run to
produce golden vectors, and its test-suite holds no golden data.  This restatement is
pinned against every known-answer / identity test the reference's own suite contains
(see ``tests/test_oracle.py``): the closed-form diagonal-K MLL (test/test_loss.jl:1-11),
the grad identity with dK=K (test/test_loss.jl:32), cache contents vs fresh cholesky/inv
(test/test_loss.jl:46-48), FD gradients (test/test_loss.jl:13-20,50-55;
test/test_covariance.jl:3-9,84-87), kernel composition identities
(test/test_covariance.jl:34-105), interpolation at the training points
(test/test_models.jl:17-32), diag-vs-full variance (test/test_models.jl:34-48), the split
distance / split kernel / split predict identities (test/test_split_kernel.jl), plus a
50-digit mpmath recomputation at small N bounding the oracle's own rounding error.

Conventions follow the reference exactly (Julia, column-major):
  * ``x`` is d x N (each sample's d features contiguous), ``hp`` a flat vector whose
    layout is the concatenation over kernel parts in ``+`` order
    (src/compose_covar.jl:21-28).
  * SE part hp = [sigma, l_1..l_d]; K = sigma^2 exp(-sum_k (l_k x_k - l_k x'_k)^2)
    (src/covariance.jl:8-12,85-95) -- l multiplies, no 1/2.
  * eps = 1e-8 is added to the diagonal, once per SE part, iff the two inputs are the
    same object (src/covariance.jl:49-58, src/compose_covar.jl:47-61).
All arrays here are numpy arrays in the same (row, col) index convention as Julia; the
memory order is irrelevant to the oracle.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import List, Sequence, Tuple

import numpy as np
import scipy.linalg as sla

SE = "SE"
WN = "WN"
EPS_DEFAULT = 1e-8
LOG2PI = math.log(2.0 * math.pi)


# ---------------------------------------------------------------------------------------
# Kernel specs (src/covariance.jl:15-27,60; src/compose_covar.jl:1-28)
# ---------------------------------------------------------------------------------------
def dim_hp(kind: str, d: int) -> int:
    """src/covariance.jl:27 (SE: d+1), :60 (WN: 1)."""
    if kind == SE:
        return d + 1
    if kind == WN:
        return 1
    raise ValueError(kind)


def split_hp(kinds: Sequence[str], hp: np.ndarray, d: int) -> List[np.ndarray]:
    """Base.split(hp, dims) src/compose_covar.jl:21-24 with dims from :26-28."""
    dims = [dim_hp(k, d) for k in kinds]
    if sum(dims) != len(hp):
        raise ValueError("Parameter size mismatch.")  # src/models.jl:27
    out, c = [], 0
    for n in dims:
        out.append(np.asarray(hp[c:c + n], dtype=np.float64))
        c += n
    return out


# ---------------------------------------------------------------------------------------
# Distances and SE kernel (src/covariance.jl:72-95)
# ---------------------------------------------------------------------------------------
def distance_euclid(xs: np.ndarray, xps: np.ndarray) -> np.ndarray:
    """distance!(Euclidean) src/covariance.jl:72-77: D[a,b] = sum_k (x[k,a]-x'[k,b])^2."""
    D = np.zeros((xs.shape[1], xps.shape[1]))
    for k in range(xs.shape[0]):  # sum over dim 1, feature by feature
        D += (xs[k][:, None] - xps[k][None, :]) ** 2
    return D


def se_kernel(hp: np.ndarray, x: np.ndarray, xp: np.ndarray, same: bool,
              eps: float = EPS_DEFAULT, dist: str = "euclid") -> np.ndarray:
    """kernel!(kern, ::SquaredExp, hp, x, xp) src/covariance.jl:49-58 -> kernel_impl! :85-95.

    Scale-then-difference: xs = x .* l, D = distance(xs, xps), K = sigma^2 * exp(-1.0*D);
    +eps on the diagonal iff x === xp.  ``dist`` selects the split metrics of
    src/split_kernel.jl:108-123.
    """
    sigma, ls = hp[0], hp[1:]
    xs = x * ls[:, None]
    xps = xp * ls[:, None]
    if dist == "euclid":
        D = distance_euclid(xs, xps)
    elif dist == "splitA":
        D = split_distance_a(xs, xps)
    elif dist == "splitC":
        D = split_distance_c(xs, xps)
    else:
        raise ValueError(dist)
    K = (sigma ** 2) * np.exp(-1.0 * D)
    if same:
        K[np.diag_indices(K.shape[0])] += eps
    return K


def kernel(kinds: Sequence[str], hp: np.ndarray, x: np.ndarray, xp: np.ndarray | None = None,
           eps: float = EPS_DEFAULT) -> np.ndarray:
    """Composed / single kernel matrix.

    kernel!(kern, K::ComposedKernel, hp, x)       src/compose_covar.jl:73-77 (xp None:
                                                  same object, + noise)
    kernel!(kern, K::ComposedKernel, hp, x, xp)   src/compose_covar.jl:47-61 (no noise; eps
                                                  per SE part iff xp is x, i.e. x === xp)
    Summation order: first SE part, then `kern .+= kernel(part_t)` for t = 2.. (each SE
    part carries its own +eps when same), then add_noise! (:63-71) adds sigma_n^2 -- only
    in the 4-arg form.  So predict(md, md.x) sees eps (not noise) on Kxp's diagonal
    (src/predict.jl:37,43), which the reference's interpolation test relies on
    (test/test_models.jl:17-24).
    """
    d = x.shape[0]
    noise = xp is None
    same = noise or xp is x
    xq = x if same else xp
    hps = split_hp(kinds, hp, d)
    se_idx = [i for i, k in enumerate(kinds) if k == SE]   # rm_noise :30-33
    if not se_idx:
        raise ValueError("kernel needs at least one SquaredExp part")
    K = se_kernel(hps[se_idx[0]], x, xq, same, eps)
    for i in se_idx[1:]:
        K = K + se_kernel(hps[i], x, xq, same, eps)
    if noise and WN in kinds:
        nidx = kinds.index(WN)  # findfirst: only the first WhiteNoise counts (:64-68)
        K[np.diag_indices(K.shape[0])] += hps[nidx][0] ** 2
    return K


def kernel_grad(kinds: Sequence[str], i: int, hp: np.ndarray, x: np.ndarray,
                eps: float = EPS_DEFAULT):
    """grad(cov, i, hp, x): src/deriv_covar.jl:2-32 + composed find_idx src/compose_covar.jl:109-123.

    ``i`` is 1-based like Julia.  SE: i==1 -> (2/|sigma|) K (K incl. eps on diag);
    i>1 -> -2 l_{i-1} K (x_{i-1,a}-x_{i-1,b})^2 with RAW x.  WN: 2 sigma_n I, returned as
    the tuple ("I", lambda).
    """
    d = x.shape[0]
    hps = split_hp(kinds, hp, d)
    dims = np.cumsum([dim_hp(k, d) for k in kinds])
    kidx = int(np.searchsorted(dims, i))  # first cdims >= i
    hpidx = i if kidx == 0 else i - dims[kidx - 1]
    part = hps[kidx]
    if kinds[kidx] == WN:
        return ("I", 2.0 * part[0])
    Kp = se_kernel(part, x, x, True, eps)
    if hpidx == 1:
        return (2.0 / abs(part[0])) * Kp
    k = hpidx - 2
    diff2 = (x[k][:, None] - x[k][None, :]) ** 2
    return -2.0 * part[hpidx - 1] * Kp * diff2


# ---------------------------------------------------------------------------------------
# Cholesky-based MLL (src/cost.jl:74-126, src/loss_grad.jl:32-52)
# ---------------------------------------------------------------------------------------
def chol_upper(K: np.ndarray) -> np.ndarray:
    """cholesky!(Hermitian(K)) = LAPACK dpotrf('U'): K = U^T U (src/cost.jl:77)."""
    return sla.cholesky(K, lower=False, check_finite=False)


def potrf_inplace_upper(K: np.ndarray) -> np.ndarray:
    """What the in-place dpotrf('U') leaves in the buffer: U in the upper triangle, the
    original K in the strict lower triangle (test/test_loss.jl:46)."""
    U = chol_upper(K)
    out = np.tril(K, -1) + np.triu(U)
    return out


def cho_solve_upper(U: np.ndarray, y: np.ndarray) -> np.ndarray:
    """ldiv!(alpha, kchol, y) = dpotrs (src/cost.jl:79)."""
    z = sla.solve_triangular(U, y, trans="T", lower=False, check_finite=False)
    return sla.solve_triangular(U, z, trans="N", lower=False, check_finite=False)


def kinv_from_upper(U: np.ndarray) -> np.ndarray:
    """K^{-1} = ldiv!(kchol, I) (src/cost.jl:90-92): dpotrs with N right-hand sides."""
    return cho_solve_upper(U, np.eye(U.shape[0]))


def get_sample(y: np.ndarray, train_axis: int = 1) -> np.ndarray:
    """src/models.jl:39-45 (train_axis is 1-based)."""
    return y if y.ndim == 1 else y[:, train_axis - 1]


def mll_value(U: np.ndarray, y: np.ndarray, alpha: np.ndarray) -> float:
    """loss(MLL, kchol, y, K^-1 y) src/loss_grad.jl:39-41: 0.5(y.alpha + logdet + N log 2pi).

    logdet(Cholesky) = 2 sum log U_ii.
    """
    n = U.shape[0]
    return 0.5 * (float(np.dot(y, alpha)) + 2.0 * float(np.sum(np.log(np.diag(U)))) + n * LOG2PI)


def mll(kinds, hp, x, y, eps=EPS_DEFAULT, train_axis=1):
    """loss(MLL, hp, md) src/cost.jl:19-22,40-43,74-81,113-117."""
    K = kernel(kinds, hp, x, None, eps)
    U = chol_upper(K)
    ys = get_sample(y, train_axis)
    alpha = cho_solve_upper(U, ys)
    return mll_value(U, ys, alpha)


def mll_grad_parts(dK, alpha: np.ndarray, Kinv: np.ndarray) -> Tuple[float, float]:
    """The two terms of grad(MLL, kchol, dK, alpha, K^-1, tt) src/loss_grad.jl:43-52:
    (alpha' dK alpha, <K^-1, dK>_F); the component is -0.5 (first - second)."""
    if isinstance(dK, tuple):  # UniformScaling lam*I: src/loss_grad.jl:50-52
        return dK[1] * float(np.sum(alpha ** 2)), dK[1] * float(np.sum(np.diag(Kinv)))
    tt = dK @ alpha
    return float(np.dot(tt, alpha)), float(np.sum(Kinv * dK))


def mll_grad_term(dK, alpha: np.ndarray, Kinv: np.ndarray) -> float:
    """grad(MLL, kchol, dK, alpha, K^-1, tt) src/loss_grad.jl:43-52."""
    if isinstance(dK, tuple):  # UniformScaling
        return -0.5 * dK[1] * float(np.sum(alpha ** 2 - np.diag(Kinv)))
    tt = dK @ alpha
    return -0.5 * (float(np.dot(tt, alpha)) - float(np.sum(Kinv * dK)))


def mll_grad(kinds, hp, x, y, eps=EPS_DEFAULT, train_axis=1, log_scale=False):
    """grad!(dL, MLL, hp, md, tc) src/cost.jl:45-48,83-111,119-126; log_loss_grad! :60-70.

    Returns the D-vector; with log_scale=True the chain rule G .*= hp is applied.
    """
    hp = np.asarray(hp, dtype=np.float64)
    K = kernel(kinds, hp, x, None, eps)
    U = chol_upper(K)
    ys = get_sample(y, train_axis)
    alpha = cho_solve_upper(U, ys)
    Kinv = kinv_from_upper(U)
    g = np.empty(len(hp))
    for i in range(1, len(hp) + 1):
        g[i - 1] = mll_grad_term(kernel_grad(kinds, i, hp, x, eps), alpha, Kinv)
    if log_scale:
        g = g * hp
    return g


def islog(kinds) -> bool:
    """islog(MLL, md) src/cost.jl:4-8: LogScale iff a SquaredExp part is present."""
    return SE in kinds


# ---------------------------------------------------------------------------------------
# Posterior (src/predict.jl)
# ---------------------------------------------------------------------------------------
def diag_prior(kinds, hp, d) -> float:
    """Diagonal-variance prior: SE alone sigma^2 (src/predict.jl:67); composed: sum over
    ALL parts of hp_part[1]^2 incl. the noise (src/predict.jl:56-58).  No eps."""
    hps = split_hp(kinds, hp, d)
    if len(kinds) == 1:
        return float(hps[0][0] ** 2)
    return float(sum(h[0] ** 2 for h in hps))


def predict(kinds, hp, x, y, xp, diagonal_var=False, eps=EPS_DEFAULT):
    """predict(md, xp; diagonal_var) src/predict.jl:14-25 with update_cache! :29-34,
    predict! :42-71, predict_mean_impl! :73-76, predict_covar_impl! :83-95.

    Returns (mu, Sigma) with Sigma an np x np matrix (full) or the np diagonal vector.
    """
    K = kernel(kinds, hp, x, None, eps)
    U = chol_upper(K)
    wt = cho_solve_upper(U, y)                    # ldiv!(pc.wt, kchol, md.y)
    return predict_from_factor(kinds, hp, x, U, wt, xp, diagonal_var, eps)


def predict_from_factor(kinds, hp, x, U, wt, xp, diagonal_var=False, eps=EPS_DEFAULT):
    """predict!(mu, Sigma, md, xp, pc) src/predict.jl:36-71 from an updated cache: U is the
    upper factor (only its upper triangle is read, like Cholesky(UpperTriangular(pc.Kxx))),
    wt = K^{-1} md.y."""
    d = x.shape[0]
    Kxp = kernel(kinds, hp, xp, x, eps)           # np x N; eps per SE part iff xp is x
    mu = Kxp @ wt
    V = sla.solve_triangular(U, Kxp.T, trans="T", lower=False, check_finite=False).T  # rdiv!(Kxp,U)
    if diagonal_var:
        var = diag_prior(kinds, hp, d) - np.sum(V * V, axis=1)
        return mu, var
    S = kernel(kinds, hp, xp, None, eps)          # kernel!(Sigma, covar, hp, xp): eps (+noise)
    S = S - V @ V.T
    return mu, S


# ---------------------------------------------------------------------------------------
# Split kernel / split prediction (src/split_kernel.jl, src/split_predict.jl)
# ---------------------------------------------------------------------------------------
def cmap_points(xe: np.ndarray, xq: np.ndarray) -> np.ndarray:
    """Cmap(+, xe, xq)[:, :] src/split_kernel.jl:1-17: column index e + (q-1)*ne (1-based),
    i.e. e fastest (test/test_split_kernel.jl:20-21)."""
    d, ne = xe.shape
    nq = xq.shape[1]
    return (xe[:, :, None] + xq[:, None, :]).reshape(d, ne * nq, order="F")


def split_distance_a(xe: np.ndarray, xq: np.ndarray) -> np.ndarray:
    """distance!(SplitDistanceA) src/split_kernel.jl:111-116: sum_k xq^2 + 2 xe xq."""
    D = np.zeros((xe.shape[1], xq.shape[1]))
    for k in range(xe.shape[0]):
        D += xq[k][None, :] ** 2 + 2.0 * xe[k][:, None] * xq[k][None, :]
    return D


def split_distance_c(xs: np.ndarray, xq: np.ndarray) -> np.ndarray:
    """distance!(SplitDistanceC) src/split_kernel.jl:118-123: sum_k -2 xs xq."""
    D = np.zeros((xs.shape[1], xq.shape[1]))
    for k in range(xs.shape[0]):
        D += -2.0 * xs[k][:, None] * xq[k][None, :]
    return D


def split_factors(kinds, hp, x, xe, xq, eps=EPS_DEFAULT):
    """kernel!(SplitKernel, ...) src/split_kernel.jl:137-159: per SE part k,
    A[:,:,k] (ne x nq, sigma=1, SplitDistanceA), B[:,:,k] (ne x ns, sigma=1, Euclidean),
    C[:,:,k] (ns x nq, sigma, SplitDistanceC).  None of them is a same-object call, so no
    eps is added."""
    d = x.shape[0]
    hps = split_hp(kinds, hp, d)
    parts = [hps[i] for i, k in enumerate(kinds) if k == SE]
    A, B, C = [], [], []
    for h in parts:
        h1 = h.copy()
        h1[0] = 1.0
        A.append(se_kernel(h1, xe, xq, False, eps, dist="splitA"))
        B.append(se_kernel(h1, xe, x, False, eps, dist="euclid"))
        C.append(se_kernel(h, x, xq, False, eps, dist="splitC"))
    return np.stack(A, 2), np.stack(B, 2), np.stack(C, 2)


def split_predict(kinds, hp, x, y, xe, xq, var_range: Tuple[int, int] | None = (1, 3),
                  eps=EPS_DEFAULT):
    """predict(md, Cmap(+,xe,xq); diagonal_var=true) src/predict.jl:14-25,51-71 with
    predict_split_mean_impl! src/split_predict.jl:10-19 and the split
    predict_covar_impl! :39-53 (var_range default 1:3, src/caches/split_kernel.jl:10).

    Returns mu as an ne x nq matrix (column-major linear index e + (q-1) ne) and the
    variance diagonal of length ne*nq whose entry (e-1)*nq + q is updated only for
    e in var_range (1-based inclusive); every other entry keeps the prior.
    """
    K = kernel(kinds, hp, x, None, eps)
    U = chol_upper(K)
    wt = cho_solve_upper(U, y)
    return split_predict_from_factor(kinds, hp, x, U, wt, xe, xq, var_range, eps)


def split_predict_from_factor(kinds, hp, x, U, wt, xe, xq, var_range=(1, 3), eps=EPS_DEFAULT,
                              mean_rows=None):
    """The split predict! (src/split_predict.jl:5-53) from an updated cache (U upper factor,
    wt = K^{-1} y).  ``mean_rows`` (0-based e indices) restricts the returned mean to those
    grid rows (a row of mu needs only its own row of A and B)."""
    d = x.shape[0]
    ne, nq = xe.shape[1], xq.shape[1]
    A, B, C = split_factors(kinds, hp, x, xe, xq, eps)
    rows = np.arange(ne) if mean_rows is None else np.asarray(mean_rows)
    mu = np.zeros((len(rows), nq))
    for k in range(A.shape[2]):
        Cw = wt[:, None] * C[:, :, k]
        BCw = B[rows, :, k] @ Cw
        mu += BCw * A[rows, :, k]
    var = np.full(ne * nq, diag_prior(kinds, hp, d))
    if var_range is not None:
        lo, hi = var_range
        lo, hi = max(lo, 1), min(hi, ne)
        for e in range(lo, hi + 1):
            Kxq = np.zeros((nq, x.shape[1]))
            for k in range(A.shape[2]):
                Kxq += A[e - 1, :, None, k] * B[e - 1, None, :, k] * C[:, :, k].T
            V = sla.solve_triangular(U, Kxq.T, trans="T", lower=False, check_finite=False).T
            var[(e - 1) * nq:e * nq] -= np.sum(V * V, axis=1)
    return mu, var


# ---------------------------------------------------------------------------------------
# Synthetic data
# ---------------------------------------------------------------------------------------
def synthetic(d: int, n: int, npred: int = 0, seed_train: int = 0, seed_test: int = 1):
    """x = U[0,1)^(d x n), y = sin(sum_k x_k)^2 (test/test_models.jl:8)."""
    x = np.random.default_rng(seed_train).random((d, n))
    y = np.sin(np.sum(x, axis=0)) ** 2
    xp = np.random.default_rng(seed_test).random((d, npred)) if npred else None
    return x, y, xp


def default_hp(kinds, d, length=None, sigma=1.0, noise=0.1):
    """sigma=1, l_k = 3 sqrt(8/d), sigma_n = 0.1."""
    l = 3.0 * math.sqrt(8.0 / d) if length is None else length
    hp = []
    for k in kinds:
        if k == SE:
            hp += [sigma] + [l] * d
        else:
            hp += [noise]
    return np.array(hp, dtype=np.float64)


# ---------------------------------------------------------------------------------------
# Bayesian quadrature of the posterior (src/integrate.jl), sample_noise = nothing
# ---------------------------------------------------------------------------------------
RT_PI_BY_2 = np.sqrt(np.pi) * 0.5


def erf2(x, y):
    """SpecialFunctions' two-argument erf(x, y) = erf(y) - erf(x) (src/integrate.jl:4,26),
    through erfc on the same side beyond 1/sqrt(2) (no cancellation)."""
    from scipy.special import erf, erfc
    x, y = np.asarray(x, dtype=np.float64), np.asarray(y, dtype=np.float64)
    t = np.sqrt(0.5)
    return np.where((x > t) & (y > t), erfc(x) - erfc(y),
                    np.where((x < -t) & (y < -t), erfc(-y) - erfc(-x), erf(y) - erf(x)))


def gauss_integ(xs, w, a, b):
    """gauss_integ(xs, w, a, b) src/integrate.jl:4-5: int_a^b exp(-w^2 (x - xs)^2) dx."""
    return (1.0 / w) * RT_PI_BY_2 * erf2(w * (a - xs), w * (b - xs))


def erf_integ(w, a, b):
    """erf_integ src/integrate.jl:6-7: int_a^b int_a^b exp(-w^2 (x - y)^2) dx dy."""
    from scipy.special import erf
    return 1.0 / w ** 2 * (np.exp(-(w * (b - a)) ** 2) - 1.0) + \
        2.0 * (RT_PI_BY_2 / w) * (b - a) * erf(w * (b - a))


def antideriv_se(xs, hp, a, b):
    """antideriv!(integ, SquaredExp(), xs, hp, a, b) src/integrate.jl:16-31 (hp[0] = sigma,
    hp[1..d] = l, the first d + 1 entries of md.params)."""
    d = xs.shape[0]
    ls = np.asarray(hp[1:d + 1], dtype=np.float64)
    prefac = hp[0] ** 2 * (RT_PI_BY_2 ** d) * np.prod(1.0 / ls)
    integ = np.ones(xs.shape[1])
    for i in range(d):
        integ = integ * erf2(ls[i] * (a[i] - xs[i]), ls[i] * (b[i] - xs[i]))
    return integ * prefac


def antideriv2_se(hp, a, b):
    """antideriv2 src/integrate.jl:33-41."""
    d = len(a)
    integ2 = 1.0
    for i in range(d):
        integ2 *= erf_integ(hp[1 + i], a[i], b[i])
    return integ2 * hp[0] ** 2


def integrate(kinds, hp, x, y, a, b, eps=EPS_DEFAULT):
    """integrate(md, hp, a, b; sample_noise=nothing) src/integrate.jl:48-167 ->
    (Iout[ne], var): wt = K^{-1} y, Iout = wt' k1, var = k2 - ||U^{-T} k1||^2."""
    K = kernel(kinds, hp, x, None, eps)
    U = chol_upper(K)
    Y = y if y.ndim == 2 else y[:, None]
    wt = cho_solve_upper(U, Y)
    k1 = antideriv_se(x, hp, a, b)
    k2 = antideriv2_se(hp, a, b)
    import scipy.linalg as sla
    tt = sla.solve_triangular(U, k1, trans="T", lower=False)
    return wt.T @ k1, k2 - float(tt @ tt)


# ---------------------------------------------------------------------------------------
# Cross-validation (src/crossval.jl) and its losses (src/loss_grad.jl:12-30)
# ---------------------------------------------------------------------------------------
def kfoldcv(n: int, k: int, nb: int | None = None, perm=None):
    """kfoldcv(n, k, nb = div(n, k)) src/crossval.jl:1-11 with 0-based indices: perm plays
    shuffle(1:n); fold i tests perm[i k : (i+1) k] and trains on perm at every OTHER
    position, in order."""
    nb = n // k if nb is None else nb
    perm = np.arange(n) if perm is None else np.asarray(perm)
    trn, tst = [], []
    for i in range(nb):
        pos = np.arange(i * k, (i + 1) * k)
        tst.append(perm[pos])
        keep = np.ones(n, dtype=bool)
        keep[pos] = False
        trn.append(perm[keep])
    return trn, tst


def cv_loss(cost: str, y, yp, S) -> float:
    """loss(::MSE | ::ChiSq | ::Mahalanobis, y, yp, Sigma_p) src/loss_grad.jl:12-30."""
    r = np.asarray(y) - np.asarray(yp)
    if cost == "MSE":
        return float(np.sum(r * r) / r.size)
    if cost == "ChiSq":
        return float(np.sum(r * r / np.diag(S)))
    if cost == "Mahalanobis":  # cholesky(Sigma_p) reads the upper triangle (uplo 'U')
        U = sla.cholesky(S, lower=False, check_finite=False)
        z = sla.solve_triangular(U, r, trans="T", lower=False, check_finite=False)
        return float(z @ z)
    raise ValueError(cost)


def cv_step(kinds, hp, cost, xtr, ytr, xtst, ytst, eps=EPS_DEFAULT) -> float:
    """cv_step / cv_step! src/crossval.jl:37-51: fit on (xtr, ytr), full-covariance predict
    at xtst, loss(cost, ytst, yp, Sigma_p)."""
    yp, S = predict(kinds, hp, xtr, ytr, xtst, diagonal_var=False, eps=eps)
    return cv_loss(cost, ytst, yp, S)


def cv_batch(kinds, hp, cost, x, y, cvset, eps=EPS_DEFAULT) -> np.ndarray:
    """cv_batch(md, cost, x, y, (trn, tst)) src/crossval.jl:13-35."""
    trn, tst = cvset
    return np.array([cv_step(kinds, hp, cost, x[:, a], y[a], x[:, b], y[b], eps)
                     for a, b in zip(trn, tst)])


def inverse_diagonal_update(lam, P, eps, y):
    """inverse_diagonal_update!(ABy, lam, P, eps, y, tmp) src/integrate.jl:81-95:
    P (lam + eps)^{-1} P' y; a vector eps applies eps[j] to column j of y."""
    eps = np.asarray(eps, dtype=np.float64)
    Pty = P.T @ y
    if eps.ndim == 0:
        return P @ (Pty / (lam + eps) if y.ndim == 1 else Pty / (lam[:, None] + eps))
    return P @ (Pty / (lam[:, None] + eps[None, :]))


def inverse_diagonal_update2(lam, P, eps, y):
    """inverse_diagonal_update2!(...) src/integrate.jl:97-111: y' (P (lam + eps)^{-1} P') y,
    one value per entry of a vector eps."""
    t = (P.T @ y) ** 2
    eps = np.asarray(eps, dtype=np.float64)
    if eps.ndim == 0:
        return float(t @ (1.0 / (lam + eps)))
    return (1.0 / (lam[None, :] + eps[:, None])) @ t


def integrate_noise(kinds, hp, x, y, a, b, noise, eps=EPS_DEFAULT):
    """integrate(md, hp, a, b; sample_noise = noise::Vector) src/integrate.jl:71-79,149-162:
    K = P Lambda P' (syevr; here numpy's eigh), wt = P (Lambda + noise_j)^{-1} P' y_j,
    Iout = wt' k1, var_j = k2 - k1' P (Lambda + noise_j)^{-1} P' k1."""
    K = kernel(kinds, hp, x, None, eps)
    lam, P = np.linalg.eigh(K)
    y2 = y[:, None] if y.ndim == 1 else y
    noise = np.asarray(noise, dtype=np.float64)
    wt = inverse_diagonal_update(lam, P, noise, y2)
    k1 = antideriv_se(x, hp, a, b)
    k2 = antideriv2_se(hp, a, b)
    return wt.T @ k1, k2 - inverse_diagonal_update2(lam, P, noise, k1)
