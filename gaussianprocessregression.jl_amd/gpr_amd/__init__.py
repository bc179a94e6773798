"""gpr_amd -- MI355X-native drop-in for the dense exact-GP hot path of
GaussianProcessRegression.jl.

Names and argument meaning follow the reference's exported API
(src/GaussianProcessRegression.jl:16-84); Julia's mutating ``f!`` functions are spelled
``f_`` here.  Every numeric operation runs in libgpr_hip.so (hand-written gfx950 HIP); there
is no CPU fallback.
"""
from ._lib import GPR_PREDICT_DIAG, GPR_PREDICT_FULL, GPR_PREDICT_MEAN, GprError, PosDefException
from .core import (
    Cmap,
    ComposedKernel,
    Context,
    GPRModel,
    GPRPredictCache,
    GPRSplitPredictCache,
    LogScale,
    MarginalLikelihood,
    MllGradCache,
    MllLossCache,
    NoLogScale,
    SquaredExp,
    UniformScaling,
    WhiteNoise,
    default_context,
    dim_hp,
    get_sample,
    grad,
    grad_,
    islog,
    kernel,
    log_loss_grad_,
    loss,
    loss_grad_,
    predict,
    predict_,
    predict_mean,
    predict_mean_,
    split_factors,
    update_cache_,
    update_predict_cache_,
    grad_cache,
    kernels,
    loss_cache,
    loss_grad_cache,
    predict_cache,
    rm_noise,
    similar,
)

from .crossval import ChiSq, Mahalanobis, MSE, cv_batch, cv_step, cv_step_, kfoldcv
from .integrate import antideriv, antideriv2, erf_integ, gauss_integ, integrate
from .train import (
    BFGS,
    LBFGS,
    BFGSQuad,
    BFGSQuadCache,
    ConjugateGradient,
    NelderMead,
    NewtonTrustRegion,
    Options,
    OptimResult,
    bfgs_hessian,
    bfgs_quad,
    bfgs_quad_,
    g_converged,
    hessian_fd,
    hessian_fd_,
    init_params,
    minimizer,
    train,
    update_sample_,
)

__all__ = [n for n in dir() if not n.startswith("_")]
