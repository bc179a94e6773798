"""Multi-GPU split-kernel block prediction: one process per GPU.

The reference runs ``predict(md, Cmap(+, xe, xq); diagonal_var=true)``
(src/predict.jl:14-25 -> src/split_predict.jl:5-53) on one CPU.  Here the e-rows of the
test grid x_{e,q} = xe_e + xq_q are independent once the training factor U and the weights
wt = K^{-1} y exist, so:

  1. rank 0 fits: K, POTRF (U), wt                        (src/predict.jl:29-34)
     fit="broadcast": U's upper triangle (packed by 128-column blocks, ~4N^2 bytes) and
     wt are broadcast from rank 0 over RCCL/xGMI;
     fit="replicate": every rank factorises K itself (no N^2 exchange; the better choice
     when the broadcast of 8N^2 bytes costs more than one K + POTRF on a GPU).
  2. rank r takes an even share of the var_range rows AND an even share of the other rows
     (shard_pieces: at most three contiguous pieces of grid rows) and computes their mean
     rows mu[e, :] and, for var_range rows, the variance (src/split_predict.jl:10-19,
     :39-53; var_range default 1:3, src/caches/split_kernel.jl:10).  Rows outside
     var_range keep the prior.  A variance row costs an N^2 triangular solve per test point
     (N = 32768, nq = 1024: ~1.1e12 flop) against ~1e8 for a mean row, so a plain split of
     the grid rows would leave every variance row of the default var_range on rank 0.
  3. every rank writes its rows straight into shard-sized buffers (mu: rows x nq, var:
     rows nq, padded to the largest share -- never a grid-sized buffer per rank); the shards
     are all-gathered and reassembled in the reference layouts: mu ne x nq column-major
     (linear e + q ne), var.diag index e nq + q.

The collective sequence (broadcast, then all_gather) is the only data exchange; the
per-rank compute is a pluggable backend so the distributed logic is tested on CPU with
gloo (tests/test_distributed.py) and runs on libgpr_hip.so with RCCL on the GPUs
(HipSplitBackend, the default).
"""
from __future__ import annotations

import ctypes
from typing import Optional, Tuple

import numpy as np
import torch
import torch.distributed as dist

from . import core
from ._lib import GprError, PosDefException, lib

__all__ = ["shard_rows", "shard_pieces", "pack_upper", "unpack_upper", "HipSplitBackend",
           "split_predict_distributed", "MultiGPU", "split_predict_mgpu"]


def shard_rows(n: int, world: int, rank: int) -> Tuple[int, int]:
    """Balanced contiguous partition of n rows: the first n % world ranks get one more."""
    q, r = divmod(n, world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def shard_pieces(n: int, world: int, rank: int, v_lo: int = 0, v_hi: int = 0):
    """Grid rows of `rank` as sorted, disjoint contiguous [lo, hi) pieces: an even share
    (shard_rows) of the variance rows [v_lo, v_hi), plus an even share of the other rows
    ([0, v_lo) then [v_hi, n), counted as one sequence).  Over all ranks the pieces
    partition [0, n)."""
    v_lo, v_hi = max(0, min(v_lo, n)), max(0, min(v_hi, n))
    nv = max(v_hi - v_lo, 0)
    pieces = []
    if nv:
        a, b = shard_rows(nv, world, rank)
        if b > a:
            pieces.append((v_lo + a, v_lo + b))
    a, b = shard_rows(n - nv, world, rank)
    # mean-only index i < v_lo is row i; i >= v_lo is row i + nv
    if a < min(b, v_lo):
        pieces.append((a, min(b, v_lo)))
    lo2, hi2 = max(a, v_lo), b
    if hi2 > lo2:
        pieces.append((lo2 + nv, hi2 + nv))
    pieces.sort()
    merged = []
    for lo, hi in pieces:  # adjacent pieces become one call
        if merged and merged[-1][1] == lo:
            merged[-1] = (merged[-1][0], hi)
        else:
            merged.append((lo, hi))
    return merged


def var_rows(var_range: Optional[Tuple[int, int]], ne: int) -> Tuple[int, int]:
    """Julia 1-based inclusive var_range -> 0-based half-open [lo, hi) clamped to ne
    (None = no variance rows)."""
    if var_range is None:
        return 0, 0
    a, b = var_range
    lo, hi = max(a, 1) - 1, min(b, ne)
    return (lo, hi) if hi > lo else (0, 0)


class HipSplitBackend:
    """Per-rank compute on libgpr_hip.so (the product path).

    fit():          gpr_fit -> (U, wt) device tensors (U column-major N x N).
    empty_fit():    receive buffers for the broadcast.
    publish():      order torch's current stream after the context stream, so a collective
                    (which waits only on the current stream) sends the finished U / wt.
    receive():      order the context stream after the current stream, so the split
                    kernels read U / wt only once the collective's copies have landed.
    received():     (receiving ranks) drop the context's cached factor inverses.
    predict_shard(): all of the rank's row pieces in one gpr_split_predict_shard call, into
                    shard-sized device buffers (mu: nq x emax tensor = emax x nq column-major,
                    var: emax nq; the pieces' rows concatenated in order).

    gpr_fit returns once the factorisation's info is known, with the wt solve still queued
    on the context stream; RCCL runs on its own stream that waits on torch's current stream
    only -- hence publish()/receive() around every collective on device buffers.
    """

    def __init__(self, md: core.GPRModel, eps: float = core.EPS_DEFAULT):
        if md.y.ndim != 1:
            raise ValueError("split prediction needs a 1-D y (Diagonal(wt), src/split_predict.jl:13)")
        self.md, self.eps, self.ctx = md, eps, md.ctx
        self.device = self.ctx.device

    def empty_fit(self):
        n = self.md.n
        return self.ctx.empty(n, n), self.ctx.empty(n)

    def fit(self):
        pc = core.GPRSplitPredictCache(self.md, 0, 0)
        core._update_predict_cache(core.pc_adapter(pc), self.md, self.eps)
        return pc.Kxx, pc.wt

    def publish(self):
        torch.cuda.current_stream(self.device).wait_stream(self.ctx.stream)

    def receive(self):
        self.ctx.stream.wait_stream(torch.cuda.current_stream(self.device))

    def received(self):
        """On the receiving ranks: the broadcast wrote U behind the context's back, so a
        cached factor keyed on the same device pointer (a re-used allocation) must not serve
        this one (the block inverses are rebuilt from the received U)."""
        self.ctx.check(lib.gpr_forget_factor(self.ctx.h), "gpr_forget_factor")

    def predict_shard(self, cm: core.Cmap, U, wt, pieces, v_lo: int, v_hi: int, emax: int):
        """All of this rank's row pieces in ONE gpr_split_predict_shard call (the ns x nq C
        factor built once) into buffers of emax rows (emax >= the shard's rows: the
        all_gather's common size)."""
        md, ctx = self.md, self.ctx
        _, ne, nq = cm.shape
        mu = ctx.zeros(nq, emax)  # emax x nq column-major (leading dimension emax)
        var = ctx.zeros(emax * nq)
        kinds, nk = core._kinds_arr(md.covar)
        _, hpp = core._hp_arr(md.params)
        dxe, dxq = ctx.colmajor(cm.xe), ctx.colmajor(cm.xq)
        flat = [v for p in pieces for v in p]
        arr = (ctypes.c_int * max(len(flat), 1))(*flat)
        ctx.check(lib.gpr_split_predict_shard(ctx.h, kinds, nk, hpp, md.d, core._ptr(md.dx()), md.n,
                                              core._ptr(U), md.n, core._ptr(wt), core._ptr(dxe), ne,
                                              core._ptr(dxq), nq, arr, len(pieces), v_lo, v_hi,
                                              self.eps, core._ptr(mu), emax, core._ptr(var)),
                  "gpr_split_predict_shard")
        ctx.sync()
        return mu, var


_PACK_NB = 128


def _packed_len(n: int, nb: int = _PACK_NB) -> int:
    return sum((j1 - j0) * j1 for j0, j1 in ((j, min(j + nb, n)) for j in range(0, n, nb)))


def pack_upper(U: torch.Tensor, nb: int = _PACK_NB) -> torch.Tensor:
    """The upper triangle of a column-major n x n factor (tensor row c = column c) by
    column blocks of nb: block [j0, j1) keeps rows [0, j1) of its columns (the diagonal
    block whole).  ~n^2/2 elements instead of n^2: what the broadcast has to move."""
    n = U.shape[0]
    return torch.cat([U[j0:min(j0 + nb, n), :min(j0 + nb, n)].reshape(-1)
                      for j0 in range(0, n, nb)]) if n else U.reshape(-1)[:0].clone()


def unpack_upper(P: torch.Tensor, U: torch.Tensor, nb: int = _PACK_NB) -> None:
    """Inverse of pack_upper into U (entries below the diagonal blocks are left as they
    are: no solve reads them)."""
    n, off = U.shape[0], 0
    for j0 in range(0, n, nb):
        j1 = min(j0 + nb, n)
        U[j0:j1, :j1] = P[off:off + (j1 - j0) * j1].view(j1 - j0, j1)
        off += (j1 - j0) * j1


def _src(group) -> int:
    return dist.get_global_rank(group, 0) if group is not None else 0


def _hook(backend, name: str):
    f = getattr(backend, name, None)
    if f is not None:
        f()


def split_predict_distributed(md: core.GPRModel, cm: core.Cmap,
                              var_range: Optional[Tuple[int, int]] = (1, 3),
                              backend=None, fit: str = "broadcast", group=None,
                              eps: float = core.EPS_DEFAULT):
    """Sharded predict(md, Cmap(+, xe, xq); diagonal_var=true) over the ranks of `group`.

    Every rank must call it with the same model and grid (SPMD).  Returns, on every rank,
    (mu, var): mu as an ne x nq numpy array (Julia indexing; linear e + q ne) and var as
    the length ne nq diagonal (index e nq + q), identical to the single-process result.
    """
    if fit not in ("broadcast", "replicate"):
        raise ValueError("fit must be 'broadcast' or 'replicate'")
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    backend = backend or HipSplitBackend(md, eps)
    _, ne, nq = cm.shape

    # 1. factor + weights: rank 0 (broadcast) or every rank (replicate).  A failed fit is
    #    turned into a status every rank sees before any data collective, so all ranks raise
    #    the same exception instead of the others blocking in a broadcast / all_gather.
    dev = getattr(backend, "device", None) or torch.device("cpu")
    U = wt = None
    err: Optional[BaseException] = None
    if fit == "replicate" or rank == 0:
        try:
            U, wt = backend.fit()
            code = 0
        except PosDefException as e:
            err, code = e, int(e.info)
        except Exception as e:  # noqa: BLE001 -- re-raised below, after the status exchange
            err, code = e, -1
    else:
        code = 0
    status = torch.tensor([code], dtype=torch.int64, device=dev)
    if fit == "broadcast":
        dist.broadcast(status, _src(group), group=group)
    else:  # any failing rank: report the first failure class (PosDef info > 0 wins)
        neg = torch.tensor([1 if code < 0 else 0], dtype=torch.int64, device=dev)
        dist.all_reduce(status, op=dist.ReduceOp.MAX, group=group)
        dist.all_reduce(neg, op=dist.ReduceOp.MAX, group=group)
        if int(status.item()) == 0 and int(neg.item()) > 0:
            status.fill_(-1)
    code_all = int(status.item())
    if code_all != 0:
        if err is not None:
            raise err
        if code_all > 0:
            raise PosDefException(code_all)
        raise GprError("split_predict_distributed: the fit failed on another rank")
    if fit == "broadcast":
        if rank != 0:
            U, wt = backend.empty_fit()
        _hook(backend, "publish")
        if world > 1:
            # the upper triangle only (by 128-column blocks): half the bytes over xGMI
            n = U.shape[0]
            P = pack_upper(U) if rank == 0 else torch.empty(_packed_len(n), dtype=U.dtype,
                                                             device=U.device)
            dist.broadcast(P, _src(group), group=group)
            if rank != 0:
                unpack_upper(P, U)
            del P
        dist.broadcast(wt, _src(group), group=group)
        _hook(backend, "receive")
        if rank != 0:
            _hook(backend, "received")

    # 2. this rank's grid rows (an even share of the variance rows and of the others) and
    #    the var_range rows inside them
    v_lo, v_hi = var_rows(var_range, ne)
    pieces = [shard_pieces(ne, world, r, v_lo, v_hi) for r in range(world)]
    rows = [sum(b - a for a, b in p) for p in pieces]

    # 3. the rank's rows (piece order) into shard-sized buffers of emax rows, all-gather,
    #    reassemble the reference layouts
    emax = max(max(rows), 1)
    mu_sh = var_sh = None
    err = None
    try:
        mine = pieces[rank]
        if mine and hasattr(backend, "predict_shard"):  # one call, shard-sized outputs
            mu_sh, var_sh = backend.predict_shard(cm, U, wt, mine, v_lo, v_hi, emax)
            if tuple(mu_sh.shape) != (nq, emax) or tuple(var_sh.shape) != (emax * nq,):
                raise GprError(f"predict_shard returned {tuple(mu_sh.shape)} / "
                               f"{tuple(var_sh.shape)}, expected ({nq}, {emax}) / ({emax * nq},)")
        elif mine:  # generic backend: full-layout rows per piece, copied into the shard
            off = 0
            for lo, hi in mine:
                mu_full, var_full = backend.predict_rows(cm, U, wt, lo, hi, v_lo, v_hi)
                if mu_sh is None:
                    mu_sh = torch.zeros(nq, emax, dtype=mu_full.dtype, device=mu_full.device)
                    var_sh = torch.zeros(emax * nq, dtype=var_full.dtype, device=var_full.device)
                mu_sh[:, off:off + hi - lo] = mu_full[:, lo:hi]
                var_sh[off * nq:(off + hi - lo) * nq] = var_full[lo * nq:hi * nq]
                off += hi - lo
    except Exception as e:  # noqa: BLE001 -- re-raised after the status exchange
        err = e
    # as for the fit: every rank learns of a failed shard before the all_gather, so all ranks
    # raise instead of the healthy ones blocking in the collective
    bad = torch.tensor([0 if err is None else 1], dtype=torch.int64, device=dev)
    dist.all_reduce(bad, op=dist.ReduceOp.MAX, group=group)
    if int(bad.item()):
        if err is not None:
            raise err
        raise GprError("split_predict_distributed: a shard failed on another rank")
    if mu_sh is None:  # no rows here (more ranks than rows)
        mu_sh = torch.zeros(nq, emax, dtype=torch.float64, device=dev)
        var_sh = torch.zeros(emax * nq, dtype=torch.float64, device=dev)
    mus = [torch.empty_like(mu_sh) for _ in range(world)]
    vars_ = [torch.empty_like(var_sh) for _ in range(world)]
    dist.all_gather(mus, mu_sh, group=group)
    dist.all_gather(vars_, var_sh, group=group)
    mu = np.empty((nq, ne))
    var = np.empty(ne * nq)
    for r in range(world):
        mr, vr = mus[r].cpu().numpy(), vars_[r].cpu().numpy()
        off = 0
        for a, b in pieces[r]:
            mu[:, a:b] = mr[:, off:off + b - a]
            var[a * nq:b * nq] = vr[off * nq:(off + b - a) * nq]
            off += b - a
    return mu.T.copy(), var


# =========================================================================================
# One process, several GPUs: the C ABI's own sharded path (gpr_split_predict_mgpu, mgpu.hip)
# =========================================================================================
class MultiGPU:
    """gpr_mgpu_create(ngpu, devices): one context per device and an RCCL communicator over
    them (ncclCommInitAll), for gpr_split_predict_mgpu.  Reuse across calls; close() frees."""

    def __init__(self, devices):
        self.devices = [int(d) for d in devices]
        arr = (ctypes.c_int * len(self.devices))(*self.devices)
        h = ctypes.c_void_p()
        rc = lib.gpr_mgpu_create(len(self.devices), arr, ctypes.byref(h))
        if rc != 0:
            raise GprError(f"gpr_mgpu_create({self.devices}) failed ({rc})")
        self.h = h

    def set_knob(self, name: str, value: float) -> None:
        """gpr_mgpu_set_knob: GPR_MGPU_STREAM / _CHUNKS / _RESERVE_CU (include/gpr_hip.h)."""
        if lib.gpr_mgpu_set_knob(self.h, name.encode(), float(value)) != 0:
            raise GprError(f"set_knob({name}): {lib.gpr_mgpu_last_error(self.h).decode()}")

    def get_knob(self, name: str) -> float:
        v = ctypes.c_double()
        if lib.gpr_mgpu_get_knob(self.h, name.encode(), ctypes.byref(v)) != 0:
            raise GprError(f"get_knob({name}): {lib.gpr_mgpu_last_error(self.h).decode()}")
        return v.value

    def close(self):
        if getattr(self, "h", None):
            lib.gpr_mgpu_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def split_predict_mgpu(md: core.GPRModel, cm: core.Cmap, mg: MultiGPU,
                       var_range: Optional[Tuple[int, int]] = (1, 3), fit: str = "broadcast",
                       eps: float = core.EPS_DEFAULT):
    """predict(md, Cmap(+, xe, xq); diagonal_var=true) over the GPUs of `mg` in this one
    process (host arrays in and out).  Returns (mu ne x nq, var ne nq) like
    split_predict_distributed."""
    if md.y.ndim != 1:
        raise ValueError("split prediction needs a 1-D y (Diagonal(wt), src/split_predict.jl:13)")
    mode = {"broadcast": 0, "replicate": 1}[fit]
    _, ne, nq = cm.shape
    v_lo, v_hi = var_rows(var_range, ne)
    kinds, nk = core._kinds_arr(md.covar)
    _, hpp = core._hp_arr(md.params)
    D = ctypes.POINTER(ctypes.c_double)
    c = lambda a: np.ascontiguousarray(a, dtype=np.float64)  # noqa: E731
    X = c(md.x.T)          # d x ns column-major == ns x d row-major
    y = c(md.y)
    Xe, Xq = c(cm.xe.T), c(cm.xq.T)
    mu = np.empty((nq, ne))  # ne x nq column-major
    var = np.empty(ne * nq)
    info = ctypes.c_int(0)
    rc = lib.gpr_split_predict_mgpu(mg.h, kinds, nk, hpp, md.d, X.ctypes.data_as(D), md.n,
                                    y.ctypes.data_as(D), Xe.ctypes.data_as(D), ne,
                                    Xq.ctypes.data_as(D), nq, v_lo, v_hi, eps, mode,
                                    mu.ctypes.data_as(D), var.ctypes.data_as(D), ctypes.byref(info))
    if info.value > 0:
        raise PosDefException(info.value)
    if rc != 0:
        raise GprError(f"gpr_split_predict_mgpu failed ({rc}): "
                       f"{lib.gpr_mgpu_last_error(mg.h).decode()}")
    return mu.T.copy(), var
