"""Multi-process split prediction (gpr_amd.distributed) on CPU with gloo.

The distributed logic under test is the product code: rank-0 fit + broadcast of (U, wt)
(or replicated fits), balanced row sharding, var_range rows per shard, padded all_gather
and reassembly into the reference layouts (mu ne x nq with linear e + q ne,
src/split_predict.jl:10-19; var.diag index e nq + q, :39-53).  Only the per-rank compute
is swapped for an oracle-backed CPU backend (test infrastructure), which fills the same
full-layout buffers the HIP backend fills.  Expected results come from the single-process
oracle split_predict.  A GPU test runs the real HIP backend over a 1-rank RCCL group.
"""
import os
import socket

import numpy as np
import pytest
import scipy.linalg as sla
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import gpr_oracle as O

gd = pytest.importorskip("gpr_amd.distributed")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _problem(ne=7, nq=5, ns=60, d=3, seed=4):
    rng = np.random.default_rng(seed)
    x = rng.random((d, ns))
    y = np.sin(x.sum(0)) ** 2
    xe, xq = 0.5 * rng.random((d, ne)), 0.5 * rng.random((d, nq))
    kinds = ["SE", "WN"]
    hp = O.default_hp(kinds, d, noise=0.05)
    return kinds, hp, x, y, xe, xq


class _Cmap:
    def __init__(self, xe, xq):
        self.xe, self.xq = xe, xq

    @property
    def shape(self):
        return (self.xe.shape[0], self.xe.shape[1], self.xq.shape[1])


class OracleBackend:
    """CPU stand-in for HipSplitBackend (same buffers, same row/var-range semantics)."""

    def __init__(self, kinds, hp, x, y, allow_fit=True):
        self.kinds, self.hp, self.x, self.y, self.allow_fit = kinds, hp, x, y, allow_fit

    def empty_fit(self):
        n = self.x.shape[1]
        return torch.empty(n, n, dtype=torch.float64), torch.empty(n, dtype=torch.float64)

    def fit(self):
        if not self.allow_fit:
            raise AssertionError("this rank must receive U/wt by broadcast")
        U = O.chol_upper(O.kernel(self.kinds, self.hp, self.x, None))
        wt = O.cho_solve_upper(U, self.y)
        return torch.from_numpy(np.ascontiguousarray(U.T)), torch.from_numpy(wt)  # column-major

    def predict_rows(self, cm, U, wt, e_lo, e_hi, v_lo, v_hi):
        _, ne, nq = cm.shape
        Un, w = U.numpy().T, wt.numpy()
        A, B, C = O.split_factors(self.kinds, self.hp, self.x, cm.xe, cm.xq)
        mu = torch.zeros(nq, ne, dtype=torch.float64)
        var = torch.zeros(ne * nq, dtype=torch.float64)
        prior = O.diag_prior(self.kinds, self.hp, self.x.shape[0])
        for e in range(e_lo, e_hi):
            m = np.zeros(nq)
            for k in range(A.shape[2]):
                m += A[e, :, k] * (B[e, :, k] @ (w[:, None] * C[:, :, k]))
            mu[:, e] = torch.from_numpy(m)
            var[e * nq:(e + 1) * nq] = prior
            if v_lo <= e < v_hi:
                Kxq = sum(A[e, :, None, k] * B[e, None, :, k] * C[:, :, k].T for k in range(A.shape[2]))
                V = sla.solve_triangular(Un, Kxq.T, trans="T", lower=False).T
                var[e * nq:(e + 1) * nq] = torch.from_numpy(prior - np.sum(V * V, axis=1))
        return mu, var


class ShardOracleBackend(OracleBackend):
    """The HIP backend's interface: predict_shard fills buffers sized to the rank's shard
    (emax rows, the pieces' rows concatenated), never a grid-sized one.  Records the calls."""

    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        self.calls = []

    def predict_shard(self, cm, U, wt, pieces, v_lo, v_hi, emax):
        _, ne, nq = cm.shape
        self.calls.append((list(pieces), emax))
        mu = torch.zeros(nq, emax, dtype=torch.float64)
        var = torch.zeros(emax * nq, dtype=torch.float64)
        off = 0
        for lo, hi in pieces:
            m_full, v_full = self.predict_rows(cm, U, wt, lo, hi, v_lo, v_hi)
            mu[:, off:off + hi - lo] = m_full[:, lo:hi]
            var[off * nq:(off + hi - lo) * nq] = v_full[lo * nq:hi * nq]
            off += hi - lo
        return mu, var


def _worker(rank, world, port, out, ne, nq, var_range, fit, kind="rows"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        kinds, hp, x, y, xe, xq = _problem(ne=ne, nq=nq)
        cls = ShardOracleBackend if kind == "shard" else OracleBackend
        be = cls(kinds, hp, x, y, allow_fit=(fit == "replicate" or rank == 0))
        mu, var = gd.split_predict_distributed(None, _Cmap(xe, xq), var_range=var_range,
                                               backend=be, fit=fit)
        np.save(os.path.join(out, f"mu{rank}.npy"), mu)
        np.save(os.path.join(out, f"var{rank}.npy"), var)
        if kind == "shard":
            with open(os.path.join(out, f"calls{rank}.txt"), "w") as f:
                f.write(repr(be.calls))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("kind", ["rows", "shard"])
@pytest.mark.parametrize("world,ne,nq,var_range,fit", [
    (2, 7, 5, (1, 3), "broadcast"),     # reference default var_range, ragged shards
    (3, 8, 4, (1, 8), "replicate"),     # full var_range, replicated factorisation
    (2, 9, 3, (3, 7), "broadcast"),     # var_range straddling the shard boundary
    (3, 2, 6, (1, 3), "broadcast"),     # more ranks than rows: an empty shard
    (3, 10, 3, (4, 9), "broadcast"),    # variance rows in the middle: 3-piece shards
    (4, 9, 2, (1, 3), "replicate"),     # fewer variance rows than ranks
])
def test_split_predict_distributed_gloo(tmp_path, world, ne, nq, var_range, fit, kind):
    port = _free_port()
    mp.spawn(_worker, args=(world, port, str(tmp_path), ne, nq, var_range, fit, kind),
             nprocs=world, join=True)
    kinds, hp, x, y, xe, xq = _problem(ne=ne, nq=nq)
    mu_o, var_o = O.split_predict(kinds, hp, x, y, xe, xq, var_range=var_range)
    for r in range(world):  # every rank holds the full result
        mu = np.load(tmp_path / f"mu{r}.npy")
        var = np.load(tmp_path / f"var{r}.npy")
        assert mu.shape == (ne, nq)
        np.testing.assert_allclose(mu, mu_o, rtol=1e-12, atol=1e-14)
        np.testing.assert_allclose(var, var_o, rtol=1e-12, atol=1e-14)
    if kind == "shard":
        # one predict_shard call per rank with rows, its buffers sized to the largest share
        # (the all_gather's common size), not to the grid's ne rows
        v_lo, v_hi = gd.var_rows(var_range, ne)
        pieces = [gd.shard_pieces(ne, world, r, v_lo, v_hi) for r in range(world)]
        emax = max(max(sum(b - a for a, b in p) for p in pieces), 1)
        assert emax <= -(-ne // world) + 1
        for r in range(world):
            calls = eval(open(tmp_path / f"calls{r}.txt").read())
            assert calls == ([(pieces[r], emax)] if pieces[r] else []), (r, calls)


class FailingBackend(OracleBackend):
    """fit() raises on the ranks listed in `fail` (PosDefException(info) or a generic error)."""

    def __init__(self, *a, fail=(), info=7, fail_rows=(), **kw):
        super().__init__(*a, **kw)
        self.fail, self.info, self.fail_rows = fail, info, fail_rows

    def predict_rows(self, *a, **kw):
        if dist.get_rank() in self.fail_rows:
            raise RuntimeError("simulated shard failure")
        return super().predict_rows(*a, **kw)

    def fit(self):
        if dist.get_rank() in self.fail:
            if self.info > 0:
                from gpr_amd._lib import PosDefException
                raise PosDefException(self.info)
            raise RuntimeError("simulated HIP failure")
        return super().fit()


class FailingShardBackend(FailingBackend, ShardOracleBackend):
    """FailingBackend behind the predict_shard interface (its predict_shard calls the
    failing predict_rows)."""


def _fail_worker(rank, world, port, out, fit, fail, info, fail_rows=(), kind="rows"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        kinds, hp, x, y, xe, xq = _problem(ne=5, nq=3)
        cls = FailingShardBackend if kind == "shard" else FailingBackend
        be = cls(kinds, hp, x, y, fail=fail, info=info, fail_rows=fail_rows)
        try:
            gd.split_predict_distributed(None, _Cmap(xe, xq), backend=be, fit=fit)
            res = "ok"
        except Exception as e:  # noqa: BLE001
            res = f"{type(e).__name__}:{getattr(e, 'info', '')}"
        with open(os.path.join(out, f"r{rank}.txt"), "w") as f:
            f.write(res)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("fit,fail,info,expect", [
    ("broadcast", (0,), 7, "PosDefException:7"),    # rank 0's PosDef reaches every rank
    ("broadcast", (0,), 0, None),                    # generic failure: no rank hangs
    ("replicate", (1,), 3, "PosDefException:3"),    # one replica fails: all raise
])
def test_split_predict_distributed_fit_failure(tmp_path, fit, fail, info, expect):
    """A failed fit raises on EVERY rank (the other ranks used to block in the
    broadcast).  mp.spawn with join=True would hang here if any rank blocked."""
    world = 3
    mp.spawn(_fail_worker, args=(world, _free_port(), str(tmp_path), fit, fail, info),
             nprocs=world, join=True)
    res = [open(tmp_path / f"r{r}.txt").read() for r in range(world)]
    assert all(r != "ok" for r in res), res
    if expect is not None:
        assert all(r == expect for r in res), res
    else:
        assert res[0].startswith("RuntimeError") and all(r.startswith("GprError") for r in res[1:])


def test_shard_rows_partition():
    for n in range(0, 40):
        for world in range(1, 9):
            parts = [gd.shard_rows(n, world, r) for r in range(world)]
            assert parts[0][0] == 0 and parts[-1][1] == n
            assert all(parts[r][1] == parts[r + 1][0] for r in range(world - 1))
            sizes = [b - a for a, b in parts]
            assert max(sizes) - min(sizes) <= 1


def test_shard_pieces_partition_and_balance():
    """Every row on exactly one rank; variance rows and mean-only rows each split evenly
    (within one row) -- the variance rows are the expensive ones (an N^2 solve per point)."""
    for n in range(0, 30):
        for world in range(1, 9):
            for v_lo in range(0, n + 1, 3):
                for v_hi in (v_lo, min(n, v_lo + 1), min(n, v_lo + 5), n):
                    parts = [gd.shard_pieces(n, world, r, v_lo, v_hi) for r in range(world)]
                    rows = sorted(e for p in parts for a, b in p for e in range(a, b))
                    assert rows == list(range(n))
                    for p in parts:
                        assert all(a < b for a, b in p)
                        assert all(p[i][1] < p[i + 1][0] for i in range(len(p) - 1))
                        assert len(p) <= 3
                    nv = [sum(1 for a, b in p for e in range(a, b) if v_lo <= e < v_hi) for p in parts]
                    nm = [sum(b - a for a, b in p) - k for p, k in zip(parts, nv)]
                    assert max(nv) - min(nv) <= 1 and max(nm) - min(nm) <= 1
    # the bench's C5 shape: 32 variance rows of 1024 over 8 ranks -> 4 each
    parts = [gd.shard_pieces(1024, 8, r, 0, 32) for r in range(8)]
    assert [sum(b - a for a, b in p if a < 32) for p in parts] == [4] * 8


@pytest.mark.parametrize("n", [0, 1, 5, 127, 128, 129, 300])
def test_pack_upper_roundtrip(n):
    """The broadcast's packed upper triangle: round trip restores every entry on or above
    the diagonal (column-major: tensor row c = column c, upper entries U[c, :c+1])."""
    U = torch.from_numpy(np.random.default_rng(n).random((n, n)))
    P = gd.pack_upper(U)
    assert P.numel() == gd._packed_len(n) <= n * (n + 128) // 2 + 128 * 128
    V = torch.full((n, n), np.nan, dtype=torch.float64)
    gd.unpack_upper(P, V)
    for c in range(n):
        assert torch.equal(V[c, :c + 1], U[c, :c + 1])


def test_var_rows_conversion():
    assert gd.var_rows((1, 3), 10) == (0, 3)        # Julia 1:3 -> [0, 3)
    assert gd.var_rows((1, 3), 2) == (0, 2)         # clamped to ne
    assert gd.var_rows(None, 5) == (0, 0)
    assert gd.var_rows((4, 3), 5) == (0, 0)         # empty range


@pytest.mark.gpu
def test_split_predict_distributed_hip_single_rank():
    """The HIP backend through the real collective path (1-rank RCCL group) equals the
    single-process split predict."""
    G = pytest.importorskip("gpr_amd")
    if dist.is_initialized():
        pytest.skip("process group already initialised")
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        kinds, hp, x, y, xe, xq = _problem(ne=11, nq=13, ns=300, d=4)
        md = G.GPRModel(G.SquaredExp() + G.WhiteNoise(), hp, x, y)
        cm = G.Cmap("+", xe, xq)
        for fit in ("broadcast", "replicate"):
            mu, var = gd.split_predict_distributed(md, cm, var_range=(1, 11), fit=fit)
            mu1, var1 = G.predict(md, cm, diagonal_var=True, var_range=(1, 11))
            np.testing.assert_allclose(mu, mu1, rtol=1e-14, atol=0)
            np.testing.assert_allclose(var, var1, rtol=1e-14, atol=0)
        mu_o, var_o = O.split_predict(kinds, hp, x, y, xe, xq, var_range=(1, 11))
        np.testing.assert_allclose(mu, mu_o, rtol=1e-8, atol=1e-10)
    finally:
        dist.destroy_process_group()


def _hp_iter(hp, it):
    hp = np.array(hp, dtype=np.float64)
    if it == 1:
        hp[1:-1] *= 1.3
        hp[-1] *= 0.7
    return hp


def _hip_gloo_worker(rank, world, port, out, fit):
    """Two ranks on ONE GPU over gloo with device tensors: the HIP backend's stream ordering
    around the collectives (gpr_fit leaves the wt solve queued on the context stream; the
    collectives order only against torch's current stream)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import gpr_amd as G
        kinds, hp, x, y, xe, xq = _problem(ne=9, nq=40, ns=4096, d=6, seed=11)
        cm = G.Cmap("+", xe, xq)
        for it in range(3):
            # iteration 1 changes the hyperparameters: a rank that receives U into a re-used
            # allocation must not solve with the previous factor's cached inverses
            md = G.GPRModel(G.SquaredExp() + G.WhiteNoise(), _hp_iter(hp, it), x, y)
            mu, var = gd.split_predict_distributed(md, cm, var_range=(1, 9), fit=fit)
            np.save(os.path.join(out, f"mu{rank}_{it}.npy"), mu)
            np.save(os.path.join(out, f"var{rank}_{it}.npy"), var)
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("fit", ["broadcast", "replicate"])
def test_split_predict_distributed_hip_two_ranks(tmp_path, fit):
    """world = 2 on the HIP backend (both ranks on cuda:0, gloo carrying device tensors),
    N = 4096 so the fit's queued solve and the broadcast overlap if unordered: every rank's
    result equals the single-process split predict (rtol 1e-12; a race shows as O(1) errors)."""
    G = pytest.importorskip("gpr_amd")
    mp.spawn(_hip_gloo_worker, args=(2, _free_port(), str(tmp_path), fit), nprocs=2, join=True)
    kinds, hp, x, y, xe, xq = _problem(ne=9, nq=40, ns=4096, d=6, seed=11)
    for it in range(3):
        md = G.GPRModel(G.SquaredExp() + G.WhiteNoise(), _hp_iter(hp, it), x, y)
        mu1, var1 = G.predict(md, G.Cmap("+", xe, xq), diagonal_var=True, var_range=(1, 9))
        for r in range(2):
            np.testing.assert_allclose(np.load(tmp_path / f"mu{r}_{it}.npy"), mu1, rtol=1e-12, atol=1e-14)
            np.testing.assert_allclose(np.load(tmp_path / f"var{r}_{it}.npy"), var1, rtol=1e-12, atol=1e-14)


@pytest.mark.parametrize("kind", ["rows", "shard"])
@pytest.mark.parametrize("fit", ["broadcast", "replicate"])
def test_split_predict_distributed_shard_failure(tmp_path, fit, kind):
    """A shard that fails on one rank (rank 1's predict_rows / predict_shard raises) raises on
    EVERY rank instead of leaving the others blocked in the all_gather."""
    world = 3
    mp.spawn(_fail_worker, args=(world, _free_port(), str(tmp_path), fit, (), 0, (1,), kind),
             nprocs=world, join=True)
    res = [open(tmp_path / f"r{r}.txt").read() for r in range(world)]
    assert res[1].startswith("RuntimeError"), res
    assert res[0].startswith("GprError") and res[2].startswith("GprError"), res


def test_c_shard_pieces_matches_python():
    """gpr_shard_pieces (mgpu.hip, host-only C) is the same partition as shard_pieces: the C
    ABI's sharded path and the torch.distributed path give every device the same rows."""
    import ctypes
    from gpr_amd import _lib
    out = (ctypes.c_int * 6)()
    for n in range(0, 34):
        for world in range(1, 9):
            for v_lo in range(0, n + 1, 3):
                for v_hi in (v_lo, min(n, v_lo + 1), min(n, v_lo + 5), n):
                    for r in range(world):
                        k = _lib.lib.gpr_shard_pieces(n, world, r, v_lo, v_hi, out)
                        assert [(out[2 * i], out[2 * i + 1]) for i in range(k)] == \
                            gd.shard_pieces(n, world, r, v_lo, v_hi)
    assert _lib.lib.gpr_shard_pieces(5, 0, 0, 0, 0, out) < 0
    for n in (0, 1, 127, 128, 129, 300, 32768):
        assert _lib.lib.gpr_packed_upper_len(n) == gd._packed_len(n)


@pytest.mark.gpu
def test_pack_unpack_upper_device_roundtrip():
    """gpr_pack_upper / gpr_unpack_upper (the broadcast's packed layout) against pack_upper,
    and the round trip restores the upper triangle, leaving the rest untouched."""
    import ctypes
    G = pytest.importorskip("gpr_amd")
    from gpr_amd import _lib
    ctx = G.Context(0)
    for n in (1, 127, 128, 300, 1000):
        U = torch.from_numpy(np.random.default_rng(n).random((n, n))).to(ctx.device)
        P = ctx.empty(_lib.lib.gpr_packed_upper_len(n))
        torch.cuda.synchronize()  # U was written on torch's stream, the calls run on ctx's
        assert _lib.lib.gpr_pack_upper(ctx.h, ctypes.c_void_p(U.data_ptr()), n, n,
                                       ctypes.c_void_p(P.data_ptr())) == 0
        ctx.sync()
        assert torch.equal(P.cpu(), gd.pack_upper(U.cpu()))
        V = torch.full((n, n), -7.0, dtype=torch.float64, device=ctx.device)
        torch.cuda.synchronize()
        assert _lib.lib.gpr_unpack_upper(ctx.h, ctypes.c_void_p(P.data_ptr()), n,
                                         ctypes.c_void_p(V.data_ptr()), n) == 0
        ctx.sync()
        Uc, Vc = U.cpu(), V.cpu()
        for c in range(n):
            assert torch.equal(Vc[c, :c + 1], Uc[c, :c + 1])
            assert torch.all(Vc[c, (c // 128 + 1) * 128:] == -7.0)


@pytest.mark.gpu
@pytest.mark.parametrize("fit", ["broadcast", "replicate"])
def test_split_predict_mgpu_one_device(fit):
    """gpr_split_predict_mgpu with ngpu = 1 equals gpr_fit + gpr_split_predict on that device
    bit for bit (the one-GPU box cannot run more; the shard partition is tested against the
    Python path above and the multi-rank logic with gloo), and matches the oracle."""
    G = pytest.importorskip("gpr_amd")
    kinds, hp, x, y, xe, xq = _problem(ne=13, nq=17, ns=700, d=4, seed=8)
    md = G.GPRModel(G.SquaredExp() + G.WhiteNoise(), hp, x, y)
    cm = G.Cmap("+", xe, xq)
    mg = gd.MultiGPU([0])
    try:
        for vr in ((1, 3), (2, 13), None):
            mu, var = gd.split_predict_mgpu(md, cm, mg, var_range=vr, fit=fit)
            mu1, var1 = G.predict(md, cm, diagonal_var=True,
                                  var_range=vr if vr is not None else (1, 0))
            assert np.array_equal(mu, mu1) and np.array_equal(var, var1)
        mu_o, var_o = O.split_predict(kinds, hp, x, y, xe, xq, var_range=(2, 13))
        mu, var = gd.split_predict_mgpu(md, cm, mg, var_range=(2, 13), fit=fit)
        np.testing.assert_allclose(mu, mu_o, rtol=1e-8, atol=1e-10)
        np.testing.assert_allclose(var, var_o, rtol=1e-8, atol=1e-8)
        # a non positive definite K (eps = -1 cancels sigma^2 = 1 on the diagonal) -> info > 0
        with pytest.raises(G.PosDefException):
            gd.split_predict_mgpu(G.GPRModel(G.SquaredExp(), np.r_[1.0, hp[1:-1]], x, y), cm, mg,
                                  fit=fit, eps=-1.0)
    finally:
        mg.close()
    with pytest.raises(G.GprError):  # one rank per GPU
        gd.MultiGPU([0, 0])


@pytest.mark.gpu
@pytest.mark.parametrize("ns,stream,chunks", [
    (1504, "1", "16"),   # streamed beside the tile-DAG launch, ragged last tile row (96 rows)
    (1504, "1", "1"),    # one chunk: everything after the last tile row
    (4096, "1", "5"),    # 32 tile rows in 5 chunks
    (1504, "0", "3"),    # chunks after the fit (GPR_MGPU_STREAM=0)
    (1500, "1", "16"),   # n % 16 != 0: the padded factorisation declines the hook -> after the fit
])
def test_split_predict_mgpu_broadcast_path_one_device(ns, stream, chunks):
    """The broadcast path of gpr_split_predict_mgpu on the one-GPU box: device 0 broadcasts to
    itself (a test-build-only switch) and predicts from the received copy; equal to the single-
    device split predict to rtol 1e-12 (tests/fault_scenarios.py mgpu_self_bcast, child process
    on libgpr_hip_testing.so)."""
    from conftest import run_fault_scenario
    run_fault_scenario("mgpu_self_bcast", ns, stream, chunks)


@pytest.mark.gpu
def test_mgpu_knobs_release_build():
    """The handle's knobs through gpr_mgpu_set_knob / gpr_mgpu_get_knob (clamped as documented);
    the release library has no self-broadcast switch (unknown knob -> GprError)."""
    G = pytest.importorskip("gpr_amd")
    mg = gd.MultiGPU([0])
    try:
        assert mg.get_knob("GPR_MGPU_STREAM") in (-1, 0, 1)
        mg.set_knob("GPR_MGPU_STREAM", 5)
        assert mg.get_knob("GPR_MGPU_STREAM") == 1
        mg.set_knob("GPR_MGPU_STREAM", -3)
        assert mg.get_knob("GPR_MGPU_STREAM") == -1
        mg.set_knob("GPR_MGPU_CHUNKS", 0)
        assert mg.get_knob("GPR_MGPU_CHUNKS") == 1
        mg.set_knob("GPR_MGPU_RESERVE_CU", 12)
        assert mg.get_knob("GPR_MGPU_RESERVE_CU") == 12
        for bad in ("GPR_MGPU_SELF_BCAST", "GPR_DAG", "nope"):
            with pytest.raises(G.GprError):
                mg.set_knob(bad, 1)
    finally:
        mg.close()


@pytest.mark.gpu
def test_split_predict_shard_compact_equals_rows():
    """gpr_split_predict_shard (outputs sized to the shard: pieces' rows concatenated, mu with
    leading dimension ldmu >= R) equals gpr_split_predict_rows' full-layout rows bit for bit,
    for every rank's pieces of a 3-way split and with a padded leading dimension; ldmu < R is
    refused."""
    import ctypes
    G = pytest.importorskip("gpr_amd")
    from gpr_amd import core
    from gpr_amd._lib import lib
    kinds, hp, x, y, xe, xq = _problem(ne=23, nq=19, ns=600, d=4, seed=21)
    md = G.GPRModel(G.SquaredExp() + G.WhiteNoise(), hp, x, y)
    cm = G.Cmap("+", xe, xq)
    be = gd.HipSplitBackend(md)
    U, wt = be.fit()
    ctx = md.ctx
    ctx.sync()
    _, ne, nq = cm.shape
    ka, nk = core._kinds_arr(md.covar)
    _, hpp = core._hp_arr(md.params)
    dxe, dxq = ctx.colmajor(cm.xe), ctx.colmajor(cm.xq)
    v_lo, v_hi = 2, 17
    for world in (1, 3):
        for r in range(world):
            pieces = gd.shard_pieces(ne, world, r, v_lo, v_hi)
            R = sum(b - a for a, b in pieces)
            flat = [v for p in pieces for v in p]
            arr = (ctypes.c_int * max(len(flat), 1))(*flat)
            mu_f, var_f = ctx.zeros(nq, ne), ctx.zeros(ne * nq)
            assert lib.gpr_split_predict_rows(ctx.h, ka, nk, hpp, md.d, core._ptr(md.dx()), md.n,
                                              core._ptr(U), md.n, core._ptr(wt), core._ptr(dxe), ne,
                                              core._ptr(dxq), nq, arr, len(pieces), v_lo, v_hi,
                                              core.EPS_DEFAULT, core._ptr(mu_f), core._ptr(var_f)) == 0
            for ld in (R, R + 5):
                mu_s, var_s = be.predict_shard(cm, U, wt, pieces, v_lo, v_hi, ld)
                mf, vf, ms, vs = mu_f.cpu(), var_f.cpu(), mu_s.cpu(), var_s.cpu()
                off = 0
                for a, b in pieces:
                    assert torch.equal(ms[:, off:off + b - a], mf[:, a:b])
                    assert torch.equal(vs[off * nq:(off + b - a) * nq], vf[a * nq:b * nq])
                    off += b - a
                assert torch.all(ms[:, R:] == 0) and torch.all(vs[R * nq:] == 0)
            if R > 1:
                mu_s, var_s = ctx.zeros(nq, R), ctx.zeros(R * nq)
                rc = lib.gpr_split_predict_shard(ctx.h, ka, nk, hpp, md.d, core._ptr(md.dx()), md.n,
                                                 core._ptr(U), md.n, core._ptr(wt), core._ptr(dxe), ne,
                                                 core._ptr(dxq), nq, arr, len(pieces), v_lo, v_hi,
                                                 core.EPS_DEFAULT, core._ptr(mu_s), R - 1,
                                                 core._ptr(var_s))
                assert rc != 0


@pytest.mark.gpu
def test_split_predict_mgpu_gate_timeout_reports_and_recovers():
    """A streamed chunk whose gate gives up is reported as an error after every stream drained
    -- no hang -- and the next call on the same handle is correct (fault_scenarios.py, child
    process on the test build libgpr_hip_testing.so)."""
    from conftest import run_fault_scenario
    run_fault_scenario("mgpu_gate_timeout")


@pytest.mark.gpu
@pytest.mark.parametrize("stream,chunk", [("1", "0"), ("1", "3"), ("0", "2")])
def test_split_predict_mgpu_unpack_failure_reports_and_recovers(stream, chunk):
    """A receiver whose unpack of one chunk fails keeps receiving every remaining chunk and wt
    and reports the error once the protocol is complete; the next call on the same handle is
    correct (fault_scenarios.py, child process on the test build libgpr_hip_testing.so)."""
    from conftest import run_fault_scenario
    run_fault_scenario("mgpu_unpack_failure", stream, chunk)


@pytest.mark.gpu
@pytest.mark.parametrize("stream", ["0", "1"])
def test_split_predict_mgpu_two_devices(stream):
    """gpr_split_predict_mgpu over two GPUs (the real receiver branch, RCCL between devices)
    against the single-device split predict.  Skips on a box with fewer than two GPUs (the
    development pool has one; no ngpu >= 2 run has happened yet)."""
    G = pytest.importorskip("gpr_amd")
    import torch
    if torch.cuda.device_count() < 2:
        pytest.skip("needs two GPUs")
    kinds, hp, x, y, xe, xq = _problem(ne=11, nq=13, ns=2048, d=4, seed=15)
    md = G.GPRModel(G.SquaredExp() + G.WhiteNoise(), hp, x, y)
    cm = G.Cmap("+", xe, xq)
    mg = gd.MultiGPU([0, 1])
    try:
        mg.set_knob("GPR_MGPU_STREAM", int(stream))
        for fit in ("broadcast", "replicate"):
            mu, var = gd.split_predict_mgpu(md, cm, mg, var_range=(2, 11), fit=fit)
            mu1, var1 = G.predict(md, cm, diagonal_var=True, var_range=(2, 11))
            np.testing.assert_allclose(mu, mu1, rtol=1e-12, atol=1e-14)
            np.testing.assert_allclose(var, var1, rtol=1e-12, atol=1e-14)
    finally:
        mg.close()
