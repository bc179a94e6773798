"""Oracle parity at BASELINE.json's full sizes (C2-C5), against committed fixtures.

The CPU oracle cannot run on the GPU box inside a test's time budget at these sizes, so
tests/golden/make_fullsize.py ran it once in the build container on the benches' exact seeded
inputs and stored compact outputs (tests/golden/fullsize_C*.npz).  Each test regenerates the
inputs from the same seeds, checks their SHA-256 against the fixture, runs the HIP path through
the C ABI (gpr_amd) and compares:

  C2  SE, N = 8192, d = 8, np = 8192: predict(md, xp; diagonal_var=true) -- mean rtol 1e-8
      (north_star), variance atol 1e-8 x prior (prior - ||V||^2 cancels), alpha = K^{-1} y
      normwise 1e-8, MLL rtol 1e-10.
  C3  SE+SE+WN, N = 32768, d = 8, np = 8192: the same quantities (the bench's gpr_fit_predict).
  C4  SE+WN, N = 16384, d = 16: MLL rtol 1e-10 and all 18 gradient components within
      1e-8 x (|a'dKa| + |<K^-1, dK>|) -- the two terms of src/loss_grad.jl:43-52, whose difference
      cancels -- plus the LogScale chain rule.
  C5  split predict, ns = 32768, ne = nq = 1024, var_range = 1:3 (the reference default): mean on
      every 32nd grid row rtol 1e-8, the three variance rows atol 1e-8 x prior.
"""
import os
import sys

import numpy as np
import pytest

from oracle import gpr_oracle as O

pytestmark = pytest.mark.gpu
G = pytest.importorskip("gpr_amd")

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import make_fullsize as MF  # noqa: E402


def _cov(kinds):
    parts = [G.SquaredExp() if k == O.SE else G.WhiteNoise() for k in kinds]
    c = parts[0]
    for p in parts[1:]:
        c = c + p
    return c


def _load(name):
    path = MF.fixture_path(name)
    if not os.path.exists(path):
        pytest.fail(f"missing fixture {path}: run tests/golden/make_fullsize.py {name}")
    fx = np.load(path)  # allow_pickle=False (default): plain arrays only
    cfg = MF.CONFIGS[name]
    inp = MF.inputs(cfg)
    keys = [k for k in ("x", "y", "xp", "xe", "xq") if k in inp]
    assert str(fx["input_sha256"]) == MF.checksum([inp[k] for k in keys]), "inputs changed"
    np.testing.assert_array_equal(fx["hp"], inp["hp"])
    return cfg, inp, fx


def _relnorm(a, b):
    return float(np.linalg.norm(a - b) / np.linalg.norm(b))


def _posterior_case(name):
    cfg, inp, fx = _load(name)
    kinds, hp = cfg["kinds"], inp["hp"]
    md = G.GPRModel(_cov(kinds), hp, inp["x"], inp["y"])
    mu, var = G.predict(md, inp["xp"], diagonal_var=True)
    prior = O.diag_prior(kinds, hp, cfg["d"])
    np.testing.assert_allclose(mu, fx["mu"], rtol=1e-8, atol=1e-10)
    assert _relnorm(mu, fx["mu"]) <= 1e-8
    np.testing.assert_allclose(var, fx["var"], rtol=1e-8, atol=1e-8 * prior)
    # alpha = K^{-1} y (update_cache!, src/predict.jl:29-34) and the MLL from the same factor
    tc = G.MllLossCache(md)
    G.update_cache_(tc, hp, md)
    alpha = md.ctx.host(tc.alpha)
    assert _relnorm(alpha, fx["alpha"]) <= 1e-8
    L = G.core._mll_value(md, tc)
    np.testing.assert_allclose(L, float(fx["mll"]), rtol=1e-10)
    del tc


def test_c2_predict_vs_oracle_fixture():
    _posterior_case("C2")


def test_c3_predict_vs_oracle_fixture():
    _posterior_case("C3")


def test_c4_mll_grad_vs_oracle_fixture():
    cfg, inp, fx = _load("C4")
    kinds, hp = cfg["kinds"], inp["hp"]
    md = G.GPRModel(_cov(kinds), hp, inp["x"], inp["y"])
    tc = G.MllGradCache(md)
    F = G.loss_grad_(G.MarginalLikelihood(), 0.0, np.zeros(len(hp)), hp, md, tc)
    np.testing.assert_allclose(F, float(fx["mll"]), rtol=1e-10)
    g = np.zeros(len(hp))
    G.loss_grad_(G.MarginalLikelihood(), None, g, hp, md, tc)
    scale = np.abs(fx["grad_p1"]) + np.abs(fx["grad_p2"])
    assert np.all(np.abs(g - fx["grad"]) <= 1e-8 * scale), (g - fx["grad"]) / scale
    alpha = md.ctx.host(tc.alpha)
    assert _relnorm(alpha, fx["alpha"]) <= 1e-8
    # log_loss_grad! (src/cost.jl:60-70): G .*= hp at hp = exp(log hp)
    gl = np.zeros(len(hp))
    G.log_loss_grad_(G.MarginalLikelihood(), None, gl, np.log(hp), md, tc)
    assert np.all(np.abs(gl - fx["grad"] * hp) <= 1e-8 * scale * hp + 1e-300)


def test_c5_split_predict_vs_oracle_fixture():
    cfg, inp, fx = _load("C5")
    kinds, hp = cfg["kinds"], inp["hp"]
    md = G.GPRModel(_cov(kinds), hp, inp["x"], inp["y"])
    cm = G.Cmap("+", inp["xe"], inp["xq"])
    mu, var = G.predict(md, cm, diagonal_var=True, var_range=cfg["var_range"])
    rows = fx["rows"]
    np.testing.assert_allclose(mu[rows], fx["mu_rows"], rtol=1e-8, atol=1e-10)
    assert _relnorm(mu[rows], fx["mu_rows"]) <= 1e-8
    prior = O.diag_prior(kinds, hp, cfg["d"])
    lo, hi = cfg["var_range"]
    nq = cfg["nq"]
    np.testing.assert_allclose(var[(lo - 1) * nq:hi * nq], fx["var_head"], rtol=1e-8,
                               atol=1e-8 * prior)
    assert np.all(var[hi * nq:] == prior)  # rows outside var_range keep the prior


@pytest.mark.parametrize("stream", ["0", "1"])
def test_c5_split_predict_mgpu_all_devices_vs_oracle_fixture(stream):
    """C5 sharded over EVERY visible device (gpr_split_predict_mgpu: one context and RCCL
    communicator per device, cost-balanced e-row shards, rows copied straight into the host
    result) against the oracle fixture -- the same rows and tolerances as the single-device
    test above -- for both fit modes (device 0 fits and broadcasts the packed factor over
    RCCL / every device fits) and both broadcast schedules (GPR_MGPU_STREAM: after the fit, or
    streamed while device 0 factors).  Skips below two devices (the development pool has one
    GPU per box; the driver's multi-GPU node runs it)."""
    import torch
    ndev = torch.cuda.device_count()
    if ndev < 2:
        pytest.skip("needs two or more GPUs")
    import gpr_amd.distributed as gd
    cfg, inp, fx = _load("C5")
    kinds, hp = cfg["kinds"], inp["hp"]
    md = G.GPRModel(_cov(kinds), hp, inp["x"], inp["y"])
    cm = G.Cmap("+", inp["xe"], inp["xq"])
    prior = O.diag_prior(kinds, hp, cfg["d"])
    lo, hi = cfg["var_range"]
    nq = cfg["nq"]
    rows = fx["rows"]
    mg = gd.MultiGPU(list(range(ndev)))
    try:
        mg.set_knob("GPR_MGPU_STREAM", int(stream))
        for fit in ("broadcast", "replicate"):
            mu, var = gd.split_predict_mgpu(md, cm, mg, var_range=cfg["var_range"], fit=fit)
            np.testing.assert_allclose(mu[rows], fx["mu_rows"], rtol=1e-8, atol=1e-10)
            assert _relnorm(mu[rows], fx["mu_rows"]) <= 1e-8
            np.testing.assert_allclose(var[(lo - 1) * nq:hi * nq], fx["var_head"], rtol=1e-8,
                                       atol=1e-8 * prior)
            assert np.all(var[hi * nq:] == prior)
    finally:
        mg.close()


def test_c5_split_predict_distributed_rccl_vs_oracle_fixture():
    """C5 through split_predict_distributed over an RCCL process group (backend "nccl"), one
    fresh process per visible device -- the torch.distributed path bench.py's C5 leg and the
    driver's SCALE runs measure, not the one-process C ABI path above -- for both fit modes
    (rank 0 fits and broadcasts the packed U + wt / every rank fits), every rank's all-gathered
    result against the oracle fixture at the single-device tolerances (tests/dist_c5_worker.py).
    Skips below two devices: RCCL refuses two ranks on one device (the one-GPU box covers the
    same path with gloo in test_distributed.py)."""
    import socket
    import subprocess

    import torch
    ndev = torch.cuda.device_count()
    if ndev < 2:
        pytest.skip("needs two or more GPUs (one RCCL rank per device)")
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(ndev):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(ndev),
                   LOCAL_WORLD_SIZE=str(ndev), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "dist_c5_worker.py")],
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                                      text=True))
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=600)[0])
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    for r, (p, out) in enumerate(zip(procs, outs)):
        assert p.returncode == 0 and f"OK rank {r}" in out, f"rank {r} rc {p.returncode}:\n{out[-3000:]}"
