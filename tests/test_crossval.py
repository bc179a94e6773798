"""Cross-validation (src/crossval.jl) with the losses of src/loss_grad.jl:12-30.

The reference has no test for cv (its test/ directory never calls cv_batch), so parity is on
the oracle restatement: CPU tests pin the oracle's losses with closed forms (Mahalanobis =
r' Sigma^{-1} r, ChiSq with a diagonal Sigma = Mahalanobis, MSE of an exact prediction = 0)
and the fold structure of kfoldcv; GPU tests compare gpr_cv_batch with the oracle's
fit + full-covariance predict + loss per fold (rtol 1e-8, SURVEY.md §8(d)'s posterior
tolerance).
"""
import numpy as np
import pytest

from oracle import gpr_oracle as O

G = pytest.importorskip("gpr_amd")


def test_kfoldcv_structure():
    """src/crossval.jl:1-11: nb folds of k test points, disjoint, training = the rest."""
    n, k = 53, 7
    trn, tst = G.kfoldcv(n, k, rng=np.random.default_rng(0))
    assert len(trn) == len(tst) == n // k
    seen = np.concatenate(tst)
    assert len(set(seen.tolist())) == seen.size == (n // k) * k
    for a, b in zip(trn, tst):
        assert b.size == k and a.size == n - k
        assert sorted(np.concatenate([a, b]).tolist()) == list(range(n))
    # the oracle restatement with the same permutation gives the same folds
    perm = np.random.default_rng(0).permutation(n)
    otrn, otst = O.kfoldcv(n, k, perm=perm)
    for a, b, c, d in zip(trn, tst, otrn, otst):
        np.testing.assert_array_equal(a, c)
        np.testing.assert_array_equal(b, d)


def test_oracle_losses_closed_forms():
    rng = np.random.default_rng(1)
    m = 12
    A = rng.standard_normal((m, m))
    S = A @ A.T + m * np.eye(m)
    y, yp = rng.standard_normal(m), rng.standard_normal(m)
    r = y - yp
    assert O.cv_loss("Mahalanobis", y, yp, S) == pytest.approx(r @ np.linalg.solve(S, r),
                                                               rel=1e-12)
    D = np.diag(rng.random(m) + 0.5)
    assert O.cv_loss("ChiSq", y, yp, D) == pytest.approx(O.cv_loss("Mahalanobis", y, yp, D),
                                                         rel=1e-12)
    assert O.cv_loss("MSE", y, yp, S) == pytest.approx(np.mean(r * r), rel=1e-14)
    assert O.cv_loss("MSE", y, y, S) == 0.0


def test_cost_type_checked():
    with pytest.raises(TypeError):
        G.crossval._cost_code(G.MarginalLikelihood())


def _data(d, n, seed):
    rng = np.random.default_rng(seed)
    x = rng.random((d, n))
    y = np.sin(x.sum(axis=0)) ** 2
    return x, y


_KINDS = {"SE": (["SE"], lambda: G.SquaredExp()),
          "SE+WN": (["SE", "WN"], lambda: G.SquaredExp() + G.WhiteNoise()),
          "SE+SE+WN": (["SE", "SE", "WN"],
                       lambda: G.SquaredExp() + G.SquaredExp() + G.WhiteNoise())}
_COSTS = {"MSE": G.MSE, "ChiSq": G.ChiSq, "Mahalanobis": G.Mahalanobis}


@pytest.mark.gpu
@pytest.mark.parametrize("kname,cname", [("SE+WN", "MSE"), ("SE+WN", "ChiSq"),
                                         ("SE+WN", "Mahalanobis"), ("SE+SE+WN", "MSE"),
                                         ("SE+SE+WN", "Mahalanobis"), ("SE+SE+WN", "ChiSq")])
@pytest.mark.parametrize("d,n,k", [(2, 200, 20), (3, 331, 37)])
def test_cv_batch_vs_oracle(kname, cname, d, n, k):
    kinds, mk = _KINDS[kname]
    x, y = _data(d, n, 11 + d)
    hp = O.default_hp(kinds, d, length=2.0)
    md = G.GPRModel(mk(), hp, x, y)
    cvset = G.kfoldcv(n, k, rng=np.random.default_rng(5))
    got = G.cv_batch(md, _COSTS[cname](), x, y, cvset)
    want = O.cv_batch(kinds, hp, cname, x, y, cvset)
    np.testing.assert_allclose(got, want, rtol=1e-8, atol=0)


@pytest.mark.gpu
def test_cv_step_vs_oracle_and_batch():
    kinds = ["SE", "WN"]
    d, ntr, nts = 4, 260, 33
    x, y = _data(d, ntr + nts, 3)
    hp = O.default_hp(kinds, d, length=2.5)
    md = G.GPRModel(G.SquaredExp() + G.WhiteNoise(), hp, x[:, :ntr], y[:ntr])
    for cname, cost in _COSTS.items():
        got = G.cv_step(md, cost(), x[:, :ntr], y[:ntr], x[:, ntr:], y[ntr:])
        want = O.cv_step(kinds, hp, cname, x[:, :ntr], y[:ntr], x[:, ntr:], y[ntr:])
        assert got == pytest.approx(want, rel=1e-8)
        assert G.cv_step_(cost(), md, x[:, ntr:], y[ntr:]) == got


@pytest.mark.gpu
def test_cv_batch_rejects_bad_indices():
    x, y = _data(2, 50, 0)
    md = G.GPRModel(G.SquaredExp() + G.WhiteNoise(), O.default_hp(["SE", "WN"], 2), x, y)
    with pytest.raises(G.GprError):
        G.cv_batch(md, G.MSE(), x, y, ([np.arange(40)], [np.arange(45, 55)]))


@pytest.mark.gpu
def test_cv_concurrent_folds_bit_identical(monkeypatch):
    """Folds spread over child contexts (default GPR_CV_STREAMS=4) give exactly the losses of
    the one-context sequential run: same kernels, per-fold deterministic reductions."""
    d, n, k = 3, 600, 40
    x, y = _data(d, n, 21)
    hp = O.default_hp(["SE", "WN"], d, length=2.0)
    cvset = G.kfoldcv(n, k, rng=np.random.default_rng(2))
    out = {}
    for streams in ("1", "4", "8"):
        monkeypatch.setenv("GPR_CV_STREAMS", streams)
        ctx = G.Context(0)
        md = G.GPRModel(G.SquaredExp() + G.WhiteNoise(), hp, x, y, ctx=ctx)
        out[streams] = G.cv_batch(md, G.Mahalanobis(), x, y, cvset)
        ctx.close()
    np.testing.assert_array_equal(out["1"], out["4"])
    np.testing.assert_array_equal(out["1"], out["8"])


@pytest.mark.gpu
@pytest.mark.parametrize("cname", ["MSE", "ChiSq", "Mahalanobis"])
def test_cv_batched_launch_vs_per_fold(cname, knobs):
    """Every fold's factorisation (and, for Mahalanobis, every Sigma_p's) in one batched tile-DAG
    launch (GPR_CV_BATCH=1; padded to multiples of 16: ntrn = 341, ntst = 31 here) against the
    per-fold path: the same losses to rounding; a one-fold memory budget (one launch per fold)
    gives the batched result bit for bit."""
    d, n, k = 3, 372, 31
    x, y = _data(d, n, 8)
    hp = O.default_hp(["SE", "WN"], d, length=2.0)
    md = G.GPRModel(G.SquaredExp() + G.WhiteNoise(), hp, x, y)
    cvset = G.kfoldcv(n, k, rng=np.random.default_rng(4))
    knobs("GPR_CV_BATCH", 0)
    seq = G.cv_batch(md, _COSTS[cname](), x, y, cvset)
    knobs("GPR_CV_BATCH", 1)
    bat = G.cv_batch(md, _COSTS[cname](), x, y, cvset)
    np.testing.assert_allclose(bat, seq, rtol=1e-9, atol=0)
    knobs("GPR_CV_BATCH_GB", 1e-9)
    one = G.cv_batch(md, _COSTS[cname](), x, y, cvset)
    np.testing.assert_array_equal(one, bat)
    want = O.cv_batch(["SE", "WN"], hp, cname, x, y, cvset)
    np.testing.assert_allclose(bat, want, rtol=1e-8, atol=0)


@pytest.mark.gpu
@pytest.mark.parametrize("cname", ["MSE", "Mahalanobis"])
def test_cv_batch_context_nb64(cname):
    """A context with 64-wide inner blocks (gpr_set_block) still takes the batched launch (its
    tiles are 128 wide whatever the context's nb) and gives the oracle's losses; the per-fold
    path of the same context agrees."""
    d, n, k = 3, 300, 25
    x, y = _data(d, n, 31)
    hp = O.default_hp(["SE", "WN"], d, length=2.0)
    cvset = G.kfoldcv(n, k, rng=np.random.default_rng(6))
    ctx = G.Context(0, nb=64)
    md = G.GPRModel(G.SquaredExp() + G.WhiteNoise(), hp, x, y, ctx=ctx)
    bat = G.cv_batch(md, _COSTS[cname](), x, y, cvset)
    ctx.set_knob("GPR_CV_BATCH", 0)
    seq = G.cv_batch(md, _COSTS[cname](), x, y, cvset)
    ctx.close()
    want = O.cv_batch(["SE", "WN"], hp, cname, x, y, cvset)
    np.testing.assert_allclose(bat, want, rtol=1e-8, atol=0)
    np.testing.assert_allclose(seq, bat, rtol=1e-9, atol=0)
