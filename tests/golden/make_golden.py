"""Generate the seeded golden fixtures under tests/golden/ (SURVEY.md 8c).

The reference (Julia, with an unfetchable unregistered dependency) cannot run in this
container and its own test-suite holds no golden data, so these vectors come from the
fp64 NumPy oracle (oracle/gpr_oracle.py), which is itself pinned by the reference's
known-answer and identity tests (tests/test_oracle.py).  They freeze inputs and expected
outputs so that (1) the oracle cannot drift silently (tests/test_golden.py recomputes and
compares) and (2) the HIP path is checked against fixed data on the GPU box without the
oracle in the loop (tests/test_golden.py, gpu-marked tests).

Run from the repository root:  python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import gpr_oracle as O  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))

KERNELS = {"SE": ["SE"], "SE+WN": ["SE", "WN"], "SE+SE": ["SE", "SE"],
           "SE+SE+WN": ["SE", "SE", "WN"]}
SIZES = [(64, 2, 16), (512, 2, 128), (256, 8, 64)]  # (N, d, np)


def hp_for(kinds, d):
    """Distinct per-part values so that composition order matters (src/compose_covar.jl)."""
    hp, nse = [], 0
    base = 3.0 * np.sqrt(8.0 / d)
    for k in kinds:
        if k == "SE":
            sig = 1.0 if nse == 0 else 0.7
            ls = base * (1.0 if nse == 0 else 0.6) * (1.0 + 0.05 * np.arange(d))
            hp += [sig] + list(ls)
            nse += 1
        else:
            hp += [0.1]
    return np.array(hp)


def case(name, kinds, n, d, npred):
    x, y, xp = O.synthetic(d, n, npred)
    hp = hp_for(kinds, d)
    K = O.kernel(kinds, hp, x, None)
    U = O.chol_upper(K)
    alpha = O.cho_solve_upper(U, y)
    out = dict(kinds=np.array(kinds), x=x, y=y, xp=xp, hp=hp,
               alpha=alpha, mll=np.array(O.mll_value(U, y, alpha)),
               grad=O.mll_grad(kinds, hp, x, y),
               grad_log=O.mll_grad(kinds, hp, x, y, log_scale=True),
               min_diag_u2=np.array(np.min(np.diag(U)) ** 2))
    mu, var = O.predict(kinds, hp, x, y, xp, diagonal_var=True)
    out.update(mu=mu, var_diag=var)
    if npred <= 128:
        _, S = O.predict(kinds, hp, x, y, xp, diagonal_var=False)
        out["var_full"] = S
    if n <= 64:
        out.update(K=K, U=U)
    np.savez_compressed(os.path.join(OUT, f"{name}.npz"), **out)


def split_case():
    kinds = ["SE", "WN"]
    ns, ne, nq, d = 256, 10, 30, 3
    x, y, _ = O.synthetic(d, ns)
    xe = np.random.default_rng(2).random((d, ne))
    xq = np.random.default_rng(3).random((d, nq))
    hp = hp_for(kinds, d)
    mu, var = O.split_predict(kinds, hp, x, y, xe, xq)             # var_range default 1:3
    _, var_full = O.split_predict(kinds, hp, x, y, xe, xq, var_range=(1, ne))
    np.savez_compressed(os.path.join(OUT, "split_SE+WN_256_10_30_3.npz"), kinds=np.array(kinds),
                        x=x, y=y, xe=xe, xq=xq, hp=hp, mu=mu, var_default=var,
                        var_full_range=var_full)


def main():
    for kname, kinds in KERNELS.items():
        for (n, d, npred) in SIZES:
            case(f"gp_{kname}_{n}_{d}_{npred}", kinds, n, d, npred)
    split_case()
    print("fixtures written to", OUT)


if __name__ == "__main__":
    main()
