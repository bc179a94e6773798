"""NumPy emulation of csrc/eigen.hip's block-Jacobi (same ordering, thresholds, rotation
formulas, R accumulation and per-round transforms), to study its accuracy on the CPU:
eigenvalue error in units of n eps ||A|| with and without the Newton-Schulz step on R.
Not a test and not the product path.   python tools/eig_emulate.py [n] [inner]
"""
import sys

import numpy as np

EB, ES = 32, 64


def circle(m, r, k):
    mm = m - 1
    L = lambda i: (i + r) % mm + 1  # noqa: E731
    return (0, L(0)) if k == 0 else (L(k), L(mm - k))


def rows(I, J):
    return np.r_[np.arange(EB * I, EB * I + EB), np.arange(EB * J, EB * J + EB)]


def subproblem(S, max_inner, reorth):
    S = S.copy()
    R = np.eye(ES)
    total = 0
    for _ in range(max_inner):
        rot = 0
        for step in range(ES - 1):
            cs = []
            for t in range(ES // 2):
                p, q = circle(ES, step, t)
                p, q = min(p, q), max(p, q)
                app, aqq, apq = S[p, p], S[q, q], S[p, q]
                c, s = 1.0, 0.0
                if apq != 0.0 and abs(apq) > 1e-15 * np.sqrt(abs(app * aqq)):
                    th = (aqq - app) / (2.0 * apq)
                    tt = (1.0 if th >= 0 else -1.0) / (abs(th) + np.sqrt(1.0 + th * th))
                    if abs(tt) >= 1e-17:
                        c = 1.0 / np.sqrt(1.0 + tt * tt)
                        s = tt * c
                        rot += 1
                cs.append((p, q, c, s))
            for p, q, c, s in cs:
                if s == 0.0:
                    continue
                sp, sq = S[p, :].copy(), S[q, :].copy()
                S[p, :], S[q, :] = c * sp - s * sq, s * sp + c * sq
            for p, q, c, s in cs:
                if s == 0.0:
                    continue
                sp, sq = S[:, p].copy(), S[:, q].copy()
                S[:, p], S[:, q] = c * sp - s * sq, s * sp + c * sq
                rp, rq = R[:, p].copy(), R[:, q].copy()
                R[:, p], R[:, q] = c * rp - s * rq, s * rp + c * rq
        total += rot
        if rot == 0:
            break
    if reorth and total:
        R = 1.5 * R - 0.5 * (R @ (R.T @ R))
    return R, total


def block_jacobi(A, max_inner=8, reorth=True, max_sweeps=60):
    n = A.shape[0]
    n2 = (n + ES - 1) // ES * ES
    W = np.zeros((n2, n2))
    W[:n, :n] = A
    nb = n2 // EB
    for sweep in range(max_sweeps):
        rotations = 0
        for r in range(nb - 1):
            Rs, P = [], []
            for k in range(nb // 2):
                idx = rows(*circle(nb, r, k))
                R, cnt = subproblem(W[np.ix_(idx, idx)], max_inner, reorth)
                Rs.append(R)
                P.append(idx)
                rotations += cnt
            Wn = W.copy()
            for k in range(nb // 2):
                for l in range(k, nb // 2):
                    T = Rs[k].T @ (W[np.ix_(P[k], P[l])] @ Rs[l])
                    if k == l:
                        T = np.triu(T) + np.triu(T, 1).T
                    Wn[np.ix_(P[k], P[l])] = T
                    Wn[np.ix_(P[l], P[k])] = T.T
            W = Wn
        if rotations == 0:
            return np.diag(W)[:n], sweep + 1
    return np.diag(W)[:n], -1


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 129
    inner = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    X = np.random.default_rng(n).standard_normal((n, n))
    A = (X + X.T) / 2
    ref = np.linalg.eigvalsh(A)
    unit = n * np.finfo(float).eps * np.abs(ref).max()
    for reorth in (False, True):
        lam, sw = block_jacobi(A, inner, reorth)
        print(f"n={n} inner={inner} reorth={reorth}: sweeps {sw}, eig err "
              f"{np.abs(np.sort(lam) - ref).max() / unit:.2f} n eps |A|")


if __name__ == "__main__":
    main()
