"""numpy emulation of the kernel's level-0 repair (qppvm_kernel.hip: level0_repair) for
debugging single instances on CPU. Not test infrastructure for parity (the oracle is)."""
import sys

import numpy as np

sys.path.insert(0, ".")
import oracle  # noqa: E402
from qppvm_amd.problem import QPPVMProblem  # noqa: E402
from qppvm_amd.synth import qppvm_instances  # noqa: E402


def rr_chol(G, kact, tol=1e-12):
    K = G.shape[0]
    L = np.tril(G.copy())
    il = np.zeros(K)
    dmx = np.max(np.diag(G))
    for c in range(K):
        dd = L[c, c] - np.dot(L[c, :c], L[c, :c])
        ind = c < kact and dd > tol * dmx
        ic = 1 / np.sqrt(dd) if ind else 0.0
        il[c] = ic
        L[c, c] = dd * ic
        for r in range(c + 1, K):
            L[r, c] = (L[r, c] - np.dot(L[r, :c], L[c, :c])) * ic
    return L, il


class PivChol:
    """Kernel's PivChol<K>: diagonal-pivoted Cholesky of a PSD Gram + min-norm LS weights."""

    def __init__(self, G, m, tol=1e-12):
        K = G.shape[0]
        self.K, self.m = K, m
        d = np.array([G[i, i] if i < m else 0.0 for i in range(K)])
        dmx = d.max()
        used = np.array([i >= m for i in range(K)])
        Lo = np.zeros((K, K))
        Lp = np.zeros((K, K))
        piv = np.zeros(K, int)
        k = 0
        for c in range(K):
            cand = np.where(~used, d, -1.0)
            p = int(np.argmax(cand))
            if not (cand[p] > tol * dmx):
                break
            used[p] = True
            piv[c] = p
            k = c + 1
            lpp = np.sqrt(cand[p])
            rp = Lo[p].copy()
            for i in range(K):
                if not used[i]:
                    Lo[i, c] = (G[i, p] - Lo[i, :c] @ rp[:c]) / lpp
                    d[i] -= Lo[i, c] ** 2
            Lo[p, c] = lpp
            Lp[c, :c] = rp[:c]
            Lp[c, c] = lpp
        self.k, self.piv, self.Lo, self.Lp, self.used = k, piv, Lo, Lp, used

    def solve(self, r):
        K, k, m = self.K, self.k, self.m
        Lp, Lo, piv = self.Lp, self.Lo, self.piv
        rP = np.array([r[piv[c]] if c < k else 0.0 for c in range(K)])
        H = np.eye(K)
        rh = rP.copy()
        pivset = set(piv[:k])
        for i in range(m):
            if i in pivset:
                continue
            ci = np.zeros(K)
            for c in range(k - 1, -1, -1):
                ci[c] = (Lo[i, c] - Lp[c + 1:k, c] @ ci[c + 1:k]) / Lp[c, c]
            H += np.outer(ci, ci)
            rh += ci * r[i]
        sv = np.linalg.solve(H, rh)
        t = np.zeros(K)
        for c in range(k):
            t[c] = (sv[c] - Lp[c, :c] @ t[:c]) / Lp[c, c]
        ws = np.zeros(K)
        for c in range(k - 1, -1, -1):
            ws[c] = (t[c] - Lp[c + 1:k, c] @ ws[c + 1:k]) / Lp[c, c]
        w = np.zeros(K)
        for c in range(k):
            w[piv[c]] = ws[c]
        return w


def bvls(A, b, lo, hi):  # A: m x n (columns a_i)
    m, n = A.shape
    x = np.clip(0, lo, hi)
    st = np.zeros(n, int)
    st[lo == hi] = -1
    ex = np.zeros(n, bool)
    wt = 1e-11 * max(1, np.abs(A.T @ b).max())
    freed, it = -1, 0
    while True:
        while True:
            it += 1
            fr = st == 0
            if not fr.any():
                break
            r = b - A[:, ~fr] @ x[~fr]
            Gm = A[:, fr] @ A[:, fr].T
            w = PivChol(Gm, m).solve(r)
            z = np.where(fr, A.T @ w, 0)
            al = np.full(n, np.inf)
            for i in np.where(fr)[0]:
                step = z[i] - x[i]
                if z[i] < lo[i] and step < 0: al[i] = (lo[i] - x[i]) / step
                elif z[i] > hi[i] and step > 0: al[i] = (hi[i] - x[i]) / step
                if not al[i] < 1: al[i] = np.inf
            jb = int(np.argmin(al))
            if al[jb] == np.inf:
                x[fr] = z[fr]; freed = -1; ex[:] = False; break
            alpha = max(al[jb], 0)
            if jb == freed and alpha == 0:
                ex[jb] = True; st[jb] = -1 if z[jb] < lo[jb] else 1; x[jb] = lo[jb] if st[jb] < 0 else hi[jb]; break
            ex[:] = False
            for i in np.where(fr)[0]:
                x[i] += alpha * (z[i] - x[i])
                if i == jb: st[i] = -1 if z[i] < lo[i] else 1
                elif x[i] <= lo[i] + 1e-14 * max(1, abs(lo[i])) and z[i] < lo[i]: st[i] = -1
                elif x[i] >= hi[i] - 1e-14 * max(1, abs(hi[i])) and z[i] > hi[i]: st[i] = 1
                if st[i] == -1: x[i] = lo[i]
                if st[i] == 1: x[i] = hi[i]
            freed = -1
        Ax = A @ x
        w = A.T @ (b - Ax)
        wt = 1e-11 * max(1, np.abs(A.T @ b).max(), np.abs(A.T @ Ax).max())
        v = np.where((st != 0) & ~ex & (lo != hi), np.where(st < 0, w, -w), -np.inf)
        best = int(np.argmax(v))
        if not v[best] > wt:
            return x, it
        st[best] = 0; freed = best


def main(n, mask, tau_max, seed, B, idx):
    prob = QPPVMProblem(n=n, tau_max=tau_max, row_mask=mask)
    inp = qppvm_instances(prob, B, seed=seed)
    one = {k: v[idx:idx + 1] for k, v in inp.items()}
    asm = oracle.assemble(prob, one, 0)
    M = one["M"][0]; h = one["h"][0]
    sel = [t * 6 + r for t in range(2) for r in range(6) if (mask[t] >> r) & 1]
    G = one["J"][0].reshape(-1, n)[sel]
    A0 = asm["A0"]; b0 = asm["b0"]
    lo = prob.tau_min - h; hi = prob.tau_max - h
    x, it = bvls(A0, b0, lo, hi)
    ys = A0 @ x
    tau_r, y0_r, st_r, _ = oracle.qppvm_one(prob, one, 0)
    return locals()


if __name__ == "__main__":
    worst = 0
    for (n, mask, tm, seed) in [(7, (0x3F, 0x3F), 1e7, 307), (3, (7, 7), 1e7, 303), (30, (7, 7), 30.0, 330),
                                (30, (0x3F, 0x3F), 10.0, 330), (39, (7, 7), 30.0, 339)]:
        for idx in range(24):
            d = main(n, mask, tm, seed, 24, idx)
            e = np.abs(d["ys"] - d["y0_r"]).max() / max(1, np.abs(d["y0_r"]).max())
            worst = max(worst, e)
            if e > 1e-8:
                print("BAD", n, mask, tm, idx, e)
    print("worst rel y* err", worst)
