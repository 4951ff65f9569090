"""Goldfarb-Idnani dual active set in QR form (design tool and numpy statement of the contact kernel's
robust fallback, qppvm_amd/csrc/qr_gi.h): the least-distance problem in the H-scaled variables
w = L^T (x - x0), H = L L^T, with an explicit orthonormal basis Q of the active scaled normals
n~ = L^-1 a and R (N~_A = Q R). The dependency test of a row is the norm of its scaled normal's
component outside span(Q), formed by two Gram-Schmidt passes -- accurate to roundoff of |n~|, not of
|n~|^2 as the Schur complement of Gamma = A H^-1 A^T is (the constraint-space loop's dual_gi.h: with
the contact form's 1 / eps_f force scale a dependent row's complement there is ~1e-7 against Gamma_pp
~1e8). Activities are recomputed from x every outer step.

    solve(H, g, A, lo, hi, kind) -> (status, x, iters)
      A [m][nx] rows, lo / hi per row (lo == hi: an equality), kind 0 off / 1 equality / 2 inequality
"""
import numpy as np

INF = 1e300


def solve(H, g, A, lo, hi, kind, maxit=None, dep=1e-14, trace=False):
    nx = H.shape[0]
    m = A.shape[0]
    L = np.linalg.cholesky(H)
    x = -np.linalg.solve(H, g)
    Nt = np.linalg.solve(L, A.T).T          # scaled normals, rows
    an2 = (A * A).sum(axis=1)               # |a|^2 (the oracle's dependency scale)
    Q = np.zeros((nx, 0))
    R = np.zeros((0, 0))
    act, sgn, lam = [], [], []
    onact = np.zeros(m, bool)
    skipped = np.zeros(m, bool)
    if maxit is None:
        maxit = 10 * (nx + m) + 50
    it = 0
    eqs = [j for j in range(m) if kind[j] == 1 or (kind[j] == 2 and lo[j] == hi[j])]
    while True:
        s = A @ x
        # next row: equalities first (in order), then the most violated inequality side
        p, sg, best = -1, 1.0, 0.0
        for j in eqs:
            if not onact[j] and not skipped[j]:
                p, sg = j, (1.0 if lo[j] - s[j] >= 0 else -1.0)
                break
        if p < 0:
            for j in range(m):
                if kind[j] != 2 or onact[j] or skipped[j]:
                    continue
                fin = lambda v: abs(v) if abs(v) < 1e299 else 0.0  # noqa: E731
                tol = 1e-10 * max(1.0, abs(s[j]), fin(lo[j]), fin(hi[j]))
                nn = np.sqrt(an2[j])
                if lo[j] - s[j] > tol and (lo[j] - s[j]) / nn > best:
                    best, p, sg = (lo[j] - s[j]) / nn, j, 1.0
                if s[j] - hi[j] > tol and (s[j] - hi[j]) / nn > best:
                    best, p, sg = (s[j] - hi[j]) / nn, j, -1.0
        if p < 0:
            return 0, x, it
        bnd = lo[p] if sg > 0 else hi[p]
        ntp = sg * Nt[p]
        lamp = 0.0
        while True:
            it += 1
            if it > maxit:
                return 1, x, it
            k = len(act)
            u = Q.T @ ntp
            w = ntp - Q @ u
            u2 = Q.T @ w
            w = w - Q @ u2
            u = u + u2
            zz = float(w @ w)
            r = np.linalg.solve(R, u) if k else np.zeros(0)
            slack = sg * (bnd - A[p] @ x)
            t1, blk = INF, -1
            rmax = np.abs(r).max() if k else 0.0
            for q in range(k):
                if not (lo[act[q]] == hi[act[q]] or kind[act[q]] == 1) and r[q] > 1e-12 * max(rmax, 1e-300):
                    if lam[q] / r[q] < t1:
                        t1, blk = lam[q] / r[q], q
            indep = zz > dep * an2[p] and k < nx
            t2 = slack / zz if indep else INF
            if trace:
                print(f"  it {it}: p={p} sg={sg:+.0f} k={k} slack={slack:.3e} zz={zz:.3e} |a|^2={an2[p]:.3e} "
                      f"t1={t1:.3e} t2={t2:.3e}")
            if t1 >= INF and t2 >= INF:
                # dependent and nothing to drop: a violation at the roundoff of the rows it depends on is
                # not an inconsistency (the oracle's rule, wbq_oracle_contact.c wbq_ref_dual_qp): skip it
                ps = np.abs(A[p] * x).sum()
                if lamp == 0.0 and slack <= 1e-9 * (1.0 + abs(bnd) + ps):
                    skipped[p] = True
                    break
                return 2, x, it
            t = min(t1, t2)
            if indep:  # a partial (t1) or full (t2) primal step; a dependent row moves the multipliers only
                x = x + t * np.linalg.solve(L.T, w)
            lam = [lam[q] - t * r[q] for q in range(k)]
            lamp += t
            if t2 <= t1:
                Q = np.hstack([Q, (w / np.sqrt(zz))[:, None]])
                Rn = np.zeros((k + 1, k + 1))
                Rn[:k, :k] = R
                Rn[:k, k] = u
                Rn[k, k] = np.sqrt(zz)
                R = Rn
                act.append(p)
                sgn.append(sg)
                lam.append(lamp)
                onact[p] = True
                break
            # drop slot blk: delete its column of R, restore the triangle by Givens rotations on rows
            # blk.. of R and the same columns of Q
            onact[act[blk]] = False
            del act[blk], sgn[blk], lam[blk]
            R = np.delete(R, blk, axis=1)
            for q in range(blk, k - 1):
                a_, b_ = R[q, q], R[q + 1, q]
                h = np.hypot(a_, b_)
                c, s_ = (a_ / h, b_ / h) if h > 0 else (1.0, 0.0)
                R[[q, q + 1], :] = np.array([[c, s_], [-s_, c]]) @ R[[q, q + 1], :]
                Q[:, [q, q + 1]] = Q[:, [q, q + 1]] @ np.array([[c, -s_], [s_, c]])
            R = R[:k - 1, :]
            Q = Q[:, :k - 1]


def solve_metric(Hinv, x0, A, lo, hi, kind, maxit=None, dep=1e-14, trace=False):
    """The same loop in the H^-1 metric with unscaled vectors (the form the contact kernel runs, where
    H^-1 A^T is at hand from its elimination and no factor of H is): the basis covectors v_q are
    H^-1-orthonormal and carried with z_q = H^-1 v_q; a row's residual w = a_p - sum u_q v_q and
    H^-1 w = H^-1 a_p - sum u_q z_q give zz = w . H^-1 w and the primal direction H^-1 w."""
    nx = A.shape[1]
    m = A.shape[0]
    x = x0.copy()
    HA = (Hinv @ A.T).T                     # H^-1 a_j, rows
    an2 = (A * A).sum(axis=1)
    V = np.zeros((0, nx))
    Z = np.zeros((0, nx))
    R = np.zeros((0, 0))
    act, lam = [], []
    onact = np.zeros(m, bool)
    skipped = np.zeros(m, bool)
    if maxit is None:
        maxit = 10 * (nx + m) + 50
    it = 0
    eqs = [j for j in range(m) if kind[j] == 1 or (kind[j] == 2 and lo[j] == hi[j])]
    sgn = []

    def refine(x):
        # x on the active rows exactly, inside range(H^-1 A_A^T): A_A H^-1 A_A^T = R^T R, so
        # dx = H^-1 A_A^T (R^T R)^-1 r_A = Z^T R^-T r_A (two passes)
        for _ in range(2):
            if not act:
                return x
            bA = np.array([lo[j] if sg_ > 0 else hi[j] for j, sg_ in zip(act, sgn)])
            rA = np.array(sgn) * (bA - A[act] @ x)
            y = np.linalg.solve(R.T, rA)
            x = x + y @ Z
        return x

    while True:
        x = refine(x)
        s = A @ x
        p, sg, best = -1, 1.0, 0.0
        for j in eqs:
            if not onact[j] and not skipped[j]:
                p, sg = j, (1.0 if lo[j] - s[j] >= 0 else -1.0)
                break
        if p < 0:
            for j in range(m):
                if kind[j] != 2 or onact[j] or skipped[j]:
                    continue
                fin = lambda v: abs(v) if abs(v) < 1e299 else 0.0  # noqa: E731
                tol = 1e-10 * max(1.0, abs(s[j]), fin(lo[j]), fin(hi[j]))
                nn = np.sqrt(an2[j])
                if lo[j] - s[j] > tol and (lo[j] - s[j]) / nn > best:
                    best, p, sg = (lo[j] - s[j]) / nn, j, 1.0
                if s[j] - hi[j] > tol and (s[j] - hi[j]) / nn > best:
                    best, p, sg = (s[j] - hi[j]) / nn, j, -1.0
        if p < 0:
            return 0, x, it
        bnd = lo[p] if sg > 0 else hi[p]
        ap, hp = sg * A[p], sg * HA[p]
        lamp = 0.0
        while True:
            it += 1
            if it > maxit:
                return 1, x, it
            k = len(act)
            u = Z @ ap
            w, hw = ap - u @ V, hp - u @ Z
            u2 = Z @ w
            w, hw = w - u2 @ V, hw - u2 @ Z
            u = u + u2
            zz = float(w @ hw)
            r = np.linalg.solve(R, u) if k else np.zeros(0)
            slack = sg * (bnd - A[p] @ x)
            t1, blk = INF, -1
            rmax = np.abs(r).max() if k else 0.0
            for q in range(k):
                if not (lo[act[q]] == hi[act[q]] or kind[act[q]] == 1) and r[q] > 1e-12 * max(rmax, 1e-300):
                    if lam[q] / r[q] < t1:
                        t1, blk = lam[q] / r[q], q
            indep = zz > dep * an2[p] and k < nx
            t2 = slack / zz if indep else INF
            if t1 >= INF and t2 >= INF:
                ps = np.abs(A[p] * x).sum()
                if lamp == 0.0 and slack <= 1e-9 * (1.0 + abs(bnd) + ps):
                    skipped[p] = True
                    break
                return 2, x, it
            t = min(t1, t2)
            if indep:
                x = x + t * hw
            lam = [lam[q] - t * r[q] for q in range(k)]
            lamp += t
            if t2 <= t1:
                nz = np.sqrt(zz)
                V = np.vstack([V, w / nz])
                Z = np.vstack([Z, hw / nz])
                Rn = np.zeros((k + 1, k + 1))
                Rn[:k, :k] = R
                Rn[:k, k] = u
                Rn[k, k] = nz
                R = Rn
                act.append(p)
                sgn.append(sg)
                lam.append(lamp)
                onact[p] = True
                break
            onact[act[blk]] = False
            del act[blk], lam[blk], sgn[blk]
            R = np.delete(R, blk, axis=1)
            for q in range(blk, k - 1):
                a_, b_ = R[q, q], R[q + 1, q]
                h = np.hypot(a_, b_)
                c, s_ = (a_ / h, b_ / h) if h > 0 else (1.0, 0.0)
                G = np.array([[c, s_], [-s_, c]])
                R[[q, q + 1], :] = G @ R[[q, q + 1], :]
                V[[q, q + 1], :] = G @ V[[q, q + 1], :]
                Z[[q, q + 1], :] = G @ Z[[q, q + 1], :]
            R = R[:k - 1, :]
            V = V[:k - 1]
            Z = Z[:k - 1]
