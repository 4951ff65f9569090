"""Step-faithful numpy emulation of the n <= 32 constraint-space dual active set (round 6,
qppvm_amd/csrc/cs_gi.h): the QPPVM level-1 least-distance problem

    min 0.5 ||u - u_hat||^2   s.t.  G u = b0,   lo <= M u <= hi

carried in the activities s = M u with Gamma = M P M (P = I - Q1^T Q1 the projector onto null(G)),
columns of Gamma formed on demand (w = P m_p, c = M w), the active-set Gram as T = L^-1 (packed
rows), a drop by re-appending the later slots, the warm batch, the final rebuild of u from the
multipliers with refinement, and the re-check. A design / debugging tool, not a test oracle: the
result is checked against the problem's KKT conditions.

    python scripts/emulate_cs_gi.py [--seed S] [--count C] [--frac F] [--warm] [--trace]
"""
import argparse

import numpy as np

INF = 1e300
KM = 22


def make_problem(rng, n=30, m0=6, frac=0.2, cond=1e3):
    Q, _ = np.linalg.qr(rng.standard_normal((n, n)))
    ev = np.exp(rng.uniform(np.log(10.0 / cond), np.log(10.0), n))
    M = (Q * ev) @ Q.T
    M = 0.5 * (M + M.T)
    G = rng.standard_normal((m0, n))
    uh = rng.standard_normal(n)
    b0 = rng.standard_normal(m0)
    # u0: the equality-constrained optimum
    Gp = np.linalg.pinv(G)
    u0 = uh + Gp @ (b0 - G @ uh)
    x0 = M @ u0
    width = np.abs(rng.standard_normal(n)) * np.abs(x0).mean()
    lo = x0 - width
    hi = x0 + width
    pick = rng.random(n) < frac
    side = rng.random(n) < 0.5
    shift = (0.2 + rng.random(n)) * width
    lo = np.where(pick & side, x0 + shift * 0.5 + 1e-3, lo)
    hi = np.where(pick & ~side, x0 - shift * 0.5 - 1e-3, hi)
    hi = np.maximum(hi, lo + 1e-3)
    return dict(M=M, G=G, uh=uh, b0=b0, u0=u0, lo=lo, hi=hi)


def q1_of(G):
    # Q1 rows: orthonormal basis of G's rows (the fast path's G^T L^-T)
    L = np.linalg.cholesky(G @ G.T)
    return np.linalg.solve(L, G)


class Slots:
    def __init__(self, n):
        self.k = 0
        self.act = np.zeros(KM, int)
        self.sg = np.ones(KM)
        self.lam = np.zeros(KM)
        self.aeq = np.zeros(KM, bool)
        self.T = np.zeros((KM, KM))   # lower triangular, T = L^-1 of the Gram of the active set
        self.GA = np.zeros((n, KM))   # GA[i, a] = Gamma[i, act_a]


def cs_solve(P, wsg=None, maxit=200, trace=False):
    M, u0, lo, hi = P["M"], P["u0"], P["lo"], P["hi"]
    n = M.shape[0]
    Q1 = q1_of(P["G"])
    dim = n - Q1.shape[0]
    nrm = np.linalg.norm(M, axis=1)
    eqb = lo == hi
    st = Slots(n)
    s = M @ u0
    iters, status, infeasible = 0, 0, False

    def ccol(p):
        mp = M[:, p]
        w = mp - Q1.T @ (Q1 @ mp)
        return M @ w, w @ w

    def append(p, sg, c, cpp):
        """T row k from the Gram column; returns d2 (the Schur complement)"""
        k = st.k
        v = st.sg[:k] * sg * c[st.act[:k]]
        l = st.T[:k, :k] @ v
        r = st.T[:k, :k].T @ l
        d2 = cpp - l @ l
        return v, l, r, d2

    def rebuild():
        k = st.k
        rho = np.zeros(n)
        rho[st.act[:k]] = st.sg[:k] * st.lam[:k]
        y = M @ rho
        u = u0 + y - Q1.T @ (Q1 @ y)
        return u, M @ u

    def refine(x):
        k = st.k
        bnd = np.where(st.sg[:k] > 0, lo[st.act[:k]], -hi[st.act[:k]])
        res = bnd - st.sg[:k] * x[st.act[:k]]
        T = st.T[:k, :k]
        st.lam[:k] += T.T @ (T @ res)
        return np.abs(res).max() if k else 0.0

    dirty = True
    onact = np.zeros(n, bool)
    # ---- warm batch
    if wsg is not None and np.any(wsg != 0):
        W = np.nonzero(wsg)[0]
        ok = len(W) <= KM and len(W) <= dim
        if ok:
            for j in W:
                c, cpp = ccol(j)
                v, l, r, d2 = append(j, wsg[j], c, cpp)
                if not d2 > 1e-14 * cpp:
                    ok = False
                    break
                k = st.k
                d = np.sqrt(d2)
                st.T[k, :k] = -r / d
                st.T[k, k] = 1.0 / d
                st.GA[:, k] = c
                st.act[k], st.sg[k], st.lam[k], st.aeq[k] = j, wsg[j], 0.0, eqb[j]
                st.k += 1
        if ok:
            k = st.k
            bnd = np.where(st.sg[:k] > 0, lo[st.act[:k]], -hi[st.act[:k]])
            res = bnd - st.sg[:k] * s[st.act[:k]]
            T = st.T[:k, :k]
            lam = T.T @ (T @ res)
            lmx = np.abs(lam).max()
            if np.any((lam < -1e-12 * (1 + lmx)) & ~st.aeq[:k]):
                ok = False
            else:
                st.lam[:k] = np.where(st.aeq[:k], lam, np.maximum(lam, 0.0))
                s = s + st.GA[:, :k] @ (st.sg[:k] * lam)
                onact[st.act[:k]] = True
                iters += 1
        if not ok:
            st.k = 0
    rounds = 0
    need_select, recheck = True, False
    have_col = False
    p = sgp = bnd = lamp = None
    peq = False
    while True:
        if need_select:
            tol = 1e-10 * np.maximum(1.0, np.maximum(np.abs(s), np.maximum(np.abs(lo), np.abs(hi))))
            viol = np.maximum(lo - s, s - hi)
            v = np.where((viol > tol) & ~onact, viol / nrm, -1.0)
            pi = int(np.argmax(v))
            if not v[pi] > 0 or recheck:
                recheck = False
                if not dirty:
                    break
                rounds += 1
                if rounds > 8:
                    infeasible = True  # hand-off
                    break
                u, x = rebuild()
                if st.k:
                    for it in range(3):
                        r = refine(x)
                        u, x = rebuild()
                        if it >= 1 and r <= 1e-14 * (1 + np.abs(x).max()):
                            break
                s = x.copy()
                dirty = False
                if trace:
                    print(f"  rebuild round {rounds}: k={st.k}")
                continue
            p = pi
            sgp = 1.0 if lo[p] - s[p] > s[p] - hi[p] else -1.0
            bnd = lo[p] if sgp > 0 else hi[p]
            peq = eqb[p]
            lamp = 0.0
            have_col = False
        if not have_col:
            c, cpp = ccol(p)
            have_col = True
        k = st.k
        v, l, r, d2 = append(p, sgp, c, cpp)
        ds = sgp * c - st.GA[:, :k] @ (st.sg[:k] * r)
        zz = sgp * ds[p]
        slack = sgp * (s[p] - bnd)
        rmax = np.abs(r).max() if k else 0.0
        cand = np.where((~st.aeq[:k]) & (r > 1e-13 * rmax), st.lam[:k] / np.where(r != 0, r, 1), INF)
        blk = int(np.argmin(cand)) if k else 0
        t1 = cand[blk] if k else INF
        t2 = -slack / zz if (k < dim and d2 > 1e-14 * cpp and zz > 0) else INF
        if t1 >= INF and t2 >= INF:
            if dirty:
                recheck = True
                need_select = True
                continue
            infeasible = True
            break
        if t2 <= t1 and k >= KM:
            infeasible = True  # storage: hand-off
            break
        dirty = True
        t = min(t1, t2)
        s = s + t * ds
        st.lam[:k] -= t * r
        lamp += t
        iters += 1
        if trace:
            print(f"  it {iters}: p={p} sg={sgp:+.0f} k={k} t1={t1:.3e} t2={t2:.3e} d2={d2:.3e}")
        if t2 <= t1:
            d = np.sqrt(d2)
            st.T[k, :k] = -r / d
            st.T[k, k] = 1.0 / d
            st.T[k, k + 1:] = 0
            st.GA[:, k] = c
            st.act[k], st.sg[k], st.lam[k], st.aeq[k] = p, sgp, lamp, peq
            st.k += 1
            onact[p] = True
            need_select = True
        else:
            cdrop = blk
            onact[st.act[cdrop]] = False
            for arr in (st.act, st.sg, st.lam, st.aeq):
                arr[cdrop:k - 1] = arr[cdrop + 1:k]
            st.GA[:, cdrop:k - 1] = st.GA[:, cdrop + 1:k]
            st.k -= 1
            # re-append slots cdrop.. (rows of T before cdrop stand)
            for a2 in range(cdrop, st.k):
                ca = st.GA[:, a2]
                va = st.sg[:a2] * st.sg[a2] * ca[st.act[:a2]]
                la = st.T[:a2, :a2] @ va
                ra = st.T[:a2, :a2].T @ la
                e2 = ca[st.act[a2]] - la @ la
                d = np.sqrt(max(e2, 1e-300))
                st.T[a2, :a2] = -ra / d
                st.T[a2, a2] = 1.0 / d
                st.T[a2, a2 + 1:] = 0
            need_select = False
        if iters >= maxit:
            status = 1
            break
    u, x = rebuild()
    side = np.zeros(n, int)
    side[st.act[:st.k]] = st.sg[:st.k].astype(int)
    side[eqb] = 0
    return dict(u=u, x=x, status=status, infeasible=infeasible, iters=iters, k=st.k,
                act=st.act[:st.k].copy(), sg=st.sg[:st.k].copy(), lam=st.lam[:st.k].copy(), side=side)


def kkt(P, out):
    """scaled KKT residuals of the result"""
    M, G, uh, lo, hi = P["M"], P["G"], P["uh"], P["lo"], P["hi"]
    u, x = out["u"], out["x"]
    sc = 1 + np.abs(x).max()
    feas = max(np.max(lo - x), np.max(x - hi), 0.0) / sc
    eq = np.abs(G @ u - P["b0"]).max() / (1 + np.abs(P["b0"]).max())
    # stationarity: u - uh = G^T mu + M^T nu, nu_j >= 0 at lower, <= 0 at upper, 0 inactive
    tol = 1e-9 * sc
    atlo = np.abs(x - lo) <= tol
    athi = np.abs(x - hi) <= tol
    on = atlo | athi
    A = np.vstack([G, M[on]])
    sol, *_ = np.linalg.lstsq(A.T, u - uh, rcond=None)
    nu = np.zeros(len(x))
    nu[on] = sol[G.shape[0]:]
    stat = np.abs(A.T @ sol - (u - uh)).max() / (1 + np.abs(u - uh).max())
    nmx = 1 + np.abs(nu).max()
    sign = np.max(np.where(atlo & ~athi, -nu, np.where(athi & ~atlo, nu, 0.0))) / nmx
    return dict(feas=feas, eq=eq, stat=stat, sign=max(sign, 0.0))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--count", type=int, default=200)
    ap.add_argument("--frac", type=float, default=0.2)
    ap.add_argument("--warm", action="store_true")
    ap.add_argument("--trace", action="store_true")
    args = ap.parse_args()
    rng = np.random.default_rng(args.seed)
    worst = dict(feas=0, eq=0, stat=0, sign=0)
    its, hand = [], 0
    for b in range(args.count):
        P = make_problem(rng, frac=args.frac)
        out = cs_solve(P, trace=args.trace)
        if args.warm and not out["infeasible"]:
            # perturb the bounds slightly and warm start from the final set
            P2 = dict(P)
            P2["lo"] = P["lo"] + 1e-3 * rng.standard_normal(P["lo"].shape) * np.isfinite(P["lo"])
            P2["hi"] = np.maximum(P["hi"] + 1e-3 * rng.standard_normal(P["hi"].shape), P2["lo"] + 1e-4)
            cold = cs_solve(P2)
            out = cs_solve(P2, wsg=out["side"], trace=args.trace)
            if not cold["infeasible"] and not out["infeasible"]:
                d = np.abs(cold["x"] - out["x"]).max() / (1 + np.abs(cold["x"]).max())
                assert d < 1e-9, (b, d)
            P = P2
        if out["infeasible"]:
            hand += 1
            # is it really infeasible? an LP feasibility check of G u = b0, lo <= M u <= hi
            from scipy.optimize import linprog
            lp = linprog(np.zeros(len(P["u0"])), A_ub=np.vstack([P["M"], -P["M"]]),
                         b_ub=np.concatenate([P["hi"], -P["lo"]]), A_eq=P["G"], b_eq=P["b0"],
                         bounds=[(None, None)] * len(P["u0"]), method="highs")
            if lp.status == 0:
                print(f"  instance {b}: handed off but feasible (k={out['k']}, iters={out['iters']})")
            continue
        r = kkt(P, out)
        for kk in worst:
            worst[kk] = max(worst[kk], r[kk])
        its.append(out["iters"])
    print(f"instances {args.count}, handed off {hand}, iters mean {np.mean(its):.2f} max {max(its)}")
    print("worst scaled KKT residuals:", {k: f"{v:.2e}" for k, v in worst.items()})


if __name__ == "__main__":
    main()
