"""Step-faithful numpy emulation of the contact kernel's active-set path (design / debugging tool,
not a test oracle): the constraint-space rows in the kernel's compact order, the batched equality
block (Cholesky of Gamma_EE, T = L^-1), and qppvm_amd/csrc/dual_gi.h's loop -- row selection, the
T-factor add / drop re-append, the dependency and rank-cap tests, the x rebuild with two
refinement passes and the final re-check -- in fp64, so a GPU status can be reproduced and
traced on the CPU.

    python scripts/emulate_dual_gi.py n q nc [b ...] [--delta D] [--trace]
      (the torque-row case of tests/test_gpu_contact.py; with instances b, trace those)
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

INF = 1e300
DROP_PIV = float(os.environ.get("DROP_PIV", "1e-9"))


class Problem:
    """The contact problem of instance b in the kernel's compact row order:
    ci < NJ joint rows (ci < 6 dynamic feasibility, an equality; then the torque rows),
    NJ..NJ+5 waist rows (equalities), then the force rows (3 per contact; disabled when the
    contact is inactive)."""

    def __init__(self, prob, inp, b):
        import oracle
        a = oracle.contact_assemble(prob, inp, b)
        n, nc = prob.n, prob.nc
        self.n, self.nc, self.nx = n, nc, n + 3 * nc
        tr = bool(prob.torque_rows)
        NJ = n if tr else 6
        mu = float(getattr(prob, "mu", 0.0))
        nfr = 4 * nc if mu > 0 else 0
        self.mu, self.nfr = mu, nfr
        self.NJ, self.ME = NJ, NJ + 6 + 3 * nc + nfr
        cm = int(inp["cmask"][b])
        rows, lo, hi, kind = [], [], [], []
        for ci in range(NJ):
            if ci < 6:
                rows.append(a["E"][6 + ci]); lo.append(a["e"][6 + ci]); hi.append(a["e"][6 + ci]); kind.append(1)
            else:
                r = 3 * nc + nfr + ci - 6
                rows.append(a["C"][r]); lo.append(a["clo"][r]); hi.append(a["chi"][r]); kind.append(2)
        for r in range(6):
            rows.append(a["E"][r]); lo.append(a["e"][r]); hi.append(a["e"][r]); kind.append(1)
        for f in range(3 * nc):
            on = (cm >> (f // 3)) & 1
            rows.append(a["C"][f]); lo.append(a["clo"][f] if on else -INF); hi.append(a["chi"][f] if on else INF)
            kind.append(2 if on else 0)
        for f in range(nfr):  # friction faces (one-sided), after the force rows as in the kernel
            on = (cm >> (f // 4)) & 1
            rows.append(a["C"][3 * nc + f]); lo.append(-INF); hi.append(0.0 if on else INF)
            kind.append(2 if on else 0)
        self.A = np.array(rows)
        for c in range(nc):  # inactive contacts: their forces appear in no row (the kernel zeroes them)
            if not (cm >> c) & 1:
                self.A[:, n + 3 * c:n + 3 * c + 3] = 0.0
        self.lo, self.hi, self.kind = np.array(lo), np.array(hi), np.array(kind)
        self.H, self.g = a["H"], a["g"]
        Hi = np.linalg.inv(self.H)
        self.Hi = Hi
        self.X = Hi @ self.A.T
        self.G = self.A @ self.X
        self.x0 = -Hi @ self.g
        self.dim = n + 3 * bin(cm & ((1 << nc) - 1)).count("1")
        self.tau_M, self.tau_h, self.Jc, self.cm = inp["M"][b], inp["h"][b], inp["Jc"][b], cm

    def tau(self, x):
        n = self.n
        t = self.tau_M @ x[:n] + self.tau_h
        for c in range(self.nc):
            if (self.cm >> c) & 1:
                t -= self.Jc[c, :3].T @ x[n + 3 * c:n + 3 * c + 3]
        return t


def solve(P, maxit=None, delta=0.0, kdep=1e-14, trace=False, rounds_max=8, wkeep=0x3f):
    """Returns (status, x, iters). delta > 0 adds delta * max diag to the waist rows' Gamma
    diagonal (the waist equalities become J_w qdd - s = b_w with a (1 / 2 delta) ||s||^2 penalty)."""
    G = P.G.copy()
    NJ, ME = P.NJ, P.ME
    m = ME
    wr = np.arange(NJ, NJ + 6)
    if delta > 0:
        G[wr, wr] += delta * max(G[wr, wr].max(), 1.0)
    lo, hi, kind = P.lo, P.hi, P.kind.copy()
    for r in range(6):
        if not (wkeep >> r) & 1:
            kind[NJ + r] = 0  # a waist row implied by the pins (repair)
    s = np.where(kind != 0, P.A @ P.x0, 0.0)
    nrm = np.sqrt(np.maximum(np.diag(G), 1e-300))
    KM = 64
    T = np.zeros((KM, KM))
    act, sgn, lam, aeq = np.zeros(KM, int), np.ones(KM), np.zeros(KM), np.zeros(KM, bool)
    onact = np.zeros(m, bool)
    if maxit is None:
        maxit = 10 * (P.nx + m) + 50
    status, iters, rounds = 0, 0, 0
    # ---- the 12 equality rows in one batch
    E = np.array(list(range(6)) + [NJ + r for r in range(6) if (wkeep >> r) & 1])
    nb = len(E)
    GE = G[np.ix_(E, E)]
    dmx = np.diag(GE).max()
    L = np.zeros((nb, nb))
    g = GE.copy()
    sing = False
    for c in range(nb):
        dcc = g[c, c]
        sing |= not (dcc > 1e-14 * dmx)
        ilc = 1.0 / np.sqrt(dcc) if dcc > 0 else 0.0
        L[c:, c] = g[c:, c] * ilc
        L[c, c] = dcc * ilc
        for j in range(c + 1, nb):
            g[j:, j] -= L[j:, c] * L[j, c]
    Tl = np.zeros((nb, nb))
    for r in range(nb):
        for i in range(nb):
            acc = (1.0 if i == r else 0.0) - sum(L[r, q] * Tl[q, i] for q in range(r))
            Tl[r, i] = acc / L[r, r] if L[r, r] > 0 else 0.0
    T[:nb, :nb] = Tl
    ye = lo[E] - s[E]
    w = Tl @ ye
    lm = Tl.T @ w
    s = s + np.where(kind != 0, G[:, E] @ lm, 0.0)
    act[:nb], sgn[:nb], lam[:nb], aeq[:nb] = E, 1.0, lm, True
    onact[E] = True
    k, iters = nb, 1
    if sing:
        return 3, None, iters
    need_select, dirty, force_rebuild = True, True, False
    just_dropped = False
    cp, sgp, bnd, lamp, peq = 0, 1.0, 0.0, 0.0, False
    x = None
    while True:
        if need_select:
            v = np.full(m, -1.0)
            for j in range(m):
                if kind[j] == 2 and not onact[j]:
                    fin = lambda v: abs(v) if abs(v) < 1e299 else 0.0  # noqa: E731 (one-sided rows)
                    tol = 1e-10 * max(1.0, abs(s[j]), fin(lo[j]), fin(hi[j]))
                    viol = max(lo[j] - s[j], s[j] - hi[j])
                    if viol > tol:
                        v[j] = viol / nrm[j]
            pi = int(np.argmax(v))
            if not v[pi] > 0.0 or force_rebuild:
                force_rebuild = False
                if not dirty:
                    break
                if rounds >= rounds_max:
                    return 1, None, iters
                rounds += 1
                dirty = False
                lo_a, hi_a = lo[act[:k]], hi[act[:k]]
                wv = sgn[:k] * lam[:k]
                x = P.x0 + P.X[:, act[:k]] @ wv
                for ps in range(1, 5):  # dual_gi.h: 2 refinement passes, up to 4 while a row misses
                    a_act = P.A[act[:k]] @ x
                    res = sgn[:k] * (np.where(sgn[:k] > 0, lo_a, hi_a) - a_act)
                    if ps > 2 and (np.abs(res) / (1 + np.abs(a_act))).max() <= 1e-13:
                        break
                    y = T[:k, :k] @ res
                    dl = T[:k, :k].T @ y
                    lam[:k] += dl
                    x = x + P.X[:, act[:k]] @ (sgn[:k] * dl)
                s = np.where(kind != 0, P.A @ x, 0.0)
                miss = 0.0
                for j in range(m):
                    if kind[j] != 0 and onact[j]:
                        miss = max(miss, min(abs(s[j] - lo[j]), abs(s[j] - hi[j])) / (1 + abs(s[j])))
                if trace:
                    print(f"  rebuild round {rounds}: k={k} miss={miss:.3e}")
                if miss > 1e-8:
                    # a nearly dependent row made the factor garbage: drop the slot with the
                    # smallest relative pivot d^2 / Gamma_pp (an implied row: the exact
                    # activities will still meet it) and rebuild, else fail
                    piv = np.array([1.0 / (T[a_, a_] ** 2 * G[act[a_], act[a_]]) for a_ in range(k)])
                    piv[:nb] = np.inf
                    blk = int(np.argmin(piv))
                    if os.environ.get("CLEAN", "1") == "1" and piv[blk] < DROP_PIV:
                        if trace:
                            print(f"  drop near-dependent slot {blk} (row {act[blk]}, pivot {piv[blk]:.2e})")
                        onact[act[blk]] = False
                        act[blk:k - 1], sgn[blk:k - 1], lam[blk:k - 1], aeq[blk:k - 1] = \
                            act[blk + 1:k].copy(), sgn[blk + 1:k].copy(), lam[blk + 1:k].copy(), aeq[blk + 1:k].copy()
                        k -= 1
                        T[blk:, :] = 0.0
                        for a2 in range(blk, k):
                            cq, sq = act[a2], sgn[a2]
                            vv2 = sgn[:a2] * sq * G[act[:a2], cq]
                            l2 = T[:a2, :a2] @ vv2
                            r2 = T[:a2, :a2].T @ l2
                            e2 = G[cq, cq] - l2 @ l2
                            id2 = 1.0 / np.sqrt(e2) if e2 > 0 else 0.0
                            T[a2, :a2] = -r2 * id2
                            T[a2, a2] = id2
                        dirty = True
                        force_rebuild = True
                        continue
                    return 3, x, iters
                continue
            cp = pi
            vl, vh = lo[cp] - s[cp], s[cp] - hi[cp]
            sgp = 1.0 if vl > vh else -1.0
            bnd = lo[cp] if sgp > 0 else hi[cp]
            peq = lo[cp] == hi[cp]
            lamp = 0.0
        iters += 1
        if iters > maxit:
            return 1, None, iters
        gpp = G[cp, cp]
        vv = sgn[:k] * sgp * G[act[:k], cp]
        l = T[:k, :k] @ vv
        r = T[:k, :k].T @ l
        d2 = gpp - l @ l
        rv = sgn[:k] * r
        ds = np.where(kind != 0, sgp * G[:, cp] - G[:, act[:k]] @ rv, 0.0)
        zz = sgp * ds[cp]
        slack = sgp * (s[cp] - bnd)
        rmax = np.abs(r).max() if k else 0.0
        cand = np.full(k, INF)
        for a_ in range(k):
            if not aeq[a_] and r[a_] > 1e-13 * rmax:
                cand[a_] = lam[a_] / r[a_]
        blk = int(np.argmin(cand)) if k else 0
        t1 = cand[blk] if k else INF
        dim = P.dim + (6 if delta > 0 else 0)  # the waist slacks add 6 primal dimensions
        # AFTERDROP: p was dependent on the slots before the drop with a positive coefficient on the
        # dropped one, so it is independent of the rest in exact arithmetic -- take its step when the
        # computed complement is at least positive (EXPERIMENT)
        after_drop = os.environ.get("AFTERDROP", "0") == "1" and just_dropped
        t2 = -slack / zz if (k < dim and (zz > kdep * gpp or (after_drop and zz > 0))) else INF
        just_dropped = False
        if trace:
            print(f"  it {iters}: cp={cp} sg={sgp:+.0f} k={k} slack={slack:.3e} zz={zz:.3e} d2={d2:.3e} "
                  f"gpp={gpp:.3e} t1={t1:.3e} (blk {blk}) t2={t2:.3e}")
        if t1 >= INF and t2 >= INF:
            # no step: the incremental activities may be off by roundoff -- confirm with an exact
            # rebuild (x from the multipliers, refined, exact activities) before reporting 2
            if dirty and os.environ.get("VERIFY", "1") == "1":
                force_rebuild = True
                need_select = True
                if trace:
                    print("  no step: exact rebuild to confirm")
                continue
            return 2, None, iters
        if t2 <= t1 and k >= KM:
            return 3, None, iters
        dirty = True  # a step is taken: the incremental activities drift from the exact ones
        t = min(t1, t2)
        s = s + t * ds
        lam[:k] -= t * r
        lamp += t
        if t2 <= t1:
            idd = 1.0 / np.sqrt(d2 if d2 > 0 else zz)
            T[k, :k] = -r * idd
            T[k, k] = idd
            act[k], sgn[k], lam[k], aeq[k] = cp, sgp, lamp, peq
            onact[cp] = True
            k += 1
            need_select = True
        else:
            just_dropped = True
            onact[act[blk]] = False
            act[blk:k - 1], sgn[blk:k - 1], lam[blk:k - 1], aeq[blk:k - 1] = \
                act[blk + 1:k].copy(), sgn[blk + 1:k].copy(), lam[blk + 1:k].copy(), aeq[blk + 1:k].copy()
            k -= 1
            T[blk:, :] = 0.0
            for a2 in range(blk, k):
                cq, sq = act[a2], sgn[a2]
                vv2 = sgn[:a2] * sq * G[act[:a2], cq]
                l2 = T[:a2, :a2] @ vv2
                r2 = T[:a2, :a2].T @ l2
                e2 = G[cq, cq] - l2 @ l2
                id2 = 1.0 / np.sqrt(e2) if e2 > 0 else 0.0
                T[a2, :a2] = -r2 * id2
                T[a2, a2] = id2
            need_select = False
    return status, x, iters


def level0(P, prob, inp, b):
    """The repair kernel's level-0 step (contact_kernel.hip:contact_level0): BVLS in
    z = (tau_a, f), y0* and the pins; returns (lo, hi) of the rows with the new targets."""
    from scipy.optimize import lsq_linear
    n, nc = P.n, P.nc
    M, h, Jw, Jc = inp["M"][b], inp["h"][b], inp["Jw"][b], inp["Jc"][b]
    W = np.linalg.solve(M, Jw.T)
    cols, zlo, zhi = [], [], []
    for a_ in range(6, n):
        cols.append(W[a_]); zlo.append(prob.tau_min[a_] if prob.torque_rows else -np.inf)
        zhi.append(prob.tau_max[a_] if prob.torque_rows else np.inf)
    for f in range(3 * nc):
        c, k = divmod(f, 3)
        on = (P.cm >> c) & 1
        cols.append(W.T @ Jc[c, k]); zlo.append(prob.f_lb[k] if on else 0.0); zhi.append(prob.f_ub[k] if on else 0.0)
    A0 = np.array(cols).T
    bw = P.lo[P.NJ:P.NJ + 6]
    bb = bw + W.T @ h
    zlo, zhi = np.array(zlo), np.array(zhi)
    fixed = zlo == zhi
    lo, hi = P.lo.copy(), P.hi.copy()
    NJ = P.NJ
    abm = max(1.0, np.abs(A0.T @ bb).max())
    if P.mu > 0:  # box + friction pyramid: the LSI of qppvm_amd/csrc/fric_lsi.h (tests/fric_lsi_ref.py)
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import fric_lsi_ref as fr
        groups = [n - 6 + 3 * c for c in range(nc) if (P.cm >> c) & 1]
        z, st, fm, it, capped, pins = fr.lsi_level0(A0, bb, zlo, zhi, groups, P.mu)
        ys = A0 @ z
        ingroup = set(j for g0 in groups for j in range(g0, g0 + 3))
        held = {}
        for key, v in pins.items():
            lamv = v if (key[0] == "face" or key[1] in ingroup) else -v
            if lamv > 1e-9 * abm:
                held[key] = True
        pin = np.zeros(len(z), int)
        for key in held:
            if key[0] == "box":
                pin[key[1]] = key[2]
            else:
                c = (key[1] - (n - 6)) // 3
                lo[NJ + 6 + 3 * nc + 4 * c + key[2]] = 0.0
        for j in range(len(z)):
            ci = 6 + j if j < n - 6 else NJ + 6 + (j - (n - 6))
            if j < n - 6 and not prob.torque_rows:
                continue
            if pin[j] > 0:
                lo[ci] = hi[ci]
            elif pin[j] < 0:
                hi[ci] = lo[ci]
        # movable columns: projector of each group onto the null space of its held constraints
        cols_m = []
        for j in range(len(z)):
            if j in ingroup or fixed[j] or pin[j] != 0:
                continue
            cols_m.append(A0[:, j])
        for g0 in groups:
            N = []
            for k in range(3):
                if pin[g0 + k] != 0 or fixed[g0 + k]:
                    e = np.zeros(3); e[k] = 1.0; N.append(e)
            for key in held:
                if key[0] == "face" and key[1] == g0:
                    N.append(fr.face_normal(key[2], P.mu))
            Pc = fr.projector(np.array(N).reshape(-1, 3))
            for k in range(3):
                cols_m.append(A0[:, g0:g0 + 3] @ Pc[:, k])
        Am = np.array(cols_m).T if cols_m else np.zeros((6, 0))
        Gu = Am @ Am.T
        lo[NJ:NJ + 6] = hi[NJ:NJ + 6] = ys - W.T @ h
        unp = [0]
    else:
        A0f = A0[:, ~fixed]
        r = lsq_linear(A0f, bb - A0[:, fixed] @ zlo[fixed], bounds=(zlo[~fixed], zhi[~fixed]), method="bvls",
                       tol=1e-14, lsmr_tol=None)
        z = zlo.copy()
        z[~fixed] = r.x
        ys = A0 @ z
        g = A0.T @ (bb - ys)
        for j in range(len(z)):
            ci = 6 + j if j < n - 6 else NJ + 6 + (j - (n - 6))
            if j < n - 6 and not prob.torque_rows:
                continue
            if g[j] > 1e-9 * abm:
                lo[ci] = hi[ci]
            elif g[j] < -1e-9 * abm:
                hi[ci] = lo[ci]
        lo[NJ:NJ + 6] = hi[NJ:NJ + 6] = ys - W.T @ h
        # waist rows to keep: a pivot basis of the span of the unpinned columns (the others are
        # implied by the pins)
        unp = [j for j in range(len(z)) if not (abs(g[j]) > 1e-9 * abm) and not fixed[j]]
        Gu = A0[:, unp] @ A0[:, unp].T if unp else np.zeros((6, 6))
    keep, d = [], np.diag(Gu).copy()
    L = np.zeros((6, 6))
    dmx = max(d.max(), 1e-300)
    for c in range(6):
        cand = [r for r in range(6) if r not in keep]
        p_ = max(cand, key=lambda r: d[r])
        if not d[p_] > 1e-10 * dmx:
            break
        L[p_, c] = np.sqrt(d[p_])
        for r in cand:
            if r != p_:
                L[r, c] = (Gu[r, p_] - L[r, :c] @ L[p_, :c]) / L[p_, c]
                d[r] -= L[r, c] ** 2
        keep.append(p_)
    wkeep = sum(1 << r for r in keep)
    return lo, hi, wkeep


def main():
    import oracle
    from qppvm_amd.problem import ContactProblem
    from qppvm_amd.synth import contact_instances
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    delta = float(sys.argv[sys.argv.index("--delta") + 1]) if "--delta" in sys.argv else 0.0
    if "--delta" in sys.argv:
        args.remove(sys.argv[sys.argv.index("--delta") + 1])
    trace = "--trace" in sys.argv
    n = int(args[0]) if args else 12
    q = float(args[1]) if len(args) > 1 else 0.8
    nc = int(args[2]) if len(args) > 2 else 4
    which = [int(b) for b in args[3:]]
    MASKS4 = [0b0011, 0b0111, 0b1111, 0b0101, 0b1010, 0b1100]
    free = ContactProblem(n=n, nc=nc)
    inp = contact_instances(free, 64, seed=70 + n, masks=MASKS4 if nc == 4 else None)
    tau_free = oracle.contact_batch(free, inp)[0]
    prob = ContactProblem(n=n, nc=nc, torque_rows=True, tau_max=float(np.quantile(np.abs(tau_free[:, 6:]), q)))
    tau_r, x_r, st_r, it_r, rep = oracle.contact_batch(prob, inp)
    bad = 0
    for b in (which or range(64)):
        P = Problem(prob, inp, b)
        st, x, it = solve(P, delta=delta, trace=trace and b in which)
        err = np.abs(P.tau(x) - tau_r[b]).max() / max(1, np.abs(tau_r[b]).max()) if (st == 0 and x is not None) else -1
        if st != st_r[b] or (st == 0 and err > 1e-6) or b in which:
            bad += st != st_r[b] or (st == 0 and err > 1e-6)
            print(f"b={b} emu st={st} it={it} | oracle st={st_r[b]} rep={rep[b]} | err={err:.3e} mask={bin(int(inp['cmask'][b]))}")
    print(f"n={n} q={q} nc={nc} delta={delta}: {bad} mismatches")


if __name__ == "__main__":
    main()
