"""KAT-4: optimality certificates for a solver output, computed from the
assembled problem alone -- no reference solution, so they hold at any batch size.

QPPVM (oracle/wbq_oracle.c:wbq_ref_assemble: A0 = G M^-1, b0, lb, ub; x = tau - h):
  level 0   x is a minimiser of 0.5 ||A0 x - b0||^2 over the box: with the gradient
            g0 = A0^T (A0 x - b0), g0_j = 0 where x_j is free, >= 0 at lb, <= 0 at ub;
  level 1   x minimises the joint task over {A0 x = A0 x, box}: M grad f1 = G^T nu + M mu
            (M grad f1 = M^-1 (x - tau_imp) for W1 = I, x - tau_imp for W1 = M), mu_j >= 0
            at lb, <= 0 at ub, 0 where free; variables level 0 pins (|g0_j| above roundoff)
            are fixed for level 1 and carry a multiplier of either sign;
  primal    lb <= x <= ub.
Contact form (oracle/wbq_oracle_contact.c:wbq_ref_contact_assemble: H, g, E x = e, clo <= C x
<= chi): H x + g = E^T nu + C^T mu with mu >= 0 on rows at clo, <= 0 at chi, and primal
feasibility. Residuals are scaled; the multipliers of a rank-deficient active set are not
unique, so their signs are checked only where the active normals are independent.
"""
import numpy as np


def _tau_imp(prob, inp, b):
    return prob.Kq * (inp["qref"][b] - inp["q"][b]) - prob.Dq * inp["qd"][b]


def _active(v, lo, hi, tol):
    at_lo = v - lo <= tol * (1.0 + np.abs(lo))
    at_hi = hi - v <= tol * (1.0 + np.abs(hi))
    return at_lo, at_hi


def qppvm_certificate(oracle, prob, inp, b, tau):
    """Scaled residuals of instance b's output tau: dict(primal, level0, stat, sign, indep).
    With a middle level (prob.task_level, the elbow tasks) the Cartesian rows form two lexicographic
    levels: level 0 over the first prob.m_l0 rows as above, then the middle level
    0.5 ||A1 x - b1||^2 over {A0 x = A0 x, box}: its gradient g1 = E^T nu + mu with E the level-0 rows,
    nu fitted on the free variables, mu_j of the right sign at bounds the earlier level does not pin;
    "level0" reports the worse of the two."""
    M = inp["M"][b]
    a = oracle.assemble(prob, inp, b)
    A0, b0, lb, ub = a["A0"], a["b0"], a["lb"], a["ub"]
    x = tau - inp["h"][b]
    scale = 1.0 + np.abs(np.concatenate([lb, ub])).max()
    primal = max(0.0, (lb - x).max(), (x - ub).max()) / scale
    at_lo, at_hi = _active(x, lb, ub, 1e-9)
    free = ~(at_lo | at_hi)
    ml = getattr(prob, "m_l0", A0.shape[0])
    levels = [(A0[:ml], b0[:ml])] + ([(A0[ml:], b0[ml:])] if ml < A0.shape[0] else [])
    pinned = lb == ub
    level0, E = 0.0, None
    for Al, bl in levels:
        g0 = Al.T @ (Al @ x - bl)
        s0 = np.abs(Al.T).sum(axis=1) * (np.abs(Al @ x).max() + np.abs(bl).max()) + 1e-300
        if E is not None:
            if free.any():
                nu = np.linalg.lstsq(E[:, free].T, g0[free], rcond=None)[0]
                g0 = g0 - E.T @ nu
        l0 = np.where(free, np.abs(g0), 0.0)
        l0 = np.maximum(l0, np.where(at_lo & ~at_hi & ~pinned, np.maximum(-g0, 0.0), 0.0))
        l0 = np.maximum(l0, np.where(at_hi & ~at_lo & ~pinned, np.maximum(g0, 0.0), 0.0))
        level0 = max(level0, float((l0 / s0).max()))
        pinned = pinned | (~free & (np.abs(g0) > 1e-7 * s0))  # this level holds these at their bound
        E = Al if E is None else np.concatenate([E, Al], axis=0)
    G = A0 @ M
    timp = _tau_imp(prob, inp, b)
    # M times the last level's gradient: W1 = I M^-1 (x - tau_imp), W1 = M x - tau_imp, and without
    # the joint task (min 0.5 ||x||^2, the reference's commented elbow stack) M x
    if not getattr(prob, "joint_task", True):
        r = M @ x
    else:
        r = np.linalg.solve(M, x - timp) if prob.joint_weight == 0 else x - timp
    act = np.where(~free)[0]
    K = np.concatenate([G.T, M[:, act]], axis=1)
    lam, *_ = np.linalg.lstsq(K, r, rcond=None)
    stat = float(np.abs(r - K @ lam).max() / (np.abs(r).max() + np.abs(K @ lam).max() + 1e-300))
    mu = lam[G.shape[0]:]
    indep = np.linalg.matrix_rank(K, tol=1e-10 * np.abs(K).max()) == K.shape[1]
    sign = 0.0
    if indep:
        mscale = np.abs(lam).max() + 1e-300
        for c, j in enumerate(act):
            if pinned[j] or lb[j] == ub[j]:
                continue
            if at_lo[j] and not at_hi[j]:
                sign = max(sign, -mu[c] / mscale)
            elif at_hi[j] and not at_lo[j]:
                sign = max(sign, mu[c] / mscale)
    return dict(primal=primal, level0=level0, stat=stat, sign=sign, indep=bool(indep))


def contact_level0_zspace(oracle, prob, inp, b, x):
    """Level 0 of the contact form in z = (tau_a, w) space (qppvm_amd/csrc/contact_kernel.hip:
    contact_level0): with tau = M qdd + h - J_c^T w every row is a box in z (plus the friction faces
    on the forces) and the waist value is y = A0 z - J_w M^-1 h. Returns (A0, b, z, lo, hi, y) for
    the output x = [qdd; w]."""
    a = oracle.contact_assemble(prob, inp, b)
    n, nc = prob.n, prob.nc
    M, h, Jw, Jc = inp["M"][b], inp["h"][b], inp["Jw"][b], inp["Jc"][b]
    cm = int(inp["cmask"][b])
    qdd, f = x[:n], x[n:]
    wd = getattr(prob, "wrench_dim", 3)
    tau = M @ qdd + h - sum(Jc[c, :wd].T @ f[wd * c:wd * c + wd] for c in range(nc))
    W = np.linalg.solve(M, Jw.T)
    cols, z, lo, hi = [], [], [], []
    for j in range(6, n):
        cols.append(W[j]); z.append(tau[j])
        lo.append(prob.tau_min[j] if prob.torque_rows else -np.inf)
        hi.append(prob.tau_max[j] if prob.torque_rows else np.inf)
    wlb, wub = (prob.w_lb, prob.w_ub) if hasattr(prob, "w_lb") else (prob.f_lb, prob.f_ub)
    for k in range(wd * nc):
        c, r = divmod(k, wd)
        on = (cm >> c) & 1
        cols.append(W.T @ Jc[c, r]); z.append(f[k])
        lo.append(wlb[r] if on else 0.0); hi.append(wub[r] if on else 0.0)
    return (np.array(cols).T, a["bw"] + W.T @ h, np.array(z), np.array(lo), np.array(hi), Jw @ qdd)


def lsi_certificate(A0, bb, z, lo, hi, groups=(), mu=0.0, act_tol=1e-8):
    """Scaled KKT violation of z for min 0.5 ||A0 z - bb||^2 over lo <= z <= hi and, for every
    friction group (start index j of an active contact's (f_x, f_y, f_z)), the pyramid faces
    s f_x - mu f_z <= 0, s f_y - mu f_z <= 0: w = A0^T (bb - A0 z) (= -gradient) vanishes on free
    variables, has the sign of the outward normal at an active bound, and on a group is a
    non-negative combination of the outward normals of its active box sides and faces (NNLS)."""
    w = A0.T @ (bb - A0 @ z)
    scale = np.abs(A0.T).sum(axis=1) * (np.abs(A0 @ z).max() + np.abs(bb).max()) + 1e-300
    at_lo, at_hi = _active(z, lo, hi, act_tol)
    v = np.where(~(at_lo | at_hi), np.abs(w), 0.0)
    v = np.maximum(v, np.where(at_lo & ~at_hi, np.maximum(w, 0.0), 0.0))
    v = np.maximum(v, np.where(at_hi & ~at_lo, np.maximum(-w, 0.0), 0.0))
    with np.errstate(invalid="ignore"):
        pl = np.where(np.isfinite(lo), (lo - z) / (1.0 + np.abs(np.where(np.isfinite(lo), lo, 0.0))), 0.0)
        ph = np.where(np.isfinite(hi), (z - hi) / (1.0 + np.abs(np.where(np.isfinite(hi), hi, 0.0))), 0.0)
    primal = max(0.0, pl.max(initial=0.0), ph.max(initial=0.0))  # relative to the bound
    for j in groups:
        from scipy.optimize import nnls
        fv, wc = z[j:j + 3], w[j:j + 3]
        nrm, tol = [], act_tol * (1.0 + np.abs(fv).max())
        for k in range(3):
            e = np.zeros(3)
            e[k] = 1.0
            if at_lo[j + k] and not at_hi[j + k]:
                nrm.append(-e)
            if at_hi[j + k] and not at_lo[j + k]:
                nrm.append(e)
        for f in range(4):
            nv = np.zeros(3)
            nv[f >> 1] = -1.0 if f & 1 else 1.0
            nv[2] = -mu
            ph = nv @ fv
            primal = max(primal, ph / (1.0 + np.abs(fv).max()))
            if ph >= -tol:
                nrm.append(nv)
        res = nnls(np.array(nrm).T, wc)[1] if nrm else np.linalg.norm(wc)
        sc = np.abs(scale[j:j + 3]).max()
        v[j:j + 3] = 0.0
        v[j] = res * scale[j] / sc
    return float(max((v / scale).max(), primal))


def contact_friction_groups(prob, inp, b):
    """z-space start indices of the active contacts' force triples (friction groups; none without mu)"""
    if float(getattr(prob, "mu", 0.0)) <= 0.0:
        return []
    wd, cm = getattr(prob, "wrench_dim", 3), int(inp["cmask"][b])
    return [prob.n - 6 + wd * c for c in range(prob.nc) if (cm >> c) & 1]


def contact_level0_certificate(oracle, prob, inp, b, x):
    """Level-0 optimality of a contact-form output whose waist row is not at b_w (level 0 not
    attainable): z must solve the level-0 LSI (lsi_certificate; the box, and with mu > 0 the friction
    pyramid faces). Returns the scaled worst violation and y."""
    A0, bb, z, lo, hi, y = contact_level0_zspace(oracle, prob, inp, b, x)
    return lsi_certificate(A0, bb, z, lo, hi, contact_friction_groups(prob, inp, b),
                           float(getattr(prob, "mu", 0.0))), y


def contact_certificate(oracle, prob, inp, b, x, waist=None):
    """Scaled residuals of instance b's contact-form output x = [qdd; f]; waist (optional) replaces
    the waist target b_w (level 1 after a level-0 repair keeps J_w qdd = y0*).

    No activity threshold decides which rows the multipliers may use (round 3 classified rows as
    active at a relative slack of 1e-8, the kernel's own re-check tolerance): every inequality row
    within a window (1e-9 .. 1e-6, the best of the four kept) of a bound is a candidate in the
    least-squares fit H x + g = E^T nu + C^T mu, and a
    multiplier on a row that is not exactly at its bound is charged through complementarity,
    |mu_j| / max|mu| * slack_j (a row 1e-7 off its bound carrying a full-size multiplier fails). Signs
    (mu >= 0 at clo, <= 0 at chi) are checked where the candidate normals are independent (the
    multipliers are unique there). Keys: primal, stat (fit residual), sign (worst wrong-signed
    multiplier, scaled), comp (complementarity), indep, window."""
    a = oracle.contact_assemble(prob, inp, b)
    H, g, E, e, C, clo, chi = a["H"], a["g"], a["E"], a["e"], a["C"], a["clo"], a["chi"]
    if waist is not None:
        e = e.copy()
        e[:6] = waist
    cx = C @ x
    fin = np.concatenate([clo, chi])
    scale = 1.0 + max(np.abs(e).max(), np.abs(fin[np.abs(fin) < 1e299]).max(initial=0.0))
    primal = max(np.abs(E @ x - e).max(), max(0.0, (clo - cx).max(initial=0.0), (cx - chi).max(initial=0.0))) / scale
    rs = 1.0 + np.abs(cx)
    s_lo, s_hi = (cx - clo) / rs, (chi - cx) / rs  # relative slacks (huge for an unbounded side)
    r = H @ x + g
    rscale = np.abs(H @ x).max() + np.abs(g).max() + 1e-300
    best = None
    # KKT asks for SOME multipliers: every candidate window is tried and the best certificate kept
    # (on a degenerate instance the min-norm fit over the widest window spreads weight onto rows that
    # are slightly off their bound, which a narrower window does not offer it)
    for win in (1e-9, 1e-8, 1e-7, 1e-6):
        cand = np.where((s_lo <= win) | (s_hi <= win))[0]
        K = np.concatenate([E.T, C[cand].T], axis=1)
        lam, *_ = np.linalg.lstsq(K, r, rcond=None)
        stat = float(np.abs(r - K @ lam).max() / rscale)
        indep = np.linalg.matrix_rank(K, tol=1e-10 * np.abs(K).max()) == K.shape[1]
        mu = lam[E.shape[0]:]
        mscale = np.abs(lam).max() + 1e-300
        near_lo = s_lo[cand] <= s_hi[cand]
        slack = np.where(near_lo, s_lo[cand], s_hi[cand])
        comp = float((np.abs(mu) / mscale * np.maximum(slack, 0.0)).max(initial=0.0))
        sign = 0.0
        if indep:
            eq = clo[cand] == chi[cand]
            wrong = np.where(near_lo, -mu, mu) / mscale
            sign = float(np.where(eq, 0.0, np.maximum(wrong, 0.0)).max(initial=0.0))
        c = dict(primal=primal, stat=stat, sign=sign, comp=comp, indep=bool(indep), window=win)
        if best is None or max(stat, sign, comp) < max(best["stat"], best["sign"], best["comp"]):
            best = c
    return best
