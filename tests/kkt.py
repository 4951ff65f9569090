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
    """Scaled residuals of instance b's output tau: dict(primal, level0, stat, sign, indep)."""
    M = inp["M"][b]
    a = oracle.assemble(prob, inp, b)
    A0, b0, lb, ub = a["A0"], a["b0"], a["lb"], a["ub"]
    x = tau - inp["h"][b]
    scale = 1.0 + np.abs(np.concatenate([lb, ub])).max()
    primal = max(0.0, (lb - x).max(), (x - ub).max()) / scale
    at_lo, at_hi = _active(x, lb, ub, 1e-9)
    free = ~(at_lo | at_hi)
    g0 = A0.T @ (A0 @ x - b0)
    s0 = np.abs(A0.T).sum(axis=1) * (np.abs(A0 @ x).max() + np.abs(b0).max()) + 1e-300
    l0 = np.where(free, np.abs(g0), 0.0)
    l0 = np.maximum(l0, np.where(at_lo & ~at_hi, np.maximum(-g0, 0.0), 0.0))
    l0 = np.maximum(l0, np.where(at_hi & ~at_lo, np.maximum(g0, 0.0), 0.0))
    level0 = float((l0 / s0).max())
    pinned = np.abs(g0) > 1e-7 * s0  # level 0 holds these at their bound
    G = A0 @ M
    timp = _tau_imp(prob, inp, b)
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


def contact_level0_certificate(oracle, prob, inp, b, x):
    """Level-0 optimality of a contact-form output whose waist row is not at b_w (level 0 not
    attainable): with tau = M qdd + h - J_c^T [f; 0] every row is a box in z = (tau_a, f) and the
    waist value is y = A0 z - J_w M^-1 h (qppvm_amd/csrc/contact_kernel.hip:contact_level0), so z
    must solve min 0.5 ||A0 z - (b_w + J_w M^-1 h)||^2 over the box: the gradient w = A0^T (b - A0 z)
    vanishes on interior variables, w <= 0 at lower and w >= 0 at upper bounds. Returns the scaled
    worst violation and y."""
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
    A0, z, lo, hi = np.array(cols).T, np.array(z), np.array(lo), np.array(hi)
    bb = a["bw"] + W.T @ h
    w = A0.T @ (bb - A0 @ z)
    scale = np.abs(A0.T).sum(axis=1) * (np.abs(A0 @ z).max() + np.abs(bb).max()) + 1e-300
    at_lo, at_hi = _active(z, lo, hi, 1e-8)
    v = np.where(~(at_lo | at_hi), np.abs(w), 0.0)
    v = np.maximum(v, np.where(at_lo & ~at_hi, np.maximum(w, 0.0), 0.0))
    v = np.maximum(v, np.where(at_hi & ~at_lo, np.maximum(-w, 0.0), 0.0))
    return float((v / scale).max()), Jw @ qdd


def contact_certificate(oracle, prob, inp, b, x, waist=None):
    """Scaled residuals of instance b's contact-form output x = [qdd; f]; waist (optional) replaces
    the waist target b_w (level 1 after a level-0 repair keeps J_w qdd = y0*)."""
    a = oracle.contact_assemble(prob, inp, b)
    H, g, E, e, C, clo, chi = a["H"], a["g"], a["E"], a["e"], a["C"], a["clo"], a["chi"]
    if waist is not None:
        e = e.copy()
        e[:6] = waist
    cx = C @ x
    scale = 1.0 + max(np.abs(e).max(), np.abs(np.concatenate([clo, chi])[np.isfinite(np.concatenate([clo, chi]))]).max(initial=0.0))
    primal = max(np.abs(E @ x - e).max(), max(0.0, (clo - cx).max(initial=0.0), (cx - chi).max(initial=0.0))) / scale
    # a row met to 1e-8 relative is active: the dual loop accepts its active rows at that level
    # (qppvm_amd/csrc/dual_gi.h, the final re-check)
    at_lo, at_hi = _active(cx, clo, chi, 1e-8)
    act = np.where(at_lo | at_hi)[0]
    K = np.concatenate([E.T, C[act].T], axis=1)
    r = H @ x + g
    lam, *_ = np.linalg.lstsq(K, r, rcond=None)
    stat = float(np.abs(r - K @ lam).max() / (np.abs(H @ x).max() + np.abs(g).max() + 1e-300))
    indep = np.linalg.matrix_rank(K, tol=1e-10 * np.abs(K).max()) == K.shape[1]
    sign = 0.0
    if indep:
        mu = lam[E.shape[0]:]
        mscale = np.abs(lam).max() + 1e-300
        for c, j in enumerate(act):
            if clo[j] == chi[j]:
                continue
            if at_lo[j] and not at_hi[j]:
                sign = max(sign, -mu[c] / mscale)
            elif at_hi[j] and not at_lo[j]:
                sign = max(sign, mu[c] / mscale)
    return dict(primal=primal, stat=stat, sign=sign, indep=bool(indep))
