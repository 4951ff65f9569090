"""Generate the golden fixtures for the contact-form solve (run in the build container).

An *independent* numpy/scipy restatement of the ForceAcc contact-form QP
(reference src/ForceAcc.cpp:58-137,181-219; SURVEY.md 8a rows a10-a12, with the build's
written spec from oracle/wbq_oracle_contact.c). It shares no code with the oracle or the
HIP kernels:

* orientation error from scipy.spatial.transform.Rotation (make_golden.cart_error_np);
* the level-1 QP by a *primal* active set started from a feasible point that
  scipy.optimize.linprog (HiGHS) finds, equality-constrained steps by numpy KKT solves;
* accepted only with a KKT certificate (stationarity, primal feasibility, multiplier
  signs, complementarity) at tight tolerance.

Only instances whose level 0 is attained at the waist target (y0* = b_w) are kept.
Output: tests/golden/contact_n{30,39}.npz (the reference's point forces) and contact_ext_n30.npz
(6-D wrenches, friction pyramid).  Usage: python tests/golden/make_golden_contact.py [base] [ext]
"""
from __future__ import annotations

import os
import sys

import numpy as np
from scipy.optimize import linprog

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, HERE)

from make_golden import cart_error_np  # noqa: E402
from qppvm_amd.problem import ContactProblem  # noqa: E402
from qppvm_amd.synth import contact_instances  # noqa: E402


def assemble_np(prob, inp, b):
    n, nc, nfb, nx = prob.n, prob.nc, prob.n_fb, prob.nx
    wd = prob.wrench_dim
    M, h, q, qd, qref = (inp[k][b] for k in ("M", "h", "q", "qd", "qref"))

    def rhs(J, jdqd, pose, pose_ref, Kp, Kd):
        return Kp * cart_error_np(pose, pose_ref) - Kd * (J @ qd) - jdqd

    H = np.zeros((nx, nx))
    g = np.zeros(nx)
    H[:n, :n] = np.eye(n)
    g[:n] = -(prob.Kp_p * (qref - q) - prob.Kd_p * qd)
    for c in range(nc):
        J = inp["Jc"][b, c]
        bc = rhs(J, inp["jdqd_c"][b, c], inp["pose_c"][b, c], inp["pose_c_ref"][b, c], prob.Kp_f, prob.Kd_f)
        H[:n, :n] += J.T @ J
        g[:n] -= J.T @ bc
    H[n:, n:] = prob.eps_f * np.eye(wd * nc)
    bw = rhs(inp["Jw"][b], inp["jdqd_w"][b], inp["pose_w"][b], inp["pose_w_ref"][b], prob.Kp_w, prob.Kd_w)
    E = np.zeros((12, nx))
    E[:6, :n] = inp["Jw"][b]
    E[6:, :n] = M[:nfb]
    for c in range(nc):
        E[6:, n + wd * c: n + wd * c + wd] = -inp["Jc"][b, c, :wd, :nfb].T
    e = np.concatenate([bw, -h[:nfb]])
    rows, lo, hi = [], [], []
    for c in range(nc):
        on = (int(inp["cmask"][b]) >> c) & 1
        for k in range(wd):
            r = np.zeros(nx)
            r[n + wd * c + k] = 1.0
            rows.append(r)
            lo.append(prob.w_lb[k] if on else 0.0)
            hi.append(prob.w_ub[k] if on else 0.0)
    if prob.mu > 0:  # friction pyramid of the active contacts (inactive: forces already zero)
        for c in range(nc):
            if not (int(inp["cmask"][b]) >> c) & 1:
                continue
            for ax in (0, 1):
                for sg in (1.0, -1.0):
                    r = np.zeros(nx)
                    r[n + wd * c + ax] = sg
                    r[n + wd * c + 2] = -prob.mu
                    rows.append(r)
                    lo.append(-np.inf)
                    hi.append(0.0)
    if prob.torque_rows:
        for a in range(nfb, n):
            r = np.zeros(nx)
            r[:n] = M[a]
            for c in range(nc):
                r[n + wd * c: n + wd * c + wd] = -inp["Jc"][b, c, :wd, a]
            rows.append(r)
            lo.append(prob.tau_min[a] - h[a])
            hi.append(prob.tau_max[a] - h[a])
    return dict(H=H, g=g, E=E, e=e, C=np.array(rows), lo=np.array(lo), hi=np.array(hi))


def primal_active_set(H, g, E, e, C, lo, hi, maxit=400):
    """min 0.5 x'Hx + g'x s.t. E x = e, lo <= C x <= hi: primal active set from an LP
    feasible point. Returns x, (mu, lam) or None when infeasible."""
    nx = H.shape[0]
    m = C.shape[0]
    fixed = lo == hi
    # strictly interior start (w.r.t. the non-fixed rows): max t s.t. E x = e,
    # lo + t w <= C x <= hi - t w, 0 <= t <= 1; the fixed rows (lo == hi) are equalities
    w = np.where(fixed, 0.0, np.minimum(1.0, (hi - lo) / 4.0))
    fl = np.isfinite(lo)  # one-sided rows (the friction faces) have no lower side
    Aub = np.vstack([np.hstack([-C[fl], w[fl, None]]), np.hstack([C, w[:, None]])])
    bub = np.concatenate([-lo[fl], hi])
    Aeq = np.hstack([E, np.zeros((E.shape[0], 1))])
    cost = np.zeros(nx + 1)
    cost[-1] = -1.0
    lp = linprog(cost, A_ub=Aub, b_ub=bub, A_eq=Aeq, b_eq=e, bounds=[(None, None)] * nx + [(0.0, 1.0)],
                 method="highs")
    if lp.status != 0:
        return None
    x = lp.x[:nx].copy()
    W = {j: 2 for j in range(m) if fixed[j]}
    for _ in range(maxit):
        idx = sorted(W)
        A = np.vstack([E] + [C[j][None] for j in idx]) if idx else E
        K = np.block([[H, A.T], [A, np.zeros((A.shape[0], A.shape[0]))]])
        rhs = np.concatenate([-(H @ x + g), np.zeros(A.shape[0])])
        try:
            sol = np.linalg.solve(K, rhs)
        except np.linalg.LinAlgError:  # dependent working-set rows
            sol = np.linalg.lstsq(K, rhs, rcond=1e-15)[0]
        p = sol[:nx]
        if np.abs(p).max() <= 1e-9 * max(1, np.abs(x).max()):
            mult = -sol[nx:]  # H x + g = A' mult at the working-set optimum
            lam = mult[E.shape[0]:]
            # lower-side rows need mult >= 0 (C x >= lo), upper-side mult <= 0
            tol = 1e-10 * max(1, np.abs(lam).max(initial=0.0))
            wj = None
            for k, j in enumerate(idx):  # smallest index with a wrong-sign multiplier (Bland)
                if W[j] != 2 and (-lam[k] if W[j] == -1 else lam[k]) > tol:
                    wj = j
                    break
            if wj is None:
                return x, mult
            del W[wj]
            continue
        # step to the first blocking row
        alpha, blk, side = 1.0, None, 0
        Cp = C @ p
        Cx = C @ x
        for j in range(m):
            if j in W:
                continue
            if Cp[j] > 1e-14 and Cx[j] + Cp[j] > hi[j]:
                a = (hi[j] - Cx[j]) / Cp[j]
                if a < alpha - 1e-15:
                    alpha, blk, side = a, j, 1
            elif Cp[j] < -1e-14 and Cx[j] + Cp[j] < lo[j]:
                a = (lo[j] - Cx[j]) / Cp[j]
                if a < alpha - 1e-15:
                    alpha, blk, side = a, j, -1
        x = x + max(alpha, 0.0) * p
        if blk is not None:
            W[blk] = side
    raise RuntimeError("primal active set did not converge")


def kkt_certificate(H, g, E, e, C, lo, hi, x, mult):
    me = E.shape[0]
    s = C @ x
    scale = max(1.0, np.abs(g).max(), np.abs(H @ x).max())
    # reconstruct full multipliers on all rows from the active ones via least squares
    act = [j for j in range(C.shape[0]) if min(abs(s[j] - lo[j]), abs(s[j] - hi[j])) <= 1e-8 * max(1, abs(s[j]))]
    A = np.vstack([E] + [C[j][None] for j in act]) if act else E
    mu = np.linalg.lstsq(A.T, H @ x + g, rcond=None)[0]
    stat = np.abs(A.T @ mu - H @ x - g).max() / scale
    feas = max(np.abs(E @ x - e).max() / max(1, np.abs(e).max()),
               max(0.0, (lo - s).max(initial=0.0)), max(0.0, (s - hi).max(initial=0.0)))
    lam = mu[me:]
    sign = 0.0
    for k, j in enumerate(act):
        if lo[j] == hi[j]:
            continue
        at_lo = abs(s[j] - lo[j]) <= abs(s[j] - hi[j])
        sign = max(sign, (-lam[k] if at_lo else lam[k]) / max(1, np.abs(lam).max()))
    return stat, feas, sign


GROUPS = [  # name, count, problem kwargs, masks
    ("double_support", 6, dict(nc=2), None),
    ("masks_2_3_4", 6, dict(nc=4), [0b0011, 0b0111, 0b1111, 0b0110, 0b1101]),
    ("torque_rows", 6, dict(nc=2, torque_rows=True, tau_max=40.0), None),
]


# full 6-D wrenches ("put 6 for full wrench", ForceAcc.cpp:67; moment box +-1, :74-76)
# and the linearised friction pyramid (tests/golden/contact_ext_n30.npz)
GROUPS_EXT = [
    ("wrench6_double", 6, dict(nc=2, wrench_dim=6), None),
    ("wrench6_masks", 6, dict(nc=4, wrench_dim=6), [0b0011, 0b0111, 0b1111, 0b0110, 0b1101]),
    ("friction_double", 6, dict(nc=2, mu=0.3), None),
    ("friction_masks", 6, dict(nc=4, mu=0.3), [0b0011, 0b0111, 0b1111, 0b0110, 0b1101]),
    ("wrench6_friction_torque", 6, dict(nc=2, wrench_dim=6, mu=0.3, torque_rows=True, tau_max=40.0), None),
    ("friction_torque_masks", 6, dict(nc=4, mu=0.5, torque_rows=True, tau_max=60.0), [0b0011, 0b0111, 0b1111]),
]


def make(n, seed, groups=GROUPS):
    out = {}
    names = []
    for gi, (name, count, kw, masks) in enumerate(groups):
        prob = ContactProblem(n=n, **kw)
        inp = contact_instances(prob, 4 * count, seed=seed * 100 + gi, masks=masks)
        keep, taus, xs = [], [], []
        for b in range(4 * count):
            a = assemble_np(prob, inp, b)
            r = primal_active_set(a["H"], a["g"], a["E"], a["e"], a["C"], a["lo"], a["hi"])
            if r is None:
                print(f"n={n} {name}[{b}] level 0 not attained at b_w: skipped")
                continue
            x, mult = r
            stat, feas, sign = kkt_certificate(a["H"], a["g"], a["E"], a["e"], a["C"], a["lo"], a["hi"], x, mult)
            assert stat < 1e-9 and feas < 1e-9 and sign < 1e-9, (name, b, stat, feas, sign)
            nn, nc = prob.n, prob.nc
            M, h = inp["M"][b], inp["h"][b]
            tau = M @ x[:nn] + h
            wd = prob.wrench_dim
            for c in range(nc):
                tau -= inp["Jc"][b, c, :wd].T @ x[nn + wd * c: nn + wd * c + wd]
            nact = int(np.sum(np.minimum(np.abs(a["C"] @ x - a["lo"]), np.abs(a["C"] @ x - a["hi"])) < 1e-8))
            print(f"n={n} {name}[{b}] active_rows={nact} kkt=({stat:.1e},{feas:.1e},{sign:.1e})")
            keep.append(b)
            taus.append(tau)
            xs.append(x)
            if len(keep) == count:
                break
        pre = f"{name}__"
        for k, v in inp.items():
            out[pre + k] = v[keep]
        out[pre + "tau"] = np.array(taus)
        out[pre + "x"] = np.array(xs)
        out[pre + "nc"] = np.int32(prob.nc)
        out[pre + "torque_rows"] = np.int32(prob.torque_rows)
        out[pre + "wrench_dim"] = np.int32(prob.wrench_dim)
        out[pre + "mu"] = np.float64(prob.mu)
        out[pre + "tau_max"] = prob.tau_max
        names.append(name)
    out["groups"] = np.array(names)
    return out


def main(which=("base", "ext")):
    jobs = []
    if "base" in which:
        jobs += [(f"contact_n{n}.npz", n, seed, GROUPS) for n, seed in ((30, 4), (39, 5))]
    if "ext" in which:
        jobs += [("contact_ext_n30.npz", 30, 6, GROUPS_EXT)]
    for fname, n, seed, groups in jobs:
        data = make(n, seed, groups)
        path = os.path.join(HERE, fname)
        np.savez_compressed(path, **data)
        print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main(tuple(sys.argv[1:]) or ("base", "ext"))
