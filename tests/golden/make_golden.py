"""Generate the golden fixtures for the QPPVM solve (run in the build container).

This is an *independent* numpy/scipy restatement of the reference's per-tick solve
(QPPVMPlugin.cpp:201-259 through OpenSoT/qpOASES). It shares
no code with oracle/wbq_oracle.c or the HIP kernels:

* Cartesian orientation error from scipy.spatial.transform.Rotation
  (quaternion of R_ref R^T, sign fixed to w >= 0);
* level 0 by scipy.optimize.lsq_linear(method="bvls") -> y* = A0 x0*;
* level 1 by a numpy guess-and-polish active set on the x-space QP, accepted only
  with a KKT certificate (stationarity, primal feasibility, multiplier signs,
  complementarity) checked at tight tolerance;
* bounds-inactive groups additionally carry the closed forms KAT-1 (W1 = I) and
  KAT-2 (W1 = M) of SURVEY.md 8c.

Output: tests/golden/qppvm_n{7,30,39}.npz (inputs + expected tau, y0, status).
Usage: python tests/golden/make_golden.py
"""
from __future__ import annotations

import os
import sys

import numpy as np
from scipy.optimize import lsq_linear
from scipy.spatial.transform import Rotation

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from qppvm_amd.problem import QPPVMProblem, SELECT_SUBTASK, SELECT_TASK  # noqa: E402
from qppvm_amd.synth import qppvm_instances  # noqa: E402


def cart_error_np(pose, pose_ref):
    P = pose.reshape(3, 4)
    Pr = pose_ref.reshape(3, 4)
    q = Rotation.from_matrix(Pr[:, :3] @ P[:, :3].T).as_quat()  # x, y, z, w
    if q[3] < 0:
        q = -q
    return np.concatenate([Pr[:, 3] - P[:, 3], q[:3]])


def assemble_np(prob, inp, b):
    n = prob.n
    M = inp["M"][b]
    Minv = np.linalg.inv(M)
    A_rows, b_rows, G_rows, y_rows = [], [], [], []
    for t in range(prob.ntasks):
        J = inp["J"][b, t]
        e = cart_error_np(inp["pose"][b, t], inp["pose_ref"][b, t])
        F = prob.Kc[t] * e - prob.Dc[t] * (J @ inp["qd"][b])
        sel = np.array([(prob.row_mask[t] >> r) & 1 for r in range(6)], dtype=bool)
        if prob.select_mode == SELECT_TASK:
            F = np.where(sel, F, 0.0)
        A6 = J @ Minv
        b6 = A6 @ (J.T @ F)
        A_rows.append(A6[sel])
        b_rows.append(b6[sel])
        G_rows.append(J[sel])
    A0 = np.vstack(A_rows)
    b0 = np.concatenate(b_rows)
    G = np.vstack(G_rows)
    timp = prob.Kq * (inp["qref"][b] - inp["q"][b]) - prob.Dq * inp["qd"][b]
    A1 = Minv
    b1 = Minv @ timp
    W = M if prob.joint_weight == 1 else np.eye(n)
    H1 = A1.T @ W @ A1
    g1 = -A1.T @ W @ b1
    lb = prob.tau_min - inp["h"][b]
    ub = prob.tau_max - inp["h"][b]
    return dict(A0=A0, b0=b0, G=G, H1=0.5 * (H1 + H1.T), g1=g1, lb=lb, ub=ub, timp=timp, M=M,
                Minv=Minv)


def level0_np(A0, b0, lb, ub):
    r = lsq_linear(A0, b0, bounds=(lb, ub), method="bvls", tol=1e-15, max_iter=10000)
    x = np.clip(r.x, lb, ub)
    # KKT certificate of the bounded least squares (gradient signs on bound variables)
    w = A0.T @ (b0 - A0 @ x)
    scale = max(1.0, np.abs(A0.T @ b0).max())
    at_lo = x <= lb + 1e-12 * np.maximum(1, np.abs(lb))
    at_hi = x >= ub - 1e-12 * np.maximum(1, np.abs(ub))
    free = ~(at_lo | at_hi)
    assert np.all(np.abs(w[free]) <= 1e-7 * scale), np.abs(w[free]).max() / scale
    assert np.all(w[at_lo & ~at_hi] <= 1e-7 * scale)
    assert np.all(w[at_hi & ~at_lo] >= -1e-7 * scale)
    return x, A0 @ x


def _null(E, k):
    if E.shape[0] == 0 or k == 0:
        return np.eye(k)
    _, S, Vt = np.linalg.svd(E, full_matrices=True)
    r = int(np.sum(S > 1e-12 * max(S.max(), 1e-300)))
    return Vt[r:].T


def level1_np(H, g, Aeq, beq, lb, ub, x0, maxit=500, gscale=None):
    """Monotone primal active set (Nocedal & Wright alg. 16.3, null-space EQP) from the
    feasible level-0 point; accepted only with a KKT certificate. gscale: the gradient scale of
    the tolerances (default max(1, |g|); a problem with g = 0 passes the scale of H x)."""
    n = H.shape[0]
    x = np.clip(x0.copy(), lb, ub)
    lo = x <= lb
    hi = (x >= ub) & ~lo
    stationary = False  # a full (unblocked) step lands on the working-set optimum
    for _ in range(maxit):
        F = ~(lo | hi)
        k = int(F.sum())
        gr = H @ x + g
        Z = _null(Aeq[:, F], k)
        p = np.zeros(n)
        if Z.shape[1]:
            HZ = Z.T @ H[np.ix_(F, F)] @ Z
            p[F] = -Z @ np.linalg.solve(HZ, Z.T @ gr[F])
        if stationary or np.abs(p).max() <= 1e-12 * max(1.0, np.abs(x).max()):
            stationary = False
            nu = np.linalg.lstsq(Aeq[:, F].T, -gr[F], rcond=None)[0] if k else \
                np.zeros(Aeq.shape[0])
            lam = gr + Aeq.T @ nu  # lambda_lo - lambda_hi on the bound variables
            wrong = np.where(lo & (lb < ub), -lam, np.where(hi, lam, -np.inf))
            gs = max(1.0, np.abs(g).max()) if gscale is None else gscale
            tol_g = 1e-9 * max(gs, np.abs(Aeq.T @ nu).max())
            if wrong.max() <= tol_g:
                # certificate: stationarity on F, feasibility, signs (checked above)
                assert np.abs(lam[F]).max(initial=0.0) <= 1e-8 * gs
                assert np.abs(Aeq @ x - beq).max() <= 1e-8 * max(1.0, np.abs(beq).max())
                assert np.all(x >= lb) and np.all(x <= ub)
                return x
            i = int(np.argmax(wrong))
            lo[i] = hi[i] = False
            continue
        alpha, j = 1.0, -1
        for i in np.where(F & (p != 0))[0]:
            t = ((lb[i] if p[i] < 0 else ub[i]) - x[i]) / p[i]
            if t < alpha:
                alpha, j = max(t, 0.0), i
        x = x + alpha * p
        stationary = j < 0
        if j >= 0:
            if p[j] < 0:
                lo[j], x[j] = True, lb[j]
            else:
                hi[j], x[j] = True, ub[j]
    raise RuntimeError("level-1 active set did not converge")


def solve_np(prob, inp, b):
    a = assemble_np(prob, inp, b)
    x0, y = level0_np(a["A0"], a["b0"], a["lb"], a["ub"])
    # variables the level-0 gradient pins to a bound are at that bound in every level-0
    # optimum, hence in every point of level 1's feasible set: fix them
    w = a["A0"].T @ (a["b0"] - y)
    tol = 1e-9 * max(1.0, np.abs(a["A0"].T @ a["b0"]).max())
    lb1, ub1 = a["lb"].copy(), a["ub"].copy()
    up = w > tol
    dn = w < -tol
    lb1[up] = ub1[up]
    ub1[dn] = lb1[dn]
    x0 = np.clip(x0, lb1, ub1)
    x = level1_np(a["H1"], a["g1"], a["A0"], y, lb1, ub1, x0)
    return x + inp["h"][b], y, a


def kat(prob, inp, b, a):
    """Closed forms for the bounds-inactive case."""
    M, Minv, G, timp = a["M"], a["Minv"], a["G"], a["timp"]
    y = a["b0"]
    if prob.joint_weight == 0:
        x = timp + M @ G.T @ np.linalg.solve(G @ G.T, y - G @ Minv @ timp)
    else:
        Lam = np.linalg.inv(G @ Minv @ G.T)
        x = timp + G.T @ Lam @ (y - G @ Minv @ timp)
    return x + inp["h"][b]


GROUPS = [
    # name, count, problem kwargs, expect bounds inactive
    ("inactive_I", 4, dict(tau_max=1e6), True),
    ("inactive_M", 2, dict(tau_max=1e6, joint_weight=1), True),
    ("inactive_task", 2, dict(tau_max=1e6, select_mode=SELECT_TASK), True),
    ("inactive_6row", 2, dict(tau_max=1e6, row_mask=(0x3F, 0x3F)), True),
    ("active1", 4, dict(tau_max=None), False),
    ("heavy1", 3, dict(tau_max=None), False),
    ("infeas0", 3, dict(tau_max=2.0), False),
]


def calibrate_tau(prob_kw, n, inp, frac):
    """tau_max such that about `frac` of the unconstrained |tau| exceed it."""
    prob = QPPVMProblem(n=n, **{**prob_kw, "tau_max": 1e6})
    taus = [solve_np(prob, inp, b)[0] for b in range(inp["h"].shape[0])]
    return float(np.quantile(np.abs(np.concatenate(taus)), 1.0 - frac))


def make(n, seed):
    out = {}
    for gi, (name, count, kw, inactive) in enumerate(GROUPS):
        kw = dict(kw)
        probe = QPPVMProblem(n=n, **{**kw, "tau_max": 1.0})
        inp = qppvm_instances(probe, count, seed=seed * 100 + gi)
        if kw.get("tau_max") is None:
            kw["tau_max"] = calibrate_tau(kw, n, inp, 0.2 if name == "active1" else 0.97)
        prob = QPPVMProblem(n=n, **kw)
        taus, ys, kats = [], [], []
        for b in range(count):
            tau, y, a = solve_np(prob, inp, b)
            taus.append(tau)
            ys.append(y)
            if inactive and prob.m0 < n:
                k = kat(prob, inp, b, a)
                assert np.abs(k - tau).max() <= 1e-8 * max(1, np.abs(k).max()), name
                kats.append(k)
            act = np.mean((tau - inp["h"][b] <= a["lb"] + 1e-9) | (tau - inp["h"][b] >= a["ub"] - 1e-9))
            resid = np.abs(y - a["b0"]).max()
            print(f"n={n} {name}[{b}] active_frac={act:.2f} level0_resid={resid:.2e}")
        pre = f"{name}__"
        for k, v in inp.items():
            out[pre + k] = v
        out[pre + "tau"] = np.array(taus)
        out[pre + "y0"] = np.array(ys)
        out[pre + "status"] = np.zeros(count, np.int32)
        if len(kats) == count:
            out[pre + "kat"] = np.array(kats)
        out[pre + "tau_max"] = prob.tau_max
        out[pre + "select_mode"] = np.int32(prob.select_mode)
        out[pre + "joint_weight"] = np.int32(prob.joint_weight)
        out[pre + "row_mask"] = np.array(prob.row_mask, np.int32)
    out["groups"] = np.array([g[0] for g in GROUPS])
    return out


def main():
    for n, seed in ((7, 1), (30, 2), (39, 3)):
        data = make(n, seed)
        path = os.path.join(HERE, f"qppvm_n{n}.npz")
        np.savez_compressed(path, **data)
        print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
