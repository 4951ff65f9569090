"""Generate the golden fixtures of the QPPVM stacks with the elbow level (run in the build container).

The elbow tasks the reference builds (QPPVMPlugin.cpp:154-166 _elbow_task_left/right) and the stack
its commented line :178 closes in place of :179:
    ((ee_r + ee_l) / (elbow_l + elbow_r)) << torque_limits          (no joint task; --literal)
i.e. task_level (0, 0, 1, 1) over four Cartesian impedance tasks and no_joint_task = 1 (include/wbq.h):
the last level's x is the minimum-norm point among its optima (the eps -> 0 limit of QPOases_sot's
regularisation, :188), min ||x||^2 over {A0 x = y0*, A1 x = y1*, box}. And the three-level extension
that keeps the joint task after the elbows:
    ((ee_r + ee_l) / (elbow_l + elbow_r)) / joint << torque_limits
An *independent* numpy/scipy restatement that shares no code with oracle/wbq_oracle.c or the HIP
kernels, built on the two-level generator (make_golden.py: its assembly, level-0 BVLS and level-1
active set):

* level 0 over the first two tasks' rows: scipy.optimize.lsq_linear(method="bvls") -> y0*;
* the middle level min ||A1 x - b1||^2 s.t. A0 x = y0*, box (level-0 pins fixed): a monotone primal
  active set whose equality-constrained steps are null-space least squares (pinv), accepted only with
  a KKT certificate (stationarity modulo the equality rows, multiplier signs) -> y1*;
* the last level over {A0 x = y0*, A1 x = y1*, box, pins} by make_golden.level1_np: the joint task
  (H1, g1), or without it min 0.5 ||x||^2 (H = I, g = 0);
* bounds-inactive groups carry a closed form with the stacked 12-row A = G M^-1 (every level
  attained), which the lexicographic answer must equal: KAT-1 with the joint task, the
  pseudo-inverse x = A^T (A A^T)^-1 b without it.

Output: tests/golden/qppvm_elbow.npz (three levels) or, with --literal, tests/golden/
qppvm_elbow_literal.npz (no joint task); groups per n in {14, 30, 39}.
Usage: python tests/golden/make_golden_elbow.py [--literal]
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from make_golden import _null, assemble_np, kat, level0_np, level1_np  # noqa: E402
from qppvm_amd.problem import QPPVMProblem  # noqa: E402
from qppvm_amd.synth import qppvm_instances  # noqa: E402

TASKS = dict(ntasks=4, row_mask=(7, 7, 7, 7), task_level=(0, 0, 1, 1))


def level_mid_np(A1, b1, E, e, lb, ub, x0, maxit=2000):
    """min 0.5 ||A1 x - b1||^2 s.t. E x = e, lb <= x <= ub from the feasible x0: monotone primal
    active set, null-space EQP steps by pseudo-inverse (the objective is only semidefinite)."""
    n = A1.shape[1]
    x = np.clip(x0.copy(), lb, ub)
    lo = x <= lb
    hi = (x >= ub) & ~lo
    stationary = False
    scale = max(1.0, np.abs(A1.T @ b1).max())
    for _ in range(maxit):
        F = ~(lo | hi)
        k = int(F.sum())
        r = b1 - A1 @ x
        Z = _null(E[:, F], k)
        p = np.zeros(n)
        if Z.shape[1]:
            B = A1[:, F] @ Z
            p[F] = Z @ (np.linalg.pinv(B, rcond=1e-12) @ r)
        if stationary or np.abs(p).max() <= 1e-12 * max(1.0, np.abs(x).max()):
            stationary = False
            g = -(A1.T @ r)  # gradient
            nu = np.linalg.lstsq(E[:, F].T, -g[F], rcond=None)[0] if k else np.zeros(E.shape[0])
            lam = g + E.T @ nu  # lambda_lo - lambda_hi on bound variables
            wrong = np.where(lo & (lb < ub), -lam, np.where(hi, lam, -np.inf))
            if wrong.max() <= 1e-10 * scale:
                assert np.abs(lam[F]).max(initial=0.0) <= 1e-7 * scale
                assert np.abs(E @ x - e).max() <= 1e-8 * max(1.0, np.abs(e).max())
                assert np.all(x >= lb) and np.all(x <= ub)
                return x, lam
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
    raise RuntimeError("middle-level active set did not converge")


def solve3_np(prob, inp, b):
    """The elbow stack: level 0, the elbow level, then the joint task (prob.joint_task) or the
    minimum-norm x."""
    a = assemble_np(prob, inp, b)  # rows in task order: tasks 0, 1 (level 0), then 2, 3 (level 1)
    ml = prob.m_l0
    A0, b0, A1, b1 = a["A0"][:ml], a["b0"][:ml], a["A0"][ml:], a["b0"][ml:]
    x0, y0 = level0_np(A0, b0, a["lb"], a["ub"])
    w = A0.T @ (b0 - y0)
    tol = 1e-9 * max(1.0, np.abs(A0.T @ b0).max())
    lb1, ub1 = a["lb"].copy(), a["ub"].copy()
    lb1[w > tol] = ub1[w > tol]
    ub1[w < -tol] = lb1[w < -tol]
    x0 = np.clip(x0, lb1, ub1)
    x1, lam = level_mid_np(A1, b1, A0, y0, lb1, ub1, x0)
    y1 = A1 @ x1
    tol1 = 1e-9 * max(1.0, np.abs(A1.T @ b1).max())
    at_lo, at_hi = x1 <= lb1, x1 >= ub1
    lb2, ub2 = lb1.copy(), ub1.copy()
    up = at_hi & (lam < -tol1)   # held at the upper bound by the middle level
    dn = at_lo & (lam > tol1)
    lb2[up] = ub2[up]
    ub2[dn] = lb2[dn]
    Aeq, beq = np.vstack([A0, A1]), np.concatenate([y0, y1])
    if prob.joint_task:
        x = level1_np(a["H1"], a["g1"], Aeq, beq, lb2, ub2, np.clip(x1, lb2, ub2))
    else:  # min 0.5 ||x||^2: the gradient is x itself
        gs = max(1.0, np.abs(a["lb"]).max(), np.abs(a["ub"]).max(), np.abs(x1).max())
        x = level1_np(np.eye(prob.n), np.zeros(prob.n), Aeq, beq, lb2, ub2, np.clip(x1, lb2, ub2), gscale=gs)
    return x + inp["h"][b], beq, a


GROUPS = [
    # name, count, tau_max quantile of the unconstrained |tau| (None: 1e6, bounds inactive)
    ("inactive", 3, None),
    ("active", 3, 0.8),
    ("heavy", 3, 0.4),
    ("tight", 3, 0.12),
]


def kat_minnorm(inp, b, a):
    """Bounds inactive, every level attained, no joint task: the minimum-norm solution of the 12
    stacked rows A x = b (A = G M^-1, the pseudo-inverse)."""
    A, y = a["A0"], a["b0"]
    return A.T @ np.linalg.solve(A @ A.T, y) + inp["h"][b]


def make(n, seed, joint=True):
    out = {}
    for gi, (name, count, q) in enumerate(GROUPS):
        probe = QPPVMProblem(n=n, tau_max=1e6, joint_task=joint, **TASKS)
        inp = qppvm_instances(probe, count, seed=seed * 100 + gi)
        if q is None:
            prob = probe
        else:
            t0 = np.concatenate([solve3_np(probe, inp, b)[0] for b in range(count)])
            prob = QPPVMProblem(n=n, tau_max=float(np.quantile(np.abs(t0), q)), joint_task=joint, **TASKS)
        taus, ys, kats = [], [], []
        for b in range(count):
            tau, y, a = solve3_np(prob, inp, b)
            taus.append(tau)
            ys.append(y)
            if q is None:
                k = kat(prob, inp, b, a) if joint else kat_minnorm(inp, b, a)  # the 12 rows all attained
                assert np.abs(k - tau).max() <= 1e-8 * max(1, np.abs(k).max()), name
                kats.append(k)
            act = np.mean((tau - inp["h"][b] <= a["lb"] + 1e-9) | (tau - inp["h"][b] >= a["ub"] - 1e-9))
            print(f"n={n} {name}[{b}] active_frac={act:.2f} level-1 resid={np.abs(y[6:] - a['b0'][6:]).max():.2e}")
        pre = f"n{n}_{name}__"
        for k, v in inp.items():
            out[pre + k] = v
        out[pre + "tau"] = np.array(taus)
        out[pre + "y"] = np.array(ys)
        if kats:
            out[pre + "kat"] = np.array(kats)
        out[pre + "tau_max"] = prob.tau_max
        out[pre + "n"] = np.int32(n)
    return out


def main():
    literal = "--literal" in sys.argv
    data, groups = {}, []
    seeds = ((14, 21), (30, 22), (39, 23)) if literal else ((14, 11), (30, 12), (39, 13))
    for n, seed in seeds:
        d = make(n, seed, joint=not literal)
        data.update(d)
        groups += [f"n{n}_{g[0]}" for g in GROUPS]
    data["groups"] = np.array(groups)
    path = os.path.join(HERE, "qppvm_elbow_literal.npz" if literal else "qppvm_elbow.npz")
    np.savez_compressed(path, **data)
    print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
