"""CPU emulation (numpy) of the W1 = M kernel's algorithm (qppvm_amd/csrc/qppvm_w1m_kernel.hip
+ dual_gi.h): Goldfarb-Idnani dual active set in constraint space with
Gamma = [G M^-1 G^T, G; G^T, M], x0 = tau_imp, equality rows added when violated and never
dropped. Compares with the oracle on the instances of tests/test_gpu_w1m.py. Diagnostic
only (not a test, not the product path)."""
import sys

import numpy as np

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
import oracle  # noqa: E402
from qppvm_amd.problem import QPPVMProblem, WEIGHT_INERTIA  # noqa: E402
from qppvm_amd.synth import qppvm_instances  # noqa: E402


def dual_gi(Gam, s0, lo, hi, maxit=200):
    m = len(s0)
    s = s0.copy()
    act, sgn, lam, aeq = [], [], [], []
    nrm = np.sqrt(np.maximum(np.diag(Gam), 1e-300))
    it = 0
    while True:
        viol = np.maximum(lo - s, s - hi)
        tol = 1e-10 * np.maximum(1, np.maximum(abs(s), np.maximum(abs(lo), abs(hi))))
        v = np.where((viol > tol) & ~np.isin(np.arange(m), act), viol / nrm, -1.0)
        p = int(np.argmax(v))
        if v[p] <= 0:
            return s, act, sgn, lam, 0, it
        sp = 1.0 if lo[p] - s[p] > s[p] - hi[p] else -1.0
        bnd = lo[p] if sp > 0 else hi[p]
        peq = lo[p] == hi[p]
        lamp = 0.0
        while True:
            it += 1
            if it > maxit:
                return s, act, sgn, lam, 1, it
            k = len(act)
            N = np.array([[sgn[a] * sgn[b] * Gam[act[a], act[b]] for b in range(k)] for a in range(k)]).reshape(k, k)
            vv = np.array([sgn[a] * sp * Gam[act[a], p] for a in range(k)])
            r = np.linalg.solve(N, vv) if k else np.zeros(0)
            ds = sp * Gam[:, p] - (Gam[:, act] @ (np.array(sgn) * r) if k else 0)
            zz = sp * ds[p]
            slack = sp * (s[p] - bnd)
            cand = [lam[a] / r[a] if (not aeq[a] and r[a] > 1e-13 * max(abs(r).max(), 0)) else np.inf for a in range(k)]
            t1 = min(cand) if k else np.inf
            blk = int(np.argmin(cand)) if k else -1
            t2 = -slack / zz if zz > 1e-10 * Gam[p, p] else np.inf
            if t1 == np.inf and t2 == np.inf:
                return s, act, sgn, lam, 2, it
            t = min(t1, t2)
            s = s + t * ds
            lam = [lam[a] - t * r[a] for a in range(k)]
            lamp += t
            if t2 <= t1:
                act.append(p); sgn.append(sp); lam.append(lamp); aeq.append(peq)
                break
            del act[blk], sgn[blk], lam[blk], aeq[blk]


def w1m_solve(prob, inp, b):
    n, m0 = prob.n, prob.m0
    M, h = inp["M"][b], inp["h"][b]
    a = oracle.assemble(prob, inp, b)
    A0, b0, lb, ub = a["A0"], a["b0"], a["lb"], a["ub"]
    G = A0 @ M  # A0 = G M^-1
    timp = -np.linalg.solve(a["H1"], a["g1"])  # H1 = M^-1, g1 = -M^-1 tau_imp
    Xg = np.linalg.solve(M, G.T)
    Gam = np.block([[G @ Xg, G], [G.T, M]])
    s0 = np.concatenate([G @ np.linalg.solve(M, timp), timp])
    lo = np.concatenate([b0, lb]); hi = np.concatenate([b0, ub])
    s, act, sgn, lam, st, it = dual_gi(Gam, s0, lo, hi)
    x = timp.copy()
    HA = np.concatenate([G, M], axis=0)  # rows: (H^-1 A^T)^T
    for c, sg, l in zip(act, sgn, lam):
        x += sg * l * HA[c]
    return x + h, st, it


if __name__ == "__main__":
    n, frac = 30, 0.1
    free = QPPVMProblem(n=n, tau_max=1e9, joint_weight=WEIGHT_INERTIA)
    inp = qppvm_instances(free, 48, seed=600 + n)
    tau0, _, _ = oracle.qppvm_batch(free, inp)
    prob = QPPVMProblem(n=n, tau_max=float(np.quantile(np.abs(tau0), 1 - frac)), joint_weight=WEIGHT_INERTIA)
    tau_r, st_r, _ = oracle.qppvm_batch(prob, inp)
    worst = 0
    for b in range(48):
        tau, st, it = w1m_solve(prob, inp, b)
        if st == 2:  # level 0 not attainable at b0: the kernel hands this one to the repair
            print(b, "-> level-0 repair")
            continue
        e = np.abs(tau - tau_r[b]).max() / max(1, np.abs(tau_r[b]).max())
        worst = max(worst, e)
        if e > 1e-6:
            print(b, st, st_r[b], it, "%.3e" % e)
    print("worst %.3e" % worst)
