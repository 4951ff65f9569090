"""GPU diagnostic for the W1 = M kernel: per-instance error / status / iterations against the
oracle on the test_gpu_w1m active-limit case (not a test)."""
import sys

import numpy as np

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
import oracle  # noqa: E402
from qppvm_amd import wbq  # noqa: E402
from qppvm_amd.problem import QPPVMProblem, WEIGHT_INERTIA  # noqa: E402
from qppvm_amd.synth import qppvm_instances  # noqa: E402

n, frac = int(sys.argv[1]) if len(sys.argv) > 1 else 30, float(sys.argv[2]) if len(sys.argv) > 2 else 0.1
if frac > 1:  # absolute torque limit (the level-0 repair cases)
    prob = QPPVMProblem(n=n, tau_max=frac, joint_weight=WEIGHT_INERTIA)
    inp = qppvm_instances(prob, 48, seed=700 + n)
else:
    free = QPPVMProblem(n=n, tau_max=1e9, joint_weight=WEIGHT_INERTIA)
    inp = qppvm_instances(free, 48, seed=600 + n)
    tau0, _, _ = oracle.qppvm_batch(free, inp)
    prob = QPPVMProblem(n=n, tau_max=float(np.quantile(np.abs(tau0), 1 - frac)), joint_weight=WEIGHT_INERTIA)
tau_r, st_r, it_r = oracle.qppvm_batch(prob, inp)
s = wbq.QPPVMSolver(prob, max_batch=48)
tau, st, it = s.solve_batch(inp)
s.close()
for b in range(48):
    e = np.abs(tau[b] - tau_r[b]).max() / max(1, np.abs(tau_r[b]).max())
    gap = np.abs(oracle.qppvm_one(prob, inp, b)[1] - oracle.assemble(prob, inp, b)["b0"]).max()
    print(b, st[b], st_r[b], it[b], it_r[b], "err %.3e gap %.2e" % (e, gap), "BAD" if e > 1e-6 else "")
for b in range(48):
    e = np.abs(tau[b] - tau_r[b]).max() / max(1, np.abs(tau_r[b]).max())
    if e <= 1e-6:
        continue
    a = oracle.assemble(prob, inp, b)
    y0 = oracle.qppvm_one(prob, inp, b)[1]
    H, g, A0, lb, ub = a["H1"], a["g1"], a["A0"], a["lb"], a["ub"]
    for name, t in (("gpu", tau[b]), ("oracle", tau_r[b])):
        x = t - inp["h"][b]
        print(b, name, "f %.10g" % (0.5 * x @ H @ x + g @ x), "eq %.2e" % np.abs(A0 @ x - y0).max(),
              "bviol %.2e" % max((lb - x).max(), (x - ub).max()),
              "at_lo", np.where(np.abs(x - lb) < 1e-9)[0].tolist(), "at_hi", np.where(np.abs(x - ub) < 1e-9)[0].tolist())
