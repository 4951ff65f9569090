"""GPU diagnostic: W1 = M config-2 batch, instances failing the KAT-4 certificate, with the
oracle's answer beside (not a test)."""
import sys

import numpy as np

ROOT = __file__.rsplit("/scripts/", 1)[0]
sys.path.insert(0, ROOT)
sys.path.insert(0, ROOT + "/tests")
import kkt  # noqa: E402
import oracle  # noqa: E402
from qppvm_amd import wbq  # noqa: E402
from qppvm_amd.problem import QPPVMProblem, WEIGHT_INERTIA  # noqa: E402
from qppvm_amd.synth import qppvm_instances  # noqa: E402

n, B = 30, 4096
inp = qppvm_instances(QPPVMProblem(n=n), B, seed=1)
s = wbq.QPPVMSolver(QPPVMProblem(n=n, tau_max=1e9, joint_weight=WEIGHT_INERTIA), max_batch=B)
t0, _, _ = s.solve_batch(inp)
s.close()
prob = QPPVMProblem(n=n, tau_max=float(np.quantile(np.abs(t0), 0.8)), joint_weight=WEIGHT_INERTIA)
s = wbq.QPPVMSolver(prob, max_batch=B)
tau, st, it = s.solve_batch(inp)
s.close()
bad = []
for b in range(B):
    c = kkt.qppvm_certificate(oracle, prob, inp, b, tau[b])
    if max(c["primal"], c["level0"], c["stat"], c["sign"]) > 1e-9:
        bad.append(b)
print("bad", len(bad), "of", B)
sub = {k: v[bad] for k, v in inp.items()}
tr, sr, ir = oracle.qppvm_batch(prob, sub)
for j, b in enumerate(bad[:20]):
    gap = np.abs(oracle.qppvm_one(prob, inp, b)[1] - oracle.assemble(prob, inp, b)["b0"]).max()
    e = np.abs(tau[b] - tr[j]).max() / max(1, np.abs(tr[j]).max())
    c = kkt.qppvm_certificate(oracle, prob, inp, b, tau[b])
    print(b, "st", st[b], sr[j], "it", it[b], ir[j], "err %.2e gap %.2e" % (e, gap),
          {k: "%.1e" % v for k, v in c.items() if k != "indep"})
# the same instances alone (batch of the bad ones): does the failure depend on the batch?
s = wbq.QPPVMSolver(prob, max_batch=len(bad))
tau2, st2, it2 = s.solve_batch(sub)
s.close()
print("alone: err", [float("%.2e" % (np.abs(tau2[j] - tr[j]).max() / max(1, np.abs(tr[j]).max()))) for j in range(min(20, len(bad)))])
