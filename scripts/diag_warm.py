import sys, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo")); sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "tests"))
import numpy as np
from qppvm_amd import wbq
from qppvm_amd.problem import ContactProblem
from qppvm_amd.synth import contact_instances
MASKS = [0b0011, 0b0111, 0b1111]
free = ContactProblem(n=30, nc=4)
inp = contact_instances(free, 512, seed=1, masks=MASKS)
s = wbq.ContactSolver(free, max_batch=512); tf, _, _ = s.solve_batch(inp); s.close()
prob = ContactProblem(n=30, nc=4, torque_rows=True, tau_max=float(np.quantile(np.abs(tf[:, 6:]), 0.85)))
w = wbq.ContactSolver(prob, max_batch=512)
t1, s1, i1 = w.solve_batch(inp)
t2, s2, i2 = w.solve_batch(inp)   # same inputs: warm = previous final set exactly
c = wbq.ContactSolver(prob, max_batch=512); tc, sc, ic = c.solve_batch(inp); c.close()
e = np.abs(t2 - tc).max(axis=1) / np.maximum(1, np.abs(tc).max(axis=1))
bad = np.where((e > 1e-9) | (s2 != sc))[0]
print("same-input warm: bad", len(bad), "of 512; iters cold mean", ic.mean(), "warm mean", i2.mean())
for b in bad[:10]:
    print(b, "st", s2[b], sc[b], "it", i2[b], ic[b], "err", e[b], "cmask", inp["cmask"][b])
# the same with the register-slot variant (no torque rows) and W1 = M
for tr in (False,):
    p2 = ContactProblem(n=30, nc=4)
    w = wbq.ContactSolver(p2, max_batch=512); w.solve_batch(inp); t2, s2, i2 = w.solve_batch(inp); w.close()
    c = wbq.ContactSolver(p2, max_batch=512); tc, sc, ic = c.solve_batch(inp); c.close()
    e = np.abs(t2 - tc).max(axis=1) / np.maximum(1, np.abs(tc).max(axis=1))
    print("no torque rows: bad", int(((e > 1e-9) | (s2 != sc)).sum()), "iters cold", ic.mean(), "warm", i2.mean())
from qppvm_amd.problem import QPPVMProblem
from qppvm_amd.synth import qppvm_instances
qi = qppvm_instances(QPPVMProblem(n=30, joint_weight=1), 512, seed=3)
s = wbq.QPPVMSolver(QPPVMProblem(n=30, tau_max=1e9, joint_weight=1), max_batch=512); tf, _, _ = s.solve_batch(qi); s.close()
pm = QPPVMProblem(n=30, tau_max=float(np.quantile(np.abs(tf), 0.8)), joint_weight=1)
w = wbq.QPPVMSolver(pm, max_batch=512); w.solve_batch(qi); t2, s2, i2 = w.solve_batch(qi); w.close()
c = wbq.QPPVMSolver(pm, max_batch=512); tc, sc, ic = c.solve_batch(qi); c.close()
e = np.abs(t2 - tc).max(axis=1) / np.maximum(1, np.abs(tc).max(axis=1))
print("W1 = M: bad", int(((e > 1e-9) | (s2 != sc)).sum()), "iters cold", ic.mean(), "warm", i2.mean())
