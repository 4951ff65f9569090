"""GPU diagnostic (not a test): the config-4 MPC workload of bench.py (4096 plant-scaled rollouts x
20 steps, limits at the 80 % quantile), step by step and repeated from the reset state as the bench
repeats it (the warm-start state carries over), recording every step's status. Instances that end
with a status != 0 are re-solved by the oracle from the same step inputs; their inputs go to
gpurun_out/mpc_fail.npz.
    python scripts/diag_mpc.py [repeats]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import oracle  # noqa: E402
from qppvm_amd.problem import QPPVMProblem  # noqa: E402
from qppvm_amd.synth import qppvm_instances  # noqa: E402
from qppvm_amd.wbq import QPPVMSolver  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
n, B, H, dt = 30, 4096, 20, 1e-3
inp = qppvm_instances(QPPVMProblem(n=n), B, seed=1, plant=True)
free = QPPVMSolver(QPPVMProblem(n=n, tau_max=1e9), max_batch=B)
tau_free, _, _ = free.solve_batch(inp)
free.close()
prob = QPPVMProblem(n=n, tau_max=float(np.quantile(np.abs(tau_free), 0.8)))
s = QPPVMSolver(prob, max_batch=B)
s.set_inputs(inp)
fails = []
hist = {}
for r in range(reps):
    s.set_state(inp["q"], inp["qd"])
    for k in range(H):
        q, qd = s.state()
        s.rollout(1, dt)
        tau, st, it = s.outputs()
        for v in np.unique(st):
            hist[int(v)] = hist.get(int(v), 0) + int((st == v).sum())
        for b in np.where(st != 0)[0]:
            one = {f: inp[f][b:b + 1].copy() for f in inp}
            one["q"], one["qd"] = q[b:b + 1], qd[b:b + 1]
            t_r, st_r, _ = oracle.qppvm_batch(prob, one)
            print(f"repeat {r} step {k} b {b}: gpu status {st[b]} iters {it[b]} | oracle status {st_r[0]}", flush=True)
            fails.append((r, k, int(b), int(st[b]), int(st_r[0]), one))
print("status histogram over all steps", hist, "tau_max", prob.tau_max[0])
if fails:
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    out = {"meta": np.array([f[:5] for f in fails]), "tau_max": prob.tau_max}
    for j, f in enumerate(fails):
        for key, v in f[5].items():
            out[f"{j}_{key}"] = v
    np.savez(os.path.join(ROOT, "gpurun_out", "mpc_fail.npz"), **out)
