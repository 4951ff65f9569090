"""Friction level-0 repair sweep (tests/test_gpu_contact_ext.py::test_contact_level0_repair_friction):
list the instances where the GPU and the oracle disagree on the status."""
import sys
import numpy as np
sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
import oracle
from qppvm_amd import wbq
from qppvm_amd.problem import ContactProblem
from qppvm_amd.synth import contact_instances
MASKS4 = [0b0011, 0b0111, 0b1111, 0b0101, 0b1010, 0b1100]
for mu in [float(a) for a in sys.argv[1:]] or [0.3, 0.5]:
    for seed in range(100, 120):
        n, nc = 12, 4
        free = ContactProblem(n=n, nc=nc, mu=mu)
        inp = contact_instances(free, 64, seed=seed, masks=MASKS4)
        tf = oracle.contact_batch(free, inp)[0]
        prob = ContactProblem(n=n, nc=nc, mu=mu, torque_rows=True, tau_max=float(np.quantile(np.abs(tf[:, 6:]), 0.4)))
        tau_r, x_r, st_r, it_r, rep = oracle.contact_batch(prob, inp)
        s = wbq.ContactSolver(prob, max_batch=64)
        tau, st, it = s.solve_batch(inp)
        s.close()
        for b in np.where((st_r == 0) & (st != 0))[0]:
            print(f"MISS mu={mu} seed={seed} b={b} gpu_status={st[b]} gpu_iters={it[b]} oracle_rep={rep[b]} oracle_iters={it_r[b]}", flush=True)
