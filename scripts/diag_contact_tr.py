"""GPU diagnostic (not a test): the torque-row contact case of tests/test_gpu_contact.py
(test_contact_torque_rows) against the oracle, optionally with another build of libwbq.
Prints the instances whose status or torques differ, with the GPU iteration count.
    python scripts/diag_contact_tr.py [n] [q] [nc] [lib.so]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402  (torch's HIP runtime first, as in bench.py)

torch.cuda.init()

import oracle  # noqa: E402
from qppvm_amd import wbq  # noqa: E402
from qppvm_amd.problem import ContactProblem  # noqa: E402
from qppvm_amd.synth import contact_instances  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 12
q = float(sys.argv[2]) if len(sys.argv) > 2 else 0.8
nc = int(sys.argv[3]) if len(sys.argv) > 3 else 4
if len(sys.argv) > 4:
    wbq.load_library(os.path.abspath(sys.argv[4]))
MASKS4 = [0b0011, 0b0111, 0b1111, 0b0101, 0b1010, 0b1100]  # as tests/test_gpu_contact.py
free = ContactProblem(n=n, nc=nc)
inp = contact_instances(free, 64, seed=70 + n, masks=MASKS4 if nc == 4 else None)
tau_free = oracle.contact_batch(free, inp)[0]
prob = ContactProblem(n=n, nc=nc, torque_rows=True, tau_max=float(np.quantile(np.abs(tau_free[:, 6:]), q)))
tau_r, x_r, st_r, it_r, rep = oracle.contact_batch(prob, inp)
s = wbq.ContactSolver(prob, max_batch=64)
tau, st, it = s.solve_batch(inp)
s.close()
bad = 0
for b in range(64):
    e = np.abs(tau[b] - tau_r[b]).max() / max(1.0, np.abs(tau_r[b]).max())
    if st[b] != (2 if rep[b] else st_r[b]) or (st[b] == 0 and e > 1e-6):
        bad += 1
        print(b, "gpu st", st[b], "it", it[b], "oracle st", st_r[b], "rep", rep[b], "err %.3e" % e,
              "mask", bin(int(inp["cmask"][b])))
print(f"n={n} q={q} nc={nc} lib={sys.argv[4] if len(sys.argv) > 4 else 'product'}: {bad} mismatches of 64")
