"""GPU diagnostic (not a test): solve the degenerate contact regime of
scripts/diag_contact_repair.py for the given seeds and save the GPU outputs (x, tau, status,
iters) to gpurun_out/contact_dump.npz for CPU-side analysis (scripts/emulate_dual_gi.py).
    python scripts/diag_contact_dump.py n q seed [seed ...]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import oracle  # noqa: E402
from qppvm_amd import wbq  # noqa: E402
from qppvm_amd.problem import ContactProblem  # noqa: E402
from qppvm_amd.synth import contact_instances  # noqa: E402

n, q = int(sys.argv[1]), float(sys.argv[2])
MASKS4 = [0b0011, 0b0111, 0b1111, 0b0101, 0b1010, 0b1100]
out = {}
for seed in map(int, sys.argv[3:]):
    free = ContactProblem(n=n, nc=4)
    inp = contact_instances(free, 64, seed=seed, masks=MASKS4)
    tau_free = oracle.contact_batch(free, inp)[0]
    prob = ContactProblem(n=n, nc=4, torque_rows=True, tau_max=float(np.quantile(np.abs(tau_free[:, 6:]), q)))
    s = wbq.ContactSolver(prob, max_batch=64)
    tau, st, it = s.solve_batch(inp)
    out[f"x{seed}"], out[f"tau{seed}"], out[f"st{seed}"], out[f"it{seed}"] = s.x(), tau, st, it
    s.close()
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez(os.path.join(ROOT, "gpurun_out", "contact_dump.npz"), **out)
print("saved", sorted(out))
