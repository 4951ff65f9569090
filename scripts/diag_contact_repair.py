"""GPU diagnostic (not a test): the degenerate contact regime of tests/test_gpu_contact.py
(test_contact_level0_repair: 6 actuated joints, torque limits at the 40 % quantile, where the
waist task is often out of reach) against the oracle, over many seeds: per seed how many
instances the oracle solves (and repairs), and how many of those the GPU does not match; with
-v the per-instance lines.
    python scripts/diag_contact_repair.py [n] [q] [seed0] [seeds] [-v]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import kkt  # noqa: E402
import oracle  # noqa: E402
from qppvm_amd import wbq  # noqa: E402
from qppvm_amd.problem import ContactProblem  # noqa: E402
from qppvm_amd.synth import contact_instances  # noqa: E402

args = [a for a in sys.argv[1:] if a != "-v"]
n = int(args[0]) if len(args) > 0 else 12
q = float(args[1]) if len(args) > 1 else 0.4
seed0 = int(args[2]) if len(args) > 2 else 100
seeds = int(args[3]) if len(args) > 3 else 20
MASKS4 = [0b0011, 0b0111, 0b1111, 0b0101, 0b1010, 0b1100]
tot = dict(solved=0, repaired=0, miss=0, miss_rep=0, wrong_st0=0, gpu_only=0, gpu_only_cert_bad=0)
for seed in range(seed0, seed0 + seeds):
    free = ContactProblem(n=n, nc=4)
    inp = contact_instances(free, 64, seed=seed, masks=MASKS4)
    tau_free = oracle.contact_batch(free, inp)[0]
    prob = ContactProblem(n=n, nc=4, torque_rows=True, tau_max=float(np.quantile(np.abs(tau_free[:, 6:]), q)))
    tau_r, x_r, st_r, it_r, rep = oracle.contact_batch(prob, inp)
    s = wbq.ContactSolver(prob, max_batch=64)
    tau, st, it = s.solve_batch(inp)
    xgpu = s.x()
    s.close()
    e = np.abs(tau - tau_r).max(axis=1) / np.maximum(1.0, np.abs(tau_r).max(axis=1))
    solved = st_r == 0
    miss = solved & ((st != 0) | (e > 1e-6))
    tot["solved"] += int(solved.sum())
    tot["repaired"] += int((solved & (rep != 0)).sum())
    tot["miss"] += int(miss.sum())
    tot["miss_rep"] += int((miss & (rep != 0)).sum())
    tot["gpu_only"] += int((~solved & (st == 0)).sum())
    tot["wrong_st0"] += int((miss & (st == 0)).sum())  # a wrong tau reported as solved
    # instances only the GPU solves: KAT-4 certificates of level 0 and level 1 (tests/kkt.py)
    for b in np.where(~solved & (st == 0))[0]:
        x = xgpu[b]
        l0, y = kkt.contact_level0_certificate(oracle, prob, inp, b, x)
        c = kkt.contact_certificate(oracle, prob, inp, b, x, waist=y)
        if l0 > 1e-9 or c["primal"] > 1e-9 or c["stat"] > 1e-9 or c["sign"] > 1e-9:
            tot["gpu_only_cert_bad"] += 1
            print(f"  b={b}: GPU-only solution fails its certificate: level0 {l0:.2e} {c}")
    print(f"seed {seed}: oracle solves {int(solved.sum())} (repaired {int((solved & (rep != 0)).sum())}), "
          f"GPU misses {int(miss.sum())} {[(int(b), int(st[b])) for b in np.where(miss)[0]]}, "
          f"GPU solves where the oracle fails "
          f"{int((~solved & (st == 0)).sum())}", flush=True)
    if "-v" in sys.argv:
        for b in range(64):
            print(f"  b={b} gpu st={st[b]} it={it[b]} | oracle st={st_r[b]} rep={rep[b]} | err={e[b]:.2e}")
print("total", tot)
