"""Experiment probe (GPU): the config-2 certificate scenario of tests/test_gpu_kkt.py with an alternative
libwbq build (argv[1]); prints the instances whose level-0 certificate fails, with their iterations."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import kkt  # noqa: E402
import oracle  # noqa: E402
from qppvm_amd import wbq  # noqa: E402
from qppvm_amd.problem import QPPVMProblem  # noqa: E402
from qppvm_amd.synth import qppvm_instances  # noqa: E402


def gpu(prob, inp):
    s = wbq.QPPVMSolver(prob, max_batch=inp["h"].shape[0])
    out = s.solve_batch(inp)
    hints = s.warm_hints()
    s.close()
    return out, hints


def main():
    wbq.load_library(os.path.abspath(sys.argv[1]))
    ol = oracle
    n, B, w = 30, 4096, int(sys.argv[2]) if len(sys.argv) > 2 else 0
    inp = qppvm_instances(QPPVMProblem(n=n), B, seed=1)
    (t0, _, _), _ = gpu(QPPVMProblem(n=n, tau_max=1e9, joint_weight=w), inp)
    prob = QPPVMProblem(n=n, tau_max=float(np.quantile(np.abs(t0), 0.8)), joint_weight=w)
    (tau, st, it), hints = gpu(prob, inp)
    tr, str_, itr = ol.qppvm_batch(prob, inp)
    bad = []
    for b in range(B):
        c = kkt.qppvm_certificate(ol, prob, inp, b, tau[b])
        if max(c["primal"], c["level0"], c["stat"], c["sign"]) > 1e-9:
            bad.append({"b": b, "st": int(st[b]), "it": int(it[b]), "hint": int(hints[b]), "oracle_it": int(itr[b]),
                        "tau_err": float(np.abs(tau[b] - tr[b]).max()), **{k: float(v) for k, v in c.items()}})
    print(json.dumps({"lib": sys.argv[1], "nbad": len(bad), "repaired": int(hints.sum()), "bad": bad[:10]}))


if __name__ == "__main__":
    main()
