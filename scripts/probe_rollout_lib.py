"""Experiment probe (GPU): load an alternative libwbq build (argv[1]), check the fused rollout against
per-step launches through the separate repair kernel (bit-equal tau / q / qd), then time both on the
config-4 and repair-free rollouts (4096 x 20)."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from qppvm_amd import wbq  # noqa: E402
from qppvm_amd.problem import QPPVMProblem  # noqa: E402
from qppvm_amd.synth import qppvm_instances  # noqa: E402


def run(prob, inp, fused, H, reps=0):
    s = wbq.QPPVMSolver(prob, max_batch=inp["h"].shape[0])
    s.set_option(s.OPT_FUSED_ROLLOUT, fused)
    s.set_option(s.OPT_INLINE_REPAIR, 0)
    s.set_inputs(inp)
    s.rollout(H, 1e-3)
    tau, st, it = s.outputs()
    q, qd = s.state()
    ts = []
    for _ in range(reps):
        s.set_state(inp["q"], inp["qd"])
        s.reset_warmstart()
        s.sync()
        t0 = time.perf_counter()
        s.rollout(H, 1e-3)
        s.sync()
        ts.append(time.perf_counter() - t0)
    s.close()
    return tau, st, q, qd, (1e3 * float(np.median(ts)) if ts else None)


def main():
    wbq.load_library(os.path.abspath(sys.argv[1]))
    out = {}
    small = qppvm_instances(QPPVMProblem(n=30), 48, seed=120)
    for tm in (1e6, 40.0):
        prob = QPPVMProblem(n=30, tau_max=tm)
        a = run(prob, small, 1, 6)
        b = run(prob, small, 0, 6)
        out[f"small_tm{tm}"] = {"st_equal": bool(np.array_equal(a[1], b[1])),
                                "tau_maxdiff": float(np.abs(a[0] - b[0]).max()),
                                "q_maxdiff": float(np.abs(a[2] - b[2]).max()), "bad": int((a[1] != 0).sum())}
        print(json.dumps(out), flush=True)
    n, B = 30, 4096
    inp = qppvm_instances(QPPVMProblem(n=n), B, seed=1, plant=True)
    free = wbq.QPPVMSolver(QPPVMProblem(n=n, tau_max=1e9), max_batch=B)
    tau_free, _, _ = free.solve_batch(inp)
    free.close()
    for name, tm in (("repair_free", 1e9), ("config4", float(np.quantile(np.abs(tau_free), 0.8)))):
        prob = QPPVMProblem(n=n, tau_max=tm)
        a = run(prob, inp, 1, 20, reps=5)
        b = run(prob, inp, 0, 20, reps=5)
        out[name] = {"fused_ms": a[4], "steps_kernel_ms": b[4], "st_equal": bool(np.array_equal(a[1], b[1])),
                     "tau_maxdiff": float(np.abs(a[0] - b[0]).max())}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
