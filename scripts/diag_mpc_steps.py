"""Config-4 rollouts step by step (GPU): one launch per step through the separate repair kernel, so
every step's iteration counts (iters = BVLS steps + dual active-set steps of the repaired instances) and
wall time can be read. Saves the (q, qd) before the step of the instances with the most iterations to
gpurun_out/mpc_worst.npz for an offline replay against the oracle."""
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


def main():
    if len(sys.argv) > 1:  # an alternative build (experiments)
        wbq.load_library(os.path.abspath(sys.argv[1]))
    n, B, H = 30, 4096, 20
    inp = qppvm_instances(QPPVMProblem(n=n), B, seed=1, plant=True)
    free = wbq.QPPVMSolver(QPPVMProblem(n=n, tau_max=1e9), max_batch=B)
    tau_free, _, _ = free.solve_batch(inp)
    free.close()
    tm = float(np.quantile(np.abs(tau_free), 0.8))
    prob = QPPVMProblem(n=n, tau_max=tm)
    out = {"tau_max": tm, "steps": []}
    worst = {}
    for inl in (0, 1):
        s = wbq.QPPVMSolver(prob, max_batch=B)
        s.set_option(s.OPT_FUSED_ROLLOUT, 0)
        s.set_option(s.OPT_INLINE_REPAIR, inl)
        s.set_inputs(inp)
        s.rollout(1, 1e-3)
        s.sync()
        s.set_state(inp["q"], inp["qd"])
        s.reset_warmstart()
        s.sync()
        rows = []
        for k in range(H):
            q0, qd0 = s.state()
            hints0 = s.warm_hints()
            t0 = time.perf_counter()
            s.rollout(1, 1e-3)
            s.sync()
            dt = time.perf_counter() - t0
            _, st, it = s.outputs()
            rep = s.warm_hints()
            r = {"step": k, "ms": 1e3 * dt, "status_bad": int((st != 0).sum()), "iters_max": int(it.max()),
                 "iters_p99": float(np.quantile(it, 0.99)), "hint_repair": int((rep & 1).sum()),
                 "iters_sum": int(it.sum())}
            rows.append(r)
            if inl == 0:
                b = int(np.argmax(it))
                if it[b] > worst.get("iters", -1):
                    worst = {"iters": int(it[b]), "b": b, "step": k, "q": q0[b].copy(), "qd": qd0[b].copy(),
                             "hint": int(hints0[b]), "iters_all": it.copy()}
        out["steps_inline" if inl else "steps_kernel"] = rows
        s.close()
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.savez(os.path.join(ROOT, "gpurun_out", "mpc_worst.npz"), b=worst["b"], step=worst["step"], q=worst["q"],
             qd=worst["qd"], hint=worst["hint"], iters=worst["iters"], iters_all=worst["iters_all"], tau_max=tm)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
