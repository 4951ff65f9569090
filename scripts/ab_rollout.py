"""A/B of the MPC rollout paths on one box (GPU): one launch per rollout (qppvm_rollout_kernel) vs one
launch per step (inline repair forced / the separate repair kernel), on repair-free rollouts (limits
far away: the common path alone) and on the bench's config-4 rollouts (plant inputs, 80 % quantile
limits). Prints ms per 20-step rollout of 4096 instances."""
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


def time_rollouts(prob, inp, fused, inl, reps=5, H=20):
    s = wbq.QPPVMSolver(prob, max_batch=inp["h"].shape[0])
    s.set_option(s.OPT_FUSED_ROLLOUT, fused)
    s.set_option(s.OPT_INLINE_REPAIR, inl)
    s.set_inputs(inp)
    s.rollout(H, 1e-3)
    s.sync()
    ts = []
    for _ in range(reps):
        s.set_state(inp["q"], inp["qd"])
        s.sync()
        t0 = time.perf_counter()
        s.rollout(H, 1e-3)
        s.sync()
        ts.append(time.perf_counter() - t0)
    hints = s.warm_hints()
    s.close()
    return 1e3 * float(np.median(ts)), float(hints.mean())


def main():
    n, B = 30, 4096
    inp = qppvm_instances(QPPVMProblem(n=n), B, seed=1, plant=True)
    free = wbq.QPPVMSolver(QPPVMProblem(n=n, tau_max=1e9), max_batch=B)
    tau_free, _, _ = free.solve_batch(inp)
    free.close()
    out = {}
    for name, tm in (("repair_free", 1e9), ("config4", float(np.quantile(np.abs(tau_free), 0.8)))):
        prob = QPPVMProblem(n=n, tau_max=tm)
        for path, fused, inl in (("fused", 1, -1), ("steps_inline", 0, 1), ("steps_kernel", 0, 0)):
            ms, rep = time_rollouts(prob, inp, fused, inl)
            out[f"{name}/{path}"] = {"ms_per_rollout": ms, "last_step_repair_share": rep}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
