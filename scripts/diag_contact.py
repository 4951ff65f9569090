"""Diagnostics (GPU box): per-phase cycles of the contact-form kernel from the stamp build
(libwbq_diag.so, -DWBQ_STAMPS), for the config-1 variant and config 2."""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from qppvm_amd import wbq  # noqa: E402
from qppvm_amd.problem import ContactProblem  # noqa: E402
from qppvm_amd.synth import contact_instances, replicate  # noqa: E402

PHASES = ["stage", "targets+H", "gauss-jordan", "gamma", "active set+refine", "output"]


def run(prob, inp, reps=10):
    s = wbq.ContactSolver(prob, max_batch=inp["h"].shape[0])
    s.set_inputs(inp)
    s.solve()
    s.sync()
    s.set_timing(True)
    for _ in range(reps):
        s.solve()
    ms, km, cnt = s.get_timing_detail()
    B = inp["h"].shape[0]
    K = 64
    buf = (ctypes.c_ulonglong * (K * B))()
    s.lib.wbq_diag_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    assert s.lib.wbq_diag_stamps(s.ctx, buf, B) == 0
    full = np.frombuffer(buf, dtype=np.uint64).reshape(B, K).astype(np.int64)
    d = np.diff(full[:, :7], axis=1)
    _, status, iters = s.outputs()
    s.close()
    steps = np.maximum(iters, 1)
    return {"us_per_launch": 1e3 * ms / cnt,
            "phase_cycles_mean": {p: float(d[:, k].mean()) for k, p in enumerate(PHASES)},
            "block_cycles_p50_p90": [float(np.percentile(full[:, 6] - full[:, 0], q)) for q in (50, 90)],
            "active_set_cycles_per_step": float((d[:, 4] / steps).mean()),
            "steps_mean_max": [float(iters.mean()), int(iters.max())],
            "refine_rounds_mean": float(full[:, 7].mean()),
            "split_active_set": {"equality batch": float((full[:, 9] - full[:, 4]).mean()),
                                 "warm extend": float((full[:, 8] - full[:, 9]).mean()),
                                 "dual loop + rebuild + refinement": float((full[:, 5] - full[:, 8]).mean())},
            "status_ok": float((status == 0).mean())}


def main():
    diag = os.path.join(ROOT, "qppvm_amd", "libwbq_diag.so")  # built beforehand, in-tree
    if not os.path.exists(diag):
        from qppvm_amd import build
        diag = build.build(force=True, diag=True)
    wbq._lib = None
    wbq.load_library(diag)
    res = {}
    p1 = ContactProblem(n=30, nc=2)
    res["cfg1_nc2"] = run(p1, replicate(contact_instances(p1, 1, seed=0), 4096))
    free = ContactProblem(n=30, nc=4)
    inp = contact_instances(free, 4096, seed=1, masks=[0b0011, 0b0111, 0b1111])
    res["nc4_masks"] = run(free, inp)
    s = wbq.ContactSolver(free, max_batch=4096)
    tau_free, _, _ = s.solve_batch(inp)
    s.close()
    p2 = ContactProblem(n=30, nc=4, torque_rows=True, tau_max=float(np.quantile(np.abs(tau_free[:, 6:]), 0.85)))
    res["cfg2_torque_rows"] = run(p2, inp)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
