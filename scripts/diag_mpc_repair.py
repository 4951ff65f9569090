"""Config-4 level-0 repair cost (GPU, the stamp build libwbq_diag.so): 8 rollout steps with one launch
per step and the separate repair kernel, then every repair block's phase stamps (Gauss-Jordan for A0,
BVLS, pins + equality block, dual active set + u) against its step counts (BVLS, dual active set): cycles
per BVLS step and per dual step by least squares."""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from qppvm_amd import wbq  # noqa: E402
from qppvm_amd.problem import QPPVMProblem  # noqa: E402
from qppvm_amd.synth import qppvm_instances  # noqa: E402


def main():
    wbq.load_library(os.path.join(ROOT, "qppvm_amd", "libwbq_diag.so"))
    n, B = 30, 4096
    inp = qppvm_instances(QPPVMProblem(n=n), B, seed=1, plant=True)
    free = wbq.QPPVMSolver(QPPVMProblem(n=n, tau_max=1e9), max_batch=B)
    tau_free, _, _ = free.solve_batch(inp)
    free.close()
    prob = QPPVMProblem(n=n, tau_max=float(np.quantile(np.abs(tau_free), 0.8)))
    s = wbq.QPPVMSolver(prob, max_batch=B)
    s.set_option(s.OPT_FUSED_ROLLOUT, 0)
    s.set_option(s.OPT_INLINE_REPAIR, 0)
    s.set_inputs(inp)
    rows = []
    nb, K = B // 2, 28
    s.lib.wbq_diag_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    for k in range(8):
        buf = (ctypes.c_ulonglong * (K * nb))()
        s.rollout(1, 1e-3)
        s.sync()
        assert s.lib.wbq_diag_stamps(s.ctx, buf, nb) == 0
        full = np.frombuffer(buf, dtype=np.uint64).reshape(nb, K).astype(np.int64)
        rows.append(full.copy())
    s.close()
    # a block's repair stamps survive until it repairs again: keep each (block, stamps) once
    allr = np.concatenate(rows)
    rep = (allr[:, 12] > allr[:, 8]) & (allr[:, 8] > 0)
    rr = np.unique(allr[rep][:, list(range(8, 15)) + list(range(20, 28))], axis=0)
    r = rr[:, :7]
    bv = rr[:, 7:].astype(float)  # BVLS split: reductions, solve, z + ratio + argmin, update, outer KKT, fast, pivoted
    ph = np.diff(r[:, :5], axis=1).astype(float)
    itb, itg = r[:, 5].astype(float), r[:, 6].astype(float)
    out = {"repairs": int(len(r)), "phase_names": ["gauss-jordan A0", "bvls", "pins+equality", "dual active set + u"],
           "phase_cycles_mean": ph.mean(axis=0).tolist(), "phase_cycles_p90": np.percentile(ph, 90, axis=0).tolist(),
           "bvls_steps_mean_max": [float(itb.mean()), float(itb.max())],
           "dual_steps_mean_max": [float(itg.mean()), float(itg.max())]}
    X = np.stack([np.ones_like(itb), itb], axis=1)
    out["bvls_cycles_fit_const_per_step"] = np.linalg.lstsq(X, ph[:, 1], rcond=None)[0].tolist()
    X = np.stack([np.ones_like(itg), itg], axis=1)
    out["dual_cycles_fit_const_per_step"] = np.linalg.lstsq(X, ph[:, 3], rcond=None)[0].tolist()
    nit = np.maximum(bv[:, 5] + bv[:, 6] + bv[:, 7], 1.0)
    out["bvls_split_cycles_per_inner_step"] = {k: float((bv[:, j] / nit).mean()) for j, k in enumerate(
        ["reductions", "solve", "z+ratio+argmin", "update"])}
    out["bvls_outer_kkt_cycles_total_mean"] = float(bv[:, 4].mean())
    out["bvls_rowfast_pivoted_column_solves_mean"] = [float(bv[:, 5].mean()), float(bv[:, 6].mean()),
                                                      float(bv[:, 7].mean())]
    out["worst"] = [dict(zip(["gj", "bvls", "pins", "dual"], p.tolist()), bvls_it=int(a), dual_it=int(g))
                    for p, a, g in sorted(zip(ph, itb, itg), key=lambda t: -t[0].sum())[:8]]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
