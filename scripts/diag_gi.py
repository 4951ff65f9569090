"""Diagnostics (GPU box, stamp build): where the dual active set's time goes (gi_solve's lap
counters, qppvm_kernel.hip) in a config-2 churned solve and a config-4 fused rollout.

Slots per block (kStamps = 64): 20-27 cycles summed per gi_solve phase (0 setup / M rows, 1 warm batch
projections, 2 warm step, 3 select, 4 project_out + |z|^2, 5 step + add/drop, 6 rebuild after a drop,
7 record + final x), 13 loop passes, 14 rebuild projections, 6 / 7 inline repairs' cycles and count,
28-29 / 30-31 the fused rollout's whole-block shader / realtime clocks."""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from qppvm_amd import wbq  # noqa: E402

K = 64
# the u-space loop (gi_solve, rounds 1-5; WBQ_GI_CS=0 builds) or the constraint-space loop (cs_gi.h, round 6:
# counts 13 = passes, 14 = x rebuilds)
LAPS = (["setup", "warm_batch", "warm_step", "select", "project_out", "step_add_drop", "rebuild", "record"]
        if os.environ.get("WBQ_DIAG_LOOP", "cs") == "gs" else
        ["setup", "warm_append", "warm_lambda", "select", "column", "step", "drop", "rebuild_refine"])


def stamps(s, nb):
    buf = (ctypes.c_ulonglong * (K * nb))()
    s.lib.wbq_diag_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    assert s.lib.wbq_diag_stamps(s.ctx, buf, nb) == 0
    return np.frombuffer(buf, dtype=np.uint64).reshape(nb, K).astype(np.int64)


def clear(s, nb):
    s.lib.wbq_diag_stamps_clear.argtypes = [ctypes.c_void_p, ctypes.c_int]
    assert s.lib.wbq_diag_stamps_clear(s.ctx, nb) == 0


def summarise(full, rollout=False):
    laps = full[:, 20:28]
    passes, rebuilds = full[:, 13], full[:, 14]
    out = {"blocks": int(full.shape[0]), "blocks_in_gi": int((laps.sum(1) > 0).sum())}
    g = laps.sum(1) > 0
    if g.any():
        out["gi_cycles_sum_mean_per_block_in_gi"] = {n: float(laps[g, k].mean()) for k, n in enumerate(LAPS)}
        out["gi_loop_passes_mean_p99_max"] = [float(passes[g].mean()), float(np.percentile(passes[g], 99)),
                                              int(passes[g].max())]
        out["gi_rebuild_projections_mean_max"] = [float(rebuilds[g].mean()), int(rebuilds[g].max())]
        per_pass = (laps[g, 3] + laps[g, 4] + laps[g, 5]) / np.maximum(passes[g], 1)
        out["gi_cycles_per_pass_select_project_step_p50"] = float(np.median(per_pass[passes[g] > 0])) \
            if (passes[g] > 0).any() else 0.0
        rb = rebuilds[g] > 0
        if rb.any():
            out["gi_cycles_per_rebuild_projection_p50"] = float(np.median(laps[g, 6][rb] / rebuilds[g][rb]))
    gi_tot = laps.sum(1)
    order = np.argsort(-gi_tot)[:6]
    out["most_gi_cycles"] = [{"block": int(b), "gi_cycles": int(gi_tot[b]), "passes": int(passes[b]),
                              "rebuilds": int(rebuilds[b]), "laps": [int(x) for x in laps[b]]} for b in order]
    rep = full[:, 7] > 0
    out["repair_blocks"] = int(rep.sum())
    if rep.any():
        out["repair_cycles_per_call_mean_max"] = [float((full[rep, 6] / full[rep, 7]).mean()),
                                                  float((full[rep, 6] / full[rep, 7]).max())]
        out["repair_calls_per_block_max"] = int(full[rep, 7].max())
    if rollout:
        cyc = full[:, 29] - full[:, 28]
        rt = (full[:, 31] - full[:, 30]) / 100.0  # us
        out["rollout_block_us_p50_p90_p99_max"] = [float(np.percentile(rt, q)) for q in (50, 90, 99, 100)]
        out["clock_ghz_median"] = float(np.median(cyc / np.maximum(rt, 1e-9)) / 1e3)
        order = np.argsort(-rt)[:8]
        gi_tot = laps.sum(1)
        out["slowest_blocks"] = [{"block": int(b), "us": float(rt[b]), "cycles": int(cyc[b]),
                                  "gi_cycles": int(gi_tot[b]), "gi_passes": int(passes[b]),
                                  "rebuild_proj": int(rebuilds[b]), "repair_cycles": int(full[b, 6]),
                                  "repairs": int(full[b, 7]),
                                  "gi_laps": [int(x) for x in laps[b]]} for b in order]
    return out


def main():
    lib = os.path.join(ROOT, "qppvm_amd", "libwbq_diag.so")
    wbq.load_library(lib)
    n, B = 30, 4096
    nb = B // 2
    res = {}
    # config 2: the second call of a churned batch (20 % of the rows re-randomised, warm start carried)
    prob, inp, Solver = bench.build_workload("qppvm", 2, n, B, 1, 0, 0)
    pool = bench.churn_pool("qppvm", prob, n, B, 1, 0)
    s = Solver(prob, max_batch=B)
    s.set_inputs(inp)
    s.solve()
    s.sync()
    sl = (B + 4) // 5
    inp2 = {k: v.copy() for k, v in inp.items()}
    for k in inp2:
        inp2[k][:sl] = pool[k][:sl]
    s.set_inputs(inp2)
    clear(s, nb)
    s.solve()
    s.sync()
    res["cfg2_churn"] = summarise(stamps(s, nb))
    _, st, it = s.outputs()
    res["cfg2_churn"]["iters_hist"] = np.bincount(it).tolist()
    s.close()
    # config 4: one fused rollout of 20 steps from the measured state, warm state from a previous one
    prob, inp, Solver = bench.build_workload("qppvm", 4, n, B, 1, 0, 0, plant=True)
    s = Solver(prob, max_batch=B)
    s.set_inputs(inp)
    s.rollout(bench.HORIZON, bench.MPC_DT)
    s.sync()
    s.set_state(inp["q"], inp["qd"])
    s.sync()
    clear(s, nb)
    s.rollout(bench.HORIZON, bench.MPC_DT)
    s.sync()
    res["cfg4_rollout"] = summarise(stamps(s, nb), rollout=True)
    s.close()
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
