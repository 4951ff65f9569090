"""Diagnostics (GPU box, stamp build): where the n > 32 active-set kernel's time goes (qppvm_active_kernel<64, ...>,
gi_solve's lap counters at stamp slots 32-39, counts 40-41) in the second call of a churned n = 39 config-2 batch
(scripts/diag_gi.py does the same for the n <= 32 loop). One instance per block: the per-block laps are per instance."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import bench  # noqa: E402
from diag_gi import clear, stamps  # noqa: E402
from qppvm_amd import wbq  # noqa: E402

LAPS = ["setup", "warm_batch", "warm_step", "select", "project_out", "step_add_drop", "rebuild", "record"]


def main():
    wbq.load_library(os.path.join(ROOT, "qppvm_amd", "libwbq_diag.so"))
    n, B = 39, 4096
    prob, inp, Solver = bench.build_workload("qppvm", 2, n, B, 1, 0, 0)
    pool = bench.churn_pool("qppvm", prob, n, B, 1, 0)
    s = Solver(prob, max_batch=B)
    s.set_inputs(inp)
    s.solve()
    s.sync()
    sl = (B + 4) // 5
    res = {}
    for call in range(3):  # three churned calls, warm state carried: the last is the steady state
        inp2 = {k: v.copy() for k, v in inp.items()}
        for k in inp2:
            inp2[k][(call * sl) % B:(call * sl) % B + sl] = pool[k][:sl]
        s.set_inputs(inp2)
        clear(s, B)
        s.solve()
        s.sync()
        full = stamps(s, B)
        laps, cnt = full[:, 32:40], full[:, 40:42]
        g = laps.sum(1) > 0
        tot = laps[g].sum(1)
        _, st, it = s.outputs()
        res[f"call{call}"] = {
            "blocks_in_gi": int(g.sum()),
            "cycles_per_block_mean": {nm: float(laps[g, k].mean()) for k, nm in enumerate(LAPS)},
            "cycles_per_block_total_p50_p90_max": [float(np.percentile(tot, 50)), float(np.percentile(tot, 90)),
                                                    int(tot.max())],
            "counts_mean_max": [[float(cnt[g, j].mean()), int(cnt[g, j].max())] for j in range(2)],
            "iters_hist": np.bincount(it).tolist(),
        }
    s.close()
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
