"""CPU: the numpy statement of the n <= 32 constraint-space dual active set (scripts/emulate_cs_gi.py, the
step-for-step restatement of qppvm_amd/csrc/cs_gi.h) solves random level-1 least-distance problems
    min 0.5 ||u - u_hat||^2  s.t.  G u = b0,  lo <= M u <= hi
to their KKT conditions (scaled residuals <= 1e-9), a warm start from the previous final active set gives the
cold result to 1e-9, and the storage hand-off (more than KM active bounds) is the only way it gives up on a
feasible problem. Checks the algorithm the kernel implements, not the kernel (the GPU parity tests do that)."""
import importlib.util
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _emu():
    spec = importlib.util.spec_from_file_location("emulate_cs_gi", os.path.join(ROOT, "scripts", "emulate_cs_gi.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_cs_statement_kkt_and_warm():
    m = _emu()
    rng = np.random.default_rng(11)
    solved = 0
    for b in range(120):
        P = m.make_problem(rng, frac=0.2)
        out = m.cs_solve(P)
        if out["infeasible"]:
            assert out["k"] >= m.KM or out["iters"] > 0  # a hand-off or a genuine no-step
            continue
        r = m.kkt(P, out)
        assert max(r.values()) <= 1e-9, (b, r)
        # warm start from the final active set on slightly moved bounds == the cold solve
        P2 = dict(P)
        P2["lo"] = P["lo"] + 1e-3 * rng.standard_normal(P["lo"].shape)
        P2["hi"] = np.maximum(P["hi"] + 1e-3 * rng.standard_normal(P["hi"].shape), P2["lo"] + 1e-4)
        cold, warm = m.cs_solve(P2), m.cs_solve(P2, wsg=out["side"])
        if not cold["infeasible"] and not warm["infeasible"]:
            d = np.abs(cold["x"] - warm["x"]).max() / (1 + np.abs(cold["x"]).max())
            assert d <= 1e-9, (b, d)
            assert warm["iters"] <= cold["iters"] + 1
        solved += 1
    assert solved >= 100
