"""Diagnostics (GPU box): where a config-0 QPPVMPlugin tick goes. Runs the dummy driver with a dump
of its first ticks' solver inputs, then re-solves those ticks one instance per solve (warm start
carried, as in the plugin) with the phase-stamp build (libwbq_diag.so): per tick the device time
of the solve, the repair phases (Gauss-Jordan, BVLS, pins + equality, dual active set) in shader
cycles, and the BVLS / active-set step counts."""
import ctypes
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    from test_plugin import read_dump

    from qppvm_amd import wbq
    from qppvm_amd.problem import QPPVMProblem
    out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "diag_plugin_tick.json")
    lib = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "qppvm_amd", "libwbq_diag.so")
    ticks = int(os.environ.get("DIAG_TICKS", "40"))
    dump = "/tmp/diag_tick_dump.bin"
    stress = ["--stress"] if os.environ.get("DIAG_STRESS") == "1" else []
    subprocess.run([os.path.join(ROOT, "qppvm_amd", "qppvm_dummy_driver"), "--ticks", str(ticks), "--dump", dump,
                    str(ticks)] + stress, check=True, capture_output=True)
    n, d = read_dump(dump)
    prob = QPPVMProblem(n=n, tau_max=150.0)
    wbq._lib = None
    wbq.load_library(lib)
    s = wbq.QPPVMSolver(prob, max_batch=1)
    s.lib.wbq_diag_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    s.lib.wbq_diag_stamps_clear.argtypes = [ctypes.c_void_p, ctypes.c_int]
    K = 64
    rows = []
    for t in range(ticks):
        inp = {k: np.ascontiguousarray(d[k][t:t + 1]) for k in ("M", "J", "pose", "pose_ref", "q", "qd", "qref", "h")}
        inp["pose"] = inp["pose"].reshape(1, 2, 12)
        inp["pose_ref"] = inp["pose_ref"].reshape(1, 2, 12)
        s.set_inputs(inp)
        s.sync()
        s.lib.wbq_diag_stamps_clear(s.ctx, 1)  # (the dual loops' lap counters add up)
        s.set_timing(True)
        s.solve()
        s.sync()
        ms, _ = s.get_timing()
        buf = (ctypes.c_ulonglong * K)()
        assert s.lib.wbq_diag_stamps(s.ctx, buf, 1) == 0
        st = np.frombuffer(buf, dtype=np.uint64).astype(np.int64)
        tau, status, iters = s.outputs()
        # the repair kernel ran for this instance when its realtime stamps are set (a repair that hands its level-1
        # loop back returns before stamp 12, so "st[12] > st[8]" missed exactly the hand-back ticks)
        rep = bool(st[29] > st[28] > 0)
        hb = bool(st[43] > st[42] > 0)
        row = {"tick": t, "us": 1e3 * ms, "status": int(status[0]), "iters": int(iters[0]), "repair": rep,
               "handback": hb, "fast_cycles": int(st[5] - st[0])}
        # the constant 100 MHz clock (s_memrealtime, global): each launch's own span (fast kernel 16-17, active-set
        # kernel 30-31, repair kernel 28-29, hand-back pass 42-43) and the gaps between consecutive launches
        spans = [("fast", 16, 17)]
        if st[31] > st[30] > 0:
            spans.append(("active", 30, 31))
        if rep:
            spans.append(("repair", 28, 29))
            row["repair_clock_ghz"] = (st[12] - st[8]) / max(1.0, (st[29] - st[28]) / 100.0) / 1e3 if st[12] > st[8] \
                else (st[11] - st[8]) / max(1.0, (st[29] - st[28]) / 100.0) / 1e3
        if hb:
            spans.append(("handback", 42, 43))
        row["rt_us"] = {}
        prev_end = None
        for nm, a0, a1 in spans:
            if prev_end is not None:
                row["rt_us"]["gap_before_" + nm] = (st[a0] - prev_end) / 100.0
            row["rt_us"][nm] = (st[a1] - st[a0]) / 100.0
            prev_end = st[a1]
        row["rt_us"]["span"] = (prev_end - st[16]) / 100.0
        row["fast_clock_ghz"] = (st[5] - st[0]) / max(1.0, (st[17] - st[16]) / 100.0) / 1e3
        # the dual loop's lap counters (gi_solve): active-set kernel slots 32-41; 48-57 the pinned level 1's loop,
        # in the hand-back pass or (hand-back off) in the repair kernel
        for nm, base, cb in (("active_gi", 32, 40), ("pinned_gi", 48, 56)):
            laps = [int(v) for v in st[base:base + 8]]
            if sum(laps) > 0:
                passes = int(st[cb])
                row[nm] = {"cycles": sum(laps), "passes": passes, "rebuild_proj": int(st[cb + 1]),
                           "cycles_per_pass": (laps[3] + laps[4] + laps[5]) / max(passes, 1),
                           "laps_setup_warm_wstep_select_proj_step_rebuild_rec": laps}
        if rep:
            row.update({"gj": int(st[9] - st[8]), "bvls": int(st[10] - st[9]), "pins_eq": int(st[11] - st[10]),
                        "bvls_it": int(st[13]), "bvls_split": [int(v) for v in st[20:28]]})
            if st[12] > st[11]:  # (the level-1 loop ran inside the repair kernel, not in the hand-back pass)
                row.update({"gi": int(st[12] - st[11]), "gi_it": int(st[14])})
        rows.append(row)
    s.close()
    json.dump(rows, open(out, "w"), indent=1)
    us = np.array([r["us"] for r in rows])
    print(json.dumps({"ticks": ticks, "us_p50_p90_p99_max": [float(np.percentile(us, q)) for q in (50, 90, 99, 100)]}))
    # stamped time vs device time: the share of each tick its launches' spans and the gaps between them account for
    # (every tick, the slowest included; the rest of a tick's device time is the first launch's dispatch)
    acc = [r["rt_us"]["span"] / r["us"] for r in rows]
    slow = sorted(rows, key=lambda r: -r["us"])[:8]
    print(json.dumps({"ticks_stamped": len(acc), "span_over_device_time_p10_p50_p90":
                      [float(np.percentile(acc, q)) for q in (10, 50, 90)],
                      "slowest8_span_over_device_time": [round(r["rt_us"]["span"] / r["us"], 3) for r in slow],
                      "repair_share": float(np.mean([r["repair"] for r in rows])),
                      "handback_share": float(np.mean([r["handback"] for r in rows]))}))
    for r in sorted(rows, key=lambda r: -r["us"])[:8]:
        print(json.dumps(r))


if __name__ == "__main__":
    main()
