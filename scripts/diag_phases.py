"""Diagnostics (GPU box): per-phase cycles from the stamp build, and launch time vs batch."""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from qppvm_amd import wbq  # noqa: E402
from qppvm_amd.problem import QPPVMProblem  # noqa: E402
from qppvm_amd.synth import qppvm_instances, replicate  # noqa: E402

PHASES = ["stage+force", "gauss-jordan", "equality block", "bound check+output"]


def run(libpath, prob, inp, reps=20, stamps=False):
    wbq._lib = None
    wbq.load_library(libpath)
    s = wbq.QPPVMSolver(prob, max_batch=inp["h"].shape[0])
    s.set_inputs(inp)
    s.solve()
    s.sync()
    s.set_timing(True)
    for _ in range(reps):
        s.solve()
    ms, cnt = s.get_timing()
    out = {"us_per_launch": 1e3 * ms / cnt}
    if stamps:
        B = inp["h"].shape[0]
        nb = B if prob.n > 32 else (B + 1) // 2  # blocks of the fast kernel: 2 instances per wave for n <= 32
        K = 64
        buf = (ctypes.c_ulonglong * (K * nb))()
        s.lib.wbq_diag_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        assert s.lib.wbq_diag_stamps(s.ctx, buf, nb) == 0
        full = np.frombuffer(buf, dtype=np.uint64).reshape(nb, K).astype(np.int64)
        st = full[:, [0, 1, 2, 3, 5]]
        d = np.diff(st, axis=1)
        out["fast_kernel_phase_cycles_mean"] = {p: float(d[:, k].mean()) for k, p in enumerate(PHASES)}
        out["fast_kernel_phase_cycles_mean"]["(stage: loads issued + forces)"] = float((full[:, 15] - full[:, 0]).mean())
        out["fast_kernel_phase_cycles_mean"]["(stage: wait for M + Y)"] = float((full[:, 1] - full[:, 15]).mean())
        out["fast_block_cycles_p50_p90"] = [float(np.percentile(st[:, -1] - st[:, 0], q)) for q in (50, 90)]
        rt = full[:, 16:18]  # s_memrealtime (100 MHz, global): start / end offsets in us
        rt = rt[(rt[:, 0] > 0) & (rt[:, 1] >= rt[:, 0])]  # blocks that wrote both stamps
        t0 = rt[:, 0].min()
        out["fast_block_start_us_p10_p50_p90_max"] = [float(np.percentile(rt[:, 0] - t0, q)) / 100 for q in (10, 50, 90, 100)]
        out["fast_block_end_us_p10_p50_p90_max"] = [float(np.percentile(rt[:, 1] - t0, q)) / 100 for q in (10, 50, 90, 100)]
        out["fast_block_dur_us_p10_p50_p90_max"] = [float(np.percentile(rt[:, 1] - rt[:, 0], q)) / 100 for q in (10, 50, 90, 100)]
        # by XCD (round-robin block dispatch: XCD = block id % 8)
        xcd = np.arange(nb) % 8
        rtf = full[:, 16:18]
        okr = (rtf[:, 0] > 0) & (rtf[:, 1] >= rtf[:, 0])
        out["fast_block_dur_us_mean_by_xcd"] = [float((rtf[okr & (xcd == x), 1] - rtf[okr & (xcd == x), 0]).mean()) / 100
                                                for x in range(8)]
        out["fast_block_cycles_mean_by_xcd"] = [float((st[xcd == x, -1] - st[xcd == x, 0]).mean()) for x in range(8)]
        _, status, iters = s.outputs()
        it_blk = iters[: 2 * nb].reshape(nb, -1).max(axis=1) if nb < B else iters[:nb]
        act = it_blk > 0
        if act.any():
            setup = full[act, 6] - full[act, 4]
            loop = full[act, 7] - full[act, 6]
            out["active_blocks"] = int(act.sum())
            out["active_setup_cycles_mean"] = float(setup.mean())
            out["active_loop_cycles_mean"] = float(loop.mean())
            out["active_cycles_per_step_mean"] = float((loop / it_blk[act]).mean())
            out["active_block_max_steps_p50_p90_max"] = [float(np.percentile(it_blk[act], q)) for q in (50, 90, 100)]
            out["iters_hist"] = np.bincount(iters).tolist()
        inl = full[:, 19] > full[:, 18]  # NP = 32: the inline dual active set (stamps 18 / 19)
        if inl.any():
            c = full[inl, 19] - full[inl, 18]
            out["inline_active_blocks"] = int(inl.sum())
            out["inline_active_cycles_p50_p90_max"] = [float(np.percentile(c, q)) for q in (50, 90, 100)]
        rep = full[:, 12] > full[:, 8]
        if rep.any():
            r = full[rep][:, 8:13]
            d = np.diff(r, axis=1)
            out["repair_blocks"] = int(rep.sum())
            out["repair_phase_cycles_mean"] = {p: float(d[:, k].mean()) for k, p in
                                               enumerate(["gauss-jordan A0", "bvls", "pins+equality", "dual active set"])}
            out["repair_iters_mean"] = float(iters[: len(iters)].mean())
    s.close()
    return out


def main():
    diag = os.path.join(ROOT, "qppvm_amd", "libwbq_diag.so")  # built beforehand, in-tree
    if not os.path.exists(diag):
        from qppvm_amd import build
        diag = build.build(force=True, diag=True)
    res = {}
    n = 30
    base = qppvm_instances(QPPVMProblem(n=n), 65536, seed=1)
    p1 = QPPVMProblem(n=n, tau_max=1e6)
    for B in (256, 1024, 4096, 16384, 65536):
        inp = replicate({k: v[:1] for k, v in base.items()}, B)
        res[f"cfg1_B{B}"] = run(wbq.LIB_PATH, p1, inp)
    for B in (256, 4096):
        inp = replicate({k: v[:1] for k, v in base.items()}, B)
        res[f"cfg1_B{B}_stamps"] = run(diag, p1, inp, stamps=True)
    free = wbq.QPPVMSolver(QPPVMProblem(n=n, tau_max=1e9), max_batch=4096)
    sub = {k: v[:4096] for k, v in base.items()}
    tau_free, _, _ = free.solve_batch(sub)
    free.close()
    p2 = QPPVMProblem(n=n, tau_max=float(np.quantile(np.abs(tau_free), 0.8)))
    res["cfg2_B4096_stamps"] = run(diag, p2, sub, stamps=True)
    # level-0 repair path (tight limits), warm after the first solve
    for nn, B in ((39, 1), (39, 64), (30, 64)):
        pr = QPPVMProblem(n=nn, tau_max=30.0)
        res[f"repair_n{nn}_B{B}"] = run(diag, pr, qppvm_instances(pr, B, seed=7), stamps=True)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
