"""Throughput bench: batched WBC-QP solves/sec (BASELINE.json metric), n = 30.

A step = one wbq_solve over the rank's batch (assemble -> 2-level QP -> tau), inputs
already resident in HBM. Default workload = BASELINE config 1 (4096 identical QPPVM
instances per GPU); ``--form contact`` runs the contact-form (ForceAcc) variant, and the
default run also measures that variant for a few hundred steps and reports it beside
the headline line. ``--config 2`` = random states (QPPVM: ~20 % of torque bounds active;
contact: 2/3/4 of 4 feet in contact + actuated torque rows); ``--config 4`` = MPC: a step is
one rollout of N = 20 sequential solves per instance with q, qd integrated on the device
(wbq_rollout), counted as B x 20 QPs.

N > 1: one process per GPU (torch.distributed.run), each rank solves its own shard of B
instances (weak scaling, no data-path collective unless --allgather). Prints ONE JSON line
on rank 0.

roofline: achieved = algorithmic bytes of one launch / the dominant kernel's average
device time (HIP events on the launch stream around that kernel only, on every 8th solve of
the timed region: event packets on every solve would pace the stream); traffic = HBM
bytes per launch of that kernel from rocprofv3 PMC passes (FETCH_SIZE x 2, the gfx950
correction of MI355X_MICROARCH.md, + WRITE_SIZE), run as child processes before this
process touches the GPU (N = 1 only; --no-pmc skips them).
"""
import argparse
import csv
import glob
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "batched WBC-QP solves/sec, ~30-DoF problem, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
DOMINANT = {"qppvm": "qppvm_fast_kernel", "contact": "contact_kernel", "qppvm_w1m": "qppvm_w1m_kernel"}
TIMING_EVERY = 8  # HIP-event pairs around every 8th solve of the timed region
HORIZON, MPC_DT = 20, 1e-3  # config 4: N = 20 sequential QPs per rollout, semi-implicit Euler


def qppvm_bytes(n, T):
    """Algorithmic bytes per QPPVM instance: inputs read once + outputs written once."""
    inputs = 8 * (n * n + T * 6 * n + 2 * T * 12 + 4 * n)  # M, J, pose, pose_ref, q, qd, qref, h
    outputs = 8 * n + 4 + 4  # tau, status, iters
    return inputs + outputs


def contact_bytes(n, nc):
    """Algorithmic bytes per contact-form instance."""
    inputs = 8 * (n * n + 4 * n + 6 * n + 6 + 24 + nc * (6 * n + 6 + 24)) + 4  # ... + cmask
    outputs = 8 * (n + n + 3 * nc) + 4 + 4  # tau, x, status, iters
    return inputs + outputs


def shard_plan(config, B, world, global_batch):
    """Weak scaling (configs 1, 2, 4): B instances per rank, rank r owns rows [r B, (r+1) B).
    Config 3: a fixed global batch (65,536) in contiguous shards over the ranks (strong)."""
    from qppvm_amd.shard import ShardPlan
    return ShardPlan(global_batch if config == 3 else B * world, world)


def build_workload(form, config, n, B, world, rank, device, weight=0, global_batch=65536, plant=False):
    """(problem, inputs, solver class) for this rank's shard (weight: joint task W1 = I / M;
    plant: the physically scaled synthetic states of config 4, qppvm_amd/synth.py)."""
    from qppvm_amd.problem import ContactProblem, QPPVMProblem
    from qppvm_amd.synth import contact_instances, qppvm_instances, replicate
    from qppvm_amd.wbq import ContactSolver, QPPVMSolver
    plan = shard_plan(config, B, world, global_batch)
    B = plan.count(rank)
    if config == 4 and form == "qppvm" and plant == "rbd":
        # MPC on a model: M, h, J, poses of a humanoid-like tree (qppvm_amd/rbd.py) from its
        # state, re-evaluated on the device every rollout step (wbq_rollout_rbd)
        from qppvm_amd.rbd import RBDModel, centauro_like, humanoid_like
        model = centauro_like() if n == 39 else humanoid_like(n)
        rng = np.random.default_rng(1000 + rank)
        q0, qd0 = rng.uniform(-0.5, 0.5, (B, n)), rng.normal(0.0, 0.5, (B, n))
        r = RBDModel(model, max_batch=B, device=device)
        M, h, J, pose = r.compute(q0, qd0)
        r.close()
        pref = pose.copy()
        pref[:, :, [3, 7, 11]] += rng.normal(0.0, 0.02, (B, model.ntasks, 3))
        inp = dict(M=M, J=J, pose=pose, pose_ref=pref, q=q0, qd=qd0, qref=q0.copy(), h=h)
        free = QPPVMSolver(QPPVMProblem(n=n, tau_max=1e9, joint_weight=weight), max_batch=B, device=device)
        tau_free, _, _ = free.solve_batch(inp)
        free.close()
        prob = QPPVMProblem(n=n, tau_max=float(np.quantile(np.abs(tau_free), 0.8)), joint_weight=weight)
        prob.rbd_model = model
        return prob, inp, QPPVMSolver
    plant = plant is True
    if config in (3, 4):
        config = 2  # config 3 shards and MPC rollouts start from the config-2 random states
    if form == "qppvm":
        if config == 1:
            prob = QPPVMProblem(n=n, tau_max=1e6, joint_weight=weight)  # bounds inactive
            return prob, replicate(qppvm_instances(prob, 1, seed=0), B), QPPVMSolver
        inp = qppvm_instances(QPPVMProblem(n=n), plan.count(rank), seed=1, offset=plan.start(rank), plant=plant)
        # ~20 % of the torque limits binding: tau_max = 80th percentile of |tau| of the first
        # B instances solved with the limits far away (same sample on every rank)
        # (the calibration sample is the first 4096 instances of the global batch, on every rank)
        calib = qppvm_instances(QPPVMProblem(n=n), min(4096, plan.total), seed=1, offset=0, plant=plant)
        free = QPPVMSolver(QPPVMProblem(n=n, tau_max=1e9, joint_weight=weight), max_batch=calib["h"].shape[0],
                           device=device)
        tau_free, _, _ = free.solve_batch(calib)
        free.close()
        return (QPPVMProblem(n=n, tau_max=float(np.quantile(np.abs(tau_free), 0.8)), joint_weight=weight), inp,
                QPPVMSolver)
    if config == 1:  # double support, identical instances
        prob = ContactProblem(n=n, nc=2)
        return prob, replicate(contact_instances(prob, 1, seed=0), B), ContactSolver
    free = ContactProblem(n=n, nc=4)
    masks = [0b0011, 0b0111, 0b1111]  # 2, 3 or 4 feet in contact
    inp = contact_instances(free, plan.count(rank), seed=1, offset=plan.start(rank), masks=masks)
    calib = contact_instances(free, min(4096, plan.total), seed=1, offset=0, masks=masks)
    s = ContactSolver(free, max_batch=calib["h"].shape[0], device=device)
    tau_free, _, _ = s.solve_batch(calib)
    s.close()
    prob = ContactProblem(n=n, nc=4, torque_rows=True, tau_max=float(np.quantile(np.abs(tau_free[:, 6:]), 0.85)))
    return prob, inp, ContactSolver


def churn_pool(form, prob, n, B, world, rank):
    """Second pool of random states for the config-2 churn (same distribution, seed 2)."""
    from qppvm_amd.problem import ContactProblem, QPPVMProblem
    from qppvm_amd.shard import ShardPlan
    from qppvm_amd.synth import contact_instances, qppvm_instances
    plan = ShardPlan(B * world, world)
    if form == "qppvm":
        return qppvm_instances(QPPVMProblem(n=n), plan.count(rank), seed=2, offset=plan.start(rank))
    return contact_instances(ContactProblem(n=n, nc=prob.nc), plan.count(rank), seed=2, offset=plan.start(rank),
                             masks=[0b0011, 0b0111, 0b1111])


def euler_stability(prob, inp, dt, sample=256):
    """dt * Dc * lambda_max(G_t M^-1 G_t^T) per instance (max over the tasks; G_t = the task's
    selected Jacobian rows): the explicit-Euler factor of the task damping. Above 2 the
    closed loop of an MPC rollout with frozen J, M is unstable at this dt."""
    out = []
    for b in range(min(sample, inp["h"].shape[0])):
        Minv = np.linalg.inv(inp["M"][b])
        worst = 0.0
        for t in range(prob.ntasks):
            rows = [r for r in range(6) if (prob.row_mask[t] >> r) & 1]
            G = inp["J"][b, t][rows]
            worst = max(worst, float(np.linalg.eigvalsh(G @ Minv @ G.T).max()) * float(prob.Dc[t].max()))
        out.append(dt * worst)
    return {"median": float(np.median(out)), "max": float(np.max(out)), "instances": len(out)}


def run(form, config, n, B, steps, warmup, world, rank, device, allgather=False, dist=False, host_io=False,
        weight=0, global_batch=65536, plant=False, repair_share=True):
    """Times `steps` solves; returns a dict of measurements (max over ranks when dist)."""
    import torch
    plan = shard_plan(config, B, world, global_batch)
    prob, inp, Solver = build_workload(form, config, n, B, world, rank, device, weight, global_batch, plant)
    B = plan.count(rank)
    solver = Solver(prob, max_batch=max(B, 1), device=device)
    solver.set_inputs(inp)
    solver.sync()
    gather_buf = None
    ag_events = []
    if allgather:
        # tau goes straight into a torch tensor on torch's stream (padded to the largest shard),
        # then one RCCL all-gather of every rank's shard over xGMI
        out = torch.zeros((plan.max_count, n), dtype=torch.float64, device="cuda")
        gather_buf = torch.empty((world * plan.max_count, n), dtype=torch.float64, device="cuda")
        solver.set_stream(torch.cuda.current_stream().cuda_stream)
        solver.set_device_outputs(out.data_ptr())

    churn = None
    if config == 2:
        # churn: every call re-randomises 20 % of the instances -- a
        # rotating fifth of the rows is refreshed in HBM from a second pool of random states
        # (seed 2; the pools alternate), warm-start state carried over. The inputs live in
        # torch tensors adopted zero-copy; the refresh (a D2D copy of 20 % of the input
        # bytes) runs on the solve stream inside the timed step.
        pool = churn_pool(form, prob, n, B, world, rank)
        keys = list(inp.keys())
        dev = f"cuda:{device}"
        # every field of a dtype lives in one flat device buffer (each field a contiguous view, the layout the
        # solver adopts), so that a refresh is one gather + one scatter over precomputed element indices per
        # dtype -- the same rows of every field -- instead of one copy dispatch per field (eight ~5 us copy
        # kernels took ~35 us of a ~140 us step: profiles/r06_v7_ab_nograph_c2.log; a captured graph of the
        # copies did not shorten it on ROCm 7.2)
        groups = {}
        for k in keys:
            groups.setdefault(np.asarray(inp[k]).dtype.str, []).append(k)
        sl = (B + 4) // 5
        flat, live, alt0, alt1, idx = {}, {}, {}, {}, {}
        for dt, ks in groups.items():
            sizes = [int(np.prod(np.asarray(inp[k]).shape)) for k in ks]
            offs = np.concatenate([[0], np.cumsum(sizes)])
            tdt = torch.from_numpy(np.zeros(1, dtype=np.dtype(dt))).dtype
            f_live = torch.empty(int(offs[-1]), dtype=tdt, device=dev)
            f_alt0, f_alt1 = torch.empty_like(f_live), torch.empty_like(f_live)
            for k, o, sz in zip(ks, offs[:-1], sizes):
                shp = np.asarray(inp[k]).shape
                live[k] = f_live[o:o + sz].view(shp)
                live[k].copy_(torch.from_numpy(np.ascontiguousarray(inp[k])).to(dev))
                f_alt0[o:o + sz].copy_(live[k].reshape(-1))
                f_alt1[o:o + sz].view(shp).copy_(torch.from_numpy(np.ascontiguousarray(pool[k])).to(dev))
            # element indices of row slice q of every field of this dtype
            idx[dt] = []
            for q in range(5):
                lo, hi = q * sl, min(B, (q + 1) * sl)
                per = [np.arange(o + lo * (sz // B), o + hi * (sz // B)) for o, sz in zip(offs[:-1], sizes)]
                idx[dt].append(torch.from_numpy(np.concatenate(per)).to(dev))
            flat[dt] = (f_live, (f_alt0, f_alt1))
        solver.set_stream(torch.cuda.current_stream(device).cuda_stream)
        solver.set_device_inputs({k: live[k].data_ptr() for k in keys}, B)
        churn = dict(flat=flat, idx=idx, calls=0)
        torch.cuda.synchronize()

    rbd = None
    if config == 4:  # each MPC step re-plans from the measured state: a D2D reset of (q, qd)
        q0 = torch.from_numpy(np.ascontiguousarray(inp["q"])).to(f"cuda:{device}")
        qd0 = torch.from_numpy(np.ascontiguousarray(inp["qd"])).to(f"cuda:{device}")
        if getattr(prob, "rbd_model", None) is not None:
            from qppvm_amd.rbd import RBDModel
            rbd = RBDModel(prob.rbd_model, max_batch=B, device=device)
            rbd.set_stream(None)
        torch.cuda.synchronize()

    def step():
        if host_io:  # PCIe-inclusive: host inputs -> pinned staging -> H2D, solve, D2H outputs
            solver.set_inputs(inp)
            solver.solve()
            solver.outputs()
            return
        if churn is not None:
            c = churn["calls"]
            for dt, (f_live, alts) in churn["flat"].items():
                ix = churn["idx"][dt][c % 5]
                src = alts[1 - (c // 5) % 2]  # pool states, then the originals, ...
                f_live.index_copy_(0, ix, src.index_select(0, ix))
            churn["calls"] = c + 1
        if config == 4:
            solver.set_state(q0.data_ptr(), qd0.data_ptr(), device=True)
            if rbd is not None:
                solver.rollout_rbd(rbd, HORIZON, MPC_DT)
            else:
                solver.rollout(HORIZON, MPC_DT)
        else:
            solver.solve()
        if gather_buf is not None:
            ev = None
            if timing_on[0] and step_no[0] % (TIMING_EVERY if config == 1 else 1) == 0:  # sampled like the kernel events
                ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                ev[0].record()
            if dist:
                import torch.distributed as tdist
                tdist.all_gather_into_tensor(gather_buf, out)
            else:
                gather_buf.copy_(out)  # world size 1: the gather is a device copy
            if ev is not None:
                ev[1].record()
                ag_events.append(ev)
        step_no[0] += 1

    timing_on, step_no = [False], [0]
    for _ in range(warmup):
        step()
    solver.sync()
    torch.cuda.synchronize()
    if dist:
        import torch.distributed as tdist
        tdist.barrier()
    # (configs 2 and 4: every solve is timed -- their kernels are long enough that the event packets do not pace
    # the stream, and the per-call time varies with the churn phase, so a 1-in-8 sample is biased)
    every = TIMING_EVERY if config == 1 else 1
    solver.set_timing(True, every=every)
    timing_on[0], step_no[0] = True, 0
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    t_enq = time.perf_counter() - t0  # host time to enqueue the steps (launch-bound if ~ dt)
    solver.sync()
    torch.cuda.synchronize()
    if dist:
        tdist.barrier()
    dt = time.perf_counter() - t0
    solve_ms, kern_ms, launches = solver.get_timing_detail()
    ag_ms = float(np.mean([a.elapsed_time(b) for a, b in ag_events])) if ag_events else 0.0
    tau, status, iters = solver.outputs()
    mpc = None
    if config == 4 and form == "qppvm" and repair_share:
        # repair share: one more rollout from the measured state, one step per call, reading the
        # warm-start hints (1 = that step's level 0 was infeasible: the BVLS repair ran)
        solver.set_state(q0.data_ptr(), qd0.data_ptr(), device=True)
        shares = []
        for _ in range(HORIZON):
            if rbd is not None:
                solver.rollout_rbd(rbd, 1, MPC_DT)
            else:
                solver.rollout(1, MPC_DT)
            shares.append(float(solver.warm_hints().mean()))
        mpc = {"repair_share_per_step": float(np.mean(shares)), "repair_share_last_step": shares[-1],
               "euler_dt_Dc_lambda_max": euler_stability(prob, inp, MPC_DT),
               "inputs": ("on-device rigid-body model re-evaluated every step (wbq_rollout_rbd), "
                          f"{prob.rbd_model.n}-joint tree" if rbd is not None else
                          "plant-scaled (lambda(M) in [0.5, 5], J ~ N(0, 0.2^2))" if plant else
                          "SURVEY 8d distribution (lambda(M) in [1e-2, 1e1], J ~ N(0, 0.5^2))")}
        if rbd is not None:
            rbd.close()
    if gather_buf is not None:  # the gathered tau holds this rank's shard where the plan puts it
        g = gather_buf[rank * plan.max_count: rank * plan.max_count + B].cpu().numpy()
        assert np.array_equal(g, tau), "all-gathered tau differs from the rank's own solve"
    solver.close()
    kavg_ms, savg_ms = kern_ms / max(launches, 1), solve_ms / max(launches, 1)
    if dist:
        t = torch.tensor([dt, kavg_ms, savg_ms, ag_ms], dtype=torch.float64, device="cuda")
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        dt, kavg_ms, savg_ms, ag_ms = float(t[0]), float(t[1]), float(t[2]), float(t[3])
    per_inst = qppvm_bytes(n, prob.ntasks) if form == "qppvm" else contact_bytes(n, prob.nc)
    qps = HORIZON if config == 4 else 1  # an MPC step counts its N sequential QPs
    return dict(prob=prob, inp=inp, dt=dt, t_enq=t_enq, kavg_ms=kavg_ms, savg_ms=savg_ms, status=status, iters=iters,
                bytes_per_instance=per_inst, total=plan.total * steps * qps, B_local=B, allgather_ms=ag_ms,
                allgather_bytes=8 * n * plan.max_count * world, mpc=mpc)


def fused_rollout(form, config, weight, n, plant):
    """Config 4 QPPVM (W1 = I, n <= 32, model frozen) runs each rollout in one launch
    (qppvm_rollout_kernel: HORIZON solves of the whole batch per launch)."""
    return form == "qppvm" and config == 4 and not weight and n <= 32 and plant != "rbd"


def dominant_kernel(form, weight, fused=False):
    if fused:
        return "qppvm_rollout_kernel"
    return DOMINANT["qppvm_w1m"] if (form == "qppvm" and weight) else DOMINANT[form]


def pmc_traffic(args, form):
    """Per-launch HBM bytes of the dominant kernel from two rocprofv3 PMC passes (one counter
    block each, kernel trace only), child processes of this not-yet-GPU-initialised process."""
    prof = shutil.which("rocprofv3")
    if prof is None:
        return None, "rocprofv3 not found"
    vals = {}
    w = 1 if args.weight == "M" else 0
    plant = ("rbd" if args.mpc_inputs == "rbd" else args.mpc_inputs == "plant") if args.config == 4 else False
    kern = dominant_kernel(form, w, fused_rollout(form, args.config, w, args.n, plant))
    with tempfile.TemporaryDirectory(dir="/tmp") as td:
        for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            out = os.path.join(td, ctr)
            cmd = [prof, "--pmc", ctr, "--output-format", "csv", "-d", out, "-o", "run", "--",
                   sys.executable, os.path.join(ROOT, "bench.py"), "--no-cpu", "--no-pmc", "--no-variant",
                   "--steps", "20", "--warmup", "2", "--form", form, "--config", str(args.config),
                   "--batch", str(args.batch), "--global-batch", str(args.global_batch), "--n", str(args.n),
                   "--weight", args.weight, "--mpc-inputs", args.mpc_inputs,
                   # (config 4: the PMC child runs only the timed twenty-step rollout launches, not the one-step
                   # launches of the repair-share pass, so the per-launch bytes are one launch shape's)
                   "--no-repair-share"]
            env = dict(os.environ, TMPDIR="/tmp")
            try:
                r = subprocess.run(cmd, cwd="/tmp", env=env, capture_output=True, text=True, timeout=150)
            except subprocess.TimeoutExpired:
                return None, f"{ctr} pass timed out"
            if r.returncode != 0:
                return None, f"{ctr} pass failed ({r.returncode})"
            per = []
            for f in glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True):
                with open(f) as fh:
                    for row in csv.DictReader(fh):
                        if kern in row.get("Kernel_Name", ""):
                            per.append(float(row["Counter_Value"]))
            if not per:
                return None, f"{ctr}: no dispatches of {kern}"
            vals[ctr] = sum(per) / len(per)  # KB per dispatch
    fetch, write = vals["FETCH_SIZE"] * 1024, vals["WRITE_SIZE"] * 1024
    return {"bytes": 2 * fetch + write, "fetch_raw": fetch, "write": write}, None


def cpu_baseline(form, prob, inp, budget_s):
    """The CPU oracle (single thread) on a bounded sample of the same workload."""
    import oracle
    oracle.build()
    fn = oracle.qppvm_batch if form == "qppvm" else oracle.contact_batch
    done, t0 = 0, time.perf_counter()
    chunk = 64
    B = inp["h"].shape[0]
    while time.perf_counter() - t0 < budget_s:
        lo = done % B
        sl = {k: v[lo:lo + chunk] for k, v in inp.items()}
        fn(prob, sl)
        done += sl["h"].shape[0]
    dt = time.perf_counter() - t0
    what = ("x-space OpenSoT-form assembly + BVLS + primal active set" if form == "qppvm" else
            "contact-form assembly + dense dual active set with LU-solved KKT")
    return {"value": done / dt, "unit": "QP-solves/s", "cores": 1, "kind": "port",
            "sample": f"{done} instances of the bench batch in {dt:.1f} s, oracle ({what}), 1 thread"}


def cpu_baseline_mpc(prob, inp, budget_s, rollouts=32):
    """Config 4 on the CPU: the oracle solves each step of a bounded sample of rollouts, numpy
    integrates (q_dd = M^-1 (tau - h), semi-implicit Euler), HORIZON steps per rollout (with a
    model: the oracle's recursions re-evaluate it every step)."""
    import oracle
    oracle.build()
    model = getattr(prob, "rbd_model", None)
    done, t0, B = 0, time.perf_counter(), inp["h"].shape[0]
    while time.perf_counter() - t0 < budget_s:
        lo = (done // HORIZON) % B
        cur = {k: v[lo:lo + rollouts].copy() for k, v in inp.items()}
        for _ in range(HORIZON):
            if model is not None:
                cur["M"], cur["h"], cur["J"], cur["pose"] = oracle.rbd_batch(model, cur["q"], cur["qd"])
            tau, st, _ = oracle.qppvm_batch(prob, cur)
            qdd = np.linalg.solve(cur["M"], (tau - cur["h"])[..., None])[..., 0]
            qdd[st != 0] = 0.0
            cur["qd"] = cur["qd"] + MPC_DT * qdd
            cur["q"] = cur["q"] + MPC_DT * cur["qd"]
        done += cur["h"].shape[0] * HORIZON
    dt = time.perf_counter() - t0
    return {"value": done / dt, "unit": "QP-solves/s", "cores": 1, "kind": "port",
            "sample": f"{done // HORIZON} rollouts x {HORIZON} steps of the bench batch in {dt:.1f} s, oracle per "
                      "step + numpy Euler, 1 thread"}


def cpu_baseline_threads(form, prob, inp, budget_s):
    """Same oracle, one independent instance stream per host thread (the
    all-cores run); the C calls release the GIL. Threads = min(16, nproc): 16 is the GPU box's CPU share."""
    import concurrent.futures as cf
    import oracle
    fn = oracle.qppvm_batch if form == "qppvm" else oracle.contact_batch
    T = max(1, min(16, len(os.sched_getaffinity(0))))  # the box's CPU share is 16 (nproc may show more)
    B = inp["h"].shape[0]

    def worker(w):
        done, t0, chunk = 0, time.perf_counter(), 32
        while time.perf_counter() - t0 < budget_s:
            lo = (w * 257 + done) % B
            fn(prob, {k: v[lo:lo + chunk] for k, v in inp.items()})
            done += min(chunk, B - lo)
        return done
    t0 = time.perf_counter()
    with cf.ThreadPoolExecutor(max_workers=T) as ex:
        done = sum(ex.map(worker, range(T)))
    dt = time.perf_counter() - t0
    return {"value": done / dt, "unit": "QP-solves/s", "cores": T, "kind": "port",
            "sample": f"{done} instances in {dt:.1f} s, {T} threads, one instance stream each",
            "cores_note": "threads = min(16, affinity): 16 is this job's CPU share on the GPU box (one GPU's "
                          "slice of the host); nproc / lscpu report the whole host, whose other cores belong "
                          "to other jobs, so an all-host-cores run is not available to this process"}


def host_cpu():
    """Host CPU description for the baseline: nproc (this process's affinity) and lscpu's model."""
    info = {"nproc": len(os.sched_getaffinity(0)), "os_cpu_count": os.cpu_count()}
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            k, _, v = line.partition(":")
            if k.strip() in ("Model name", "CPU(s)", "Thread(s) per core", "Socket(s)"):
                info["lscpu_" + k.strip().lower().replace(" ", "_").replace("(s)", "s")] = v.strip()
    except (OSError, subprocess.SubprocessError):
        pass
    return info


def relaunch(args):
    """--gpus N > 1 from a plain process: one rank per GPU under torch.distributed.run, as a
    child process started before this process touches the GPU (never an exec). Fails loudly
    when the node has fewer GPUs."""
    import socket

    import torch
    have = torch.cuda.device_count()  # counting devices does not initialise the GPU here
    if have < args.gpus:
        print(f"bench.py: --gpus {args.gpus} requested but only {have} GPU(s) are visible", file=sys.stderr)
        return 2
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd).returncode


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=4096, help="instances per GPU (configs 1, 2, 4)")
    ap.add_argument("--global-batch", type=int, default=65536, help="config 3: instances over all GPUs")
    ap.add_argument("--n", type=int, default=30)
    ap.add_argument("--form", choices=("qppvm", "contact"), default="qppvm")
    ap.add_argument("--config", type=int, default=1, choices=(1, 2, 3, 4),
                    help="1: identical instances; 2: random states, bounds / contacts churn; "
                         "3: a fixed global batch of random states sharded over the GPUs + all-gather of tau; "
                         "4: MPC, each step = HORIZON sequential solves per rollout (wbq_rollout)")
    ap.add_argument("--allgather", action="store_true", help="RCCL all-gather of tau per step (config 3: always)")
    ap.add_argument("--mpc-inputs", choices=("plant", "survey", "rbd"), default="plant",
                    help="config 4 states: plant-scaled (stable explicit Euler at the reference gains, default), "
                         "the SURVEY 8d distribution (its rollouts diverge into level-0 repairs), or a rigid-body "
                         "model re-evaluated on the device every step (wbq_rollout_rbd)")
    ap.add_argument("--weight", choices=("I", "M"), default="I", help="QPPVM joint-task weight W1 (SURVEY 8a a6)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline budget")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-pmc", action="store_true", help="skip the rocprofv3 traffic passes")
    ap.add_argument("--no-variant", action="store_true", help="skip the contact-form variant line")
    ap.add_argument("--no-repair-share", action="store_true",
                    help="config 4: skip the one-step-per-call rollout that measures the repair share (the PMC child "
                         "uses this, so its counters see the timed launch shape only)")
    ap.add_argument("--host-io", action="store_true",
                    help="PCIe-inclusive rate: host inputs copied in and outputs copied out every step "
                         "(never the headline value; DESIGN.md reports it beside it)")
    args = ap.parse_args()
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(relaunch(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}: launch one rank per GPU", file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1
    allgather = args.allgather or args.config == 3
    traffic, traffic_note = None, "skipped (--no-pmc or N > 1)"
    if not dist and not args.no_pmc:
        traffic, traffic_note = pmc_traffic(args, args.form)  # before this process touches the GPU
    import torch
    if local >= torch.cuda.device_count():
        print(f"bench.py: rank {rank} has LOCAL_RANK {local} but only {torch.cuda.device_count()} GPU(s)",
              file=sys.stderr)
        sys.exit(2)
    if dist:
        import torch.distributed as tdist
        torch.cuda.set_device(local)
        tdist.init_process_group("nccl", device_id=torch.device("cuda", local))
    device = local if dist else 0
    n, B = args.n, args.batch
    weight = 1 if args.weight == "M" else 0
    plant = ("rbd" if args.mpc_inputs == "rbd" else args.mpc_inputs == "plant") if args.config == 4 else False
    fused = fused_rollout(args.form, args.config, weight, n, plant)
    kern = dominant_kernel(args.form, weight, fused)
    m = run(args.form, args.config, n, B, args.steps, args.warmup, world, rank, device, allgather, dist,
            args.host_io, weight, args.global_batch, plant, repair_share=not args.no_repair_share)
    value = m["total"] / m["dt"]
    # algorithmic bytes of one launch of the dominant kernel: the fused rollout kernel solves the batch
    # HORIZON times (each solve stages its instance's inputs again: nothing is skipped)
    bpl = m["bytes_per_instance"] * m["B_local"] * (HORIZON if fused else 1)
    achieved = bpl / (m["kavg_ms"] * 1e-3) / 1e9
    wl = {("qppvm", 1): "QPPVM 2-level torque QP, identical instances, bounds inactive (BASELINE config 1)",
          ("qppvm", 2): "QPPVM 2-level torque QP, random states, ~20% torque bounds active, 20% of the "
                        "instances re-randomised per call (D2D refresh in the step), warm start carried (config 2)",
          ("qppvm", 3): f"QPPVM 2-level torque QP, {args.global_batch} random states (~20% torque bounds active) "
                        "in contiguous shards over the GPUs, RCCL all-gather of tau every step (config 3)",
          ("contact", 1): "ForceAcc contact-form QP, double support (nc=2), identical instances (config 1 variant)",
          ("contact", 2): "ForceAcc contact-form QP, random states, 2-4 of 4 feet, torque rows, 20% of the "
                          "instances re-randomised per call (config 2)",
          ("contact", 3): f"ForceAcc contact-form QP, {args.global_batch} random states (2-4 of 4 feet, torque rows) "
                          "in contiguous shards over the GPUs, RCCL all-gather of tau every step (config 3)",
          ("qppvm", 4): f"MPC: rollouts x N={HORIZON} sequential QPPVM QPs, on-device semi-implicit Euler "
                        "(dt=1e-3), J/M/h frozen, warm-start carry (config 4)",
          ("contact", 4): f"MPC: rollouts x N={HORIZON} sequential contact-form QPs, on-device Euler (config 4)"}
    if args.config == 4 and args.mpc_inputs == "rbd":
        wl[("qppvm", 4)] = (f"MPC: rollouts x N={HORIZON} sequential QPPVM QPs, M/h/J/poses re-evaluated on the device "
                            "every step from the integrated state (rigid-body model, wbq_rollout_rbd), semi-implicit "
                            "Euler (dt=1e-3), warm-start carry (config 4)")
    per_gpu = f"batch={m['B_local']}/GPU" if args.config != 3 else f"global batch={args.global_batch}"
    st, it = m["status"], m["iters"]
    line = {
        "metric": METRIC,
        "value": value,
        "unit": "QP-solves/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": m["dt"] * 1e3 / args.steps,
        "higher_is_better": True,
        "scaling": "strong" if args.config == 3 else "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic randomized robot states (SURVEY 8d), " + (
            "host inputs/outputs over PCIe every step (--host-io)" if args.host_io else "inputs resident in HBM"),
        "config": {"workload": f"{wl[(args.form, args.config)]}{', W1 = M' if weight else ''}, n={n}, {per_gpu}",
                   "global_batch": m["total"] // (args.steps * (HORIZON if args.config == 4 else 1)), "n": n,
                   "parallelism": f"shard{world}", "allgather": bool(allgather)},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS,
                     "traffic": None if traffic is None else traffic["bytes"],
                     "kernel": kern, "kernel_avg_us": m["kavg_ms"] * 1e3,
                     "solve_avg_us": m["savg_ms"] * 1e3, "algorithmic_bytes_per_launch": bpl,
                     "solves_per_launch": (HORIZON if fused else 1) * m["B_local"],
                     "algorithmic_bytes_per_instance": m["bytes_per_instance"],
                     "traffic_note": traffic_note if traffic is None else
                     "rocprofv3 PMC per launch: 2 x FETCH_SIZE (gfx950 correction) + WRITE_SIZE"
                     f"; raw fetch {traffic['fetch_raw']:.0f} B, write {traffic['write']:.0f} B"},
        "status_ok_frac": float(np.mean(st == 0)),
        "status_histogram": {str(k): int(v) for k, v in zip(*np.unique(st, return_counts=True))},
        "mean_active_set_steps": float(np.mean(it)) if it.size else 0.0,
        "max_active_set_steps": int(it.max()) if it.size else 0,
        "host_enqueue_us_per_step": m["t_enq"] * 1e6 / args.steps,
    }
    if m["mpc"] is not None:
        line["mpc"] = m["mpc"]
    if allgather:
        line["allgather"] = {"avg_ms": m["allgather_ms"], "bytes": m["allgather_bytes"],
                             "note": "torch.cuda events around all_gather_into_tensor (RCCL) on every "
                                     + ("step" if args.config != 1 else f"{TIMING_EVERY}th step")
                                     + " of the timed region, max over ranks; at N = 1 a device copy"}
    if not args.no_variant and args.form == "qppvm" and args.config != 3:
        # the contact-form variant of the same config, same process, same protocol
        v = run("contact", args.config, n, B, max(50, args.steps // 2), args.warmup, world, rank, device,
                False, dist)
        va = v["bytes_per_instance"] * v["B_local"] / (v["kavg_ms"] * 1e-3) / 1e9
        line["contact_variant"] = {"workload": wl[("contact", args.config)], "value": v["total"] / v["dt"],
                                   "ms_per_step": v["dt"] * 1e3 / max(50, args.steps // 2),
                                   "kernel_avg_us": v["kavg_ms"] * 1e3, "roofline_frac": va / HBM_PEAK_GBS,
                                   "status_ok_frac": float(np.mean(v["status"] == 0)),
                                   "mean_active_set_steps": float(np.mean(v["iters"]))}
    if rank == 0 and world == 1 and not args.no_cpu:
        if args.config == 4 and args.form == "qppvm":
            line["cpu_baseline"] = cpu_baseline_mpc(m["prob"], m["inp"], args.cpu_seconds)
        else:
            line["cpu_baseline"] = cpu_baseline(args.form, m["prob"], m["inp"], args.cpu_seconds)
            line["cpu_baseline_threads"] = cpu_baseline_threads(args.form, m["prob"], m["inp"], args.cpu_seconds / 2)
        line["cpu_host"] = host_cpu()
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist:
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
