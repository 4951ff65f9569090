"""Throughput bench: batched WBC-QP solves/sec (BASELINE.json metric), QPPVM form, n = 30.

A step = one wbq_solve over the rank's batch (assemble -> 2-level QP -> tau), inputs
already resident in HBM. N > 1: one process per GPU (torch.distributed.run), each rank
solves its own shard of B instances (weak scaling, no data-path collective unless
--allgather). Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# algorithmic bytes per instance (n = 30, 2 tasks): inputs read once + outputs written once
def algorithmic_bytes(n, T):
    inputs = 8 * (n * n + T * 6 * n + 2 * T * 12 + 4 * n)  # M, J, pose, pose_ref, q, qd, qref, h
    outputs = 8 * n + 4 + 4  # tau, status, iters
    return inputs + outputs


HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=4096, help="instances per GPU")
    ap.add_argument("--n", type=int, default=30)
    ap.add_argument("--config", type=int, default=1, choices=(1, 2),
                    help="1: identical instances, bounds inactive; 2: random, ~20%% active bounds")
    ap.add_argument("--allgather", action="store_true", help="RCCL all-gather of tau per step")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline budget")
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1
    import torch
    if dist:
        import torch.distributed as tdist
        torch.cuda.set_device(local)
        tdist.init_process_group("nccl", device_id=torch.device("cuda", local))
    from qppvm_amd.problem import QPPVMProblem
    from qppvm_amd.shard import ShardPlan
    from qppvm_amd.synth import qppvm_instances, replicate
    from qppvm_amd.wbq import QPPVMSolver

    n, B = args.n, args.batch
    device = local if dist else 0
    if args.config == 1:
        prob = QPPVMProblem(n=n, tau_max=1e6)  # bounds inactive
        inp = replicate(qppvm_instances(prob, 1, seed=0), B)
    else:
        plan = ShardPlan(B * world, world)  # weak scaling: rank r solves rows [r B, (r+1) B)
        inp = qppvm_instances(QPPVMProblem(n=n), plan.count(rank), seed=1, offset=plan.start(rank))
        # ~20 % of the torque limits binding: tau_max = 80th percentile of |tau| of the first
        # B instances solved with the limits far away (same sample on every rank, so all ranks
        # solve one global problem)
        calib = inp if rank == 0 else qppvm_instances(QPPVMProblem(n=n), B, seed=1, offset=0)
        free = QPPVMSolver(QPPVMProblem(n=n, tau_max=1e9), max_batch=B, device=device)
        tau_free, _, _ = free.solve_batch(calib)
        free.close()
        prob = QPPVMProblem(n=n, tau_max=float(np.quantile(np.abs(tau_free), 0.8)))
    solver = QPPVMSolver(prob, max_batch=B, device=device)
    solver.set_inputs(inp)
    solver.sync()

    gather_buf = None
    if args.allgather:
        # tau goes straight into a torch tensor on torch's stream, then one RCCL all-gather
        out = torch.empty((B, n), dtype=torch.float64, device="cuda")
        gather_buf = torch.empty((world * B, n), dtype=torch.float64, device="cuda")
        solver.set_stream(torch.cuda.current_stream().cuda_stream)
        solver.set_device_outputs(out.data_ptr())

    def step():
        solver.solve()
        if gather_buf is not None:
            if dist:
                tdist.all_gather_into_tensor(gather_buf, out)
            else:
                gather_buf.copy_(out)

    for _ in range(args.warmup):
        step()
    solver.sync()
    torch.cuda.synchronize()
    if dist:
        tdist.barrier()
    solver.set_timing(True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    solver.sync()
    torch.cuda.synchronize()
    if dist:
        tdist.barrier()
    dt = time.perf_counter() - t0
    kern_ms, launches = solver.get_timing()
    tau, status, iters = solver.outputs()
    if dist:
        t = torch.tensor([dt, kern_ms / max(launches, 1)], dtype=torch.float64, device="cuda")
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        dt, kavg_ms = float(t[0]), float(t[1])
    else:
        kavg_ms = kern_ms / max(launches, 1)

    total = B * world * args.steps
    value = total / dt
    bytes_per_launch = algorithmic_bytes(n, prob.ntasks) * B
    achieved = bytes_per_launch / (kavg_ms * 1e-3) / 1e9
    line = {
        "metric": "batched WBC-QP solves/sec, ~30-DoF problem, 1/2/4/8 MI355X",
        "value": value,
        "unit": "QP-solves/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt * 1e3 / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic randomized robot states (SURVEY 8d), inputs resident in HBM",
        "config": {"workload": f"QPPVM 2-level torque QP, n={n}, batch={B}/GPU, "
                               + ("identical instances, bounds inactive (BASELINE config 1)"
                                  if args.config == 1 else "random states, ~20% bounds active (config 2)"),
                   "global_batch": B * world, "n": n, "parallelism": f"shard{world}",
                   "allgather": bool(args.allgather)},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                     "kernel_avg_us": kavg_ms * 1e3,
                     "algorithmic_bytes_per_instance": algorithmic_bytes(n, prob.ntasks)},
        "status_ok_frac": float(np.mean(status == 0)),
        "mean_active_set_steps": float(np.mean(iters)),
    }
    if rank == 0 and not args.no_cpu:
        line["cpu_baseline"] = cpu_baseline(prob, inp, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist:
        tdist.destroy_process_group()


def cpu_baseline(prob, inp, budget_s):
    """The CPU oracle (single thread) on a bounded sample of the same workload."""
    import oracle
    oracle.build()
    done, t0 = 0, time.perf_counter()
    chunk = 64
    B = inp["h"].shape[0]
    while time.perf_counter() - t0 < budget_s:
        lo = done % B
        sl = {k: v[lo:lo + chunk] for k, v in inp.items()}
        oracle.qppvm_batch(prob, sl)
        done += sl["h"].shape[0]
    dt = time.perf_counter() - t0
    return {"value": done / dt, "unit": "QP-solves/s", "cores": 1, "kind": "port",
            "sample": f"{done} instances of the bench batch in {dt:.1f} s, oracle/wbq_oracle.c "
                      "(x-space OpenSoT-form assembly + BVLS + primal active set), 1 thread"}


if __name__ == "__main__":
    main()
