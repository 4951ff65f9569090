"""One bench-style rank (RANK / WORLD_SIZE / MASTER_* from the environment) for
tests/test_gpu_shard.py: solve this rank's shard with tau written straight into a torch tensor on
torch's stream (wbq_set_outputs), all-gather it over RCCL, and save the gathered shard beside the
solver's own copy of its outputs."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(out_path):
    import torch
    import torch.distributed as dist

    from qppvm_amd.problem import QPPVMProblem
    from qppvm_amd.shard import ShardPlan
    from qppvm_amd.synth import qppvm_instances
    from qppvm_amd.wbq import QPPVMSolver

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    try:
        n, total = 30, 3000
        plan = ShardPlan(total, world)
        prob = QPPVMProblem(n=n, tau_max=120.0)  # some limits bind
        inp = qppvm_instances(prob, plan.count(rank), seed=21, offset=plan.start(rank))
        s = QPPVMSolver(prob, max_batch=plan.max_count, device=local)
        s.set_inputs(inp)
        out = torch.zeros((plan.max_count, n), dtype=torch.float64, device="cuda")
        status = torch.full((plan.max_count,), -9, dtype=torch.int32, device="cuda")
        s.set_stream(torch.cuda.current_stream().cuda_stream)
        s.set_device_outputs(out.data_ptr(), status.data_ptr())
        s.solve()
        buf = torch.empty((world * plan.max_count, n), dtype=torch.float64, device="cuda")
        dist.all_gather_into_tensor(buf, out)  # same stream: ordered behind the solve
        torch.cuda.synchronize()
        tau, st, _ = s.outputs()
        s.close()
        c = plan.count(rank)
        mine = buf[rank * plan.max_count: rank * plan.max_count + c].cpu().numpy()
        if rank == 0:
            np.savez(out_path, gathered=mine, direct=tau, status=st)
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1])
