"""Worker for the multi-process (gloo, CPU) sharding tests; spawned by tests/test_shard.py.
The shard's solve is the CPU oracle (test infrastructure): what is under test is the
partition, the per-shard instance generation and the padded all-gather."""
import os

import numpy as np


def shard_worker(rank, world, port, total, n, out_path):
    import torch
    import torch.distributed as dist

    import oracle
    from qppvm_amd.problem import QPPVMProblem
    from qppvm_amd.shard import ShardPlan, gather_shards, max_over_ranks
    from qppvm_amd.synth import qppvm_instances

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        plan = ShardPlan(total, world)
        s, e = plan.bounds(rank)
        prob = QPPVMProblem(n=n, tau_max=100.0)
        if e > s:
            inp = qppvm_instances(prob, e - s, seed=11, offset=s)
            tau, st, _ = oracle.qppvm_batch(prob, inp)
        else:
            tau, st = np.zeros((0, n)), np.zeros(0, dtype=np.int32)
        full_tau = gather_shards(torch.from_numpy(tau), plan, rank)
        full_st = gather_shards(torch.from_numpy(st.astype(np.int64))[:, None], plan, rank)
        # a plan with an empty shard (total < world)
        tiny = ShardPlan(1, world)
        t = torch.full((tiny.count(rank), 2), float(rank))
        tiny_all = gather_shards(t, tiny, rank)
        mx = max_over_ranks([rank + 0.5, -float(rank)])
        if rank == 0:
            np.savez(out_path, tau=full_tau.numpy(), st=full_st.numpy()[:, 0], tiny=tiny_all.numpy(),
                     mx=np.array(mx))
    finally:
        dist.destroy_process_group()
