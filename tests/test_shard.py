"""Multi-GPU path on CPU: the shard plan, and world_size-2 (and 3) gloo runs of the
sharded solve + padded all-gather, checked against the single-process oracle on the whole
batch (weak-scaling shards, the only collective is the optional gather)."""
import os
import socket
import sys

import numpy as np
import pytest

from qppvm_amd.shard import ShardPlan

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.parametrize("total,world", [(0, 1), (1, 2), (37, 2), (4096, 8), (5, 3), (8, 8)])
def test_shard_plan_partitions(total, world):
    p = ShardPlan(total, world)
    covered = []
    for r in range(world):
        s, e = p.bounds(r)
        assert e - s == p.count(r) and p.count(r) in (total // world, total // world + 1)
        covered.extend(range(s, e))
    assert covered == list(range(total))
    assert p.max_count == max(p.count(r) for r in range(world))


def test_shard_plan_rejects_bad():
    with pytest.raises(ValueError):
        ShardPlan(10, 0)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world,total", [(2, 37), (3, 10)])
def test_gloo_sharded_solve_matches_single_process(tmp_path, oracle_lib, world, total):
    import torch.multiprocessing as mp

    from qppvm_amd.problem import QPPVMProblem
    from qppvm_amd.synth import qppvm_instances

    sys.path.insert(0, HERE)
    from _dist_worker import shard_worker

    n = 12
    out = str(tmp_path / "gathered.npz")
    mp.spawn(shard_worker, args=(world, _free_port(), total, n, out), nprocs=world, join=True)
    got = np.load(out)
    prob = QPPVMProblem(n=n, tau_max=100.0)
    tau, st, _ = oracle_lib.qppvm_batch(prob, qppvm_instances(prob, total, seed=11))
    np.testing.assert_array_equal(got["tau"], tau)  # shards reproduce the global batch exactly
    np.testing.assert_array_equal(got["st"], st)
    np.testing.assert_array_equal(got["tiny"], np.zeros((1, 2)))
    np.testing.assert_array_equal(got["mx"], [world - 0.5, 0.0])


def test_bench_refuses_more_gpus_than_visible():
    """bench.py --gpus N relaunches itself as N ranks only when N GPUs are visible; otherwise it
    exits non-zero with a clear message before touching any GPU."""
    import subprocess
    root = os.path.dirname(HERE)
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "64", "--no-pmc"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2
    assert "--gpus 64 requested but only" in r.stderr


def test_bench_refuses_world_size_mismatch():
    import subprocess
    root = os.path.dirname(HERE)
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "4", "--no-pmc"],
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 2 and "WORLD_SIZE=2 but --gpus 4" in r.stderr
