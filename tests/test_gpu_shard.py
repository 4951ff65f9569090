"""GPU side of the multi-GPU path (BASELINE config 3: 65,536 instances in 8 contiguous
shards + an all-gather of tau) on the one GPU a test box has:

* the HIP path at the config-3 shard size (8,192) carries the KAT-4 certificates on every instance;
* the whole 65,536-instance batch on one GPU: every instance solves, and each one's tau is
  bit-identical to the same instance solved inside its own 8,192-instance shard (sharding never
  changes an answer, so the 8-rank run returns exactly this batch), certificates on a sample;
* n = 64 at 70,000 instances: M alone is 2.3 GB, past the 2^31-byte reach of a 32-bit buffer
  offset -- every instance of a replicated batch must return the first one's tau;
* the all-gather path at world size 1 over RCCL (`wbq_set_outputs` into a torch tensor on torch's
  stream, then `all_gather_into_tensor`), run as its own process like a bench rank.
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import kkt
from qppvm_amd.problem import QPPVMProblem
from qppvm_amd.shard import ShardPlan
from qppvm_amd.synth import qppvm_instances

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
TOL = 1e-9
GLOBAL, WORLD = 65536, 8


@pytest.fixture(scope="module")
def wbq_mod():
    from qppvm_amd import build, wbq
    build.build()
    return wbq


def solve(wbq_mod, prob, inp):
    s = wbq_mod.QPPVMSolver(prob, max_batch=max(1, inp["h"].shape[0]))
    try:
        return s.solve_batch(inp)
    finally:
        s.close()


@pytest.fixture(scope="module")
def config3(wbq_mod):
    """The config-3 batch (config-2 random states, seed 1) and its limits (~20 % binding),
    calibrated like bench.py on the first 4096 instances."""
    inp = qppvm_instances(QPPVMProblem(n=30), GLOBAL, seed=1)
    calib = {k: v[:4096] for k, v in inp.items()}
    t0, _, _ = solve(wbq_mod, QPPVMProblem(n=30, tau_max=1e9), calib)
    return QPPVMProblem(n=30, tau_max=float(np.quantile(np.abs(t0), 0.8))), inp


def certify(oracle_lib, prob, inp, tau, idx):
    cs = [kkt.qppvm_certificate(oracle_lib, prob, inp, int(b), tau[b]) for b in idx]
    w = {k: max(c[k] for c in cs) for k in ("primal", "level0", "stat", "sign")}
    assert max(w.values()) <= TOL, w


def test_config3_shard_certificates(wbq_mod, oracle_lib, config3):
    prob, inp = config3
    plan = ShardPlan(GLOBAL, WORLD)
    s, e = plan.bounds(WORLD - 1)  # the last rank's shard
    shard = {k: v[s:e] for k, v in inp.items()}
    tau, st, it = solve(wbq_mod, prob, shard)
    assert e - s == 8192 and (st == 0).all(), np.bincount(st.clip(0))
    assert (it > 0).mean() > 0.5  # the active set runs on most instances
    certify(oracle_lib, prob, shard, tau, range(e - s))


def test_config3_full_batch_one_gpu(wbq_mod, oracle_lib, config3):
    prob, inp = config3
    tau, st, _ = solve(wbq_mod, prob, inp)
    assert (st == 0).all() and np.isfinite(tau).all()
    plan = ShardPlan(GLOBAL, WORLD)
    for r in (0, 3, WORLD - 1):  # shard answers are bit-identical to the full batch's rows
        s, e = plan.bounds(r)
        t_r, st_r, _ = solve(wbq_mod, prob, {k: v[s:e] for k, v in inp.items()})
        np.testing.assert_array_equal(t_r, tau[s:e])
        np.testing.assert_array_equal(st_r, st[s:e])
    rng = np.random.default_rng(3)
    certify(oracle_lib, prob, inp, tau, rng.choice(GLOBAL, 512, replace=False))


def test_large_batch_past_32bit_offsets(wbq_mod):
    """n = 64, B = 70,000: M is 2.3e9 bytes. Device inputs (torch), replicated instance."""
    import torch
    n, B = 64, 70000
    prob = QPPVMProblem(n=n, tau_max=1e6)
    one = qppvm_instances(prob, 1, seed=5)
    dev = {k: torch.from_numpy(np.ascontiguousarray(v)).to("cuda").expand((B,) + v.shape[1:]).contiguous()
           for k, v in one.items()}
    assert int(dev["M"].numel()) * 8 > 2 ** 31
    s = wbq_mod.QPPVMSolver(prob, max_batch=B)
    try:
        s.set_device_inputs({k: t.data_ptr() for k, t in dev.items()}, B)
        s.solve()
        tau, st, _ = s.outputs()
    finally:
        s.close()
    assert (st == 0).all()
    assert np.array_equal(tau, np.broadcast_to(tau[:1], tau.shape))
    t1, st1, _ = solve(wbq_mod, prob, one)
    np.testing.assert_array_equal(tau[-1], t1[0])


def _free_port():
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def test_allgather_rccl_world1(wbq_mod, tmp_path):
    out = str(tmp_path / "ag.npz")
    env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(_free_port()))
    r = subprocess.run([sys.executable, os.path.join(HERE, "_allgather_worker.py"), out], env=env, cwd=ROOT,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    d = np.load(out)
    np.testing.assert_array_equal(d["gathered"], d["direct"])
    assert (d["status"] == 0).all()


def test_bench_config3_allgather_line(tmp_path):
    """bench.py --config 3 at N = 1 (the global batch on one GPU, the all-gather a device copy):
    one JSON line with the all-gather timing and the strong-scaling tag."""
    import json
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--config", "3", "--global-batch", "8192",
                        "--steps", "10", "--warmup", "2", "--no-pmc", "--no-cpu"], cwd=ROOT,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["scaling"] == "strong" and line["config"]["allgather"] is True
    assert line["config"]["global_batch"] == 8192 and line["allgather"]["avg_ms"] > 0
    assert line["status_ok_frac"] == 1.0
