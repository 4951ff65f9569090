"""BASELINE config 0 end to end: the XBot plugin shell (QPPVMPlugin over the C ABI) driven by
the dummy-mode loop on the synthetic n = 39 robot. The driver dumps each tick's solver
inputs and the torque the plugin applied; the oracle re-solves every dumped tick
(tolerance 1e-6 relative, statuses equal). With 150 Nm limits most ticks are level-0
infeasible, so this also covers the repair kernel through the plugin path."""
import os
import subprocess

import numpy as np
import pytest

from conftest import rel_err
from qppvm_amd.problem import QPPVMProblem

pytestmark = pytest.mark.gpu
TOL = 1e-6


def read_dump(path):
    raw = open(path, "rb").read()
    n, ticks = np.frombuffer(raw[:8], dtype=np.int32)
    off = 8
    f64 = lambda k: np.frombuffer(raw[off:off + 8 * k], dtype=np.float64)  # noqa: E731
    qref = f64(n).copy(); off += 8 * n
    pose_ref = f64(24).copy(); off += 8 * 24
    rec = {k: [] for k in ("M", "J", "pose", "q", "qd", "h", "tau", "status")}
    for _ in range(ticks):
        rec["M"].append(f64(n * n).reshape(n, n)); off += 8 * n * n
        rec["J"].append(f64(12 * n).reshape(2, 6, n)); off += 8 * 12 * n
        rec["pose"].append(f64(24)); off += 8 * 24
        for k in ("q", "qd", "h", "tau"):
            rec[k].append(f64(n)); off += 8 * n
        rec["status"].append(int(np.frombuffer(raw[off:off + 4], dtype=np.int32)[0])); off += 4
    assert off == len(raw)
    out = {k: np.array(v) for k, v in rec.items()}
    B = len(out["q"])
    out["qref"] = np.tile(qref, (B, 1))
    out["pose_ref"] = np.tile(pose_ref, (B, 1))
    return int(n), out


def test_dummy_driver_matches_oracle(tmp_path, oracle_lib):
    from qppvm_amd import build
    _, driver = build.build_plugins()
    dump = str(tmp_path / "dump.bin")
    r = subprocess.run([driver, "--ticks", "300", "--dump", dump, "40"], capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    n, d = read_dump(dump)
    prob = QPPVMProblem(n=n, tau_max=150.0)
    inp = {k: np.ascontiguousarray(d[k]) for k in ("M", "J", "pose", "pose_ref", "q", "qd", "qref", "h")}
    tau_r, st_r, _ = oracle_lib.qppvm_batch(prob, inp)
    np.testing.assert_array_equal(d["status"], st_r)
    ok = st_r == 0
    assert ok.sum() >= len(ok) - 2
    assert rel_err(d["tau"][ok], tau_r[ok]) <= TOL, rel_err(d["tau"][ok], tau_r[ok])
