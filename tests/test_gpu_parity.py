"""GPU parity: the HIP path (libwbq through the C ABI) against the CPU oracle and the
golden fixtures. Tolerance (BASELINE north_star): tau within 1e-6 relative,
rel = ||tau_gpu - tau_ref||_inf / max(1, ||tau_ref||_inf) per instance; statuses equal.
"""
import numpy as np
import pytest

from conftest import load_golden, rel_err
from qppvm_amd.problem import QPPVMProblem, SELECT_TASK
from qppvm_amd.synth import qppvm_instances, replicate

pytestmark = pytest.mark.gpu
TOL = 1e-6


@pytest.fixture(scope="module")
def wbq_mod():
    from qppvm_amd import build, wbq
    build.build()
    return wbq


def gpu_solve(wbq_mod, prob, inp):
    s = wbq_mod.QPPVMSolver(prob, max_batch=inp["h"].shape[0])
    try:
        return s.solve_batch(inp)
    finally:
        s.close()


def calibrated(prob_kw, n, inp, oracle_lib, frac):
    probe = QPPVMProblem(n=n, **{**prob_kw, "tau_max": 1e6})
    tau, _, _ = oracle_lib.qppvm_batch(probe, inp)
    return QPPVMProblem(n=n, **{**prob_kw, "tau_max": float(np.quantile(np.abs(tau), 1 - frac))})


@pytest.mark.parametrize("n", [7, 30, 39])
def test_golden_fixtures(wbq_mod, n):
    for g, prob, inp, exp in load_golden(n):
        tau, st, it = gpu_solve(wbq_mod, prob, inp)
        # includes the level-0-infeasible groups (infeas0; the n = 7 groups with m0 > n),
        # which go through the in-kernel BVLS repair
        np.testing.assert_array_equal(st, exp["status"], err_msg=g)
        ok = exp["status"] == 0
        assert rel_err(tau[ok], exp["tau"][ok]) <= TOL, (g, rel_err(tau[ok], exp["tau"][ok]))
        np.testing.assert_array_equal(tau[~ok], inp["h"][~ok], err_msg=g)


def level0_gap(prob, inp):
    """max_a |y*_a - b0_a| per instance (oracle): > 0 where level 0 is infeasible at b0."""
    import oracle
    out = []
    for b in range(inp["h"].shape[0]):
        _, y0, _, _ = oracle.qppvm_one(prob, inp, b)
        b0 = oracle.assemble(prob, inp, b)["b0"]
        out.append(np.abs(y0 - b0).max() / max(1.0, np.abs(b0).max()))
    return np.array(out)


@pytest.mark.parametrize("n,kw,tau_max", [
    (7, dict(row_mask=(0x3F, 0x3F)), 1e7),    # m0 = 12 > n: level 0 never attainable (M0 = 12 path)
    (3, dict(), 1e7),                          # m0 = 6 > n = 3
    (30, dict(), 30.0),                        # torque limits too tight for the level-0 targets
    (30, dict(), 100.0),
    (30, dict(row_mask=(0x3F, 0x3F)), 10.0),
    (39, dict(), 30.0),                        # n > 32: split fast / active-set kernels
])
def test_level0_infeasible_repair(wbq_mod, oracle_lib, n, kw, tau_max):
    """y* != b0: the kernel's BVLS level-0 repair, pinning and fresh active set against the
    oracle's wbq_ref_level0 + pinning + level 1 (oracle/wbq_oracle.c:wbq_ref_qppvm_one)."""
    prob = QPPVMProblem(n=n, tau_max=tau_max, **kw)
    inp = qppvm_instances(prob, 24, seed=300 + n)
    tau_r, st_r, _ = oracle_lib.qppvm_batch(prob, inp)
    tau, st, _ = gpu_solve(wbq_mod, prob, inp)
    assert (level0_gap(prob, inp) > 1e-6).sum() >= len(st) // 2  # the case really is exercised
    np.testing.assert_array_equal(st, st_r)
    ok = st_r == 0
    assert ok.sum() >= len(st) - 2
    assert rel_err(tau[ok], tau_r[ok]) <= TOL, rel_err(tau[ok], tau_r[ok])


@pytest.mark.parametrize("n", [1, 3, 6, 12, 24, 30, 31, 32, 33, 39, 48, 64])
def test_random_vs_oracle_bounds_inactive(wbq_mod, oracle_lib, n):
    # level 0 stays feasible (m0 <= n): single task with n rows for tiny n
    kw = dict(ntasks=2, row_mask=(0x7, 0x7)) if n >= 6 else dict(ntasks=1, row_mask=((1 << n) - 1,))
    prob = QPPVMProblem(n=n, tau_max=1e7, **kw)
    inp = qppvm_instances(prob, 37, seed=100 + n)
    tau_r, st_r, _ = oracle_lib.qppvm_batch(prob, inp)
    tau, st, _ = gpu_solve(wbq_mod, prob, inp)
    ok = st_r == 0
    assert np.all(st[ok] == 0)
    assert rel_err(tau[ok], tau_r[ok]) <= TOL


@pytest.mark.parametrize("n,frac", [(12, 0.1), (30, 0.1), (30, 0.25), (30, 0.5), (39, 0.2), (64, 0.2)])
def test_random_vs_oracle_active_bounds(wbq_mod, oracle_lib, n, frac):
    inp = qppvm_instances(QPPVMProblem(n=n), 64, seed=200 + n)
    prob = calibrated({}, n, inp, oracle_lib, frac)
    tau_r, st_r, _ = oracle_lib.qppvm_batch(prob, inp)
    tau, st, it = gpu_solve(wbq_mod, prob, inp)
    assert np.all(st_r == 0)
    assert np.all(st == 0), st
    assert rel_err(tau, tau_r) <= TOL, rel_err(tau, tau_r)
    assert it.max() > 0  # the active set really moved


@pytest.mark.parametrize("n,frac", [(33, 0.5), (40, 0.5), (40, 0.8), (47, 0.6), (64, 0.6)])
def test_saturated_sets_n_sized_layout(wbq_mod, oracle_lib, n, frac):
    """n > 32 with most limits active: the 64-lane active-set kernel's layout holds NR = n rounded up to 8 basis / M / T
    rows (qppvm_repair.h ActiveLayout; n = 40: NR = n, the basis can fill every row). Statuses equal to the oracle's,
    tau within TOL where it solves."""
    inp = qppvm_instances(QPPVMProblem(n=n), 48, seed=700 + n)
    prob = calibrated({}, n, inp, oracle_lib, frac)
    tau_r, st_r, _ = oracle_lib.qppvm_batch(prob, inp)
    tau, st, it = gpu_solve(wbq_mod, prob, inp)
    np.testing.assert_array_equal(st, st_r)
    ok = st_r == 0
    assert ok.sum() >= len(st) // 2
    assert rel_err(tau[ok], tau_r[ok]) <= TOL, rel_err(tau[ok], tau_r[ok])
    assert it.max() > 0


def test_select_task_mode_and_six_rows(wbq_mod, oracle_lib):
    for kw in (dict(select_mode=SELECT_TASK), dict(row_mask=(0x3F, 0x3F)), dict(row_mask=(0x5, 0x38))):
        prob = QPPVMProblem(n=30, tau_max=1e7, **kw)
        inp = qppvm_instances(prob, 16, seed=7)
        tau_r, _, _ = oracle_lib.qppvm_batch(prob, inp)
        tau, st, _ = gpu_solve(wbq_mod, prob, inp)
        assert np.all(st == 0) and rel_err(tau, tau_r) <= TOL, kw


def test_edge_cases(wbq_mod):
    prob = QPPVMProblem(n=30, tau_max=1e7)
    inp = qppvm_instances(prob, 5, seed=3)
    s = wbq_mod.QPPVMSolver(prob, max_batch=8)
    try:
        # empty batch
        s.set_inputs({k: v[:0] for k, v in inp.items()})
        s.solve()
        tau, st, _ = s.outputs()
        assert tau.shape == (0, 30)
        # non-SPD inertia -> status 3, tau = h
        bad = {k: v.copy() for k, v in inp.items()}
        bad["M"][1] = -np.eye(30)
        tau, st, _ = s.solve_batch(bad)
        assert st[1] == 3 and np.array_equal(tau[1], bad["h"][1])
        assert np.all(st[[0, 2, 3, 4]] == 0)
        # capacity
        with pytest.raises(wbq_mod.WbqError):
            s.set_inputs(qppvm_instances(prob, 9, seed=1))
    finally:
        s.close()


def test_crossed_limits_fallback(wbq_mod):
    prob = QPPVMProblem(n=10, tau_max=-1.0, tau_min=1.0)
    inp = qppvm_instances(prob, 3, seed=5)
    tau, st, _ = gpu_solve(wbq_mod, prob, inp)
    assert np.all(st == 2)
    np.testing.assert_array_equal(tau, inp["h"])


def test_config1_identical_full_size(wbq_mod, oracle_lib):
    """BASELINE config 1: 4096 identical instances -> identical outputs == oracle."""
    prob = QPPVMProblem(n=30, tau_max=1e4)
    inp = replicate(qppvm_instances(prob, 1, seed=0), 4096)
    tau_r, st_r, _ = oracle_lib.qppvm_batch(prob, {k: v[:1] for k, v in inp.items()})
    tau, st, _ = gpu_solve(wbq_mod, prob, inp)
    assert np.all(st == 0)
    assert np.all(tau == tau[0])  # bitwise identical across the batch
    assert rel_err(tau[:1], tau_r) <= TOL


def test_full_size_properties(wbq_mod, oracle_lib):
    """B = 8192 random instances, ~20 % active bounds: feasibility on every instance,
    oracle parity on a sample (the oracle is too slow for the whole batch)."""
    n = 30
    inp = qppvm_instances(QPPVMProblem(n=n), 8192, seed=9)
    small = {k: v[:64] for k, v in inp.items()}
    prob = calibrated({}, n, small, oracle_lib, 0.2)
    tau, st, it = gpu_solve(wbq_mod, prob, inp)
    assert np.all(st == 0)
    x = tau - inp["h"]
    lb = prob.tau_min - inp["h"]
    ub = prob.tau_max - inp["h"]
    slack = 1e-9 * np.maximum(1, np.abs(x))
    assert np.all(x >= lb - slack) and np.all(x <= ub + slack)
    idx = np.arange(0, 8192, 97)
    sample = {k: v[idx] for k, v in inp.items()}
    tau_r, st_r, _ = oracle_lib.qppvm_batch(prob, sample)
    assert rel_err(tau[idx], tau_r) <= TOL


@pytest.mark.parametrize("n", [30, 39])
def test_warm_start_changes_path_not_result(wbq_mod, oracle_lib, n):
    """Per-instance warm start (repair hint + BVLS state) carried across solves of one
    context, including stale hints from a different batch, gives the cold results."""
    prob = QPPVMProblem(n=n, tau_max=30.0)
    x = qppvm_instances(prob, 24, seed=400 + n)
    y = qppvm_instances(prob, 24, seed=500 + n)
    tau_c, st_c, _ = gpu_solve(wbq_mod, prob, y)
    s = wbq_mod.QPPVMSolver(prob, max_batch=24)
    try:
        s.solve_batch(x)                 # hints from x
        tau_w, st_w, _ = s.solve_batch(y)  # stale hints on y
        tau_w2, st_w2, _ = s.solve_batch(y)  # own hints
        s.reset_warmstart()
        tau_r, st_r, _ = s.solve_batch(y)
    finally:
        s.close()
    for t, st in ((tau_w, st_w), (tau_w2, st_w2), (tau_r, st_r)):
        np.testing.assert_array_equal(st, st_c)
        assert rel_err(t, tau_c) <= 1e-9
    tau_o, st_o, _ = oracle_lib.qppvm_batch(prob, y)
    np.testing.assert_array_equal(st_c, st_o)
    assert rel_err(tau_c[st_o == 0], tau_o[st_o == 0]) <= TOL
    # stale "repair" hints on instances whose level 0 is feasible: zero task error and
    # velocity give b0 = 0, attainable at x = 0 when |h| <= tau_max
    z = {k: v.copy() for k, v in x.items()}
    z["pose_ref"] = z["pose"].copy()
    z["qd"][:] = 0.0
    z["h"] = np.clip(z["h"], -20.0, 20.0)
    s = wbq_mod.QPPVMSolver(prob, max_batch=24)
    try:
        s.solve_batch(x)
        tau_z, st_z, _ = s.solve_batch(z)
    finally:
        s.close()
    tau_zo, st_zo, _ = oracle_lib.qppvm_batch(prob, z)
    np.testing.assert_array_equal(st_z, st_zo)
    assert rel_err(tau_z, tau_zo) <= TOL
