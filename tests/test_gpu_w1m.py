"""GPU: the inertia-weighted joint task W1 = M (SURVEY.md 8a row a6, KAT-2;
qppvm_amd/csrc/qppvm_w1m_kernel.hip) against the oracle, which solves level 1 in x-space with
H1 = A1^T M A1 = M^-1 (oracle/wbq_oracle.c:wbq_ref_assemble / wbq_ref_level1). Same
tolerance as the W1 = I path: tau within 1e-6 relative, statuses equal."""
import numpy as np
import pytest

from conftest import rel_err
from qppvm_amd.problem import QPPVMProblem, WEIGHT_INERTIA
from qppvm_amd.synth import qppvm_instances

pytestmark = pytest.mark.gpu
TOL = 1e-6


@pytest.fixture(scope="module")
def wbq_mod():
    from qppvm_amd import build, wbq
    build.build()
    return wbq


def solve_both(wbq_mod, oracle_lib, prob, inp):
    tau_r, st_r, _ = oracle_lib.qppvm_batch(prob, inp)
    s = wbq_mod.QPPVMSolver(prob, max_batch=inp["h"].shape[0])
    try:
        tau, st, it = s.solve_batch(inp)
    finally:
        s.close()
    return tau, st, it, tau_r, st_r


def check(tau, st, tau_r, st_r, inp, min_ok):
    np.testing.assert_array_equal(st, st_r)
    ok = st_r == 0
    assert ok.sum() >= min_ok
    assert rel_err(tau[ok], tau_r[ok]) <= TOL, rel_err(tau[ok], tau_r[ok])
    np.testing.assert_array_equal(tau[~ok], inp["h"][~ok])


@pytest.mark.parametrize("n,kw", [(7, {}), (30, {}), (30, dict(row_mask=(0x3F, 0x3F))), (39, {}),
                                  (52, dict(row_mask=(0x3F, 0x3F)))])
def test_w1m_unconstrained(wbq_mod, oracle_lib, n, kw):
    """No binding limit: x = KAT-2's J^T F + (I - J^T Lambda J M^-1) tau_imp."""
    prob = QPPVMProblem(n=n, tau_max=1e9, joint_weight=WEIGHT_INERTIA, **kw)
    inp = qppvm_instances(prob, 40, seed=500 + n)
    tau, st, it, tau_r, st_r = solve_both(wbq_mod, oracle_lib, prob, inp)
    check(tau, st, tau_r, st_r, inp, 40 if prob.m0 <= n else 0)


@pytest.mark.parametrize("n,kw,frac", [(30, {}, 0.1), (30, {}, 0.3), (30, dict(row_mask=(0x3F, 0x3F)), 0.2),
                                       (39, {}, 0.2), (52, dict(row_mask=(0x3F, 0x07)), 0.25)])
def test_w1m_active_limits(wbq_mod, oracle_lib, n, kw, frac):
    """Torque limits calibrated so that about frac of the unconstrained torques bind."""
    free = QPPVMProblem(n=n, tau_max=1e9, joint_weight=WEIGHT_INERTIA, **kw)
    inp = qppvm_instances(free, 48, seed=600 + n)
    tau0, _, _ = oracle_lib.qppvm_batch(free, inp)
    prob = QPPVMProblem(n=n, tau_max=float(np.quantile(np.abs(tau0), 1 - frac)),
                        joint_weight=WEIGHT_INERTIA, **kw)
    tau, st, it, tau_r, st_r = solve_both(wbq_mod, oracle_lib, prob, inp)
    check(tau, st, tau_r, st_r, inp, 40)
    assert (it > 0).sum() >= 24  # the active set really ran


@pytest.mark.parametrize("n,kw,tau_max", [(7, dict(row_mask=(0x3F, 0x3F)), 1e7), (30, {}, 30.0),
                                          (30, dict(row_mask=(0x3F, 0x3F)), 10.0), (39, {}, 30.0)])
def test_w1m_level0_repair(wbq_mod, oracle_lib, n, kw, tau_max):
    """Level 0 not attainable at b0: BVLS y* and pins, then the W1 = M level 1 again."""
    prob = QPPVMProblem(n=n, tau_max=tau_max, joint_weight=WEIGHT_INERTIA, **kw)
    inp = qppvm_instances(prob, 24, seed=700 + n)
    tau, st, it, tau_r, st_r = solve_both(wbq_mod, oracle_lib, prob, inp)
    check(tau, st, tau_r, st_r, inp, 20)


def test_w1m_differs_from_identity(wbq_mod, oracle_lib):
    """The weight matters once limits bind (with none binding both give the same level-1
    optimum only when level 0 fixes it), so a silent W1 = I fallback would be caught."""
    free = QPPVMProblem(n=30, tau_max=1e9, joint_weight=WEIGHT_INERTIA)
    inp = qppvm_instances(free, 32, seed=808)
    tm = float(np.quantile(np.abs(oracle_lib.qppvm_batch(free, inp)[0]), 0.8))
    pm = QPPVMProblem(n=30, tau_max=tm, joint_weight=WEIGHT_INERTIA)
    pi = QPPVMProblem(n=30, tau_max=tm)
    tm_gpu = solve_both(wbq_mod, oracle_lib, pm, inp)[0]
    ti_gpu = solve_both(wbq_mod, oracle_lib, pi, inp)[0]
    assert rel_err(tm_gpu, ti_gpu) > 1e-3


def test_w1m_rollout(wbq_mod, oracle_lib):
    prob = QPPVMProblem(n=30, tau_max=60.0, joint_weight=WEIGHT_INERTIA)
    inp = qppvm_instances(prob, 24, seed=909)
    steps, dt = 4, 1e-3
    ref = {k: v.copy() for k, v in inp.items()}
    for _ in range(steps):
        tau_r, st_r, _ = oracle_lib.qppvm_batch(prob, ref)
        qdd = np.linalg.solve(ref["M"], (tau_r - ref["h"])[..., None])[..., 0]
        qdd[st_r != 0] = 0.0
        ref["qd"] = ref["qd"] + dt * qdd
        ref["q"] = ref["q"] + dt * ref["qd"]
    s = wbq_mod.QPPVMSolver(prob, max_batch=24)
    s.set_inputs(inp)
    s.rollout(steps, dt)
    tau, st, _ = s.outputs()
    q, qd = s.state()
    s.close()
    np.testing.assert_array_equal(st, st_r)
    assert rel_err(tau[st == 0], tau_r[st_r == 0]) <= TOL
    assert rel_err(qd, ref["qd"]) <= 1e-9 and rel_err(q, ref["q"]) <= 1e-9
