"""GPU parity of the QPPVM stacks with the elbow level (src/QPPVMPlugin.cpp:154-166
_elbow_task_left/right, task_level (0, 0, 1, 1)):
* the reference's commented stack, closed at :178 in place of :179,
  ((ee_r + ee_l) / (elbow_l + elbow_r)) << torque_limits -- no joint task (wbq_desc no_joint_task),
  x the minimum-norm point of the last level's optima (the eps -> 0 limit of QPOases_sot's
  regularisation, :188): the constraint-space kernel with H = I (qppvm_w1m_kernel.hip);
* the three-level extension ((ee_r + ee_l) / (elbow_l + elbow_r)) / joint << torque_limits: the fast
  kernel with the 12 stacked rows (W1 = I) or the constraint-space kernel (W1 = M).
Level repairs: the level-0 BVLS, then the middle level by bvls_eq in the null space of the level-0
rows (qppvm_amd/csrc/qppvm_repair.h). Against the independent numpy/scipy fixtures
(tests/golden/make_golden_elbow.py) and the oracle (oracle/wbq_oracle.c:wbq_ref_level_mid).
Tolerance: tau within 1e-6 relative, statuses equal."""
import numpy as np
import pytest

from conftest import load_golden_elbow, rel_err
from qppvm_amd.problem import QPPVMProblem
from qppvm_amd.synth import qppvm_instances

pytestmark = pytest.mark.gpu
TOL = 1e-6
TASKS = dict(ntasks=4, row_mask=(7, 7, 7, 7), task_level=(0, 0, 1, 1))


@pytest.fixture(scope="module")
def wbq_mod():
    from qppvm_amd import build, wbq
    build.build()
    return wbq


def gpu(wbq_mod, prob, inp):
    s = wbq_mod.QPPVMSolver(prob, max_batch=max(1, inp["h"].shape[0]))
    try:
        return s.solve_batch(inp)
    finally:
        s.close()


@pytest.mark.parametrize("literal", [True, False])
def test_elbow_golden(wbq_mod, literal):
    for g, prob, inp, exp in load_golden_elbow(literal):
        tau, st, _ = gpu(wbq_mod, prob, inp)
        assert (st == 0).all(), (g, st)
        assert rel_err(tau, exp["tau"]) <= TOL, (g, rel_err(tau, exp["tau"]))


@pytest.mark.parametrize("joint", [False, True])
@pytest.mark.parametrize("n,q", [(14, 0.8), (14, 0.5), (14, 0.2), (30, 0.5), (30, 0.15), (39, 0.3), (39, 0.12),
                                 (20, 0.3)])
def test_elbow_vs_oracle(wbq_mod, oracle_lib, n, q, joint):
    """Random states with the torque limits at a quantile of the free |tau|: the elbow level is
    unattained on part of the instances (n = 14, 20 and the tight n = 39 groups); statuses equal the
    oracle's, tau within 1e-6, and the lexicographic certificate (tests/kkt.py) holds on every one.
    joint = False: the reference's commented stack (no joint task, min-norm x)."""
    import kkt
    free = QPPVMProblem(n=n, tau_max=1e9, joint_task=joint, **TASKS)
    inp = qppvm_instances(free, 64, seed=500 + n + int(100 * q))
    t0, _, _ = oracle_lib.qppvm_batch(free, inp)
    prob = QPPVMProblem(n=n, tau_max=float(np.quantile(np.abs(t0), q)), joint_task=joint, **TASKS)
    tau_r, st_r, _ = oracle_lib.qppvm_batch(prob, inp)
    tau, st, it = gpu(wbq_mod, prob, inp)
    np.testing.assert_array_equal(st, st_r)
    ok = st == 0
    assert ok.sum() >= 60
    assert rel_err(tau[ok], tau_r[ok]) <= TOL, rel_err(tau[ok], tau_r[ok])
    for b in np.where(ok)[0][:24]:
        c = kkt.qppvm_certificate(oracle_lib, prob, inp, b, tau[b])
        assert max(c["primal"], c["level0"], c["stat"], c["sign"]) <= 1e-9, (b, c)


@pytest.mark.parametrize("n", [14, 39])
def test_split_six_row_stack_vs_oracle(wbq_mod, oracle_lib, n):
    """Two 3-row tasks on two levels (6 rows in total): both the n <= 32 and the n > 32 launch must
    take the instantiation that carries the middle level -- the 6-row one would solve the rows as
    one summed level (the n > 32 branch once did)."""
    tasks = dict(ntasks=2, row_mask=(7, 7), task_level=(0, 1))
    free = QPPVMProblem(n=n, tau_max=1e9, **tasks)
    inp = qppvm_instances(free, 64, seed=900 + n)
    t0, _, _ = oracle_lib.qppvm_batch(free, inp)
    for q in (0.9, 0.3):
        prob = QPPVMProblem(n=n, tau_max=float(np.quantile(np.abs(t0), q)), **tasks)
        tau_r, st_r, _ = oracle_lib.qppvm_batch(prob, inp)
        tau, st, _ = gpu(wbq_mod, prob, inp)
        np.testing.assert_array_equal(st, st_r)
        ok = st == 0
        assert ok.sum() >= 60
        assert rel_err(tau[ok], tau_r[ok]) <= TOL, (q, rel_err(tau[ok], tau_r[ok]))


def test_elbow_differs_from_summed_stack(wbq_mod, oracle_lib):
    """Where the limits bind at n = 14 the lexicographic elbow level gives other torques than the four
    tasks summed on one level (the reference's live stack with the elbows added to level 0)."""
    n = 14
    free = QPPVMProblem(n=n, tau_max=1e9, **TASKS)
    inp = qppvm_instances(free, 64, seed=5)
    t0, _, _ = oracle_lib.qppvm_batch(free, inp)
    tm = float(np.quantile(np.abs(t0), 0.4))
    t3, s3, _ = gpu(wbq_mod, QPPVMProblem(n=n, tau_max=tm, **TASKS), inp)
    t2, s2, _ = gpu(wbq_mod, QPPVMProblem(n=n, tau_max=tm, ntasks=4, row_mask=(7, 7, 7, 7)), inp)
    assert (s3 == 0).all() and (s2 == 0).all()
    assert (np.abs(t3 - t2).max(axis=1) > 1e-6 * np.abs(t2).max(axis=1)).sum() >= 16


@pytest.mark.parametrize("n", [14, 30, 39])
def test_elbow_w1m_vs_oracle(wbq_mod, oracle_lib, n):
    """The three-level extension with the inertia-weighted joint task (W1 = M, KAT-2's weight): the
    constraint-space kernel with every Cartesian row an equality and the two-level repair."""
    import kkt
    free = QPPVMProblem(n=n, tau_max=1e9, joint_weight=1, **TASKS)
    inp = qppvm_instances(free, 64, seed=700 + n)
    t0, _, _ = oracle_lib.qppvm_batch(free, inp)
    for q in (0.9, 0.3):
        prob = QPPVMProblem(n=n, tau_max=float(np.quantile(np.abs(t0), q)), joint_weight=1, **TASKS)
        tau_r, st_r, _ = oracle_lib.qppvm_batch(prob, inp)
        tau, st, _ = gpu(wbq_mod, prob, inp)
        np.testing.assert_array_equal(st, st_r)
        ok = st == 0
        assert ok.sum() >= 60
        assert rel_err(tau[ok], tau_r[ok]) <= TOL, (q, rel_err(tau[ok], tau_r[ok]))
        for b in np.where(ok)[0][:16]:
            c = kkt.qppvm_certificate(oracle_lib, prob, inp, b, tau[b])
            assert max(c["primal"], c["level0"], c["stat"], c["sign"]) <= 1e-9, (b, c)


def test_elbow_unsupported_shapes(wbq_mod):
    """At most 6 rows per Cartesian level, m0 + n <= 64 for the constraint-space stacks, and no
    rollout without the joint task (its qdd = M^-1 x is not carried): other shapes are refused
    (WBQ_E_UNSUPPORTED), never solved as a different stack."""
    with pytest.raises(wbq_mod.WbqError):
        wbq_mod.QPPVMSolver(QPPVMProblem(n=30, ntasks=4, row_mask=(0x3F, 0x3F, 7, 7), task_level=(0, 0, 1, 1)),
                            max_batch=4)
    with pytest.raises(wbq_mod.WbqError):
        wbq_mod.QPPVMSolver(QPPVMProblem(n=60, joint_task=False, **TASKS), max_batch=4)
    prob = QPPVMProblem(n=14, joint_task=False, **TASKS)
    s = wbq_mod.QPPVMSolver(prob, max_batch=4)
    try:
        s.set_inputs(qppvm_instances(prob, 4, seed=1))
        with pytest.raises(wbq_mod.WbqError):
            s.rollout(2, 1e-3)
    finally:
        s.close()
