"""CPU oracle (oracle/wbq_oracle.c) pinned to the golden fixtures and closed forms.

The fixtures come from the independent numpy/scipy restatement in
tests/golden/make_golden.py. Tolerance: 1e-9 relative
on tau (the oracle is fp64 throughout; observed <= 2e-11).
"""
import numpy as np
import pytest

from conftest import load_golden, rel_err
from qppvm_amd.problem import QPPVMProblem, SELECT_TASK
from qppvm_amd.synth import qppvm_instances

TOL = 1e-9


@pytest.mark.parametrize("n", [7, 30, 39])
def test_oracle_matches_golden(oracle_lib, n):
    for g, prob, inp, exp in load_golden(n):
        tau, st, it = oracle_lib.qppvm_batch(prob, inp)
        assert np.all(st == exp["status"]), (g, st)
        assert rel_err(tau, exp["tau"]) <= TOL, (g, rel_err(tau, exp["tau"]))
        if "kat" in exp:  # closed form (bounds inactive)
            assert rel_err(tau, exp["kat"]) <= TOL, g


@pytest.mark.parametrize("n", [7, 30, 39])
def test_oracle_level0_value(oracle_lib, n):
    """y* = A0 x0* is unique; compare with scipy's BVLS (fixtures)."""
    for g, prob, inp, exp in load_golden(n):
        for b in range(inp["h"].shape[0]):
            _, y0, st, _ = oracle_lib.qppvm_one(prob, inp, b)
            assert rel_err(y0, exp["y0"][b]) <= TOL, g


def test_cart_error_small_rotation(oracle_lib):
    """e_o ~ theta/2 * axis for a small rotation error; position error p_ref - p."""
    th = 1e-3
    axis = np.array([0.3, -0.5, 0.81])
    axis /= np.linalg.norm(axis)
    K = np.array([[0, -axis[2], axis[1]], [axis[2], 0, -axis[0]], [-axis[1], axis[0], 0]])
    Rd = np.eye(3) + np.sin(th) * K + (1 - np.cos(th)) * K @ K
    pose = np.hstack([np.eye(3), [[1.0], [2.0], [3.0]]]).ravel()
    pose_ref = np.hstack([Rd, [[1.5], [2.0], [2.0]]]).ravel()
    e = oracle_lib.cart_error(pose, pose_ref)
    np.testing.assert_allclose(e[:3], [0.5, 0.0, -1.0], atol=1e-15)
    np.testing.assert_allclose(e[3:], np.sin(th / 2) * axis, rtol=1e-12)


def test_cart_error_half_turn_branches(oracle_lib):
    """Shepperd branches (trace <= 0): 180-degree errors about each axis give |e_o| = 1."""
    for k in range(3):
        Rd = -np.eye(3)
        Rd[k, k] = 1.0
        pose = np.hstack([np.eye(3), np.zeros((3, 1))]).ravel()
        e = oracle_lib.cart_error(pose, np.hstack([Rd, np.zeros((3, 1))]).ravel())
        assert abs(abs(e[3 + k]) - 1.0) < 1e-14


def test_select_modes_differ_only_with_rotation(oracle_lib):
    """SUBTASK vs TASK selection coincide when the task-space force has no rotational part."""
    p1 = QPPVMProblem(n=12, tau_max=1e6, Kc=[700, 700, 700, 0, 0, 0], Dc=0.0)
    p2 = QPPVMProblem(n=12, tau_max=1e6, Kc=[700, 700, 700, 0, 0, 0], Dc=0.0, select_mode=SELECT_TASK)
    inp = qppvm_instances(p1, 4, seed=11)
    t1, s1, _ = oracle_lib.qppvm_batch(p1, inp)
    t2, s2, _ = oracle_lib.qppvm_batch(p2, inp)
    assert np.all(s1 == 0) and np.all(s2 == 0)
    # not equal in general: J M^-1 J^T couples translational rows with the (zero) rotational F
    # only through F, which is zero here -> identical
    assert rel_err(t1, t2) <= 1e-10


def test_infeasible_bounds_fallback(oracle_lib):
    """tau_min > tau_max -> solver failure -> tau = h (QPPVMPlugin.cpp:246-249)."""
    prob = QPPVMProblem(n=10, tau_max=-1.0, tau_min=1.0)
    inp = qppvm_instances(prob, 3, seed=5)
    tau, st, _ = oracle_lib.qppvm_batch(prob, inp)
    assert np.all(st == 2)
    np.testing.assert_array_equal(tau, inp["h"])


@pytest.mark.parametrize("literal", [True, False])
def test_oracle_elbow_stacks(oracle_lib, literal):
    """The oracle's lexicographic elbow stacks against the independent numpy/scipy fixtures
    (tests/golden/make_golden_elbow.py), including the groups where the elbow level is not attained:
    the reference's commented stack ((ee_r + ee_l) / (elbow_l + elbow_r)) << limits with no joint task
    and the minimum-norm x (QPPVMPlugin.cpp:177-178 in place of :179; closed form: the pseudo-inverse
    of the 12 stacked rows), and the three-level extension with the joint task (KAT-1)."""
    from conftest import load_golden_elbow, rel_err
    seen_unattained = 0
    for g, prob, inp, exp in load_golden_elbow(literal):
        tau, st, _ = oracle_lib.qppvm_batch(prob, inp)
        assert (st == 0).all(), g
        assert rel_err(tau, exp["tau"]) <= 1e-8, (g, rel_err(tau, exp["tau"]))
        if "kat" in exp:
            assert rel_err(tau, exp["kat"]) <= 1e-8, g
        for b in range(tau.shape[0]):
            a = oracle_lib.assemble(prob, inp, b)
            seen_unattained += np.abs(exp["y"][b][6:] - a["b0"][6:]).max() > 1e-6 * max(1, np.abs(a["b0"]).max())
    assert seen_unattained >= 4  # the middle level binds in the fixtures


def test_oracle_elbow_literal_minnorm(oracle_lib):
    """Without the joint task the stack's x is the minimum-norm point of the last level's optima: any
    feasible move along the null space of the 12 rows that keeps the box raises ||x|| (checked on the
    bounds-inactive groups by perturbation), and the joint-task stack gives other torques."""
    from conftest import load_golden_elbow, rel_err
    rng = np.random.default_rng(3)
    for g, prob, inp, exp in load_golden_elbow(True):
        if "kat" not in exp:
            continue
        tau, _, _ = oracle_lib.qppvm_batch(prob, inp)
        for b in range(tau.shape[0]):
            a = oracle_lib.assemble(prob, inp, b)
            x = tau[b] - inp["h"][b]
            _, S, Vt = np.linalg.svd(a["A0"])
            Z = Vt[int((S > 1e-12 * S[0]).sum()):].T
            # x lies in the row space of the 12 rows (orthogonal to every feasible direction)
            assert np.abs(Z.T @ x).max() <= 1e-9 * np.linalg.norm(x), g
            for _ in range(8):
                d = Z @ rng.normal(size=Z.shape[1])
                d *= 1e-3 * np.linalg.norm(x) / np.linalg.norm(d)
                assert np.linalg.norm(x + d) > np.linalg.norm(x)
        joint = type(prob)(**{**{k: getattr(prob, k) for k in ("n", "ntasks", "row_mask", "task_level")},
                              "tau_max": prob.tau_max, "joint_task": True})
        tj, _, _ = oracle_lib.qppvm_batch(joint, inp)
        assert rel_err(tj, tau) > 1e-6, g
