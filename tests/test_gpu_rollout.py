"""GPU: MPC-style rollouts through wbq_rollout. Each step solves the
batch, then q_dd = M^-1 (tau - h) (contact form: x[0:n]) and semi-implicit Euler
qd += dt q_dd, q += dt qd on the device; J, M, h and poses are frozen per rollout. The CPU
check runs the same loop with the oracle and numpy: the torques of the last step within the
1e-6 relative tolerance, the states to 1e-9 relative."""
import numpy as np
import pytest

from conftest import rel_err
from qppvm_amd.problem import ContactProblem, QPPVMProblem
from qppvm_amd.synth import contact_instances, qppvm_instances

pytestmark = pytest.mark.gpu
TOL = 1e-6


@pytest.fixture(scope="module")
def wbq_mod():
    from qppvm_amd import build, wbq
    build.build()
    return wbq


def cpu_rollout_qppvm(oracle_lib, prob, inp, steps, dt):
    inp = {k: v.copy() for k, v in inp.items()}
    for _ in range(steps):
        tau, st, _ = oracle_lib.qppvm_batch(prob, inp)
        qdd = np.linalg.solve(inp["M"], (tau - inp["h"])[..., None])[..., 0]
        qdd[st != 0] = 0.0
        inp["qd"] = inp["qd"] + dt * qdd
        inp["q"] = inp["q"] + dt * inp["qd"]
    return tau, st, inp["q"], inp["qd"]


@pytest.mark.parametrize("n,tau_max", [(30, 1e6), (30, None), (39, None)])
def test_rollout_qppvm_matches_cpu_loop(wbq_mod, oracle_lib, n, tau_max):
    base = QPPVMProblem(n=n)
    inp = qppvm_instances(base, 48, seed=90 + n)
    if tau_max is None:  # ~20 % of the torque limits binding along the rollout
        free = QPPVMProblem(n=n, tau_max=1e9)
        tau0, _, _ = oracle_lib.qppvm_batch(free, inp)
        tau_max = float(np.quantile(np.abs(tau0), 0.8))
    prob = QPPVMProblem(n=n, tau_max=tau_max)
    steps, dt = 6, 1e-3
    tau_r, st_r, q_r, qd_r = cpu_rollout_qppvm(oracle_lib, prob, inp, steps, dt)
    s = wbq_mod.QPPVMSolver(prob, max_batch=48)
    s.set_inputs(inp)
    s.rollout(steps, dt)
    tau, st, _ = s.outputs()
    q, qd = s.state()
    s.close()
    np.testing.assert_array_equal(st, st_r)
    ok = st == 0
    assert rel_err(tau[ok], tau_r[ok]) <= TOL
    assert rel_err(qd, qd_r) <= 1e-9 and rel_err(q, q_r) <= 1e-9
    assert np.abs(qd - inp["qd"]).max() > 0.0  # the state did move


def test_rollout_contact_matches_cpu_loop(wbq_mod, oracle_lib):
    prob = ContactProblem(n=30, nc=4)
    inp = contact_instances(prob, 32, seed=77, masks=[0b0011, 0b0111, 0b1111])
    steps, dt = 5, 1e-3
    ref = {k: v.copy() for k, v in inp.items()}
    for _ in range(steps):
        tau_r, x_r, st_r, _, _ = oracle_lib.contact_batch(prob, ref)
        qdd = np.where((st_r == 0)[:, None], x_r[:, :30], 0.0)
        ref["qd"] = ref["qd"] + dt * qdd
        ref["q"] = ref["q"] + dt * ref["qd"]
    s = wbq_mod.ContactSolver(prob, max_batch=32)
    s.set_inputs(inp)
    s.rollout(steps, dt)
    tau, st, _ = s.outputs()
    q, qd = s.state()
    s.close()
    np.testing.assert_array_equal(st, st_r)
    assert rel_err(tau[st == 0], tau_r[st_r == 0]) <= TOL
    assert rel_err(qd, ref["qd"]) <= 1e-9 and rel_err(q, ref["q"]) <= 1e-9


def test_rollout_zero_steps_and_plain_solve_leave_state(wbq_mod):
    prob = QPPVMProblem(n=30, tau_max=1e6)
    inp = qppvm_instances(prob, 8, seed=3)
    s = wbq_mod.QPPVMSolver(prob, max_batch=8)
    s.set_inputs(inp)
    s.rollout(0)
    s.solve()
    q, qd = s.state()
    s.close()
    np.testing.assert_array_equal(q, inp["q"])
    np.testing.assert_array_equal(qd, inp["qd"])


def test_set_state_restarts_rollout(wbq_mod):
    """wbq_set_state: two rollouts from the same start state agree (the second starts warm: the
    warm start changes the path, not the solution, so agreement is to roundoff)."""
    prob = QPPVMProblem(n=30, tau_max=60.0)
    inp = qppvm_instances(prob, 16, seed=5)
    s = wbq_mod.QPPVMSolver(prob, max_batch=16)
    s.set_inputs(inp)
    s.rollout(4, 1e-3)
    q1, qd1 = s.state()
    tau1, _, _ = s.outputs()
    s.set_state(inp["q"], inp["qd"])
    q0, qd0 = s.state()
    np.testing.assert_array_equal(q0, inp["q"])
    s.rollout(4, 1e-3)
    q2, qd2 = s.state()
    tau2, _, _ = s.outputs()
    s.close()
    assert rel_err(q1, q2) <= 1e-12 and rel_err(qd1, qd2) <= 1e-12
    assert rel_err(tau1, tau2) <= 1e-9


def test_rollout_config4_full_size_properties(wbq_mod, oracle_lib):
    """The bench's config-4 workload at full size (4096 plant-scaled rollouts x N = 20, limits at
    the 80 % quantile, repeated from the reset state so the warm start carries over, as bench.py
    runs it): every step of every rollout ends with status 0 -- the level-0 repair's single-point
    case once ended at "no step" (status 2) inside rollouts (scripts/diag_mpc.py) -- and the last
    step's torques carry the KAT-4 certificates (tests/kkt.py): every instance whose last solve
    went through the level-0 repair, plus 128 others."""
    import kkt
    n, B, H, dt = 30, 4096, 20, 1e-3
    inp = qppvm_instances(QPPVMProblem(n=n), B, seed=1, plant=True)
    free = wbq_mod.QPPVMSolver(QPPVMProblem(n=n, tau_max=1e9), max_batch=B)
    tau_free, _, _ = free.solve_batch(inp)
    free.close()
    prob = QPPVMProblem(n=n, tau_max=float(np.quantile(np.abs(tau_free), 0.8)))
    s = wbq_mod.QPPVMSolver(prob, max_batch=B)
    try:
        s.set_inputs(inp)
        repaired = 0
        for rep in range(2):
            s.set_state(inp["q"], inp["qd"])
            for k in range(H):
                if k == H - 1:
                    q_last, qd_last = s.state()
                s.rollout(1, dt)
                tau, st, _ = s.outputs()
                assert np.all(st == 0), (rep, k, np.bincount(st))
                hints = s.warm_hints()
                repaired += int(hints.sum())
        q, qd = s.state()
    finally:
        s.close()
    assert repaired > 0  # the repair path runs along the rollouts
    assert np.all(np.isfinite(q)) and np.all(np.isfinite(qd))
    last = dict(inp, q=q_last, qd=qd_last)
    rng = np.random.default_rng(0)
    check = set(np.where(hints != 0)[0].tolist()) | set(rng.choice(B, 128, replace=False).tolist())
    for b in sorted(check):
        c = kkt.qppvm_certificate(oracle_lib, prob, last, b, tau[b])
        assert max(c["primal"], c["level0"], c["stat"], c["sign"]) <= 1e-9, (b, c)


@pytest.mark.parametrize("plant", [False, True])
def test_rollout_paths_agree(wbq_mod, plant):
    """The execution paths of a rollout give the same answer (include/wbq.h wbq_set_option): one
    launch for the whole rollout (qppvm_rollout_kernel, the default), one launch per step with the
    level-0 repair inline in the fast kernel, and one launch per step with the repair in its own
    kernel. plant=False is the SURVEY 8d distribution, where most instance-steps go through the
    level-0 repair (bench.py --mpc-inputs survey), so every path's repair runs; the statuses and
    warm-start hints agree exactly, the torques and states to roundoff."""
    n, B, H, dt = 30, 256, 8, 1e-3
    inp = qppvm_instances(QPPVMProblem(n=n), B, seed=21, plant=plant)
    free = wbq_mod.QPPVMSolver(QPPVMProblem(n=n, tau_max=1e9), max_batch=B)
    tau_free, _, _ = free.solve_batch(inp)
    free.close()
    prob = QPPVMProblem(n=n, tau_max=float(np.quantile(np.abs(tau_free), 0.8)))
    out = {}
    for name, fused, inl in (("fused", 1, -1), ("steps_inline", 0, 1), ("steps_kernel", 0, 0)):
        s = wbq_mod.QPPVMSolver(prob, max_batch=B)
        try:
            s.set_option(s.OPT_FUSED_ROLLOUT, fused)
            s.set_option(s.OPT_INLINE_REPAIR, inl)
            s.set_inputs(inp)
            s.rollout(H, dt)
            tau, st, _ = s.outputs()
            q, qd = s.state()
            out[name] = (tau, st, q, qd, s.warm_hints())
        finally:
            s.close()
    tau0, st0, q0, qd0, h0 = out["fused"]
    if not plant:
        assert h0.sum() > B // 4  # the repair path carries many of the rollouts
    for name in ("steps_inline", "steps_kernel"):
        tau, st, q, qd, h = out[name]
        np.testing.assert_array_equal(st, st0, err_msg=name)
        np.testing.assert_array_equal(h, h0, err_msg=name)
        assert rel_err(tau, tau0) <= 1e-9, (name, rel_err(tau, tau0))
        assert rel_err(q, q0) <= 1e-12 and rel_err(qd, qd0) <= 1e-10, name


def test_set_option_rejects_bad_values(wbq_mod):
    s = wbq_mod.QPPVMSolver(QPPVMProblem(n=30), max_batch=4)
    try:
        with pytest.raises(wbq_mod.WbqError):
            s.set_option(s.OPT_INLINE_REPAIR, 2)
        with pytest.raises(wbq_mod.WbqError):
            s.set_option(99, 0)
        s.set_option(s.OPT_FUSED_ROLLOUT, 0)
    finally:
        s.close()
