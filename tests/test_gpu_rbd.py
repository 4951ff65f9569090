"""GPU: batched rigid-body dynamics (qppvm_amd/csrc/rbd.hip) against the oracle's
link-frame recursions (oracle/wbq_oracle_rbd.c, itself pinned to closed forms and derivative
properties in tests/test_rbd_oracle.py), and MPC rollouts that re-evaluate the model every step
(wbq_rollout_rbd) against the same loop on the CPU. fp64: 1e-11 relative for the model
quantities, the solver's 1e-6 for the torques."""
import numpy as np
import pytest

import oracle
from conftest import rel_err
from qppvm_amd.problem import QPPVMProblem
from qppvm_amd.rbd import centauro_like, random_tree, serial_chain

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rbd_mod():
    from qppvm_amd import build, rbd
    build.build()
    return rbd


@pytest.mark.parametrize("maker,B", [(centauro_like, 256), (serial_chain, 128), (lambda: serial_chain(64, 4), 32),
                                     (lambda: random_tree([-1, 0, 0, 1, 1, 2, 5, -1, 7], seed=9, task_link=(6, 8)), 64)])
def test_rbd_matches_oracle(rbd_mod, maker, B):
    model = maker()
    rng = np.random.default_rng(11)
    q, qd = rng.uniform(-np.pi, np.pi, (B, model.n)), rng.normal(0, 1.5, (B, model.n))
    r = rbd_mod.RBDModel(model, max_batch=B)
    M, h, J, pose = r.compute(q, qd)
    r.close()
    Mr, hr, Jr, Pr = oracle.rbd_batch(model, q, qd)
    assert rel_err(M, Mr) <= 1e-11, rel_err(M, Mr)
    assert rel_err(h, hr) <= 1e-11, rel_err(h, hr)
    assert rel_err(J, Jr) <= 1e-11, rel_err(J, Jr)
    assert rel_err(pose, Pr) <= 1e-12, rel_err(pose, Pr)


def test_rbd_closed_forms(rbd_mod):
    from test_rbd_oracle import pendulum, two_link, two_link_closed_form
    r = rbd_mod.RBDModel(two_link(), max_batch=16)
    rng = np.random.default_rng(3)
    q, qd = rng.uniform(-np.pi, np.pi, (16, 2)), rng.normal(0, 2, (16, 2))
    M, h, _, _ = r.compute(q, qd)
    r.close()
    for b in range(16):
        Mc, hc = two_link_closed_form(q[b], qd[b])
        np.testing.assert_allclose(M[b], Mc, rtol=1e-13, atol=1e-13)
        np.testing.assert_allclose(h[b], hc, rtol=1e-12, atol=1e-12)
    r = rbd_mod.RBDModel(pendulum(), max_batch=4)
    M, h, _, _ = r.compute(np.array([[0.3], [1.1], [-2.0], [3.0]]), np.zeros((4, 1)))
    r.close()
    np.testing.assert_allclose(M[:, 0, 0], 0.05 + 2.0 * 0.49, rtol=1e-14)
    np.testing.assert_allclose(h[:, 0], 2.0 * 9.81 * 0.7 * np.sin([0.3, 1.1, -2.0, 3.0]), rtol=1e-13, atol=1e-13)


def test_rbd_device_pointers(rbd_mod):
    import torch
    model = centauro_like()
    B, n, T = 64, model.n, model.ntasks
    rng = np.random.default_rng(2)
    q, qd = rng.uniform(-1, 1, (B, n)), rng.normal(0, 1, (B, n))
    dev = torch.device("cuda:0")
    tq, tqd = torch.from_numpy(q).to(dev), torch.from_numpy(qd).to(dev)
    out = [torch.empty(s, dtype=torch.float64, device=dev) for s in ((B, n, n), (B, n), (B, T, 6, n), (B, T, 12))]
    r = rbd_mod.RBDModel(model, max_batch=B)
    r.set_stream(torch.cuda.current_stream().cuda_stream)
    r.compute_device(B, tq.data_ptr(), tqd.data_ptr(), *[o.data_ptr() for o in out])
    torch.cuda.synchronize()
    M, h, J, pose = r.compute(q, qd)
    r.close()
    for a, b_ in zip(out, (M, h, J, pose)):
        np.testing.assert_array_equal(a.cpu().numpy(), b_)


def test_rollout_rbd_matches_cpu_loop(rbd_mod, oracle_lib):
    """wbq_rollout_rbd: every step M, h, J, poses from the integrated state, then the QPPVM solve
    and semi-implicit Euler -- physically consistent rollouts."""
    from qppvm_amd import wbq
    model = centauro_like()
    B, n, steps, dt = 32, model.n, 12, 1e-3
    rng = np.random.default_rng(4)
    q0, qd0 = rng.uniform(-0.5, 0.5, (B, n)), rng.normal(0, 0.5, (B, n))
    M, h, J, pose = oracle.rbd_batch(model, q0, qd0)
    # references: the start poses moved by 2 cm, joint reference the start posture
    pref = pose.copy()
    pref[:, :, [3, 7, 11]] += rng.normal(0, 0.02, (B, 2, 3))
    inp = dict(M=M, J=J, pose=pose, pose_ref=pref, q=q0, qd=qd0, qref=q0.copy(), h=h)
    prob = QPPVMProblem(n=n, tau_max=400.0)
    cur = {k: v.copy() for k, v in inp.items()}
    for _ in range(steps):  # CPU: oracle model + oracle solve + Euler
        cur["M"], cur["h"], cur["J"], cur["pose"] = oracle.rbd_batch(model, cur["q"], cur["qd"])
        tau_r, st_r, _ = oracle_lib.qppvm_batch(prob, cur)
        qdd = np.linalg.solve(cur["M"], (tau_r - cur["h"])[..., None])[..., 0]
        qdd[st_r != 0] = 0.0
        cur["qd"] = cur["qd"] + dt * qdd
        cur["q"] = cur["q"] + dt * cur["qd"]
    r = rbd_mod.RBDModel(model, max_batch=B)
    s = wbq.QPPVMSolver(prob, max_batch=B)
    s.set_inputs(inp)
    s.rollout_rbd(r, steps, dt)
    tau, st, _ = s.outputs()
    q, qd = s.state()
    s.close()
    r.close()
    np.testing.assert_array_equal(st, st_r)
    assert (st == 0).all()
    assert rel_err(tau, tau_r) <= 1e-6, rel_err(tau, tau_r)
    assert rel_err(qd, cur["qd"]) <= 1e-9 and rel_err(q, cur["q"]) <= 1e-9
    assert np.abs(qd - qd0).max() > 1e-3  # the state moved


def _urdf(name, tasks, fb):
    import os
    from qppvm_amd.urdf import load_urdf
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", name)
    return load_urdf(path, task_links=tasks, floating_base=fb).model


FEET = ["foot_fl", "foot_fr", "foot_hr", "foot_hl"]


@pytest.mark.parametrize("name,tasks,fb", [("quadruped.urdf", ["pelvis"] + FEET, True),
                                           ("centauro_arms.urdf", ["arm2_ee", "arm1_ee"], False)])
def test_rbd_urdf_matches_oracle(rbd_mod, name, tasks, fb):
    """URDF models (tests/golden/*.urdf through qppvm_amd/urdf.py): the six-joint floating base,
    a prismatic joint, task frames behind fixed joints, and Jdot qd (wbq_rbd_compute_ex)."""
    model = _urdf(name, tasks, fb)
    B = 96
    rng = np.random.default_rng(12)
    q, qd = rng.uniform(-0.8, 0.8, (B, model.n)), rng.normal(0, 1.5, (B, model.n))
    r = rbd_mod.RBDModel(model, max_batch=B)
    M, h, J, pose, jd = r.compute_jdqd(q, qd)
    r.close()
    Mr, hr, Jr, Pr = oracle.rbd_batch(model, q, qd)
    jdr = oracle.task_jdqd(model, q, qd)
    assert rel_err(M, Mr) <= 1e-11, rel_err(M, Mr)
    assert rel_err(h, hr) <= 1e-11, rel_err(h, hr)
    assert rel_err(J.reshape(B, -1), Jr.reshape(B, -1)) <= 1e-11
    assert rel_err(pose.reshape(B, -1), Pr.reshape(B, -1)) <= 1e-12
    assert rel_err(jd.reshape(B, -1), jdr.reshape(B, -1)) <= 1e-11, rel_err(jd.reshape(B, -1), jdr.reshape(B, -1))


def test_contact_rollout_rbd_matches_cpu_loop(rbd_mod, oracle_lib):
    """ForceAcc on the device model: every step M, h, the waist (pelvis) and the four foot frames
    (Jacobian, pose, Jdot qd) are re-evaluated from the integrated state on the floating-base URDF
    quadruped, then the contact-form solve integrates qdd = x[0:n] (wbq_rollout_rbd) -- against the
    oracle model + oracle contact solve + Euler on the CPU (ForceAcc.cpp:184-226)."""
    from qppvm_amd import wbq
    from qppvm_amd.problem import ContactProblem
    model = _urdf("quadruped.urdf", ["pelvis"] + FEET, True)
    B, n, nc, steps, dt = 32, model.n, 4, 8, 1e-3
    rng = np.random.default_rng(4)
    q0 = rng.uniform(-0.3, 0.3, (B, n))
    q0[:, 2] += 0.6
    qd0 = rng.normal(0, 0.3, (B, n))

    def model_inputs(q, qd):
        M, h, J, pose = oracle.rbd_batch(model, q, qd)
        jd = oracle.task_jdqd(model, q, qd)
        return dict(M=M, h=h, Jw=J[:, 0], jdqd_w=jd[:, 0], pose_w=pose[:, 0], Jc=np.ascontiguousarray(J[:, 1:]),
                    jdqd_c=np.ascontiguousarray(jd[:, 1:]), pose_c=np.ascontiguousarray(pose[:, 1:]))
    mi = model_inputs(q0, qd0)
    pw_ref = mi["pose_w"].copy()
    pw_ref[:, 11] -= 0.1  # ForceAcc.cpp:181: the pelvis 10 cm below its start
    inp = dict(q=q0.copy(), qd=qd0.copy(), qref=q0.copy(), pose_w_ref=pw_ref, pose_c_ref=mi["pose_c"].copy(),
               cmask=np.full(B, 15, np.int32), **mi)
    prob = ContactProblem(n=n, nc=nc)
    cur = {k: v.copy() for k, v in inp.items()}
    for _ in range(steps):
        cur.update(model_inputs(cur["q"], cur["qd"]))
        tau_r, x_r, st_r, _, _ = oracle_lib.contact_batch(prob, cur)
        qdd = x_r[:, :n].copy()
        qdd[st_r != 0] = 0.0
        cur["qd"] = cur["qd"] + dt * qdd
        cur["q"] = cur["q"] + dt * cur["qd"]
    r = rbd_mod.RBDModel(model, max_batch=B)
    s = wbq.ContactSolver(prob, max_batch=B)
    s.set_inputs(inp)
    s.rollout_rbd(r, steps, dt)
    tau, st, _ = s.outputs()
    q, qd = s.state()
    s.close()
    r.close()
    np.testing.assert_array_equal(st, st_r)
    assert (st == 0).all()
    assert rel_err(tau, tau_r) <= 1e-6, rel_err(tau, tau_r)
    assert rel_err(qd, cur["qd"]) <= 1e-9 and rel_err(q, cur["q"]) <= 1e-9
    assert np.abs(qd - qd0).max() > 1e-3
