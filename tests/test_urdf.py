"""CPU: the URDF reader (qppvm_amd/urdf.py) and the rigid-body oracle's extensions for it
(oracle/wbq_oracle_rbd.c: prismatic joints, the six-joint floating base, task frames behind fixed
joints, Jdot qd), SURVEY.md 8f-1. Fixtures: tests/golden/{quadruped,centauro_arms}.urdf (written by
tests/golden/make_urdf.py). Closed forms (prismatic mass, pendulum centripetal acceleration) and the
properties every correct model satisfies: M symmetric positive definite, RNEA = M qdd + h,
J = d pose / dq and Jdot qd = (d/dt J) qd by finite differences, the floating base carries the total
weight, gravity torques = dU/dq."""
import os

import numpy as np
import pytest

import oracle
from qppvm_amd.rbd import PRISMATIC, RobotModel, with_floating_base
from qppvm_amd.urdf import load_urdf, rpy_matrix

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FEET = ["foot_fl", "foot_fr", "foot_hr", "foot_hl"]


def quadruped():
    return load_urdf(os.path.join(GOLDEN, "quadruped.urdf"), task_links=["pelvis"] + FEET, floating_base=True)


def arms():
    return load_urdf(os.path.join(GOLDEN, "centauro_arms.urdf"), task_links=["arm2_ee", "arm1_ee"])


def test_rpy_convention():
    # URDF: R = Rz(y) Ry(p) Rx(r); a pure yaw of 90 deg maps x to y
    np.testing.assert_allclose(rpy_matrix((0, 0, np.pi / 2)) @ [1, 0, 0], [0, 1, 0], atol=1e-15)
    np.testing.assert_allclose(rpy_matrix((np.pi / 2, 0, 0)) @ [0, 1, 0], [0, 0, 1], atol=1e-15)


def test_urdf_structure():
    ur = quadruped()
    m = ur.model
    assert m.n == 30 and list(m.jtype[:6]) == [PRISMATIC] * 3 + [0] * 3
    assert int((m.jtype[6:] == PRISMATIC).sum()) == 1  # the hr slider
    # every link's mass lands on some body (fixed feet and soles lumped into the ankles)
    assert m.mass.sum() == pytest.approx(18.0 + sum(2.5 - 0.3 * k + 0.1 * li for li in range(4) for k in range(6))
                                         + 4 * (0.3 + 0.2))
    assert ur.effort[:6].tolist() == [0.0] * 6 and ur.effort[6] == 120.0
    assert [ur.frames[f][0] for f in FEET] == [11, 17, 23, 29]
    a = arms().model
    assert a.n == 15 and list(a.task_link) == [14, 7]


def test_prismatic_closed_form():
    m = RobotModel(parent=np.array([-1], np.int32), X_fixed=np.array([[1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0.]]),
                   axis=np.array([[0, 0, 1.0]]), mass=np.array([3.0]), com=np.array([[0.1, 0, 0]]),
                   inertia=np.array([[0.1, 0.1, 0.1, 0, 0, 0]]), task_link=np.array([0], np.int32),
                   jtype=np.array([PRISMATIC], np.int32))
    M, h, J, pose = oracle.rbd_batch(m, [[0.4]], [[1.5]])
    np.testing.assert_allclose(M[0], [[3.0]], rtol=1e-15)
    np.testing.assert_allclose(h[0], [3.0 * 9.81], rtol=1e-15)
    np.testing.assert_allclose(J[0, 0, :, 0], [0, 0, 1, 0, 0, 0], atol=1e-15)
    np.testing.assert_allclose(pose[0, 0, 11], 0.4, rtol=1e-15)


def test_jdqd_pendulum_closed_form():
    """A frame at distance l on a pendulum: Jdot qd = the centripetal acceleration -qd^2 l toward
    the axis, zero angular part."""
    from test_rbd_oracle import pendulum
    m = pendulum()
    l = 0.7
    m.task_offset = np.array([[1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, -l]], dtype=float)
    for q, qd in ((0.3, 1.2), (-1.0, 2.5)):
        jd = oracle.task_jdqd(m, [[q]], [[qd]])[0, 0]
        _, _, _, pose = oracle.rbd_batch(m, [[q]], [[qd]])
        p = pose[0, 0, [3, 7, 11]]
        np.testing.assert_allclose(jd[:3], -qd * qd * p, atol=1e-14)
        np.testing.assert_allclose(jd[3:], 0.0, atol=1e-15)


def _frames(model, q):
    _, _, J, pose = oracle.rbd_batch(model, q[None], np.zeros((1, model.n)))
    return J[0], pose[0]


@pytest.mark.parametrize("which", ["quadruped", "arms"])
def test_urdf_model_properties(which):
    model = quadruped().model if which == "quadruped" else arms().model
    n, T = model.n, model.ntasks
    rng = np.random.default_rng(8)
    q, qd, qdd = rng.uniform(-0.6, 0.6, n), rng.normal(0, 1, n), rng.normal(0, 1, n)
    M, h, J, pose = (v[0] for v in oracle.rbd_batch(model, q, qd))
    np.testing.assert_allclose(M, M.T, rtol=0, atol=1e-12 * np.abs(M).max())
    assert np.linalg.eigvalsh(M).min() > 0
    np.testing.assert_allclose(oracle.rnea(model, q, qd, qdd), M @ qdd + h, rtol=1e-11, atol=1e-10)
    eps = 1e-6
    for j in range(n):  # J = d pose / dq (task frames behind fixed joints included)
        dq = np.zeros(n); dq[j] = eps
        _, Pp = _frames(model, q + dq)
        _, Pm = _frames(model, q - dq)
        for t in range(T):
            R = pose[t].reshape(3, 4)[:, :3]
            lin = (Pp[t].reshape(3, 4)[:, 3] - Pm[t].reshape(3, 4)[:, 3]) / (2 * eps)
            W = (Pp[t].reshape(3, 4)[:, :3] - Pm[t].reshape(3, 4)[:, :3]) / (2 * eps) @ R.T
            np.testing.assert_allclose(J[t, :3, j], lin, atol=1e-8)
            np.testing.assert_allclose(J[t, 3:, j], [W[2, 1], W[0, 2], W[1, 0]], atol=1e-8)
    # Jdot qd = d/ds [J(q + s qd) qd] at s = 0
    jd = oracle.task_jdqd(model, q[None], qd[None])[0]
    Jp, _ = _frames(model, q + eps * qd)
    Jm, _ = _frames(model, q - eps * qd)
    np.testing.assert_allclose(jd, np.einsum("trn,n->tr", (Jp - Jm) / (2 * eps), qd), rtol=1e-6, atol=1e-7)


def test_floating_base_weight_and_gravity():
    """Floating base at rest: the base's three force rows carry the total weight; the gravity
    torques are dU/dq (U = -sum m_i g . c_i, COMs by forward kinematics)."""
    model = quadruped().model
    n = model.n
    rng = np.random.default_rng(3)
    q = rng.uniform(-0.5, 0.5, n)
    _, g0, _, _ = oracle.rbd_batch(model, q[None], np.zeros((1, n)))
    g0 = g0[0]
    # translation joints: world x, y, z (the prismatic base joints come first, unrotated)
    np.testing.assert_allclose(g0[:3], [0, 0, 9.81 * model.mass.sum()], rtol=1e-12, atol=1e-9)

    def U(qq):
        tot = 0.0
        for i in range(n):
            mi = RobotModel(parent=model.parent, X_fixed=model.X_fixed, axis=model.axis, mass=model.mass,
                            com=model.com, inertia=model.inertia, task_link=np.array([i], np.int32), jtype=model.jtype)
            P = _frames(mi, qq)[1][0].reshape(3, 4)
            tot -= model.mass[i] * np.dot(model.gravity, P[:, :3] @ model.com[i] + P[:, 3])
        return tot
    for j in (3, 4, 5, 7, 14, 25, 28):
        dq = np.zeros(n); dq[j] = 1e-6
        np.testing.assert_allclose(g0[j], (U(q + dq) - U(q - dq)) / 2e-6, rtol=1e-6, atol=1e-6)


def test_with_floating_base_free_body():
    """A single free body: M at the zero configuration is blockdiag(m I, I_com) for a COM at the
    base origin (the ZYX Euler rates are body rates there)."""
    body = RobotModel(parent=np.zeros(0, np.int32), X_fixed=np.zeros((0, 12)), axis=np.zeros((0, 3)),
                      mass=np.zeros(0), com=np.zeros((0, 3)), inertia=np.zeros((0, 6)), task_link=np.zeros(0, np.int32))
    fb = with_floating_base(body, base_mass=7.0, base_inertia=(0.3, 0.4, 0.5, 0.0, 0.0, 0.0))
    fb.task_link = np.array([5], np.int32)
    M, h, _, _ = oracle.rbd_batch(fb, np.zeros((1, 6)), np.zeros((1, 6)))
    np.testing.assert_allclose(M[0][:3, :3], 7.0 * np.eye(3), atol=1e-14)
    np.testing.assert_allclose(np.diag(M[0])[3:], [0.5, 0.4, 0.3], atol=1e-14)  # z, y, x rotations
    np.testing.assert_allclose(h[0], [0, 0, 7.0 * 9.81, 0, 0, 0], atol=1e-12)
