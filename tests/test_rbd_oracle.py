"""CPU checks of the rigid-body-dynamics oracle (oracle/wbq_oracle_rbd.c, the checker of
qppvm_amd/csrc/rbd.hip): closed forms of a pendulum and a planar two-link arm (KAT), and on the
n = 39 CENTAURO-like tree the properties every correct model satisfies -- M symmetric positive
definite, RNEA(q, qd, qdd) = M qdd + h (CRBA vs RNEA), J = d pose / dq (finite differences),
h(q, 0) = dU/dq (finite differences of the potential energy)."""
import numpy as np
import pytest

import oracle
from qppvm_amd.rbd import RobotModel, centauro_like, serial_chain


def pendulum(m=2.0, l=0.7, I0=0.05):
    return RobotModel(parent=np.array([-1], np.int32), X_fixed=np.array([[1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0.]]),
                      axis=np.array([[1.0, 0, 0]]), mass=np.array([m]), com=np.array([[0, 0, -l]]),
                      inertia=np.array([[I0, 0.01, 0.01, 0, 0, 0]]), task_link=np.array([0], np.int32))


def two_link(m1=3.0, m2=2.0, l1=0.6, lc1=0.3, lc2=0.25, I1=0.04, I2=0.03):
    X = np.array([[1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0.], [1, 0, 0, l1, 0, 1, 0, 0, 0, 0, 1, 0.]])
    return RobotModel(parent=np.array([-1, 0], np.int32), X_fixed=X, axis=np.array([[0, 0, 1.0], [0, 0, 1.0]]),
                      mass=np.array([m1, m2]), com=np.array([[lc1, 0, 0], [lc2, 0, 0]]),
                      inertia=np.array([[0.01, 0.01, I1, 0, 0, 0], [0.01, 0.01, I2, 0, 0, 0]]),
                      task_link=np.array([1], np.int32), gravity=(0.0, -9.81, 0.0))


def two_link_closed_form(q, qd, m1=3.0, m2=2.0, l1=0.6, lc1=0.3, lc2=0.25, I1=0.04, I2=0.03, g=9.81):
    c2, s2 = np.cos(q[1]), np.sin(q[1])
    M = np.array([[m1 * lc1 ** 2 + I1 + m2 * (l1 ** 2 + lc2 ** 2 + 2 * l1 * lc2 * c2) + I2,
                   m2 * (lc2 ** 2 + l1 * lc2 * c2) + I2],
                  [m2 * (lc2 ** 2 + l1 * lc2 * c2) + I2, m2 * lc2 ** 2 + I2]])
    hh = m2 * l1 * lc2 * s2
    grav = np.array([(m1 * lc1 + m2 * l1) * g * np.cos(q[0]) + m2 * lc2 * g * np.cos(q[0] + q[1]),
                     m2 * lc2 * g * np.cos(q[0] + q[1])])
    h = np.array([-hh * (2 * qd[0] * qd[1] + qd[1] ** 2), hh * qd[0] ** 2]) + grav
    return M, h


def test_pendulum_closed_form():
    m, l, I0 = 2.0, 0.7, 0.05
    for q in (0.0, 0.4, -1.3, 2.9):
        M, h, J, pose = oracle.rbd_batch(pendulum(m, l, I0), [q], [0.8])
        np.testing.assert_allclose(M[0], [[I0 + m * l * l]], rtol=1e-14)
        np.testing.assert_allclose(h[0], [m * 9.81 * l * np.sin(q)], rtol=1e-13, atol=1e-13)
        np.testing.assert_allclose(J[0, 0, :, 0], [0, 0, 0, 1, 0, 0], atol=1e-15)  # link origin on the axis


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_two_link_closed_form(seed):
    rng = np.random.default_rng(seed)
    q, qd = rng.uniform(-np.pi, np.pi, 2), rng.normal(0, 2, 2)
    M, h, J, pose = oracle.rbd_batch(two_link(), q, qd)
    Mc, hc = two_link_closed_form(q, qd)
    np.testing.assert_allclose(M[0], Mc, rtol=1e-13, atol=1e-13)
    np.testing.assert_allclose(h[0], hc, rtol=1e-12, atol=1e-12)
    # the task link (link 1) origin sits at l1 (cos q1, sin q1)
    np.testing.assert_allclose(pose[0, 0, [3, 7]], [0.6 * np.cos(q[0]), 0.6 * np.sin(q[0])], atol=1e-15)


def _fk_pose(model, q):
    _, _, _, pose = oracle.rbd_batch(model, q, np.zeros_like(q))
    return pose[0]


@pytest.mark.parametrize("maker", [centauro_like, serial_chain])
def test_tree_properties(maker):
    model = maker()
    n = model.n
    rng = np.random.default_rng(5)
    q, qd, qdd = rng.uniform(-np.pi, np.pi, n), rng.normal(0, 1, n), rng.normal(0, 1, n)
    M, h, J, pose = oracle.rbd_batch(model, q, qd)
    M, h, J, pose = M[0], h[0], J[0], pose[0]
    np.testing.assert_allclose(M, M.T, rtol=0, atol=1e-12 * np.abs(M).max())
    assert np.linalg.eigvalsh(M).min() > 0
    # RNEA with qdd = M qdd + h (CRBA and RNEA are separate recursions)
    np.testing.assert_allclose(oracle.rnea(model, q, qd, qdd), M @ qdd + h, rtol=1e-11, atol=1e-10)
    # Jacobian = d(pose)/dq by central differences: linear rows from p, angular rows from R
    eps = 1e-6
    for j in range(n):
        dq = np.zeros(n); dq[j] = eps
        Pp, Pm = _fk_pose(model, q + dq), _fk_pose(model, q - dq)
        for t in range(model.ntasks):
            Rp, Rm = Pp[t].reshape(3, 4)[:, :3], Pm[t].reshape(3, 4)[:, :3]
            R = pose[t].reshape(3, 4)[:, :3]
            lin = (Pp[t].reshape(3, 4)[:, 3] - Pm[t].reshape(3, 4)[:, 3]) / (2 * eps)
            W = (Rp - Rm) / (2 * eps) @ R.T  # skew(omega)
            ang = np.array([W[2, 1], W[0, 2], W[1, 0]])
            np.testing.assert_allclose(J[t, :3, j], lin, atol=1e-8)
            np.testing.assert_allclose(J[t, 3:, j], ang, atol=1e-8)
    # gravity torques = dU/dq, U = -sum_i m_i g . c_i(q)
    def U(qq):
        tot = 0.0
        for i in range(n):  # world COM of link i through a one-link task on it
            mi = RobotModel(parent=model.parent, X_fixed=model.X_fixed, axis=model.axis, mass=model.mass,
                            com=model.com, inertia=model.inertia, task_link=np.array([i], np.int32))
            P = _fk_pose(mi, qq)[0].reshape(3, 4)
            c = P[:, :3] @ model.com[i] + P[:, 3]
            tot -= model.mass[i] * np.dot(model.gravity, c)
        return tot
    _, g0, _, _ = oracle.rbd_batch(model, q, np.zeros(n))
    for j in rng.choice(n, 4, replace=False):
        dq = np.zeros(n); dq[j] = 1e-6
        np.testing.assert_allclose(g0[0, j], (U(q + dq) - U(q - dq)) / 2e-6, rtol=1e-6, atol=1e-6)
