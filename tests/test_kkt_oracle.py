"""The KAT-4 optimality certificates (tests/kkt.py) themselves, on CPU: the oracle's solutions
pass them; perturbed solutions and the solution of the other joint weight fail them."""
import numpy as np
import pytest

import kkt
from qppvm_amd.problem import ContactProblem, QPPVMProblem, WEIGHT_IDENTITY, WEIGHT_INERTIA
from qppvm_amd.synth import contact_instances, qppvm_instances

TOL = 1e-9


def worst(cs, keys):
    return {k: max(c[k] for c in cs) for k in keys}


@pytest.mark.parametrize("weight", [WEIGHT_IDENTITY, WEIGHT_INERTIA])
def test_qppvm_certificate_accepts_oracle_and_rejects_others(oracle_lib, weight):
    free = QPPVMProblem(n=30, tau_max=1e9, joint_weight=weight)
    inp = qppvm_instances(free, 24, seed=11)
    t0, _, _ = oracle_lib.qppvm_batch(free, inp)
    prob = QPPVMProblem(n=30, tau_max=float(np.quantile(np.abs(t0), 0.8)), joint_weight=weight)
    tau, st, _ = oracle_lib.qppvm_batch(prob, inp)
    assert (st == 0).all()
    ok = worst([kkt.qppvm_certificate(oracle_lib, prob, inp, b, tau[b]) for b in range(24)],
               ("primal", "level0", "stat", "sign"))
    assert max(ok.values()) <= TOL, ok
    bad = [kkt.qppvm_certificate(oracle_lib, prob, inp, b, tau[b] * (1 + 1e-6)) for b in range(8)]
    assert all(max(c["primal"], c["level0"], c["stat"]) > 1e-8 for c in bad)
    other = QPPVMProblem(n=30, tau_max=prob.tau_max, joint_weight=1 - weight)
    tau_o, st_o, _ = oracle_lib.qppvm_batch(other, inp)
    wrong = [kkt.qppvm_certificate(oracle_lib, prob, inp, b, tau_o[b]) for b in range(24) if st_o[b] == 0]
    assert sum(c["stat"] > 1e-6 for c in wrong) >= len(wrong) // 2


def test_contact_certificate_accepts_oracle_and_rejects_perturbed(oracle_lib):
    prob = ContactProblem(n=30, nc=4)
    inp = contact_instances(prob, 16, seed=12, masks=[0b0011, 0b0111, 0b1111])
    _, x, st, _, _ = oracle_lib.contact_batch(prob, inp)
    ok = worst([kkt.contact_certificate(oracle_lib, prob, inp, b, x[b]) for b in range(16) if st[b] == 0],
               ("primal", "stat", "sign", "comp"))
    assert max(ok.values()) <= TOL, ok
    bad = [kkt.contact_certificate(oracle_lib, prob, inp, b, x[b] * (1 + 1e-6)) for b in range(8)]
    assert all(max(c["primal"], c["stat"]) > 1e-9 for c in bad)


@pytest.mark.parametrize("mu", [0.3, 0.5])
def test_friction_lsi_certificate_and_reference(oracle_lib, mu):
    """The level-0 LSI over the box and the friction pyramid (kernel: qppvm_amd/csrc/fric_lsi.h) as
    its numpy statement (tests/fric_lsi_ref.py) solves it: the certificate (kkt.lsi_certificate)
    accepts those points and rejects perturbed ones, and the waist value y0* agrees with the
    oracle's level-0 QP (a 1e-10 ridge, oracle/wbq_oracle_contact.c) to 1e-6 relative."""
    import fric_lsi_ref as ref
    n, nc = 12, 4
    free = ContactProblem(n=n, nc=nc, mu=mu)
    inp = contact_instances(free, 64, seed=101, masks=ref.MASKS4)
    tf = oracle_lib.contact_batch(free, inp)[0]
    prob = ContactProblem(n=n, nc=nc, mu=mu, torque_rows=True, tau_max=float(np.quantile(np.abs(tf[:, 6:]), 0.4)))
    _, x_r, st_r, _, rep = oracle_lib.contact_batch(prob, inp)
    cases = np.where((st_r == 0) & (rep != 0))[0][:12]
    assert len(cases) >= 8
    faces_held = 0
    for b in cases:
        A, bb, lo, hi, groups, wth = ref.zspace(prob, inp, b)
        z, st, fm, it, capped, pins = ref.lsi_level0(A, bb, lo, hi, groups, mu)
        assert not capped
        faces_held += sum(bin(m).count("1") for m in fm.values())
        assert kkt.lsi_certificate(A, bb, z, lo, hi, groups, mu) <= TOL
        zp = z.copy()
        zp[groups[0] + 2] *= 1.0 + 1e-4  # one contact's normal force off its optimum
        assert kkt.lsi_certificate(A, bb, zp, lo, hi, groups, mu) > TOL
        y = A @ z - wth
        yr = inp["Jw"][b] @ x_r[b, :n]
        assert np.abs(y - yr).max() <= 1e-6 * max(1.0, np.abs(yr).max()), (b, np.abs(y - yr).max())
    assert faces_held > 0  # the pyramid really binds in this sweep


@pytest.mark.parametrize("n,q", [(14, 0.6), (20, 0.3), (30, 0.5)])
def test_three_level_certificate_accepts_oracle(oracle_lib, n, q):
    """The elbow level (task_level (0, 0, 1, 1): ((ee_r + ee_l) / (elbow_l + elbow_r)) / joint,
    QPPVMPlugin.cpp:154-166,177-178): the oracle's lexicographic chain (level-0 BVLS, the middle level
    by BVLS in the null space of the level-0 rows, oracle/wbq_oracle.c:wbq_ref_level_mid, the joint
    task last) carries the three-level certificate, and differs from the two-level stack that sums
    the four tasks where the limits bind; the two-level answer fails the three-level certificate."""
    rm = (7, 7, 7, 7)
    free = QPPVMProblem(n=n, ntasks=4, row_mask=rm, tau_max=1e9)
    inp = qppvm_instances(free, 32, seed=31 + n)
    t0, _, _ = oracle_lib.qppvm_batch(free, inp)
    tm = float(np.quantile(np.abs(t0), q))
    p3 = QPPVMProblem(n=n, ntasks=4, row_mask=rm, tau_max=tm, task_level=(0, 0, 1, 1))
    p2 = QPPVMProblem(n=n, ntasks=4, row_mask=rm, tau_max=tm)
    t3, s3, _ = oracle_lib.qppvm_batch(p3, inp)
    t2, s2, _ = oracle_lib.qppvm_batch(p2, inp)
    assert (s3 == 0).all() and (s2 == 0).all()
    cs = [kkt.qppvm_certificate(oracle_lib, p3, inp, b, t3[b]) for b in range(32)]
    ok = worst(cs, ("primal", "level0", "stat", "sign"))
    assert max(ok.values()) <= TOL, ok
    differ = np.abs(t3 - t2).max(axis=1) > 1e-6 * np.abs(t2).max(axis=1)
    if n < 30:
        assert differ.sum() >= 4
        bad = [kkt.qppvm_certificate(oracle_lib, p3, inp, b, t2[b])["level0"] for b in np.where(differ)[0]]
        assert max(bad) > 1e-6


def test_certificate_elbow_literal(oracle_lib):
    """The lexicographic certificate of the reference's commented elbow stack (no joint task: the last
    level's gradient is x itself, QPPVMPlugin.cpp:177-178): the oracle's outputs pass on every
    fixture group, and the three-level stack's torques (joint task kept) fail its stationarity where
    the two differ."""
    import kkt
    from conftest import load_golden_elbow
    fails = 0
    for g, prob, inp, exp in load_golden_elbow(True):
        tau, st, _ = oracle_lib.qppvm_batch(prob, inp)
        joint = QPPVMProblem(n=prob.n, ntasks=4, row_mask=(7, 7, 7, 7), task_level=(0, 0, 1, 1), tau_max=prob.tau_max)
        tj, _, _ = oracle_lib.qppvm_batch(joint, inp)
        for b in range(tau.shape[0]):
            c = kkt.qppvm_certificate(oracle_lib, prob, inp, b, tau[b])
            assert max(c["primal"], c["level0"], c["stat"], c["sign"]) <= 1e-9, (g, b, c)
            if np.abs(tj[b] - tau[b]).max() > 1e-6 * np.abs(tau[b]).max():
                cj = kkt.qppvm_certificate(oracle_lib, prob, inp, b, tj[b])
                fails += max(cj["stat"], cj["sign"]) > 1e-6
    assert fails >= 10
