"""GPU, full BASELINE sizes: every output of a config-2 batch (B = 4096) carries
the KAT-4 optimality certificate (tests/kkt.py): level-0 optimality, level-1 stationarity,
multiplier signs and primal feasibility, scaled residuals <= 1e-9. This needs no reference
solution, so it covers the sizes the oracle comparison (test_gpu_parity) samples."""
import numpy as np
import pytest

import kkt
from qppvm_amd.problem import ContactProblem, QPPVMProblem, WEIGHT_IDENTITY, WEIGHT_INERTIA
from qppvm_amd.synth import contact_instances, qppvm_instances

pytestmark = pytest.mark.gpu
TOL = 1e-9


@pytest.fixture(scope="module")
def wbq_mod():
    from qppvm_amd import build, wbq
    build.build()
    return wbq


def gpu(wbq_mod, prob, inp):
    s = wbq_mod.QPPVMSolver(prob, max_batch=inp["h"].shape[0])
    try:
        return s.solve_batch(inp)
    finally:
        s.close()


@pytest.mark.parametrize("n,B,weight", [(30, 4096, WEIGHT_IDENTITY), (30, 4096, WEIGHT_INERTIA),
                                        (39, 1024, WEIGHT_IDENTITY)])
def test_qppvm_config2_certificates(wbq_mod, oracle_lib, n, B, weight):
    inp = qppvm_instances(QPPVMProblem(n=n), B, seed=1)
    t0, _, _ = gpu(wbq_mod, QPPVMProblem(n=n, tau_max=1e9, joint_weight=weight), inp)
    prob = QPPVMProblem(n=n, tau_max=float(np.quantile(np.abs(t0), 0.8)), joint_weight=weight)
    tau, st, it = gpu(wbq_mod, prob, inp)
    assert (st == 0).all(), np.bincount(st.clip(0))
    assert (it > 0).mean() > 0.5  # the active set really ran on most instances
    cs = [kkt.qppvm_certificate(oracle_lib, prob, inp, b, tau[b]) for b in range(B)]
    w = {k: max(c[k] for c in cs) for k in ("primal", "level0", "stat", "sign")}
    assert max(w.values()) <= TOL, w
    assert sum(c["indep"] for c in cs) >= 0.9 * B  # signs checked on (almost) every instance


def test_contact_config2_certificates(wbq_mod, oracle_lib):
    n, B = 30, 4096
    masks = [0b0011, 0b0111, 0b1111]
    inp = contact_instances(ContactProblem(n=n, nc=4), B, seed=1, masks=masks)
    s = wbq_mod.ContactSolver(ContactProblem(n=n, nc=4), max_batch=B)
    t0, _, _ = s.solve_batch(inp)
    s.close()
    prob = ContactProblem(n=n, nc=4, torque_rows=True, tau_max=float(np.quantile(np.abs(t0[:, 6:]), 0.85)))
    s = wbq_mod.ContactSolver(prob, max_batch=B)
    tau, st, _ = s.solve_batch(inp)
    x = s.x()
    s.close()
    assert (st == 0).all(), np.bincount(st.clip(0))
    cs = [kkt.contact_certificate(oracle_lib, prob, inp, b, x[b]) for b in range(B)]
    w = {k: max(c[k] for c in cs) for k in ("primal", "stat", "sign", "comp")}
    assert max(w.values()) <= TOL, w
