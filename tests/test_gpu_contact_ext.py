"""GPU parity of the SURVEY.md 8f-2 contact-form extensions: full 6-D wrenches ("put 6 for full
wrench", reference src/ForceAcc.cpp:67; moment box +-1, :74-76) and the linearised friction
pyramid |f_x| <= mu f_z, |f_y| <= mu f_z (4 rows per active contact). The HIP kernel through the C
ABI against the oracle (oracle/wbq_oracle_contact.c) and the KKT-certified fixture
tests/golden/contact_ext_n30.npz. Tolerance as tests/test_gpu_contact.py: tau within 1e-6 relative
per instance, statuses equal."""
import numpy as np
import pytest

from conftest import load_golden_contact, rel_err
from qppvm_amd.problem import ContactProblem
from qppvm_amd.synth import contact_instances, replicate
from test_gpu_contact import MASKS4, TOL, check_against_oracle, gpu_solve

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def wbq_mod():
    from qppvm_amd import build, wbq
    build.build()
    return wbq


def test_contact_ext_golden(wbq_mod):
    for g, prob, inp, exp in load_golden_contact(30, "contact_ext_n30.npz"):
        tau, x, st, _ = gpu_solve(wbq_mod, prob, inp)
        assert np.all(st == 0), (g, st)
        assert rel_err(tau, exp["tau"]) <= TOL, (g, rel_err(tau, exp["tau"]))
        assert rel_err(x, exp["x"]) <= 1e-5, (g, rel_err(x, exp["x"]))


# (nc, wrench_dim, mu, torque rows): every kernel variant the shapes select (contact_kernel.hip
# launch_wd: register slots 18 / 24, LDS slots for friction rows and four full wrenches, torque rows)
CASES = [
    (2, 6, 0.0, False), (4, 6, 0.0, False), (2, 3, 0.3, False), (4, 3, 0.3, False),
    (2, 6, 0.3, False), (4, 6, 0.5, False), (2, 6, 0.0, True), (2, 3, 0.3, True), (4, 3, 0.5, True),
]


@pytest.mark.parametrize("nc,wd,mu,tr", CASES)
def test_contact_ext_random(wbq_mod, oracle_lib, nc, wd, mu, tr):
    kw = dict(torque_rows=True, tau_max=60.0) if tr else {}
    prob = ContactProblem(n=30, nc=nc, wrench_dim=wd, mu=mu, **kw)
    masks = MASKS4 if nc == 4 else None
    inp = contact_instances(prob, 48, seed=40 + nc + wd + int(10 * mu) + int(tr), masks=masks)
    tau, x, st, _ = check_against_oracle(wbq_mod, oracle_lib, prob, inp, min_ok=40)
    n = prob.n
    w = x[:, n:].reshape(-1, nc, wd)
    act = ((inp["cmask"][:, None] >> np.arange(nc)[None]) & 1).astype(bool)
    ok = st == 0
    sel = act & ok[:, None]
    assert np.all(w[sel][:, 2] >= 10.0 - 1e-8)
    if wd == 6:
        assert np.all(np.abs(w[sel][:, 3:]) <= 1.0 + 1e-9)
    if mu > 0:
        f = w[sel]
        assert np.all(np.abs(f[:, :2]) <= mu * f[:, 2:3] + 1e-8)
    assert np.all(w[~act & ok[:, None]] == 0.0)


def test_contact_ext_n39(wbq_mod, oracle_lib):
    """CENTAURO-sized (n = 39, one instance per 64 lanes) with two full wrenches and the cone."""
    prob = ContactProblem(n=39, nc=2, wrench_dim=6, mu=0.4)
    inp = contact_instances(prob, 32, seed=77)
    check_against_oracle(wbq_mod, oracle_lib, prob, inp, min_ok=28)


def test_contact_ext_config1_identical(wbq_mod, oracle_lib):
    """Double support with full wrenches and the cone, identical instances (config 1 shape)."""
    prob = ContactProblem(n=30, nc=2, wrench_dim=6, mu=0.3)
    inp = replicate(contact_instances(prob, 1, seed=0), 64)
    tau, x, st, _ = check_against_oracle(wbq_mod, oracle_lib, prob, inp, min_ok=64)
    assert np.abs(tau - tau[0]).max() == 0.0
