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


@pytest.mark.parametrize("mu", [0.3, 0.5])
def test_contact_level0_repair_friction(wbq_mod, oracle_lib, mu):
    """Level 0 not attainable with the friction pyramid on (the reference's stack
    waist / (postural + feet), ForceAcc.cpp:131-137, keeps the waist at its level-0 optimum under
    every constraint and returns false only when infeasible, :189-193): the GPU solves level 0 over the
    box AND the pyramid faces (fric_lsi.h, an LSI in the BVLS pattern) as the oracle's level-0 QP does
    (oracle/wbq_oracle_contact.c:413-447), and level 1 holds the faces and box sides its multipliers
    pin. The test_contact_level0_repair sweep (n = 12, nc = 4, torque rows at the 40 % quantile, 20
    seeds, 1,280 instances) with the cone on: every instance the oracle solves, the GPU solves with the
    oracle's tau (no miss allowed). Near a degenerate vertex the constraint-space dual loop cannot tell
    a dependent row from an independent one (its Schur complements in Gamma carry the 1 / eps_f force
    scale's roundoff); there the repair kernel finishes level 1 with the QR-form loop
    (qppvm_amd/csrc/qr_gi.h: an explicit H^-1-orthonormal basis of the active normals, numpy
    statement scripts/qr_gi.py). Where the oracle fails, a GPU solution carries the level-1 KKT
    certificate (1e-9) and the level-0 LSI certificate at 1e-8: those are the degenerate instances
    (the oracle's own dual loop ends numerically there), where the final point's waist value carries
    the level-0 step's roundoff (observed 2e-9)."""
    import kkt
    n, nc = 12, 4
    tot = dict(solved=0, repaired=0, miss=0, extra=0, l0_worst=0.0)
    for seed in range(100, 120):
        free = ContactProblem(n=n, nc=nc, mu=mu)
        inp = contact_instances(free, 64, seed=seed, masks=MASKS4)
        tau_free = oracle_lib.contact_batch(free, inp)[0]
        prob = ContactProblem(n=n, nc=nc, mu=mu, torque_rows=True,
                              tau_max=float(np.quantile(np.abs(tau_free[:, 6:]), 0.4)))
        tau_r, x_r, st_r, _, rep = oracle_lib.contact_batch(prob, inp)
        tau, x, st, it = gpu_solve(wbq_mod, prob, inp)
        solved = st_r == 0
        tot["solved"] += int(solved.sum())
        tot["repaired"] += int((solved & (rep != 0)).sum())
        ok = solved & (st == 0)
        assert rel_err(tau[ok], tau_r[ok]) <= TOL, (seed, rel_err(tau[ok], tau_r[ok]))
        tot["miss"] += int((solved & (st != 0)).sum())
        np.testing.assert_array_equal(tau[st != 0], inp["h"][st != 0])
        w = x[:, n:].reshape(-1, nc, 3)
        act = ((inp["cmask"][:, None] >> np.arange(nc)[None]) & 1).astype(bool) & (st == 0)[:, None]
        assert np.all(np.abs(w[act][:, :2]) <= mu * w[act][:, 2:3] + 1e-8)
        for b in np.where(~solved & (st == 0))[0]:
            tot["extra"] += 1
            l0, y = kkt.contact_level0_certificate(oracle_lib, prob, inp, b, x[b])
            c = kkt.contact_certificate(oracle_lib, prob, inp, b, x[b], waist=y)
            tot["l0_worst"] = max(tot["l0_worst"], l0)
            # complementarity: 1e-9, or 1e-8 where the candidate normals are dependent (indep False: the
            # multipliers are not unique and the fit's own choice among them spreads weight onto rows a
            # few 1e-9 off their bound; primal, stationarity and signs stay at 1e-9)
            comp_tol = 1e-9 if c["indep"] else 1e-8
            assert l0 <= 1e-8 and max(c["primal"], c["stat"], c["sign"]) <= 1e-9 and c["comp"] <= comp_tol, \
                (seed, b, l0, c)
    print("friction level-0 repair sweep:", tot)
    assert tot["repaired"] >= 500, tot  # the friction-aware repair path really runs
    assert tot["miss"] == 0, tot
