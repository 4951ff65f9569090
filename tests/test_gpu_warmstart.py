"""GPU: the per-instance warm start of the dual active set (the qpOASES hot-start analogue,
SURVEY.md 8b ownership row; qppvm_amd/csrc/dual_gi.h warm_start). A context keeps every
instance's final active set and the next solve batch-adds it (kept only when dual feasible). It
changes the path, never the solution: under the config-2 churn (20 % of the instances re-drawn
between solves) the warm results equal a cold context's to 1e-9, statuses equal, and the
unchanged instances take fewer active-set steps."""
import numpy as np
import pytest

from conftest import rel_err
from qppvm_amd.problem import ContactProblem, QPPVMProblem
from qppvm_amd.synth import contact_instances, qppvm_instances

pytestmark = pytest.mark.gpu
MASKS = [0b0011, 0b0111, 0b1111]


@pytest.fixture(scope="module")
def wbq_mod():
    from qppvm_amd import build, wbq
    build.build()
    return wbq


def churn(inp, alt, frac, seed):
    rng = np.random.default_rng(seed)
    B = inp["h"].shape[0]
    pick = rng.choice(B, int(frac * B), replace=False)
    out = {k: v.copy() for k, v in inp.items()}
    for k in out:
        out[k][pick] = alt[k][pick]
    return out, pick


def run_churn(wbq_mod, Solver, prob, inp, alt, calls=4):
    warm = Solver(prob, max_batch=inp["h"].shape[0])
    try:
        cur = inp
        warm.solve_batch(cur)
        results = []
        for c in range(calls):
            cur, pick = churn(cur, alt if c % 2 == 0 else inp, 0.2, 100 + c)
            tw, sw, iw = warm.solve_batch(cur)
            cold = Solver(prob, max_batch=inp["h"].shape[0])
            try:
                tc, sc, ic = cold.solve_batch(cur)
            finally:
                cold.close()
            results.append((tw, sw, iw, tc, sc, ic, pick))
        return results
    finally:
        warm.close()


@pytest.mark.parametrize("torque_rows,nc,wd,mu", [(False, 4, 3, 0.0), (True, 4, 3, 0.0),
                                                   (False, 2, 6, 0.0), (False, 4, 6, 0.0),
                                                   (False, 2, 3, 0.4), (False, 4, 3, 0.4),
                                                   (False, 2, 6, 0.4), (True, 2, 6, 0.5), (True, 4, 3, 0.4)])
def test_contact_warm_equals_cold(wbq_mod, torque_rows, nc, wd, mu):
    """Every contact-form variant the shapes select (register slots, LDS slots with one-sided friction
    faces, 6-D wrench boxes, torque rows): dual_gi.h warm_extend over repeated solves on one context
    gives the cold answer."""
    free = ContactProblem(n=30, nc=nc, wrench_dim=wd, mu=mu)
    masks = MASKS if nc == 4 else None
    inp = contact_instances(free, 512, seed=1, masks=masks)
    alt = contact_instances(free, 512, seed=2, masks=masks)
    prob = free
    if torque_rows:
        s = wbq_mod.ContactSolver(free, max_batch=512)
        tf, _, _ = s.solve_batch(inp)
        s.close()
        prob = ContactProblem(n=30, nc=nc, wrench_dim=wd, mu=mu, torque_rows=True,
                              tau_max=float(np.quantile(np.abs(tf[:, 6:]), 0.85)))
    saved = 0
    for tw, sw, iw, tc, sc, ic, pick in run_churn(wbq_mod, wbq_mod.ContactSolver, prob, inp, alt):
        np.testing.assert_array_equal(sw, sc)
        ok = sw == 0
        assert rel_err(tw[ok], tc[ok]) <= 1e-9, rel_err(tw[ok], tc[ok])
        same = np.ones(len(sw), bool)
        same[pick] = False
        saved += int(ic[same & ok].sum() - iw[same & ok].sum())
    assert saved > 0  # the unchanged instances skip steps


def test_w1m_warm_equals_cold(wbq_mod):
    base = QPPVMProblem(n=30, joint_weight=1)
    inp = qppvm_instances(base, 512, seed=3)
    alt = qppvm_instances(base, 512, seed=4)
    s = wbq_mod.QPPVMSolver(QPPVMProblem(n=30, tau_max=1e9, joint_weight=1), max_batch=512)
    tf, _, _ = s.solve_batch(inp)
    s.close()
    prob = QPPVMProblem(n=30, tau_max=float(np.quantile(np.abs(tf), 0.8)), joint_weight=1)
    saved = 0
    for tw, sw, iw, tc, sc, ic, pick in run_churn(wbq_mod, wbq_mod.QPPVMSolver, prob, inp, alt):
        np.testing.assert_array_equal(sw, sc)
        ok = sw == 0
        assert rel_err(tw[ok], tc[ok]) <= 1e-9, rel_err(tw[ok], tc[ok])
        same = np.ones(len(sw), bool)
        same[pick] = False
        saved += int(ic[same & ok].sum() - iw[same & ok].sum())
    assert saved > 0


@pytest.mark.parametrize("n", [30, 39])
def test_w1i_warm_equals_cold(wbq_mod, oracle_lib, n):
    """W1 = I (the reference's stack): the bound active set of the last solve is added first
    (qppvm_kernel.hip gi_solve); n = 30 runs it inline in the fast kernel, n = 39 in the active-set
    kernel. Warm == cold to 1e-9, and == the oracle."""
    base = QPPVMProblem(n=n)
    inp = qppvm_instances(base, 512, seed=5)
    alt = qppvm_instances(base, 512, seed=6)
    s = wbq_mod.QPPVMSolver(QPPVMProblem(n=n, tau_max=1e9), max_batch=512)
    tf, _, _ = s.solve_batch(inp)
    s.close()
    prob = QPPVMProblem(n=n, tau_max=float(np.quantile(np.abs(tf), 0.8)))
    saved = 0
    for k, (tw, sw, iw, tc, sc, ic, pick) in enumerate(run_churn(wbq_mod, wbq_mod.QPPVMSolver, prob, inp, alt)):
        np.testing.assert_array_equal(sw, sc)
        ok = sw == 0
        assert rel_err(tw[ok], tc[ok]) <= 1e-9, rel_err(tw[ok], tc[ok])
        same = np.ones(len(sw), bool)
        same[pick] = False
        saved += int(ic[same & ok].sum() - iw[same & ok].sum())
    assert saved > 0
