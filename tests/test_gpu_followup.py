"""The on-demand follow-up (include/wbq.h WBQ_OPT_FOLLOWUP): while the last solves of a context listed no
level-0 repair, a QPPVM W1 = I solve with n <= 32 enqueues its fast kernel alone, and a solve that does list
one is completed (qppvm_repair_kernel over its list) by the next call that reads outputs. The outputs must
equal the always-enqueued follow-up's, bit for bit, in every order of calls; against the oracle as
tests/test_gpu_parity.py (tau within 1e-6 relative, statuses equal)."""
import numpy as np
import pytest

from conftest import rel_err
from qppvm_amd.problem import QPPVMProblem
from qppvm_amd.synth import qppvm_instances

pytestmark = pytest.mark.gpu
TOL = 1e-6


@pytest.fixture(scope="module")
def wbq_mod():
    from qppvm_amd import build, wbq
    build.build()
    return wbq


def cases(oracle_lib):
    """(problem, repair-free batch, repair-heavy batch): the same problem with loose and tight limits."""
    n = 30
    tight = QPPVMProblem(n=n, tau_max=30.0)  # level 0 not attainable for most instances
    heavy = qppvm_instances(tight, 64, seed=331)
    loose = QPPVMProblem(n=n, tau_max=1e6)
    free = qppvm_instances(loose, 64, seed=332)
    return tight, loose, free, heavy


def test_followup_modes_agree(wbq_mod, oracle_lib):
    tight, _, _, heavy = cases(oracle_lib)
    tau_r, st_r, _ = oracle_lib.qppvm_batch(tight, heavy)
    outs = []
    for mode in (0, 1):
        s = wbq_mod.QPPVMSolver(tight, max_batch=64)
        try:
            s.set_option(s.OPT_FOLLOWUP, mode)
            outs.append(s.solve_batch(heavy))
        finally:
            s.close()
    (t0, s0, i0), (t1, s1, i1) = outs
    np.testing.assert_array_equal(s0, s1)
    np.testing.assert_array_equal(t0, t1)
    np.testing.assert_array_equal(s1, st_r)
    ok = st_r == 0
    assert (s1 != 0).sum() <= 2 and rel_err(t1[ok], tau_r[ok]) <= TOL


def test_followup_deferred_completion(wbq_mod, oracle_lib):
    """A context whose solves needed no repair enqueues the fast kernel alone; a batch that then needs the
    repair is finished when its outputs are read (and by wbq_sync), never returned half done; a solve
    superseded before its outputs were read is simply replaced by the next one's."""
    tight, _, free_l, heavy = cases(oracle_lib)
    # the loose batch under the tight problem's limits would need repairs too: use it under a wide box
    wide = QPPVMProblem(n=30, tau_max=1e6)
    tau_w, st_w, _ = oracle_lib.qppvm_batch(wide, free_l)
    assert (st_w == 0).all()
    s = wbq_mod.QPPVMSolver(wide, max_batch=64)
    try:
        s.set_option(s.OPT_FOLLOWUP, 1)
        for _ in range(4):  # repair-free solves: the follow-up kernel is skipped from here on
            tau, st, _ = s.solve_batch(free_l)
        assert (st == 0).all() and rel_err(tau, tau_w) <= TOL
    finally:
        s.close()
    tau_r, st_r, _ = oracle_lib.qppvm_batch(tight, heavy)
    s = wbq_mod.QPPVMSolver(tight, max_batch=64)
    try:
        s.set_option(s.OPT_FOLLOWUP, 1)
        # a fresh context starts in the on-demand mode: the first solve lists repairs it does not run
        s.set_inputs(heavy)
        s.solve()
        s.sync()  # completes it
        tau, st, _ = s.outputs()
        np.testing.assert_array_equal(st, st_r)
        ok = st_r == 0
        assert rel_err(tau[ok], tau_r[ok]) <= TOL
    finally:
        s.close()


def test_followup_superseded_pending_solve(wbq_mod, oracle_lib):
    """A fresh context starts in the on-demand mode: two solves of the repair-heavy batch without a read in
    between leave the first pending and let the second supersede it (its listing flag, the stale counters
    the second solve's fast kernel clears); the outputs read once at the end equal OPT_FOLLOWUP = 0 bit for
    bit, and a third solve after the read (now with the follow-up enqueued) agrees too."""
    tight, _, _, heavy = cases(oracle_lib)
    tau_r, st_r, _ = oracle_lib.qppvm_batch(tight, heavy)
    ref = wbq_mod.QPPVMSolver(tight, max_batch=64)
    try:
        ref.set_option(ref.OPT_FOLLOWUP, 0)
        t0, s0, i0 = ref.solve_batch(heavy)
    finally:
        ref.close()
    s = wbq_mod.QPPVMSolver(tight, max_batch=64)
    try:
        s.set_option(s.OPT_FOLLOWUP, 1)
        s.set_inputs(heavy)
        s.solve()
        s.solve()
        t1, s1, i1 = s.outputs()
        s.solve()
        t2, s2, i2 = s.outputs()
    finally:
        s.close()
    np.testing.assert_array_equal(s1, s0)
    np.testing.assert_array_equal(t1, t0)
    np.testing.assert_array_equal(s1, st_r)
    ok = st_r == 0
    assert rel_err(t1[ok], tau_r[ok]) <= TOL
    # (the third solve starts warm from the second: the path may change, the solution may not)
    np.testing.assert_array_equal(s2, st_r)
    assert rel_err(t2[ok], tau_r[ok]) <= TOL


def test_followup_device_inputs_refilled_after_solve(wbq_mod, oracle_lib):
    """WBQ_MEM_DEVICE inputs live in the caller's buffers: a solve's repair must read them in stream order,
    so a refill the caller enqueues on the stream after wbq_solve and before reading the outputs must not
    reach the solve (with device inputs every solve enqueues its follow-up kernel)."""
    torch = pytest.importorskip("torch")
    tight, _, _, heavy = cases(oracle_lib)
    tau_r, st_r, _ = oracle_lib.qppvm_batch(tight, heavy)
    other = qppvm_instances(tight, 64, seed=333)
    live = {k: torch.from_numpy(np.ascontiguousarray(v)).to("cuda:0") for k, v in heavy.items()}
    alt = {k: torch.from_numpy(np.ascontiguousarray(v)).to("cuda:0") for k, v in other.items()}
    s = wbq_mod.QPPVMSolver(tight, max_batch=64)
    try:
        s.set_option(s.OPT_FOLLOWUP, 1)
        s.set_stream(torch.cuda.current_stream().cuda_stream)
        s.set_device_inputs({k: v.data_ptr() for k, v in live.items()}, 64)
        s.solve()
        for k in live:  # the caller refills its buffers on the same stream
            live[k].copy_(alt[k])
        t1, s1, _ = s.outputs()
    finally:
        s.close()
    np.testing.assert_array_equal(s1, st_r)
    ok = st_r == 0
    assert rel_err(t1[ok], tau_r[ok]) <= TOL
