"""ctypes loader for the CPU oracle (TEST INFRASTRUCTURE ONLY).

Only tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg may
import this package; the product path (``qppvm_amd``) never does.
Parity status: pinned to closed-form KATs + an independent numpy/scipy restatement
(tests/golden), not to reference binaries (unbuildable here).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
SRCS = [os.path.join(HERE, f) for f in ("wbq_oracle.c", "wbq_oracle_contact.c", "wbq_oracle_rbd.c")]


def build(force: bool = False) -> str:
    """Compile the C restatement with gcc (host only)."""
    deps = SRCS + [os.path.join(HERE, "wbq_oracle.h")]
    if force or not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < max(map(os.path.getmtime, deps)):
        subprocess.check_call(["gcc", "-O2", "-std=c99", "-fPIC", "-shared", "-Wall", "-Wextra",
                               "-Wno-unused-parameter", *SRCS, "-o", LIB_PATH + ".tmp", "-lm"])
        os.replace(LIB_PATH + ".tmp", LIB_PATH)
    return LIB_PATH


class _Desc(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int), ("ntasks", ctypes.c_int), ("row_mask", ctypes.c_int * 4),
                ("select_mode", ctypes.c_int), ("joint_weight", ctypes.c_int),
                ("Kc", ctypes.c_void_p), ("Dc", ctypes.c_void_p), ("Kq", ctypes.c_void_p),
                ("Dq", ctypes.c_void_p), ("tau_max", ctypes.c_void_p), ("tau_min", ctypes.c_void_p),
                ("joint_limits", ctypes.c_int), ("q_min", ctypes.c_void_p), ("q_max", ctypes.c_void_p),
                ("Kjl", ctypes.c_void_p), ("Djl", ctypes.c_void_p), ("task_level", ctypes.c_int * 4),
                ("no_joint_task", ctypes.c_int)]


class _Inst(ctypes.Structure):
    _fields_ = [(k, ctypes.c_void_p) for k in ("M", "J", "pose", "pose_ref", "q", "qd", "qref", "h")]


_lib = None


def lib():
    global _lib
    if _lib is None:
        _lib = ctypes.CDLL(build())
        P = ctypes.c_void_p
        _lib.wbq_ref_cart_error.argtypes = [P, P, P]
        _lib.wbq_ref_assemble.argtypes = [P, P, P, P, P, P, P, P]
        _lib.wbq_ref_assemble.restype = ctypes.c_int
        _lib.wbq_ref_level0.argtypes = [ctypes.c_int, ctypes.c_int, P, P, P, P, P, P, P]
        _lib.wbq_ref_level0.restype = ctypes.c_int
        _lib.wbq_ref_level1.argtypes = [ctypes.c_int, P, P, ctypes.c_int, P, P, P, P, P, P, P]
        _lib.wbq_ref_level1.restype = ctypes.c_int
        _lib.wbq_ref_level_mid.argtypes = [ctypes.c_int, P, ctypes.c_int, ctypes.c_int, P, P, P, P, P, P, P, P]
        _lib.wbq_ref_level_mid.restype = ctypes.c_int
        _lib.wbq_ref_qppvm_one.argtypes = [P, P, P, P, P]
        _lib.wbq_ref_qppvm_one.restype = ctypes.c_int
        _lib.wbq_ref_qppvm_batch.argtypes = [P, ctypes.c_int] + [P] * 8 + [P, P, P]
        I = ctypes.c_int
        _lib.wbq_ref_dual_qp.argtypes = [I, P, P, I, P, P, I, P, P, P, P, P]
        _lib.wbq_ref_dual_qp.restype = I
        _lib.wbq_ref_contact_assemble.argtypes = [P, P] + [P] * 8
        _lib.wbq_ref_contact_assemble.restype = I
        _lib.wbq_ref_contact_one.argtypes = [P, P, P, P, P, P]
        _lib.wbq_ref_contact_one.restype = I
        _lib.wbq_ref_contact_batch.argtypes = [P, I] + [P] * 14 + [P, P, P, P, P]
        _lib.wbq_ref_rbd_one.argtypes = [P] * 7
        _lib.wbq_ref_rbd_one.restype = None
        _lib.wbq_ref_rnea.argtypes = [P] * 5
        _lib.wbq_ref_task_jdqd.argtypes = [P, P, P, I, P]
        _lib.wbq_ref_task_jdqd.restype = None
        _lib.wbq_ref_rnea.restype = None
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _desc(prob):
    d = _Desc()
    d.n, d.ntasks = prob.n, prob.ntasks
    for t in range(4):
        d.row_mask[t] = prob.row_mask[t] if t < prob.ntasks else 0
    d.select_mode, d.joint_weight = prob.select_mode, prob.joint_weight
    for t, lv in enumerate(getattr(prob, "task_level", None) or ()):
        d.task_level[t] = int(lv)
    d.no_joint_task = 0 if getattr(prob, "joint_task", True) else 1
    keep = [np.ascontiguousarray(getattr(prob, k), dtype=np.float64)
            for k in ("Kc", "Dc", "Kq", "Dq", "tau_max", "tau_min")]
    d.Kc, d.Dc, d.Kq, d.Dq, d.tau_max, d.tau_min = [a.ctypes.data for a in keep]
    if getattr(prob, "joint_limits", False):
        jl = [np.ascontiguousarray(getattr(prob, k), dtype=np.float64) for k in ("q_min", "q_max", "Kjl", "Djl")]
        keep += jl
        d.joint_limits = 1
        d.q_min, d.q_max, d.Kjl, d.Djl = [a.ctypes.data for a in jl]
    return d, keep


def _c(a):
    return np.ascontiguousarray(a, dtype=np.float64)


def cart_error(pose, pose_ref):
    e = np.zeros(6)
    lib().wbq_ref_cart_error(_p(_c(pose)), _p(_c(pose_ref)), _p(e))
    return e


def _inst(inputs, b):
    arrs = {k: _c(inputs[k][b]) for k in ("M", "J", "pose", "pose_ref", "q", "qd", "qref", "h")}
    s = _Inst(**{k: v.ctypes.data for k, v in arrs.items()})
    return s, arrs


def assemble(prob, inputs, b=0):
    """A0 [m0][n] / b0: the Cartesian rows, level-0 rows first, then the middle level's (prob.m_l0
    of them are level 0)."""
    n = prob.n
    d, keep = _desc(prob)
    s, arrs = _inst(inputs, b)
    A0 = np.zeros((prob.m0, n))
    b0 = np.zeros(prob.m0)
    H1 = np.zeros((n, n))
    g1, lb, ub = np.zeros(n), np.zeros(n), np.zeros(n)
    m0 = lib().wbq_ref_assemble(ctypes.byref(d), ctypes.byref(s), _p(A0), _p(b0), _p(H1), _p(g1),
                                _p(lb), _p(ub))
    if m0 < 0:
        raise np.linalg.LinAlgError("M not SPD")
    return dict(A0=A0, b0=b0, H1=H1, g1=g1, lb=lb, ub=ub)


def level0(A, b, lb, ub, state=None):
    m, n = A.shape
    x = np.zeros(n)
    st = np.zeros(n, dtype=np.int32) if state is None else np.ascontiguousarray(state, dtype=np.int32)
    it = ctypes.c_int(0)
    rc = lib().wbq_ref_level0(m, n, _p(_c(A)), _p(_c(b)), _p(_c(lb)), _p(_c(ub)), _p(x), _p(st),
                              ctypes.byref(it))
    return rc, x, st, it.value


def level1(H, g, Aeq, beq, lb, ub, x0, state):
    n = H.shape[0]
    me = Aeq.shape[0]
    x = _c(x0).copy()
    st = np.ascontiguousarray(state, dtype=np.int32).copy()
    it = ctypes.c_int(0)
    rc = lib().wbq_ref_level1(n, _p(_c(H)), _p(_c(g)), me, _p(_c(Aeq)), _p(_c(beq)), _p(_c(lb)),
                              _p(_c(ub)), _p(x), _p(st), ctypes.byref(it))
    return rc, x, st, it.value


def qppvm_one(prob, inputs, b=0):
    d, keep = _desc(prob)
    s, arrs = _inst(inputs, b)
    tau = np.zeros(prob.n)
    y0 = np.zeros(prob.m0)
    it = ctypes.c_int(0)
    st = lib().wbq_ref_qppvm_one(ctypes.byref(d), ctypes.byref(s), _p(tau), _p(y0), ctypes.byref(it))
    return tau, y0, st, it.value


def qppvm_batch(prob, inputs):
    """tau[B, n], status[B], iters[B] for a whole batch (single thread)."""
    d, keep = _desc(prob)
    arrs = [_c(inputs[k]) for k in ("M", "J", "pose", "pose_ref", "q", "qd", "qref", "h")]
    B = arrs[-1].shape[0]
    tau = np.zeros((B, prob.n))
    status = np.zeros(B, dtype=np.int32)
    iters = np.zeros(B, dtype=np.int32)
    lib().wbq_ref_qppvm_batch(ctypes.byref(d), B, *[_p(a) for a in arrs], _p(tau), _p(status),
                              _p(iters))
    return tau, status, iters


# ------------------------------------------------------------------ contact form (ForceAcc)
class _CDesc(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int), ("n_fb", ctypes.c_int), ("nc", ctypes.c_int),
                ("Kp_w", ctypes.c_double), ("Kd_w", ctypes.c_double), ("Kp_f", ctypes.c_double),
                ("Kd_f", ctypes.c_double), ("Kp_p", ctypes.c_double), ("Kd_p", ctypes.c_double),
                ("f_lb", ctypes.c_double * 3), ("f_ub", ctypes.c_double * 3), ("eps_f", ctypes.c_double),
                ("torque_rows", ctypes.c_int), ("tau_max", ctypes.c_void_p), ("tau_min", ctypes.c_void_p),
                ("wrench_dim", ctypes.c_int), ("m_lb", ctypes.c_double * 3), ("m_ub", ctypes.c_double * 3),
                ("mu", ctypes.c_double)]


class _CInst(ctypes.Structure):
    _fields_ = [(k, ctypes.c_void_p) for k in ("M", "h", "q", "qd", "qref", "Jw", "jdqd_w", "pose_w",
                                               "pose_w_ref", "Jc", "jdqd_c", "pose_c", "pose_c_ref")] + \
               [("contact_mask", ctypes.c_int)]


CONTACT_ARRAYS = ("M", "h", "q", "qd", "qref", "Jw", "jdqd_w", "pose_w", "pose_w_ref", "Jc", "jdqd_c",
                  "pose_c", "pose_c_ref")


def _cdesc(prob):
    d = _CDesc()
    d.n, d.n_fb, d.nc = prob.n, prob.n_fb, prob.nc
    for k in ("Kp_w", "Kd_w", "Kp_f", "Kd_f", "Kp_p", "Kd_p", "eps_f"):
        setattr(d, k, float(getattr(prob, k)))
    for k in range(3):
        d.f_lb[k], d.f_ub[k] = prob.f_lb[k], prob.f_ub[k]
        d.m_lb[k], d.m_ub[k] = prob.m_lb[k], prob.m_ub[k]
    d.wrench_dim = int(getattr(prob, "wrench_dim", 3))
    d.mu = float(getattr(prob, "mu", 0.0))
    d.torque_rows = int(bool(prob.torque_rows))
    keep = [np.ascontiguousarray(prob.tau_max, dtype=np.float64), np.ascontiguousarray(prob.tau_min, dtype=np.float64)]
    d.tau_max, d.tau_min = keep[0].ctypes.data, keep[1].ctypes.data
    return d, keep


def _cinst(inputs, b):
    s = _CInst()
    arrs = [np.ascontiguousarray(inputs[k][b], dtype=np.float64) for k in CONTACT_ARRAYS]
    for k, a in zip(CONTACT_ARRAYS, arrs):
        setattr(s, k, a.ctypes.data)
    s.contact_mask = int(inputs["cmask"][b])
    return s, arrs


def dual_qp(H, g, E, e, C, clo, chi):
    """Dense dual active-set QP (oracle): min 0.5 x'Hx + g'x, E x = e, clo <= C x <= chi."""
    n = H.shape[0]
    H, g, E, e = _c(H), _c(g), _c(E).reshape(-1, n), _c(e)
    C, clo, chi = _c(C).reshape(-1, n), _c(clo), _c(chi)
    x = np.zeros(n)
    it = ctypes.c_int(0)
    st = lib().wbq_ref_dual_qp(n, _p(H), _p(g), E.shape[0], _p(E), _p(e), C.shape[0], _p(C), _p(clo), _p(chi),
                               _p(x), ctypes.byref(it))
    return x, st, it.value


def contact_assemble(prob, inputs, b=0):
    d, keep = _cdesc(prob)
    s, arrs = _cinst(inputs, b)
    nx = prob.nx
    mi = (prob.wrench_dim + (4 if prob.mu > 0 else 0)) * prob.nc + (prob.n - prob.n_fb if prob.torque_rows else 0)
    H, g, E, e = np.zeros((nx, nx)), np.zeros(nx), np.zeros((12, nx)), np.zeros(12)
    C, clo, chi, bw = np.zeros((max(mi, 1), nx)), np.zeros(max(mi, 1)), np.zeros(max(mi, 1)), np.zeros(6)
    lib().wbq_ref_contact_assemble(ctypes.byref(d), ctypes.byref(s), _p(H), _p(g), _p(E), _p(e), _p(C),
                                   _p(clo), _p(chi), _p(bw))
    return dict(H=H, g=g, E=E, e=e, C=C[:mi], clo=clo[:mi], chi=chi[:mi], bw=bw)


def contact_one(prob, inputs, b=0):
    d, keep = _cdesc(prob)
    s, arrs = _cinst(inputs, b)
    tau, x = np.zeros(prob.n), np.zeros(prob.nx)
    it, rep = ctypes.c_int(0), ctypes.c_int(0)
    st = lib().wbq_ref_contact_one(ctypes.byref(d), ctypes.byref(s), _p(tau), _p(x), ctypes.byref(it),
                                   ctypes.byref(rep))
    return dict(tau=tau, x=x, status=st, iters=it.value, l0_repaired=rep.value)


def contact_batch(prob, inputs):
    """tau[B, n], x[B, nx], status[B], iters[B], l0_repaired[B] (single thread)."""
    d, keep = _cdesc(prob)
    arrs = [_c(inputs[k]) for k in CONTACT_ARRAYS]
    cm = np.ascontiguousarray(inputs["cmask"], dtype=np.int32)
    B = arrs[1].shape[0]
    tau, x = np.zeros((B, prob.n)), np.zeros((B, prob.nx))
    st, it, rep = (np.zeros(B, dtype=np.int32) for _ in range(3))
    lib().wbq_ref_contact_batch(ctypes.byref(d), B, *[_p(a) for a in arrs], _p(cm), _p(tau), _p(x), _p(st),
                                _p(it), _p(rep))
    return tau, x, st, it, rep


# ---------------------------------------------------------------- rigid-body dynamics
class _RbdModel(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int), ("parent", ctypes.c_void_p), ("X_fixed", ctypes.c_void_p),
                ("axis", ctypes.c_void_p), ("mass", ctypes.c_void_p), ("com", ctypes.c_void_p),
                ("inertia", ctypes.c_void_p), ("gravity", ctypes.c_double * 3), ("ntasks", ctypes.c_int),
                ("task_link", ctypes.c_void_p), ("jtype", ctypes.c_void_p), ("task_offset", ctypes.c_void_p)]


def _rbd_model(model):
    """model: qppvm_amd.rbd.RobotModel (or any object with its fields; jtype / task_offset optional)."""
    keep = {k: np.ascontiguousarray(getattr(model, k), dtype=np.int32 if k in ("parent", "task_link") else np.float64)
            for k in ("parent", "X_fixed", "axis", "mass", "com", "inertia", "task_link")}
    for k, dt in (("jtype", np.int32), ("task_offset", np.float64)):
        v = getattr(model, k, None)
        if v is not None:
            keep[k] = np.ascontiguousarray(v, dtype=dt)
    m = _RbdModel()
    m.n = int(model.n)
    for k, v in keep.items():
        setattr(m, k, v.ctypes.data)
    m.gravity = (ctypes.c_double * 3)(*[float(g) for g in model.gravity])
    m.ntasks = int(len(keep["task_link"]))
    return m, keep


def task_jdqd(model, q, qd):
    """Jdot qd [B][T][6] of every task frame (rows [linear; angular], world frame)."""
    L = lib()
    m, keep = _rbd_model(model)
    q = np.ascontiguousarray(np.atleast_2d(q), dtype=np.float64)
    qd = np.ascontiguousarray(np.atleast_2d(qd), dtype=np.float64)
    B, T = q.shape[0], len(model.task_link)
    out = np.zeros((B, T, 6))
    for b in range(B):
        for t in range(T):
            L.wbq_ref_task_jdqd(ctypes.byref(m), _p(q[b]), _p(qd[b]), t, _p(out[b, t]))
    return out


def rbd_batch(model, q, qd):
    """M [B][n][n], h [B][n], J [B][T][6][n], pose [B][T][12] for each (q, qd) row."""
    L = lib()
    m, keep = _rbd_model(model)
    q = np.ascontiguousarray(np.atleast_2d(q), dtype=np.float64)
    qd = np.ascontiguousarray(np.atleast_2d(qd), dtype=np.float64)
    B, n, T = q.shape[0], model.n, len(model.task_link)
    M = np.zeros((B, n, n)); h = np.zeros((B, n)); J = np.zeros((B, T, 6, n)); pose = np.zeros((B, T, 12))
    for b in range(B):
        L.wbq_ref_rbd_one(ctypes.byref(m), _p(q[b]), _p(qd[b]), _p(M[b]), _p(h[b]), _p(J[b]), _p(pose[b]))
    return M, h, J, pose


def rnea(model, q, qd, qdd):
    L = lib()
    m, keep = _rbd_model(model)
    tau = np.zeros(model.n)
    L.wbq_ref_rnea(ctypes.byref(m), _p(np.ascontiguousarray(q, dtype=np.float64)),
                   _p(np.ascontiguousarray(qd, dtype=np.float64)), _p(np.ascontiguousarray(qdd, dtype=np.float64)),
                   _p(tau))
    return tau
