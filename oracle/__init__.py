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
SRC = os.path.join(HERE, "wbq_oracle.c")


def build(force: bool = False) -> str:
    """Compile the C restatement with gcc (host only)."""
    if force or not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < max(
            os.path.getmtime(SRC), os.path.getmtime(os.path.join(HERE, "wbq_oracle.h"))):
        subprocess.check_call(["gcc", "-O2", "-std=c99", "-fPIC", "-shared", "-Wall", "-Wextra",
                               "-Wno-unused-parameter", SRC, "-o", LIB_PATH, "-lm"])
    return LIB_PATH


class _Desc(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int), ("ntasks", ctypes.c_int), ("row_mask", ctypes.c_int * 4),
                ("select_mode", ctypes.c_int), ("joint_weight", ctypes.c_int),
                ("Kc", ctypes.c_void_p), ("Dc", ctypes.c_void_p), ("Kq", ctypes.c_void_p),
                ("Dq", ctypes.c_void_p), ("tau_max", ctypes.c_void_p), ("tau_min", ctypes.c_void_p)]


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
        _lib.wbq_ref_qppvm_one.argtypes = [P, P, P, P, P]
        _lib.wbq_ref_qppvm_one.restype = ctypes.c_int
        _lib.wbq_ref_qppvm_batch.argtypes = [P, ctypes.c_int] + [P] * 8 + [P, P, P]
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _desc(prob):
    d = _Desc()
    d.n, d.ntasks = prob.n, prob.ntasks
    for t in range(4):
        d.row_mask[t] = prob.row_mask[t] if t < prob.ntasks else 0
    d.select_mode, d.joint_weight = prob.select_mode, prob.joint_weight
    keep = [np.ascontiguousarray(getattr(prob, k), dtype=np.float64)
            for k in ("Kc", "Dc", "Kq", "Dq", "tau_max", "tau_min")]
    d.Kc, d.Dc, d.Kq, d.Dq, d.tau_max, d.tau_min = [a.ctypes.data for a in keep]
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
