"""ctypes binding of libwbq (include/wbq.h). The product path: HIP kernels on the GPU.

There is no CPU fallback: constructing a solver without the built library or without a
GPU raises ``WbqError``.
"""
from __future__ import annotations

import ctypes
import os
import sys

import numpy as np

from .problem import (CONTACT_INPUT_FIELDS, INPUT_FIELDS, ContactProblem, QPPVMProblem,
                      check_contact_inputs, check_inputs)

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libwbq.so")

SUCCESS, E_INVALID, E_DEVICE, E_UNSUPPORTED, E_CAPACITY = 0, -1, -2, -3, -4
NULL_STREAM = 1  # include/wbq.h WBQ_NULL_STREAM: the device's null stream (torch's default, handle 0)


def stream_arg(handle):
    """wbq_set_stream argument for a stream handle: None -> the context's own stream, 0 (the null
    stream, e.g. torch.cuda.current_stream().cuda_stream of the default stream) -> WBQ_NULL_STREAM."""
    if handle is None:
        return None
    return NULL_STREAM if int(handle) == 0 else int(handle)
MEM_HOST, MEM_DEVICE = 0, 1
FORM_QPPVM, FORM_CONTACT = 0, 1

# every symbol include/wbq.h declares (checked by tests/test_abi.py)
EXPORTS = ("wbq_create", "wbq_set_stream", "wbq_set_inputs", "wbq_solve", "wbq_sync",
           "wbq_get_outputs", "wbq_set_outputs", "wbq_get_device_outputs", "wbq_reset_warmstart", "wbq_set_timing",
           "wbq_get_timing", "wbq_destroy", "wbq_last_error", "wbq_version", "wbq_create_contact",
           "wbq_set_contact_inputs", "wbq_get_contact_outputs", "wbq_get_timing_detail", "wbq_rollout",
           "wbq_get_state", "wbq_set_state", "wbq_get_warmstart_hints", "wbq_rbd_create", "wbq_rbd_compute",
           "wbq_rbd_set_stream", "wbq_rbd_destroy", "wbq_rollout_rbd", "wbq_rbd_compute_ex", "wbq_set_option")


class WbqError(RuntimeError):
    pass


class Desc(ctypes.Structure):
    _fields_ = [("form", ctypes.c_int), ("n", ctypes.c_int), ("ntasks", ctypes.c_int),
                ("row_mask", ctypes.c_int * 4), ("select_mode", ctypes.c_int),
                ("joint_weight", ctypes.c_int), ("max_batch", ctypes.c_int),
                ("max_iter", ctypes.c_int),
                ("Kc", ctypes.c_void_p), ("Dc", ctypes.c_void_p), ("Kq", ctypes.c_void_p),
                ("Dq", ctypes.c_void_p), ("tau_max", ctypes.c_void_p), ("tau_min", ctypes.c_void_p),
                ("joint_limits", ctypes.c_int), ("q_min", ctypes.c_void_p), ("q_max", ctypes.c_void_p),
                ("Kjl", ctypes.c_void_p), ("Djl", ctypes.c_void_p), ("task_level", ctypes.c_int * 4),
                ("no_joint_task", ctypes.c_int)]


class Inputs(ctypes.Structure):
    _fields_ = [("batch", ctypes.c_int), ("memory", ctypes.c_int)] + \
               [(k, ctypes.c_void_p) for k in INPUT_FIELDS]


class ContactDesc(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int), ("n_fb", ctypes.c_int), ("nc", ctypes.c_int),
                ("torque_rows", ctypes.c_int), ("max_batch", ctypes.c_int), ("max_iter", ctypes.c_int)] + \
               [(k, ctypes.c_double) for k in ("Kp_w", "Kd_w", "Kp_f", "Kd_f", "Kp_p", "Kd_p")] + \
               [("f_lb", ctypes.c_double * 3), ("f_ub", ctypes.c_double * 3), ("eps_f", ctypes.c_double),
                ("tau_max", ctypes.c_void_p), ("tau_min", ctypes.c_void_p),
                ("wrench_dim", ctypes.c_int), ("m_lb", ctypes.c_double * 3), ("m_ub", ctypes.c_double * 3),
                ("mu", ctypes.c_double)]


_CONTACT_F64 = tuple(k for k in CONTACT_INPUT_FIELDS if k != "cmask")


class ContactInputs(ctypes.Structure):
    _fields_ = [("batch", ctypes.c_int), ("memory", ctypes.c_int)] + \
               [(k, ctypes.c_void_p) for k in _CONTACT_F64] + [("cmask", ctypes.c_void_p)]


_lib = None


def _preload_hip_runtime():
    """One HIP runtime per process. torch ships its own libamdhip64 (soname libamdhip64.so.7, as
    /opt/rocm's): whichever copy loads first serves every later user of that soname. If libwbq
    pulled /opt/rocm's copy in first, a later `import torch` would find that runtime already in the
    process and see no GPU. So when torch is installed, its copy is loaded here by path -- without
    importing torch -- and libwbq, torch tensors and torch streams share it; without torch,
    /opt/rocm's copy is the runtime."""
    if "torch" in sys.modules:  # its runtime is in the process already
        return
    import importlib.util
    spec = importlib.util.find_spec("torch")
    if spec is None or not spec.submodule_search_locations:
        return
    rt = os.path.join(list(spec.submodule_search_locations)[0], "lib", "libamdhip64.so")
    if os.path.exists(rt):
        ctypes.CDLL(rt, mode=ctypes.RTLD_GLOBAL)


def load_library(path: str = LIB_PATH):
    """Load libwbq.so; raises WbqError (never falls back) when it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise WbqError(f"{path} not built: run `python -m qppvm_amd.build` (hipcc, gfx950)")
    _preload_hip_runtime()
    lib = ctypes.CDLL(path)
    P, I = ctypes.c_void_p, ctypes.c_int
    lib.wbq_create.argtypes = [ctypes.POINTER(Desc), I, ctypes.POINTER(P)]
    lib.wbq_set_stream.argtypes = [P, P]
    lib.wbq_set_inputs.argtypes = [P, ctypes.POINTER(Inputs)]
    lib.wbq_solve.argtypes = [P]
    lib.wbq_sync.argtypes = [P]
    lib.wbq_get_outputs.argtypes = [P, P, P, P]
    lib.wbq_set_outputs.argtypes = [P, P, P, P]
    lib.wbq_get_device_outputs.argtypes = [P, ctypes.POINTER(P), ctypes.POINTER(P), ctypes.POINTER(P)]
    lib.wbq_reset_warmstart.argtypes = [P, P]
    lib.wbq_set_timing.argtypes = [P, I]
    lib.wbq_get_timing.argtypes = [P, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(I)]
    lib.wbq_get_timing_detail.argtypes = [P, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                          ctypes.POINTER(I)]
    lib.wbq_destroy.argtypes = [P]
    lib.wbq_destroy.restype = None
    lib.wbq_last_error.argtypes = [P]
    lib.wbq_last_error.restype = ctypes.c_char_p
    lib.wbq_version.restype = ctypes.c_char_p
    lib.wbq_create_contact.argtypes = [ctypes.POINTER(ContactDesc), I, ctypes.POINTER(P)]
    lib.wbq_set_contact_inputs.argtypes = [P, ctypes.POINTER(ContactInputs)]
    lib.wbq_get_contact_outputs.argtypes = [P, P]
    lib.wbq_rollout.argtypes = [P, I, ctypes.c_double]
    lib.wbq_set_option.argtypes = [P, I, I]
    lib.wbq_get_state.argtypes = [P, P, P]
    lib.wbq_set_state.argtypes = [P, P, P, I]
    lib.wbq_get_warmstart_hints.argtypes = [P, P]
    lib.wbq_rbd_create.argtypes = [P, I, ctypes.POINTER(P)]
    lib.wbq_rbd_compute.argtypes = [P, I, P, P, P, P, P, P, I]
    lib.wbq_rbd_compute_ex.argtypes = [P, I, P, P, P, P, P, P, P, I]
    lib.wbq_rbd_set_stream.argtypes = [P, P]
    lib.wbq_rbd_destroy.argtypes = [P]
    lib.wbq_rbd_destroy.restype = None
    lib.wbq_rollout_rbd.argtypes = [P, P, I, ctypes.c_double]
    for f in ("wbq_create", "wbq_set_stream", "wbq_set_inputs", "wbq_solve", "wbq_sync",
              "wbq_get_outputs", "wbq_set_outputs", "wbq_get_device_outputs",
              "wbq_reset_warmstart", "wbq_create_contact", "wbq_set_contact_inputs",
              "wbq_get_contact_outputs", "wbq_set_timing", "wbq_get_timing", "wbq_get_timing_detail",
              "wbq_rollout", "wbq_get_state", "wbq_set_state", "wbq_get_warmstart_hints", "wbq_rbd_create",
              "wbq_rbd_compute", "wbq_rbd_set_stream", "wbq_rollout_rbd", "wbq_rbd_compute_ex"):
        getattr(lib, f).restype = I
    _lib = lib
    return lib


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


class QPPVMSolver:
    """Batched drop-in for QPPVMPlugin's per-tick solve (tasks + AutoStack + QPOases_sot).

    One context = one device, one HIP stream, buffers sized for ``max_batch``.
    """

    def __init__(self, prob: QPPVMProblem, max_batch: int, device: int = 0):
        self.lib = load_library()
        self.prob = prob
        self.max_batch = int(max_batch)
        d = Desc()
        d.form, d.n, d.ntasks = FORM_QPPVM, prob.n, prob.ntasks
        for t in range(4):
            d.row_mask[t] = prob.row_mask[t] if t < prob.ntasks else 0
        d.select_mode, d.joint_weight = prob.select_mode, prob.joint_weight
        for t, lv in enumerate(prob.task_level):
            d.task_level[t] = int(lv)
        d.no_joint_task = 0 if prob.joint_task else 1
        d.max_batch, d.max_iter = self.max_batch, int(prob.max_iter)
        self._keep = [np.ascontiguousarray(getattr(prob, k), dtype=np.float64)
                      for k in ("Kc", "Dc", "Kq", "Dq", "tau_max", "tau_min")]
        d.Kc, d.Dc, d.Kq, d.Dq, d.tau_max, d.tau_min = [_ptr(a) for a in self._keep]
        if prob.joint_limits:
            jl = [np.ascontiguousarray(getattr(prob, k), dtype=np.float64) for k in ("q_min", "q_max", "Kjl", "Djl")]
            self._keep += jl
            d.joint_limits = 1
            d.q_min, d.q_max, d.Kjl, d.Djl = [_ptr(a) for a in jl]
        h = ctypes.c_void_p()
        rc = self.lib.wbq_create(ctypes.byref(d), int(device), ctypes.byref(h))
        if rc != SUCCESS:
            raise WbqError(f"wbq_create failed ({rc}): check the GPU / problem support")
        self.ctx = h
        self.batch = 0
        self._host_inputs = None

    # -- errors
    def _check(self, rc, what):
        if rc != SUCCESS:
            msg = self.lib.wbq_last_error(self.ctx).decode()
            raise WbqError(f"{what} failed ({rc}): {msg}")

    def close(self):
        if getattr(self, "ctx", None):
            self.lib.wbq_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- inputs
    def set_inputs(self, inputs: dict):
        """Host numpy arrays (copied async H2D into context buffers)."""
        B = check_inputs(self.prob, inputs)
        arrs = {k: np.ascontiguousarray(inputs[k], dtype=np.float64) for k in INPUT_FIELDS}
        self._host_inputs = arrs  # keep alive until the async copy completes
        s = Inputs(batch=B, memory=MEM_HOST, **{k: _ptr(v) for k, v in arrs.items()})
        self._check(self.lib.wbq_set_inputs(self.ctx, ctypes.byref(s)), "wbq_set_inputs")
        self.batch = B

    def set_device_inputs(self, ptrs: dict, batch: int):
        """Device pointers (e.g. torch tensors' data_ptr()) adopted without copy."""
        s = Inputs(batch=int(batch), memory=MEM_DEVICE, **{k: int(ptrs[k]) for k in INPUT_FIELDS})
        self._check(self.lib.wbq_set_inputs(self.ctx, ctypes.byref(s)), "wbq_set_inputs")
        self.batch = int(batch)

    def set_stream(self, stream_handle: int | None):
        """Launch on this HIP stream handle (None: the context's own stream; 0: the null stream, which is
        torch's default stream)."""
        self._check(self.lib.wbq_set_stream(self.ctx, stream_arg(stream_handle)), "wbq_set_stream")

    # -- solve
    def solve(self):
        self._check(self.lib.wbq_solve(self.ctx), "wbq_solve")

    def sync(self):
        self._check(self.lib.wbq_sync(self.ctx), "wbq_sync")

    def outputs(self):
        B, n = self.batch, self.prob.n
        tau = np.empty((B, n))
        status = np.empty(B, dtype=np.int32)
        iters = np.empty(B, dtype=np.int32)
        self._check(self.lib.wbq_get_outputs(self.ctx, _ptr(tau), _ptr(status), _ptr(iters)),
                    "wbq_get_outputs")
        return tau, status, iters

    def set_device_outputs(self, tau_ptr, status_ptr=None, iters_ptr=None):
        """Write outputs straight into caller-owned device buffers (e.g. torch tensors)."""
        self._check(self.lib.wbq_set_outputs(self.ctx, tau_ptr or None, status_ptr or None,
                                             iters_ptr or None), "wbq_set_outputs")

    def device_outputs(self):
        t, s, i = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
        self._check(self.lib.wbq_get_device_outputs(self.ctx, ctypes.byref(t), ctypes.byref(s),
                                                    ctypes.byref(i)), "wbq_get_device_outputs")
        return t.value, s.value, i.value

    OPT_INLINE_REPAIR = 1  # include/wbq.h WBQ_OPT_*
    OPT_FUSED_ROLLOUT = 2
    OPT_FOLLOWUP = 3  # on-demand follow-up kernel (completed when outputs are read)
    OPT_HANDBACK = 4  # n > 32: a repaired instance's dual loop in the hand-back pass
    OPT_GI_HANDOFF = 5  # n > 32: active-set steps before the level-0 repair takes over (0 = never)

    def set_option(self, option: int, value: int):
        """Per-context execution option (wbq_set_option): a path choice, never a result change."""
        self._check(self.lib.wbq_set_option(self.ctx, int(option), int(value)), "wbq_set_option")

    def rollout(self, steps: int, dt: float = 1e-3):
        """``steps`` solves with q, qd integrated on the device between them (wbq_rollout)."""
        self._check(self.lib.wbq_rollout(self.ctx, int(steps), float(dt)), "wbq_rollout")

    def state(self):
        """The batch's current (q, qd) on the device."""
        q = np.empty((self.batch, self.prob.n))
        qd = np.empty((self.batch, self.prob.n))
        self._check(self.lib.wbq_get_state(self.ctx, _ptr(q), _ptr(qd)), "wbq_get_state")
        return q, qd

    def set_state(self, q=None, qd=None, device: bool = False):
        """Overwrite (q, qd): numpy arrays, or device pointers (ints) with device=True."""
        if device:
            self._check(self.lib.wbq_set_state(self.ctx, q or None, qd or None, MEM_DEVICE), "wbq_set_state")
            return
        qa = None if q is None else np.ascontiguousarray(q, dtype=np.float64)
        qda = None if qd is None else np.ascontiguousarray(qd, dtype=np.float64)
        self._check(self.lib.wbq_set_state(self.ctx, None if qa is None else _ptr(qa),
                                           None if qda is None else _ptr(qda), MEM_HOST), "wbq_set_state")

    def solve_batch(self, inputs: dict):
        self.set_inputs(inputs)
        self.solve()
        return self.outputs()

    def reset_warmstart(self, mask=None):
        """Drop the warm start of the instances with mask[b] != 0 (one entry per instance of the
        current batch; None = all)."""
        m = None if mask is None else np.ascontiguousarray(mask, dtype=np.uint8)
        if m is not None and m.shape != (self.batch,):
            raise ValueError(f"mask must have one entry per instance of the batch ({self.batch}), got {m.shape}")
        self._check(self.lib.wbq_reset_warmstart(self.ctx, None if m is None else _ptr(m)),
                    "wbq_reset_warmstart")

    def rollout_rbd(self, rbd, steps: int, dt: float):
        """MPC rollout with M, h, J and poses re-evaluated on the device every step from the
        integrated state (``rbd``: qppvm_amd.rbd.RBDModel on the same device)."""
        self._check(self.lib.wbq_rollout_rbd(self.ctx, rbd.ctx, int(steps), float(dt)), "wbq_rollout_rbd")

    def warm_hints(self) -> np.ndarray:
        """Per-instance warm-start hints of the current batch (1 = the last solve went through
        the level-0 repair with level 0 infeasible at b0)."""
        out = np.zeros(self.batch, dtype=np.uint8)
        if self.batch:
            self._check(self.lib.wbq_get_warmstart_hints(self.ctx, _ptr(out)), "wbq_get_warmstart_hints")
        return out

    # -- timing (HIP events around every launch, on the launch stream)
    def set_timing(self, enable: bool, every: int = 1):
        """Time every ``every``-th solve with HIP events (0 / False disables)."""
        self._check(self.lib.wbq_set_timing(self.ctx, int(every) if enable else 0), "wbq_set_timing")

    def get_timing(self):
        ms = ctypes.c_double()
        cnt = ctypes.c_int()
        self._check(self.lib.wbq_get_timing(self.ctx, ctypes.byref(ms), ctypes.byref(cnt)),
                    "wbq_get_timing")
        return ms.value, cnt.value

    def get_timing_detail(self):
        """(summed solve ms, summed dominant-kernel ms, timed solves) since the last read."""
        ms, km = ctypes.c_double(), ctypes.c_double()
        cnt = ctypes.c_int()
        self._check(self.lib.wbq_get_timing_detail(self.ctx, ctypes.byref(ms), ctypes.byref(km),
                                                   ctypes.byref(cnt)), "wbq_get_timing_detail")
        return ms.value, km.value, cnt.value


class ContactSolver(QPPVMSolver):
    """Batched drop-in for ForceAccExample's per-tick solve (OptvarHelper variables, feet /
    postural / waist acceleration tasks, DynamicFeasibility, wrench bounds, QPOases_sot, and
    the inverse-dynamics post-step; reference src/ForceAcc.cpp:31-141,181-219).
    Same context semantics as QPPVMSolver; outputs add x = [qdd; w] (w: 3 forces or the 6-D
    wrench per contact)."""

    def __init__(self, prob: ContactProblem, max_batch: int, device: int = 0):
        self.lib = load_library()
        self.prob = prob
        self.max_batch = int(max_batch)
        d = ContactDesc()
        d.n, d.n_fb, d.nc, d.torque_rows = prob.n, prob.n_fb, prob.nc, int(bool(prob.torque_rows))
        d.max_batch, d.max_iter = self.max_batch, int(prob.max_iter)
        for k in ("Kp_w", "Kd_w", "Kp_f", "Kd_f", "Kp_p", "Kd_p", "eps_f"):
            setattr(d, k, float(getattr(prob, k)))
        for k in range(3):
            d.f_lb[k], d.f_ub[k] = prob.f_lb[k], prob.f_ub[k]
            d.m_lb[k], d.m_ub[k] = prob.m_lb[k], prob.m_ub[k]
        d.wrench_dim, d.mu = prob.wrench_dim, prob.mu
        self._keep = [np.ascontiguousarray(prob.tau_max, dtype=np.float64),
                      np.ascontiguousarray(prob.tau_min, dtype=np.float64)]
        d.tau_max, d.tau_min = _ptr(self._keep[0]), _ptr(self._keep[1])
        h = ctypes.c_void_p()
        rc = self.lib.wbq_create_contact(ctypes.byref(d), int(device), ctypes.byref(h))
        if rc != SUCCESS:
            raise WbqError(f"wbq_create_contact failed ({rc}): check the GPU / problem support")
        self.ctx = h
        self.batch = 0
        self._host_inputs = None

    def set_inputs(self, inputs: dict):
        B = check_contact_inputs(self.prob, inputs)
        arrs = {k: np.ascontiguousarray(inputs[k], dtype=np.float64) for k in _CONTACT_F64}
        arrs["cmask"] = np.ascontiguousarray(inputs["cmask"], dtype=np.int32)
        self._host_inputs = arrs
        s = ContactInputs(batch=B, memory=MEM_HOST, **{k: _ptr(v) for k, v in arrs.items()})
        self._check(self.lib.wbq_set_contact_inputs(self.ctx, ctypes.byref(s)), "wbq_set_contact_inputs")
        self.batch = B

    def set_device_inputs(self, ptrs: dict, batch: int):
        s = ContactInputs(batch=int(batch), memory=MEM_DEVICE, **{k: int(ptrs[k]) for k in CONTACT_INPUT_FIELDS})
        self._check(self.lib.wbq_set_contact_inputs(self.ctx, ctypes.byref(s)), "wbq_set_contact_inputs")
        self.batch = int(batch)

    def x(self):
        out = np.empty((self.batch, self.prob.nx))
        self._check(self.lib.wbq_get_contact_outputs(self.ctx, _ptr(out)), "wbq_get_contact_outputs")
        return out


def version() -> str:
    return load_library().wbq_version().decode()
