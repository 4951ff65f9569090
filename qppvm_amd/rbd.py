"""Robot models for the on-GPU rigid-body dynamics (qppvm_amd/csrc/rbd.hip).

``RobotModel`` is the host description behind ``wbq_rbd_desc`` (include/wbq.h): a kinematic
tree of revolute or prismatic joints, one per link, ``parent[i] < i``; a floating base is six
virtual joints (``with_floating_base``: x, y, z prismatic, then z, y, x revolute, massless links
between), task frames are a link times a fixed offset (a frame on a fixed joint of the URDF).
``qppvm_amd.urdf.load_urdf`` builds one from a URDF file. ``centauro_like()`` builds the
synthetic stand-in for the CENTAURO model the reference loads from its URDF/YAML
(QPPVMPlugin.cpp:50-51; not in the container): a pelvis-fixed torso joint with two 7-DoF arms
(links ``arm1_1..7`` = 1..7, ``arm2_1..7`` = 8..14, the dof order of the dummy robot) and four
6-DoF legs, n = 39, tasks on ``arm2_7`` and ``arm1_7`` as QPPVMPlugin's stack.
``RBDModel`` wraps a device context (wbq_rbd_create / wbq_rbd_compute).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field

import numpy as np

from . import wbq


@dataclass
class RobotModel:
    parent: np.ndarray       # [n] int32
    X_fixed: np.ndarray      # [n][12] joint frame in the parent link frame at q = 0, [R | p]
    axis: np.ndarray         # [n][3] unit, joint frame
    mass: np.ndarray         # [n]
    com: np.ndarray          # [n][3] link frame
    inertia: np.ndarray      # [n][6] Ixx Iyy Izz Ixy Ixz Iyz about the COM, link frame
    task_link: np.ndarray    # [T] int32
    gravity: tuple = (0.0, 0.0, -9.81)
    names: list = field(default_factory=list)
    jtype: np.ndarray | None = None        # [n] int32, 0 revolute / 1 prismatic (None: revolute)
    task_offset: np.ndarray | None = None  # [T][12] task frame in its link's frame (None: identity)
    task_names: list = field(default_factory=list)

    @property
    def n(self) -> int:
        return int(len(self.parent))

    @property
    def ntasks(self) -> int:
        return int(len(self.task_link))


def _rot(rng, scale):
    w = rng.normal(0.0, scale, 3)
    th = np.linalg.norm(w)
    if th == 0.0:
        return np.eye(3)
    k = w / th
    K = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + np.sin(th) * K + (1 - np.cos(th)) * K @ K


def random_tree(parent, seed=0, task_link=(), names=None, link_len=(0.08, 0.3)):
    """Random but physical kinematics and inertias on a given tree: link lengths ``link_len`` m,
    joint frames rotated by up to ~60 deg, masses 0.5-5 kg, COMs inside the link, principal
    inertias of a rod-like body (positive definite, triangle inequality holds)."""
    rng = np.random.default_rng(seed)
    n = len(parent)
    X = np.zeros((n, 12)); axis = np.zeros((n, 3)); mass = np.zeros(n); com = np.zeros((n, 3))
    inertia = np.zeros((n, 6))
    for i in range(n):
        R = _rot(rng, 0.6)
        p = rng.normal(0.0, 1.0, 3)
        p *= rng.uniform(*link_len) / np.linalg.norm(p)
        X[i] = np.concatenate([R, p[:, None]], axis=1).reshape(-1)
        a = rng.normal(0.0, 1.0, 3)
        axis[i] = a / np.linalg.norm(a)
        mass[i] = rng.uniform(0.5, 5.0)
        com[i] = rng.normal(0.0, 0.05, 3)
        # rod of length l along a random direction: principal moments m l^2/12 (two) + a small one
        l = rng.uniform(0.1, 0.4)
        lam = mass[i] * np.array([l * l / 12, l * l / 12, 0.002 + 0.01 * rng.random()])
        Q = _rot(rng, 2.0)
        Ib = Q @ np.diag(lam) @ Q.T
        inertia[i] = [Ib[0, 0], Ib[1, 1], Ib[2, 2], Ib[0, 1], Ib[0, 2], Ib[1, 2]]
    return RobotModel(parent=np.asarray(parent, dtype=np.int32), X_fixed=X, axis=axis, mass=mass, com=com,
                      inertia=inertia, task_link=np.asarray(task_link, dtype=np.int32), names=names or [])


REVOLUTE, PRISMATIC = 0, 1


def with_floating_base(model: RobotModel, base_mass: float = 20.0, base_com=(0.0, 0.0, 0.0),
                       base_inertia=(0.6, 0.5, 0.3, 0.0, 0.0, 0.0)) -> RobotModel:
    """The model on a floating base: six virtual joints first (translation x, y, z, then rotation
    z, y, x about the moving axes: q[0:3] base position, q[3:6] ZYX Euler angles), the base body
    (mass, COM, inertia in its frame) on the sixth; the model's roots hang off the base body. The
    ForceAcc contact form's first n_fb = 6 coordinates (ForceAcc.cpp:256-282 set the base state
    from the simulator)."""
    n0 = model.n
    eye = np.array([1.0, 0, 0, 0, 0, 1.0, 0, 0, 0, 0, 1.0, 0])
    X = np.vstack([np.tile(eye, (6, 1)), model.X_fixed])
    axis = np.vstack([np.eye(3), np.array([[0, 0, 1.0], [0, 1.0, 0], [1.0, 0, 0]]), model.axis])
    parent = np.concatenate([np.arange(-1, 5), np.where(model.parent < 0, 5, model.parent + 6)]).astype(np.int32)
    mass = np.concatenate([np.zeros(5), [base_mass], model.mass])
    com = np.vstack([np.zeros((5, 3)), np.asarray(base_com, dtype=float)[None], model.com])
    inertia = np.vstack([np.zeros((5, 6)), np.asarray(base_inertia, dtype=float)[None], model.inertia])
    jt = np.concatenate([[PRISMATIC] * 3, [REVOLUTE] * 3,
                         model.jtype if model.jtype is not None else np.zeros(n0, np.int32)]).astype(np.int32)
    return RobotModel(parent=parent, X_fixed=X, axis=axis, mass=mass, com=com, inertia=inertia,
                      task_link=np.asarray(model.task_link, np.int32) + 6, gravity=model.gravity,
                      names=["base_x", "base_y", "base_z", "base_yaw", "base_pitch", "base_roll"] + list(model.names),
                      jtype=jt, task_offset=model.task_offset, task_names=list(model.task_names))


def centauro_like(seed=7) -> RobotModel:
    """n = 39: torso (0), arm1 1-7, arm2 8-14 (both on the torso), four 6-DoF legs on the
    pelvis (the fixed base here). Tasks: arm2_7 (14), arm1_7 (7) -- QPPVMPlugin's right/left."""
    parent = [-1]
    names = ["torso_yaw"]
    for arm in (1, 2):
        for j in range(7):
            parent.append(0 if j == 0 else len(parent) - 1)
            names.append(f"arm{arm}_{j + 1}")
    for leg in range(4):
        for j in range(6):
            parent.append(-1 if j == 0 else len(parent) - 1)
            names.append(f"leg{leg + 1}_{j + 1}")
    return random_tree(parent, seed=seed, task_link=(14, 7), names=names)


def humanoid_like(n=30, seed=5) -> RobotModel:
    """A floating-base-free humanoid-like tree of n >= 16 joints: a torso chain on the fixed
    pelvis, two 7-DoF arms on the torso top, the remaining joints as two legs on the pelvis.
    Tasks on the two arm ends (right first, as QPPVMPlugin's stack)."""
    if n < 16:
        raise ValueError("humanoid_like needs n >= 16")
    legs = n - 14 - 2
    parent, names = [-1, 0], ["torso_1", "torso_2"]
    ends = []
    for arm in (1, 2):
        for j in range(7):
            parent.append(1 if j == 0 else len(parent) - 1)
            names.append(f"arm{arm}_{j + 1}")
        ends.append(len(parent) - 1)
    for leg in range(2):
        cnt = legs // 2 + (leg < legs % 2)
        for j in range(cnt):
            parent.append(-1 if j == 0 else len(parent) - 1)
            names.append(f"leg{leg + 1}_{j + 1}")
    return random_tree(parent, seed=seed, task_link=(ends[1], ends[0]), names=names)


def serial_chain(n=30, seed=3, ntasks=2) -> RobotModel:
    """A serial chain (depth n) with tasks on the last link and the middle link."""
    parent = [-1] + list(range(n - 1))
    tl = (n - 1, n // 2)[:ntasks]
    return random_tree(parent, seed=seed, task_link=tl)


class _Desc(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int), ("parent", ctypes.c_void_p), ("X_fixed", ctypes.c_void_p),
                ("axis", ctypes.c_void_p), ("mass", ctypes.c_void_p), ("com", ctypes.c_void_p),
                ("inertia", ctypes.c_void_p), ("gravity", ctypes.c_double * 3), ("ntasks", ctypes.c_int),
                ("task_link", ctypes.c_void_p), ("max_batch", ctypes.c_int), ("jtype", ctypes.c_void_p),
                ("task_offset", ctypes.c_void_p)]


class RBDModel:
    """Device context computing M, h, J, poses for batches of (q, qd) (wbq_rbd_* C ABI)."""

    def __init__(self, model: RobotModel, max_batch: int, device: int = 0):
        self.lib = wbq.load_library()
        self.model = model
        self.max_batch = int(max_batch)
        self._keep = {k: np.ascontiguousarray(getattr(model, k),
                                              dtype=np.int32 if k in ("parent", "task_link") else np.float64)
                      for k in ("parent", "X_fixed", "axis", "mass", "com", "inertia", "task_link")}
        for k, dt in (("jtype", np.int32), ("task_offset", np.float64)):
            if getattr(model, k, None) is not None:
                self._keep[k] = np.ascontiguousarray(getattr(model, k), dtype=dt)
        d = _Desc()
        d.n = model.n
        for k, v in self._keep.items():
            setattr(d, k, v.ctypes.data)
        d.gravity = (ctypes.c_double * 3)(*[float(g) for g in model.gravity])
        d.ntasks = model.ntasks
        d.max_batch = self.max_batch
        h = ctypes.c_void_p()
        rc = self.lib.wbq_rbd_create(ctypes.byref(d), int(device), ctypes.byref(h))
        if rc != wbq.SUCCESS:
            raise wbq.WbqError(f"wbq_rbd_create failed ({rc})")
        self.ctx = h

    def compute(self, q, qd):
        """Host (q, qd) [B][n] -> M [B][n][n], h [B][n], J [B][T][6][n], pose [B][T][12]."""
        q = np.ascontiguousarray(np.atleast_2d(q), dtype=np.float64)
        qd = np.ascontiguousarray(np.atleast_2d(qd), dtype=np.float64)
        B, n, T = q.shape[0], self.model.n, self.model.ntasks
        M = np.empty((B, n, n)); h = np.empty((B, n)); J = np.empty((B, T, 6, n)); pose = np.empty((B, T, 12))
        rc = self.lib.wbq_rbd_compute(self.ctx, B, q.ctypes.data, qd.ctypes.data, M.ctypes.data, h.ctypes.data,
                                      J.ctypes.data, pose.ctypes.data, wbq.MEM_HOST)
        if rc != wbq.SUCCESS:
            raise wbq.WbqError(f"wbq_rbd_compute failed ({rc})")
        return M, h, J, pose

    def compute_jdqd(self, q, qd):
        """Host (q, qd) -> (M, h, J, pose, jdqd [B][T][6]) (wbq_rbd_compute_ex)."""
        q = np.ascontiguousarray(np.atleast_2d(q), dtype=np.float64)
        qd = np.ascontiguousarray(np.atleast_2d(qd), dtype=np.float64)
        B, n, T = q.shape[0], self.model.n, self.model.ntasks
        M = np.empty((B, n, n)); h = np.empty((B, n)); J = np.empty((B, T, 6, n)); pose = np.empty((B, T, 12))
        jd = np.empty((B, T, 6))
        rc = self.lib.wbq_rbd_compute_ex(self.ctx, B, q.ctypes.data, qd.ctypes.data, M.ctypes.data, h.ctypes.data,
                                         J.ctypes.data, pose.ctypes.data, jd.ctypes.data, wbq.MEM_HOST)
        if rc != wbq.SUCCESS:
            raise wbq.WbqError(f"wbq_rbd_compute_ex failed ({rc})")
        return M, h, J, pose, jd

    def compute_device(self, B, q_ptr, qd_ptr, M_ptr, h_ptr, J_ptr, pose_ptr):
        """Device pointers (e.g. torch tensors' data_ptr()), asynchronous on the context stream."""
        rc = self.lib.wbq_rbd_compute(self.ctx, int(B), q_ptr, qd_ptr, M_ptr, h_ptr, J_ptr, pose_ptr, wbq.MEM_DEVICE)
        if rc != wbq.SUCCESS:
            raise wbq.WbqError(f"wbq_rbd_compute failed ({rc})")

    def set_stream(self, stream_handle):
        self.lib.wbq_rbd_set_stream(self.ctx, wbq.stream_arg(stream_handle))

    def close(self):
        if getattr(self, "ctx", None):
            self.lib.wbq_rbd_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
