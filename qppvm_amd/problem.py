"""Host-side problem descriptor for the QPPVM torque solve.

Mirrors the configuration that ``demo::QPPVMPlugin::init_control_plugin`` wires into
OpenSoT (reference ``src/QPPVMPlugin.cpp``):

* level 0 = ``ee_task_right + ee_task_left`` (summed Cartesian impedance tasks,
  ``:129-152``, ``:177``), gains ``Kc = 700 I6``, ``Dc = 70 I6`` (``:136-137``,
  ``:148-149``), rows ``OpenSoT::Indices::range(0,2)`` (``:134``, ``:147``),
  ``useInertiaMatrix(true)`` (``:139``, ``:151``);
* level 1 = ``joint_task`` (``:114-118``), ``K = 5 I``, ``D = 2 I`` (``:105-106``);
* global bounds = ``TorqueLimits(tau_max - h, tau_min - h)`` with
  ``tau_min = -tau_max`` (``:56-58``, ``:66-67``, ``:112``, ``:203-205``);
* solver = ``QPOases_sot(stack, bounds, eps_regularisation = 1.0)`` (``:188``).

The structure is static per controller (it is the "AutoStack" of the reference);
only per-tick numbers travel to the device.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

SELECT_SUBTASK = 0  # full 6-D task built, then rows selected (OpenSoT SubTask semantics)
SELECT_TASK = 1  # task-space force masked before J^T F

WEIGHT_IDENTITY = 0  # joint task weight W1 = I
WEIGHT_INERTIA = 1  # joint task weight W1 = M

STATUS_OK = 0
STATUS_MAXITER = 1
STATUS_INFEASIBLE = 2
STATUS_NUMERICAL = 3

STATUS_NAMES = {0: "ok", 1: "max-iterations", 2: "infeasible", 3: "numerical"}


def _vec(x, n, name):
    a = np.asarray(x, dtype=np.float64)
    if a.ndim == 0:
        a = np.full(n, float(a))
    if a.shape != (n,):
        raise ValueError(f"{name} must have shape ({n},), got {a.shape}")
    return np.ascontiguousarray(a)


@dataclass
class QPPVMProblem:
    """Batch-shared structure + gains of the QPPVM stack.

    Defaults are the reference literals (QPPVMPlugin.cpp); ``tau_max`` defaults to
    150 N m per joint because the CENTAURO effort limits (URDF) are not in the
    container.
    """

    n: int
    ntasks: int = 2
    row_mask: tuple = (0x7, 0x7)
    select_mode: int = SELECT_SUBTASK
    joint_weight: int = WEIGHT_IDENTITY
    Kc: np.ndarray | float = 700.0
    Dc: np.ndarray | float = 70.0
    Kq: np.ndarray | float = 5.0
    Dq: np.ndarray | float = 2.0
    tau_max: np.ndarray | float = 150.0
    tau_min: np.ndarray | float | None = None
    max_iter: int = 0  # 0 = default cap (4 n + 32 active-set steps)
    # JointLimits toggle (QPPVMPlugin.cpp:169-171, commented out of the reference stack): the box
    # also holds Kjl (q_min - q) - Djl qd <= tau <= Kjl (q_max - q) - Djl qd (include/wbq.h)
    joint_limits: bool = False
    q_min: np.ndarray | float = -np.pi
    q_max: np.ndarray | float = np.pi
    Kjl: np.ndarray | float = 50.0
    Djl: np.ndarray | float = 20.0
    # priority level per Cartesian task: 0 = the first level (summed), 1 = a second Cartesian level --
    # the elbow tasks of QPPVMPlugin.cpp:154-166 (include/wbq.h task_level). None: all 0.
    task_level: tuple | None = None
    # False: no joint task -- the stack ends at the last Cartesian level, the reference's commented
    # elbow stack ((ee_r + ee_l) / (elbow_l + elbow_r)) << limits (QPPVMPlugin.cpp:177-178 in place of
    # :179), x the minimum-norm point among that level's optima (include/wbq.h no_joint_task)
    joint_task: bool = True
    extra: dict = field(default_factory=dict)

    def __post_init__(self):
        n, T = int(self.n), int(self.ntasks)
        if not (1 <= n <= 64):
            raise ValueError("n must be in [1, 64]")
        if not (1 <= T <= 4):
            raise ValueError("ntasks must be in [1, 4]")
        self.n, self.ntasks = n, T
        rm = tuple(int(m) for m in self.row_mask)
        if len(rm) == 1 and T > 1:
            rm = rm * T
        if len(rm) != T or any(not (0 < m < 64) for m in rm):
            raise ValueError("row_mask needs one non-empty 6-bit mask per task")
        self.row_mask = rm
        tl = (0,) * T if self.task_level is None else tuple(int(v) for v in self.task_level)
        if len(tl) != T or any(v not in (0, 1) for v in tl) or 0 not in tl:
            raise ValueError("task_level needs one level (0 or 1) per task, at least one task on level 0")
        self.task_level = tl
        kc = np.asarray(self.Kc, dtype=np.float64)
        dc = np.asarray(self.Dc, dtype=np.float64)
        self.Kc = np.ascontiguousarray(np.broadcast_to(kc, (T, 6)).astype(np.float64))
        self.Dc = np.ascontiguousarray(np.broadcast_to(dc, (T, 6)).astype(np.float64))
        self.Kq = _vec(self.Kq, n, "Kq")
        self.Dq = _vec(self.Dq, n, "Dq")
        self.tau_max = _vec(self.tau_max, n, "tau_max")
        self.tau_min = -self.tau_max if self.tau_min is None else _vec(self.tau_min, n, "tau_min")
        self.joint_limits = bool(self.joint_limits)
        self.joint_task = bool(self.joint_task)
        for k in ("q_min", "q_max", "Kjl", "Djl"):
            setattr(self, k, _vec(getattr(self, k), n, k))
        if self.select_mode not in (SELECT_SUBTASK, SELECT_TASK):
            raise ValueError("select_mode must be SELECT_SUBTASK or SELECT_TASK")
        if self.joint_weight not in (WEIGHT_IDENTITY, WEIGHT_INERTIA):
            raise ValueError("joint_weight must be WEIGHT_IDENTITY or WEIGHT_INERTIA")

    @property
    def m0(self) -> int:
        """Rows of the Cartesian levels (sum of selected task rows, the middle level included)."""
        return sum(bin(m).count("1") for m in self.row_mask)

    @property
    def m_l0(self) -> int:
        """Rows of the first level alone (m0 in the reference stack)."""
        return sum(bin(m).count("1") for m, lv in zip(self.row_mask, self.task_level) if lv == 0)


# per-instance input arrays and their shapes (B = batch)
INPUT_FIELDS = ("M", "J", "pose", "pose_ref", "q", "qd", "qref", "h")


def input_shapes(prob: QPPVMProblem, B: int) -> dict:
    n, T = prob.n, prob.ntasks
    return {
        "M": (B, n, n),
        "J": (B, T, 6, n),
        "pose": (B, T, 12),
        "pose_ref": (B, T, 12),
        "q": (B, n),
        "qd": (B, n),
        "qref": (B, n),
        "h": (B, n),
    }


def check_inputs(prob: QPPVMProblem, inputs: dict) -> int:
    """Validate shapes/dtypes of a batch; returns B. Raises ValueError like the C ABI."""
    B = int(np.asarray(inputs["h"]).shape[0])
    for k, shp in input_shapes(prob, B).items():
        a = inputs[k]
        if tuple(a.shape) != shp:
            raise ValueError(f"input {k}: expected shape {shp}, got {tuple(a.shape)}")
        if a.dtype != np.float64:
            raise ValueError(f"input {k}: expected float64, got {a.dtype}")
    return B


# ------------------------------------------------------------------ contact form (ForceAcc)
@dataclass
class ContactProblem:
    """Batch-shared structure of the ForceAcc contact-form stack (reference
    ``src/ForceAcc.cpp``):

    * variables ``x = [qdd (n); f_c (3) per contact]`` (``:58-72``), wrench ``[f; 0_3]`` (``:81``);
    * level 0 = waist (pelvis) acceleration task (``:118-122``);
    * level 1 = postural + feet acceleration tasks (``:83-89``, ``:105-107``, ``:131``)
      + ``eps_f ||f||^2``, the explicit minimum-norm tie-break on the contact forces;
    * both levels: DynamicFeasibility on the ``n_fb`` floating-base rows (``:109-114``),
      force box ``f_lb <= f <= f_ub`` (``:74-76``), zero force for inactive contacts,
      and (``torque_rows``, row a12, an extension) actuated torque limits;
    * ``tau = M qdd + h - sum_c J_c^T [f_c; 0]`` (``:206-218``).

    SURVEY.md 8f-2 options (defaults = the reference's stack): ``wrench_dim = 6`` makes every
    contact variable the full wrench ``w_c = [f_c; m_c]`` ("put 6 for full wrench", ``:67``) with
    the reference's 6-D box ``[f_lb, m_lb] <= w_c <= [f_ub, m_ub]`` (``:74-76``: moments +-1) and
    ``J_c^T w_c`` over all six Jacobian rows; ``mu > 0`` adds the linearised friction pyramid
    ``|f_x| <= mu f_z, |f_y| <= mu f_z`` (world frame, four rows per active contact; the reference
    has no cone).

    The acceleration-task gains are OpenSoT defaults upstream (not in the reference); here
    they are named options (critically damped unit stiffness by default).
    """

    n: int
    nc: int = 2
    n_fb: int = 6
    Kp_w: float = 1.0
    Kd_w: float = 2.0
    Kp_f: float = 1.0
    Kd_f: float = 2.0
    Kp_p: float = 1.0
    Kd_p: float = 2.0
    f_lb: tuple = (-1000.0, -1000.0, 10.0)
    f_ub: tuple = (1000.0, 1000.0, 1000.0)
    eps_f: float = 1e-8
    wrench_dim: int = 3
    m_lb: tuple = (-1.0, -1.0, -1.0)
    m_ub: tuple = (1.0, 1.0, 1.0)
    mu: float = 0.0
    torque_rows: bool = False
    tau_max: np.ndarray | float = 150.0
    tau_min: np.ndarray | float | None = None
    max_iter: int = 0  # 0 = default cap

    def __post_init__(self):
        n, nc = int(self.n), int(self.nc)
        if not (1 <= nc <= 4):
            raise ValueError("nc must be in [1, 4]")
        if self.n_fb != 6 or n <= self.n_fb:
            raise ValueError("the contact form needs a 6-DoF floating base and n > 6")
        if int(self.wrench_dim) not in (3, 6):
            raise ValueError("wrench_dim must be 3 or 6")
        self.wrench_dim = int(self.wrench_dim)
        if n + self.wrench_dim * nc > 64:
            raise ValueError("n + wrench_dim * nc must be <= 64 (one instance per wavefront)")
        if not self.eps_f > 0:
            raise ValueError("eps_f must be > 0")
        if not self.mu >= 0:
            raise ValueError("mu must be >= 0")
        self.n, self.nc, self.mu = n, nc, float(self.mu)
        self.f_lb = tuple(float(v) for v in self.f_lb)
        self.f_ub = tuple(float(v) for v in self.f_ub)
        self.m_lb = tuple(float(v) for v in self.m_lb)
        self.m_ub = tuple(float(v) for v in self.m_ub)
        self.tau_max = _vec(self.tau_max, n, "tau_max")
        self.tau_min = -self.tau_max if self.tau_min is None else _vec(self.tau_min, n, "tau_min")

    @property
    def nx(self) -> int:
        return self.n + self.wrench_dim * self.nc

    @property
    def w_lb(self) -> tuple:
        """Box of one active contact's variables (3 forces, or the 6-D wrench)."""
        return self.f_lb + (self.m_lb if self.wrench_dim == 6 else ())

    @property
    def w_ub(self) -> tuple:
        return self.f_ub + (self.m_ub if self.wrench_dim == 6 else ())


CONTACT_INPUT_FIELDS = ("M", "h", "q", "qd", "qref", "Jw", "jdqd_w", "pose_w", "pose_w_ref",
                        "Jc", "jdqd_c", "pose_c", "pose_c_ref", "cmask")


def contact_input_shapes(prob: ContactProblem, B: int) -> dict:
    n, nc = prob.n, prob.nc
    return {"M": (B, n, n), "h": (B, n), "q": (B, n), "qd": (B, n), "qref": (B, n),
            "Jw": (B, 6, n), "jdqd_w": (B, 6), "pose_w": (B, 12), "pose_w_ref": (B, 12),
            "Jc": (B, nc, 6, n), "jdqd_c": (B, nc, 6), "pose_c": (B, nc, 12), "pose_c_ref": (B, nc, 12),
            "cmask": (B,)}


def check_contact_inputs(prob: ContactProblem, inputs: dict) -> int:
    B = int(np.asarray(inputs["h"]).shape[0])
    for k, shp in contact_input_shapes(prob, B).items():
        a = inputs[k]
        if tuple(a.shape) != shp:
            raise ValueError(f"input {k}: expected shape {shp}, got {tuple(a.shape)}")
        want = np.int32 if k == "cmask" else np.float64
        if a.dtype != want:
            raise ValueError(f"input {k}: expected {np.dtype(want).name}, got {a.dtype}")
    return B
