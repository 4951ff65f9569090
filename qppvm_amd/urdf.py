"""URDF reader for the on-GPU rigid-body model: a URDF file -> ``RobotModel``
(``wbq_rbd_desc``), the model the reference's plugins load through XBotInterface
(``ModelInterface::getModel(path)``, QPPVMPlugin.cpp:50-51 / ForceAcc.cpp:43; RBDL backend
[upstream]).

Supported: ``revolute``, ``continuous`` and ``prismatic`` joints (one degree of freedom each, in
depth-first order from the root link, children in file order), ``fixed`` joints (the child link's
inertia is lumped into the body that carries it, and its frame stays addressable as a task frame
with a fixed offset), ``<inertial>`` with origin xyz/rpy, ``<limit effort lower upper>``.
``floating_base=True`` puts the root link on six virtual joints (``rbd.with_floating_base``: the
ForceAcc contact form's ``n_fb = 6`` first coordinates); otherwise the root link is the fixed
world. ``floating`` / ``planar`` joints below the root and closed loops are rejected.

Conventions (URDF): a joint's child link frame is the joint frame, ``origin`` = parent link frame
-> joint frame (xyz, then fixed-axis roll-pitch-yaw), ``axis`` in the joint frame.
"""
from __future__ import annotations

import xml.etree.ElementTree as ET
from dataclasses import dataclass, field

import numpy as np

from .rbd import PRISMATIC, REVOLUTE, RobotModel, with_floating_base


def rpy_matrix(rpy) -> np.ndarray:
    """URDF rotation: R = Rz(yaw) Ry(pitch) Rx(roll)."""
    r, p, y = (float(v) for v in rpy)
    cr, sr, cp, sp, cy, sy = np.cos(r), np.sin(r), np.cos(p), np.sin(p), np.cos(y), np.sin(y)
    Rx = np.array([[1, 0, 0], [0, cr, -sr], [0, sr, cr]])
    Ry = np.array([[cp, 0, sp], [0, 1, 0], [-sp, 0, cp]])
    Rz = np.array([[cy, -sy, 0], [sy, cy, 0], [0, 0, 1]])
    return Rz @ Ry @ Rx


def _vec(s, default):
    return np.array([float(v) for v in s.split()]) if s is not None else np.array(default, dtype=float)


def _origin(el) -> np.ndarray:
    """4x4 homogeneous transform of an <origin> element (identity when absent)."""
    T = np.eye(4)
    o = el.find("origin") if el is not None else None
    if o is not None:
        T[:3, :3] = rpy_matrix(_vec(o.get("rpy"), (0, 0, 0)))
        T[:3, 3] = _vec(o.get("xyz"), (0, 0, 0))
    return T


@dataclass
class _Body:
    """Rigid body of one degree of freedom (or the root): its mass properties in its frame."""
    mass: float = 0.0
    com: np.ndarray = field(default_factory=lambda: np.zeros(3))
    inertia: np.ndarray = field(default_factory=lambda: np.zeros((3, 3)))  # about the COM

    def add(self, m, c, I):
        """Lump a body of mass m, COM c and inertia I (about c, this frame) into this one."""
        if m <= 0.0:
            return
        M = self.mass + m
        cn = (self.mass * self.com + m * c) / M

        def shift(mm, cc, II):
            d = cc - cn
            return II + mm * (np.dot(d, d) * np.eye(3) - np.outer(d, d))
        self.inertia = shift(self.mass, self.com, self.inertia) + shift(m, c, I)
        self.mass, self.com = M, cn


@dataclass
class UrdfRobot:
    """What the URDF yields: the model, joint names in dof order, effort and position limits, and
    every link's (dof body, offset) so any link frame can become a task frame."""
    model: RobotModel
    joint_names: list
    effort: np.ndarray
    q_min: np.ndarray
    q_max: np.ndarray
    frames: dict  # link name -> (body index or -1 for the root, 4x4 offset in that body's frame)

    def with_tasks(self, task_links) -> RobotModel:
        """The model with task frames on the named links (their frame origins)."""
        links, offs = [], []
        for name in task_links:
            if name not in self.frames:
                raise KeyError(f"unknown link {name!r}")
            b, T = self.frames[name]
            if b < 0:
                raise ValueError(f"link {name!r} is fixed to the world: no task frame")
            links.append(b)
            offs.append(T[:3, :].reshape(-1))
        m = self.model
        return RobotModel(parent=m.parent, X_fixed=m.X_fixed, axis=m.axis, mass=m.mass, com=m.com,
                          inertia=m.inertia, task_link=np.asarray(links, np.int32), gravity=m.gravity,
                          names=list(m.names), jtype=m.jtype, task_offset=np.asarray(offs, dtype=float),
                          task_names=list(task_links))


def load_urdf(path_or_text: str, task_links=(), floating_base: bool = False, gravity=(0.0, 0.0, -9.81)) -> UrdfRobot:
    """Parse a URDF file (or its text) into a ``UrdfRobot``; ``task_links`` become the model's task
    frames (their order is the task order)."""
    text = path_or_text
    if not path_or_text.lstrip().startswith("<"):
        with open(path_or_text) as f:
            text = f.read()
    root_el = ET.fromstring(text)
    if root_el.tag != "robot":
        raise ValueError("not a URDF <robot>")
    links = {}
    for l in root_el.findall("link"):
        inert = l.find("inertial")
        m, c, I = 0.0, np.zeros(3), np.zeros((3, 3))
        if inert is not None:
            T = _origin(inert)
            m = float(inert.find("mass").get("value"))
            ie = inert.find("inertia")
            g = {k: float(ie.get(k, 0.0)) for k in ("ixx", "iyy", "izz", "ixy", "ixz", "iyz")}
            Il = np.array([[g["ixx"], g["ixy"], g["ixz"]], [g["ixy"], g["iyy"], g["iyz"]], [g["ixz"], g["iyz"], g["izz"]]])
            I = T[:3, :3] @ Il @ T[:3, :3].T
            c = T[:3, 3]
        links[l.get("name")] = (m, c, I)
    children, child_of = {}, {}
    for j in root_el.findall("joint"):
        par, ch = j.find("parent").get("link"), j.find("child").get("link")
        if ch in child_of:
            raise ValueError(f"link {ch!r} has two parent joints (closed loop)")
        child_of[ch] = j
        children.setdefault(par, []).append(j)
    roots = [name for name in links if name not in child_of]
    if len(roots) != 1:
        raise ValueError(f"expected one root link, found {roots}")
    root = roots[0]

    bodies = [_Body()]  # index 0 = the root body (fixed world or the floating base)
    parent, X, axis, jtype, names, effort, qmin, qmax = [], [], [], [], [], [], [], []
    frames = {}

    def visit(link, body, T_in_body):
        """link's frame is T_in_body in body `body` (index into bodies; 0 = root)."""
        frames[link] = (body, T_in_body)
        m, c, I = links[link]
        R = T_in_body[:3, :3]
        bodies[body].add(m, R @ c + T_in_body[:3, 3], R @ I @ R.T)
        for j in children.get(link, []):
            typ = j.get("type")
            ch = j.find("child").get("link")
            Tj = T_in_body @ _origin(j)
            if typ == "fixed":
                visit(ch, body, Tj)
                continue
            if typ not in ("revolute", "continuous", "prismatic"):
                raise ValueError(f"joint {j.get('name')!r}: type {typ!r} not supported")
            a = _vec(j.find("axis").get("xyz") if j.find("axis") is not None else None, (1, 0, 0))
            a = a / np.linalg.norm(a)
            lim = j.find("limit")
            dof = len(parent)
            parent.append(body - 1)  # dof index of the carrying body (-1: the root)
            X.append(Tj[:3, :].reshape(-1))
            axis.append(a)
            jtype.append(PRISMATIC if typ == "prismatic" else REVOLUTE)
            names.append(j.get("name"))
            effort.append(float(lim.get("effort", np.inf)) if lim is not None else np.inf)
            cont = typ == "continuous" or lim is None
            qmin.append(-np.inf if cont else float(lim.get("lower", -np.inf)))
            qmax.append(np.inf if cont else float(lim.get("upper", np.inf)))
            bodies.append(_Body())
            assert len(bodies) - 2 == dof
            visit(ch, dof + 1, np.eye(4))

    visit(root, 0, np.eye(4))
    n = len(parent)
    mass = np.array([b.mass for b in bodies[1:]])
    com = np.array([b.com for b in bodies[1:]]).reshape(n, 3)
    inertia = np.array([[b.inertia[0, 0], b.inertia[1, 1], b.inertia[2, 2], b.inertia[0, 1], b.inertia[0, 2],
                         b.inertia[1, 2]] for b in bodies[1:]]).reshape(n, 6)
    model = RobotModel(parent=np.asarray(parent, np.int32), X_fixed=np.asarray(X, dtype=float).reshape(n, 12),
                       axis=np.asarray(axis, dtype=float).reshape(n, 3), mass=mass, com=com, inertia=inertia,
                       task_link=np.zeros(0, np.int32), gravity=tuple(gravity), names=names,
                       jtype=np.asarray(jtype, np.int32))
    frames = {k: (b - 1, T) for k, (b, T) in frames.items()}  # body -> dof index (root -> -1)
    effort, qmin, qmax = np.array(effort), np.array(qmin), np.array(qmax)
    if floating_base:
        b0 = bodies[0]
        I0 = b0.inertia
        model = with_floating_base(model, base_mass=b0.mass, base_com=b0.com,
                                   base_inertia=(I0[0, 0], I0[1, 1], I0[2, 2], I0[0, 1], I0[0, 2], I0[1, 2]))
        frames = {k: (b + 6 if b >= 0 else 5, T) for k, (b, T) in frames.items()}  # the root rides joint 5
        effort = np.concatenate([np.zeros(6), effort])  # unactuated virtual joints (tau limit 0)
        qmin = np.concatenate([np.full(6, -np.inf), qmin])
        qmax = np.concatenate([np.full(6, np.inf), qmax])
    ur = UrdfRobot(model=model, joint_names=list(model.names), effort=effort, q_min=qmin, q_max=qmax, frames=frames)
    if task_links:
        ur.model = ur.with_tasks(task_links)
    return ur
