"""Synthetic randomized robot states (no URDF/checkpoints in the container).

* M = Q diag(lam) Q^T, Q Haar-orthogonal, lam log-uniform in [1e-2, 1e1]  (cond 1e3)
* J ~ N(0, 0.5^2) per task (6 x n)
* q, q_ref ~ U(-pi, pi), qd ~ N(0, 1), h ~ N(0, 10^2)
* poses: R Haar, p ~ U(-1, 1); reference = pose perturbed by N(0, 0.05^2) in
  position and by a rotation vector ~ N(0, 0.05^2)
Counter-based RNG (numpy Philox) keyed by ``seed``; ``offset`` skips instances so a
shard on rank r reproduces exactly the rows [offset, offset+B) of the global batch.
"""
from __future__ import annotations

import numpy as np

from .problem import QPPVMProblem


def _rng(seed: int, stream: int) -> np.random.Generator:
    return np.random.Generator(np.random.Philox(key=[int(seed) & 0xFFFFFFFFFFFFFFFF, int(stream)]))


def _haar(rng, B, n):
    Z = rng.standard_normal((B, n, n))
    Q, R = np.linalg.qr(Z)
    d = np.sign(np.diagonal(R, axis1=1, axis2=2))
    d[d == 0] = 1.0
    return Q * d[:, None, :]


def _rotvec_to_R(w):
    th = np.linalg.norm(w, axis=-1, keepdims=True)
    k = np.where(th > 0, w / np.where(th > 0, th, 1.0), 0.0)
    K = np.zeros(w.shape[:-1] + (3, 3))
    K[..., 0, 1], K[..., 0, 2] = -k[..., 2], k[..., 1]
    K[..., 1, 0], K[..., 1, 2] = k[..., 2], -k[..., 0]
    K[..., 2, 0], K[..., 2, 1] = -k[..., 1], k[..., 0]
    s, c = np.sin(th)[..., None], np.cos(th)[..., None]
    eye = np.broadcast_to(np.eye(3), K.shape)
    return eye + s * K + (1 - c) * (K @ K)


def _pose(R, p):
    out = np.zeros(R.shape[:-2] + (3, 4))
    out[..., :3] = R
    out[..., 3] = p
    return out.reshape(R.shape[:-2] + (12,))


# The physically scaled variant (``plant=True``): M eigenvalues in [0.5, 5] and Jacobian entries
# N(0, 0.2^2), i.e. lever arms of ~0.2 m and an operational-space inverse inertia J M^-1 J^T of
# O(1). The SURVEY distribution (J ~ N(0, 0.5^2), lambda(M) down to 1e-2) puts dt * Dc *
# lambda_max(J M^-1 J^T) at ~10-100 for the reference gains (Dc = 70) at 1 kHz: explicit Euler
# rollouts of it diverge within a few steps (config 4); the plant variant keeps it below 2.
PLANT_LAM_LO, PLANT_COND, PLANT_JSCALE = 0.5, 10.0, 0.2


def qppvm_instances(prob: QPPVMProblem, B: int, seed: int = 0, offset: int = 0,
                    cond_max: float = 1e3, plant: bool = False) -> dict:
    """B independent random instances (rows [offset, offset+B) of stream ``seed``)."""
    lam_lo, jscale = (PLANT_LAM_LO, PLANT_JSCALE) if plant else (1e-2, 0.5)
    if plant:
        cond_max = PLANT_COND
    n, T = prob.n, prob.ntasks
    out = {k: [] for k in ("M", "J", "pose", "pose_ref", "q", "qd", "qref", "h")}
    # generate in chunks keyed by absolute chunk index so offsets are reproducible
    CH = 256
    first, last = offset // CH, (offset + B - 1) // CH if B > 0 else -1
    for c in range(first, last + 1):
        rng = _rng(seed, c)
        Q = _haar(rng, CH, n)
        lam = np.exp(rng.uniform(np.log(lam_lo), np.log(lam_lo * cond_max), (CH, n)))
        M = (Q * lam[:, None, :]) @ Q.transpose(0, 2, 1)
        M = 0.5 * (M + M.transpose(0, 2, 1))
        J = rng.normal(0.0, jscale, (CH, T, 6, n))
        R = _haar(rng, CH * T, 3).reshape(CH, T, 3, 3)
        det = np.linalg.det(R)
        R[det < 0, :, 0] *= -1.0
        p = rng.uniform(-1.0, 1.0, (CH, T, 3))
        Rref = _rotvec_to_R(rng.normal(0.0, 0.05, (CH, T, 3))) @ R
        pref = p + rng.normal(0.0, 0.05, (CH, T, 3))
        q = rng.uniform(-np.pi, np.pi, (CH, n))
        qref = rng.uniform(-np.pi, np.pi, (CH, n))
        qd = rng.normal(0.0, 1.0, (CH, n))
        h = rng.normal(0.0, 10.0, (CH, n))
        lo = max(offset, c * CH) - c * CH
        hi = min(offset + B, (c + 1) * CH) - c * CH
        for k, v in (("M", M), ("J", J), ("pose", _pose(R, p)), ("pose_ref", _pose(Rref, pref)),
                     ("q", q), ("qd", qd), ("qref", qref), ("h", h)):
            out[k].append(v[lo:hi])
    return {k: np.ascontiguousarray(np.concatenate(v, axis=0)) if v else
            np.zeros((0,)) for k, v in out.items()}


def replicate(inputs: dict, B: int) -> dict:
    """Config 1: B identical copies of instance 0."""
    return {k: np.ascontiguousarray(np.broadcast_to(v[:1], (B,) + v.shape[1:])) for k, v in inputs.items()}


def contact_instances(prob, B: int, seed: int = 0, offset: int = 0, masks=None, cond_max: float = 1e3) -> dict:
    """Synthetic floating-base states for the contact form. Per instance:
    M as in qppvm_instances; h ~ N(0, 10^2) with the floating-base rows carrying a
    weight-like +z component; waist Jacobian = [R_w-blocks | 0] (the base link moves with
    the floating base only); feet Jacobians ~ N(0, 0.5^2); Jdot qd ~ N(0, 1); poses Haar,
    references perturbed; ``masks``: None = all contacts active, else a list of allowed
    contact masks drawn uniformly per instance (config 2: 2, 3 or 4 feet)."""
    n, nc = prob.n, prob.nc
    out = {k: [] for k in ("M", "h", "q", "qd", "qref", "Jw", "jdqd_w", "pose_w", "pose_w_ref",
                           "Jc", "jdqd_c", "pose_c", "pose_c_ref", "cmask")}
    CH = 256
    first, last = offset // CH, (offset + B - 1) // CH if B > 0 else -1
    for c in range(first, last + 1):
        rng = _rng(seed, (1 << 20) + c)
        Q = _haar(rng, CH, n)
        lam = np.exp(rng.uniform(np.log(1e-2), np.log(1e-2 * cond_max), (CH, n)))
        M = (Q * lam[:, None, :]) @ Q.transpose(0, 2, 1)
        M = 0.5 * (M + M.transpose(0, 2, 1))
        h = rng.normal(0.0, 10.0, (CH, n))
        h[:, 2] += 50.0  # gravity on the base z row: the feet push up (f_z >= 10)
        R = _haar(rng, CH * (1 + nc), 3).reshape(CH, 1 + nc, 3, 3)
        det = np.linalg.det(R)
        R[det < 0, :, 0] *= -1.0
        Jw = np.zeros((CH, 6, n))
        Jw[:, :3, :3] = R[:, 0]
        Jw[:, 3:, 3:6] = R[:, 0]
        Jw[:, :3, 3:6] = rng.normal(0.0, 0.2, (CH, 3, 3))
        Jc = rng.normal(0.0, 0.5, (CH, nc, 6, n))
        p = rng.uniform(-1.0, 1.0, (CH, 1 + nc, 3))
        Rref = _rotvec_to_R(rng.normal(0.0, 0.05, (CH, 1 + nc, 3))) @ R
        pref = p + rng.normal(0.0, 0.05, (CH, 1 + nc, 3))
        poses, poses_ref = _pose(R, p), _pose(Rref, pref)
        q = rng.uniform(-np.pi, np.pi, (CH, n))
        qref = q + rng.normal(0.0, 0.1, (CH, n))
        qd = rng.normal(0.0, 1.0, (CH, n))
        jw = rng.normal(0.0, 1.0, (CH, 6))
        jc = rng.normal(0.0, 1.0, (CH, nc, 6))
        if masks is None:
            cm = np.full(CH, (1 << nc) - 1, dtype=np.int32)
        else:
            cm = np.asarray(masks, dtype=np.int32)[rng.integers(0, len(masks), CH)]
        lo = max(offset, c * CH) - c * CH
        hi = min(offset + B, (c + 1) * CH) - c * CH
        for k, v in (("M", M), ("h", h), ("q", q), ("qd", qd), ("qref", qref), ("Jw", Jw), ("jdqd_w", jw),
                     ("pose_w", poses[:, 0]), ("pose_w_ref", poses_ref[:, 0]), ("Jc", Jc), ("jdqd_c", jc),
                     ("pose_c", poses[:, 1:]), ("pose_c_ref", poses_ref[:, 1:]), ("cmask", cm)):
            out[k].append(v[lo:hi])
    return {k: np.ascontiguousarray(np.concatenate(v, axis=0)) for k, v in out.items()}
