import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")
INPUT_KEYS = ("M", "J", "pose", "pose_ref", "q", "qd", "qref", "h")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")


def load_golden(n):
    """Yield (group, QPPVMProblem, inputs, expected dict) from tests/golden/qppvm_n{n}.npz."""
    from qppvm_amd.problem import QPPVMProblem
    z = np.load(os.path.join(GOLDEN, f"qppvm_n{n}.npz"))
    for g in z["groups"]:
        g = str(g)
        pre = g + "__"
        prob = QPPVMProblem(n=n, tau_max=z[pre + "tau_max"],
                            select_mode=int(z[pre + "select_mode"]),
                            joint_weight=int(z[pre + "joint_weight"]),
                            row_mask=tuple(int(m) for m in z[pre + "row_mask"]))
        inp = {k: np.ascontiguousarray(z[pre + k]) for k in INPUT_KEYS}
        exp = {k: z[pre + k] for k in ("tau", "y0", "status", "kat") if pre + k in z}
        yield g, prob, inp, exp


def rel_err(a, b):
    """max_i ||a_i - b_i||_inf / max(1, ||b_i||_inf) over a batch."""
    a = np.atleast_2d(a)
    b = np.atleast_2d(b)
    return float((np.abs(a - b).max(axis=1) / np.maximum(1.0, np.abs(b).max(axis=1))).max())


@pytest.fixture(scope="session")
def oracle_lib():
    import oracle
    oracle.build()
    return oracle


def load_golden_contact(n, fname=None):
    """Yield (group, ContactProblem, inputs, expected) from tests/golden/contact_n{n}.npz (or
    fname: contact_ext_n30.npz holds the SURVEY 8f-2 groups, 6-D wrenches and friction rows)."""
    from qppvm_amd.problem import ContactProblem, CONTACT_INPUT_FIELDS
    z = np.load(os.path.join(GOLDEN, fname or f"contact_n{n}.npz"))
    for g in z["groups"]:
        g = str(g)
        pre = g + "__"
        ext = {k: (int(z[pre + k]) if k == "wrench_dim" else float(z[pre + k]))
               for k in ("wrench_dim", "mu") if pre + k in z}
        prob = ContactProblem(n=n, nc=int(z[pre + "nc"]), torque_rows=bool(z[pre + "torque_rows"]),
                              tau_max=z[pre + "tau_max"], **ext)
        inp = {k: np.ascontiguousarray(z[pre + k]) for k in CONTACT_INPUT_FIELDS}
        yield g, prob, inp, {"tau": z[pre + "tau"], "x": z[pre + "x"]}


def load_golden_elbow(literal=False):
    """Yield (group, QPPVMProblem, inputs, expected) of the elbow-stack fixtures (make_golden_elbow.py):
    task_level (0, 0, 1, 1) with the elbow tasks of QPPVMPlugin.cpp:154-166. literal: the reference's
    commented stack ((ee_r + ee_l) / (elbow_l + elbow_r)) << limits, no joint task (:177-178 in place
    of :179; tests/golden/qppvm_elbow_literal.npz); else the three-level extension with the joint task
    (tests/golden/qppvm_elbow.npz)."""
    from qppvm_amd.problem import QPPVMProblem
    z = np.load(os.path.join(GOLDEN, "qppvm_elbow_literal.npz" if literal else "qppvm_elbow.npz"))
    for g in z["groups"]:
        g = str(g)
        pre = g + "__"
        prob = QPPVMProblem(n=int(z[pre + "n"]), ntasks=4, row_mask=(7, 7, 7, 7), task_level=(0, 0, 1, 1),
                            tau_max=z[pre + "tau_max"], joint_task=not literal)
        inp = {k: np.ascontiguousarray(z[pre + k]) for k in INPUT_KEYS}
        exp = {k: z[pre + k] for k in ("tau", "y", "kat") if pre + k in z}
        yield g, prob, inp, exp
