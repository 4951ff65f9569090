"""C-ABI checks that need no GPU: the library builds for gfx950, loads, exports every
symbol include/wbq.h declares, and its struct layouts match the ctypes mirror."""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import ROOT
from qppvm_amd import build as wbq_build
from qppvm_amd import wbq

HEADER = os.path.join(ROOT, "include", "wbq.h")


def declared_symbols():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\**\s*(wbq_\w+)\s*\(", src, re.M)))


@pytest.fixture(scope="module")
def lib():
    wbq_build.build()
    return wbq.load_library()


def test_header_declares_expected_api():
    assert declared_symbols() == sorted(wbq.EXPORTS)


def test_library_exports_every_declared_symbol(lib):
    for name in declared_symbols():
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", wbq.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    for name in declared_symbols():
        assert re.search(rf"\bT {name}$", out, re.M), name


def test_code_object_is_gfx950(lib, tmp_path):
    # --offloading extracts the bundled code objects next to its input: work on a copy
    import shutil
    copy = str(tmp_path / "libwbq.so")
    shutil.copy(wbq.LIB_PATH, copy)
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", copy],
                         capture_output=True, text=True, cwd=str(tmp_path))
    if out.returncode != 0:
        pytest.skip("llvm-objdump --offloading unavailable")
    assert "gfx950" in out.stdout + out.stderr


def test_struct_layout_matches_c(tmp_path):
    prog = tmp_path / "sz.c"
    prog.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "wbq.h"\n'
                    'int main(void){printf("%zu %zu %zu %zu\\n", sizeof(wbq_desc), '
                    'offsetof(wbq_desc, Kc), sizeof(wbq_inputs), offsetof(wbq_inputs, h));return 0;}\n')
    exe = tmp_path / "sz"
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), str(prog), "-o", str(exe)])
    got = [int(x) for x in subprocess.check_output([str(exe)]).split()]
    assert got == [ctypes.sizeof(wbq.Desc), wbq.Desc.Kc.offset, ctypes.sizeof(wbq.Inputs),
                   wbq.Inputs.h.offset]


def test_version_string(lib):
    assert lib.wbq_version().decode().startswith("wbq ")


def test_null_arguments_rejected(lib):
    h = ctypes.c_void_p()
    assert lib.wbq_create(None, 0, ctypes.byref(h)) == wbq.E_INVALID
    assert lib.wbq_solve(None) == wbq.E_INVALID
    assert lib.wbq_sync(None) == wbq.E_INVALID
    assert lib.wbq_last_error(None) == b"null context"
    lib.wbq_destroy(None)


def test_unsupported_problem_rejected_before_device(lib):
    d = wbq.Desc()
    d.form, d.n, d.ntasks, d.max_batch = 7, 30, 2, 4  # unknown form
    h = ctypes.c_void_p()
    assert lib.wbq_create(ctypes.byref(d), 0, ctypes.byref(h)) == wbq.E_UNSUPPORTED
    d.form, d.n = wbq.FORM_QPPVM, 65  # n too large
    assert lib.wbq_create(ctypes.byref(d), 0, ctypes.byref(h)) == wbq.E_INVALID


def test_plugin_shells_export_factories():
    """libQPPVMPlugin.so / libForceAccPlugin.so (the reference's target names,
    CMakeLists.txt:48-49) build with g++ against the compat XCM header and export the
    REGISTER_XBOT_PLUGIN factory symbols XBotCore dlopens."""
    plugin, driver, forceacc = wbq_build.build_plugins()
    # REGISTER_XBOT_PLUGIN(QPPVMPlugin, ..) (QPPVMPlugin.cpp:29) names its factory pair;
    # REGISTER_XBOT_PLUGIN_(XBotPlugin::ForceAccExample) (ForceAcc.cpp:26) emits the fixed pair
    for lib, syms in ((plugin, ("create_instance_QPPVMPlugin", "destroy_instance_QPPVMPlugin")),
                      (forceacc, ("create_instance", "destroy_instance"))):
        out = subprocess.run(["nm", "-D", "--defined-only", lib], capture_output=True, text=True, check=True).stdout
        for sym in syms:
            assert re.search(rf"\bT {sym}$", out, re.M), (lib, sym)
    assert os.access(driver, os.X_OK)


def test_w1m_capacity_rejected_before_device(lib):
    """W1 = M runs one lane per level-0 row and torque limit: m0 + n > 64 is refused (before
    any device call, so this runs without a GPU); an unknown weight is invalid."""
    import numpy as np
    d = wbq.Desc()
    d.form, d.n, d.ntasks, d.max_batch = wbq.FORM_QPPVM, 60, 2, 4
    d.row_mask[0] = d.row_mask[1] = 0x3F  # m0 = 12
    d.select_mode, d.joint_weight = 0, 1
    keep = [np.ones(12), np.ones(12), np.ones(60), np.ones(60), np.full(60, 1.0), np.full(60, -1.0)]
    d.Kc, d.Dc, d.Kq, d.Dq, d.tau_max, d.tau_min = [a.ctypes.data for a in keep]
    h = ctypes.c_void_p()
    assert lib.wbq_create(ctypes.byref(d), 0, ctypes.byref(h)) == wbq.E_UNSUPPORTED
    d.joint_weight = 2
    assert lib.wbq_create(ctypes.byref(d), 0, ctypes.byref(h)) == wbq.E_INVALID


def test_rbd_model_validated_before_device(lib):
    """wbq_rbd_create rejects a model that is not a topologically ordered tree of unit joint
    axes, or task links outside it, before any device call (CPU)."""
    import numpy as np
    from qppvm_amd.rbd import _Desc, centauro_like

    m = centauro_like()

    def create(parent=None, axis=None, task_link=None, n=None):
        keep = {k: np.ascontiguousarray(getattr(m, k), dtype=np.int32 if k in ("parent", "task_link") else np.float64)
                for k in ("parent", "X_fixed", "axis", "mass", "com", "inertia", "task_link")}
        if parent is not None:
            keep["parent"] = np.ascontiguousarray(parent, dtype=np.int32)
        if axis is not None:
            keep["axis"] = np.ascontiguousarray(axis, dtype=np.float64)
        if task_link is not None:
            keep["task_link"] = np.ascontiguousarray(task_link, dtype=np.int32)
        d = _Desc()
        d.n = m.n if n is None else n
        for k, v in keep.items():
            setattr(d, k, v.ctypes.data)
        d.ntasks, d.max_batch = len(keep["task_link"]), 4
        h = ctypes.c_void_p()
        return lib.wbq_rbd_create(ctypes.byref(d), 0, ctypes.byref(h))

    bad_parent = m.parent.copy()
    bad_parent[3] = 5  # a parent after its child
    assert create(parent=bad_parent) == wbq.E_INVALID
    bad_axis = m.axis.copy()
    bad_axis[2] *= 2.0  # not unit
    assert create(axis=bad_axis) == wbq.E_INVALID
    assert create(task_link=[m.n]) == wbq.E_INVALID
    assert create(n=65) == wbq.E_INVALID


def test_plant_states_are_euler_stable():
    """Config 4's plant-scaled synthetic states keep dt * Dc * lambda_max(G M^-1 G^T) below 2 at
    the reference gains, the SURVEY distribution does not (bench.py euler_stability)."""
    import sys

    sys.path.insert(0, ROOT)
    import bench
    from qppvm_amd.problem import QPPVMProblem
    from qppvm_amd.synth import qppvm_instances
    prob = QPPVMProblem(n=30)
    plant = bench.euler_stability(prob, qppvm_instances(prob, 64, seed=1, plant=True), 1e-3)
    survey = bench.euler_stability(prob, qppvm_instances(prob, 64, seed=1), 1e-3)
    assert plant["max"] < 2.0 < survey["median"]
