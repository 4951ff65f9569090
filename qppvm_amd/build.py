"""Build libwbq.so (HIP, gfx950) in-tree with hipcc. No JIT cache, no pip install:
the .so lives next to this file so it travels to the GPU box with the repo snapshot."""
from __future__ import annotations

import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libwbq.so")
SOURCES = ["wbq_api.hip", "qppvm_kernel.hip", "qppvm_w1m_kernel.hip", "contact_kernel.hip", "rbd.hip"]
HEADERS = ["wbq_kernels.h", "wbq_device.h", "dual_gi.h", "qppvm_repair.h"]
ARCH = os.environ.get("WBQ_ARCH", "gfx950")


def _stale() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, s) for s in SOURCES + HEADERS] + [os.path.join(ROOT, "include", "wbq.h")]
    return any(os.path.getmtime(p) > t for p in deps)


def build(force: bool = False, verbose: bool = False, diag: bool = False, defines: tuple = (),
          out: str | None = None) -> str:
    """diag=True builds libwbq_diag.so with in-kernel phase stamps (never the product);
    defines/out build an experiment variant (scripts/ab_bench.py) at another path."""
    lib = out or (LIB.replace("libwbq.so", "libwbq_diag.so") if diag else LIB)
    if not force and not diag and out is None and not _stale():
        return LIB
    flags = ["hipcc", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
             "-Wall", "-Wno-unused-function", "-munsafe-fp-atomics",
             "-I", os.path.join(ROOT, "include"),
             *(["-DWBQ_STAMPS"] if diag else []), *[f"-D{d}" for d in defines]]
    # one translation unit per process (each holds its own kernels), then one link. Objects are
    # kept per flag set; a source is recompiled only when it or a header it includes is newer
    objdir = os.path.join(HERE, "build", "obj_" + hashlib.md5(" ".join(flags).encode()).hexdigest()[:10])
    os.makedirs(objdir, exist_ok=True)
    objs = [os.path.join(objdir, os.path.splitext(s)[0] + ".o") for s in SOURCES]
    procs = []
    for s, o in zip(SOURCES, objs):
        src = os.path.join(CSRC, s)
        deps = [src] + [os.path.join(CSRC, h) for h in HEADERS] + [os.path.join(ROOT, "include", "wbq.h")]
        if not force or os.environ.get("WBQ_INCREMENTAL"):
            if os.path.exists(o) and all(os.path.getmtime(d) <= os.path.getmtime(o) for d in deps):
                continue
        cmd = flags + ["-c", src, "-o", o]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        procs.append((cmd, subprocess.Popen(cmd)))
    failed = [c for c, p in procs if p.wait() != 0]
    if failed:
        raise subprocess.CalledProcessError(1, failed[0])
    subprocess.check_call(["hipcc", f"--offload-arch={ARCH}", "-shared", *objs, "-o", lib + ".tmp"])
    os.replace(lib + ".tmp", lib)
    return lib


PLUGIN_DIR = os.path.join(HERE, "plugins")
PLUGIN_LIB = os.path.join(HERE, "libQPPVMPlugin.so")
FORCEACC_LIB = os.path.join(HERE, "libForceAccPlugin.so")
DRIVER = os.path.join(HERE, "qppvm_dummy_driver")
# the same driver and shells against a row-major compat MatrixXd (tests/test_plugin.py: the
# torques must not depend on the matrix storage order)
DRIVER_RM = os.path.join(HERE, "qppvm_dummy_driver_rowmajor")


def _plugin_sources():
    out = []
    for d in ("src", "include/QPPVM_RT_plugin", "include/ForceAccPlugin", "compat/XCM", "compat/XBotInterface"):
        base = os.path.join(PLUGIN_DIR, d)
        out += [os.path.join(base, f) for f in os.listdir(base)]
    return out


def build_plugins(verbose: bool = False, force: bool = False) -> tuple:
    """The XBot plugin shells (libQPPVMPlugin.so and libForceAccPlugin.so, the reference's
    target names, CMakeLists.txt:48-49) and the config-0 dummy-mode drivers, host C++ over
    libwbq.so. Skipped when every output is newer than its sources and libwbq.so."""
    lib = build()
    outs = (PLUGIN_LIB, FORCEACC_LIB, DRIVER, DRIVER_RM)
    deps = _plugin_sources() + [lib, os.path.join(ROOT, "include", "wbq.h")]
    if not force and all(os.path.exists(o) for o in outs):
        t = min(os.path.getmtime(o) for o in outs)
        if all(os.path.getmtime(p) <= t for p in deps):
            return PLUGIN_LIB, DRIVER, FORCEACC_LIB
    inc = ["-I", os.path.join(ROOT, "include"), "-I", os.path.join(PLUGIN_DIR, "compat"),
           "-I", os.path.join(PLUGIN_DIR, "include"), "-I", os.path.join(PLUGIN_DIR, "src")]
    link = ["-L", HERE, "-lwbq", "-Wl,-rpath,$ORIGIN", "-Wl,-rpath,/opt/rocm/lib"]
    src = os.path.join(PLUGIN_DIR, "src", "QPPVMPlugin.cpp")
    fsrc = os.path.join(PLUGIN_DIR, "src", "ForceAcc.cpp")
    drv = os.path.join(PLUGIN_DIR, "src", "dummy_driver.cpp")
    cmds = [
        ["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", *inc, src, "-o", PLUGIN_LIB, *link],
        ["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", *inc, fsrc, "-o", FORCEACC_LIB, *link],
        ["g++", "-O2", "-std=c++17", "-Wall", *inc, drv, src, fsrc, "-o", DRIVER, *link],
        ["g++", "-O2", "-std=c++17", "-Wall", "-DXBOT_COMPAT_ROW_MAJOR", *inc, drv, src, fsrc, "-o", DRIVER_RM, *link],
    ]
    for c in cmds:
        if verbose:
            print(" ".join(c), file=sys.stderr)
        subprocess.check_call(c)
    return PLUGIN_LIB, DRIVER, FORCEACC_LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True, diag="--diag" in sys.argv))
    if "--plugins" in sys.argv:
        print(build_plugins(verbose=True))
