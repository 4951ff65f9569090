"""Build libwbq.so (HIP, gfx950) in-tree with hipcc. No JIT cache, no pip install:
the .so lives next to this file so it travels to the GPU box with the repo snapshot."""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libwbq.so")
SOURCES = ["wbq_api.hip", "qppvm_kernel.hip", "qppvm_w1m_kernel.hip", "contact_kernel.hip"]
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
    cmd = ["hipcc", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-Wall", "-Wno-unused-function", "-munsafe-fp-atomics",
           "-I", os.path.join(ROOT, "include"),
           *(["-DWBQ_STAMPS"] if diag else []), *[f"-D{d}" for d in defines],
           *[os.path.join(CSRC, s) for s in SOURCES], "-o", lib + ".tmp"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd)
    os.replace(lib + ".tmp", lib)
    return lib


PLUGIN_DIR = os.path.join(HERE, "plugins")
PLUGIN_LIB = os.path.join(HERE, "libQPPVMPlugin.so")
FORCEACC_LIB = os.path.join(HERE, "libForceAccPlugin.so")
DRIVER = os.path.join(HERE, "qppvm_dummy_driver")


def build_plugins(verbose: bool = False) -> tuple:
    """The XBot plugin shells (libQPPVMPlugin.so and libForceAccPlugin.so, the reference's
    target names, CMakeLists.txt:48-49) and the config-0 dummy-mode driver, host C++ over
    libwbq.so."""
    build()
    inc = ["-I", os.path.join(ROOT, "include"), "-I", os.path.join(PLUGIN_DIR, "compat"),
           "-I", os.path.join(PLUGIN_DIR, "include"), "-I", os.path.join(PLUGIN_DIR, "src")]
    link = ["-L", HERE, "-lwbq", "-Wl,-rpath,$ORIGIN", "-Wl,-rpath,/opt/rocm/lib"]
    src = os.path.join(PLUGIN_DIR, "src", "QPPVMPlugin.cpp")
    fsrc = os.path.join(PLUGIN_DIR, "src", "ForceAcc.cpp")
    cmds = [
        ["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", *inc, src, "-o", PLUGIN_LIB, *link],
        ["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", *inc, fsrc, "-o", FORCEACC_LIB, *link],
        ["g++", "-O2", "-std=c++17", "-Wall", *inc, os.path.join(PLUGIN_DIR, "src", "dummy_driver.cpp"), src, fsrc,
         "-o", DRIVER, *link],
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
