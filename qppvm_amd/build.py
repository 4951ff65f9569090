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
ARCH = os.environ.get("WBQ_ARCH", "gfx950")


def _headers(src: str | None = None) -> list:
    """The local headers a translation unit includes, followed recursively through its
    #include "..." lines (src None: every csrc/*.h), and the C ABI header."""
    inc = [os.path.join(ROOT, "include", "wbq.h")]
    if src is None:
        return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")) + inc
    seen, todo = [], [src]
    while todo:
        with open(todo.pop()) as f:
            for line in f:
                line = line.strip()
                if line.startswith("#include \"") or line.startswith("#include <wbq"):
                    name = line.split('"')[1] if '"' in line else line.split("<")[1].split(">")[0]
                    for d in (CSRC, os.path.join(ROOT, "include")):
                        h = os.path.join(d, name)
                        if os.path.exists(h):
                            if h not in seen:
                                seen.append(h)
                                todo.append(h)
                            break
    return sorted(seen)


def _digest(flags: list, paths: list) -> str:
    """Content hash of the compile flags and the files (not their modification times: a copied
    tree with reset timestamps must not relink stale objects)."""
    h = hashlib.sha256(" ".join(flags).encode())
    for p in paths:
        h.update(os.path.basename(p).encode())
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def _stamp(lib: str) -> str:
    return lib + ".srchash"


def _flags(diag: bool = False, defines: tuple = ()) -> list:
    return ["hipcc", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
            "-Wall", "-Wno-unused-function", "-munsafe-fp-atomics",
            "-I", os.path.join(ROOT, "include"),
            *(["-DWBQ_STAMPS"] if diag else []), *[f"-D{d}" for d in defines]]


def _stale() -> bool:
    """The product library is stale when the content hash of its compile flags and sources differs
    from the one recorded beside it at link time (no record: fall back to modification times)."""
    if not os.path.exists(LIB):
        return True
    deps = [os.path.join(CSRC, s) for s in SOURCES] + _headers()
    if os.path.exists(_stamp(LIB)):
        with open(_stamp(LIB)) as f:
            return f.read().strip() != _digest(_flags(), deps)
    t = os.path.getmtime(LIB)
    return any(os.path.getmtime(p) > t for p in deps)


def build(force: bool = False, verbose: bool = False, diag: bool = False, defines: tuple = (),
          out: str | None = None, diag_tus: tuple | None = None) -> str:
    """diag=True builds libwbq_diag.so with in-kernel phase stamps (never the product);
    defines/out build an experiment variant (scripts/ab_bench.py) at another path. diag_tus: stamp
    only these translation units (plus wbq_api.hip, which holds the stamp buffers and the read-out),
    the others link their product objects (the argument structs do not depend on the flag; a stamped
    qppvm or contact unit compiles for ~25 min)."""
    if defines and out is None:
        raise ValueError("an experiment build (defines) needs its own output path: the product "
                         "library and its source stamp describe the product flags only")
    lib = out or (LIB.replace("libwbq.so", "libwbq_diag.so") if diag else LIB)
    if not force and not diag and out is None and not _stale():
        return LIB
    flags = _flags(diag, defines)
    # one translation unit per process (each holds its own kernels), then one link. An object is
    # keyed by the content hash of its flags, its source and every header, so it is reused only
    # when none of them changed (WBQ_INCREMENTAL=1 reuses objects on a forced build too)
    objdir = os.path.join(HERE, "build", "obj")
    os.makedirs(objdir, exist_ok=True)
    hdrs = _headers()
    # the record is taken before compiling: an edit made while the build runs leaves it stale
    record = _digest(flags, [os.path.join(CSRC, s) for s in SOURCES] + hdrs)
    def tu_flags(src):
        if diag and diag_tus is not None and os.path.basename(src) not in tuple(diag_tus) + ("wbq_api.hip",):
            return _flags(False, defines)
        # an experiment define reaches only the translation units whose sources name its macro, so the
        # others keep their cached objects
        if not defines:
            return flags
        text = "".join(open(p).read() for p in [src] + _headers(src))
        keep = [d for d in defines if d.split("=")[0] in text]
        return _flags(diag, tuple(keep))
    tus = [(os.path.join(CSRC, s), tu_flags(os.path.join(CSRC, s))) for s in SOURCES]
    objs = [os.path.join(objdir, os.path.splitext(os.path.basename(src))[0] + "_" +
                         _digest(fl, [src] + _headers(src)) + ".o")
            for src, fl in tus]
    procs = []
    for (src, fl), o in zip(tus, objs):
        if (not force or os.environ.get("WBQ_INCREMENTAL")) and os.path.exists(o):
            continue
        cmd = fl + ["-c", src, "-o", o + ".tmp"]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        procs.append((cmd, subprocess.Popen(cmd)))
    failed = [c for c, p in procs if p.wait() != 0]
    if failed:
        raise subprocess.CalledProcessError(1, failed[0])
    for c, _ in procs:
        os.replace(c[-1], c[-1][:-4])
    subprocess.check_call(["hipcc", f"--offload-arch={ARCH}", "-shared", *objs, "-o", lib + ".tmp"])
    os.replace(lib + ".tmp", lib)
    if lib == LIB:
        with open(_stamp(LIB), "w") as f:
            f.write(record + "\n")
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
