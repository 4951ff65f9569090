"""A/B helper: run bench.py against an experiment build of libwbq (qppvm_amd.build.build(
defines=..., out=...)) instead of the in-tree product library. Usage:
    python scripts/ab_bench.py <lib.so> [bench.py arguments]"""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402  (torch's HIP runtime first, as in bench.py)

torch.cuda.init()
from qppvm_amd import wbq  # noqa: E402

wbq.load_library(os.path.abspath(sys.argv[1]))  # cached: every solver in bench.py uses it
sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[2:]
runpy.run_path(sys.argv[0], run_name="__main__")
