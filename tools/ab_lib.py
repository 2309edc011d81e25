"""Run a tool script against another build of the library: ILQR_LIB=<path.so> python
tools/ab_lib.py tools/bench_rbd.py [args] (A/B of two builds on one box, alternated)."""
import os
import runpy
import sys

import torch  # noqa: F401  (torch's HIP runtime first, as in the tools themselves)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ilqr.jl_amd")]
from ilqr_amd import _lib  # noqa: E402

if os.environ.get("ILQR_LIB"):
    _lib._lib = _lib.load(os.environ["ILQR_LIB"])
sys.argv = sys.argv[1:]
runpy.run_path(sys.argv[0], run_name="__main__")
