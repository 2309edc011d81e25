"""CPU tests of the floating-base RBD family's host side (include/ilqr.h
ilqr_floating_*): the ctypes struct matches the C layout, the URDF's root link is read,
the script's problem is assembled as written, and argument checks need no GPU."""
import ctypes as C
import os
import shutil
import subprocess

import numpy as np
import pytest

from ilqr_amd import _lib
from ilqr_amd.floating import (RBD_Q_WEIGHT, RBD_TARGET_POSE, FloatingProblem, rbd_example_problem,
                               rbd_initial_state)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("gcc") is None, reason="no gcc")
def test_struct_layout_matches_header(tmp_path):
    fields = [f[0] for f in _lib.FloatingStruct._fields_]
    src = tmp_path / "lay.c"
    src.write_text('#include <stddef.h>\n#include <stdio.h>\n#include "ilqr.h"\nint main(void){\n'
                   '  printf("%zu\\n", sizeof(ilqr_floating));\n'
                   + "".join(f'  printf("%zu\\n", offsetof(ilqr_floating, {f}));\n' for f in fields)
                   + "  return 0;\n}\n")
    exe = tmp_path / "lay"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), "-I", "/opt/rocm/include", str(src), "-o", str(exe)],
                   check=True, capture_output=True)
    out = [int(v) for v in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    assert out[0] == C.sizeof(_lib.FloatingStruct)
    assert out[1:] == [getattr(_lib.FloatingStruct, f).offset for f in fields]


def test_rbd_example_problem_as_the_script_writes_it():
    p = rbd_example_problem()
    ch = p.chain
    # 2Dof_arm.urdf: a 30 kg base with 50·1 inertia, two 3 kg links with 0.5·1
    assert ch.base_mass == 30.0 and np.allclose(ch.base_Ic, 50.0 * np.eye(3)) and not ch.base_com.any()
    assert list(ch.mass) == [3.0, 3.0]
    assert np.allclose(ch.p, [[0.5, 0.5, 0.0], [1.0, 0.0, 0.0]])
    assert np.allclose(ch.axis, [[0, 0, 1], [0, 1, 0]])
    assert (p.nx, p.nu, p.dt) == (16, 8, 0.01)
    s = p.struct()
    assert list(s.target) == list(RBD_TARGET_POSE) and list(s.q_weight) == list(RBD_Q_WEIGHT)
    assert (s.q_scale, s.r_scale, s.qf_scale) == (10.0, 1.0, 100000.0)
    assert s.base_mass == 30.0 and list(s.base_inertia) == [50.0, 0, 0, 0, 50.0, 0, 0, 0, 50.0]
    x0 = rbd_initial_state()
    assert list(x0[:8]) == [0.0, 0.0, 1.0, 0.5, 0.75, 1.0, 0.0, 0.0] and not x0[8:].any()


def test_create_checks_need_no_gpu():
    lib = _lib.load()
    assert lib.ilqr_floating_supported(2) == 1 and lib.ilqr_floating_supported(1) == 0
    s = rbd_example_problem().struct()
    h = C.c_void_p()
    assert lib.ilqr_floating_create(C.byref(h), 0, C.byref(s), 0, 1) == _lib.ERR_BAD_DIMS
    assert lib.ilqr_floating_create(None, 0, C.byref(s), 10, 1) == _lib.ERR_BAD_ARG
    g = rbd_example_problem().struct()
    g.gravity[2] = -9.81
    assert lib.ilqr_floating_create(C.byref(h), 0, C.byref(g), 10, 1) == _lib.ERR_UNSUPPORTED
    assert b"gravity" in lib.ilqr_floating_last_error()
    j = rbd_example_problem().struct()
    j.n_joints = 1
    assert lib.ilqr_floating_create(C.byref(h), 0, C.byref(j), 10, 1) == _lib.ERR_UNSUPPORTED
    assert lib.ilqr_floating_destroy(None) == _lib.OK


def test_no_base_mass_is_refused():
    p = rbd_example_problem()
    p.chain.base_mass = 0.0
    with pytest.raises(ValueError):
        FloatingProblem(p.chain).struct()


def _julia_struct_layout(name):
    """(size, [offsets]) of a Julia isbits struct of Int32 / Float64 / NTuple{n,Float64}
    fields as declared in the shim, under C alignment rules (what ccall passes)."""
    import re
    src = open(os.path.join(ROOT, "ilqr.jl_amd", "julia", "iLQRHIP.jl")).read()
    body = src[src.index(f"struct {name}"):]
    body = body[body.index("\n") + 1:body.index("\nend")]
    fields = re.findall(r"(\w+)::(Int32|Float64|NTuple\{(\d+),Float64\})", body)
    off, offs, align = 0, [], 1
    for _, ty, n in fields:
        size, a = (4, 4) if ty == "Int32" else ((8, 8) if ty == "Float64" else (8 * int(n), 8))
        off = (off + a - 1) // a * a
        offs.append(off)
        off += size
        align = max(align, a)
    return (off + align - 1) // align * align, offs, [f[0] for f in fields]


def test_julia_floating_model_matches_the_c_layout():
    """The shim's FloatingModel (passed by Ref to ilqr_floating_create) has the C struct's
    field order, offsets and size (the shim cannot run here)."""
    size, offs, names = _julia_struct_layout("FloatingModel")
    assert names == [f[0] for f in _lib.FloatingStruct._fields_]
    assert size == C.sizeof(_lib.FloatingStruct)
    assert offs == [getattr(_lib.FloatingStruct, f).offset for f in names]


def test_julia_constructor_equals_the_python_problem():
    """The shim's rbd_2dof_arm_floating() and ilqr_amd.floating.rbd_example_problem()
    (whose fits the GPU tests pin to the oracle) hand create the same bytes."""
    from julia_layout import rbd_2dof_arm_floating
    j = rbd_2dof_arm_floating()
    p = rbd_example_problem().struct()
    assert bytes(j) == bytes(p)
