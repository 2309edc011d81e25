"""CPU tests of the drop-in boundary: libilqr_hip.so loads and exports every symbol
include/ilqr.h declares; argument validation works without touching a GPU."""
import ctypes as C
import os
import re

import pytest

from ilqr_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "ilqr.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(ilqr_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_the_bound_symbols():
    names = declared_functions()
    assert "ilqr_fit" in names and "ilqr_backward" in names and "ilqr_forward" in names
    assert set(names) == set(_lib.SIGNATURES), set(names) ^ set(_lib.SIGNATURES)


def test_library_loads_and_exports_every_symbol():
    lib = _lib.load()
    for name in declared_functions():
        assert hasattr(lib, name), name
    assert lib.ilqr_abi_version() == _lib.ABI_VERSION == 2


def test_status_strings_and_defaults():
    lib = _lib.load()
    for s in range(7):
        assert lib.ilqr_status_string(s)
    o = _lib.default_options()
    # the reference's defaults: max_iter=100, tol=1e-6 (forward_pass.jl:152),
    # μ = 0.01 (backward_pass.jl:214), α₀ = 1 (forward_pass.jl:66), α /= 2 (:82)
    assert (o.max_iter, o.tol, o.mu, o.alpha0, o.shrink) == (100, 1e-6, 0.01, 1.0, 0.5)
    assert o.max_trials >= 30


def test_supported_shapes():
    lib = _lib.load()
    assert lib.ilqr_supported(_lib.PROBLEM_LQ, 12, 4) == 1
    assert lib.ilqr_supported(_lib.PROBLEM_LQ, 5, 3) == 1   # zero-padded onto (12, 4)
    assert lib.ilqr_supported(_lib.PROBLEM_LQ, 13, 3) == 0
    assert lib.ilqr_supported(_lib.PROBLEM_LQ, 12, 5) == 0
    assert lib.ilqr_supported(99, 12, 4) == 0
    assert lib.ilqr_supported(_lib.PROBLEM_TWO_LINK, 4, 2) == 1
    assert lib.ilqr_supported(_lib.PROBLEM_TWO_LINK, 12, 4) == 0
    assert lib.ilqr_supported(_lib.PROBLEM_LQ, 4, 2) == 1
    assert lib.ilqr_supported(_lib.PROBLEM_TILES, 7, 3) == 1
    assert lib.ilqr_supported(_lib.PROBLEM_TILES, 13, 1) == 1   # the wide tiles kernel
    assert lib.ilqr_supported(_lib.PROBLEM_TILES, 16, 8) == 1   # animate_RBD_2_link.jl's shape
    assert lib.ilqr_supported(_lib.PROBLEM_TILES, 17, 1) == 0
    assert lib.ilqr_supported(_lib.PROBLEM_TILES, 16, 9) == 0


def test_header_problem_kinds_match_binding():
    import re
    hdr = open(os.path.join(ROOT, "include", "ilqr.h")).read()
    kinds = dict(re.findall(r"ILQR_PROBLEM_(\w+) = (\d+)", hdr))
    assert int(kinds["LQ"]) == _lib.PROBLEM_LQ and int(kinds["TWO_LINK"]) == _lib.PROBLEM_TWO_LINK


def test_argument_validation_needs_no_gpu():
    lib = _lib.load()
    h = C.c_void_p()
    # reference: @assert N == M+1 / positive sizes → ILQR_ERR_BAD_DIMS before any HIP call
    assert lib.ilqr_create(C.byref(h), 0, 12, 4, 0, 16) == _lib.ERR_BAD_DIMS
    assert lib.ilqr_create(C.byref(h), 0, 12, 4, 100, 0) == _lib.ERR_BAD_DIMS
    assert lib.ilqr_create(None, 0, 12, 4, 100, 16) == _lib.ERR_BAD_ARG
    o = _lib.default_options()
    p = _lib.Problem(_lib.PROBLEM_LQ, 0, None, None, None, None, None)
    assert lib.ilqr_backward(None, C.byref(p), C.byref(o), None, None, None, None, None) == _lib.ERR_BAD_ARG
    assert lib.ilqr_fit(None, C.byref(p), C.byref(o), None, None, None, None, None, None, None,
                        None) == _lib.ERR_BAD_ARG
    assert lib.ilqr_destroy(None) == _lib.OK


def test_missing_library_fails_loudly(tmp_path):
    with pytest.raises(ImportError):
        _lib.load(str(tmp_path / "nope.so"))


def test_no_oracle_in_the_product_path():
    """The product (ilqr.jl_amd/) must never import or link the oracle."""
    pkg = os.path.join(ROOT, "ilqr.jl_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".hip", ".cpp", ".h", ".jl")) or f == "Makefile":
                txt = open(os.path.join(dirpath, f), encoding="utf-8").read()
                for bad in ("import oracle", "from oracle", "libilqr_oracle", "ilqr_ref"):
                    assert bad not in txt, (f, bad)


def test_julia_shim_ccalls_declared_symbols():
    """Every `ccall((:ilqr_…, libilqr), …)` of the Julia shim names a function that
    include/ilqr.h declares and the library exports (the shim cannot run here)."""
    src = open(os.path.join(ROOT, "ilqr.jl_amd", "julia", "iLQRHIP.jl")).read()
    called = set(re.findall(r"ccall\(\(:(ilqr_[a-z0-9_]+),\s*libilqr\)", src))
    assert {"ilqr_fit_ex", "ilqr_backward", "ilqr_forward", "ilqr_backward_tiles",
            "ilqr_chain_fit", "ilqr_chain_set_dynamics", "ilqr_multi_set_problem", "ilqr_multi_load",
            "ilqr_multi_fit_resident", "ilqr_multi_gather", "ilqr_linearize"} <= called, called
    declared = set(declared_functions())
    assert called <= declared, called - declared
    lib = _lib.load()
    for name in called:
        assert hasattr(lib, name), name


def test_julia_shim_exposes_reference_api():
    """The shim defines the reference's public functions (docs/src/documentation.md:13-51)
    and the resident Solver's methods; the per-call paths no longer create handles
    (they run on a cached workspace through with_cached, the closures' tiles path
    included): only Solver(), TilesSolver(), the linearize helper and solve!(prob)
    construct a Handle."""
    src = open(os.path.join(ROOT, "ilqr.jl_amd", "julia", "iLQRHIP.jl")).read()
    for fn in ("fit", "backward_pass", "forward_pass", "linearize_dynamics", "immediate_cost_quadratization",
               "final_cost_quadratization", "optimal_controller_param", "feedback_parameters", "step_back",
               "fit!", "backward!", "forward!", "set_problem!", "solve!", "clear_cache!"):
        assert re.search(r"^(function )?" + re.escape(fn) + r"\(", src, re.M), fn
    assert re.search(r"^Base\.close\(s::Solver\)", src, re.M)
    body = lambda name: src[src.index(f"function {name}("):src.index("\nend", src.index(f"function {name}("))]
    for name in ("fit", "backward_pass", "forward_pass"):
        assert "Handle(" not in body(name) and "with_cached(SOLVER_CACHE" in body(name), name
    assert re.search(r"^Base\.close\(s::TilesSolver\)", src, re.M)
    assert "Handle(" not in body("backward_tiles_device")
    assert "with_cached(TILES_CACHE" in body("backward_tiles_device")
    # every cached workspace carries the lock with_cached holds for a call
    assert src.count("ReentrantLock()") >= 5
    # the floating-base family (the reference's RBD script) and the chain family: their
    # entry points run on cached workspaces too (floating_fit / chain_fit
    # created and destroyed a handle per call); the reference API reaches the floating
    # kernels through its recognised callables
    for name in ("floating_fit1", "floating_backward", "floating_forward", "floating_linearize", "floating_fit"):
        assert "Handle(" not in body(name) and "ilqr_floating_create" not in body(name), name
        assert "floating_cached(" in body(name), name
    assert "Handle(" not in body("chain_fit") and "ilqr_chain_create" not in body("chain_fit")
    assert "with_cached(CHAIN_CACHE" in body("chain_fit")
    assert "floating_cached(" in src[src.index("function (f::FloatingDynamics)"):]
    for name, call in (("fit", "floating_fit1("), ("backward_pass", "floating_backward("),
                       ("forward_pass", "floating_forward(")):
        assert "fam == :floating" in body(name) and call in body(name), name
    assert "is_floating(f, l, lf) ? :floating" in src
    assert "FLOATING_CACHE" in body("clear_cache!") and "CHAIN_CACHE" in body("clear_cache!")
