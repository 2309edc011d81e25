"""ctypes binding of libilqr_hip.so (include/ilqr.h).

The library is built in-tree (ilqr.jl_amd/lib/libilqr_hip.so) by
`make -C ilqr.jl_amd/csrc` or `__graft_entry__.build()`. There is no fallback:
if the library is missing, importing the device API raises.
"""
from __future__ import annotations

import ctypes as C
import os

LIB_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lib",
                        "libilqr_hip.so")
# test-only builds (csrc/Makefile `variants`): the cooperative search's timeout exit forced
WAIT0_LIB_PATH = os.path.join(os.path.dirname(LIB_PATH), "variants", "libilqr_hip_wait0.so")

ABI_VERSION = 2  # ILQR_ABI_VERSION of include/ilqr.h

# ilqr_status
OK = 0
ERR_BAD_DIMS = 1
ERR_BAD_ARG = 2
ERR_UNSUPPORTED = 3
ERR_HIP = 4
ERR_NAN = 5
ERR_LS_EXHAUSTED = 6

# per-trajectory status
TRAJ_OK = 0
TRAJ_CONVERGED = 1
TRAJ_MAX_ITER = 2
TRAJ_LS_EXHAUSTED = 3
TRAJ_NAN = 4

# ilqr_set_schedule flags (LQ family)
SCHED_PIPELINED = 1
SCHED_RING_FORWARD = 2
SCHED_BACKWARD_WAVE = 4
SCHED_BACKWARD_BLOCK = 8
SCHED_FUSED = 16
SCHED_FORWARD_MFMA = 32
SCHED_SEQUENTIAL_SEARCH = 64
MULTI_WARM_START = 1
MULTI_USE_X_TRAJ = 2

PROBLEM_LQ = 1
PROBLEM_TWO_LINK = 2
PROBLEM_TILES = 3
PROBLEM_CHAIN = 4

# ilqr_dtype / ilqr_linearization (chain family)
F64 = 0
F32 = 1
LINEARIZE_DUAL = 0
LINEARIZE_CENTRAL_FD = 1
CHAIN_DYN_AUTO = 0          # ilqr_chain_dynamics_mode
CHAIN_DYN_RNEA = 1
CHAIN_DYN_CLOSED_FORM = 2
CHAIN_COST_JOINT = 0            # ilqr_chain_cost_mode (cost_functions.jl's factories)
CHAIN_COST_SIMPLE = 1
CHAIN_COST_SIMPLE_EUCLIDEAN = 2
CHAIN_MAX_JOINTS = 8


class Problem(C.Structure):
    _fields_ = [("kind", C.c_int32), ("reserved", C.c_int32),
                ("A", C.c_void_p), ("B", C.c_void_p), ("Q", C.c_void_p),
                ("R", C.c_void_p), ("Qf", C.c_void_p)]


class Tiles(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in ("A", "B", "lx", "lu", "lxx", "lux", "luu", "lfx", "lfxx")]


class Options(C.Structure):
    _fields_ = [("max_iter", C.c_int32), ("max_trials", C.c_int32), ("tol", C.c_double),
                ("mu", C.c_double), ("alpha0", C.c_double), ("shrink", C.c_double)]


class History(C.Structure):
    """ilqr_history (include/ilqr.h): device arrays (max_iter, batch), each may be NULL."""
    _fields_ = [("cost", C.c_void_p), ("trials", C.c_void_p), ("alpha", C.c_void_p), ("du2", C.c_void_p)]


class ChainStruct(C.Structure):
    """ilqr_chain (include/ilqr.h)."""
    J = CHAIN_MAX_JOINTS
    _fields_ = [("n_joints", C.c_int32), ("nu", C.c_int32), ("dt", C.c_double),
                ("gravity", C.c_double * 3),
                ("joint_rot", (C.c_double * 9) * J), ("joint_pos", (C.c_double * 3) * J),
                ("axis", (C.c_double * 3) * J), ("mass", C.c_double * J),
                ("com", (C.c_double * 3) * J), ("inertia", (C.c_double * 9) * J),
                ("target", C.c_double * J), ("q_weight", C.c_double * J),
                ("r_weight", C.c_double * J), ("qf_weight", C.c_double * J)]


FLOATING_MAX_JOINTS = 2
FLOATING_MAX_POSE = 6 + FLOATING_MAX_JOINTS


class FloatingStruct(C.Structure):
    """ilqr_floating (include/ilqr.h): the floating-base RBD family."""
    J, Q = FLOATING_MAX_JOINTS, FLOATING_MAX_POSE
    _fields_ = [("n_joints", C.c_int32), ("dt", C.c_double), ("gravity", C.c_double * 3),
                ("base_mass", C.c_double), ("base_com", C.c_double * 3), ("base_inertia", C.c_double * 9),
                ("joint_rot", (C.c_double * 9) * J), ("joint_pos", (C.c_double * 3) * J),
                ("axis", (C.c_double * 3) * J), ("mass", C.c_double * J),
                ("com", (C.c_double * 3) * J), ("inertia", (C.c_double * 9) * J),
                ("target", C.c_double * Q), ("q_weight", C.c_double * Q),
                ("r_weight", C.c_double * Q), ("qf_weight", C.c_double * Q),
                ("q_scale", C.c_double), ("r_scale", C.c_double), ("qf_scale", C.c_double)]


# every symbol declared in include/ilqr.h, with its ctypes signature
P = C.c_void_p
SIGNATURES = {
    "ilqr_abi_version": (C.c_int, []),
    "ilqr_status_string": (C.c_char_p, [C.c_int]),
    "ilqr_last_error": (C.c_char_p, []),
    "ilqr_default_options": (None, [C.POINTER(Options)]),
    "ilqr_supported": (C.c_int, [C.c_int32, C.c_int, C.c_int]),
    "ilqr_create": (C.c_int, [C.POINTER(P), C.c_int, C.c_int, C.c_int, C.c_int, C.c_int]),
    "ilqr_destroy": (C.c_int, [P]),
    "ilqr_set_stream": (C.c_int, [P, P]),
    "ilqr_sync": (C.c_int, [P]),
    "ilqr_set_schedule": (C.c_int, [P, C.c_int]),
    "ilqr_multi_create": (C.c_int, [P, P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int]),
    "ilqr_multi_destroy": (C.c_int, [P]),
    "ilqr_multi_set_schedule": (C.c_int, [P, C.c_int]),
    "ilqr_multi_devices": (C.c_int, [P]),
    "ilqr_multi_fit": (C.c_int, [P, C.POINTER(Problem), C.POINTER(Options), P, P, P, P, P, P, P, P]),
    "ilqr_multi_set_problem": (C.c_int, [P, C.POINTER(Problem)]),
    "ilqr_multi_load": (C.c_int, [P, P, P, P]),
    "ilqr_multi_fit_resident": (C.c_int, [P, C.POINTER(Options), C.c_int, C.POINTER(History)]),
    "ilqr_multi_gather": (C.c_int, [P, P, P, P, P, P]),
    "ilqr_host_alloc": (C.c_int, [C.c_size_t, C.POINTER(P)]),
    "ilqr_host_free": (C.c_int, [P]),
    "ilqr_backward": (C.c_int, [P, C.POINTER(Problem), C.POINTER(Options), P, P, P, P, P]),
    "ilqr_backward_tiles": (C.c_int, [P, C.POINTER(Tiles), C.POINTER(Options), P, P, P]),
    "ilqr_linearize": (C.c_int, [P, C.POINTER(Problem), P, P, P, P]),
    "ilqr_forward": (C.c_int, [P, C.POINTER(Problem), C.POINTER(Options), P, P, P, P, P, P,
                               P, P, P, P, P]),
    "ilqr_iterate": (C.c_int, [P, C.POINTER(Problem), C.POINTER(Options), P, P, P, P, P, P,
                               P, P, P, P]),
    "ilqr_fit": (C.c_int, [P, C.POINTER(Problem), C.POINTER(Options), P, P, P, P, P, P, P, P]),
    "ilqr_fit_ex": (C.c_int, [P, C.POINTER(Problem), C.POINTER(Options), P, P, P, P, P, P, P, P,
                              C.POINTER(History)]),
    "ilqr_malloc": (C.c_int, [P, C.c_size_t, C.POINTER(P)]),
    "ilqr_free": (C.c_int, [P, P]),
    "ilqr_memcpy_h2d": (C.c_int, [P, P, P, C.c_size_t]),
    "ilqr_memcpy_d2h": (C.c_int, [P, P, P, C.c_size_t]),
    "ilqr_selftest": (C.c_int, [C.c_int, C.POINTER(C.c_int32)]),
    "ilqr_chain_supported": (C.c_int, [C.c_int, C.c_int]),
    "ilqr_chain_last_error": (C.c_char_p, []),
    "ilqr_chain_create": (C.c_int, [C.POINTER(P), C.c_int, C.POINTER(ChainStruct), C.c_int,
                                    C.c_int, C.c_int32, C.c_int32]),
    "ilqr_chain_destroy": (C.c_int, [P]),
    "ilqr_chain_set_stream": (C.c_int, [P, P]),
    "ilqr_chain_set_dynamics": (C.c_int, [P, C.c_int32]),
    "ilqr_chain_get_dynamics": (C.c_int32, [P]),
    "ilqr_chain_closed_form_error": (C.c_double, [P]),
    "ilqr_chain_set_simple_costs": (C.c_int, [P, C.c_int32, C.c_int32, C.POINTER(C.c_double),
                                              C.POINTER(C.c_double), C.c_double]),
    "ilqr_chain_get_cost_mode": (C.c_int32, [P]),
    "ilqr_chain_sync": (C.c_int, [P]),
    "ilqr_chain_dynamics": (C.c_int, [P, P, P, P, C.c_int]),
    "ilqr_chain_linearize": (C.c_int, [P, P, P, P, P]),
    "ilqr_chain_backward": (C.c_int, [P, C.POINTER(Options), P, P, P, P, P]),
    "ilqr_chain_forward": (C.c_int, [P, C.POINTER(Options), P, P, P, P, P, P, P, P, P, P, P]),
    "ilqr_chain_iterate": (C.c_int, [P, C.POINTER(Options), P, P, P, P, P, P, P, P, P, P]),
    "ilqr_chain_fit": (C.c_int, [P, C.POINTER(Options), P, P, P, P, P, P, P, P]),
    "ilqr_chain_fit_ex": (C.c_int, [P, C.POINTER(Options), P, P, P, P, P, P, P, P, C.POINTER(History)]),
    "ilqr_floating_supported": (C.c_int, [C.c_int]),
    "ilqr_floating_last_error": (C.c_char_p, []),
    "ilqr_floating_create": (C.c_int, [C.POINTER(P), C.c_int, C.POINTER(FloatingStruct), C.c_int, C.c_int]),
    "ilqr_floating_destroy": (C.c_int, [P]),
    "ilqr_floating_set_stream": (C.c_int, [P, P]),
    "ilqr_floating_sync": (C.c_int, [P]),
    "ilqr_floating_dynamics": (C.c_int, [P, P, P, P, C.c_int]),
    "ilqr_floating_linearize": (C.c_int, [P, P, P, P, P]),
    "ilqr_floating_backward": (C.c_int, [P, C.POINTER(Options), P, P, P, P, P]),
    "ilqr_floating_forward": (C.c_int, [P, C.POINTER(Options), P, P, P, P, P, P, P, P, P, P, P]),
    "ilqr_floating_fit": (C.c_int, [P, C.POINTER(Options), P, P, P, P, P, P, P, P]),
    "ilqr_floating_fit_ex": (C.c_int, [P, C.POINTER(Options), P, P, P, P, P, P, P, P, C.POINTER(History)]),
}

_lib = None


def load(path: str = LIB_PATH) -> C.CDLL:
    """Load libilqr_hip.so and declare every exported signature (raises if absent)."""
    global _lib
    if _lib is not None and path == LIB_PATH:
        return _lib
    if not os.path.exists(path):
        raise ImportError(f"{path} not built: run `make -C ilqr.jl_amd/csrc` "
                          "(the HIP path has no CPU fallback)")
    lib = C.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.ilqr_abi_version() != ABI_VERSION:
        raise ImportError("libilqr_hip.so ABI version mismatch")
    if path == LIB_PATH:
        _lib = lib
    return lib


class IlqrError(RuntimeError):
    def __init__(self, status: int, where: str):
        lib = load()
        msg = lib.ilqr_status_string(status).decode()
        extra = (lib.ilqr_last_error().decode() or lib.ilqr_chain_last_error().decode()
                 or lib.ilqr_floating_last_error().decode())
        super().__init__(f"{where}: {msg}" + (f" ({extra})" if extra and status == ERR_HIP else ""))
        self.status = status


def check(status: int, where: str, allow=()) -> int:
    if status != OK and status not in allow:
        raise IlqrError(status, where)
    return status


def default_options(**overrides) -> Options:
    o = Options()
    load().ilqr_default_options(C.byref(o))
    for k, v in overrides.items():
        if v is not None:
            setattr(o, k, v)
    return o
