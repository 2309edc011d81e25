"""ctypes wrapper of oracle/ilqr_ref.c (C restatement of the reference's hot
path for the LQ family and the 2-link arm) — TEST INFRASTRUCTURE ONLY: the checker for large parity tests and the
bench's cpu_baseline leg. Build with `make -C oracle`."""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(_HERE, "lib", "libilqr_oracle.so")
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        _lib = C.CDLL(LIB)
        _lib.oracle_max_threads.restype = C.c_int
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def _f64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


def max_threads():
    return load().oracle_max_threads()


def lq_backward(lq, x, u, mu=0.01, symmetrize=False, nthreads=0):
    """→ (d (B,T,m), K (B,T,m,n), status (B,))"""
    lib = load()
    nb, n, m = lq.B.shape
    T = u.shape[1]
    x, u = _f64(x), _f64(u)
    d = np.empty((nb, T, m))
    K = np.empty((nb, T, m, n))
    st = np.empty(nb, dtype=np.int32)
    rc = lib.oracle_lq_backward(nb, T, n, m, _p(lq.A), _p(lq.B), _p(lq.Q), _p(lq.R), _p(lq.Qf),
                                _p(x), _p(u), C.c_double(mu), int(symmetrize), _p(d), _p(K), _p(st),
                                nthreads)
    assert rc >= 0
    return d, K, st


def lq_forward(lq, x, u, x_traj, d, K, prev_cost, max_trials=64, alpha0=1.0, shrink=0.5,
               nthreads=0):
    """→ (x_new, u_new, cost, trials) ; trials < 0 means exhausted."""
    lib = load()
    nb, n, m = lq.B.shape
    T = u.shape[1]
    x, u, d, K = _f64(x), _f64(u), _f64(d), _f64(K)
    xt = None if x_traj is None else _f64(x_traj)
    pc = _f64(np.broadcast_to(np.asarray(prev_cost, dtype=np.float64), (nb,)))
    xn = np.empty((nb, T + 1, n))
    un = np.empty((nb, T, m))
    cost = np.empty(nb)
    tr = np.empty(nb, dtype=np.int32)
    lib.oracle_lq_forward(nb, T, n, m, _p(lq.A), _p(lq.B), _p(lq.Q), _p(lq.R), _p(lq.Qf), _p(x),
                          _p(u), _p(xt), _p(d), _p(K), _p(pc), _p(xn), _p(un), _p(cost), _p(tr),
                          max_trials, C.c_double(alpha0), C.c_double(shrink), nthreads)
    return xn, un, cost, tr


def lq_fit(lq, x_init, u_init, x_traj=None, max_iter=100, tol=1e-6, mu=0.01, max_trials=64,
           symmetrize=False, nthreads=0):
    """→ (x, u, cost, iters, status)   status: 1 converged, 2 max_iter, 3 LS exhausted, 4 NaN"""
    lib = load()
    nb, n, m = lq.B.shape
    T = u_init.shape[1]
    xi, ui = _f64(x_init), _f64(u_init)
    xt = None if x_traj is None else _f64(x_traj)
    xo = np.empty((nb, T + 1, n))
    uo = np.empty((nb, T, m))
    cost = np.empty(nb)
    iters = np.empty(nb, dtype=np.int32)
    st = np.empty(nb, dtype=np.int32)
    lib.oracle_lq_fit(nb, T, n, m, _p(lq.A), _p(lq.B), _p(lq.Q), _p(lq.R), _p(lq.Qf), _p(xi),
                      _p(ui), _p(xt), max_iter, C.c_double(tol), C.c_double(mu), int(symmetrize), max_trials,
                      _p(xo), _p(uo), _p(cost), _p(iters), _p(st), nthreads)
    return xo, uo, cost, iters, st


def host_threads():
    """Threads for a CPU-baseline leg: every CPU this process may run on, capped at the
    operator's per-GPU share when OMP_NUM_THREADS is set (16 on the GPU pool)."""
    n = len(os.sched_getaffinity(0))
    share = os.environ.get("OMP_NUM_THREADS", "")
    return min(n, int(share)) if share.isdigit() and int(share) > 0 else n


# -- 2-link arm (test/2_link_example) ---------------------------------------------
def tl_backward(x, u, mu=0.01, symmetrize=False, nthreads=0):
    lib = load()
    x, u = _f64(x), _f64(u)
    nb, T, nu = u.shape
    d = np.empty((nb, T, nu))
    K = np.empty((nb, T, nu, 4))
    st = np.empty(nb, dtype=np.int32)
    lib.oracle_tl_backward(nb, T, nu, _p(x), _p(u), C.c_double(mu), int(symmetrize), _p(d), _p(K),
                           _p(st), nthreads)
    return d, K, st


def tl_forward(x, u, x_traj, d, K, prev_cost, max_trials=64, alpha0=1.0, shrink=0.5, nthreads=0):
    lib = load()
    x, u, d, K = _f64(x), _f64(u), _f64(d), _f64(K)
    nb, T, nu = u.shape
    xt = None if x_traj is None else _f64(x_traj)
    pc = _f64(np.broadcast_to(np.asarray(prev_cost, dtype=np.float64), (nb,)))
    xn = np.empty((nb, T + 1, 4))
    un = np.empty((nb, T, nu))
    cost = np.empty(nb)
    tr = np.empty(nb, dtype=np.int32)
    lib.oracle_tl_forward(nb, T, nu, _p(x), _p(u), _p(xt), _p(d), _p(K), _p(pc), _p(xn), _p(un),
                          _p(cost), _p(tr), max_trials, C.c_double(alpha0), C.c_double(shrink),
                          nthreads)
    return xn, un, cost, tr


def tl_fit(x_init, u_init, x_traj=None, max_iter=100, tol=1e-6, mu=0.01, max_trials=64,
           symmetrize=False, nthreads=0, history=False):
    """→ (x, u, cost, iters, status), plus with history=True a dict of (max_iter, B)
    arrays "cost" (NaN: not run / failed), "trials" (0: not run), "du2" — the layout of
    ilqr_fit_ex's record (include/ilqr.h)."""
    lib = load()
    xi, ui = _f64(x_init), _f64(u_init)
    nb, T, nu = ui.shape
    xt = None if x_traj is None else _f64(x_traj)
    xo = np.empty((nb, T + 1, 4))
    uo = np.empty((nb, T, nu))
    cost = np.empty(nb)
    iters = np.empty(nb, dtype=np.int32)
    st = np.empty(nb, dtype=np.int32)
    h = None
    if history:
        h = {"cost": np.full((nb, max_iter), np.nan), "trials": np.zeros((nb, max_iter), dtype=np.int32),
             "du2": np.full((nb, max_iter), np.nan)}
    lib.oracle_tl_fit(nb, T, nu, _p(xi), _p(ui), _p(xt), max_iter, C.c_double(tol), C.c_double(mu),
                      int(symmetrize), max_trials, _p(xo), _p(uo), _p(cost), _p(iters), _p(st),
                      nthreads, *((_p(h["cost"]), _p(h["trials"]), _p(h["du2"])) if h else (None, None, None)))
    if history:
        return xo, uo, cost, iters, st, {k: np.ascontiguousarray(v.T) for k, v in h.items()}
    return xo, uo, cost, iters, st


def tl_set_physical_coriolis(on=False):
    """Test-only: the textbook Coriolis matrix in place of the script's quirk (ilqr_ref.c)."""
    load().oracle_tl_set_physical_coriolis(int(on))


def set_fit_return_post_update(on=False):
    """Test-only: fit returns the iterate that met tol, not the previous one (ilqr_ref.c)."""
    load().oracle_set_fit_return_post_update(int(on))


def tl_set_target(x=0.6, y=-0.5):
    """The 2-link target_tool_loc of the C restatement (test-only; default the script's)."""
    load().oracle_tl_set_target(C.c_double(x), C.c_double(y))


def twolink_cpu_baseline(x, u, batch, budget_s):
    """bench_twolink's cpu_baseline leg: one cold-start iteration (backward +
    forward) per trajectory of the 2-link workload (nu from u), OpenMP over trajectories."""
    import time
    threads = host_threads()
    n = 64
    while True:
        idx = np.arange(n) % x.shape[0]
        t0 = time.perf_counter()
        d, K, _ = tl_backward(x[idx], u[idx], nthreads=threads)
        tl_forward(x[idx], u[idx], None, d, K, np.inf, nthreads=threads)
        el = time.perf_counter() - t0
        if el > budget_s / 4 or n >= 1 << 18:
            break
        n *= 2
    rate = n / el
    return {"value": rate / batch, "unit": f"batched iterations/s (batch={batch})", "cores": threads,
            "kind": "port",
            "sample": f"{n} trajectories x 1 cold-start iteration (C restatement oracle/ilqr_ref.c, "
                      f"dual-number linearisation, OpenMP {threads} threads), {el:.2f} s; "
                      f"trajectory-iterations/s={rate:.1f}"}


# -- caller-supplied tiles (ilqr_backward_tiles) ------------------------------------
TILE_NAMES = ("A", "B", "lx", "lu", "lxx", "lux", "luu", "lfx", "lfxx")


def tiles_backward(tiles, mu=0.01, symmetrize=False, nthreads=0):
    """tiles: dict of arrays with ilqr_tiles' shapes (lux may be None) → (d, K, status)."""
    lib = load()
    t = {k: (None if tiles.get(k) is None else _f64(tiles[k])) for k in TILE_NAMES}
    nb, T, n, m = t["B"].shape
    d = np.empty((nb, T, m))
    K = np.empty((nb, T, m, n))
    st = np.empty(nb, dtype=np.int32)
    rc = lib.oracle_tiles_backward(nb, T, n, m, *(_p(t[k]) for k in TILE_NAMES), C.c_double(mu),
                                   int(symmetrize), _p(d), _p(K), _p(st), nthreads)
    assert rc >= 0
    return d, K, st


# -- RBD chain (ILQR_PROBLEM_CHAIN, BASELINE config 5) ------------------------------
def _chain_args(pr):
    """ChainProblem (ilqr_amd.chain) → the C restatement's chain arguments."""
    ch = pr.chain
    arrs = [_f64(ch.R0), _f64(ch.p), _f64(ch.axis), _f64(ch.mass), _f64(ch.com), _f64(ch.Ic),
            _f64(ch.gravity)]
    tail = [_f64(pr.target), _f64(pr.q_weight), _f64(pr.r_weight), _f64(pr.qf_weight)]
    args = [ch.n, pr.nu] + [_p(a) for a in arrs] + [C.c_double(pr.dt)] + [_p(a) for a in tail]
    return args, arrs + tail  # keep the arrays alive for the call


def chain_dynamics(pr, x, u):
    """One RK4 step of the chain for n points: x (n, 2nj), u (n, nu) → (n, 2nj)."""
    lib = load()
    x, u = _f64(x), _f64(u)
    out = np.empty_like(x)
    args, keep = _chain_args(pr)
    rc = lib.oracle_chain_dynamics(x.shape[0], *args, _p(x), _p(u), _p(out))
    assert rc == 0, "oracle_chain_dynamics: bad chain"
    return out


def chain_iterate(pr, x, u, mu=0.01, symmetrize=True, max_trials=64, nthreads=0):
    """One cold-start iteration per trajectory (central-difference linearisation,
    backward_pass, forward_pass) → (d, K, x_new, u_new, cost, trials)."""
    lib = load()
    x, u = _f64(x), _f64(u)
    nb, T, m = u.shape
    n = x.shape[2]
    d = np.empty((nb, T, m))
    K = np.empty((nb, T, m, n))
    xn, un = np.empty_like(x), np.empty_like(u)
    cost = np.empty(nb)
    trials = np.empty(nb, dtype=np.int32)
    args, keep = _chain_args(pr)
    rc = lib.oracle_chain_iterate(nb, T, *args, _p(x), _p(u), C.c_double(mu), int(symmetrize),
                                  max_trials, _p(d), _p(K), _p(xn), _p(un), _p(cost), _p(trials),
                                  nthreads)
    assert rc >= 0, "oracle_chain_iterate: bad chain"
    return d, K, xn, un, cost, trials
