"""Generate the golden vectors in tests/golden/ from the CPU restatement of the
reference (oracle/ilqr_oracle.py, numpy + dual-number AD).

The reference (aabouman/iLQR.jl) is pure Julia and cannot run here (no Julia
toolchain), and its own tests pin no numeric outputs (unseeded rand(), broken
as written — SURVEY.md §4), so these fixtures are the oracle's outputs on
seeded inputs. The oracle itself is pinned by the known-answer tests in
tests/test_oracle.py. Regenerate with:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ilqr.jl_amd")]

from ilqr_amd.chain import (coupled_2dof_problem, load_robot, rbd_2dof_problem,  # noqa: E402
                            rbd_initial_states)
from ilqr_amd.problems import quadrotor_batch, random_lq_batch  # noqa: E402
from oracle import ilqr_oracle as O  # noqa: E402
from oracle import cost_functions as OC  # noqa: E402
from oracle import rbd as RBD  # noqa: E402

MAX_TRIALS = 60


def lq_case(name, lq, x, u, xtraj=None, symmetrize=False, fit_iters=30, tol=1e-6):
    nb = lq.batch
    T = u.shape[1]
    out = {"A": lq.A, "B": lq.B, "Q": lq.Q, "R": lq.R, "Qf": lq.Qf, "x": x, "u": u}
    if xtraj is not None:
        out["xtraj"] = xtraj
    d = np.empty_like(u)
    K = np.empty((nb, T, lq.nu, lq.nx))
    xn, un = np.empty_like(x), np.empty_like(u)
    cost = np.empty(nb)
    trials = np.empty(nb, dtype=np.int32)
    fx, fu = np.empty_like(x), np.empty_like(u)
    fcost = np.full((nb, fit_iters), np.nan)
    fiters = np.empty(nb, dtype=np.int32)
    for b in range(nb):
        f, l, lf = O.lq_closures(lq.A[b], lq.B[b], lq.Q[b], lq.R[b], lq.Qf[b])
        xt = np.zeros_like(x[b]) if xtraj is None else xtraj[b]
        d[b], K[b] = O.backward_pass(x[b], u[b], f, l, lf, symmetrize=symmetrize)
        if not symmetrize:
            # the literal recursion must be numerically healthy on a literal fixture
            ds, Ks = O.backward_pass(x[b], u[b], f, l, lf, symmetrize=True)
            rel = np.abs(K[b] - Ks).max() / np.abs(Ks).max()
            assert rel < 1e-9, (name, b, rel)
        st = {}
        xn[b], un[b], cost[b] = O.forward_pass(x[b], u[b], xt, d[b], K[b], np.inf, f, l, lf,
                                               max_trials=MAX_TRIALS, stats=st)
        trials[b] = st["trials"]
        hist = []
        fx[b], fu[b] = O.fit(x[b], u[b], f, l, lf, x_traj=xt, max_iter=fit_iters, tol=tol,
                             max_trials=MAX_TRIALS, history=hist, symmetrize=symmetrize)
        fiters[b] = len(hist)
        fcost[b, :len(hist)] = [h["cost"] for h in hist]
    out.update(d=d, K=K, fw_x=xn, fw_u=un, fw_cost=cost, fw_trials=trials, fit_x=fx, fit_u=fu,
               fit_cost=fcost, fit_iters=fiters,
               meta=np.array(json.dumps({"symmetrize": symmetrize, "fit_max_iter": fit_iters,
                                         "tol": tol, "max_trials": MAX_TRIALS})))
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)
    print(name, "fit iters", fiters.tolist(), "trials", trials.tolist())


def twolink_case(name, x0s, T, fit_iters=40, tol=1e-6, nu=2):
    """2-link arm; nu = 1 is the build-defined f(x, [u₁, 0]) variant (not reference-pinned)."""
    TL = O.TwoLink
    f = TL.dynamicsf if nu == 2 else TL.dynamicsf_nu1
    nb = len(x0s)
    x = np.stack([O.rollout(np.asarray(x0, float), np.zeros((T, nu)), f) for x0 in x0s])
    u = np.zeros((nb, T, nu))
    d = np.empty_like(u)
    K = np.empty((nb, T, nu, 4))
    xn, un = np.empty_like(x), np.empty_like(u)
    cost = np.empty(nb)
    fx, fu = np.empty_like(x), np.empty_like(u)
    fcost = np.full((nb, fit_iters), np.nan)
    fiters = np.empty(nb, dtype=np.int32)
    for b in range(nb):
        d[b], K[b] = O.backward_pass(x[b], u[b], f, TL.immediate_cost, TL.final_cost)
        xn[b], un[b], cost[b] = O.forward_pass(x[b], u[b], np.zeros_like(x[b]), d[b], K[b], np.inf,
                                               f, TL.immediate_cost, TL.final_cost,
                                               max_trials=MAX_TRIALS)
        hist = []
        fx[b], fu[b] = O.fit(x[b], u[b], f, TL.immediate_cost, TL.final_cost,
                             max_iter=fit_iters, tol=tol, max_trials=MAX_TRIALS, history=hist)
        fiters[b] = len(hist)
        fcost[b, :len(hist)] = [h["cost"] for h in hist]
    np.savez_compressed(os.path.join(HERE, name + ".npz"), x=x, u=u, d=d, K=K, fw_x=xn, fw_u=un,
                        fw_cost=cost, fit_x=fx, fit_u=fu, fit_cost=fcost, fit_iters=fiters,
                        meta=np.array(json.dumps({"T": T, "nu": nu, "fit_max_iter": fit_iters, "tol": tol})))
    print(name, "fit iters", fiters.tolist())


def chain_case(name, nu, x0s, T, fit_iters=20, tol=1e-6, pr=None, robot="2dof_arm", simple=None):
    """RBD family (ILQR_PROBLEM_CHAIN) on the fixed-base 2Dof_arm (or `pr`): oracle.rbd
    dynamics (RNEA + RK4, exact Jacobians by forward-mode AD) through the generic
    oracle passes. `simple` = dict(body, point, final_target, weight, euclidean): the
    costs of cost_functions.jl's factories (oracle.cost_functions, differentiated by
    the ForwardDiff restatement) instead of the joint-space ones."""
    pr = rbd_2dof_problem(nu) if pr is None else pr
    model = RBD.ChainModel(pr.chain, pr.dt)
    cost = RBD.ChainCost(pr.target, pr.q_weight, pr.r_weight, pr.qf_weight)
    f, l, lf = RBD.chain_closures(model, cost)
    if simple is not None:
        a = (pr.chain, simple["body"], simple["point"], simple["final_target"], simple["weight"])
        l = OC.simple_immediate_cost(*a)
        lf = OC.simple_final_cost(*a, euclidean=simple["euclidean"])
    nb, nx = len(x0s), pr.nx
    u = np.zeros((nb, T, nu))
    x = np.empty((nb, T + 1, nx))
    x[:, 0] = x0s
    for t in range(T):
        x[:, t + 1] = model.step(x[:, t], u[:, t])
    A, Bm = model.linearize(x[:, :T].reshape(-1, nx), u.reshape(-1, nu))
    d, K = np.empty_like(u), np.empty((nb, T, nu, nx))
    xn, un, fwc = np.empty_like(x), np.empty_like(u), np.empty(nb)
    fx, fu = np.empty_like(x), np.empty_like(u)
    fcost = np.full((nb, fit_iters), np.nan)
    fiters = np.empty(nb, dtype=np.int32)
    fstatus = np.empty(nb, dtype=np.int32)  # ILQR_TRAJ_*: 1 converged, 2 max_iter, 3 exhausted
    for b in range(nb):
        d[b], K[b] = O.backward_pass(x[b], u[b], f, l, lf)
        ds, Ks = O.backward_pass(x[b], u[b], f, l, lf, symmetrize=True)
        assert np.abs(K[b] - Ks).max() <= 1e-9 * np.abs(Ks).max(), name
        xn[b], un[b], fwc[b] = O.forward_pass(x[b], u[b], np.zeros_like(x[b]), d[b], K[b], np.inf,
                                              f, l, lf, max_trials=MAX_TRIALS)
        hist = []
        try:
            fx[b], fu[b] = O.fit(x[b], u[b], f, l, lf, max_iter=fit_iters, tol=tol,
                                 max_trials=MAX_TRIALS, history=hist)
            fiters[b] = len(hist)
            fstatus[b] = 1 if hist[-1]["du2"] <= tol else 2
        except O.LineSearchExhausted:
            # the reference would loop forever; the device stops this trajectory at the
            # iterate its failing iteration started from (len(hist) accepted updates)
            fx[b], fu[b] = O.fit(x[b], u[b], f, l, lf, max_iter=len(hist), tol=-1.0,
                                 max_trials=MAX_TRIALS)
            fiters[b] = len(hist) + 1
            fstatus[b] = 3
        fcost[b, :len(hist)] = [h["cost"] for h in hist]
    np.savez_compressed(os.path.join(HERE, name + ".npz"), x=x, u=u,
                        A=A.reshape(nb, T, nx, nx), B=Bm.reshape(nb, T, nx, nu), d=d, K=K,
                        fw_x=xn, fw_u=un, fw_cost=fwc, fit_x=fx, fit_u=fu, fit_cost=fcost,
                        fit_iters=fiters, fit_status=fstatus,
                        meta=np.array(json.dumps({"T": T, "nu": nu, "fit_max_iter": fit_iters,
                                                  "tol": tol, "robot": robot, "simple": simple})))
    print(name, "fit iters", fiters.tolist(), "status", fstatus.tolist())


def chain6_dynamics_case(name, n=24, seed=5):
    """One RK4 step of the coupled 6-DoF arm (test/urdf/6Dof_arm.urdf) at random states."""
    ch = load_robot("6dof_arm")
    model = RBD.ChainModel(ch, 0.01)
    rng = np.random.default_rng(seed)
    x = np.concatenate([rng.uniform(-2, 2, (n, 6)), rng.uniform(-1, 1, (n, 6))], axis=1)
    u = rng.uniform(-5, 5, (n, 6))
    M = np.stack([model.mass_matrix_np(q) for q in x[:, :6]])
    bias = np.stack([model.bias_np(q, qd) for q, qd in zip(x[:, :6], x[:, 6:])])
    np.savez_compressed(os.path.join(HERE, name + ".npz"), x=x, u=u, x_next=model.step(x, u),
                        M=M, bias=bias)
    print(name, "points", n)


def main(only=()):
    def want(n):
        return not only or n in only
    if want("chain2"):
        # RBD family, fixed-base 2Dof_arm (BASELINE config 5 shape: T = 100)
        chain_case("chain2_t100", 2, rbd_initial_states(3, 2, seed0=0), T=100)
        chain_case("chain2_nu1_t50", 1, rbd_initial_states(2, 2, seed0=10), T=50)
        chain6_dynamics_case("chain6_dynamics")
    if want("chain2_nu1_t100"):
        # BASELINE config 5 as stated: nu = 1 (joint 1 driven), T = 100
        chain_case("chain2_nu1_t100", 1, rbd_initial_states(3, 2, seed0=20), T=100)
    if want("chain2c"):
        # a coupled 2-joint chain (dense q-dependent M, Coriolis and gravity bias): the
        # 2Dof_arm's own M is constant, so it cannot pin the recursion's coupling terms
        chain_case("chain2c_t40", 2, rbd_initial_states(4, 2, seed0=30), T=40,
                   pr=coupled_2dof_problem(2), robot="coupled_2dof")
        chain_case("chain2c_nu1_t40", 1, rbd_initial_states(3, 2, seed0=40), T=40,
                   pr=coupled_2dof_problem(1), robot="coupled_2dof")
    if want("chaintask"):
        # cost_functions.jl's simple_final_cost / simple_immediate_cost: the tip point's
        # z against every target component (the reference's reading), and the squared
        # distance (euclidean) on the coupled chain
        chain_case("chaintask_t60", 2, rbd_initial_states(3, 2, seed0=50), T=60, robot="2dof_arm",
                   simple=dict(body=1, point=[0.0, 0.0, 0.5], final_target=[0.3, 0.5, 0.4],
                               weight=2e4, euclidean=False))
        chain_case("chaintask_c_nu1_t40", 1, rbd_initial_states(2, 2, seed0=60), T=40,
                   pr=coupled_2dof_problem(1), robot="coupled_2dof",
                   simple=dict(body=1, point=[0.2, 0.1, 0.3], final_target=[0.6, 0.2, 0.7],
                               weight=2e5, euclidean=False))
        chain_case("chaintask_c_euc_t40", 2, rbd_initial_states(2, 2, seed0=70), T=40,
                   pr=coupled_2dof_problem(2), robot="coupled_2dof",
                   simple=dict(body=1, point=[0.2, 0.1, 0.3], final_target=[1.2, 1.0, 0.5],
                               weight=2e5, euclidean=True))
    if want("twolink_nu1"):
        # the nu = 1 variant of configs 1-2: f(x, [u₁, 0]), T = 50
        rng = np.random.default_rng(2025)
        twolink_case("twolink_nu1_t50", [[0.1, -0.1, 0.0, 0.0], rng.random(4), rng.random(4)], T=50, nu=1)
    if only:
        return
    # headline family, short horizon: the literal recursion is healthy for T ≲ 16 (rounding asymmetry grows ~3×/step)
    lq, x, u = quadrotor_batch(4, T=16, seed0=0)
    lq_case("quad_t16", lq, x, u)
    # headline family, full horizon: the literal recursion diverges (~step 32), so
    # the fixture uses the symmetrised oracle (identity in exact arithmetic)
    lq, x, u = quadrotor_batch(2, T=100, seed0=100)
    lq_case("quad_t100_sym", lq, x, u, symmetrize=True, fit_iters=12)
    # dense per-instance LQ with random initial controls
    lq, x, u = random_lq_batch(3, 12, 4, 16, seed=7)
    lq_case("dense_t16", lq, x, u)
    # dense, full horizon, symmetrised oracle
    lq, x, u = random_lq_batch(3, 12, 4, 64, seed=9)
    lq_case("dense_t64_sym", lq, x, u, symmetrize=True, fit_iters=12)
    # x_traj enters only the line-search objective (forward_pass.jl:187-190)
    lq, x, u = random_lq_batch(2, 12, 4, 16, seed=11)
    xtraj = 0.3 * np.random.default_rng(12).standard_normal(x.shape)
    lq_case("dense_xtraj", lq, x, u, xtraj=xtraj)
    # 2-link arm (test/2_link_example): animate_2_link.jl:13's x0 and two seeded rand(4)
    rng = np.random.default_rng(2024)
    twolink_case("twolink_t50", [[0.1, -0.1, 0.0, 0.0], rng.random(4), rng.random(4)], T=50)
    kat = {
        "alpha": O.TwoLink.alpha, "beta": O.TwoLink.beta, "delta": O.TwoLink.delta,
        "theta_star": O.TwoLink.inverse_kinematics(O.TwoLink.target_tool_loc).tolist(),
    }
    with open(os.path.join(HERE, "twolink_constants.json"), "w") as f:
        json.dump(kat, f, indent=1)


if __name__ == "__main__":
    main(tuple(sys.argv[1:]))
