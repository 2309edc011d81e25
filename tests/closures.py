"""Nonlinear test problems written once against a tiny math namespace, so the same
closure runs as torch code (the device path's generic-closure mode) and on the
oracle's dual numbers (oracle.dual, the ForwardDiff restatement). Test helper."""
from __future__ import annotations

import types

import numpy as np


def torch_ns():
    import torch
    return types.SimpleNamespace(sin=torch.sin, cos=torch.cos, stack=torch.stack)


def oracle_ns():
    from oracle import dual
    return types.SimpleNamespace(sin=dual.sin, cos=dual.cos,
                                 stack=lambda v: np.array(list(v), dtype=object))


def coupled_pendula(ns, dt=0.05):
    """Two coupled pendula, nx = 4, nu = 2, explicit Euler; a cost with
    state-input cross terms (𝐏 ≠ 0) and a nonlinear term."""
    def dynamicsf(x, u):
        th1, th2, w1, w2 = x[0], x[1], x[2], x[3]
        cpl = ns.sin(th1 - th2)
        a1 = -9.81 * ns.sin(th1) - 0.4 * cpl * w2 * w2 - 0.1 * w1 + u[0]
        a2 = -9.81 * ns.sin(th2) + 0.4 * cpl * w1 * w1 - 0.1 * w2 + u[1] * ns.cos(th2)
        return ns.stack([th1 + dt * w1, th2 + dt * w2, w1 + dt * a1, w2 + dt * a2])

    def immediate_cost(x, u):
        return (0.5 * (x[0] * x[0] + x[1] * x[1]) + 0.1 * (x[2] * x[2] + x[3] * x[3])
                + u[0] * u[0] + u[1] * u[1] + 0.2 * u[0] * x[2] + 0.1 * ns.sin(x[0]) * u[1])

    def final_cost(x):
        return 5.0 * (x[0] * x[0] + x[1] * x[1]) + x[2] * x[2] + x[3] * x[3]

    return dynamicsf, immediate_cost, final_cost


def two_link_torch():
    """test/2_link_example/2_link_helper_functions.jl's arm written with torch ops
    (the Coriolis quirk included) — what a user of the generic path would write."""
    import math

    import torch
    l1 = l2 = math.sqrt(2.0) / 2.0
    r2 = 0.5 * l2
    Iz1 = Iz2 = 1.0 / 12.0 * l1 ** 2
    al = Iz1 + Iz2 + (0.5 * l1) ** 2 + (l1 ** 2 + r2 ** 2)
    be = l1 * r2
    de = Iz2 + r2 ** 2
    x_, y_ = 0.6, -0.5
    q2 = math.acos((x_ ** 2 + y_ ** 2 - l1 ** 2 - l2 ** 2) / (2 * l1 * l2))
    q1 = math.atan2(y_, x_) - math.atan2(l2 * math.sin(q2), l1 + l2 * math.cos(q2))

    def cd(s, w):
        c2, s2 = torch.cos(s[1]), torch.sin(s[1])
        m00, m01 = al + 2 * be * c2, de + be * c2
        c00, c01 = 0.5 * (2 * be * -s2) * s[3], 0.5 * (be * -s2) * s[3]
        det = m00 * de - m01 * m01
        i00, i01, i11 = de / det, -m01 / det, m00 / det
        a0 = -((i00 * c00 + i01 * c01) * s[2] + (i00 * c01) * s[3]) + (i00 * w[0] + i01 * w[1])
        a1 = -((i01 * c00 + i11 * c01) * s[2] + (i01 * c01) * s[3]) + (i01 * w[0] + i11 * w[1])
        return torch.stack([s[2], s[3], a0, a1])

    def dynamicsf(x, u):
        dt = 0.01
        k1 = dt * cd(x, u)
        k2 = dt * cd(x + k1 / 2, u)
        k3 = dt * cd(x + k2 / 2, u)
        k4 = dt * cd(x + k3, u)
        return x + (1 / 6) * (k1 + 2 * k2 + 2 * k3 + k4)

    def immediate_cost(x, u):
        return ((q1 - x[0]) ** 2 + (q2 - x[1]) ** 2) * 1.0 + (u[0] ** 2 + u[1] ** 2) * 1.0

    def final_cost(x):
        return ((q1 - x[0]) ** 2 + (q2 - x[1]) ** 2) * 1.0

    return dynamicsf, immediate_cost, final_cost


# -- the reference's RBD example, floating base -------------------------------------
def jet_ns():
    """numpy arrays and oracle.jet Jets (array-valued forward-mode AD)."""
    from oracle import jet
    return types.SimpleNamespace(sin=jet.sin, cos=jet.cos, cat=jet.cat, solve=jet.solve, tr=jet.tr,
                                 const=lambda a: np.asarray(a, dtype=np.float64))


def torch_arr_ns(device="cuda"):
    import torch
    return types.SimpleNamespace(
        sin=torch.sin, cos=torch.cos, cat=lambda parts, axis=-1: torch.cat(parts, dim=axis),
        solve=lambda M, b: torch.linalg.solve(M, b.unsqueeze(-1)).squeeze(-1),
        tr=lambda a: a.transpose(-1, -2),
        const=lambda a: torch.as_tensor(np.asarray(a, dtype=np.float64), device=device))


def _skew(a):
    return np.array([[0.0, -a[2], a[1]], [a[2], 0.0, -a[0]], [-a[1], a[0], 0.0]])


def _skew_basis():
    """E (9, 3) with (E @ a).reshape(3, 3) = [a×]."""
    return np.stack([_skew(e).ravel() for e in np.eye(3)], axis=1)


def _crm_basis():
    """E (36, 6) with (E @ v).reshape(6, 6) = crm(v) = [[ω×, 0], [v×, ω×]] (Featherstone)."""
    cols = []
    for e in np.eye(6):
        m = np.zeros((6, 6))
        m[:3, :3] = m[3:, 3:] = _skew(e[:3])
        m[3:, :3] = _skew(e[3:])
        cols.append(m.ravel())
    return np.stack(cols, axis=1)


ARM_2DOF = {  # test/urdf/2Dof_arm.urdf (ilqr_amd/robots/2dof_arm.json)
    "base_mass": 30.0, "base_com": (0.0, 0.0, 0.0), "base_Ic": 50.0 * np.eye(3),
    "R0": (np.eye(3), np.eye(3)), "p": ((0.5, 0.5, 0.0), (1.0, 0.0, 0.0)),
    "axis": ((0.0, 0.0, 1.0), (0.0, 1.0, 0.0)), "mass": (3.0, 3.0),
    "com": ((0.0, 0.0, 0.0), (0.0, 0.0, 0.0)), "Ic": (0.5 * np.eye(3), 0.5 * np.eye(3))}


def spatial_inertia(m, c, Ic):
    """Featherstone's rigid-body inertia about the body origin, angular first:
    [[Ic + m[c×][c×]ᵀ, m[c×]], [m[c×]ᵀ, m1]]."""
    cx = _skew(np.asarray(c, float))
    return np.block([[np.asarray(Ic, float) + m * cx @ cx.T, m * cx], [m * cx.T, m * np.eye(3)]])


def rbd_floating_arm(ns, dt=0.01, model=None):
    """test/RBD_2_link_example/RBD_helper_functions.jl:48-116 written with array ops —
    the closures a user of the generic path would write for animate_RBD_2_link.jl:
    nx = 16 ([MRP p (3); base position r (3); θ (2); ω (3); v (3); θ̇ (2)]), nu = 8
    (base torque (3), base force (3), joint torques (2)).

    The mechanism is test/urdf/2Dof_arm.urdf parsed floating with zero gravity (:6-8):
    a 30 kg base (I = 50·1), link_1 at (.5, .5, 0) about z, link_2 at (1, 0, 0) of
    link_1 about y, 3 kg and I = .5·1 each, COMs on the joint origins. RigidBodyDynamics.jl
    (absent) is restated with Featherstone's algorithms in body coordinates: the mass
    matrix by the composite-rigid-body algorithm, dynamics_bias by recursive
    Newton-Euler at zero acceleration; the base twist (ω, v) is body-frame, angular
    first (RBD.jl's QuaternionFloating). The reference's kinematics (:64) are kept as
    written: q̇ = [pdot_from_w(p, ω); v; θ̇] (Attitude.jl's MRP rate; the base position
    integrates v as is). Parity vs RigidBodyDynamics.jl: unpinned (not runnable here).
    Works on 1-D tensors (torch.func) and on (P, n) numpy arrays / oracle.jet Jets."""
    md = ARM_2DOF if model is None else model
    if model is None:
        I0 = np.diag([50.0, 50.0, 50.0, 30.0, 30.0, 30.0])
        I1 = I2 = np.diag([0.5, 0.5, 0.5, 3.0, 3.0, 3.0])
    else:  # another mechanism of the same shape (a floating base, two revolute joints)
        I0 = spatial_inertia(md["base_mass"], md["base_com"], md["base_Ic"])
        I1, I2 = (spatial_inertia(md["mass"][i], md["com"][i], md["Ic"][i]) for i in (0, 1))

    def joint(r, a, R0):
        r, a, R0 = np.asarray(r, float), np.asarray(a, float), np.asarray(R0, float)
        Xt = np.eye(6)
        Xt[3:, :3] = -_skew(r)
        aa = np.outer(a, a)
        bd = lambda m: np.block([[m, np.zeros((3, 3))], [np.zeros((3, 3)), m]])  # noqa: E731
        S = np.concatenate([a, np.zeros(3)])
        # X(θ) = blockdiag(E, E)·Xt, E = (R0·Rot(a, θ))ᵀ = (cos θ (1 − aaᵀ) − sin θ [a×] + aaᵀ)·R0ᵀ
        return bd((np.eye(3) - aa) @ R0.T) @ Xt, bd(-_skew(a) @ R0.T) @ Xt, bd(aa @ R0.T) @ Xt, S

    C1a, C1b, C1c, S1n = joint(md["p"][0], md["axis"][0], md["R0"][0])
    C2a, C2b, C2c, S2n = joint(md["p"][1], md["axis"][1], md["R0"][1])
    m22 = float(S2n @ I2 @ S2n)
    K = ns.const
    I0c, I1c, I2c = K(I0), K(I1), K(I2)
    C1a, C1b, C1c, C2a, C2b, C2c = (K(a) for a in (C1a, C1b, C1c, C2a, C2b, C2c))
    S1, S2 = K(S1n), K(S2n)
    F2 = K(I2 @ S2n)
    ECRM, ESKEW = K(_crm_basis()), K(_skew_basis())
    target = K([0.0, 0.0, 0.0, 5.0, 1.0, 2.0, 1.0, 0.3])             # animate_RBD_2_link.jl:10
    Qw = K([100.0, 100.0, 100.0, 1.0, 1.0, 1.0, 10.0, 10.0])           # :89-91
    Rw = K([1.0, 1.0, 1.0, 100.0, 100.0, 100.0, 10.0, 10.0])           # :96-97
    Qfw = K([100.0, 100.0, 100.0, 1000.0, 1000.0, 1000.0, 10.0, 10.0])  # :111-112

    def mv(M, v):
        return (M @ v[..., None])[..., 0]

    def crm(v):
        w = mv(ECRM, v)
        return w.reshape(tuple(w.shape[:-1]) + (6, 6))

    def cross(a, b):
        w = mv(ESKEW, a)
        return mv(w.reshape(tuple(w.shape[:-1]) + (3, 3)), b)

    def xform(c, s, Ca, Cb, Cc):
        return c[..., None, None] * Ca + s[..., None, None] * Cb + Cc

    def kinematics(x):
        th = x[..., 6:8]
        X1 = xform(ns.cos(th[..., 0]), ns.sin(th[..., 0]), C1a, C1b, C1c)
        X2 = xform(ns.cos(th[..., 1]), ns.sin(th[..., 1]), C2a, C2b, C2c)
        return X1, X2, ns.tr(X1), ns.tr(X2)

    def mass_matrix(x, kin=None):                                      # :60, CRBA
        X1, X2, X1T, X2T = kin if kin is not None else kinematics(x)
        Ic1 = I1c + X2T @ I2c @ X2
        Ic0 = I0c + X1T @ Ic1 @ X1
        F1 = mv(Ic1, S1)
        F21 = mv(X2T, F2)
        m11 = (F1 * S1).sum(-1)[..., None, None]
        m12 = (F21 * S1).sum(-1)[..., None, None]
        M01, M02 = mv(X1T, F1), mv(X1T, F21)
        top = ns.cat([Ic0, M01[..., :, None], M02[..., :, None]])
        r6 = ns.cat([M01[..., None, :], m11, m12])
        r7 = ns.cat([M02[..., None, :], m12, m12 * 0.0 + m22])
        return ns.cat([top, r6, r7], axis=-2)

    def dynamics_bias(x, kin=None):                                    # :64, RNEA at q̈ = 0
        X1, X2, X1T, X2T = kin if kin is not None else kinematics(x)
        w, vl, thd = x[..., 8:11], x[..., 11:14], x[..., 14:16]
        v0 = ns.cat([w, vl])
        v1 = mv(X1, v0) + S1 * thd[..., 0:1]
        v2 = mv(X2, v1) + S2 * thd[..., 1:2]
        a1 = mv(crm(v1), S1) * thd[..., 0:1]
        a2 = mv(X2, a1) + mv(crm(v2), S2) * thd[..., 1:2]
        f2 = mv(I2c, a2) - mv(ns.tr(crm(v2)), mv(I2c, v2))
        f1 = mv(I1c, a1) - mv(ns.tr(crm(v1)), mv(I1c, v1)) + mv(X2T, f2)
        f0 = -mv(ns.tr(crm(v0)), mv(I0c, v0)) + mv(X1T, f1)
        return ns.cat([f0, (f1 * S1).sum(-1)[..., None], (f2 * S2).sum(-1)[..., None]])

    def continuous_dynamics(x, u):                                     # :52-68
        p, w, vl, thd = x[..., 0:3], x[..., 8:11], x[..., 11:14], x[..., 14:16]
        kin = kinematics(x)
        M = mass_matrix(x, kin)
        vdot = ns.solve(M, u - dynamics_bias(x, kin))                  # :64
        pp = (p * p).sum(-1)[..., None]
        pw = (p * w).sum(-1)[..., None]
        pdot = 0.25 * ((1.0 - pp) * w + 2.0 * cross(p, w) + 2.0 * pw * p)   # pdot_from_w
        return ns.cat([pdot, vl, thd, vdot])                           # :65-67

    def dynamicsf(x, u):                                               # RK4, :70-78
        k1 = dt * continuous_dynamics(x, u)
        k2 = dt * continuous_dynamics(x + k1 / 2, u)
        k3 = dt * continuous_dynamics(x + k2 / 2, u)
        k4 = dt * continuous_dynamics(x + k3, u)
        return x + (1 / 6) * (k1 + 2 * k2 + 2 * k3 + k4)

    def immediate_cost(x, u):                                          # :85-101
        dx = target - x[..., 0:8]
        return (dx * Qw * dx).sum(-1) * 10.0 + (u * Rw * u).sum(-1) * 1.0

    def final_cost(x):                                                 # :107-116
        dx = target - x[..., 0:8]
        return (dx * Qfw * dx).sum(-1) * 100000.0

    dynamicsf.mass_matrix, dynamicsf.dynamics_bias = mass_matrix, dynamics_bias
    return dynamicsf, immediate_cost, final_cost


def rbd_initial_state():
    """RBD_to_iLQR_state of set_configuration!(state, [0,0,0,1, .5,.75,1, 0,0]) at rest
    (RBD_helper_functions.jl:9, :26-29; animate_RBD_2_link.jl:22): quaternion (0, 0, 0, 1)
    → MRP p = q_v / (1 + q_s) = (0, 0, 1)."""
    return np.array([0.0, 0.0, 1.0, 0.5, 0.75, 1.0, 0.0, 0.0] + [0.0] * 8)


def rbd_cost_quads():
    """Exact quadratizations of rbd_floating_arm's costs (RBD_helper_functions.jl:85-116
    are weighted sums of squares): what ForwardDiff's gradient / hessian return, batched
    over points — lx, lu, lxx, lux (= 0), luu and lfx, lfxx."""
    tgt = np.array([0.0, 0.0, 0.0, 5.0, 1.0, 2.0, 1.0, 0.3])
    Qw = np.array([100.0, 100.0, 100.0, 1.0, 1.0, 1.0, 10.0, 10.0])
    Rw = np.array([1.0, 1.0, 1.0, 100.0, 100.0, 100.0, 10.0, 10.0])
    Qfw = np.array([100.0, 100.0, 100.0, 1000.0, 1000.0, 1000.0, 10.0, 10.0])

    def quad(x, u):
        P = x.shape[0]
        lx = np.zeros((P, 16))
        lx[:, :8] = -20.0 * Qw * (tgt - x[:, :8])
        lxx = np.zeros((P, 16, 16))
        lxx[:, np.arange(8), np.arange(8)] = 20.0 * Qw
        luu = np.broadcast_to(np.diag(2.0 * Rw), (P, 8, 8)).copy()
        return lx, 2.0 * Rw * u, lxx, np.zeros((P, 8, 16)), luu

    def fquad(xN):
        P = xN.shape[0]
        lfx = np.zeros((P, 16))
        lfx[:, :8] = -200000.0 * Qfw * (tgt - xN[:, :8])
        lfxx = np.zeros((P, 16, 16))
        lfxx[:, np.arange(8), np.arange(8)] = 200000.0 * Qfw
        return lfx, lfxx
    return quad, fquad


def coupled_pendula_arr(ns, dt=0.05):
    """coupled_pendula's dynamics written on arrays (x[..., i]): the same arithmetic in the
    same order, for batched numpy / oracle.jet evaluation."""
    def dynamicsf(x, u):
        th1, th2, w1, w2 = x[..., 0], x[..., 1], x[..., 2], x[..., 3]
        cpl = ns.sin(th1 - th2)
        a1 = -9.81 * ns.sin(th1) - 0.4 * cpl * w2 * w2 - 0.1 * w1 + u[..., 0]
        a2 = -9.81 * ns.sin(th2) + 0.4 * cpl * w1 * w1 - 0.1 * w2 + u[..., 1] * ns.cos(th2)
        return ns.cat([(th1 + dt * w1)[..., None], (th2 + dt * w2)[..., None],
                       (w1 + dt * a1)[..., None], (w2 + dt * a2)[..., None]])

    def immediate_cost(x, u):
        return (0.5 * (x[..., 0] * x[..., 0] + x[..., 1] * x[..., 1]) + 0.1 * (x[..., 2] * x[..., 2] + x[..., 3] * x[..., 3])
                + u[..., 0] * u[..., 0] + u[..., 1] * u[..., 1] + 0.2 * u[..., 0] * x[..., 2]
                + 0.1 * ns.sin(x[..., 0]) * u[..., 1])

    def final_cost(x):
        return 5.0 * (x[..., 0] * x[..., 0] + x[..., 1] * x[..., 1]) + x[..., 2] * x[..., 2] + x[..., 3] * x[..., 3]

    return dynamicsf, immediate_cost, final_cost


def coupled_floating_model():
    """A floating two-joint mechanism without the 2Dof_arm's symmetries (not a reference
    robot): the base's COM off its origin with products of inertia, joint 1 tilted about
    x, joint 2 turned about z with an oblique axis, COMs off the joint origins,
    anisotropic link inertias — every term of the floating-base dynamics nonzero."""
    def rx(a):
        c, s = np.cos(a), np.sin(a)
        return np.array([[1.0, 0.0, 0.0], [0.0, c, -s], [0.0, s, c]])

    def rz(a):
        c, s = np.cos(a), np.sin(a)
        return np.array([[c, -s, 0.0], [s, c, 0.0], [0.0, 0.0, 1.0]])
    ax2 = np.array([0.0, 1.0, 0.2]) / np.linalg.norm([0.0, 1.0, 0.2])
    return {"base_mass": 20.0, "base_com": (0.1, -0.05, 0.02),
            "base_Ic": np.array([[8.0, 0.3, -0.2], [0.3, 6.0, 0.1], [-0.2, 0.1, 7.0]]),
            "R0": (rx(0.3), rz(0.2)), "p": ((0.5, 0.5, 0.0), (1.0, 0.0, 0.1)),
            "axis": ((0.0, 0.0, 1.0), tuple(ax2)), "mass": (3.0, 2.0),
            "com": ((0.10, 0.05, 0.20), (0.30, 0.05, -0.15)),
            "Ic": (np.array([[0.40, 0.02, 0.01], [0.02, 0.60, 0.03], [0.01, 0.03, 0.30]]),
                   np.array([[0.20, 0.01, -0.02], [0.01, 0.35, 0.015], [-0.02, 0.015, 0.25]]))}


def floating_energy(x, model=None):
    """½ vᵀ M(θ) v of floating states x (P, 16) under rbd_floating_arm's model: conserved
    by the continuous dynamics at u = 0 and zero gravity (a check that the mass matrix
    and the bias are one mechanism's)."""
    ns = jet_ns()
    f, _, _ = rbd_floating_arm(ns, model=model)
    M = f.mass_matrix(np.asarray(x, float))
    v = np.asarray(x, float)[:, 8:16]
    return 0.5 * np.einsum("pi,pij,pj->p", v, M, v)


# -- an independent formulation of the floating mechanism ----------
def _rodrigues(a, th):
    """Rot(a, θ) = 1 + sin θ [a×] + (1 − cos θ)[a×]² (a unit)."""
    ax = _skew(np.asarray(a, float))
    return np.eye(3) + np.sin(th) * ax + (1.0 - np.cos(th)) * ax @ ax


def floating_mass_matrix_jacobians(x, model=None):
    """M(q) of rbd_floating_arm's mechanism as Σᵢ mᵢ Jvᵢᵀ Jvᵢ + Jωᵢᵀ (Rᵢ Icᵢ Rᵢᵀ) Jωᵢ: the
    kinetic energy ½ vᵀ M v summed over the three bodies from each body's COM velocity
    and angular velocity. Nothing of the CRBA / spatial-algebra restatement is used:
    the bodies' poses come from composing the URDF transforms (joint origin p, fixed
    rotation R0, Rodrigues rotation about the axis) as 3×3 rotations and 3-vectors, and
    the Jacobians from the geometric rule v_c = v₀ + ω₀ × c + Σ_joints (aⱼ θ̇ⱼ) × (c − oⱼ).
    Everything is expressed in the base frame, where the base twist (ω₀, v₀) of the
    generalised velocity lives (body-frame twist, angular first; x[8:16] = [ω₀, v₀, θ̇]).
    x: (P, 16) → (P, 8, 8)."""
    md = ARM_2DOF if model is None else model
    x = np.asarray(x, float)
    out = np.zeros((x.shape[0], 8, 8))
    cb = np.asarray(md["base_com"], float)
    for k, xk in enumerate(x):
        th = xk[6:8]
        Js = []   # (m, Jv (3, 8), Jw (3, 8), R, Ic) per body
        # base: COM velocity v₀ + ω₀ × c = v₀ − [c×] ω₀
        Jv = np.zeros((3, 8))
        Jw = np.zeros((3, 8))
        Jv[:, 0:3] = -_skew(cb)
        Jv[:, 3:6] = np.eye(3)
        Jw[:, 0:3] = np.eye(3)
        Js.append((md["base_mass"], Jv, Jw, np.eye(3), np.asarray(md["base_Ic"], float)))
        R, o = np.eye(3), np.zeros(3)            # the parent body's pose in the base frame
        axes = []                                 # (joint origin, world-of-base axis)
        for j in range(2):
            Rj0 = R @ np.asarray(md["R0"][j], float)
            o = o + R @ np.asarray(md["p"][j], float)
            axes.append((o.copy(), Rj0 @ np.asarray(md["axis"][j], float)))  # Rot(a, θ) a = a
            R = Rj0 @ _rodrigues(md["axis"][j], th[j])
            c = o + R @ np.asarray(md["com"][j], float)
            Jv = np.zeros((3, 8))
            Jw = np.zeros((3, 8))
            Jv[:, 0:3] = -_skew(c)
            Jv[:, 3:6] = np.eye(3)
            Jw[:, 0:3] = np.eye(3)
            for i, (oi, ai) in enumerate(axes):
                Jv[:, 6 + i] = np.cross(ai, c - oi)
                Jw[:, 6 + i] = ai
            Js.append((md["mass"][j], Jv, Jw, R, np.asarray(md["Ic"][j], float)))
        for m, Jv, Jw, Rb, Ic in Js:
            out[k] += m * Jv.T @ Jv + Jw.T @ (Rb @ Ic @ Rb.T) @ Jw
    return out


def mrp_to_dcm(p):
    """Body-to-world rotation of MRPs p (P, 3) (the attitude kinematics rbd_floating_arm
    integrates, pdot_from_w): R = 1 + (8[p×]² + 4(1 − pᵀp)[p×]) / (1 + pᵀp)²."""
    p = np.asarray(p, float)
    out = np.zeros((p.shape[0], 3, 3))
    for k, pk in enumerate(p):
        S = _skew(pk)
        pp = float(pk @ pk)
        out[k] = np.eye(3) + (8.0 * S @ S + 4.0 * (1.0 - pp) * S) / (1.0 + pp) ** 2
    return out


def floating_linear_momentum_world(x, model=None, M=None):
    """The mechanism's total linear momentum in the world frame: R(p) · (M(q) v)[3:6]
    (the base rows of M v are the system's spatial momentum in the base frame). Conserved
    at u = 0 with zero gravity. x: (P, 16) → (P, 3)."""
    x = np.asarray(x, float)
    M = floating_mass_matrix_jacobians(x, model) if M is None else M
    h = np.einsum("pij,pj->pi", M, x[:, 8:16])
    return np.einsum("pij,pj->pi", mrp_to_dcm(x[:, 0:3]), h[:, 3:6])
