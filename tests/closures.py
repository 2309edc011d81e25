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
