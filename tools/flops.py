"""Algorithmic FLOP counts of the secondary configurations' dynamics, for the roofline
objects of tools/bench_twolink.py and tools/bench_rbd.py.

The count is taken by evaluating the restated reference formulas once on counting
scalars: `Flop` counts every +, −, ×, ÷ (and 1 per sin/cos) the formula performs; `FDual`
is a forward-mode dual over ND directions that counts what each primitive costs on its
value and partials (add 1+ND, multiply 1+3ND, divide 2+4ND, sin/cos 2+2ND, scaling
by a constant 1+ND) — the arithmetic ForwardDiff (and the device's Dual<N>) performs.
Central differences cost 2·ND primal evaluations plus ND divisions. These are counts of
the reference's arithmetic, not of the device's instruction stream (which reassociates,
fuses into FMAs and skips structural zeros).
"""
from __future__ import annotations

import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ilqr.jl_amd")]


class Counter:
    n = 0


class Flop:
    """A float that counts the arithmetic done on it."""
    __slots__ = ("v",)

    def __init__(self, v):
        self.v = float(v)

    @staticmethod
    def _v(o):
        return o.v if isinstance(o, Flop) else float(o)

    def _op(self, v, k=1):
        Counter.n += k
        return Flop(v)

    def __add__(self, o): return self._op(self.v + self._v(o))
    __radd__ = __add__
    def __sub__(self, o): return self._op(self.v - self._v(o))
    def __rsub__(self, o): return self._op(self._v(o) - self.v)
    def __mul__(self, o): return self._op(self.v * self._v(o))
    __rmul__ = __mul__
    def __truediv__(self, o): return self._op(self.v / self._v(o))
    def __rtruediv__(self, o): return self._op(self._v(o) / self.v)
    def __neg__(self): return Flop(-self.v)
    def sin(self): return self._op(math.sin(self.v))
    def cos(self): return self._op(math.cos(self.v))


def chain_dynamics_flops(problem):
    """Primal FLOPs of one RK4 step of the chain family (oracle/rbd.py's restatement of
    RBD_helper_functions.jl:48-79 on the fixed-base chain)."""
    from oracle import rbd
    m = rbd.ChainModel(problem.chain, problem.dt)
    x = [Flop(0.3 * (i + 1)) for i in range(problem.nx)]
    u = [Flop(0.1 * (i + 1)) for i in range(problem.nu)]
    Counter.n = 0
    m.dynamicsf(x, u)
    return Counter.n


# the 2-link arm's dynamicsf as the device functor evaluates it (ilqr_twolink.hip:
# continuous_dynamics + rk4, the formulas of 2_link_helper_functions.jl:29-79)
def twolink_dynamics_flops(nu=2):
    P_alpha, P_beta, P_delta, dt = 0.83, 0.25, 0.17, 0.01

    def cd(x, u):
        s2, c2 = x[1].sin(), x[1].cos()
        m00 = P_alpha + (2.0 * P_beta) * c2
        m01 = P_delta + P_beta * c2
        ns2 = -s2
        dm00 = (2.0 * P_beta) * ns2
        dm01 = P_beta * ns2
        c00 = (0.5 * dm00) * x[3]
        c01 = (0.5 * dm01) * x[3]
        det = P_delta * m00 - m01 * m01
        idet = 1.0 / det
        i00, i01, i11 = P_delta * idet, -(m01 * idet), m00 * idet
        mc00 = i00 * c00 + i01 * c01
        mc01 = i00 * c01
        mc10 = i01 * c00 + i11 * c01
        mc11 = i01 * c01
        u1 = u[1] if nu == 2 else 0.0
        return [x[2], x[3], -(mc00 * x[2] + mc01 * x[3]) + (i00 * u[0] + i01 * u1),
                -(mc10 * x[2] + mc11 * x[3]) + (i01 * u[0] + i11 * u1)]

    x = [Flop(0.1), Flop(-0.2), Flop(0.3), Flop(0.4)]
    u = [Flop(0.5), Flop(0.6)][:nu]
    Counter.n = 0
    k1 = [dt * v for v in cd(x, u)]
    k2 = [dt * v for v in cd([x[i] + 0.5 * k1[i] for i in range(4)], u)]
    k3 = [dt * v for v in cd([x[i] + 0.5 * k2[i] for i in range(4)], u)]
    k4 = [dt * v for v in cd([x[i] + k3[i] for i in range(4)], u)]
    [x[i] + (1.0 / 6.0) * (((k1[i] + 2.0 * k2[i]) + 2.0 * k3[i]) + k4[i]) for i in range(4)]
    return Counter.n


def chain_closed_form_flops(nu=1):
    """Primal FLOPs of one RK4 step of the 2-joint chain's closed form, the evaluator the
    iteration kernels run by default (ilqr_chain.hip chain_qdd_trig / chain_xdot_trig:
    M(q₂) and dM/dq₂ as trigonometric polynomials, bilinear gravity, the Christoffel
    velocity term, a 2×2 solve). The recursion's count (chain_dynamics_flops) is what the
    reference's RigidBodyDynamics.jl calls perform; the closed form does ~16× fewer, so
    a roofline priced on the recursion's count would exceed the peak."""
    Mc = [[Flop(0.1 * (e + 1) + 0.01 * k) for k in range(5)] for e in range(3)]
    Gc = [[[Flop(0.2 + 0.01 * (i + a + b)) for b in range(3)] for a in range(3)] for i in range(2)]
    dt = 0.01

    def xdot(x, u):
        s1, c1, s2, c2 = x[0].sin(), x[0].cos(), x[1].sin(), x[1].cos()
        w0, w1 = x[2], x[3]
        C2, S2 = c2 * c2 - s2 * s2, 2.0 * (s2 * c2)
        m, dm = [], []
        for e in range(3):
            m.append(Mc[e][0] + (((Mc[e][1] * c2 + Mc[e][2] * s2) + Mc[e][3] * C2) + Mc[e][4] * S2))
            dm.append((Mc[e][2] * c2 - Mc[e][1] * s2) + 2.0 * (Mc[e][4] * C2 - Mc[e][3] * S2))
        g = []
        for i in range(2):
            h = [Gc[i][a][0] + (Gc[i][a][1] * c2 + Gc[i][a][2] * s2) for a in range(3)]
            g.append(h[0] + (h[1] * c1 + h[2] * s1))
        p0, p1 = dm[0] * w0 + dm[1] * w1, dm[1] * w0 + dm[2] * w1
        qq = w0 * p0 + w1 * p1
        r0 = u[0] - (w1 * p0 + g[0])
        r1 = (w1 * p1 - 0.5 * qq) + g[1]
        r1 = u[-1] - r1 if nu > 1 else -r1
        idet = 1.0 / (m[0] * m[2] - m[1] * m[1])
        return [w0, w1, (m[2] * r0 - m[1] * r1) * idet, (m[0] * r1 - m[1] * r0) * idet]

    x = [Flop(0.3), Flop(-0.4), Flop(0.5), Flop(0.6)]
    u = [Flop(0.1), Flop(0.2)][:nu]
    Counter.n = 0
    k1 = [dt * v for v in xdot(x, u)]
    k2 = [dt * v for v in xdot([x[i] + 0.5 * k1[i] for i in range(4)], u)]
    k3 = [dt * v for v in xdot([x[i] + 0.5 * k2[i] for i in range(4)], u)]
    k4 = [dt * v for v in xdot([x[i] + k3[i] for i in range(4)], u)]
    [x[i] + (1.0 / 6.0) * (((k1[i] + 2.0 * k2[i]) + 2.0 * k3[i]) + k4[i]) for i in range(4)]
    return Counter.n


def dual_factor(nd):
    """FLOPs of a forward-mode dual evaluation per primal FLOP (mix-weighted average of
    add 1+ND, mul 1+3ND, div 2+4ND, constant scaling 1+ND): ~1 + 2ND."""
    return 1.0 + 2.0 * nd


def riccati_flops_per_step(n, m):
    """SURVEY.md §8(d)'s backward-step count (FMA × 2)."""
    return 2 * (2 * n**3 + 4 * n * n * m + 2 * n * m * m + 2 * n * n + 4 * n * m + m**3 / 3 + (n + 3) * m * m)


def forward_flops_per_step(n, m, f_dyn):
    """One line-search trial step: the control law (2nm + 2m), the dynamics, the stage
    cost (≈ 3n + 3m for the diagonal costs of these families)."""
    return 2 * n * m + 2 * m + f_dyn + 3 * n + 3 * m


if __name__ == "__main__":
    from ilqr_amd.chain import rbd_2dof_problem
    for nu in (2, 1):
        print("2-link nu", nu, "RK4 flops", twolink_dynamics_flops(nu))
        print("chain 2dof nu", nu, "RK4 flops", chain_dynamics_flops(rbd_2dof_problem(nu)),
              "closed form", chain_closed_form_flops(nu))
