"""Array-valued forward-mode AD for the CPU oracle — TEST INFRASTRUCTURE ONLY.

The same algorithm as oracle.dual (the restatement of ForwardDiff.jl 0.10.14's
`jacobian`, the reference's call at src/backward_pass.jl:32-33): every input
component is seeded with a unit partial, the closure is evaluated ONCE, and the
Jacobian is read from the output partials. The difference is the data layout: a
`Jet` is a whole numpy array `val` with its partials `der` stacked in front
(der.shape == (k,) + val.shape), so a closure written with array operations (slices,
`@`, `solve`, `sin`, `cat`) is differentiated at many points at once — every step
of every trajectory of a T = 1000 fit in one evaluation — where oracle.dual carries
one Python object per scalar. Only first derivatives (the cost Hessians of the
closures that use this come from their analytic `.quad` forms, cross-checked by
tests/test_closures.py).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
anything under oracle/.
"""
from __future__ import annotations

import numpy as np


class Jet:
    __slots__ = ("val", "der")
    __array_ufunc__ = None   # ndarray (op) Jet defers to Jet's reflected operators

    def __init__(self, val, der):
        self.val = np.asarray(val, dtype=np.float64)
        self.der = np.asarray(der, dtype=np.float64)

    # -- shape -----------------------------------------------------------------
    @property
    def shape(self):
        return self.val.shape

    @property
    def ndim(self):
        return self.val.ndim

    def __getitem__(self, idx):
        idx = idx if isinstance(idx, tuple) else (idx,)
        return Jet(self.val[idx], self.der[(slice(None),) + idx])

    def reshape(self, *shape):
        shape = shape[0] if len(shape) == 1 and isinstance(shape[0], tuple) else shape
        return Jet(self.val.reshape(shape), self.der.reshape((self.der.shape[0],) + tuple(shape)))

    def sum(self, axis=-1):
        ax = axis if axis < 0 else axis + 1
        return Jet(self.val.sum(axis=axis), self.der.sum(axis=ax))

    # -- arithmetic (broadcasting like numpy; the partials axis leads) -----------
    def __add__(self, o):
        if isinstance(o, Jet):
            return Jet(self.val + o.val, self.der + o.der)
        return Jet(self.val + o, np.broadcast_to(self.der, (self.der.shape[0],) +
                                                  np.broadcast_shapes(self.val.shape, np.shape(o))))

    __radd__ = __add__

    def __neg__(self):
        return Jet(-self.val, -self.der)

    def __sub__(self, o):
        return self + (-o)

    def __rsub__(self, o):
        return (-self) + o

    def __mul__(self, o):
        if isinstance(o, Jet):
            return Jet(self.val * o.val, self.der * o.val + self.val * o.der)
        return Jet(self.val * o, self.der * o)

    __rmul__ = __mul__

    def __truediv__(self, o):
        if isinstance(o, Jet):
            q = self.val / o.val
            return Jet(q, (self.der - q * o.der) / o.val)
        return Jet(self.val / o, self.der / o)

    def __rtruediv__(self, o):
        q = o / self.val
        return Jet(q, -q / self.val * self.der)

    def __pow__(self, k):
        assert k == 2
        return self * self

    def __matmul__(self, o):
        if isinstance(o, Jet):
            return Jet(self.val @ o.val, self.der @ o.val + self.val @ o.der)
        return Jet(self.val @ o, self.der @ o)

    def __rmatmul__(self, o):
        return Jet(o @ self.val, o @ self.der)

    @property
    def T(self):
        return Jet(np.swapaxes(self.val, -1, -2), np.swapaxes(self.der, -1, -2))


def _vd(a):
    return (a.val, a.der) if isinstance(a, Jet) else (np.asarray(a, dtype=np.float64), None)


def sin(a):
    if not isinstance(a, Jet):
        return np.sin(a)
    return Jet(np.sin(a.val), np.cos(a.val) * a.der)


def cos(a):
    if not isinstance(a, Jet):
        return np.cos(a)
    return Jet(np.cos(a.val), -np.sin(a.val) * a.der)


def cat(parts, axis=-1):
    """concatenate along a (negative) axis, Jets and constants mixed."""
    assert axis < 0
    if not any(isinstance(p, Jet) for p in parts):
        return np.concatenate([np.asarray(p, dtype=np.float64) for p in parts], axis=axis)
    k = next(p.der.shape[0] for p in parts if isinstance(p, Jet))
    vals, ders = [], []
    for p in parts:
        v, d = _vd(p)
        vals.append(v)
        ders.append(np.zeros((k,) + v.shape) if d is None else d)
    return Jet(np.concatenate(vals, axis=axis), np.concatenate(ders, axis=axis))


def tr(a):
    """swap the last two axes (a batched matrix transpose)."""
    return a.T if isinstance(a, Jet) else np.swapaxes(a, -1, -2)


def solve(M, b):
    """M⁻¹ b for a vector b (..., n): y = M⁻¹b, ẏ = M⁻¹(ḃ − Ṁ y) (LAPACK gesv per point)."""
    Mv, Md = _vd(M)
    bv, bd = _vd(b)
    y = np.linalg.solve(Mv, bv[..., None])[..., 0]
    if Md is None and bd is None:
        return y
    k = (Md if Md is not None else bd).shape[0]
    rhs = np.zeros((k,) + y.shape) if bd is None else np.array(bd, copy=True)
    if Md is not None:
        rhs = rhs - (Md @ y[..., None])[..., 0]
    dy = np.linalg.solve(np.broadcast_to(Mv, (k,) + Mv.shape), rhs[..., None])[..., 0]
    return Jet(y, dy)


def seed(xs):
    """Jets for the inputs xs (each (P, n_i)), partials over all their components
    stacked: the seeding of ForwardDiff's jacobian (one chunk holding every input)."""
    k = sum(x.shape[-1] for x in xs)
    out, o = [], 0
    for x in xs:
        n = x.shape[-1]
        d = np.zeros((k,) + x.shape)
        for j in range(n):
            d[o + j, ..., j] = 1.0
        out.append(Jet(x, d))
        o += n
    return out


def jacobians(f, x, u):
    """(∂f/∂x, ∂f/∂u) of f(x, u) at every point: x (P, nx), u (P, nu) → A (P, nx', nx),
    B (P, nx', nu) — linearize_dynamics (src/backward_pass.jl:25-40) at P points at once."""
    nx = x.shape[-1]
    xj, uj = seed([np.asarray(x, dtype=np.float64), np.asarray(u, dtype=np.float64)])
    y = f(xj, uj)
    J = np.moveaxis(y.der, 0, -1)          # (P, nx', nx + nu)
    return np.ascontiguousarray(J[..., :nx]), np.ascontiguousarray(J[..., nx:])
