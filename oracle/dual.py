"""Forward-mode dual-number AD for the CPU oracle — TEST INFRASTRUCTURE ONLY.

The reference differentiates every user closure with ForwardDiff.jl 0.10.14
(pinned at /root/reference docs/Manifest.toml:77-81; call sites
src/backward_pass.jl:32-33, :95-99, :142-143 and
test/2_link_example/2_link_helper_functions.jl:37). ForwardDiff is not
vendored and Julia is absent, so this module restates its published algorithm:
a value carries a vector of partials; `jacobian(f, x)` seeds x_i with the unit
partial e_i, evaluates f once and reads the partials back (matrix outputs are
vectorised column-major, Julia's `vec`); `gradient` is the scalar case;
`hessian(f, x)` = jacobian of gradient via nested duals.

Nesting follows ForwardDiff's tag rule: every derivative call gets a fresh,
larger tag; when two duals meet, the one with the larger (newer) tag is the
outer structure and the older one is a constant at that level, so an inner
derivative never reads an outer perturbation.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import anything under oracle/.
"""
from __future__ import annotations

import itertools
import math

import numpy as np

_TAGS = itertools.count(1)


class Dual:
    __slots__ = ("val", "der", "tag")

    def __init__(self, val, der, tag):
        self.val = val   # float, or an older-tag Dual
        self.der = der   # numpy array of partials (float or object dtype)
        self.tag = tag

    def _level(self, other):
        """(value, partials-or-None) of `other` at this dual's level, or None if
        `other` must handle the operation itself (ndarray, or newer tag)."""
        if isinstance(other, np.ndarray):
            return None
        if isinstance(other, Dual):
            if other.tag == self.tag:
                return other.val, other.der
            if other.tag > self.tag:
                return None
        return other, None

    def __add__(self, other):
        lv = self._level(other)
        if lv is None:
            return _defer(other, "__radd__", self)
        ov, od = lv
        return Dual(self.val + ov, self.der if od is None else self.der + od, self.tag)

    __radd__ = __add__

    def __neg__(self):
        return Dual(-self.val, -self.der, self.tag)

    def __pos__(self):
        return self

    def __sub__(self, other):
        lv = self._level(other)
        if lv is None:
            return _defer(other, "__rsub__", self)
        ov, od = lv
        return Dual(self.val - ov, self.der if od is None else self.der - od, self.tag)

    def __rsub__(self, other):
        lv = self._level(other)
        if lv is None:
            return _defer(other, "__sub__", self)
        ov, od = lv
        return Dual(ov - self.val, -self.der if od is None else od - self.der, self.tag)

    def __mul__(self, other):
        lv = self._level(other)
        if lv is None:
            return _defer(other, "__rmul__", self)
        ov, od = lv
        if od is None:
            return Dual(self.val * ov, self.der * ov, self.tag)
        return Dual(self.val * ov, self.der * ov + od * self.val, self.tag)

    def __rmul__(self, other):
        lv = self._level(other)
        if lv is None:
            return _defer(other, "__mul__", self)
        ov, od = lv
        if od is None:
            return Dual(ov * self.val, ov * self.der, self.tag)
        return Dual(ov * self.val, od * self.val + ov * self.der, self.tag)

    def __truediv__(self, other):
        lv = self._level(other)
        if lv is None:
            return _defer(other, "__rtruediv__", self)
        ov, od = lv
        v = self.val / ov
        if od is None:
            return Dual(v, self.der / ov, self.tag)
        return Dual(v, (self.der - od * v) / ov, self.tag)

    def __rtruediv__(self, other):
        lv = self._level(other)
        if lv is None:
            return _defer(other, "__truediv__", self)
        ov, od = lv
        v = ov / self.val
        if od is None:
            return Dual(v, self.der * (-v / self.val), self.tag)
        return Dual(v, (od - self.der * v) / self.val, self.tag)

    def __pow__(self, p):
        if p == 2:
            return self * self
        if isinstance(p, (int, float)):
            return Dual(self.val ** p, self.der * (p * self.val ** (p - 1)), self.tag)
        raise TypeError("Dual ** Dual is not used by the reference path")

    def __lt__(self, o):
        return primal(self) < primal(o)

    def __gt__(self, o):
        return primal(self) > primal(o)

    def __float__(self):
        return float(primal(self))

    def __repr__(self):
        return f"Dual[{self.tag}]({self.val!r}, {self.der!r})"


def _defer(other, method, me):
    # Python never tries the reflected method between two instances of one class,
    # so a newer-tag dual (the outer structure) is handed the operation directly.
    if isinstance(other, Dual):
        return getattr(other, method)(me)
    return NotImplemented


def primal(x):
    while isinstance(x, Dual):
        x = x.val
    return x


# -- elementary functions (DiffRules as used by ForwardDiff) ------------------------
def sin(x):
    if isinstance(x, Dual):
        return Dual(sin(x.val), x.der * cos(x.val), x.tag)
    return math.sin(x)


def cos(x):
    if isinstance(x, Dual):
        return Dual(cos(x.val), x.der * (-sin(x.val)), x.tag)
    return math.cos(x)


def sqrt(x):
    if isinstance(x, Dual):
        r = sqrt(x.val)
        return Dual(r, x.der / (2 * r), x.tag)
    return math.sqrt(x)


def acos(x):
    if isinstance(x, Dual):
        return Dual(acos(x.val), x.der * (-1.0 / sqrt(1 - x.val * x.val)), x.tag)
    return math.acos(x)


def atan2(y, x):
    if isinstance(y, Dual) or isinstance(x, Dual):
        raise NotImplementedError("atan2 of duals is not used by the reference path")
    return math.atan2(y, x)


# -- derivative drivers (ForwardDiff.jacobian / gradient / hessian) -----------------
def _seed(x):
    xs = list(np.asarray(x, dtype=object).reshape(-1))
    n = len(xs)
    tag = next(_TAGS)
    eye = np.eye(n)
    out = np.empty(n, dtype=object)
    for i, xi in enumerate(xs):
        out[i] = Dual(xi, eye[i].copy(), tag)
    return out, tag


def _partials(y, tag, n):
    if isinstance(y, Dual):
        if y.tag == tag:
            return list(y.der)
        if y.tag > tag:
            raise RuntimeError("perturbation confusion")
    return [0.0] * n


def _pack(rows):
    arr = np.empty((len(rows), len(rows[0]) if rows else 0), dtype=object)
    for i, r in enumerate(rows):
        for j, v in enumerate(r):
            arr[i, j] = v
    if all(not isinstance(v, Dual) for v in arr.flat):
        return arr.astype(float)
    return arr


def jacobian(f, x):
    xs, tag = _seed(x)
    y = np.asarray(f(xs), dtype=object)
    flat = y.flatten(order="F") if y.ndim > 1 else y.reshape(-1)
    return _pack([_partials(yi, tag, len(xs)) for yi in flat])


def gradient(f, x):
    xs, tag = _seed(x)
    y = f(xs)
    return _pack([_partials(y, tag, len(xs))])[0]


def hessian(f, x):
    return jacobian(lambda z: gradient(f, z), x)
