"""Restatement of ilqr.jl_amd/julia/iLQRHIP.jl's memory-layout conventions on numpy
arrays, for tests/test_gpu_julia_layout.py (Julia is not installed here).

A Julia `Array` is column-major, and `ccall` passes a pointer to that memory. Here a
Julia array of shape (d1, d2, ...) is a Fortran-ordered numpy array of the same shape;
`memory(a)` is the flat buffer `ccall` would hand to the C ABI and `from_memory` reads a
buffer back into a Julia-shaped array. The functions below are the shim's, line for
line: `permutedims(a, perm)` is np.transpose with the 1-based perm made 0-based.
"""
import ctypes as C

import numpy as np

from ilqr_amd import _lib
from oracle import dual


def jl(a):
    """A Julia array with this shape and these values."""
    return np.asfortranarray(np.asarray(a, dtype=np.float64))


def memory(a):
    """The column-major buffer a Julia array occupies (what ccall passes)."""
    return np.asarray(a).ravel(order="F").copy()


def from_memory(buf, shape):
    """Julia's `download!(h, zeros(shape...), p)`: the buffer as a column-major array."""
    return np.asfortranarray(np.asarray(buf).reshape(shape, order="F"))


def permutedims(a, perm=(2, 1)):
    return np.asfortranarray(np.transpose(a, [p - 1 for p in perm]))


# -- iLQRHIP.jl: layouts ------------------------------------------------------------
def to_abi(x):                      # Array{Float64}(permutedims(x))
    return permutedims(jl(x))


def from_abi(a):                    # permutedims(a)
    return permutedims(a)


def gains_from_abi(K):              # permutedims(K, (3, 2, 1))
    return permutedims(K, (3, 2, 1))


def gains_to_abi(K):                # Array{Float64}(permutedims(K, (3, 2, 1)))
    return permutedims(jl(K), (3, 2, 1))


def rowmajor(M):                    # Array{Float64}(permutedims(M))
    return permutedims(jl(M))


def rowmajor3(A):                   # Array{Float64}(permutedims(A, (2, 1, 3)))
    return permutedims(jl(A), (2, 1, 3))


def derivative_tiles(x, u, f, l, lf):
    """iLQRHIP.derivative_tiles with the oracle's forward-mode duals (oracle.dual, the
    ForwardDiff restatement) in place of ForwardDiff: per step, the transposes of the
    reference's jacobian/gradient/hessian results (backward_pass.jl:32-33, 95-99,
    142-143) stored in Julia arrays (nx, nx, M), (nu, nx, M), (nx, M), ..."""
    x, u = np.asarray(x, float), np.asarray(u, float)
    N, nx = x.shape
    M, nu = u.shape
    A = jl(np.zeros((nx, nx, M))); B = jl(np.zeros((nu, nx, M)))
    lx = jl(np.zeros((nx, M))); lu = jl(np.zeros((nu, M)))
    lxx = jl(np.zeros((nx, nx, M))); lux = jl(np.zeros((nx, nu, M))); luu = jl(np.zeros((nu, nu, M)))
    for i in range(M):
        xi, ui = x[i], u[i]
        A[:, :, i] = dual.jacobian(lambda z: f(z, ui), xi).T
        B[:, :, i] = dual.jacobian(lambda v: f(xi, v), ui).T
        dLdu = lambda z, v: dual.gradient(lambda w: l(z, w), v)  # noqa: E731
        lx[:, i] = dual.gradient(lambda z: l(z, ui), xi)
        lu[:, i] = dLdu(xi, ui)
        lxx[:, :, i] = dual.hessian(lambda z: l(z, ui), xi).T
        lux[:, :, i] = dual.jacobian(lambda z: dLdu(z, ui), xi).T
        luu[:, :, i] = dual.hessian(lambda v: l(xi, v), ui).T
    xN = x[N - 1]
    return dict(A=A, B=B, lx=lx, lu=lu, lxx=lxx, lux=lux, luu=luu, lfx=jl(dual.gradient(lf, xN)),
                lfxx=jl(dual.hessian(lf, xN).T))


# -- iLQRHIP.jl: the floating-base model ----------------------------------------------

def rbd_2dof_arm_floating(target=(0., 0., 0., 5., 1., 2., 1., .3)):
    """The shim's rbd_2dof_arm_floating() (ilqr.jl_amd/julia/iLQRHIP.jl:958-966), field
    for field, as the ctypes struct ccall would pass by Ref."""
    I3 = (1., 0., 0., 0., 1., 0., 0., 0., 1.)
    vals = [2, 0.01, (0., 0., 0.), 30.0, (0., 0., 0.), tuple(50.0 * v for v in I3),
            I3 + I3, (.5, .5, 0., 1., 0., 0.), (0., 0., 1., 0., 1., 0.),
            (3.0, 3.0), (0.0,) * 6, tuple(0.5 * v for v in I3) * 2,
            tuple(float(v) for v in target), (100., 100., 100., 1., 1., 1., 10., 10.),
            (1., 1., 1., 100., 100., 100., 10., 10.),
            (100., 100., 100., 1000., 1000., 1000., 10., 10.), 10.0, 1.0, 100000.0]
    s = _lib.FloatingStruct()
    for (name, ty), v in zip(_lib.FloatingStruct._fields_, vals):
        if isinstance(v, tuple):
            n = C.sizeof(ty) // 8
            assert len(v) == n, name
            C.memmove(C.addressof(s) + getattr(_lib.FloatingStruct, name).offset,
                      (C.c_double * n)(*v), 8 * n)
        else:
            setattr(s, name, v)
    return s
