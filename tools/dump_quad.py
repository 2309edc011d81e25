"""Writes tools/quad256.bin for tools/bw4_probe.hip (not part of the product): the
headline quadrotor batch (256 instances, T=100) and the symmetrised C oracle's
backward gains on it, raw float64 in the order A B Q R Qf x u K d."""
import os, sys
import numpy as np
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, "ilqr.jl_amd")]
from ilqr_amd.problems import quadrotor_batch
from oracle import cref

lq, x, u = quadrotor_batch(256, T=100, seed0=7)
d, K, st = cref.lq_backward(lq, x, u, symmetrize=True)
assert (st == 0).all()
with open(os.path.join(R, "tools", "quad256.bin"), "wb") as f:
    for a in (lq.A, lq.B, lq.Q, lq.R, lq.Qf, x, u, K, d):
        f.write(np.ascontiguousarray(a, dtype=np.float64).tobytes())
print("wrote quad256.bin", x.shape, K.shape)
