"""Accuracy of a Newton-Schulz (H + μI)⁻¹ in the LQ backward:
numpy restatement of backward_pass.jl:324-357 (symmetrised step_back) where each step's
gains come from X ≈ (H + μI)⁻¹ warm-started from the previous step's inverse, with the
residual check of tools/archive/ablation/bw4_newton_schulz.patch (per wave of four trajectories:
the factorisation when max|I − HX| ≥ 2.5e-3 anywhere, else 3 NS steps, 2 below 2.5e-5),
against the exact solve. Measured: quadrotor 256 trajectories max rel 1.06e-12 (15.6 %
factorised / 29 % NS2 / 55 % NS3 steps), dense T = 64 1.7e-13. Fixed schedules without
the check diverge or miss the 1e-11 gate (e.g. 16 exact steps then NS2: 6e-10)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ilqr.jl_amd")]
from ilqr_amd.problems import quadrotor_batch, random_lq_batch  # noqa: E402

MU = 0.01


def run(lq, x, u, T, adaptive, t2=2.5e-5, t3=2.5e-3, W=4):
    B = lq.A.shape[0]
    out, cnt = [], np.zeros(3)
    for b0 in range(0, B, W):  # a wave of W trajectories decides together
        Xs = [None] * W
        Ss = [lq.Qf[b] + lq.Qf[b].T for b in range(b0, b0 + W)]
        ss = [Ss[w] @ x[b0 + w, T] for w in range(W)]
        Kall = [[] for _ in range(W)]
        for t in range(T - 1, -1, -1):
            Hs, Gs, gs, Hraw = [], [], [], []
            for w in range(W):
                b = b0 + w
                A, Bm, R = lq.A[b], lq.B[b], lq.R[b]
                Hraw.append((R + R.T) + Bm.T @ Ss[w] @ Bm)
                Hs.append(Hraw[-1] + MU * np.eye(4))
                Gs.append(Bm.T @ Ss[w] @ A)
                gs.append((R + R.T) @ u[b, t] + Bm.T @ ss[w])
            r = max(np.abs(np.eye(4) - Hs[w] @ Xs[w]).max() if Xs[w] is not None else 1.0 for w in range(W))
            mode = 0 if (not adaptive or r >= t3) else (2 if r < t2 else 3)
            cnt[{0: 0, 2: 1, 3: 2}[mode]] += 1
            for w in range(W):
                b = b0 + w
                A, Q = lq.A[b], lq.Q[b]
                Gg = np.column_stack([Gs[w], gs[w]])
                if mode == 0:
                    Kaug = -np.linalg.solve(Hs[w], Gg)
                    Xs[w] = np.linalg.inv(Hs[w])
                else:
                    X = Xs[w]
                    for _ in range(mode):
                        X = 0.5 * (X + X.T)
                        X = 2 * X - X @ (Hs[w] @ X)
                    X = 0.5 * (X + X.T)
                    Xs[w] = X
                    Kaug = -X @ Gg
                K, d = Kaug[:, :12], Kaug[:, 12]
                Kall[w].append(Kaug)
                H, G, g = Hraw[w], Gs[w], gs[w]
                S = (Q + Q.T) + A.T @ Ss[w] @ A + K.T @ H @ K + K.T @ G + G.T @ K
                ss[w] = (Q + Q.T) @ x[b, t] + A.T @ ss[w] + K.T @ H @ d + K.T @ g + G.T @ d
                Ss[w] = 0.5 * (S + S.T)
        out += [np.array(k) for k in Kall]
    return np.array(out), cnt / cnt.sum()


if __name__ == "__main__":
    cases = {"quadrotor T=100 (256)": quadrotor_batch(256, T=100, seed0=0) + (100,),
             "dense T=64 (64)": random_lq_batch(64, 12, 4, 64, seed=7) + (64,)}
    for name, (lq, x, u, T) in cases.items():
        Kr, _ = run(lq, x, u, T, False)
        Km, frac = run(lq, x, u, T, True)
        e = np.abs(Km - Kr).max(axis=(1, 2, 3)) / np.abs(Kr).max(axis=(1, 2, 3))
        print(f"{name}: max rel {e.max():.3g}, median {np.median(e):.3g}, steps factorised / NS2 / NS3 "
              f"{frac.round(3).tolist()}")
