"""The floating forward alone (ilqr_floating_forward) at T = 1000 on the RBD script's
start, after 1 s of forwards: host-timed median / min of 15 calls per batch size, and
the outputs (x̄, ū, cost, trials of a forward that must shrink α) saved for a bit-for-bit
comparison of two builds. Not product code.

    ILQR_LIB=<build.so> python tools/ab_lib.py tools/floating_fw_ab.py OUT.npz [B ...]
    python tools/floating_fw_ab.py --compare A.npz B.npz
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "ilqr.jl_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402


def compare(a, b):
    A, B = np.load(a), np.load(b)
    same = {k: bool(np.array_equal(A[k], B[k], equal_nan=True)) for k in A.files}
    print(json.dumps({"bit_equal": all(same.values()), "arrays": same}), flush=True)
    for k in A.files:
        a, b = A[k], B[k]
        if same[k] or a.ndim != 3:
            continue
        d = (a != b) & ~(np.isnan(a) & np.isnan(b))
        t0 = int(np.argmax(d.any(axis=(0, 2))))
        rel = np.abs(a - b) / np.maximum(np.abs(a), 1e-300)
        print(json.dumps({"array": k, "first_step": t0, "components": np.argwhere(d[:, t0].any(axis=0)).ravel().tolist(),
                          "rel_at_first": float(np.nanmax(rel[:, t0])), "rel_max": float(np.nanmax(rel))}), flush=True)
    return all(same.values())


def main():
    import torch
    from ilqr_amd.floating import FloatingSolver, rbd_example_problem, rbd_initial_state

    out = sys.argv[1]
    batches = [int(v) for v in sys.argv[2:]] or [1, 64, 1024]
    T = 1000
    saved = {}
    for nb in batches:
        s = FloatingSolver(rbd_example_problem(), T, nb)
        x0 = np.tile(rbd_initial_state(), (nb, 1))
        x0[:, 8:] += 0.05 * np.random.default_rng(nb).standard_normal((nb, 8))  # spin the arm
        x0 = torch.from_numpy(x0).cuda()
        u = torch.zeros(nb, T, 8, dtype=torch.float64, device="cuda")
        x = s.rollout(x0, u)
        d, K, _ = s.backward(x, u)
        pc = torch.full((nb,), float("inf"), dtype=torch.float64, device="cuda")
        t_end = time.perf_counter() + 1.0  # settle the clock: 1 s of forwards first
        while time.perf_counter() < t_end:
            s.forward(x, u, d, K, pc)
        ts = []
        for _ in range(15):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            s.forward(x, u, d, K, pc)
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        # a search that must shrink α: the previous cost just above trial 3's
        r1 = [v.clone() for v in s.forward(x, u, d, K, pc)]
        c1 = r1[2]
        # trial 1's x̄ against fb_step (the dynamics kernel) stepped under its ū
        xr = s.rollout(r1[0][:, 0], r1[1])
        dstep = (xr != r1[0]).sum().item()
        relm = (xr - r1[0]).abs() / r1[0].abs().clamp_min(1e-300)
        rstep = relm.max().item()
        big = (relm > 1e-12).any(dim=2).any(dim=0).nonzero()  # first step off by more than 1e-12
        t_off = int(big[0].item()) if big.numel() else -1
        r1b = s.forward(x, u, d, K, pc)  # the same call again: the same bits
        again = bool(torch.equal(r1b[0].view(torch.int64), r1[0].view(torch.int64)) and
                     torch.equal(r1b[2].view(torch.int64), r1[2].view(torch.int64)))  # bits: NaN too
        r = s.forward(x, u, d, K, c1 * (1 - 1e-9))
        for k, v in zip(("x", "u", "cost", "trials", "status"), r):
            saved[f"B{nb}_{k}"] = v[:4].cpu().numpy()  # a few trajectories: the files travel back
        for k, v in zip(("x1", "u1", "cost1"), r1[:3]):
            saved[f"B{nb}_{k}"] = v[:4].cpu().numpy()
        s.close()
        print(json.dumps({"B": nb, "forward_ms": float(np.median(ts)), "min_ms": float(np.min(ts)),
                          "trials_shrunk": int(r[3].max()),
                          "x1_vs_fb_step_differing": dstep, "x1_vs_fb_step_rel": rstep,
                          "x1_vs_fb_step_first_step_off_1e-12": t_off, "repeat_bit_equal": again}), flush=True)
    np.savez(out, **saved)


if __name__ == "__main__":
    if sys.argv[1] == "--compare":
        sys.exit(0 if compare(sys.argv[2], sys.argv[3]) else 1)
    main()
