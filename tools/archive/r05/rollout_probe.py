"""Per-step cost of rolling out the reference RBD caller's dynamics closure (nx = 16,
nu = 8: tests/closures.py rbd_floating_arm) at B = 1, four ways: vmap on the device (what
ilqr_amd.tiles.rollout_forward does), the closure called on the batch directly, one
step captured in a HIP graph and replayed, and a graph of S unrolled steps.

    PYTHONPATH=.:ilqr.jl_amd:tests python tools/archive/r05/rollout_probe.py
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
for p in (ROOT, os.path.join(ROOT, "ilqr.jl_amd"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402
from torch.func import vmap  # noqa: E402

from closures import rbd_floating_arm, rbd_initial_state, torch_arr_ns  # noqa: E402


def per_step(fn, n):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e6


def main():
    dev = "cuda"
    f, _, _ = rbd_floating_arm(torch_arr_ns())
    x = torch.tensor(rbd_initial_state(), dtype=torch.float64, device=dev)[None].clone()
    u = torch.zeros(1, 8, dtype=torch.float64, device=dev)
    fv = vmap(f)
    out = {}
    out["vmap_us"] = per_step(lambda: fv(x, u), 20)
    out["direct_us"] = per_step(lambda: f(x, u), 20)
    try:
        out.update(graphs(fv, x, u, "solve"))
    except Exception as e:  # linalg.solve checks its info on the host: no capture
        out["graph_solve_error"] = str(e)[:200]
    ns = torch_arr_ns()
    ns.solve = lambda M, b: torch.linalg.solve_ex(M, b.unsqueeze(-1))[0].squeeze(-1)
    f2, _, _ = rbd_floating_arm(ns)
    torch.cuda.synchronize()
    out.update(graphs(vmap(f2), x, u, "solve_ex"))
    print(json.dumps(out))


def graphs(fv, x, u, tag):
    out = {}
    ref = fv(x, u)
    xs, us = x.clone(), u.clone()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            fv(xs, us)
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g):
        y = fv(xs, us)
    out[tag + "_graph1_us"] = per_step(g.replay, 200)
    out[tag + "_graph1_equal"] = bool(torch.equal(y, ref))
    S = 20
    g2 = torch.cuda.CUDAGraph()
    xw = x.clone()
    with torch.cuda.graph(g2):
        z = xw
        for _ in range(S):
            z = fv(z, us)
        xw.copy_(z)
    out[tag + "_graphS_us_per_step"] = per_step(g2.replay, 20) / S
    return out


if __name__ == "__main__":
    main()
