"""Throughput of ilqr_backward_tiles (row f3: backward_pass from caller-supplied
derivative tiles): B trajectories × T steps of random tiles on the narrow kernel
(nx ≤ 12, nu ≤ 4) and the wide one (nx ≤ 16, nu ≤ 8). The kernel streams every step's
tiles once: algorithmic bytes = B·T·8·(nx² + nx·nu + nx + nu + nx² + nu·nx + nu²) read
+ B·T·8·(nu·nx + nu) written + B·8·(nx + nx²) terminal, against the 8 TB/s HBM spec.
`python tools/bench_tiles.py [B] [T]` prints one JSON line per shape; bench.py's
secondary section calls measure() for the reference RBD caller's shape."""
import ctypes as C
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ilqr.jl_amd")]
from ilqr_amd import _lib  # noqa: E402
from ilqr_amd.solver import Solver, _ptr  # noqa: E402

HBM_PEAK = 8.0e12


def measure(nx, nu, B, T, reps=50, device=0):
    dev = torch.device("cuda", device)
    g = torch.Generator(device=dev).manual_seed(0)

    def rnd(*shape, scale=1.0):
        return scale * torch.randn(*shape, dtype=torch.float64, device=dev, generator=g)
    eye = torch.eye(nx, dtype=torch.float64, device=dev)
    Mq = rnd(B, T, nx, nx)
    tiles = {"A": eye + rnd(B, T, nx, nx, scale=0.03), "B": rnd(B, T, nx, nu, scale=0.2),
             "lx": rnd(B, T, nx), "lu": rnd(B, T, nu),
             "lxx": 0.1 * Mq @ Mq.transpose(-1, -2) / nx + eye, "lux": rnd(B, T, nu, nx, scale=0.05),
             "luu": 0.2 * torch.eye(nu, dtype=torch.float64, device=dev).expand(B, T, nu, nu).contiguous(),
             "lfx": rnd(B, nx), "lfxx": 2 * eye.expand(B, nx, nx).contiguous()}
    del Mq
    s = Solver(nx, nu, T, B, device=device, kind=_lib.PROBLEM_TILES)
    try:
        s._bind_stream()
        names = ("A", "B", "lx", "lu", "lxx", "lux", "luu", "lfx", "lfxx")
        tl = _lib.Tiles(*(tiles[k].data_ptr() for k in names))
        d = torch.empty((B, T, nu), dtype=torch.float64, device=dev)
        K = torch.empty((B, T, nu, nx), dtype=torch.float64, device=dev)
        st = torch.empty((B,), dtype=torch.int32, device=dev)
        o = _lib.default_options()

        def run(status=None):
            rc = s.lib.ilqr_backward_tiles(s.h, C.byref(tl), C.byref(o), _ptr(d), _ptr(K), status)
            assert rc == 0, rc
        run(_ptr(st))
        ok = bool((st == 0).all().item())
        if os.environ.get("TILES_SAVE"):  # the gains of a few trajectories, for a bit comparison of two builds
            import numpy as np
            np.savez(f"{os.environ['TILES_SAVE']}_{nx}x{nu}_B{B}.npz", d=d[:8].cpu().numpy(), K=K[:8].cpu().numpy())
        for _ in range(5):
            run()
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        stream = torch.cuda.current_stream(dev)
        e0.record(stream)
        for _ in range(reps):
            run()
        e1.record(stream)
        torch.cuda.synchronize(dev)
        ms = e0.elapsed_time(e1) / reps
    finally:
        s.close()
    per_step = 8 * (nx * nx + nx * nu + nx + nu + nx * nx + nu * nx + nu * nu)
    byts = B * T * per_step + B * T * 8 * (nu * nx + nu) + B * 8 * (nx + nx * nx)
    kernel = "tiles_backward_kernel" if nx <= 12 and nu <= 4 else "tiles_backward_wide_kernel"
    return {"kernel": kernel, "nx": nx, "nu": nu, "B": B, "T": T, "avg_launch_ms": ms, "status_ok": ok,
            "algorithmic_bytes": byts, "achieved_gbps": byts / (ms * 1e-3) / 1e9,
            "hbm_frac": byts / (ms * 1e-3) / HBM_PEAK, "us_per_step": ms * 1e3 / T}


if __name__ == "__main__":
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    T = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    for nx, nu in ((12, 4), (16, 8), (4, 1)):
        print(json.dumps(measure(nx, nu, B, T)), flush=True)
        torch.cuda.empty_cache()
