"""Extract the reference's own executed output from the animations it ships — TEST
FIXTURE GENERATOR (run here, where /root/reference exists; the GPU box only reads the
committed tests/golden/reference_gifs.npz).

/root/reference/test/2_link_example/animate_2_link.jl:7-41 fits the 2-link arm (T = 900,
x₀ = [.1, −.1, 0, 0], u₀ = 0, tol = 1e-6) with iLQR.fit and saves every 10th state of
the result, t = 1:10:901, as a 91-frame GIF of the arm (Plots.jl, 400×400, xlims = ylims =
(−2, 2), aspect equal: each frame draws base → elbow → tool). The shipped
figures/iLQR_2_link_quad_4.gif is that script's output for its target_tool_loc
[0.6, −0.5]; quad_1..3 are the same script with the target in the other quadrants
((0.6, 0.5), (−0.6, 0.5), (−0.6, −0.5): read off their last frames); iLQR_2_link.gif
(an earlier copy, also in docs/extras/) is recorded for completeness. These are the only
numeric outputs of the executed reference anywhere in it.

Per frame: the arm's pixels (the red/blue blend: R − G > 40) are fitted by the polyline
base → elbow → tool of link lengths l₁ = l₂ = √2/2 (2_link_helper_functions.jl:5) over
(θ₁, θ₂), least squares of the pixels' distances to the polyline (a grid start, then
Nelder-Mead, each frame from the previous one's answer). The pixel ↔ data map comes
from the plot's own grid lines at x, y ∈ {−1, 0, 1} (intensity centroids): ≈88.2 px per
unit. Stored: θ per frame, the fit's RMS pixel distance, the calibration. GIF decoding is
PIL's (a data format, nothing executed from the files).

    python tests/golden/make_gif_golden.py
"""
import hashlib
import json
import math
import os

import numpy as np
from PIL import Image, ImageSequence
from scipy.optimize import minimize

REF = "/root/reference"
FIG = os.path.join(REF, "test", "2_link_example", "figures")
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_gifs.npz")
L = math.sqrt(2.0) / 2.0   # l₁ = l₂ (2_link_helper_functions.jl:5)
GIFS = {"quad_4": "iLQR_2_link_quad_4.gif", "quad_1": "iLQR_2_link_quad_1.gif",
        "quad_2": "iLQR_2_link_quad_2.gif", "quad_3": "iLQR_2_link_quad_3.gif",
        "ilqr_2_link": "iLQR_2_link.gif"}


def frames(path):
    return [np.array(f.convert("RGB")).astype(float) for f in ImageSequence.Iterator(Image.open(path))]


def calibrate(f):
    """Grid-line centroids (pixel-index coordinates) of x, y ∈ {−1, 0, 1}."""
    g = f.sum(2)

    def centroid(profile, c):
        idx = np.arange(c - 3, c + 4)
        w = np.clip(765.0 - profile[idx], 0.0, None)
        return float((w * idx).sum() / w.sum())
    cols = g[20:90].mean(0)            # rows near the top: only vertical grid lines
    rows = g[:, 40:110].mean(1)        # columns at the left: only horizontal grid lines
    xs = [centroid(cols, c) for c in (122, 210, 298)]
    ys = [centroid(rows, r) for r in (101, 189, 277)]
    return {"x0": xs[1], "y0": ys[1], "sx": (xs[2] - xs[0]) / 2, "sy": (ys[2] - ys[0]) / 2}


def arm_pixels(f, cal):
    yy, xx = np.nonzero(f[..., 0] - f[..., 1] > 40.0)
    return (xx - cal["x0"]) / cal["sx"], -(yy - cal["y0"]) / cal["sy"]


def seg_dist(px, py, ax, ay, bx, by):
    vx, vy = bx - ax, by - ay
    t = np.clip(((px - ax) * vx + (py - ay) * vy) / (vx * vx + vy * vy), 0.0, 1.0)
    return np.hypot(px - ax - t * vx, py - ay - t * vy)


def points(th):
    th = np.atleast_2d(th)
    e = np.stack([L * np.cos(th[:, 0]), L * np.sin(th[:, 0])], 1)
    t = e + np.stack([L * np.cos(th[:, 0] + th[:, 1]), L * np.sin(th[:, 0] + th[:, 1])], 1)
    return e, t


def misfit(th, X, Y):
    e, t = points(th)
    d = np.minimum(seg_dist(X, Y, 0.0, 0.0, *e[0]), seg_dist(X, Y, *e[0], *t[0]))
    return float((d * d).mean())


def extract(path):
    fr = frames(path)
    cal = calibrate(fr[0])
    out, rms, prev = [], [], None
    grid = [(a, b) for a in np.linspace(-math.pi, math.pi, 73) for b in np.linspace(-math.pi, math.pi, 73)]
    for f in fr:
        X, Y = arm_pixels(f, cal)
        starts = sorted(grid, key=lambda th: misfit(th, X, Y))[:3] if prev is None else [prev]
        best = None
        for s in starts:
            r = minimize(misfit, s, args=(X, Y), method="Nelder-Mead", options={"xatol": 1e-7, "fatol": 1e-14})
            if best is None or r.fun < best.fun:
                best = r
        prev = best.x
        out.append(best.x)
        rms.append(math.sqrt(best.fun) * cal["sx"])
    return np.array(out), np.array(rms), cal


def main():
    arrays, meta = {}, {"stride": 10, "T": 900, "x0": [0.1, -0.1, 0.0, 0.0], "tol": 1e-6, "link": L,
                        "source": "animate_2_link.jl:7-41 output GIFs shipped in /root/reference", "gifs": {}}
    for key, name in GIFS.items():
        path = os.path.join(FIG, name)
        th, rms, cal = extract(path)
        arrays[key + "_theta"] = th
        arrays[key + "_rms_px"] = rms
        e, t = points(th[-1])
        meta["gifs"][key] = {"file": "test/2_link_example/figures/" + name, "frames": len(th),
                             "md5": hashlib.md5(open(path, "rb").read()).hexdigest(), "calibration": cal,
                             "final_tool": [float(t[0, 0]), float(t[0, 1])], "max_rms_px": float(rms.max())}
        print(key, len(th), "final tool", t[0].round(4), "max rms px", rms.max().round(3))
    np.savez_compressed(OUT, meta=np.array(json.dumps(meta)), **arrays)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
