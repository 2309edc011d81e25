"""Parse the reference's URDFs (test/urdf/*.urdf) into the chain descriptions the
RBD family loads at run time (ilqr.jl_amd/ilqr_amd/robots/*.json): the GPU box has
no /root/reference. Run here: python tools/make_robots.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ilqr.jl_amd")]
from ilqr_amd.urdf import parse_urdf  # noqa: E402

SRC = "/root/reference/test/urdf"
OUT = os.path.join(ROOT, "ilqr.jl_amd", "ilqr_amd", "robots")
for name in ("2Dof_arm", "6Dof_arm"):
    ch = parse_urdf(os.path.join(SRC, name + ".urdf"))
    doc = {"source": f"test/urdf/{name}.urdf (ilqr_amd.urdf.parse_urdf: joints, bodies and the root link)",
           "names": ch.names, "R0": ch.R0.tolist(), "p": ch.p.tolist(), "axis": ch.axis.tolist(),
           "mass": ch.mass.tolist(), "com": ch.com.tolist(), "Ic": ch.Ic.tolist(),
           "gravity": ch.gravity.tolist(), "base_mass": ch.base_mass, "base_com": ch.base_com.tolist(),
           "base_Ic": ch.base_Ic.tolist()}
    with open(os.path.join(OUT, name.lower() + ".json"), "w") as f:
        json.dump(doc, f, indent=1)
    print(name, ch.n, "joints")
