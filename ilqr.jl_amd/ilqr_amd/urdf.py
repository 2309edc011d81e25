"""URDF → serial revolute chain, the robot description the RBD problem family
(ILQR_PROBLEM_CHAIN, include/ilqr.h `ilqr_chain`) runs on the device.

The reference builds its RBD dynamics with RigidBodyDynamics.jl's
`parse_urdf(urdf; gravity = [0, 0, 0], floating = true)`
(/root/reference/test/RBD_2_link_example/RBD_helper_functions.jl:7) and calls
`mass_matrix` / `dynamics_bias` on the resulting mechanism (:61-66). This module
is the host half of that restatement for a FIXED base (BASELINE.json config 5,
SURVEY.md §8 f2): the chain of revolute/continuous joints from the root link,
with fixed joints merged into their parent body, in URDF conventions —

* joint i's frame sits at `origin xyz` with orientation `Rz(y)·Ry(p)·Rx(r)` of
  `origin rpy` in its parent link's frame; the child link frame is the joint
  frame rotated by qᵢ about `axis` (unit, joint-frame coordinates);
* a link's `inertial` gives mass, the COM (`origin xyz`) and the inertia tensor
  about the COM in axes rotated by `origin rpy`.

Everything is expressed in each body's own frame: `Chain.R0[i]` (joint frame →
parent body frame), `p[i]` (joint origin in the parent body frame), `axis[i]`,
`mass[i]`, `com[i]` and `Ic[i]` (3×3 about the COM, body axes).
"""
from __future__ import annotations

import math
import xml.etree.ElementTree as ET
from dataclasses import dataclass, field

import numpy as np

MOVABLE = ("revolute", "continuous")


def rpy_matrix(rpy):
    """URDF fixed-axis roll-pitch-yaw: R = Rz(yaw) · Ry(pitch) · Rx(roll)."""
    r, p, y = (float(v) for v in rpy)
    cr, sr, cp, sp, cy, sy = math.cos(r), math.sin(r), math.cos(p), math.sin(p), math.cos(y), math.sin(y)
    return np.array([[cy * cp, cy * sp * sr - sy * cr, cy * sp * cr + sy * sr],
                     [sy * cp, sy * sp * sr + cy * cr, sy * sp * cr - cy * sr],
                     [-sp, cp * sr, cp * cr]])


def _vec(s, default="0 0 0"):
    return np.array([float(v) for v in (s if s is not None else default).split()])


def _origin(el):
    o = el.find("origin") if el is not None else None
    if o is None:
        return np.eye(3), np.zeros(3)
    return rpy_matrix(_vec(o.get("rpy"))), _vec(o.get("xyz"))


@dataclass
class Body:
    mass: float = 0.0
    com: np.ndarray = field(default_factory=lambda: np.zeros(3))
    Ic: np.ndarray = field(default_factory=lambda: np.zeros((3, 3)))

    def merged(self, other: "Body", R: np.ndarray, p: np.ndarray) -> "Body":
        """self ∪ other, `other` given in a frame at (R, p) of this body's frame."""
        if other.mass <= 0.0:
            return self
        c2 = R @ other.com + p
        I2 = R @ other.Ic @ R.T
        m = self.mass + other.mass
        c = (self.mass * self.com + other.mass * c2) / m
        def shift(I, mk, ck):
            d = ck - c
            return I + mk * (float(d @ d) * np.eye(3) - np.outer(d, d))
        return Body(m, c, shift(self.Ic, self.mass, self.com) + shift(I2, other.mass, c2))


def _link_body(link) -> Body:
    inr = link.find("inertial")
    if inr is None:
        return Body()
    R, c = _origin(inr)
    m = float(inr.find("mass").get("value"))
    it = inr.find("inertia")
    g = {k: float(it.get(k, "0")) for k in ("ixx", "ixy", "ixz", "iyy", "iyz", "izz")}
    I = np.array([[g["ixx"], g["ixy"], g["ixz"]], [g["ixy"], g["iyy"], g["iyz"]],
                  [g["ixz"], g["iyz"], g["izz"]]])
    return Body(m, c, R @ I @ R.T)


@dataclass
class Chain:
    """A fixed-base serial chain of revolute joints (root to tip)."""
    names: list
    R0: np.ndarray    # (n, 3, 3) joint frame orientation in the parent body frame
    p: np.ndarray     # (n, 3)    joint origin in the parent body frame
    axis: np.ndarray  # (n, 3)    unit rotation axis, joint/child frame
    mass: np.ndarray  # (n,)
    com: np.ndarray   # (n, 3)    COM in the body frame
    Ic: np.ndarray    # (n, 3, 3) inertia about the COM, body axes
    gravity: np.ndarray = field(default_factory=lambda: np.zeros(3))
    # the root link (fixed children merged): only a floating base's dynamics see it
    base_mass: float = 0.0
    base_com: np.ndarray = field(default_factory=lambda: np.zeros(3))
    base_Ic: np.ndarray = field(default_factory=lambda: np.zeros((3, 3)))

    @property
    def n(self) -> int:
        return len(self.names)


def parse_urdf(path: str, gravity=(0.0, 0.0, 0.0)) -> Chain:
    """Serial-chain URDF → Chain: the joints and their bodies, and the root link's body
    (base_mass, base_com, base_Ic) — which a fixed base ignores and a floating base
    (ilqr_amd.floating, `parse_urdf(...; floating = true)` in the reference) moves.
    Branching trees and prismatic joints are rejected."""
    root = ET.parse(path).getroot()
    links = {l.get("name"): l for l in root.findall("link")}
    joints = root.findall("joint")
    children = {j.find("child").get("link") for j in joints}
    roots = [n for n in links if n not in children]
    if len(roots) != 1:
        raise ValueError(f"expected one root link, found {roots}")
    by_parent = {}
    for j in joints:
        by_parent.setdefault(j.find("parent").get("link"), []).append(j)

    # link name → (owning body index, R_off, p_off): pose of the link frame in the
    # owner's frame (-1 = the fixed base)
    place = {roots[0]: (-1, np.eye(3), np.zeros(3))}
    names, R0s, ps, axes, bodies = [], [], [], [], []
    base = _link_body(links[roots[0]])
    frontier = [roots[0]]
    while frontier:
        lname = frontier.pop()
        kids = by_parent.get(lname, [])
        if len(kids) > 1:
            raise ValueError(f"link {lname} branches: only serial chains are supported")
        for j in kids:
            child = j.find("child").get("link")
            owner, Ro, po = place[lname]
            Rj, pj = _origin(j)
            R, p = Ro @ Rj, Ro @ pj + po       # joint frame in the owner body's frame
            jtype = j.get("type")
            if jtype in MOVABLE:
                if owner != len(bodies) - 1:
                    raise ValueError("joint order does not follow the chain")
                ax = _vec(j.find("axis").get("xyz") if j.find("axis") is not None else None, "1 0 0")
                names.append(j.get("name"))
                R0s.append(R)
                ps.append(p)
                axes.append(ax / np.linalg.norm(ax))
                bodies.append(_link_body(links[child]))
                place[child] = (len(bodies) - 1, np.eye(3), np.zeros(3))
            elif jtype == "fixed":
                if owner >= 0:
                    bodies[owner] = bodies[owner].merged(_link_body(links[child]), R, p)
                else:
                    base = base.merged(_link_body(links[child]), R, p)
                place[child] = (owner, R, p)
            else:
                raise ValueError(f"joint type {jtype!r} is not supported")
            frontier.append(child)
    if not names:
        raise ValueError("no movable joints")
    return Chain(names, np.array(R0s), np.array(ps), np.array(axes),
                 np.array([b.mass for b in bodies]), np.array([b.com for b in bodies]),
                 np.array([b.Ic for b in bodies]), np.asarray(gravity, dtype=float),
                 float(base.mass), np.asarray(base.com, float), np.asarray(base.Ic, float))
