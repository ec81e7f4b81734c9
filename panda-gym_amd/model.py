"""Articulated Panda model tables: URDF -> Bullet-equivalent multibody description.

This module turns a robot URDF into the constant tables the step kernels and the
CPU oracle consume (`pgx_model` in include/pgx.h).  It restates what pybullet's
``loadURDF`` builds for the reference (``PyBulletRobot._load_robot``,
panda_gym/envs/core.py:53-67, called with ``useFixedBase=True`` and no flags):

* Link numbering is Bullet's DFS pre-order over URDF joints in file order
  (verified against test/pybullet_test.py:135, link 1 = panda_link2).
* Each multibody link frame sits at the URDF inertial origin (COM), so
  ``getLinkState()[0]`` (panda_gym/pybullet.py:259) is a COM position.
* Without ``URDF_USE_INERTIA_FROM_FILE`` Bullet ignores the URDF ``<inertia>``
  and recomputes the principal inertia from the AABB of the link's collision
  compound (box formula ``m/12*(ly^2+lz^2)``), margins included.  Links with
  mass but no collision get the empty-compound AABB (2*margin per side).
* Joint-limit constraints exist for every revolute/prismatic joint with
  lower <= upper; one joint motor exists per movable joint; the solver sees
  the constraints in the order Bullet's (unstable) quicksort on equal island
  ids leaves them (``bullet_constraint_order``).

The URDF is parsed once in the build container (``tools/build_models.py``);
the resulting JSON tables in ``assets/`` are what ships to the GPU box.
"""
from __future__ import annotations

import json
import math
import os
import xml.etree.ElementTree as ET
from dataclasses import dataclass, field, asdict
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

JOINT_REVOLUTE = 0
JOINT_PRISMATIC = 1
JOINT_FIXED = 4

MAX_LINKS = 16
MAX_DOFS = 9

# Bullet's URDF importer default collision margin (gUrdfDefaultCollisionMargin).
URDF_MARGIN = 0.001

ASSET_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "assets")


def rpy_to_matrix(rpy: Sequence[float]) -> np.ndarray:
    """URDF fixed-axis roll-pitch-yaw -> rotation matrix Rz(y) Ry(p) Rx(r)."""
    r, p, y = rpy
    cr, sr = math.cos(r), math.sin(r)
    cp, sp = math.cos(p), math.sin(p)
    cy, sy = math.cos(y), math.sin(y)
    rx = np.array([[1, 0, 0], [0, cr, -sr], [0, sr, cr]])
    ry = np.array([[cp, 0, sp], [0, 1, 0], [-sp, 0, cp]])
    rz = np.array([[cy, -sy, 0], [sy, cy, 0], [0, 0, 1]])
    return rz @ ry @ rx


def _vec(s: Optional[str], default=(0.0, 0.0, 0.0)) -> np.ndarray:
    if s is None:
        return np.array(default, dtype=np.float64)
    return np.array([float(v) for v in s.split()], dtype=np.float64)


@dataclass
class Model:
    """Constant multibody tables (float64), one entry per Bullet link index."""

    name: str
    link_names: List[str]
    parent: List[int]
    jtype: List[int]
    dof_of_link: List[int]
    link_of_dof: List[int]
    jpos: List[List[float]]          # joint origin translation in parent URDF link frame
    jrot: List[List[float]]          # joint origin rotation (row-major 3x3)
    axis: List[List[float]]          # joint axis in joint frame
    com: List[List[float]]           # inertial origin in URDF link frame
    mass: List[float]
    inertia: List[List[float]]       # principal inertia in COM frame (Bullet AABB rule)
    lower: List[float]               # per dof
    upper: List[float]
    has_limit: List[int]
    effort: List[float]
    base_com: List[float]
    # collision primitives per link, in the link COM frame: (kind, link, pos[3], rot[9], size[3])
    collision: List[dict] = field(default_factory=list)
    # constraint order after Bullet's island quicksort: list of (kind, dof) with kind 'limit'|'motor'
    constraint_order: List[Tuple[str, int]] = field(default_factory=list)
    # per link: Bullet's link compound AABB in the link COM frame, the compound margin included
    # (btCompoundShape::getAabb with the identity): centre [3], half extents [3]
    aabb_center: List[List[float]] = field(default_factory=list)
    aabb_half: List[List[float]] = field(default_factory=list)

    @property
    def n_links(self) -> int:
        return len(self.parent)

    @property
    def n_dofs(self) -> int:
        return len(self.link_of_dof)

    def to_json(self) -> str:
        return json.dumps(asdict(self), indent=1)

    @staticmethod
    def from_json(text: str) -> "Model":
        d = json.loads(text)
        d["constraint_order"] = [tuple(x) for x in d.get("constraint_order", [])]
        return Model(**d)

    def row_table(self) -> Tuple[np.ndarray, np.ndarray]:
        """Solver rows in Bullet order: (kind[r], dof[r]); kind 0 motor, 1 limit-lower, 2 limit-upper."""
        kinds, dofs = [], []
        for kind, dof in self.constraint_order:
            if kind == "limit":
                kinds += [1, 2]
                dofs += [dof, dof]
            else:
                kinds.append(0)
                dofs.append(dof)
        return np.array(kinds, dtype=np.int32), np.array(dofs, dtype=np.int32)

    def capsules(self, table_from_link: int = 1, object_from_link: int = 4, base_capsule: bool = False) -> List[dict]:
        """Contact geometry: every <collision> cylinder with the spheres capping its ends
        fused into a capsule, spheres not contained in a capsule as zero-length capsules.

        In franka_panda_custom_0 every cylinder is capped by two spheres of its own
        radius (panda.urdf:21-438), so the union Bullet collides (one compound child per
        primitive) is exactly a set of capsules; the only exception is panda_link7's
        r=0.025 sphere on the r=0.04 cylinder's top face, which the capsule's end cap
        contains.  Endpoints are in the URDF frame of the owning link.  Flags: links
        below ``table_from_link`` (panda_link1, whose sphere rests on the joint-1 axis
        inside the table top) do not touch the table -- like reach_ao.py:898, and
        dynamically inert in Bullet because the contact point lies on the joint axis;
        links from ``object_from_link`` (panda_link5) on can touch the object."""
        caps, spheres = [], []
        for p in self.collision:
            li = p["link"]
            rot = np.array(p["rot"]).reshape(3, 3)
            center = np.array(p["pos"]) + np.array(self.com[li])   # inertial frame -> URDF frame
            if p["kind"] == "cylinder":
                r, h = p["size"][0], p["size"][1]
                ax = rot @ np.array([0.0, 0.0, 1.0])
                caps.append(dict(link=li, a=(center - ax * h / 2), b=(center + ax * h / 2), r=r))
            elif p["kind"] == "sphere":
                spheres.append(dict(link=li, c=center, r=p["size"][0]))
        for s in spheres:
            inside = False
            for c in caps:
                if c["link"] != s["link"]:
                    continue
                ab = c["b"] - c["a"]
                t = np.clip(np.dot(s["c"] - c["a"], ab) / max(np.dot(ab, ab), 1e-300), 0.0, 1.0)
                if np.linalg.norm(s["c"] - (c["a"] + t * ab)) + s["r"] <= c["r"] + 1e-9:
                    inside = True
                    break
            if not inside:
                caps.append(dict(link=s["link"], a=s["c"].copy(), b=s["c"].copy(), r=s["r"]))
        if base_capsule:
            # panda_link0's cylinder (r 0.06, length 0.03 along x) capped by its two spheres
            # (panda.urdf:21-36), in the base frame; it only takes part in whole-robot distance
            # queries (ReachAO's collision-free sampling), never in contacts
            caps.append(dict(link=-1, a=np.array([-0.09, 0.0, 0.06]), b=np.array([-0.06, 0.0, 0.06]), r=0.06))
        out = []
        for c in sorted(caps, key=lambda c: c["link"]):
            flags = 0 if c["link"] < 0 else ((1 if c["link"] >= table_from_link else 0) |
                                             (2 if c["link"] >= object_from_link else 0))
            out.append(dict(link=int(c["link"]), a=[float(x) for x in c["a"]], b=[float(x) for x in c["b"]],
                            r=float(c["r"]), flags=flags))
        return out


def bullet_quicksort_equal_keys(items: List) -> List:
    """btAlignedObjectArray::quickSortInternal on a list whose keys all compare equal.

    The reference's solver receives its multibody constraints after
    ``m_sortedMultiBodyConstraints.quickSort(btSortMultiBodyConstraintOnIslandPredicate())``;
    every constraint of one robot has the same island id, so the predicate is
    always false and only the swap pattern of the partition loop remains.
    """
    a = list(items)

    def rec(lo: int, hi: int) -> None:
        i, j = lo, hi
        # x = a[(lo+hi)//2]; CompareFunc(.., x) is always false for equal keys
        while True:
            if i <= j:
                a[i], a[j] = a[j], a[i]
                i += 1
                j -= 1
            if not (i <= j):
                break
        if lo < j:
            rec(lo, j)
        if i < hi:
            rec(i, hi)

    if len(a) > 1:
        rec(0, len(a) - 1)
    return a


def _aabb_of_transformed_box(center: np.ndarray, half: np.ndarray, rot: np.ndarray,
                             pos: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    """btTransformAabb: AABB of a local box (center, half) under (rot, pos)."""
    c = rot @ center + pos
    e = np.abs(rot) @ half
    return c - e, c + e


def _obj_vertices(path: str) -> np.ndarray:
    verts = []
    used = set()
    with open(path, "r", errors="ignore") as f:
        lines = f.readlines()
    for ln in lines:
        if ln.startswith("v "):
            p = ln.split()
            verts.append([float(p[1]), float(p[2]), float(p[3])])
    for ln in lines:
        if ln.startswith("f "):
            for tok in ln.split()[1:]:
                idx = int(tok.split("/")[0])
                used.add(idx - 1 if idx > 0 else len(verts) + idx)
    v = np.array(verts, dtype=np.float64)
    if used:
        v = v[sorted(used)]
    return v


def parse_urdf(path: str, mesh_root: Optional[str] = None, name: Optional[str] = None) -> Model:
    """Parse a URDF into Bullet link order and compute Bullet's AABB inertia."""
    tree = ET.parse(path)
    root = tree.getroot()
    mesh_root = mesh_root or os.path.dirname(path)
    links = {l.get("name"): l for l in root.findall("link")}
    joints = root.findall("joint")
    child_links = {j.find("child").get("link") for j in joints}
    roots = [n for n in links if n not in child_links]
    assert len(roots) == 1, roots
    root_link = roots[0]
    children: Dict[str, List[ET.Element]] = {n: [] for n in links}
    for j in joints:
        children[j.find("parent").get("link")].append(j)

    order: List[Tuple[str, ET.Element]] = []  # (child link name, joint)

    def dfs(lname: str) -> None:
        for j in children[lname]:
            c = j.find("child").get("link")
            order.append((c, j))
            dfs(c)

    dfs(root_link)
    index = {c: i for i, (c, _) in enumerate(order)}

    def inertial(lname: str):
        el = links[lname].find("inertial")
        if el is None:
            return np.zeros(3), np.eye(3), 0.0
        o = el.find("origin")
        xyz = _vec(o.get("xyz") if o is not None else None)
        rpy = _vec(o.get("rpy") if o is not None else None)
        m = el.find("mass")
        return xyz, rpy_to_matrix(rpy), float(m.get("value")) if m is not None else 0.0

    def collision_aabb_and_prims(lname: str, li: int):
        """AABB of Bullet's link compound in the inertial frame (+margins), and primitives."""
        com_xyz, com_rot, _ = inertial(lname)
        inv_rot = com_rot.T
        inv_pos = -inv_rot @ com_xyz
        mins, maxs, prims = [], [], []
        for col in links[lname].findall("collision"):
            o = col.find("origin")
            xyz = _vec(o.get("xyz") if o is not None else None)
            rot = rpy_to_matrix(_vec(o.get("rpy") if o is not None else None))
            # child transform in compound = inertialFrame^-1 * collisionOrigin
            crot = inv_rot @ rot
            cpos = inv_rot @ xyz + inv_pos
            g = col.find("geometry")
            sph, cyl, box, mesh = g.find("sphere"), g.find("cylinder"), g.find("box"), g.find("mesh")
            if sph is not None:
                r = float(sph.get("radius"))
                # btSphereShape::getAabb uses getMargin() == radius
                lo, hi = cpos - r, cpos + r
                prims.append(dict(kind="sphere", link=li, pos=cpos.tolist(), rot=crot.ravel().tolist(),
                                  size=[r, 0.0, 0.0]))
            elif cyl is not None:
                r = float(cyl.get("radius"))
                h = float(cyl.get("length"))
                # convex hull of 32x2 points, margin set then recalcLocalAabb (+m),
                # btTransformAabb adds the child margin again (+m)
                k = np.arange(32)
                px = r * np.sin(2 * np.pi * k / 32)
                py = r * np.cos(2 * np.pi * k / 32)
                half_local = np.array([px.max() - px.min(), py.max() - py.min(), h]) * 0.5
                center_local = np.array([(px.max() + px.min()) * 0.5, (py.max() + py.min()) * 0.5, 0.0])
                half_local = half_local + 2 * URDF_MARGIN
                lo, hi = _aabb_of_transformed_box(center_local, half_local, crot, cpos)
                prims.append(dict(kind="cylinder", link=li, pos=cpos.tolist(), rot=crot.ravel().tolist(),
                                  size=[r, h, 0.0]))
            elif box is not None:
                he = _vec(box.get("size")) * 0.5
                lo, hi = _aabb_of_transformed_box(np.zeros(3), he + URDF_MARGIN, crot, cpos)
                prims.append(dict(kind="box", link=li, pos=cpos.tolist(), rot=crot.ravel().tolist(),
                                  size=he.tolist()))
            elif mesh is not None:
                fn = mesh.get("filename").replace("package://", "")
                v = _obj_vertices(os.path.join(mesh_root, fn))
                vmin, vmax = v.min(axis=0), v.max(axis=0)
                # hull local aabb (+m), hull in mesh-compound (+m), mesh compound margin (+m)
                half_local = (vmax - vmin) * 0.5 + 3 * URDF_MARGIN
                center_local = (vmax + vmin) * 0.5
                lo, hi = _aabb_of_transformed_box(center_local, half_local, crot, cpos)
                prims.append(dict(kind="mesh_aabb", link=li, pos=cpos.tolist(), rot=crot.ravel().tolist(),
                                  size=((vmax - vmin) * 0.5).tolist(), center=center_local.tolist()))
            else:
                continue
            mins.append(lo)
            maxs.append(hi)
        if mins:
            lo, hi = np.min(mins, axis=0), np.max(maxs, axis=0)
            half = (hi - lo) * 0.5 + URDF_MARGIN     # link compound margin
            center = (hi + lo) * 0.5
        else:
            half = np.full(3, URDF_MARGIN)          # empty compound: zero extents + margin
            center = np.zeros(3)
        return half, prims, center

    parent, jtype, dof_of_link, link_of_dof = [], [], [], []
    jpos, jrot, axis, com, mass, inertia = [], [], [], [], [], []
    lower, upper, has_limit, effort, names, prims_all = [], [], [], [], [], []
    aabb_center, aabb_half = [], []
    for li, (cname, j) in enumerate(order):
        pname = j.find("parent").get("link")
        parent.append(index.get(pname, -1))
        t = j.get("type")
        jt = {"revolute": JOINT_REVOLUTE, "continuous": JOINT_REVOLUTE,
              "prismatic": JOINT_PRISMATIC, "fixed": JOINT_FIXED}[t]
        jtype.append(jt)
        o = j.find("origin")
        xyz = _vec(o.get("xyz") if o is not None else None)
        rot = rpy_to_matrix(_vec(o.get("rpy") if o is not None else None))
        # URDF joint origin is given in the parent's URDF link frame
        jpos.append(xyz.tolist())
        jrot.append(rot.ravel().tolist())
        a = j.find("axis")
        ax = _vec(a.get("xyz") if a is not None else None, (1.0, 0.0, 0.0))
        if jt != JOINT_FIXED:
            ax = ax / np.linalg.norm(ax)
        axis.append(ax.tolist())
        cxyz, crot, m = inertial(cname)
        assert np.allclose(crot, np.eye(3)), "rotated inertial frames are not supported"
        com.append(cxyz.tolist())
        mass.append(m)
        half, prims, center = collision_aabb_and_prims(cname, li)
        prims_all += prims
        aabb_center.append(center.tolist())
        aabb_half.append(half.tolist())
        lx, ly, lz = 2 * half
        if m != 0.0:
            inertia.append([m / 12.0 * (ly * ly + lz * lz), m / 12.0 * (lx * lx + lz * lz),
                            m / 12.0 * (lx * lx + ly * ly)])
        else:
            inertia.append([0.0, 0.0, 0.0])
        names.append(cname)
        if jt != JOINT_FIXED:
            dof_of_link.append(len(link_of_dof))
            link_of_dof.append(li)
            lim = j.find("limit")
            lo_, hi_ = 0.0, -1.0
            eff = 0.0
            if lim is not None:
                lo_ = float(lim.get("lower", "0"))
                hi_ = float(lim.get("upper", "-1"))
                eff = float(lim.get("effort", "0"))
            lower.append(lo_)
            upper.append(hi_)
            has_limit.append(1 if (t != "continuous" and lo_ <= hi_) else 0)
            effort.append(eff)
        else:
            dof_of_link.append(-1)

    bxyz, _, _ = inertial(root_link)
    # solver constraint list as the world holds it: URDF import adds limit constraints
    # in link order, then createJointMotors adds one motor per movable joint.
    cons = [("limit", d) for d in range(len(link_of_dof)) if has_limit[d]]
    cons += [("motor", d) for d in range(len(link_of_dof))]
    cons = bullet_quicksort_equal_keys(cons)
    return Model(name=name or os.path.basename(os.path.dirname(path)), link_names=names, parent=parent,
                 jtype=jtype, dof_of_link=dof_of_link, link_of_dof=link_of_dof, jpos=jpos, jrot=jrot,
                 axis=axis, com=com, mass=mass, inertia=inertia, lower=lower, upper=upper,
                 has_limit=has_limit, effort=effort, base_com=bxyz.tolist(), collision=prims_all,
                 constraint_order=cons, aabb_center=aabb_center, aabb_half=aabb_half)


def load_model(name: str = "panda_custom0") -> Model:
    """Load a prebuilt model table from ``assets/<name>.json``."""
    with open(os.path.join(ASSET_DIR, name + ".json")) as f:
        return Model.from_json(f.read())


def forward_kinematics(model: Model, q: Sequence[float], base_pos=(0.0, 0.0, 0.0)) -> Dict[str, np.ndarray]:
    """Reference-side FK in float64 (numpy), for tests and host-side queries.

    Returns per-link URDF-frame rotation/origin and COM position (world frame).
    """
    n = model.n_links
    R = np.zeros((n, 3, 3))
    P = np.zeros((n, 3))
    C = np.zeros((n, 3))
    base_R, base_P = np.eye(3), np.asarray(base_pos, dtype=np.float64)
    for i in range(n):
        p = model.parent[i]
        pr, pp = (base_R, base_P) if p < 0 else (R[p], P[p])
        jr = np.array(model.jrot[i]).reshape(3, 3)
        r = pr @ jr
        o = pp + pr @ np.array(model.jpos[i])
        d = model.dof_of_link[i]
        if d >= 0 and model.jtype[i] == JOINT_REVOLUTE:
            ax = np.array(model.axis[i])
            c, s = math.cos(q[d]), math.sin(q[d])
            K = np.array([[0, -ax[2], ax[1]], [ax[2], 0, -ax[0]], [-ax[1], ax[0], 0]])
            r = r @ (np.eye(3) + s * K + (1 - c) * K @ K)
        elif d >= 0 and model.jtype[i] == JOINT_PRISMATIC:
            o = o + r @ (np.array(model.axis[i]) * q[d])
        R[i], P[i] = r, o
        C[i] = o + r @ np.array(model.com[i])
    return {"R": R, "P": P, "C": C}
