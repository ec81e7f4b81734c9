"""PandaReachAO-v3 ("reachao_rand") host side: the seeded reset of the fork's
collision-avoidance reach task, drawn from the reference's own numpy stream.

``RobotTaskEnv.reset(seed)`` seeds a fresh ``PCG64(SeedSequence(seed))`` (core.py:302)
and ReachAO.reset (reach_ao.py:965-1000) then draws, in this order:

  * ``set_coll_free_goal(["table", "robot"])`` (reach_ao.py:1101-1123): goal samples
    ``sample_within_hollow_sphere(0.5, 0.8, upper_half_only=True)`` (:1188-1211,
    scenario reachao3 :573-580) until the 0.05 m dummy sphere at the sample keeps
    more than 0.1 m from the table and the robot; after 10000 rejections the
    10001st sample is drawn and the goal falls back to the EE position;
  * ``set_coll_free_obs(0.03)`` (:1137-1161): per obstacle (sphere_0..2, cuboid_3..5,
    ``create_scenario_reachao_rand`` :587-599) ``sample_obstacle_experimental``
    (:635-644: ``random() > 0.5`` picks the goal or the EE as centre, then a
    ``hollow_sphere(0.1, 0.5)`` offset) until it keeps more than 0.03 m from the
    robot, the table and the dummy sphere (overlapping obstacles allowed);
  * ``set_random_num_obs`` (:1062-1082): ``integers(4, 6)`` active obstacles,
    ``shuffle`` of the 6 names, the first ``6 - n`` parked at (99.9, 99.9, -99.9).

numpy's own Generator produces the draws here (uniform, random, integers, shuffle),
so the stream is the reference's by construction; the geometry (signed distances
of the capsule robot to spheres and rounded boxes) restates the kernel's
(``pgx_kernels.hip``) in float64.  The device reset draws the same sequence from the
env's PCG64 record (``reset_rng="pcg64"``: numpy's draws, bit for bit) or from the
counter-based Philox stream.
"""
from __future__ import annotations

from typing import Optional, Tuple

import numpy as np

from . import abi
from .model import Model, forward_kinematics

AO_KIND = (0, 0, 0, 1, 1, 1)        # 3 spheres then 3 cuboids
AO_SIZE = 0.05                      # sphere radius / cuboid half extent (reach_ao.py:66, :583)
DUMMY_R = 0.05                      # reach_ao.py:284-287
MARGIN = 0.001                      # btBoxShape margin of the created boxes (rounded edges)
PARKED = (99.9, 99.9, -99.9)        # reach_ao.py:1078
GOAL_MARGIN = 0.1                   # set_coll_free_goal default margin
OBST_MARGIN = 0.03                  # set_coll_free_obs(0.03) + safety_distance 0.0
TABLE_CENTER = np.array([0.0, 0.0, -0.2])   # create_table(2.0, 1.3, 0.4) (reach_ao.py:272)
TABLE_HALF = np.array([1.0, 0.65, 0.2])


def box_sd(P: np.ndarray, c: np.ndarray, h: np.ndarray) -> np.ndarray:
    """Signed distance of points P[..., 3] to the axis-aligned box (c, h)."""
    d = np.abs(P - c) - h
    pos = np.where(d > 0, d, 0.0)
    o = pos[..., 0] * pos[..., 0] + pos[..., 1] * pos[..., 1] + pos[..., 2] * pos[..., 2]
    inner = np.max(d, axis=-1)
    return np.sqrt(o) + np.where(inner < 0, inner, 0.0)


def rbox_sd(P, c, h):
    return box_sd(P, c, np.asarray(h) - MARGIN) - MARGIN


def capsule_sphere_dist(A: np.ndarray, B: np.ndarray, r: np.ndarray, C: np.ndarray, R: float) -> np.ndarray:
    ab = B - A
    l2 = np.sum(ab * ab, axis=-1)
    num = (C[0] - A[:, 0]) * ab[:, 0] + (C[1] - A[:, 1]) * ab[:, 1] + (C[2] - A[:, 2]) * ab[:, 2]
    t = np.where(l2 > 0, np.clip(num / np.where(l2 > 0, l2, 1.0), 0.0, 1.0), 0.0)
    P = A + t[:, None] * ab
    v = C - P
    return np.sqrt(v[:, 0] * v[:, 0] + v[:, 1] * v[:, 1] + v[:, 2] * v[:, 2]) - r - R


def capsule_box_dist(A: np.ndarray, B: np.ndarray, r: np.ndarray, c: np.ndarray, h) -> np.ndarray:
    """Capsule vs rounded box: 40 ternary-search steps on the inner box's signed distance."""
    hi_box = np.asarray(h, dtype=np.float64) - MARGIN
    ab = B - A
    nz = np.sum(ab * ab, axis=-1) > 0
    lo, hi = np.zeros(len(A)), np.ones(len(A))
    for _ in range(40):
        m1 = lo + (hi - lo) / 3.0
        m2 = hi - (hi - lo) / 3.0
        f1 = box_sd(A + m1[:, None] * ab, c, hi_box)
        f2 = box_sd(A + m2[:, None] * ab, c, hi_box)
        left = f1 <= f2
        hi = np.where(left, m2, hi)
        lo = np.where(left, lo, m1)
    t = np.where(nz, 0.5 * (lo + hi), 0.0)
    P = A + t[:, None] * ab
    outside = (box_sd(P, c, hi_box) > 0) & nz
    # two alternating projections (box -> segment) where the distance is flat to second order
    l2 = np.sum(ab * ab, axis=-1)
    for _ in range(2):
        q = np.clip(P, c - hi_box, c + hi_box)
        num = (q[:, 0] - A[:, 0]) * ab[:, 0] + (q[:, 1] - A[:, 1]) * ab[:, 1] + (q[:, 2] - A[:, 2]) * ab[:, 2]
        tq = np.clip(num / np.where(nz, l2, 1.0), 0.0, 1.0)
        P = np.where(outside[:, None], A + tq[:, None] * ab, P)
    return box_sd(P, c, hi_box) - MARGIN - r


class RobotGeometry:
    """World-frame capsules of the robot at its neutral pose (every capsule, base and
    hand included: reset-time queries use the whole robot body)."""

    def __init__(self, model: Model, base_pos=(0.0, 0.0, 0.0), neutral_q=None, ee_link: int = 11):
        q = list(abi.NEUTRAL_Q[:model.n_dofs]) if neutral_q is None else list(neutral_q)
        fk = forward_kinematics(model, q, base_pos)
        base = np.asarray(base_pos, dtype=np.float64)
        A, B, r = [], [], []
        for c in model.capsules(base_capsule=True):
            a, b = np.array(c["a"]), np.array(c["b"])
            if c["link"] < 0:
                A.append(base + a)
                B.append(base + b)
            else:
                R, P = fk["R"][c["link"]], fk["P"][c["link"]]
                A.append(R @ a + P)
                B.append(R @ b + P)
            r.append(c["r"])
        self.A, self.B, self.r = np.array(A), np.array(B), np.array(r)
        self.ee = fk["C"][ee_link].copy()

    def distance(self, kind: int, center: np.ndarray, size: float) -> float:
        if kind == 0:
            return float(np.min(capsule_sphere_dist(self.A, self.B, self.r, center, size)))
        return float(np.min(capsule_box_dist(self.A, self.B, self.r, center, (size, size, size))))


def _hollow_sphere(rng: np.random.Generator, rmin: float, rmax: float, upper_half_only: bool) -> np.ndarray:
    """sample_within_hollow_sphere (reach_ao.py:1188-1211)."""
    phi = rng.uniform(0, 2 * np.pi)
    theta = rng.uniform(0, 0.5 * np.pi) if upper_half_only else rng.uniform(0, np.pi)
    r = np.cbrt(rng.uniform(rmin ** 3, rmax ** 3))
    return np.array([r * np.sin(theta) * np.cos(phi), r * np.sin(theta) * np.sin(phi), r * np.cos(theta)])


def reset_draws(rng: np.random.Generator, geom: RobotGeometry, trace: Optional[list] = None,
                margins: Optional[list] = None) -> Tuple[np.ndarray, np.ndarray]:
    """(goal[3], obstacles[6, 3]) of one ReachAO.reset drawn from ``rng``.  ``trace`` collects the
    draws in order (("double", k), ("integers", 1), ("shuffle", 6)); ``margins`` every accept /
    reject test's distance minus its threshold (a test within rounding of 0 may decide otherwise
    in another precision)."""
    th = TABLE_HALF
    goal = None
    dummy = None
    i = 0
    rec = trace.append if trace is not None else (lambda _x: None)
    mrg = margins.extend if margins is not None else (lambda _x: None)
    while True:
        goal = _hollow_sphere(rng, 0.5, 0.8, True)
        rec(("double", 3))
        if i > 9999:
            goal = geom.ee.copy()
            break
        i += 1
        dummy = goal
        d = (float(rbox_sd(goal, TABLE_CENTER, th)) - DUMMY_R - GOAL_MARGIN,
             geom.distance(0, goal, DUMMY_R) - GOAL_MARGIN)
        mrg(d)
        if not any(x <= 0.0 for x in d):
            break
    obst = np.zeros((6, 3))
    hcube = np.array([AO_SIZE] * 3)
    for o, kind in enumerate(AO_KIND):
        for _ in range(10000):
            rnd = rng.random()
            s = _hollow_sphere(rng, 0.1, 0.5, False)
            rec(("double", 4))
            P = s + goal if rnd > 0.5 else geom.ee + s
            if kind == 0:
                dtab = float(rbox_sd(P, TABLE_CENTER, th)) - AO_SIZE
                v = P - dummy
                ddum = float(np.sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2])) - AO_SIZE - DUMMY_R
            else:
                dtab = float(box_sd(P, TABLE_CENTER, th + AO_SIZE - 2 * MARGIN)) - 2 * MARGIN
                ddum = float(rbox_sd(dummy, P, hcube)) - DUMMY_R
            d = (geom.distance(kind, P, AO_SIZE) - OBST_MARGIN, dtab - OBST_MARGIN, ddum - OBST_MARGIN)
            mrg(d)
            obst[o] = P
            if not any(x <= 0.0 for x in d):
                break
        else:   # set_coll_free_obs (reach_ao.py:1143-1145): the 10001st attempt raises
            raise StopIteration("Couldn't find collision free obstacle!")
    n_active = int(rng.integers(4, 6))
    keys = list(range(6))
    rng.shuffle(keys)
    rec(("integers", 1))
    rec(("shuffle", 6))
    for k in keys[:abs(n_active - 6)]:
        obst[k] = PARKED
    return goal, obst


def seeded_reset(seed: Optional[int], geom: RobotGeometry) -> Optional[Tuple[np.ndarray, np.ndarray]]:
    """(goal, obstacles) of PandaReachAO-v3's reset(seed) (core.py:302 then reach_ao.py:965-1000)."""
    if seed is None:
        return None
    rng = np.random.Generator(np.random.PCG64(np.random.SeedSequence(seed)))
    return reset_draws(rng, geom)
