"""Physical sanity of the oracle's contact restatement (cube / table / plane / robot).

Bullet's contact dynamics have no known answer in the reference (SURVEY §8c:
"contact dynamics" is parity-unpinned), so these tests pin the restatement by
closed-form physics instead: a cube comes to rest on the table top and on the
plane, stays at rest, slides to a stop after v^2 / (2 mu g), the robot's tool
bar cannot sink into the table, and the robot can push the cube.
"""
import math

import numpy as np
import pytest

from panda_gym_amd import abi
from panda_gym_amd.model import load_model

KEEP = []


def _cfg(task=abi.TASK_PUSH, n=1, contacts=True, block_gripper=True):
    model = abi.make_model(load_model("panda_custom0"), ee_link=11)
    params = abi.default_sim_params()
    spec = abi.EnvSpec(task=task, block_gripper=block_gripper)
    cfg = abi.make_config(spec, n, model, params, contacts=contacts)
    KEEP.append((model, params, cfg))
    return cfg


def _motors(oracle, q):
    return oracle.make_motors(7, {d: (q[d], 0.0, 0.1, 1.0, abi.JOINT_FORCES[d] / 500.0) for d in range(7)})


def _obj(pos, vel=(0, 0, 0), w=(0, 0, 0), quat=(0, 0, 0, 1)):
    from oracle import oracle as orc

    o = np.zeros(orc.OBJ_N)
    o[0:3], o[3:7], o[7:10], o[10:13] = pos, quat, vel, w
    o[orc.OBJ_CACHE:orc.OBJ_AO:2] = -1.0
    return o


def _run(oracle, cfg, obj, steps, q=None):
    q = np.array(abi.NEUTRAL_Q[:7]) if q is None else np.array(q, dtype=np.float64)
    qd = np.zeros(7)
    mot = _motors(oracle, q)
    for _ in range(steps):
        q, qd, obj, st = oracle.world_substep(cfg, q, qd, obj, mot)
    return q, qd, obj, st


def test_cube_falls_and_rests_on_table(oracle):
    cfg = _cfg()
    _, _, o, st = _run(oracle, cfg, _obj((0.0, 0.1, 0.07)), 400)
    assert abs(o[2] - 0.02) < 1e-3
    assert np.linalg.norm(o[7:13]) < 1e-2
    assert st.n_contacts == 4
    assert abs(o[6]) > 0.999            # still upright


def test_cube_at_rest_stays_at_rest(oracle):
    cfg = _cfg()
    o0 = _obj((0.05, -0.05, 0.02))
    _, _, o, _ = _run(oracle, cfg, o0.copy(), 500)
    assert np.abs(o[0:3] - o0[0:3]).max() < 2e-4
    assert np.linalg.norm(o[7:10]) < 1e-3


def test_cube_off_the_table_lands_on_the_plane(oracle):
    cfg = _cfg()
    _, _, o, _ = _run(oracle, cfg, _obj((0.5, 0.0, -0.3)), 400)
    assert abs(o[2] - (-0.4 + 0.02)) < 1e-3


def test_sliding_cube_stops_after_coulomb_distance(oracle):
    """v0 = 0.4 m/s on the table: Coulomb friction mu = 0.25 stops it after v0^2 / (2 mu g)."""
    cfg = _cfg()
    v0 = 0.4
    o = _obj((-0.1, 0.0, 0.02), vel=(v0, 0.0, 0.0))
    _, _, o, _ = _run(oracle, cfg, o, 400)
    want = v0 * v0 / (2 * 0.25 * 9.81)
    got = o[0] + 0.1
    assert np.linalg.norm(o[7:10]) < 1e-3
    assert abs(got - want) < 0.15 * want, (got, want)


def test_tool_bar_stays_on_the_table(oracle):
    """Drive the EE down to z = 0 (a Reach goal on the table top): with contacts the tool
    bar (capsule r = 0.02 at the EE) stops at the table, without them it sinks."""
    from oracle import oracle as O

    res = {}
    for contacts in (True, False):
        cfg = _cfg(task=abi.TASK_REACH, contacts=contacts)
        env = O.OracleVecEnv(cfg, 1)
        env.reset(inject_goal=np.array([[0.0, 0.0, 0.0]]))
        for _ in range(30):
            ee = env.step(np.array([[0.0, 0.0, -1.0]], np.float32))
        res[contacts] = float(ee["ag"][0, 2])
    assert res[False] < 0.02            # no table: the EE goes (almost) to the IK target z = 0
    assert res[True] > 0.035            # the bar, 0.0416 below the EE point, rests on the top


def test_robot_pushes_cube(oracle):
    """Lower the EE beside the cube and sweep it in +y: the bar strikes the cube, which
    slides (and turns) on the table top instead of being penetrated."""
    from oracle import oracle as O

    cfg = _cfg(task=abi.TASK_PUSH)
    env = O.OracleVecEnv(cfg, 1)
    env.reset(inject_goal=np.array([[0.0, 0.1, 0.02]]), inject_obj=np.array([[0.0, 0.0, 0.02]]))
    start = env.obj[0, 0:3].copy()
    acts = [[1, 0, 0]] * 2 + [[0, -1, 0]] * 2 + [[0, 0, -1]] * 5 + [[0, 1, 0]] * 6
    for a in acts:
        b = env.step(np.array([a], np.float32))
    moved = env.obj[0, 0:3] - start
    assert np.linalg.norm(moved[:2]) > 0.02, moved
    assert abs(env.obj[0, 2] - 0.02) < 2e-3
    assert b["obs"][0, 2] > 0.035          # the EE rides on the table top (tool bar contact)


def test_push_obs_layout(oracle):
    from oracle import oracle as O

    cfg = _cfg(task=abi.TASK_PUSH)
    env = O.OracleVecEnv(cfg, 2)
    b = env.reset(inject_goal=np.array([[0.1, 0.1, 0.02]] * 2), inject_obj=np.array([[0.05, -0.05, 0.02]] * 2))
    assert b["obs"].shape == (2, 18)
    assert np.allclose(b["obs"][:, 6:9], [0.05, -0.05, 0.02])
    assert np.allclose(b["obs"][:, 9:18], 0.0)
    assert np.array_equal(b["ag"], b["obs"][:, 6:9])
    cfg = _cfg(task=abi.TASK_PICK_AND_PLACE, block_gripper=False)
    env = O.OracleVecEnv(cfg, 1)
    b = env.reset()
    assert b["obs"].shape == (1, 19) and b["obs"][0, 6] == 0.0


@pytest.mark.parametrize("rpy", [(0.3, -0.2, 1.1), (-1.0, 0.5, -2.5), (0.0, 0.0, 0.0)])
def test_euler_matches_pybullet_convention(oracle, rpy):
    """getEulerFromQuaternion inverts getQuaternionFromEuler (roll about x, pitch y, yaw z)."""
    from oracle import oracle as O

    r, p, y = rpy
    cr, sr, cp, sp, cy, sy = math.cos(r / 2), math.sin(r / 2), math.cos(p / 2), math.sin(p / 2), \
        math.cos(y / 2), math.sin(y / 2)
    q = (sr * cp * cy - cr * sp * sy, cr * sp * cy + sr * cp * sy, cr * cp * sy - sr * sp * cy,
         cr * cp * cy + sr * sp * sy)
    cfg = _cfg(task=abi.TASK_PUSH)
    env = O.OracleVecEnv(cfg, 1)
    env.reset()
    env.obj[0, 3:7] = q
    env.obj[0, 0:3] = (0.0, 0.0, 0.5)
    b = env.step(np.zeros((1, 3), np.float32))   # one step in free fall: orientation unchanged (w = 0)
    assert np.allclose(b["obs"][0, 9:12], rpy, atol=1e-5)


# ---------------------------------------------------------------- manifold rule + row budget
# Bullet keeps one btPersistentManifold of <= 4 points per colliding pair (a capsule -- a child
# shape of its link's compound -- against the table, the plane, the cube or an obstacle); the
# build then keeps the deepest points up to a per-env budget (include/pgx.h: with
# PGX_CONTACTS_FULL 8 robot points in Reach / ReachAO, 12 in Push / PickAndPlace; else 4).  Poses: a resting arm
# with the hand and a finger on the table (found by sampling joint space), and the cube at the
# closed fingertips.
TWO_LINKS_ON_TABLE_Q = [-1.1690350756013894, 0.6106566125901616, 0.23087389083588095, -2.3777880820996167,
                        0.6961929207547803, 1.5588531369310048, -0.6269433985552224]
# the same case at Bullet's relative thresholds (round 6, found by sampling joint space, every end at
# least 3e-4 from its pair's threshold): panda_link8's three capsules and the hand, 5 points within
# 1.5 mm of the table top
TWO_LINKS_ON_TABLE_REL_Q = [0.526566, 1.546148, -1.128492, -1.578053, 2.257213, 0.547753, 0.653782]


def _detect(oracle, cfg, q, obj, budget=-1):
    """one substep from rest at q (motors holding q); the detection's points and the number the
    per-pair rule keeps before the budget"""
    oracle.set_robot_budget(budget)
    try:
        oracle.pair_hist(clear=True)
        _run(oracle, cfg, obj, 1, q=q)
        h = oracle.pair_hist(clear=True)
        return oracle.last_contacts(), int(np.nonzero(h)[0][0])
    finally:
        oracle.set_robot_budget(-1)


def _robot(pts):
    g, i, l, d = pts
    r = g != 0
    return i[r], l[r], d[r]


def test_two_links_on_table_keep_all_points(oracle):
    """The budget's mechanics on five table points of two links (at the global 0.02 threshold of the
    study flag, which reports them all); at Bullet's relative per-pair threshold (the default) the
    same pose reports the subset within each link's own threshold."""
    cfg = _cfg(task=abi.TASK_REACH)
    cfg.contacts = abi.CONTACTS_FULL
    cfg.params.contents.flags = abi.FLAG_GLOBAL_BREAKING
    obj = _obj((0.0, 0.0, 0.0))
    pts, n_pair = _detect(oracle, cfg, TWO_LINKS_ON_TABLE_Q, obj)
    ids, links, d = _robot(pts)
    assert n_pair == 5 and len(ids) == 5                        # all of them (budget 8)
    assert len(set(links.tolist())) == 2 and np.all(ids < 32)   # two links, capsule ends vs the table
    assert np.all(d < 0.02) and np.all(np.diff(ids) > 0)        # within tau, rows in id order
    cfg.contacts = 1                                            # the default budget: the 4 deepest
    pts4, _ = _detect(oracle, cfg, TWO_LINKS_ON_TABLE_Q, obj)
    ids4, _, d4 = _robot(pts4)
    assert len(ids4) == 4 and d4.max() <= np.sort(d)[3]
    cfg.contacts = abi.CONTACTS_FULL
    cfg.params.contents.flags = 0                               # Bullet's relative threshold
    ptsr, _ = _detect(oracle, cfg, TWO_LINKS_ON_TABLE_Q, obj)
    idsr, linksr, dr = _robot(ptsr)
    thr = oracle.breaking_thresholds(cfg)["table"]
    caps = idsr // 2
    keep = np.array([dd < thr[(i // 2)] for i, dd in zip(ids, d)])
    assert np.array_equal(idsr, ids[keep]) and np.all(dr < thr[caps])
    # the relative-threshold pose: all five kept at budget 8, the 4 deepest at the default budget
    ptsr, n_pair = _detect(oracle, cfg, TWO_LINKS_ON_TABLE_REL_Q, obj)
    idsr, linksr, dr = _robot(ptsr)
    assert n_pair == 5 and len(idsr) == 5 and len(set(linksr.tolist())) == 2 and np.all(idsr < 32)
    assert np.all(dr < thr[idsr // 2]) and np.all(np.diff(idsr) > 0)
    cfg.contacts = 1
    ids4, _, d4 = _robot(_detect(oracle, cfg, TWO_LINKS_ON_TABLE_REL_Q, obj)[0])
    assert len(ids4) == 4 and d4.max() <= np.sort(dr)[3]


def test_link_on_cube_keeps_all_points_per_pair_cap(oracle):
    """The fresh per-pair rule (round 4's, now the study flag PGX_FLAG_FRESH_MANIFOLD): every capsule
    on the cube brings its 4 deepest samples at once; Bullet's persistent manifold (the default)
    starts each pair from its one new point."""
    cfg = _cfg(task=abi.TASK_PUSH)
    cfg.contacts = abi.CONTACTS_FULL
    env = oracle.OracleVecEnv(cfg, 1)
    env.reset()   # cfg seed 0
    ee = env.step(np.zeros((1, 3)))["obs"][0, :3]   # the cube at the closed fingertips, in the air
    q = env.q[0].copy()
    cfg.params.contents.flags = abi.FLAG_FRESH_MANIFOLD
    pts, n_pair = _detect(oracle, cfg, q, _obj(tuple(ee)))
    ids, links, d = _robot(pts)
    assert np.all(ids >= 32)                                    # capsule spheres vs the cube
    caps = (ids - 32) // 16
    per_pair = np.bincount(caps)
    assert per_pair.max() == 4 and (per_pair > 0).sum() >= 2    # >= 2 capsules, each capped at 4
    assert n_pair == len(ids) > 4                               # the budget (12) cuts nothing
    cfg.params.contents.flags = 0                               # Bullet's manifolds, from empty ones
    ptsp, _ = _detect(oracle, cfg, q, _obj(tuple(ee)))
    idsp = _robot(ptsp)[0]
    assert len(idsp) == (per_pair > 0).sum() and np.all((idsp - 32) % 16 == 0)   # one per pair, slot 0
    cfg.contacts = 1
    pts4, _ = _detect(oracle, cfg, q, _obj(tuple(ee)))
    assert len(_robot(pts4)[0]) == 4


# ---------------------------------------------------------------- persistent manifold
# Bullet's btPersistentManifold for the robot's cube / obstacle pairs (the default with
# PGX_CONTACTS_FULL): a pool of points per env, pgx.h PGX_MANIFOLD_POOL.
def _pt(a, dist, normal=(0.0, 0.0, 1.0), imp=0.0):
    a, n = np.asarray(a, float), np.asarray(normal, float)
    return np.concatenate([[0.0], a, a - n * dist, n, [dist, imp]])


def _pool(oracle, cap=16):
    return np.zeros(1 + cap * oracle.MAN_PT)


def _P(oracle, P, i):
    return P[1 + i * oracle.MAN_PT:1 + (i + 1) * oracle.MAN_PT]


def test_manifold_merges_appends_and_replaces_by_area(oracle):
    P = _pool(oracle)
    key = 32
    assert oracle.manifold_add(P, key, _pt((0, 0, 0), -0.003)) == 0 and P[0] == 1
    _P(oracle, P, 0)[oracle.MP_IMP] = 5.0                       # the solver wrote an impulse back
    # within the breaking threshold (0.02) of the cached point in A's frame: replaces it, impulse kept
    assert oracle.manifold_add(P, key, _pt((0.01, 0, 0), -0.002)) == 0 and P[0] == 1
    assert _P(oracle, P, 0)[oracle.MP_IMP] == 5.0 and _P(oracle, P, 0)[1] == 0.01
    for a in ((0.05, 0, 0), (0, 0.05, 0), (0.05, 0.05, 0)):   # farther apart: appended
        oracle.manifold_add(P, key, _pt(a, -0.001))
    assert P[0] == 4
    assert [int(_P(oracle, P, i)[0]) for i in range(4)] == [32, 33, 34, 35]   # kid = key + slot
    pts = np.stack([_P(oracle, P, i).copy() for i in range(4)])
    # a fifth point: sortCachedPoints -- never the deepest (slot 0), else the largest remaining area
    new = _pt((0.1, 0.1, 0), -0.0005)
    res = []
    for i, (ia, ib, ic) in enumerate(((1, 3, 2), (0, 3, 2), (0, 3, 1), (0, 2, 1))):
        x = np.cross(new[1:4] - pts[ia, 1:4], pts[ib, 1:4] - pts[ic, 1:4])
        res.append(0.0 if i == 0 else float(x @ x))
    want = int(np.argmax(res))
    assert want != 0 and oracle.manifold_add(P, key, new) == want and P[0] == 4
    got = _P(oracle, P, want)
    assert got[0] == 32 + want and np.array_equal(got[1:11], new[1:11]) and got[oracle.MP_IMP] == 0.0
    # another pair's manifold shares the pool; a full pool drops a point that needs a new entry
    Q = _pool(oracle, cap=2)
    assert oracle.manifold_add(Q, 48, _pt((0, 0, 0), -0.001), cap=2) == 0
    assert oracle.manifold_add(Q, 64, _pt((0, 0, 0), -0.001), cap=2) == 0
    assert oracle.manifold_add(Q, 48, _pt((0.05, 0, 0), -0.001), cap=2) == -1 and Q[0] == 2


def test_manifold_refresh_breaks_points(oracle):
    P = _pool(oracle)
    for a in ((0, 0, 0), (0.05, 0, 0), (0, 0.05, 0)):
        oracle.manifold_add(P, 32, _pt(a, -0.001))
    _P(oracle, P, 1)[4:7] = _P(oracle, P, 1)[1:4] - np.array([0, 0, 0.03])    # B 0.03 below A: separated past 0.02
    _P(oracle, P, 2)[4:7] = _P(oracle, P, 2)[1:4] + np.array([0.03, 0, 0.001])  # slid 0.03 sideways
    oracle.manifold_refresh_static(P)
    assert P[0] == 1 and np.allclose(_P(oracle, P, 0)[1:4], 0.0)
    assert abs(_P(oracle, P, 0)[oracle.MP_D] - (-0.001)) < 1e-15


def test_manifold_removal_renumbers_slots_as_bullet(oracle):
    """removeContactPoint in reverse slot order, the last slot's point filling the hole: dropping
    slots 1 and 3 of four leaves the old slot 0 at 0 and the old slot 2 at 1; the pool keeps the
    survivors' order and another manifold's points are untouched."""
    P = _pool(oracle)
    for a in ((0, 0, 0), (0.05, 0, 0), (0, 0.05, 0), (0.05, 0.05, 0)):
        oracle.manifold_add(P, 32, _pt(a, -0.001))
    oracle.manifold_add(P, 48, _pt((0.3, 0, 0), -0.001))
    for i in (1, 3):
        _P(oracle, P, i)[4:7] = _P(oracle, P, i)[1:4] - np.array([0, 0, 0.05])
    oracle.manifold_refresh_static(P)
    assert P[0] == 3
    kids = [int(_P(oracle, P, i)[0]) for i in range(3)]
    las = [tuple(_P(oracle, P, i)[1:4]) for i in range(3)]
    assert kids == [32, 33, 48] and las == [(0, 0, 0), (0, 0.05, 0), (0.3, 0, 0)]


def test_persistent_manifold_builds_over_substeps(oracle):
    """The cube at the closed fingertips (test_link_on_cube_keeps_all_points_per_pair_cap): the
    fresh rule (PGX_FLAG_FRESH_MANIFOLD) gives each colliding capsule its 4 deepest samples at once;
    Bullet's manifold (the default) starts from the pair's one closest point and gains at most one
    point per pair per substep, never more than 4."""
    from oracle import oracle as orc

    cfg = _cfg(task=abi.TASK_PUSH)
    cfg.contacts = abi.CONTACTS_FULL
    env = oracle.OracleVecEnv(cfg, 1)
    env.reset()
    ee = env.step(np.zeros((1, 3)))["obs"][0, :3]
    q0 = env.q[0].copy()
    q, qd, obj, mot = q0.copy(), np.zeros(7), _obj(tuple(ee)), _motors(oracle, q0)
    counts = []
    for t in range(12):
        q, qd, obj, _ = oracle.world_substep(cfg, q, qd, obj, mot)
        cube = {key: len(pts) for key, pts in orc.manifolds(obj)}
        assert all(32 <= key < 32 + 16 * 16 and (key - 32) % 16 == 0 for key in cube)
        counts.append(cube)
    assert counts[0] and all(v == 1 for v in counts[0].values())      # one closest point per pair first
    for a, b in zip(counts, counts[1:]):
        for key, v in b.items():
            assert v <= a.get(key, 0) + 1 and v <= 4
    assert max(max(c.values(), default=0) for c in counts) >= 2       # and it builds up
    # the fresh rule from the same start holds up to 4 per pair at once
    cff = _cfg(task=abi.TASK_PUSH)
    cff.contacts = abi.CONTACTS_FULL
    cff.params.contents.flags = abi.FLAG_FRESH_MANIFOLD
    q1, qd1, obj1, _ = oracle.world_substep(cff, q0.copy(), np.zeros(7), _obj(tuple(ee)), mot)
    assert int(obj1[orc.OBJ_MAN]) == 0                                   # (no pool in that mode)
    g, ids, _, _ = orc.last_contacts()
    per_cap = {}
    for gg, i in zip(g, ids):
        if gg == 2:
            per_cap[(i - 32) // 16] = per_cap.get((i - 32) // 16, 0) + 1
    assert max(per_cap.values()) > 1


def test_table_manifolds_equal_the_fresh_table_rule(oracle):
    """The fresh table / plane rule stands for Bullet's manifolds of the end spheres (each re-reports
    its one point every substep, which merges into itself with its impulse): Reach with the tool bar
    on the table, 60 substeps, the default (fresh table pairs) against the study flag
    PGX_FLAG_PERSISTENT_MANIFOLD (every robot pair through manifolds) -- the same trajectory to
    rounding."""
    from oracle import oracle as orc

    outs = []
    for flags in (0, abi.FLAG_PERSISTENT_MANIFOLD):
        cfg = _cfg(task=abi.TASK_REACH)
        cfg.contacts = abi.CONTACTS_FULL
        cfg.params.contents.flags = flags
        q = np.array(abi.NEUTRAL_Q[:7])
        q[1], q[3] = 0.6, -1.55           # EE low over the table
        target = q.copy()
        target[1] += 0.35                 # drive it down into the table
        qd, obj = np.zeros(7), _obj((5.0, 5.0, 5.0))
        mot = _motors(oracle, target)
        pts = 0
        for _ in range(60):
            q, qd, obj, st = oracle.world_substep(cfg, q, qd, obj, mot)
            pts = max(pts, st.n_contacts)
        outs.append((q.copy(), qd.copy(), pts, int(obj[orc.OBJ_MAN])))
    (q0, qd0, n0, pool0), (q1, qd1, n1, pool1) = outs
    assert n0 >= 1 and n0 == n1          # the bar touches the table in both
    assert pool0 == 0 and pool1 >= 1     # only the study mode keeps manifolds for the table
    assert np.abs(q0 - q1).max() < 1e-9 and np.abs(qd0 - qd1).max() < 1e-7


# ---------------------------------------------------------------- contact breaking threshold
def test_relative_breaking_thresholds(oracle):
    """Bullet's relative per-pair rule (btCollisionDispatcher::getNewManifold's default
    CD_USE_RELATIVE_CONTACT_BREAKING_THRESHOLD): min over the pair of (|AABB half| + |AABB centre|)
    x 0.02, the link compounds' AABBs from the URDF import, the scene's createMultiBody boxes as
    compounds with margin 0.001.  Restated by hand here, against the oracle's table; the device
    block (pgx_dev_model_bytes, host only) carries the same values in float; the study flag gives
    the global 0.02 everywhere."""
    from panda_gym_amd._native import load

    model = load_model("panda_custom0")
    m = 0.001
    disc = lambda *h: float(np.linalg.norm(np.array(h) + m))  # noqa: E731
    for task in (abi.TASK_REACH, abi.TASK_PUSH):
        cfg = _cfg(task=task)
        thr = oracle.breaking_thresholds(cfg)
        caps = model.capsules(base_capsule=True)
        for c, cap in enumerate(caps):
            li = cap["link"]
            t_link = 0.02 if li < 0 else 0.02 * (np.linalg.norm(model.aabb_half[li]) + np.linalg.norm(model.aabb_center[li]))
            assert thr["table"][c] == pytest.approx(min(t_link, 0.02 * disc(0.55, 0.35, 0.2)), rel=1e-12)
            assert thr["plane"][c] == pytest.approx(min(t_link, 0.02 * disc(3.0, 3.0, 0.01)), rel=1e-12)
            assert thr["cube"][c] == pytest.approx(min(t_link, 0.02 * disc(0.02, 0.02, 0.02)), rel=1e-12)
            assert thr["obstacle"][c] == pytest.approx(min(t_link, 0.02 * disc(0.05, 0.05, 0.05)), rel=1e-12)
        assert thr["cube_table"] == pytest.approx(0.02 * disc(0.02, 0.02, 0.02), rel=1e-12)
        # the robot's links: 2.2 - 7.4 mm against the table; every robot / cube pair at the cube's 0.73 mm
        arm = [c for c, cap in enumerate(caps) if cap["flags"]]
        assert 0.002 < thr["table"][arm].min() and thr["table"][arm].max() < 0.008
        assert np.allclose(thr["cube"][arm], 0.02 * disc(0.02, 0.02, 0.02))
        lib = load()
        import ctypes as C
        lib.pgx_dev_model_bytes.argtypes = [C.c_void_p, C.c_void_p, C.c_int64]
        buf = np.zeros(320, dtype=np.float32)
        assert lib.pgx_dev_model_bytes(C.byref(cfg), buf.ctypes.data_as(C.c_void_p), buf.nbytes) == 0
        for k, name in enumerate(("table", "plane", "cube", "obstacle")):
            dev = buf[246 + 16 * k: 246 + 16 * k + len(caps)]
            assert np.array_equal(dev, thr[name][:len(caps)].astype(np.float32)), name
        assert buf[310] == np.float32(thr["cube_table"]) and buf[311] == np.float32(thr["cube_plane"])
        # then the scene's table box and plane top (round 6: compile-time in the default build)
        tc, th = np.array(cfg.table_center[:]), np.array(cfg.table_half[:])
        assert np.array_equal(buf[312:319], np.float32([tc[0], tc[1], th[0], th[1], tc[2] + th[2], cfg.plane_z, th[2]]))
        cfg.params.contents.flags = abi.FLAG_GLOBAL_BREAKING
        g = oracle.breaking_thresholds(cfg)
        assert np.all(g["table"][:len(caps)] == 0.02) and g["cube_table"] == 0.02


# ---------------------------------------------------------------- the table's side walls
def test_cube_stops_at_the_table_side_wall(oracle):
    """Round 6: the cube's vertices meet the whole table box, its side walls included.  A cube on the
    plane sliding into the table's +x wall (x = 0.25) stops against it instead of being thrown onto
    the top (rounds 2-5 took each vertex against the top face of the box under it)."""
    cfg = _cfg()
    o = _obj((0.25 + 0.02 + 0.03, 0.0, -0.4 + 0.02), vel=(-0.6, 0.0, 0.0))
    q = np.array(abi.NEUTRAL_Q[:7])
    qd = np.zeros(7)
    mot = _motors(oracle, q)
    vmax = 0.0
    for _ in range(400):
        q, qd, o, st = oracle.world_substep(cfg, q, qd, o, mot)
        vmax = max(vmax, float(np.abs(o[7:10]).max()))
    assert vmax <= 0.6 + 1e-6, vmax                       # never thrown
    assert 0.25 + 0.02 - 2e-3 < o[0] < 0.25 + 0.02 + 0.01, o[0]   # resting against the wall
    assert abs(o[2] - (-0.38)) < 2e-3, o[2]               # still on the plane


def test_cube_slides_off_the_table_edge_and_lands(oracle):
    """A cube sliding over the table's +x edge tips and falls past it at free-fall speeds (0.4 m:
    ~2.8 m/s), never thrown back up by the top face.  (Its fall is not a parabola: the restated
    floating base carries btMultiBody's base bias m (w x v) in the spinning base's frame, so a cube
    that tipped at the edge swings its velocity round as it spins.)"""
    cfg = _cfg()
    o = _obj((0.22, 0.0, 0.02), vel=(0.8, 0.0, 0.0))
    q = np.array(abi.NEUTRAL_Q[:7])
    qd = np.zeros(7)
    mot = _motors(oracle, q)
    vmax, zmax = 0.0, -1.0
    for _ in range(600):
        q, qd, o, st = oracle.world_substep(cfg, q, qd, o, mot)
        vmax = max(vmax, float(np.linalg.norm(o[7:10])))
        zmax = max(zmax, float(o[2]))
    assert vmax < 3.5 and zmax < 0.03, (vmax, zmax)
    assert o[0] > 0.27 and o[2] < -0.05, o[:3]     # over the edge and falling beside the table
