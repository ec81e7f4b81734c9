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
    o = np.zeros(29)
    o[0:3], o[3:7], o[7:10], o[10:13] = pos, quat, vel, w
    o[13::2] = -1.0
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
