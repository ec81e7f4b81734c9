"""Pin the fp64 oracle against the reference's own known-answer tests.

The reference's physics is pybullet (absent here); test/pybullet_test.py holds
the only numeric answers for it, all on the upstream franka_panda URDF at
atol=1e-3.  These tests replay the same scenarios through the oracle.
"""
import math

import numpy as np
import pytest

from panda_gym_amd import abi
from panda_gym_amd.model import load_model, forward_kinematics

ATOL = 1e-3  # the reference tests' tolerance


def test_link_position_com_convention(oracle, upstream_model):
    """test/pybullet_test.py:124-136: link 1 position at q=0 is the COM [0, 0.060, 0.373]."""
    com, _, _ = oracle.fk(upstream_model, np.zeros(9))
    assert np.allclose(com[1], [0.000, 0.060, 0.373], atol=ATOL)


def test_inverse_kinematics_known_answer(oracle, upstream_model):
    """test/pybullet_test.py:254-266 (IK of link 6 to pos/orn from q=0)."""
    p = abi.default_sim_params()
    q, st = oracle.ik(upstream_model, p, np.zeros(9), 6, [0.4, 0.5, 0.6], [0.707, -0.02, 0.02, 0.707])
    expected = [1.000, 1.223, -1.113, -0.021, -0.917, 0.666, -0.499, 0.0, 0.0]
    assert np.allclose(q, expected, atol=ATOL), q
    assert st.ik_iterations == 20


def test_ik_alternative_hypothesis_rejected(oracle, upstream_model):
    """Targeting the link COM (instead of the joint pivot) misses the known answer."""
    p = abi.default_sim_params(flags=abi.FLAG_IK_COM)
    q, _ = oracle.ik(upstream_model, p, np.zeros(9), 6, [0.4, 0.5, 0.6], [0.707, -0.02, 0.02, 0.707])
    expected = [1.000, 1.223, -1.113, -0.021, -0.917, 0.666, -0.499, 0.0, 0.0]
    assert not np.allclose(q, expected, atol=ATOL)


def _control_joint5_step(oracle, model, flags=0, history=False):
    """control_joints("panda", [5], [0.3], [5.0]) then PyBullet.step(): POSITION_CONTROL on joint 5
    (kp 0.1, kd 1, max force 5); every other joint keeps pybullet's default velocity motor
    (target 0, kd 1, max impulse 1); 20 substeps of 1/500 s.  ``history``: also the pose the
    last substep started from (getLinkState's cached link pose, pgx_oracle.c link_state_cached)."""
    p = abi.default_sim_params(flags=flags)
    entries = {d: (0.0, 0.0, 0.0, 1.0, 1.0) for d in range(9)}
    entries[5] = (0.3, 0.0, 0.1, 1.0, 5.0 * p.dt)
    motors = oracle.make_motors(9, entries)
    q, qd = np.zeros(9), np.zeros(9)
    qc = q
    for _ in range(20):
        qc = q
        q, qd, _ = oracle.substep(model, p, q, qd, motors)
    return (q, qd, qc) if history else (q, qd)


def _link_state(oracle, model, q, qd, qc, link):
    """getLinkState(link, computeLinkVelocity=1): the cached pose qc for position / orientation,
    the local velocity at (q, qd) turned to world with the cached rotation."""
    from scipy.spatial.transform import Rotation

    _, rot, _ = oracle.fk(model, q)
    _, rotc, _ = oracle.fk(model, qc)
    lin, ang = oracle.link_velocity(model, q, qd, link)
    Rrel = rotc[link] @ rot[link].T
    quat = Rotation.from_matrix(rotc[link]).as_quat()
    return quat if quat[3] >= 0 else -quat, Rrel @ lin, Rrel @ ang


def test_joint_angle_known_answer(oracle, upstream_model):
    """test/pybullet_test.py:190-204: joint 5 angle 0.063 after one env step (getJointState: the
    current pose)."""
    q, _ = _control_joint5_step(oracle, upstream_model)
    assert abs(q[5] - 0.063) < ATOL, q[5]


def test_link_state_known_answers_jointly(oracle, upstream_model):
    """test/pybullet_test.py:139-187 after the same step: link 5's orientation
    [0.707, -0.02, 0.02, 0.707], COM velocity [-0.0068, 0, 0.1186] and angular velocity
    [0, -2.969, 0], all at atol 1e-3, together with the joint angle 0.063 of :190-204 -- which
    holds only with getLinkState reporting Bullet's cached link pose (the pose the last substep
    was solved at; velocities from the current local state, turned with the cached rotation)."""
    q, qd, qc = _control_joint5_step(oracle, upstream_model, history=True)
    quat, lin, ang = _link_state(oracle, upstream_model, q, qd, qc, 5)
    assert abs(q[5] - 0.063) < ATOL
    assert np.allclose(quat, [0.707, -0.02, 0.02, 0.707], atol=ATOL), quat
    assert np.allclose(lin, [-0.0068, 0.0, 0.1186], atol=ATOL), lin
    assert np.allclose(ang, [0.0, -2.969, 0.0], atol=ATOL), ang
    assert np.abs(lin - [-0.0068, 0.0, 0.1186]).max() < 1e-4   # 3e-5 off (current-pose rule: 6.7e-4)


def test_link_state_at_current_pose_rejected(oracle, upstream_model):
    """The alternative -- link states at the pose after the last substep -- misses the orientation
    answer: y = -0.7068 sin(0.0627 / 2) = -0.0222, 2.2e-3 from -0.02 (the joint angle answer pins
    q5 within 1e-3, so no pose consistent with :190-204 gives -0.02 at 1e-3 this way)."""
    q, qd = _control_joint5_step(oracle, upstream_model)
    quat, lin, _ = _link_state(oracle, upstream_model, q, qd, q, 5)
    assert not np.allclose(quat, [0.707, -0.02, 0.02, 0.707], atol=ATOL)
    assert abs(quat[1] + 0.7068 * math.sin(q[5] / 2)) < 1e-3


def test_vec_step_reports_the_cached_link_pose(oracle, custom_model):
    """The env step (pgxo_vec_step) reports the EE from the cached pose: obs = COM at the pose
    before the last substep (oracle.qc), velocity turned with its rotation; with
    PGX_FLAG_LINKSTATE_CURRENT it reports the current pose instead."""
    from oracle import oracle as O

    outs = {}
    for flags in (0, abi.FLAG_LINKSTATE_CURRENT):
        p = abi.default_sim_params(flags=flags)
        cfg = abi.make_config(abi.EnvSpec(control=abi.CONTROL_JOINTS), 4, custom_model, p, seed=3)
        env = O.OracleVecEnv(cfg, 4)
        env.reset()
        a = env.sample_actions(0)
        b = env.step(a)
        com_c, _, _ = O.fk(custom_model, env.qc[0], base=(-0.6, 0, 0))
        com, _, _ = O.fk(custom_model, env.q[0], base=(-0.6, 0, 0))
        outs[flags] = (b["obs"][0, :3].astype(np.float64), com_c[11], com[11])
    got, at_qc, at_q = outs[0]
    assert np.allclose(got, at_qc, atol=1e-6) and np.abs(at_q - at_qc).max() > 1e-4
    got2, _, at_q2 = outs[abi.FLAG_LINKSTATE_CURRENT]
    assert np.allclose(got2, at_q2, atol=1e-6)


def test_double_bias_hypothesis_rejected(oracle, upstream_model):
    """Re-applying velocity bias in Bullet's constraint pass misses the angular-velocity answer."""
    q, qd = _control_joint5_step(oracle, upstream_model, flags=abi.FLAG_CONSTRAINT_PASS_BIAS)
    _, ang = oracle.link_velocity(upstream_model, q, qd, 5)
    assert abs(ang[1] - (-2.969)) > ATOL


def test_dt():
    """test/pybullet_test.py:30-35: env dt = timestep * n_substeps = 0.04."""
    p = abi.default_sim_params()
    assert math.isclose(p.dt * p.n_substeps, 0.04)


def test_mass_matrix_symmetric_positive(oracle, custom_model):
    q = [0.0, -0.3, 0.0, -2.2, 0.0, 2.0, math.pi / 4]
    M = oracle.mass_matrix(custom_model, q, base=(-0.6, 0, 0))
    assert np.allclose(M, M.T, atol=1e-12)
    assert np.all(np.linalg.eigvalsh(M) > 0)


def test_gravity_bias_matches_potential_gradient(oracle, custom_model):
    """b(q, 0) with gravity equals dV/dq of the link masses (finite differences)."""
    model = load_model("panda_custom0")
    p = abi.default_sim_params()
    q = np.array([0.1, -0.3, 0.2, -2.2, 0.1, 2.0, 0.7])

    def V(qq):
        C = forward_kinematics(model, qq, base_pos=(-0.6, 0, 0))["C"]
        return sum(m * 9.81 * C[i][2] for i, m in enumerate(model.mass))

    grad = np.array([(V(q + e) - V(q - e)) / 2e-6 for e in np.eye(7) * 1e-6])
    b = oracle.bias(custom_model, p, q, np.zeros(7), True, base=(-0.6, 0, 0))
    assert np.allclose(b, grad, atol=1e-5)


def test_free_fall_base_velocity_known_answer(oracle):
    """test/pybullet_test.py:56-64: a 1 kg box (half extents 0.5) created at rest, one env step
    (20 substeps of 1/500 s) later, has base velocity [0, 0, -0.392] at atol 1e-3 -- the
    floating-base path the cube takes (gravity, the base's damping m v (k + k|v|), the
    semi-implicit update).  The oracle's scene has a table and a plane, so the box starts 10 m
    up, far from both and from the robot; the reference's PyBullet() has neither."""
    from oracle import oracle as orc

    model = abi.make_model(load_model("panda_custom0"), ee_link=11)
    params = abi.default_sim_params()
    cfg = abi.make_config(abi.EnvSpec(task=abi.TASK_PUSH), 1, model, params)
    cfg.object_half, cfg.object_mass = 0.5, 1.0
    cfg.object_inertia = 1.0 * (2 * 0.5) ** 2 / 6.0   # box formula, 1 m edge
    obj = np.zeros(orc.OBJ_N)
    obj[0:3], obj[3:7] = (0.0, 0.0, 10.0), (0.0, 0.0, 0.0, 1.0)
    obj[orc.OBJ_CACHE:orc.OBJ_AO:2] = -1.0
    q, qd = np.array(abi.NEUTRAL_Q[:7]), np.zeros(7)
    mot = oracle.make_motors(7, {d: (q[d], 0.0, 0.1, 1.0, abi.JOINT_FORCES[d] / 500.0) for d in range(7)})
    for _ in range(20):
        q, qd, obj, st = oracle.world_substep(cfg, q, qd, obj, mot)
        assert st.n_contacts == 0
    assert np.allclose(obj[7:10], [0.0, 0.0, -0.392], atol=ATOL), obj[7:10]
    assert np.array_equal(obj[10:13], np.zeros(3))
    # without the base's damping the same step gives g * 0.04 = -0.3924 exactly: the answer pins
    # gravity and the update, and the damping keeps it within the tolerance (-0.39209)
    assert -0.3924 < obj[9] < -0.3920
    # the velocity the damping leaves, in closed form: v <- v + dt (g - (k + k|v|) v) twenty times
    v = 0.0
    for _ in range(20):
        v = v + (1.0 / 500.0) * (-9.81 - (0.04 + 0.04 * abs(v)) * v)
    assert abs(obj[9] - v) < 1e-12
