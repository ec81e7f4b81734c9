"""ctypes mirror of include/pgx.h and builders for its structs.

Only plain C structs cross the boundary (no torch types): the same structs are
handed to libpgx.so (the HIP product) and, in tests, to the oracle library.
Default constants are the ones the reference uses; each carries its citation.
"""
from __future__ import annotations

import ctypes as C
import math
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np

from .model import Model, MAX_LINKS, MAX_DOFS, load_model

MAX_ROWS = 27
MAX_CAPSULES = 16
OBJECT_POINTS = 4             # PGX_OBJECT_POINTS: object vs table / plane contact budget
ROBOT_POINTS = 12             # PGX_ROBOT_POINTS: robot contact budget, Push / PickAndPlace (16 lanes)
ROBOT_POINTS_ARM = 8          # PGX_ROBOT_POINTS_ARM: Reach / ReachAO (16 lanes)
ROBOT_POINTS_ONE_LANE = 4     # PGX_ROBOT_POINTS_ONE_LANE: the one-lane layout
CONTACT_SLOTS = OBJECT_POINTS + ROBOT_POINTS
CONTACTS_FULL = 2             # PGX_CONTACTS_FULL: pgx_config.contacts for the full manifold budget
MANIFOLD_POOL = 16            # PGX_MANIFOLD_POOL: persistent manifold points per env (Push / PickAndPlace)
MANIFOLD_POOL_AO = 8          # PGX_MANIFOLD_POOL_AO: ReachAO
MANIFOLD_POINT = 12           # PGX_MANIFOLD_POINT: kid, local A[3], local B[3], normal[3], distance, impulse
PCG64_WORDS = 6               # PGX_PCG64_WORDS: state_lo, state_hi, inc_lo, inc_hi, has_uint32, uinteger
CAP_VS_TABLE, CAP_VS_OBJECT = 1, 2

TASK_REACH, TASK_PUSH, TASK_PICK_AND_PLACE, TASK_REACH_AO = 0, 1, 2, 3
AO_OBSTACLES, AO_LINKS = 6, 9
CONTROL_EE, CONTROL_JOINTS = 0, 1
REWARD_SPARSE, REWARD_DENSE, REWARD_SPARSE_AO = 0, 1, 2
REWARD_CODES = {"sparse": REWARD_SPARSE, "dense": REWARD_DENSE, "sparse_ao": REWARD_SPARSE_AO}

FLAG_CONSTRAINT_PASS_BIAS = 1
FLAG_IK_COM = 2
FLAG_NO_RESIDUAL_EXIT = 4
FLAG_LINKSTATE_CURRENT = 8   # getLinkState at the pose after the last substep (rejected hypothesis)
FLAG_DYN_RECURSIVE = 16      # oracle: M, b by CRBA + Newton-Euler (the kernel's formulation), for the op count
FLAG_PERSISTENT_MANIFOLD = 32  # oracle study: the table / plane pairs through persistent manifolds too
FLAG_FRESH_MANIFOLD = 64       # oracle study: round 4's per-substep rule for the cube / obstacle pairs
FLAG_GLOBAL_BREAKING = 128     # oracle study: the global 0.02 breaking threshold for every pair (rounds 2-5)

HER_FUTURE, HER_FINAL, HER_EPISODE = 0, 1, 2

PGX_OK = 0
PGX_E_INVALID, PGX_E_HIP, PGX_E_UNSUPPORTED, PGX_E_NOMEM = -1, -2, -3, -4


class PgxModel(C.Structure):
    _fields_ = [
        ("n_links", C.c_int32), ("n_dofs", C.c_int32), ("ee_link", C.c_int32), ("n_rows", C.c_int32),
        ("parent", C.c_int32 * MAX_LINKS), ("jtype", C.c_int32 * MAX_LINKS),
        ("dof_of_link", C.c_int32 * MAX_LINKS), ("link_of_dof", C.c_int32 * MAX_DOFS),
        ("has_limit", C.c_int32 * MAX_DOFS), ("row_kind", C.c_int32 * MAX_ROWS),
        ("row_dof", C.c_int32 * MAX_ROWS), ("pad0", C.c_int32),
        ("jpos", (C.c_double * 3) * MAX_LINKS), ("jrot", (C.c_double * 9) * MAX_LINKS),
        ("axis", (C.c_double * 3) * MAX_LINKS), ("com", (C.c_double * 3) * MAX_LINKS),
        ("mass", C.c_double * MAX_LINKS), ("inertia", (C.c_double * 3) * MAX_LINKS),
        ("lower", C.c_double * MAX_DOFS), ("upper", C.c_double * MAX_DOFS),
        ("n_capsules", C.c_int32), ("pad1", C.c_int32),
        ("cap_link", C.c_int32 * MAX_CAPSULES), ("cap_flags", C.c_int32 * MAX_CAPSULES),
        ("cap_a", (C.c_double * 3) * MAX_CAPSULES), ("cap_b", (C.c_double * 3) * MAX_CAPSULES),
        ("cap_radius", C.c_double * MAX_CAPSULES),
        ("link_aabb_center", (C.c_double * 3) * MAX_LINKS), ("link_aabb_half", (C.c_double * 3) * MAX_LINKS),
    ]


class PgxSimParams(C.Structure):
    _fields_ = [
        ("dt", C.c_double), ("gravity", C.c_double * 3), ("lin_damping", C.c_double),
        ("ang_damping", C.c_double), ("max_coord_vel", C.c_double), ("residual_threshold", C.c_double),
        ("erp", C.c_double), ("limit_max_impulse", C.c_double), ("motor_kp", C.c_double),
        ("motor_kd", C.c_double), ("ik_residual", C.c_double), ("ik_damping", C.c_double),
        ("ik_max_angle", C.c_double), ("n_substeps", C.c_int32), ("num_iterations", C.c_int32),
        ("ik_max_iters", C.c_int32), ("flags", C.c_int32),
        ("contact_distance", C.c_double), ("contact_erp", C.c_double), ("friction", C.c_double),
        ("warmstart", C.c_double), ("link_friction", C.c_double * MAX_LINKS),
    ]


class PgxConfig(C.Structure):
    _fields_ = [
        ("task", C.c_int32), ("control", C.c_int32), ("reward", C.c_int32), ("n_envs", C.c_int32),
        ("max_episode_steps", C.c_int32), ("block_gripper", C.c_int32), ("no_auto_reset", C.c_int32),
        ("pad1", C.c_int32), ("seed", C.c_uint64), ("env_id_offset", C.c_uint64),
        ("base_pos", C.c_double * 3), ("distance_threshold", C.c_double),
        ("goal_low", C.c_double * 3), ("goal_high", C.c_double * 3),
        ("joint_forces", C.c_double * MAX_DOFS), ("neutral_q", C.c_double * MAX_DOFS),
        ("ee_step", C.c_double), ("joint_step", C.c_double),
        ("model", C.POINTER(PgxModel)), ("params", C.POINTER(PgxSimParams)),
        ("contacts", C.c_int32), ("lanes_per_env", C.c_int32),
        ("goal_offset", C.c_double * 3), ("goal_z_zero_prob", C.c_double),
        ("obj_low", C.c_double * 3), ("obj_high", C.c_double * 3), ("obj_offset", C.c_double * 3),
        ("object_half", C.c_double), ("object_mass", C.c_double), ("object_inertia", C.c_double),
        ("table_center", C.c_double * 3), ("table_half", C.c_double * 3), ("plane_z", C.c_double),
        ("terminate_on_success", C.c_int32), ("pad3", C.c_int32), ("collision_reward", C.c_double),
        ("ao_ee_neutral", C.c_double * 3),
        ("ao_capsules_neutral", (C.c_double * 7) * MAX_CAPSULES),
    ]


ERR_AO_OBSTACLE = 1   # PGX_ERR_AO_OBSTACLE (include/pgx.h): pgx_state_view.errors bit


class PgxStepOut(C.Structure):
    _fields_ = [
        ("obs", C.c_void_p), ("achieved_goal", C.c_void_p), ("desired_goal", C.c_void_p),
        ("reward", C.c_void_p), ("success", C.c_void_p), ("terminated", C.c_void_p),
        ("truncated", C.c_void_p), ("terminal_obs", C.c_void_p), ("terminal_achieved_goal", C.c_void_p),
        ("terminal_desired_goal", C.c_void_p), ("task_truncated", C.c_void_p),
    ]


class PgxStateView(C.Structure):
    _fields_ = [
        ("q", C.c_void_p), ("qd", C.c_void_p), ("qc", C.c_void_p), ("goal", C.c_void_p), ("object", C.c_void_p),
        ("contacts", C.c_void_p), ("obstacles", C.c_void_p), ("elapsed", C.c_void_p), ("episode", C.c_void_p),
        ("errors", C.c_void_p), ("robot_points", C.c_int32),
        ("env_order", C.c_void_p), ("manifolds", C.c_void_p), ("manifold_pool", C.c_int32),
    ]


class PgxReplayConfig(C.Structure):
    _fields_ = [
        ("n_envs", C.c_int32), ("capacity", C.c_int32), ("obs_dim", C.c_int32), ("action_dim", C.c_int32),
        ("reward_type", C.c_int32), ("strategy", C.c_int32), ("distance_threshold", C.c_double),
        ("her_ratio", C.c_double), ("seed", C.c_uint64),
    ]


class PgxTransition(C.Structure):
    _fields_ = [
        ("obs", C.c_void_p), ("achieved_goal", C.c_void_p), ("desired_goal", C.c_void_p), ("action", C.c_void_p),
        ("reward", C.c_void_p), ("next_obs", C.c_void_p), ("next_achieved_goal", C.c_void_p),
        ("next_desired_goal", C.c_void_p), ("done", C.c_void_p), ("timeout", C.c_void_p),
    ]


class PgxReplayBatch(C.Structure):
    _fields_ = [("rows", C.c_void_p), ("slot", C.c_void_p), ("env", C.c_void_p), ("goal_slot", C.c_void_p)]


def replay_row_fields(obs_dim: int, action_dim: int):
    """(name, offset, width) of the batch row layout of include/pgx.h, plus row_dim."""
    f, o = [], 0
    for name, w in (("obs", obs_dim), ("achieved_goal", 3), ("desired_goal", 3), ("action", action_dim),
                    ("reward", 1), ("next_obs", obs_dim), ("next_achieved_goal", 3), ("next_desired_goal", 3),
                    ("done", 1)):
        f.append((name, o, w))
        o += w
    return f, o


def make_model(model: Model, ee_link: int = 11) -> PgxModel:
    m = PgxModel()
    m.n_links, m.n_dofs, m.ee_link = model.n_links, model.n_dofs, ee_link
    assert model.n_links <= MAX_LINKS and model.n_dofs <= MAX_DOFS
    kinds, dofs = model.row_table()
    m.n_rows = len(kinds)
    for i in range(model.n_links):
        m.parent[i] = model.parent[i]
        m.jtype[i] = model.jtype[i]
        m.dof_of_link[i] = model.dof_of_link[i]
        for c in range(3):
            m.jpos[i][c] = model.jpos[i][c]
            m.axis[i][c] = model.axis[i][c]
            m.com[i][c] = model.com[i][c]
            m.inertia[i][c] = model.inertia[i][c]
        for c in range(9):
            m.jrot[i][c] = model.jrot[i][c]
        m.mass[i] = model.mass[i]
    for d in range(model.n_dofs):
        m.link_of_dof[d] = model.link_of_dof[d]
        m.has_limit[d] = model.has_limit[d]
        m.lower[d] = model.lower[d]
        m.upper[d] = model.upper[d]
    for r, (k, d) in enumerate(zip(kinds, dofs)):
        m.row_kind[r], m.row_dof[r] = int(k), int(d)
    caps = model.capsules(base_capsule=model.name == "panda_custom0")
    assert len(caps) <= MAX_CAPSULES
    m.n_capsules = len(caps)
    for i, c in enumerate(caps):
        m.cap_link[i], m.cap_flags[i], m.cap_radius[i] = c["link"], c["flags"], c["r"]
        for k in range(3):
            m.cap_a[i][k], m.cap_b[i][k] = c["a"][k], c["b"][k]
    assert len(model.aabb_half) == model.n_links, "model table without link AABBs: rerun tools/build_models.py"
    for i in range(model.n_links):
        for k in range(3):
            m.link_aabb_center[i][k] = model.aabb_center[i][k]
            m.link_aabb_half[i][k] = model.aabb_half[i][k]
    return m


def default_sim_params(n_substeps: int = 20, flags: int = 0) -> PgxSimParams:
    """pybullet defaults as configured by the reference's PyBullet facade."""
    p = PgxSimParams()
    p.dt = 1.0 / 500                         # panda_gym/pybullet.py:50
    p.gravity[0], p.gravity[1], p.gravity[2] = 0.0, 0.0, -9.81   # pybullet.py:54
    p.lin_damping = 0.04                     # btMultiBody m_linearDamping
    p.ang_damping = 0.04                     # btMultiBody m_angularDamping
    p.max_coord_vel = 100.0                  # btMultiBody m_maxCoordinateVelocity
    p.residual_threshold = 1e-7              # pybullet solverResidualThreshold
    p.erp = 0.2                              # btContactSolverInfo m_erp
    p.limit_max_impulse = 100.0              # btMultiBodyConstraint m_maxAppliedImpulse
    p.motor_kp = 0.1                         # setJointMotorControlArray positionGains default
    p.motor_kd = 1.0                         # setJointMotorControlArray velocityGains default
    p.ik_residual = 1e-4                     # calculateInverseKinematics residualThreshold
    p.ik_damping = 0.5                       # per-joint DLS damping default
    p.ik_max_angle = math.pi / 4             # BussIK Jacobian::MaxAngleDLS
    p.n_substeps = n_substeps                # pybullet.py:25
    p.num_iterations = 50                    # pybullet numSolverIterations
    p.ik_max_iters = 20                      # calculateInverseKinematics maxNumIterations
    p.flags = flags
    p.contact_distance = 0.02                # gContactBreakingThreshold (scaled per pair: pgx.h)
    p.contact_erp = 0.2                      # btMultiBodyConstraintSolver: contacts use m_erp
    p.friction = 0.5 * 0.5                   # default lateral friction 0.5 per body, product combine
    p.warmstart = 0.85                       # btContactSolverInfo m_warmstartingFactor
    # robot links against the scene (0.5 each): 0.5 x the link's lateral friction; Panda.__init__
    # sets links 9, 10 (fingers_indices: panda_ee, panda_leftfinger in custom_0) to 1.0 (panda.py:69-70)
    for i in range(MAX_LINKS):
        p.link_friction[i] = 0.5 * (1.0 if i in FINGER_FRICTION_LINKS else 0.5)
    return p


NEUTRAL_Q = [0.0, -0.3, 0.0, -2.2, 0.0, 2.0, math.pi / 4, 0.0, 0.0]        # panda.py:67
FINGER_FRICTION_LINKS = (9, 10)   # Panda.fingers_indices (panda.py:66), lateral friction 1.0 (panda.py:69-70)
JOINT_FORCES = [87.0, 87.0, 87.0, 87.0, 12.0, 120.0, 120.0, 170.0, 170.0]  # panda.py:63


@dataclass
class EnvSpec:
    """Task/robot configuration of one registered env id (panda_gym/__init__.py:23-91)."""

    task: int = TASK_REACH
    control: int = CONTROL_EE
    reward: int = REWARD_SPARSE
    max_episode_steps: int = 50
    block_gripper: bool = True
    base_pos: Sequence[float] = (-0.6, 0.0, 0.0)       # panda_tasks.py:49,66,85
    distance_threshold: float = 0.05                   # reach.py:15
    goal_range: float = 0.3                            # reach.py:16
    collision_reward: float = -100.0                   # ReachAO only: train_config.py:33

    @classmethod
    def reach_ao(cls, max_episode_steps: int = 50) -> "EnvSpec":
        """PandaReachAO-v3 with TrainConfig defaults (panda_tasks.py:132-159,
        train_config.py:25-59): base at the origin, joint control, sparse reward,
        terminate on success, ee_error_threshold float32(0.05) (reach_ao.py:71)."""
        import numpy as np
        return cls(task=TASK_REACH_AO, control=CONTROL_JOINTS, reward=REWARD_SPARSE,
                   max_episode_steps=max_episode_steps, block_gripper=True, base_pos=(0.0, 0.0, 0.0),
                   distance_threshold=float(np.float32(0.05)))

    def obj_bounds(self):
        """push.py:24-25 / pick_and_place.py:26-27: noise ranges of the object position."""
        return [-0.15, -0.15, 0.0], [0.15, 0.15, 0.0]

    def goal_bounds(self):
        if self.task == TASK_REACH:   # reach.py:24-25
            g = self.goal_range
            return [-g / 2, -g / 2, 0.0], [g / 2, g / 2, g]
        if self.task == TASK_PUSH:    # push.py:22-23 (+ z offset object_size/2 added at sample)
            return [-0.15, -0.15, 0.0], [0.15, 0.15, 0.0]
        return [-0.15, -0.15, 0.0], [0.15, 0.15, 0.2]  # pick_and_place.py:24-25

    @property
    def obs_dim(self) -> int:
        if self.task == TASK_REACH_AO:   # ("ee","js") 20 + vectors+closest_per_link 36
            return 20 + 4 * AO_LINKS
        return 6 + (0 if self.block_gripper else 1) + (0 if self.task == TASK_REACH else 12)

    @property
    def action_dim(self) -> int:
        return (3 if self.control == CONTROL_EE else 7) + (0 if self.block_gripper else 1)


def make_config(spec: EnvSpec, n_envs: int, model: PgxModel, params: PgxSimParams, seed: int = 0,
                env_id_offset: int = 0, contacts: bool = True, lanes_per_env: int = 0,
                full_manifold: bool = False) -> PgxConfig:
    c = PgxConfig()
    c.lanes_per_env = lanes_per_env   # step layout: 0 auto, 1 or 16 (include/pgx.h)
    c.task, c.control, c.reward = spec.task, spec.control, spec.reward
    c.n_envs = n_envs
    c.max_episode_steps = spec.max_episode_steps
    c.block_gripper = 1 if spec.block_gripper else 0
    c.seed = seed & 0xFFFFFFFFFFFFFFFF
    c.env_id_offset = env_id_offset
    for i in range(3):
        c.base_pos[i] = spec.base_pos[i]
    c.distance_threshold = spec.distance_threshold
    lo, hi = spec.goal_bounds()
    for i in range(3):
        c.goal_low[i], c.goal_high[i] = lo[i], hi[i]
    for d in range(MAX_DOFS):
        c.joint_forces[d] = JOINT_FORCES[d]
        c.neutral_q[d] = NEUTRAL_Q[d]
    c.ee_step = 0.05        # panda.py:235
    c.joint_step = 0.05     # panda.py:74 max_change_position
    c.model = C.pointer(model)
    c.params = C.pointer(params)
    c.contacts = (CONTACTS_FULL if full_manifold else 1) if contacts else 0
    half = OBJECT_SIZE / 2
    if spec.task != TASK_REACH:
        c.goal_offset[2] = half                   # push.py:77 / pick_and_place.py:73 (cube centre)
        c.obj_offset[2] = half
        olo, ohi = spec.obj_bounds()
        for i in range(3):
            c.obj_low[i], c.obj_high[i] = olo[i], ohi[i]
    c.goal_z_zero_prob = 0.3 if spec.task == TASK_PICK_AND_PLACE else 0.0   # pick_and_place.py:75-76
    c.object_half = half
    c.object_mass = 1.0                           # push.py:36
    c.object_inertia = box_inertia(OBJECT_MASS, half)
    ao = spec.task == TASK_REACH_AO
    for i in range(3):  # create_table(1.1, 0.7, 0.4, x_offset=-0.3); ReachAO create_table(2.0, 1.3, 0.4) (reach_ao.py:272)
        c.table_center[i] = ((0.0, 0.0, -0.2) if ao else (-0.3, 0.0, -0.2))[i]
        c.table_half[i] = ((1.0, 0.65, 0.2) if ao else (0.55, 0.35, 0.2))[i]
    c.plane_z = -0.4                              # create_plane(z_offset=-0.4): box top
    c.terminate_on_success = 1 if ao else 0       # core.py:265 / train_config.py:28
    c.collision_reward = spec.collision_reward if ao else 0.0    # train_config.py:33
    return c


OBJECT_SIZE = 0.04     # push.py:21
OBJECT_MASS = 1.0


def box_inertia(mass: float, half: float) -> float:
    """Principal inertia of the cube as pybullet computes it for createMultiBody: the
    URDF importer's compound (margin 0.001) around the box child, inertia from the
    compound AABB (btCompoundShape::calculateLocalInertia): half extents h + 0.001."""
    from .model import URDF_MARGIN
    e = 2.0 * (half + URDF_MARGIN)
    return mass / 12.0 * (e * e + e * e)


def ptr(a: Optional[np.ndarray]):
    """Raw pointer of a host numpy array (or None)."""
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(C.c_void_p)
