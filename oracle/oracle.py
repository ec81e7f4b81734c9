"""TEST INFRASTRUCTURE ONLY: ctypes wrapper of the fp64 CPU oracle (oracle/_build/libpgx_oracle.so).

Importable only from tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg.  The product path (panda-gym_amd) never imports this module.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from typing import Optional, Tuple

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "libpgx_oracle.so")
FLOPS_LIB_PATH = os.path.join(HERE, "_build", "libpgx_oracle_flops.so")   # operation-counting build
FP32_LIB_PATH = os.path.join(HERE, "_build", "libpgx_oracle_fp32.so")     # the algorithm in fp32 arithmetic

_lib = None
_flops_lib = None
_fp32_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = C.CDLL(LIB_PATH)
        _lib.pgxo_ik.restype = C.c_int
        _lib.pgxo_distance_f32_f64.restype = C.c_double
        _lib.pgxo_distance_f32_f32.restype = C.c_float
        _lib.pgxo_vec_step.restype = C.c_int
        _lib.pgxo_vec_reset.restype = C.c_int
    return _lib


def flops_lib():
    """The operation-counting build of the same oracle (oracle/flops_count.cpp)."""
    global _flops_lib
    if _flops_lib is None:
        if not os.path.exists(FLOPS_LIB_PATH):
            build()
        _flops_lib = C.CDLL(FLOPS_LIB_PATH)
        for f in ("pgxo_vec_step", "pgxo_vec_reset", "pgxo_flops_nphase"):
            getattr(_flops_lib, f).restype = C.c_int
    return _flops_lib


def fp32_lib():
    """The same oracle evaluated in fp32 arithmetic (oracle/fp32_emul.cpp): every operation's
    result rounded to float -- the restated algorithm's own rounding envelope at the device's
    precision."""
    global _fp32_lib
    if _fp32_lib is None:
        if not os.path.exists(FP32_LIB_PATH):
            build()
        _fp32_lib = C.CDLL(FP32_LIB_PATH)
        for f in ("pgxo_vec_step", "pgxo_vec_reset"):
            getattr(_fp32_lib, f).restype = C.c_int
    return _fp32_lib


class PgxoFlops(C.Structure):
    _fields_ = [(k, C.c_int64) for k in ("add", "mul", "div", "sqrt", "trans", "cmp")]


FLOP_PHASES = ("action_ik", "detection", "dynamics", "row_setup", "pgs_sweeps", "integrate", "obs_reward",
               "reset", "ao_collision_check")


def read_flops(clear: bool = True) -> dict:
    """Per-phase operation counters of the counting build since the last clear."""
    lb = flops_lib()
    n = lb.pgxo_flops_nphase()
    assert n == len(FLOP_PHASES), n
    arr = (PgxoFlops * n)()
    lb.pgxo_flops_read(arr, int(clear))
    return {FLOP_PHASES[i]: {k: int(getattr(arr[i], k)) for k, _ in PgxoFlops._fields_} for i in range(n)}


class PgxoMotor(C.Structure):
    _fields_ = [("target_q", C.c_double), ("target_qd", C.c_double), ("kp", C.c_double), ("kd", C.c_double),
                ("max_impulse", C.c_double)]


class PgxoStats(C.Structure):
    _fields_ = [("solver_iterations", C.c_int32), ("ik_iterations", C.c_int32), ("ik_residual", C.c_double),
                ("limits_far", C.c_int32), ("n_contacts", C.c_int32)]


# obj[] (pgx_oracle.h): pos3 quat4 linvel3 angvel3, the contact cache (feature id, normal impulse)
# x (OBJECT_POINTS + ROBOT_MAX), ReachAO obstacles, the cached link pose qc[7] (getLinkState's
# pose: before the last substep)
OBJECT_POINTS = 4     # PGX_OBJECT_POINTS
ROBOT_POINTS = 12     # PGX_ROBOT_POINTS: robot slots of the kernels' cache (largest budget)
ROBOT_MAX = 16        # PGXO_ROBOT_MAX: the oracle's robot slots (its largest budget)
OBJ_CACHE = 13
OBJ_CACHE1 = OBJ_CACHE + 2 * OBJECT_POINTS
OBJ_AO = OBJ_CACHE1 + 2 * ROBOT_MAX   # ReachAO: obstacle centres [6][3], active flags [6] at OBJ_AO + 18
OBJ_QC = OBJ_AO + 24
POOL_MAX, MAN_PT = 48, 12     # PGXO_POOL_MAX, PGX_MANIFOLD_POINT: the persistent manifold pool
OBJ_MAN = OBJ_QC + 7          # count, then POOL_MAX x (kid, local A, local B, normal, distance, impulse)
OBJ_N = OBJ_MAN + 1 + POOL_MAX * MAN_PT
MP_KID, MP_LA, MP_LB, MP_N, MP_D, MP_IMP = 0, 1, 4, 7, 10, 11
ROBOT_HIST = 33


def set_robot_budget(budget: int = -1) -> None:
    """The oracle's robot contact budget (default / -1: the configuration's -- pgx_config.contacts 1:
    4 points, PGX_CONTACTS_FULL: 12 with an object, else 8); PandaVecEnv.robot_contact_budget()
    gives a handle's."""
    lib().pgxo_set_robot_budget(int(budget))


def pair_hist(clear: bool = True) -> np.ndarray:
    """Per substep since the last clear: how many robot points Bullet's per-pair manifold rule
    keeps before the budget (index = count, the last bin = that many or more)."""
    h = np.zeros(ROBOT_HIST, dtype=np.int64)
    lib().pgxo_pair_hist_read(h.ctypes.data_as(C.c_void_p), int(clear))
    return h


def breaking_thresholds(cfg) -> dict:
    """The contact breaking threshold of every pair the oracle uses (Bullet's relative rule,
    pgx_oracle.c breaking_thresholds; the global contact_distance under FLAG_GLOBAL_BREAKING):
    per capsule against the table / plane / cube / an obstacle, and the cube against the table /
    plane."""
    nc = 16
    out = np.zeros(4 * nc + 2)
    lib().pgxo_breaking_thresholds(C.byref(cfg), out.ctypes.data_as(C.c_void_p))
    return {"table": out[:nc], "plane": out[nc:2 * nc], "cube": out[2 * nc:3 * nc], "obstacle": out[3 * nc:4 * nc],
            "cube_table": float(out[4 * nc]), "cube_plane": float(out[4 * nc + 1])}


def last_contacts():
    """The points of the oracle's last contact detection: (group, feature id, link, separation) arrays."""
    m = OBJECT_POINTS + ROBOT_MAX
    g, i, l = (np.zeros(m, dtype=np.int32) for _ in range(3))
    d = np.zeros(m)
    n = lib().pgxo_last_contacts(*(a.ctypes.data_as(C.c_void_p) for a in (g, i, l, d)))
    return g[:n], i[:n], l[:n], d[:n]


def manifold_add(P: np.ndarray, key: int, point: np.ndarray, thr: float = 0.02, cap: int = POOL_MAX) -> int:
    """btPersistentManifold addContactPoint of point (MAN_PT: kid, local A, local B, normal, distance,
    impulse -- kid and impulse ignored) to manifold `key` of pool P [1 + cap * MAN_PT] (in place);
    the slot it went to, -1 when the pool was full."""
    lib().pgxo_manifold_add.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_double]
    return int(lib().pgxo_manifold_add(_p(P), int(cap), int(key), _p(_d(point)), thr))


def manifold_refresh_static(P: np.ndarray, thr: float = 0.02) -> None:
    """refreshContactPoints of every manifold in pool P whose bodies did not move (local = world)."""
    lib().pgxo_manifold_refresh_static.argtypes = [C.c_void_p, C.c_double]
    lib().pgxo_manifold_refresh_static(_p(P), thr)


def pool(obj_row: np.ndarray) -> np.ndarray:
    """The manifold pool of one env's obj row: its points [count, MAN_PT] in pool order."""
    n = int(obj_row[OBJ_MAN])
    return obj_row[OBJ_MAN + 1:OBJ_MAN + 1 + n * MAN_PT].reshape(n, MAN_PT).copy()


def manifolds(obj_row: np.ndarray) -> list:
    """The persistent manifolds of one env's obj row: [(key, points [n, MAN_PT] by slot)], keys in
    order of first appearance in the pool."""
    pts = pool(obj_row)
    out = {}
    for p in pts:
        kid = int(p[MP_KID])
        out.setdefault(kid & ~3, {})[kid & 3] = p
    return [(k, np.stack([v[s] for s in sorted(v)])) for k, v in out.items()]


def set_manifolds(obj: np.ndarray, man: np.ndarray) -> None:
    """obj[:, pool] from the kernels' pool [1 + pool * MAN_PT] per env (pgx_state_view.manifolds)."""
    man = np.asarray(man, dtype=np.float64)
    obj[:, OBJ_MAN:OBJ_N] = 0.0
    obj[:, OBJ_MAN:OBJ_MAN + man.shape[1]] = man


def set_contact_cache(obj: np.ndarray, cache: np.ndarray) -> None:
    """obj[:, cache] from the kernel's cache [2 * (OBJECT_POINTS + ROBOT_POINTS)] per env
    (object-scene slots, then robot slots); the oracle's remaining robot slots are empty."""
    cache = np.asarray(cache, dtype=np.float64)
    obj[:, OBJ_CACHE:OBJ_AO:2] = -1.0
    obj[:, OBJ_CACHE + 1:OBJ_AO:2] = 0.0
    obj[:, OBJ_CACHE:OBJ_CACHE1] = cache[:, :2 * OBJECT_POINTS]
    obj[:, OBJ_CACHE1:OBJ_CACHE1 + 2 * ROBOT_POINTS] = cache[:, 2 * OBJECT_POINTS:]


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def _d(a):
    return np.ascontiguousarray(a, dtype=np.float64)


def _base(base):
    return (C.c_double * 3)(*base)


def fk(model, q, base=(0.0, 0.0, 0.0)) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    n = model.n_links
    com = np.zeros((n, 3))
    rot = np.zeros((n, 9))
    org = np.zeros((n, 3))
    lib().pgxo_fk(C.byref(model), _base(base), _p(_d(q)), _p(com), _p(rot), _p(org))
    return com, rot.reshape(n, 3, 3), org


def link_velocity(model, q, qd, link, base=(0.0, 0.0, 0.0)):
    lin, ang = np.zeros(3), np.zeros(3)
    lib().pgxo_link_velocity(C.byref(model), _base(base), _p(_d(q)), _p(_d(qd)), link, _p(lin), _p(ang))
    return lin, ang


def mass_matrix(model, q, base=(0.0, 0.0, 0.0)):
    nd = model.n_dofs
    M = np.zeros((nd, nd))
    lib().pgxo_mass_matrix(C.byref(model), _base(base), _p(_d(q)), _p(M))
    return M


def bias(model, params, q, qd, with_gravity=True, base=(0.0, 0.0, 0.0)):
    b = np.zeros(model.n_dofs)
    lib().pgxo_bias(C.byref(model), C.byref(params), _base(base), _p(_d(q)), _p(_d(qd)), int(with_gravity), _p(b))
    return b


def dyn_recursive(model, params, q, qd, with_gravity=True, base=(0.0, 0.0, 0.0)):
    """(M, b) by composite rigid bodies + Newton-Euler (pgxo_dyn_recursive): the kernel's formulation."""
    nd = model.n_dofs
    M, b = np.zeros((nd, nd)), np.zeros(nd)
    lib().pgxo_dyn_recursive(C.byref(model), C.byref(params), _base(base), _p(_d(q)), _p(_d(qd)), int(with_gravity),
                             _p(M), _p(b))
    return M, b


def ik(model, params, q_start, link, target_pos, target_orn, base=(0.0, 0.0, 0.0)):
    out = np.zeros(model.n_dofs)
    st = PgxoStats()
    lib().pgxo_ik(C.byref(model), C.byref(params), _base(base), _p(_d(q_start)), link, _p(_d(target_pos)),
                  _p(_d(target_orn)), _p(out), C.byref(st))
    return out, st


def make_motors(n, entries):
    arr = (PgxoMotor * n)()
    for d, e in entries.items():
        arr[d].target_q, arr[d].target_qd, arr[d].kp, arr[d].kd, arr[d].max_impulse = e
    return arr


def substep(model, params, q, qd, motors, base=(0.0, 0.0, 0.0)):
    q = _d(q).copy()
    qd = _d(qd).copy()
    st = PgxoStats()
    lib().pgxo_substep(C.byref(model), C.byref(params), _base(base), _p(q), _p(qd), motors, C.byref(st))
    return q, qd, st


def world_substep(cfg, q, qd, obj, motors):
    """One substep of the task scene (contacts, object); returns new (q, qd, obj, stats)."""
    q = _d(q).copy()
    qd = _d(qd).copy()
    obj = _d(obj).copy()
    if obj.shape != (OBJ_N,):
        raise ValueError(f"obj must have the oracle layout ({OBJ_N} doubles), got {obj.shape}")
    st = PgxoStats()
    lib().pgxo_world_substep(C.byref(cfg), _p(q), _p(qd), _p(obj), motors, C.byref(st))
    return q, qd, obj, st


def ao_capsule_sphere(A, B, r, ctr, R):
    pa, pb = np.zeros(3), np.zeros(3)
    lib().pgxo_ao_capsule_sphere.restype = C.c_double
    d = lib().pgxo_ao_capsule_sphere(_p(_d(A)), _p(_d(B)), C.c_double(r), _p(_d(ctr)), C.c_double(R), _p(pa), _p(pb))
    return d, pa, pb


def ao_capsule_box(A, B, r, c, h):
    pa, pb = np.zeros(3), np.zeros(3)
    lib().pgxo_ao_capsule_box.restype = C.c_double
    d = lib().pgxo_ao_capsule_box(_p(_d(A)), _p(_d(B)), C.c_double(r), _p(_d(c)), _p(_d(h)), _p(pa), _p(pb))
    return d, pa, pb


def ao_link_distances(cfg, q, obstacles):
    """(dist[9], pa[9,3], pb[9,3], table distance) of ReachAO's collision links at q."""
    dist, pa, pb = np.zeros(9), np.zeros((9, 3)), np.zeros((9, 3))
    lib().pgxo_ao_link_distances.restype = C.c_double
    dt = lib().pgxo_ao_link_distances(C.byref(cfg), _p(_d(q)), _p(_d(obstacles)), _p(dist), _p(pa), _p(pb))
    return dist, pa, pb, dt


def ao_collided(cfg, q, obstacles) -> bool:
    return bool(lib().pgxo_ao_collided(C.byref(cfg), _p(_d(q)), _p(_d(obstacles))))


def distance_f32_f64(ag, g) -> float:
    a = np.ascontiguousarray(ag, dtype=np.float32)
    b = _d(g)
    return lib().pgxo_distance_f32_f64(_p(a), _p(b))


def compute_reward_f32(ag, dg, reward_type, thr=0.05):
    ag = np.ascontiguousarray(ag, dtype=np.float32).reshape(-1, 3)
    dg = np.ascontiguousarray(dg, dtype=np.float32).reshape(-1, 3)
    out = np.zeros(len(ag), dtype=np.float32)
    lib().pgxo_compute_reward_f32(_p(ag), _p(dg), C.c_int64(len(ag)), reward_type, C.c_double(thr), _p(out))
    return out


def philox(ctr, key):
    c = (C.c_uint32 * 4)(*ctr)
    k = (C.c_uint32 * 2)(*key)
    o = (C.c_uint32 * 4)()
    lib().pgxo_philox(c, k, o)
    return list(o)


class OracleVecEnv:
    """Host-side fp64 mirror of one libpgx handle (AoS state), same vec-env semantics."""

    def __init__(self, cfg, n: int, counting: bool = False, fp32: bool = False):
        """``counting``: run on the operation-counting build (read_flops) instead; ``fp32``: on
        the build that rounds every operation to float (fp32_lib)."""
        self._lib = flops_lib() if counting else (fp32_lib() if fp32 else lib())
        self.cfg = cfg
        self.n = n
        self.nd = cfg.model.contents.n_dofs
        from panda_gym_amd.abi import EnvSpec  # noqa: F401  (layout helpers only)
        if cfg.task == 3:
            self.od = 56
        else:
            self.od = 6 + (0 if cfg.block_gripper else 1) + (0 if cfg.task == 0 else 12)
        self.stats = PgxoStats()
        self.ad = (3 if cfg.control == 0 else 7) + (0 if cfg.block_gripper else 1)
        self.q = np.zeros((n, self.nd))
        self.qd = np.zeros((n, self.nd))
        self.goal = np.zeros((n, 3))
        self.obj = np.zeros((n, OBJ_N))
        self.obj[:, 6] = 1.0
        self.obj[:, OBJ_CACHE:OBJ_AO:2] = -1.0
        self.elapsed = np.zeros(n, dtype=np.int32)
        self.episode = np.zeros(n, dtype=np.uint32)

    def _bufs(self):
        n, od = self.n, self.od
        return dict(obs=np.zeros((n, od), np.float32), ag=np.zeros((n, 3), np.float32),
                    dg=np.zeros((n, 3), np.float32))

    def reset(self, mask: Optional[np.ndarray] = None, inject_goal: Optional[np.ndarray] = None,
              inject_obj: Optional[np.ndarray] = None):
        b = self._bufs()
        m = None if mask is None else np.ascontiguousarray(mask, dtype=np.uint8)
        g = None if inject_goal is None else _d(inject_goal)
        io = None if inject_obj is None else _d(inject_obj)
        rc = self._lib.pgxo_vec_reset(C.byref(self.cfg), C.c_int64(self.n), None if m is None else _p(m),
                                  None if g is None else _p(g), None if io is None else _p(io), _p(self.q),
                                  _p(self.qd), _p(self.goal),
                                  _p(self.obj), _p(self.elapsed), _p(self.episode), _p(b["obs"]), _p(b["ag"]),
                                  _p(b["dg"]))
        assert rc == 0, rc
        return b

    def step(self, action: np.ndarray, margins: bool = False):
        """One vec step.  ``margins`` (ReachAO): also return, per env, the smallest |margin| of
        check_collided over the substep checks that ran ("margin_abs") and the margin at the last
        one ("margin_last"); collided <=> margin <= 0 (pgxo_diag_collision_margin)."""
        a = np.ascontiguousarray(action, dtype=np.float32)
        b = self._bufs()
        n = self.n
        b.update(reward=np.zeros(n, np.float32), success=np.zeros(n, np.uint8), terminated=np.zeros(n, np.uint8),
                 truncated=np.zeros(n, np.uint8), terminal_obs=np.zeros((n, self.od), np.float32))
        if margins:
            b.update(margin_abs=np.full(n, np.inf), margin_last=np.full(n, np.inf))
            self._lib.pgxo_diag_collision_margin(_p(b["margin_abs"]), _p(b["margin_last"]), C.c_int64(n))
        rc = self._lib.pgxo_vec_step(C.byref(self.cfg), C.c_int64(n), _p(self.q), _p(self.qd), _p(self.goal),
                                 _p(self.obj), _p(self.elapsed), _p(self.episode), _p(a), _p(b["obs"]), _p(b["ag"]),
                                 _p(b["dg"]), _p(b["reward"]), _p(b["success"]), _p(b["terminated"]),
                                 _p(b["truncated"]), _p(b["terminal_obs"]))
        if margins:
            self._lib.pgxo_diag_collision_margin(None, None, C.c_int64(0))
        assert rc == 0, rc
        return b

    @property
    def obstacles(self) -> np.ndarray:
        """ReachAO obstacle centres [n, 6, 3] (a view)."""
        return self.obj[:, OBJ_AO:OBJ_AO + 18].reshape(self.n, 6, 3)

    @property
    def qc(self) -> np.ndarray:
        """The cached link pose [n, 7] getLinkState reports (a view)."""
        return self.obj[:, OBJ_QC:OBJ_QC + 7]

    @property
    def active(self) -> np.ndarray:
        return self.obj[:, OBJ_AO + 18:OBJ_AO + 24]

    def take_errors(self) -> int:
        """PGX_ERR_* bits the resets set since the last call (the device errors word)."""
        self._lib.pgxo_take_errors.restype = C.c_uint32
        return int(self._lib.pgxo_take_errors())

    def sample_actions(self, step: int) -> np.ndarray:
        a = np.zeros((self.n, self.ad), np.float32)
        self._lib.pgxo_sample_actions(C.byref(self.cfg), C.c_int64(self.n), C.c_uint64(step), _p(a))
        return a
