"""Vectorised Panda environments on MI355X: the reference's env surface over libpgx.

Mirrors the reference's interfaces for the hot path:
  * ``register_envs`` / ``make`` -- env ids and kwargs of panda_gym/__init__.py:23-91
    (``PandaReach{,Joints}{,Dense}-v3``, max_episode_steps);
  * ``PandaEnv`` -- one env with the ``RobotTaskEnv`` surface (core.py:255-414):
    ``reset(seed, options)``, ``step(action)`` -> (obs dict, float reward,
    terminated, truncated, info{"is_success","is_truncated"}), ``compute_reward``,
    ``save_state/restore_state/remove_state``, gymnasium TimeLimit truncation;
  * ``PandaVecEnv`` -- N lockstep envs on one GPU with SB3's VecEnv protocol
    (``reset``, ``step_async/step_wait``, ``env_method("compute_reward", ...)``,
    ``get_attr/set_attr``, auto-reset with ``terminal_observation`` and
    ``TimeLimit.truncated`` infos) plus a device-resident ``step_tensors`` path.

State lives in one device allocation owned by libpgx; observations come back
as torch tensors on the env's device.  There is no CPU physics fallback.
"""
from __future__ import annotations

import ctypes as C
import importlib
import math
import os
from dataclasses import replace
from typing import Any, Dict, List, Optional, Sequence, Tuple, Union

import numpy as np

from . import abi, reach_ao
from ._native import PgxError, check, load
from .model import load_model

try:
    import torch
except ImportError:  # pragma: no cover - torch is part of the image
    torch = None


# ------------------------------------------------- gymnasium / SB3 identity
def _optional(name: str):
    try:
        return importlib.import_module(name)
    except ImportError:
        return None


# Where gymnasium / stable-baselines3 are importable, the env classes ARE their classes' subclasses
# and the spaces are gymnasium's (RobotTaskEnv(gym.Env) with spaces.Dict of spaces.Box, core.py:4-7,
# 255, 274-280; SB3's make_vec_env(..., SubprocVecEnv) consumer, setup_training.py:43-47), so SB3's
# isinstance checks (VecEnv wrapping, spaces.Dict for MultiInputPolicy) accept them; elsewhere the
# stand-ins below keep the same surface.
_gym = _optional("gymnasium")
_gym_spaces = _optional("gymnasium.spaces") if _gym is not None else None
_sb3_vec = _optional("stable_baselines3.common.vec_env")
_EnvBase = _gym.Env if _gym is not None else object
_VecEnvBase = _sb3_vec.VecEnv if _sb3_vec is not None else object


# ----------------------------------------------------------------- spaces
class Box:
    """Minimal gymnasium.spaces.Box stand-in (used where gymnasium is not installed)."""

    def __init__(self, low: float, high: float, shape: Tuple[int, ...], dtype=np.float32):
        self.low = np.full(shape, low, dtype=dtype)
        self.high = np.full(shape, high, dtype=dtype)
        self.shape = tuple(shape)
        self.dtype = np.dtype(dtype)
        self._rng = np.random.default_rng()

    def seed(self, seed: Optional[int] = None) -> None:
        self._rng = np.random.default_rng(seed)

    def sample(self) -> np.ndarray:
        return self._rng.uniform(self.low, self.high).astype(self.dtype)

    def contains(self, x) -> bool:
        x = np.asarray(x)
        return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))


class DictSpace(dict):
    """Minimal gymnasium.spaces.Dict stand-in."""

    @property
    def spaces(self) -> Dict[str, Box]:
        return dict(self)


def make_spaces(obs_dim: int, action_dim: int):
    """(observation_space, action_space) of RobotTaskEnv (core.py:274-280): Dict(observation,
    desired_goal, achieved_goal) of Box(-10, 10) and Box(-1, 1) of the action, float32 --
    gymnasium's classes where gymnasium imports, the stand-ins otherwise."""
    if _gym_spaces is not None:
        box = lambda lo, hi, n: _gym_spaces.Box(lo, hi, shape=(n,), dtype=np.float32)  # noqa: E731
        obs = _gym_spaces.Dict(dict(observation=box(-10.0, 10.0, obs_dim), desired_goal=box(-10.0, 10.0, 3),
                                    achieved_goal=box(-10.0, 10.0, 3)))
        return obs, box(-1.0, 1.0, action_dim)
    obs = DictSpace(observation=Box(-10.0, 10.0, (obs_dim,)), desired_goal=Box(-10.0, 10.0, (3,)),
                    achieved_goal=Box(-10.0, 10.0, (3,)))
    return obs, Box(-1.0, 1.0, (action_dim,))


# --------------------------------------------------------------- registry
_REGISTRY: Dict[str, abi.EnvSpec] = {}


def register_envs(max_ep_steps: int = 50) -> None:
    """panda_gym.register_envs (panda_gym/__init__.py:23-91) for the tasks this build runs."""
    for reward in (abi.REWARD_SPARSE, abi.REWARD_DENSE):
        for control in (abi.CONTROL_EE, abi.CONTROL_JOINTS):
            rs = "Dense" if reward == abi.REWARD_DENSE else ""
            cs = "Joints" if control == abi.CONTROL_JOINTS else ""
            _REGISTRY[f"PandaReach{cs}{rs}-v3"] = abi.EnvSpec(task=abi.TASK_REACH, control=control, reward=reward,
                                                             max_episode_steps=max_ep_steps, block_gripper=True)
            # panda_tasks.py:50-58 (Push: block_gripper=True), :37-48 (PickAndPlace: block_gripper=False)
            _REGISTRY[f"PandaPush{cs}{rs}-v3"] = abi.EnvSpec(task=abi.TASK_PUSH, control=control, reward=reward,
                                                            max_episode_steps=max_ep_steps, block_gripper=True)
            _REGISTRY[f"PandaPickAndPlace{cs}{rs}-v3"] = abi.EnvSpec(
                task=abi.TASK_PICK_AND_PLACE, control=control, reward=reward, max_episode_steps=max_ep_steps,
                block_gripper=False)
    # panda_gym/__init__.py:15-20, 51-56; PandaReachAOEnv (panda_tasks.py:132-159) with TrainConfig
    # defaults and scenario "reachao_rand" (the config this build runs)
    _REGISTRY["PandaReachAO-v3"] = abi.EnvSpec.reach_ao(max_episode_steps=max_ep_steps)
    if _gym is not None:   # gym.make("PandaReach-v3") as the reference registers it (__init__.py:23-91)
        for env_id in _REGISTRY:
            if env_id not in getattr(_gym, "registry", {}):
                _gym.register(id=env_id, entry_point="panda_gym_amd.envs:PandaEnv", kwargs={"env_id": env_id},
                              max_episode_steps=max_ep_steps)


def registered_ids() -> List[str]:
    return sorted(_REGISTRY)


def spec(env_id: str) -> abi.EnvSpec:
    if not _REGISTRY:
        register_envs(50)
    if env_id not in _REGISTRY:
        raise KeyError(f"{env_id} is not registered (call register_envs); known: {registered_ids()}")
    return _REGISTRY[env_id]


def seeded_goal(env_spec: abi.EnvSpec, seed: Optional[int]) -> Optional[np.ndarray]:
    """Goal draw of RobotTaskEnv.reset(seed) (core.py:302 reseeds PCG64 every reset; reach.py:75-78)."""
    r = seeded_reset(env_spec, seed)
    return None if r is None else r[0]


_AO_GEOM: Dict[tuple, "reach_ao.RobotGeometry"] = {}


def _ao_geometry(base_pos: tuple, model_name: str = "panda_custom0") -> "reach_ao.RobotGeometry":
    key = (base_pos, model_name)
    if key not in _AO_GEOM:
        _AO_GEOM[key] = reach_ao.RobotGeometry(load_model(model_name), base_pos)
    return _AO_GEOM[key]


def seeded_reset(env_spec: abi.EnvSpec, seed: Optional[int]) -> Optional[Tuple[np.ndarray, Optional[np.ndarray]]]:
    """(goal, object position) of RobotTaskEnv.reset(seed): a fresh PCG64(SeedSequence(seed))
    (core.py:302), then the task's draws in its own order -- Reach reach.py:75-78; Push
    push.py:69-87 (goal noise, object noise, both around the cube centre height);
    PickAndPlace pick_and_place.py:65-85 (goal noise, random() < 0.3 zeroes its z, object)."""
    if seed is None:
        return None
    if env_spec.task == abi.TASK_REACH_AO:   # (goal, obstacle centres [6, 3])
        return reach_ao.seeded_reset(seed, _ao_geometry(tuple(env_spec.base_pos)))
    return task_draws(env_spec, np.random.Generator(np.random.PCG64(np.random.SeedSequence(seed))))


def task_draws(env_spec: abi.EnvSpec, rng: np.random.Generator) -> Tuple[np.ndarray, Optional[np.ndarray]]:
    """(goal, object position) of one Task.reset of Reach / Push / PickAndPlace drawn from ``rng``
    (env.np_random): the order the device reset follows in its PCG64 mode (pgx_set_rng_streams)."""
    lo, hi = env_spec.goal_bounds()
    if env_spec.task == abi.TASK_REACH:
        return rng.uniform(np.array(lo), np.array(hi)), None
    half = abi.OBJECT_SIZE / 2
    goal = np.array([0.0, 0.0, half])
    noise = rng.uniform(np.array(lo), np.array(hi))
    if env_spec.task == abi.TASK_PICK_AND_PLACE and rng.random() < 0.3:
        noise[2] = 0.0
    goal += noise
    obj = np.array([0.0, 0.0, half])
    olo, ohi = env_spec.obj_bounds()
    obj += rng.uniform(np.array(olo), np.array(ohi))
    return goal, obj


def pcg64_record(gen: Union[np.random.Generator, np.random.PCG64]) -> np.ndarray:
    """[abi.PCG64_WORDS] uint64 {state_lo, state_hi, inc_lo, inc_hi, has_uint32, uinteger}: numpy's
    PCG64 bit_generator.state, the record pgx_set_rng_streams takes per env (pgx.h)."""
    bg = gen.bit_generator if isinstance(gen, np.random.Generator) else gen
    st = bg.state
    m = (1 << 64) - 1
    s = st["state"]
    has = int(st["has_uint32"])   # (a spent uinteger, which numpy keeps, is recorded as 0)
    return np.array([s["state"] & m, s["state"] >> 64, s["inc"] & m, s["inc"] >> 64, has,
                     int(st["uinteger"]) if has else 0], dtype=np.uint64)


def pcg64_records(seeds: Sequence[int]) -> np.ndarray:
    """[N, abi.PCG64_WORDS] records of PCG64(SeedSequence(seed)) per seed: gymnasium's
    seeding.np_random(seed) (core.py:302)."""
    out = np.empty((len(seeds), abi.PCG64_WORDS), dtype=np.uint64)
    for i, sd in enumerate(seeds):
        out[i] = pcg64_record(np.random.PCG64(np.random.SeedSequence(int(sd))))
    return out


def pcg64_from_record(rec: np.ndarray) -> np.random.Generator:
    """numpy Generator at a record's stream position (inverse of pcg64_record)."""
    bg = np.random.PCG64()
    st = bg.state
    st["state"] = {"state": int(rec[0]) | (int(rec[1]) << 64), "inc": int(rec[2]) | (int(rec[3]) << 64)}
    st["has_uint32"], st["uinteger"] = int(rec[4]), int(rec[5])
    bg.state = st
    return np.random.Generator(bg)


# ------------------------------------------------------------ vec env
class PandaVecEnv(_VecEnvBase):
    """N independent Panda envs stepped in lockstep by one HIP kernel launch (an SB3 ``VecEnv``
    subclass where stable-baselines3 imports).

    ``lanes_per_env`` picks the kernel layout (results agree to fp32 rounding): 16 gives
    each env a 16-lane DPP row (the solver's coordinates split over the lanes; fastest
    while the batch is too small to fill the chip one lane per env), 1 one env per lane,
    0 (default) chooses: 16 with contacts at every batch size, and up to 8192 envs without).
    ``full_manifold`` (default: on wherever the layout has it, i.e. with contacts in the 16-lane
    layout) keeps Bullet's per-pair manifolds (<= 4 points per colliding pair) up to 8 robot points
    per env in Reach / ReachAO and 12 in Push / PickAndPlace; ``False`` keeps the 4 deepest robot
    points (the one-lane layout's budget; DESIGN.md section 4: budget, rates, cost).

    ``reset_rng``: where the reset draws (goal, object) come from.  ``"philox"`` (default): a
    device counter stream; a seeded ``reset`` injects the reference's numpy draws for that reset
    only.  ``"pcg64"``: every env keeps a numpy PCG64 stream on the device, and a seeded reset
    (env i with seed + i, as SB3 seeds a VecEnv) reseeds it and draws the reference's goal / object
    on the device, bit for bit -- RobotTaskEnv.reset reseeds ``task.np_random`` on every reset
    (core.py:302).  A reset without a seed, the auto-reset included, gets fresh OS entropy in the
    reference, so there is no reference value to match: here it continues the env's stream (a
    reproducible stand-in with the reference's distribution).  ReachAO draws its rejection sampler
    (reach_ao.py:965-1082) from the stream with numpy's uniform / random / integers / shuffle, and
    decides every accept / reject test in fp64 on the host's capsules with the host sampler's
    arithmetic (``reach_ao.reset_draws``), so it takes the same branches and draws; its goal agrees
    to a few ulp (the device's sin / cos / cbrt against the host libm)."""

    metadata = {"render_modes": []}
    render_mode = None

    def __init__(self, env_id: str = "PandaReach-v3", num_envs: int = 4096, device: Any = "cuda:0", seed: int = 0,
                 env_id_offset: int = 0, max_episode_steps: Optional[int] = None, auto_reset: bool = True,
                 n_substeps: int = 20, model_name: str = "panda_custom0", contacts: bool = True,
                 lanes_per_env: int = 0, full_manifold: Optional[bool] = None,
                 sim_params: Optional[Dict[str, Any]] = None, lib_path: Optional[str] = None,
                 reset_rng: str = "philox"):
        """``sim_params``: pgx_sim_params fields to override (the default library runs only the
        compiled parameters and refuses others; ``lib_path`` = libpgx_rtmodel.so reads them from
        the handle)."""
        if torch is None:
            raise PgxError("PandaVecEnv needs torch for device buffers")
        self.lib = load(lib_path)
        self.env_id = env_id
        base_spec = spec(env_id)
        if reset_rng not in ("philox", "pcg64"):
            raise ValueError(f"reset_rng must be 'philox' or 'pcg64', got {reset_rng!r}")
        if max_episode_steps is not None:
            base_spec = replace(base_spec, max_episode_steps=max_episode_steps)
        self.spec = base_spec
        self.num_envs = int(num_envs)
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise PgxError("PandaVecEnv runs on a HIP device only (no CPU physics fallback)")
        self._model = abi.make_model(load_model(model_name), ee_link=11)
        self._params = abi.default_sim_params(n_substeps=n_substeps)
        for k, v in (sim_params or {}).items():
            field = getattr(self._params, k)
            if hasattr(field, "__len__"):
                for i, x in enumerate(v):
                    field[i] = x
            else:
                setattr(self._params, k, v)
        if full_manifold is None:   # the per-pair manifold budget wherever the 16-lane kernels run
            full_manifold = bool(contacts) and lanes_per_env != 1 and os.environ.get("PGX_LANES_PER_ENV") != "1"
        self._cfg = abi.make_config(self.spec, self.num_envs, self._model, self._params, seed=seed,
                                    env_id_offset=env_id_offset, contacts=contacts, lanes_per_env=lanes_per_env,
                                    full_manifold=full_manifold)
        if self.spec.task == abi.TASK_REACH_AO:
            # the reset sampler's EE centre and its capsules at the neutral pose, fp64 (pgx.h
            # ao_ee_neutral, ao_capsules_neutral): the device's accept / reject tests run on these values
            geom = _ao_geometry(tuple(self.spec.base_pos), model_name)
            for i in range(3):
                self._cfg.ao_ee_neutral[i] = float(geom.ee[i])
            for c in range(len(geom.r)):
                for k in range(3):
                    self._cfg.ao_capsules_neutral[c][k] = float(geom.A[c][k])
                    self._cfg.ao_capsules_neutral[c][3 + k] = float(geom.B[c][k])
                self._cfg.ao_capsules_neutral[c][6] = float(geom.r[c])
        # auto_reset=False: a finished env keeps its terminal state until reset (one gymnasium env)
        self._cfg.no_auto_reset = 0 if auto_reset else 1
        self.auto_reset = bool(auto_reset)
        self.obs_dim = self.lib.pgx_obs_dim(C.byref(self._cfg))
        self.action_dim = self.lib.pgx_action_dim(C.byref(self._cfg))
        h = C.c_void_p()
        torch.cuda.set_device(self.device)
        self._check(self.lib.pgx_create(C.byref(self._cfg), self.device.index or 0, C.byref(h)), "pgx_create")
        self._h = h
        self.seed_value = seed
        n, od = self.num_envs, self.obs_dim
        kw = dict(device=self.device)
        # every step output is a view into one device buffer (f32 arrays, then the u8 flags), so
        # the SB3 path brings a step back with a single D2H copy
        f32 = [("obs", (n, od)), ("achieved_goal", (n, 3)), ("desired_goal", (n, 3)), ("reward", (n,)),
               ("terminal_obs", (n, od)), ("terminal_ag", (n, 3)), ("terminal_dg", (n, 3))]
        # Task.is_truncated (task_trunc, ReachAO is_collided): written by the kernel; zero for the others
        u8 = ["success", "terminated", "truncated", "task_trunc"]
        nf = sum(int(np.prod(shape)) for _, shape in f32)
        self._outbuf = torch.zeros(4 * nf + len(u8) * n, dtype=torch.uint8, **kw)
        self._out_f32 = self._outbuf[:4 * nf].view(torch.float32)
        self._out_u8 = self._outbuf[4 * nf:].view(len(u8), n)
        o = 0
        for name, shape in f32:
            k = int(np.prod(shape))
            setattr(self, name, self._out_f32[o:o + k].view(shape))
            o += k
        for i, name in enumerate(u8):
            setattr(self, name, self._out_u8[i])
        self._actions = torch.zeros((n, self.action_dim), dtype=torch.float32, **kw)
        self._out = abi.PgxStepOut(self.obs.data_ptr(), self.achieved_goal.data_ptr(), self.desired_goal.data_ptr(),
                                   self.reward.data_ptr(), self.success.data_ptr(), self.terminated.data_ptr(),
                                   self.truncated.data_ptr(), self.terminal_obs.data_ptr(), self.terminal_ag.data_ptr(),
                                   self.terminal_dg.data_ptr(),
                                   self.task_trunc.data_ptr() if self.spec.task == abi.TASK_REACH_AO else None)
        self.observation_space, self.action_space = make_spaces(od, self.action_dim)
        self.distance_threshold = self.spec.distance_threshold
        if self.spec.task == abi.TASK_REACH_AO:
            self.reward_type = "sparse_ao"   # ReachAO.compute_reward sparse/reach (reach_ao.py:1317-1320)
        else:
            self.reward_type = "dense" if self.spec.reward == abi.REWARD_DENSE else "sparse"
        self._pending: Optional[torch.Tensor] = None
        self._pending_seed: Optional[int] = None
        self._step_index = 0
        self.reset_rng = reset_rng
        if reset_rng == "pcg64":
            try:
                self._set_rng_streams(pcg64_records([seed + i for i in range(n)]))
            except Exception:
                self.close()
                raise
        if _VecEnvBase is not object:   # SB3's VecEnv bookkeeping (reset_infos, seeds, render_mode)
            _VecEnvBase.__init__(self, n, self.observation_space, self.action_space)

    # ---------------------------------------------------------------- core
    def _check(self, rc: int, what: str) -> None:
        check(rc, what, self.lib)

    def _stream(self):
        return C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def close(self) -> None:
        if getattr(self, "_h", None):
            torch.cuda.synchronize(self.device)
            self.lib.pgx_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def state(self) -> Dict[str, torch.Tensor]:
        """Device views of the SoA state (q, qd [7,N] f32; qc [7,N] f32 the pose getLinkState reports;
        goal [3,N] f64; object [13,N] f32 =
        pos, quat (x,y,z,w), linvel, angvel; contacts [2 * abi.CONTACT_SLOTS, N] f32 warm-start cache
        (feature id, normal impulse): object-scene slots, then robot slots; elapsed, episode [N])."""
        v = abi.PgxStateView()
        self._check(self.lib.pgx_get_state(self._h, C.byref(v)), "pgx_get_state")
        n = self.num_envs
        return {
            "q": _view(v.q, (7, n), torch.float32, self.device),
            "qd": _view(v.qd, (7, n), torch.float32, self.device),
            "qc": _view(v.qc, (7, n), torch.float32, self.device),
            "goal": _view(v.goal, (3, n), torch.float64, self.device),
            "object": _view(v.object, (13, n), torch.float32, self.device),
            "contacts": _view(v.contacts, (2 * abi.CONTACT_SLOTS, n), torch.float32, self.device),
            **({"obstacles": _view(v.obstacles, (4 * abi.AO_OBSTACLES, n), torch.float32, self.device)}
               if v.obstacles else {}),
            "elapsed": _view(v.elapsed, (n,), torch.int32, self.device),
            "episode": _view(v.episode, (n,), torch.int32, self.device),
            "errors": _view(v.errors, (1,), torch.int32, self.device),
            # Bullet's persistent manifolds (pgx.h PGX_MANIFOLD_POOL): count, then per point kid, local A,
            # local B, normal, distance, impulse
            **({"manifolds": _view(v.manifolds, (1 + v.manifold_pool * abi.MANIFOLD_POINT, n), torch.float32,
                                   self.device)} if v.manifolds else {}),
            # not state: the env order of the last sorted step launch (heavy-first)
            **({"env_order": _view(v.env_order, (n,), torch.int32, self.device)} if v.env_order else {}),
        }

    def robot_contact_budget(self) -> int:
        """Robot contact points this handle's kernels keep per env (the deepest of Bullet's <= 4 per
        colliding pair; abi.ROBOT_POINTS / ROBOT_POINTS_ARM / ROBOT_POINTS_ONE_LANE; 0 without contacts)."""
        v = abi.PgxStateView()
        self._check(self.lib.pgx_get_state(self._h, C.byref(v)), "pgx_get_state")
        return int(v.robot_points)

    def raise_device_errors(self, errors: Optional[int] = None) -> None:
        """Raise what the kernels flagged (pgx_state_view.errors) and clear it.  The device path
        (step_tensors / reset_tensors) never synchronises to look; the SB3 path (reset,
        step_wait) looks at every call.  PGX_ERR_AO_OBSTACLE: ReachAO.set_coll_free_obs raises
        StopIteration after 10000 rejected obstacle draws (reach_ao.py:1143-1145)."""
        err = self.state()["errors"]
        if errors is None:
            errors = int(err.item())
        if errors:
            err.zero_()
            if errors & abi.ERR_AO_OBSTACLE:
                raise PgxError("Couldn't find collision free obstacle! (device reset of a ReachAO env gave up "
                               "after 10000 obstacle draws; reach_ao.py:1143-1145 raises StopIteration)")
            raise PgxError(f"device error flags 0x{errors:x}")

    def _obs_dict(self) -> Dict[str, torch.Tensor]:
        return {"observation": self.obs, "achieved_goal": self.achieved_goal, "desired_goal": self.desired_goal}

    def _set_rng_streams(self, records: np.ndarray) -> None:
        rec = torch.as_tensor(np.ascontiguousarray(records, dtype=np.uint64).view(np.int64), device=self.device)
        self._check(self.lib.pgx_set_rng_streams(self._h, C.c_void_p(rec.data_ptr()), self._stream()),
                    "pgx_set_rng_streams")
        self._rng_keep = rec   # read by the queued copy

    def rng_streams(self) -> np.ndarray:
        """[N, abi.PCG64_WORDS] uint64 PCG64 records of the envs' reset streams (``reset_rng="pcg64"``):
        where each env's np_random stands (pcg64_from_record rebuilds the numpy Generator)."""
        out = torch.empty((self.num_envs, abi.PCG64_WORDS), dtype=torch.int64, device=self.device)
        self._check(self.lib.pgx_get_rng_streams(self._h, C.c_void_p(out.data_ptr()), self._stream()),
                    "pgx_get_rng_streams")
        return out.cpu().numpy().view(np.uint64)

    def reset_tensors(self, seed: Optional[int] = None, mask: Optional[torch.Tensor] = None,
                      goals: Optional[np.ndarray] = None, objects: Optional[np.ndarray] = None,
                      episode_phase: Optional[str] = None) -> Dict[str, torch.Tensor]:
        """Reset (masked) envs on device; ``seed`` reproduces the reference's PCG64 goal (and
        object) draws for env i with seed+i (SB3 VecEnv seeding): injected into the kernel, or
        with ``reset_rng="pcg64"`` the envs' device streams are reseeded and drawn from.

        ``episode_phase="staggered"`` (benchmarks only): global env g starts its TimeLimit counter
        at g mod max_episode_steps instead of 0, so its first episode is shorter and from then on
        every step auto-resets about N / max_episode_steps envs -- the steady state of a long
        VecEnv rollout (auto-reset and TimeLimit: core.py:352-368, __init__.py:30-35) in any window
        of steps, instead of all envs resetting on the same step."""
        if episode_phase not in (None, "staggered"):
            raise ValueError(f"episode_phase must be None or 'staggered', got {episode_phase!r}")
        inj, inj_obj = None, None
        if goals is None and objects is None and seed is not None and self.reset_rng == "pcg64":
            rec = pcg64_records([seed + i for i in range(self.num_envs)])
            if mask is not None:   # only the masked envs are reseeded
                keep = ~mask.detach().to("cpu", torch.bool).numpy()
                rec[keep] = self.rng_streams()[keep]
            self._set_rng_streams(rec)
        elif goals is None and objects is None and seed is not None:
            draws = [seeded_reset(self.spec, seed + i) for i in range(self.num_envs)]
            goals = np.stack([d[0] for d in draws])
            if self.spec.task != abi.TASK_REACH:
                objects = np.stack([d[1] for d in draws])
        if goals is not None:
            inj = torch.as_tensor(np.asarray(goals, dtype=np.float64).reshape(self.num_envs, 3), device=self.device)
        if objects is not None:   # object position [N,3] or ReachAO obstacle centres [N,6,3]
            w = 3 * abi.AO_OBSTACLES if self.spec.task == abi.TASK_REACH_AO else 3
            inj_obj = torch.as_tensor(np.asarray(objects, dtype=np.float64).reshape(self.num_envs, w),
                                      device=self.device)
        m = None
        if mask is not None:
            m = mask.to(device=self.device, dtype=torch.uint8).contiguous()
        self._check(self.lib.pgx_reset(self._h, None if m is None else C.c_void_p(m.data_ptr()),
                                 None if inj is None else C.c_void_p(inj.data_ptr()),
                                 None if inj_obj is None else C.c_void_p(inj_obj.data_ptr()), C.byref(self._out),
                                 self._stream()), "pgx_reset")
        self._keep = (m, inj, inj_obj)  # keep the buffers alive until the stream consumes them
        if episode_phase == "staggered":   # stream-ordered after the reset (torch's current stream)
            T = int(self.spec.max_episode_steps)
            g = torch.arange(self.num_envs, device=self.device, dtype=torch.int64) + int(self._cfg.env_id_offset)
            el = self.state()["elapsed"]
            phase = (g % T).to(torch.int32)
            el.copy_(phase if m is None else torch.where(m.bool(), phase, el))
        return self._obs_dict()

    def step_kernel(self) -> Optional[str]:
        """Name of the step kernel the last step launched (pgx_step_kernel; rocprof's spelling)."""
        name = self.lib.pgx_step_kernel(self._h)
        return None if name is None else name.decode()

    def step_tensors(self, actions: torch.Tensor):
        """Device-resident step: actions [N,A] f32 on device -> (obs dict, reward, terminated, truncated, success).

        Returned tensors are the env's persistent buffers (overwritten by the next step)."""
        a = actions
        if a.dtype != torch.float32 or a.device != self.device or not a.is_contiguous():
            a = a.to(device=self.device, dtype=torch.float32).contiguous()
        if tuple(a.shape) != (self.num_envs, self.action_dim):
            raise ValueError(f"actions must be [{self.num_envs}, {self.action_dim}], got {tuple(a.shape)}")
        self._check(self.lib.pgx_step(self._h, C.c_void_p(a.data_ptr()), C.byref(self._out), self._stream()), "pgx_step")
        self._step_index += 1
        return self._obs_dict(), self.reward, self.terminated, self.truncated, self.success

    def sample_actions(self, step: Optional[int] = None) -> torch.Tensor:
        """Random policy U[-1,1) from the device Philox stream (benchmark workload)."""
        s = self._step_index if step is None else step
        self._check(self.lib.pgx_sample_actions(self._h, C.c_void_p(self._actions.data_ptr()), C.c_uint64(s),
                                          self._stream()), "pgx_sample_actions")
        return self._actions

    def capture_steps(self, k: int, actions: Optional[torch.Tensor] = None):
        """Capture ``k`` lockstep env steps into one HIP graph (torch.cuda.CUDAGraph); ``replay()``
        runs them with no host launch in between (graph capture of the step loop).
        ``actions``: a static [k, N, A] f32 device buffer step i reads (refill it between replays),
        or None: the device Philox random policy, drawn inside the graph with the step counters of
        capture time (every replay repeats those draws; the env state moves on).  The step's outputs
        land in the env's usual buffers (obs, reward, ... of the last captured step).  Capture runs
        nothing: the state changes only on replay."""
        if actions is not None:
            if tuple(actions.shape) != (k, self.num_envs, self.action_dim) or actions.dtype != torch.float32 \
                    or actions.device != self.device or not actions.is_contiguous():
                raise ValueError(f"actions must be a contiguous f32 [{k}, {self.num_envs}, {self.action_dim}] "
                                 f"tensor on {self.device}")
        torch.cuda.synchronize(self.device)
        g = torch.cuda.CUDAGraph()
        base = self._step_index
        with torch.cuda.graph(g):
            for i in range(k):
                a = actions[i] if actions is not None else self.sample_actions(base + i)
                self._check(self.lib.pgx_step(self._h, C.c_void_p(a.data_ptr()), C.byref(self._out), self._stream()),
                            "pgx_step (capture)")
        g._pgx_keep = actions   # the graph reads the buffer at replay
        return g

    # ------------------------------------------------------- SB3 VecEnv API
    def reset(self, seed: Optional[int] = None, options: Optional[dict] = None):
        """SB3 VecEnv.reset: a seed given to ``seed()`` beforehand applies to this reset only."""
        if seed is None:
            seed = self._pending_seed
        self._pending_seed = None
        self.reset_tensors(seed=seed)
        self.raise_device_errors()
        return self._numpy_obs()

    def seed(self, seed: Optional[int] = None) -> List[Optional[int]]:
        """SB3 VecEnv.seed: env i is seeded with seed + i at the next reset()."""
        self._pending_seed = seed
        return [None if seed is None else seed + i for i in range(self.num_envs)]

    def _host_stage(self):
        """Pinned host mirrors of the step outputs (allocated on first use): the SB3 path
        copies every output with one async DMA each on the env's stream and waits once,
        instead of a blocking pageable copy (and a stream sync) per tensor."""
        if getattr(self, "_hs", None) is None:
            n, od, ad = self.num_envs, self.obs_dim, self.action_dim
            pin = dict(dtype=torch.float32, pin_memory=True)
            self._hs = {
                "act": torch.empty((n, ad), **pin), "act_dev": torch.empty((n, ad), dtype=torch.float32,
                                                                           device=self.device),
                "packed": torch.empty(self._outbuf.numel(), dtype=torch.uint8, pin_memory=True),
                "errors": torch.zeros(1, dtype=torch.int32, pin_memory=True),
                "errors_dev": self.state()["errors"],   # a view of the library's word (stable)
            }
            nf = self._out_f32.numel()
            hf = self._hs["packed"][:4 * nf].view(torch.float32)
            o = 0
            for name, shape in (("observation", (n, od)), ("achieved_goal", (n, 3)), ("desired_goal", (n, 3)),
                                ("reward", (n,)), ("t_observation", (n, od)), ("t_achieved_goal", (n, 3)),
                                ("t_desired_goal", (n, 3))):
                k = int(np.prod(shape))
                self._hs[name] = hf[o:o + k].view(shape)
                o += k
            self._hs["flags"] = self._hs["packed"][4 * nf:].view(4, n)   # success, terminated, truncated, task
        return self._hs

    def step_async(self, actions) -> None:
        if torch.is_tensor(actions) and actions.device == self.device:
            self._pending = actions
            return
        hs = self._host_stage()
        a = np.asarray(actions.cpu() if torch.is_tensor(actions) else actions, dtype=np.float32)
        if a.shape != (self.num_envs, self.action_dim):
            raise ValueError(f"actions must be [{self.num_envs}, {self.action_dim}], got {a.shape}")
        # the previous step's H2D copy has completed: step_wait synchronised the stream
        hs["act"].numpy()[...] = a
        hs["act_dev"].copy_(hs["act"], non_blocking=True)
        self._pending = hs["act_dev"]

    def step_wait(self):
        """SB3 VecEnv.step_wait: (obs dict, rewards, dones, infos) as numpy, with auto-reset
        ``terminal_observation`` / ``TimeLimit.truncated`` infos (SB3 DummyVecEnv semantics).
        Host-facing path: PCIe-inclusive (bench.py ``sb3_host_path`` times it)."""
        obs, rew, term, trunc, succ = self.step_tensors(self._pending)
        self._pending = None
        hs = self._host_stage()
        stream = torch.cuda.current_stream(self.device)
        hs["packed"].copy_(self._outbuf, non_blocking=True)   # every output, one DMA
        hs["errors"].copy_(hs["errors_dev"], non_blocking=True)
        # SB3's per-env infos list is built while the step kernel runs: a fresh dict per env copied
        # in C from the common template, the few envs whose flags differ patched after the sync
        infos: List[Dict[str, Any]] = list(map(dict.copy, [_INFO_TEMPLATES[0]] * self.num_envs))
        stream.synchronize()
        if hs["errors"].item():
            self.raise_device_errors(int(hs["errors"].item()))
        # copies: the pinned mirrors are overwritten by the next step
        o = {k: hs[k].numpy().copy() for k in ("observation", "achieved_goal", "desired_goal")}
        r = hs["reward"].numpy().copy()
        fl = hs["flags"].numpy() != 0
        sc, te, tr, col = fl[0], fl[1].copy(), fl[2].copy(), fl[3]
        d = te | tr
        code = sc.view(np.uint8) + 2 * col.view(np.uint8)
        for i in np.flatnonzero(code).tolist():
            infos[i] = _INFO_TEMPLATES[int(code[i])].copy()
        idx = np.nonzero(d)[0]
        if len(idx):
            tobs, tag, tdg = hs["t_observation"].numpy(), hs["t_achieved_goal"].numpy(), hs["t_desired_goal"].numpy()
            for i in idx.tolist():
                infos[i]["terminal_observation"] = {"observation": tobs[i].copy(), "achieved_goal": tag[i].copy(),
                                                    "desired_goal": tdg[i].copy()}
                infos[i]["TimeLimit.truncated"] = bool(tr[i] and not te[i])
        return o, r, d, infos

    def step(self, actions):
        self.step_async(actions)
        return self.step_wait()

    def task_truncated(self) -> np.ndarray:
        """Task.is_truncated of the last step per env: False for Reach / Push / PickAndPlace
        (reach.py:53-54); ReachAO's is_collided (reach_ao.py:1263-1264), the kernel's own
        collision flag (pgx_step_out.task_truncated), whatever collision_reward is."""
        return self.task_trunc.cpu().numpy() != 0

    def _numpy_obs(self) -> Dict[str, np.ndarray]:
        return {k: v.cpu().numpy().copy() for k, v in self._obs_dict().items()}

    def compute_reward(self, achieved_goal, desired_goal, info=None):
        """Task.compute_reward over a batch (HER relabel path), on device.

        Float32 inputs follow the reference's float32 numpy arithmetic bit for bit."""
        is_np = not torch.is_tensor(achieved_goal)
        ag = torch.as_tensor(np.asarray(achieved_goal, dtype=np.float32) if is_np else achieved_goal)
        dg = torch.as_tensor(np.asarray(desired_goal, dtype=np.float32) if is_np else desired_goal)
        shape = ag.shape[:-1]
        ag = ag.to(self.device, torch.float32).reshape(-1, 3).contiguous()
        dg = dg.to(self.device, torch.float32).reshape(-1, 3).contiguous()
        out = torch.empty(ag.shape[0], dtype=torch.float32, device=self.device)
        rt = abi.REWARD_CODES[self.reward_type]
        self._check(self.lib.pgx_compute_reward(C.c_void_p(ag.data_ptr()), C.c_void_p(dg.data_ptr()),
                                          C.c_int64(ag.shape[0]), rt, C.c_double(self.distance_threshold),
                                          C.c_void_p(out.data_ptr()), self._stream()), "pgx_compute_reward")
        out = out.reshape(shape)
        return out.cpu().numpy() if is_np else out

    def env_method(self, method_name: str, *args, indices=None, **kwargs):
        if method_name == "compute_reward":
            return [self.compute_reward(*args, **kwargs)]
        return [getattr(self, method_name)(*args, **kwargs)]

    def env_is_wrapped(self, wrapper_class, indices=None) -> List[bool]:
        """SB3 VecEnv.env_is_wrapped: the envs are kernel lanes, wrapped in nothing."""
        n = self.num_envs if indices is None else len(list(indices))
        return [False] * n

    def get_attr(self, attr_name: str, indices=None):
        val = getattr(self, attr_name)
        n = self.num_envs if indices is None else len(list(indices))
        return [val] * n

    def set_attr(self, attr_name: str, value, indices=None) -> None:
        setattr(self, attr_name, value)

    # ----------------------------------------------------- save / restore
    def save_state(self) -> int:
        """Device snapshot of the whole SoA state (RobotTaskEnv.save_state, core.py:310-321 ->
        PyBullet.save_state, pybullet.py:79-86): the id is libpgx's, the first non-negative
        integer not in use."""
        sid = C.c_int32()
        self._check(self.lib.pgx_snapshot(self._h, C.byref(sid), self._stream()), "pgx_snapshot")
        return int(sid.value)

    def restore_state(self, state_id: int) -> None:
        """Restore a snapshot; an id that was removed (or never saved) raises PgxError, as
        pybullet.error in the reference (test/save_and_restore_test.py:30-36)."""
        self._check(self.lib.pgx_restore(self._h, int(state_id), self._stream()), "pgx_restore")

    def remove_state(self, state_id: int) -> None:
        """Free a snapshot; its id becomes available again (PyBullet.remove_state, pybullet.py:96-102)."""
        self._check(self.lib.pgx_release(self._h, int(state_id)), "pgx_release")


_INFO_TEMPLATES = [{"is_success": s, "is_truncated": c} for c in (False, True) for s in (False, True)]


def _view(addr: int, shape, dtype, device):
    """Wrap a libpgx-owned device buffer as a torch tensor (no copy)."""
    typestr = {torch.float32: "<f4", torch.float64: "<f8", torch.int32: "<i4"}[dtype]

    class _Iface:  # torch has no public from-pointer constructor; use __cuda_array_interface__
        __cuda_array_interface__ = {"shape": tuple(shape), "typestr": typestr, "data": (int(addr), False),
                                    "version": 2, "strides": None}

    return torch.as_tensor(_Iface(), device=device)


# --------------------------------------------------------- single env
class _RobotView:
    """Read-only `env.robot` (Panda, panda.py:264-312): the state the kernels keep for the one env.
    Control goes through `env.step` (set_action and the motors run inside the step kernel)."""

    def __init__(self, env: "PandaEnv"):
        self._env = env

    def _obs(self) -> np.ndarray:
        return self._env._vec.obs[0].cpu().numpy().copy()

    @property
    def neutral_joint_values(self) -> np.ndarray:   # panda.py:67
        return np.array(abi.NEUTRAL_Q, dtype=np.float64)

    @property
    def block_gripper(self) -> bool:
        return bool(self._env._vec.spec.block_gripper)

    def get_obs(self) -> np.ndarray:
        """Panda.get_obs (panda.py:264-288): EE position, EE velocity (+ fingers width; ReachAO:
        + q, qd, the "js" observation)."""
        o = self._obs()
        n = 20 if self._env._vec.spec.task == abi.TASK_REACH_AO else 6 + (0 if self.block_gripper else 1)
        return o[:n]

    def get_ee_position(self) -> np.ndarray:   # panda.py:306-308 (getLinkState's cached pose)
        return self._obs()[0:3]

    def get_ee_velocity(self) -> np.ndarray:   # panda.py:310-312
        return self._obs()[3:6]

    def get_joint_angle(self, joint: int) -> float:   # core.py:151-160 (fixed finger joints: 0)
        st = self._env._vec.state()
        return float(st["q"][joint, 0].item()) if joint < st["q"].shape[0] else 0.0

    def get_joint_velocity(self, joint: int) -> float:
        st = self._env._vec.state()
        return float(st["qd"][joint, 0].item()) if joint < st["qd"].shape[0] else 0.0

    def get_fingers_width(self) -> float:   # panda.py:300-304: custom_0's finger joints are fixed
        return 0.0


class _TaskView:
    """Read-only `env.task` (Reach / Push / PickAndPlace / ReachAO): goal, achieved goal, the task
    observation, obstacles, and the task's is_success / compute_reward."""

    def __init__(self, env: "PandaEnv"):
        self._env = env

    @property
    def goal(self) -> np.ndarray:   # Task.goal: fp64, as the reference keeps it
        return self._env._vec.state()["goal"][:, 0].cpu().numpy().astype(np.float64)

    def get_goal(self) -> np.ndarray:   # core.py:236-241
        return self.goal.copy()

    def get_achieved_goal(self) -> np.ndarray:
        return self._env._vec.achieved_goal[0].cpu().numpy().copy()

    def get_obs(self) -> np.ndarray:
        o = self._env._vec.obs[0].cpu().numpy().copy()
        return o[len(self._env.robot.get_obs()):]

    @property
    def distance_threshold(self) -> float:
        return float(self._env._vec.spec.distance_threshold)

    @property
    def reward_type(self) -> str:
        return self._env._vec.reward_type

    @property
    def obstacles(self) -> Optional[np.ndarray]:
        """ReachAO: the obstacle centres [6, 3] (inactive ones parked at (99.9, 99.9, -99.9))."""
        st = self._env._vec.state()
        if "obstacles" not in st:
            return None
        return st["obstacles"][:18, 0].cpu().numpy().reshape(6, 3).astype(np.float64)

    def is_success(self, achieved_goal, desired_goal, info=None) -> np.ndarray:
        """utils.distance < distance_threshold (reach.py:80-82)."""
        a, b = np.asarray(achieved_goal), np.asarray(desired_goal)   # (numpy's promotion, as utils.py:4-16)
        d = np.round(np.linalg.norm(a - b, axis=-1), 6)
        return np.array(d < self.distance_threshold, dtype=bool)

    def compute_reward(self, achieved_goal, desired_goal, info=None):
        return self._env.compute_reward(achieved_goal, desired_goal, info)


class _SimView:
    """Read-only `env.sim` (the PyBullet facade, pybullet.py:15-102): timing and the state ids."""

    def __init__(self, env: "PandaEnv"):
        self._env = env

    @property
    def timestep(self) -> float:   # pybullet.py:50
        return float(self._env._vec._params.dt)

    @property
    def n_substeps(self) -> int:
        return int(self._env._vec._params.n_substeps)

    @property
    def dt(self) -> float:   # pybullet.py:63-66
        return self.timestep * self.n_substeps

    def save_state(self) -> int:
        return self._env.save_state()

    def restore_state(self, state_id: int) -> None:
        self._env.restore_state(state_id)

    def remove_state(self, state_id: int) -> None:
        self._env.remove_state(state_id)


class PandaEnv(_EnvBase):
    """One env with the RobotTaskEnv + TimeLimit surface (gym.make("PandaReach-v3") in the reference;
    a ``gymnasium.Env`` subclass where gymnasium imports)."""

    metadata = {"render_modes": []}
    render_mode = None

    def __init__(self, env_id: str = "PandaReach-v3", device: Any = "cuda:0", max_episode_steps: Optional[int] = None,
                 seed: int = 0, reset_rng: str = "philox"):
        """``reset_rng="pcg64"``: reset(seed) reseeds the env's device PCG64 stream and draws the
        reference's goal / object for that seed (core.py:302); a later reset() without a seed
        continues the stream -- a reproducible stand-in for the fresh OS entropy the reference
        draws there, not a reference value (PandaVecEnv)."""
        self._vec = PandaVecEnv(env_id, num_envs=1, device=device, seed=seed, auto_reset=False,
                                max_episode_steps=max_episode_steps, reset_rng=reset_rng)
        # (gymnasium.make replaces env.spec with its registry EnvSpec: the env reads self._vec.spec)
        self.spec = self._vec.spec
        self.observation_space = self._vec.observation_space
        self.action_space = self._vec.action_space
        # RobotTaskEnv's attributes callers read (evaluation/evaluate.py:242-247): read-only views
        self.robot, self.task, self.sim = _RobotView(self), _TaskView(self), _SimView(self)

    def reset(self, seed: Optional[int] = None, options: Optional[dict] = None):
        r = None if self._vec.reset_rng == "pcg64" else seeded_reset(self._vec.spec, seed)
        if self._vec.reset_rng == "pcg64":   # reseed the device stream (seed given) or continue it
            self._vec.reset_tensors(seed=seed)
        elif r is None:
            self._vec.reset_tensors()
        else:
            self._vec.reset_tensors(goals=r[0][None, :], objects=None if r[1] is None else r[1][None, :])
        self._vec.raise_device_errors()
        obs = self._vec._numpy_obs()
        obs = {k: v[0] for k, v in obs.items()}
        return obs, {"is_success": bool(self._vec.success[0].item())}

    def step(self, action):
        a = torch.as_tensor(np.asarray(action, dtype=np.float32).reshape(1, -1), device=self._vec.device)
        obs, rew, term, trunc, succ = self._vec.step_tensors(a)
        o = {k: v[0].cpu().numpy().copy() for k, v in obs.items()}
        r = float(rew[0].item())
        # the kernel's truncated flag = Task.is_truncated (ReachAO collision) or the TimeLimit
        # (gymnasium TimeLimit.step ORs them); info carries the task's own flag (core.py:363-365)
        info = {"is_success": bool(succ[0].item()), "is_truncated": bool(self._vec.task_truncated()[0])}
        return o, r, bool(term[0].item()), bool(trunc[0].item()), info

    def compute_reward(self, achieved_goal, desired_goal, info=None):
        return self._vec.compute_reward(achieved_goal, desired_goal, info)

    def save_state(self) -> int:
        """Snapshot of the env's device state, TimeLimit counter included."""
        return self._vec.save_state()

    def restore_state(self, state_id: int) -> None:
        self._vec.restore_state(state_id)

    def remove_state(self, state_id: int) -> None:
        self._vec.remove_state(state_id)

    def close(self) -> None:
        self._vec.close()


def make(env_id: str, **kwargs) -> PandaEnv:
    """gym.make equivalent for the registered ids (single env with TimeLimit)."""
    spec(env_id)
    return PandaEnv(env_id, **kwargs)
