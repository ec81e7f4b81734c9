"""Device HER replay buffer: the goal-relabelling buffer the reference trains with, on MI355X.

Mirrors stable-baselines3's ``HerReplayBuffer`` as the reference configures it
(training/utils/setup_training.py:14,176-179; classes/train_config.py:2,15:
``replay_buffer_class=HerReplayBuffer``, ``n_sampled_goal=4``,
``goal_selection_strategy="future"``) with the same public surface --
``add(obs, next_obs, action, reward, done, infos)``, ``sample(batch_size)``
returning ``DictReplayBufferSamples``-shaped tensors (real rows first, then the
relabelled ones), ``size()``, ``full``, ``pos``, ``ep_start``/``ep_length``
views -- plus a device-resident path (``add_tensors``, ``add_from_vec_env``)
that never leaves HBM.  Storage, episode bookkeeping, relabelling and reward
recomputation run in libpgx.so (pgx_her.hip); there is no CPU fallback.

Draws: the device Philox stream (key = buffer seed, counter = (sample, call))
replaces numpy's global RNG, so a sample is a pure function of (seed, call
index, buffer contents) -- the oracle (oracle/her.py) reproduces it exactly.
"""
from __future__ import annotations

import ctypes as C
from typing import Any, Dict, List, NamedTuple, Optional, Sequence, Union

import numpy as np

from . import abi
from ._native import PgxError, check, load

try:
    import torch
except ImportError:  # pragma: no cover
    torch = None

STRATEGIES = {"future": abi.HER_FUTURE, "final": abi.HER_FINAL, "episode": abi.HER_EPISODE}


class DictReplayBufferSamples(NamedTuple):
    """stable_baselines3.common.type_aliases.DictReplayBufferSamples (torch tensors on device)."""

    observations: Dict[str, "torch.Tensor"]
    actions: "torch.Tensor"
    next_observations: Dict[str, "torch.Tensor"]
    dones: "torch.Tensor"
    rewards: "torch.Tensor"


class HerReplayBuffer:
    """SB3 HerReplayBuffer over a device ring of ``buffer_size // n_envs`` slots x ``n_envs``.

    ``env`` may be a ``PandaVecEnv`` (reward type, threshold and dims are read
    from it, as SB3 reads them through ``env.env_method("compute_reward")``).
    """

    def __init__(self, buffer_size: int, observation_space: Any = None, action_space: Any = None, env: Any = None,
                 device: Any = "cuda:0", n_envs: int = 1, n_sampled_goal: int = 4,
                 goal_selection_strategy: str = "future", copy_info_dict: bool = False,
                 handle_timeout_termination: bool = True, seed: int = 0, obs_dim: Optional[int] = None,
                 action_dim: Optional[int] = None, reward_type: Optional[str] = None,
                 distance_threshold: Optional[float] = None):
        if torch is None:
            raise PgxError("HerReplayBuffer needs torch for device buffers")
        if goal_selection_strategy not in STRATEGIES:
            raise ValueError(f"Invalid goal selection strategy, please use one of {list(STRATEGIES)}")
        if copy_info_dict:
            raise NotImplementedError("copy_info_dict: infos are not needed by Task.compute_reward")
        self.lib = load()
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise PgxError("HerReplayBuffer lives on a HIP device only (no CPU fallback)")
        if env is not None:
            n_envs = env.num_envs
            obs_dim = env.obs_dim if obs_dim is None else obs_dim
            action_dim = env.action_dim if action_dim is None else action_dim
            reward_type = env.reward_type if reward_type is None else reward_type
            distance_threshold = env.distance_threshold if distance_threshold is None else distance_threshold
        if observation_space is not None and obs_dim is None:
            obs_dim = int(np.prod(observation_space["observation"].shape))
        if action_space is not None and action_dim is None:
            action_dim = int(np.prod(action_space.shape))
        if obs_dim is None or action_dim is None:
            raise ValueError("obs_dim/action_dim: pass env, the spaces, or the dims")
        self.n_envs = int(n_envs)
        self.buffer_size = max(int(buffer_size) // self.n_envs, 1)   # SB3 BaseBuffer: per-env slots
        self.obs_dim, self.action_dim = int(obs_dim), int(action_dim)
        self.reward_type = reward_type or "sparse"
        self.distance_threshold = 0.05 if distance_threshold is None else float(distance_threshold)
        self.n_sampled_goal = n_sampled_goal
        self.her_ratio = 1 - (1.0 / (n_sampled_goal + 1))            # SB3 HerReplayBuffer.__init__
        self.goal_selection_strategy = goal_selection_strategy
        self.handle_timeout_termination = handle_timeout_termination
        self.env = env
        cfg = abi.PgxReplayConfig()
        cfg.n_envs, cfg.capacity = self.n_envs, self.buffer_size
        cfg.obs_dim, cfg.action_dim = self.obs_dim, self.action_dim
        cfg.reward_type = abi.REWARD_CODES[self.reward_type]
        cfg.strategy = STRATEGIES[goal_selection_strategy]
        cfg.distance_threshold, cfg.her_ratio, cfg.seed = self.distance_threshold, self.her_ratio, int(seed)
        self._cfg = cfg
        self._fields, self.row_dim = abi.replay_row_fields(self.obs_dim, self.action_dim)
        self.row_stride = self.lib.pgx_replay_row_stride(C.byref(cfg))
        if self.lib.pgx_replay_row_dim(C.byref(cfg)) != self.row_dim:
            raise PgxError("libpgx batch row layout differs from abi.replay_row_fields")
        h = C.c_void_p()
        torch.cuda.set_device(self.device)
        check(self.lib.pgx_replay_create(C.byref(cfg), self.device.index or 0, C.byref(h)), "pgx_replay_create")
        self._h = h
        self._draw = 0
        self._seen_valid = False
        self._keep: List[Any] = []

    # ------------------------------------------------------------ plumbing
    def _stream(self):
        return C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def close(self) -> None:
        if getattr(self, "_h", None):
            torch.cuda.synchronize(self.device)
            self.lib.pgx_replay_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def _dev(self, x, shape, dtype) -> "torch.Tensor":
        t = x if torch.is_tensor(x) else torch.as_tensor(np.asarray(x))
        t = t.to(device=self.device, dtype=dtype).reshape(shape).contiguous()
        return t

    def _arrays(self):
        s, l, nv = C.c_void_p(), C.c_void_p(), C.c_void_p()
        check(self.lib.pgx_replay_episode_arrays(self._h, C.byref(s), C.byref(l), C.byref(nv)),
              "pgx_replay_episode_arrays")
        from .envs import _view
        shp = (self.buffer_size, self.n_envs)
        return _view(s.value, shp, torch.int32, self.device), _view(l.value, shp, torch.int32, self.device), \
            _view(nv.value, (1,), torch.int32, self.device)

    # ---------------------------------------------------------------- state
    @property
    def ep_start(self) -> "torch.Tensor":
        return self._arrays()[0]

    @property
    def ep_length(self) -> "torch.Tensor":
        return self._arrays()[1]

    @property
    def pos(self) -> int:
        return int(self.lib.pgx_replay_size(self._h) % self.buffer_size)

    @property
    def full(self) -> bool:
        return self.lib.pgx_replay_size(self._h) >= self.buffer_size

    def size(self) -> int:
        """SB3 BaseBuffer.size: transitions stored per env."""
        return self.buffer_size if self.full else self.pos

    # ------------------------------------------------------------------ add
    def add_tensors(self, obs, achieved_goal, desired_goal, action, reward, next_obs, next_achieved_goal,
                    next_desired_goal, done, timeout=None) -> None:
        """Store one transition per env from device (or host) arrays, SB3 HerReplayBuffer.add order."""
        N, od, ad = self.n_envs, self.obs_dim, self.action_dim
        f, u8 = torch.float32, torch.uint8
        t = [self._dev(obs, (N, od), f), self._dev(achieved_goal, (N, 3), f), self._dev(desired_goal, (N, 3), f),
             self._dev(action, (N, ad), f), self._dev(reward, (N,), f), self._dev(next_obs, (N, od), f),
             self._dev(next_achieved_goal, (N, 3), f), self._dev(next_desired_goal, (N, 3), f),
             self._dev(done, (N,), u8)]
        to = None
        if timeout is not None and self.handle_timeout_termination:
            to = self._dev(timeout, (N,), u8)
        tr = abi.PgxTransition(*[x.data_ptr() for x in t], None if to is None else to.data_ptr())
        check(self.lib.pgx_replay_add(self._h, C.byref(tr), self._stream()), "pgx_replay_add")
        self._keep = t + [to]  # alive until the stream has consumed them (same-stream allocator reuse is safe)

    def add(self, obs: Dict[str, Any], next_obs: Dict[str, Any], action, reward, done,
            infos: Sequence[Dict[str, Any]]) -> None:
        """SB3 signature: obs/next_obs dicts of [n_envs, ...] arrays; timeouts from infos."""
        timeout = np.array([bool(i.get("TimeLimit.truncated", False)) for i in infos], dtype=np.uint8)
        self.add_tensors(obs["observation"], obs["achieved_goal"], obs["desired_goal"], action, reward,
                         next_obs["observation"], next_obs["achieved_goal"], next_obs["desired_goal"],
                         np.asarray(done).astype(np.uint8) if not torch.is_tensor(done) else done, timeout)

    def add_from_vec_env(self, venv, obs: Dict[str, "torch.Tensor"], action: "torch.Tensor") -> None:
        """Store the step just taken by ``venv.step_tensors(action)`` from ``obs``, on device.

        ``obs`` is a copy of the observation the action was taken from.  next_obs is
        the terminal observation for every env that was auto-reset, terminated or truncated
        (SB3 off_policy_algorithm _store_transition reads infos["terminal_observation"] of
        any done env), dones = terminated | truncated, timeouts = truncated & ~terminated."""
        tr = venv.truncated.bool()
        te = venv.terminated.bool()
        done = (tr | te).to(torch.uint8)
        m = (tr | te).unsqueeze(1)   # every auto-reset env (time limit, collision, terminate_on_success)
        next_o = torch.where(m, venv.terminal_obs, venv.obs)
        next_ag = torch.where(m, venv.terminal_ag, venv.achieved_goal)
        next_dg = torch.where(m, venv.terminal_dg, venv.desired_goal)
        timeout = (tr & ~te).to(torch.uint8)
        self.add_tensors(obs["observation"], obs["achieved_goal"], obs["desired_goal"], action, venv.reward,
                         next_o, next_ag, next_dg, done, timeout)

    # --------------------------------------------------------------- sample
    def alloc_batch(self, batch_size: int, with_indices: bool = True) -> Dict[str, "torch.Tensor"]:
        """Batch tensors: ``rows`` [B, row_stride] plus per-field views into it (include/pgx.h layout)."""
        B = int(batch_size)
        rows = torch.empty((B, self.row_stride), dtype=torch.float32, device=self.device)
        out = {"rows": rows}
        for name, off, w in self._fields:
            out[name] = rows[:, off] if name in ("reward", "done") else rows[:, off:off + w]
        for k in ("slot", "env", "goal_slot"):
            out[k] = torch.empty((B,), dtype=torch.int32, device=self.device) if with_indices else None
        return out

    def sample_raw(self, batch_size: int, draw: Optional[int] = None) -> Dict[str, "torch.Tensor"]:
        """One relabelled batch: field views (obs, achieved_goal, ..., done) plus the drawn slot/env/goal_slot."""
        out = self.alloc_batch(batch_size)
        self.sample_into(out, draw)
        return out

    def sample_into(self, out: Dict[str, "torch.Tensor"], draw: Optional[int] = None) -> None:
        """Fill a batch from alloc_batch() (no allocation; the benchmark's timed call)."""
        rows = out["rows"]
        d = self._draw if draw is None else int(draw)
        self._draw = d + 1
        ptr = lambda k: out[k].data_ptr() if out.get(k) is not None else None  # noqa: E731
        b = abi.PgxReplayBatch(rows.data_ptr(), ptr("slot"), ptr("env"), ptr("goal_slot"))
        check(self.lib.pgx_replay_sample(self._h, C.c_int64(rows.shape[0]), C.c_uint64(d), C.byref(b),
                                         self._stream()), "pgx_replay_sample")
        if not self._seen_valid:
            # SB3 raises before the first episode has ended; check once (one sync) until it has
            if int(self._arrays()[2].item()) == 0:
                raise RuntimeError("Unable to sample before the end of the first episode. We recommend choosing "
                                   "a value for learning_starts that is greater than the maximum number of "
                                   "timesteps in the environment.")
            self._seen_valid = True

    def sample(self, batch_size: int, env: Any = None) -> DictReplayBufferSamples:
        """SB3 HerReplayBuffer.sample: real rows first, then int(her_ratio * B) relabelled rows."""
        r = self.sample_raw(batch_size)
        return DictReplayBufferSamples(
            observations={"observation": r["obs"], "achieved_goal": r["achieved_goal"],
                          "desired_goal": r["desired_goal"]},
            actions=r["action"],
            next_observations={"observation": r["next_obs"], "achieved_goal": r["next_achieved_goal"],
                               "desired_goal": r["next_desired_goal"]},
            dones=r["done"].reshape(-1, 1), rewards=r["reward"].reshape(-1, 1))
