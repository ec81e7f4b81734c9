"""TEST INFRASTRUCTURE ONLY: numpy restatement of SB3's HerReplayBuffer (the checker for pgx_her.hip).

Importable only from tests/ and bench.py's cpu_baseline leg; the product path
(panda-gym_amd/her.py -> libpgx.so) never imports it.

What it restates.  The reference trains with stable-baselines3's HerReplayBuffer
(training/utils/setup_training.py:14,176-179; classes/train_config.py:2,15;
the fork pinned at requirements.txt:142 is not in the container and SB3 is not
installed -- see DESIGN.md "HER relabelling": parity is anchored on the
published SB3 >= 2.0 algorithm, on the reference's own compute_reward
(reach.py:84-89, utils.py:18-30, pinned by tests/golden/reward_golden.npz) and
on SB3's test invariants (tests/test_her.py upstream: virtual goals come from
the same episode at or after t; rewards equal compute_reward).

  add()      HerReplayBuffer.add: for every env, if ep_length[pos] > 0 zero
             ep_length over arange(pos, ep_start[pos] + ep_length[pos]) % C;
             ep_start[pos] = current episode start; DictReplayBuffer.add
             stores the transition (timeouts = infos["TimeLimit.truncated"]);
             pos += 1 (wrap); for done envs _compute_episode_length writes
             the episode length over [start, pos) (unwrapped by + C) and the
             next episode starts at pos.
  sample()   valid = flatnonzero(ep_length > 0) over the [C, N] array;
             the b-th draw takes valid[floor(u0_b * n_valid)] (the
             np.random.choice of SB3 with the device's Philox stream in
             place of numpy's global RNG); the first int(her_ratio * B)
             draws are virtual, the rest real; the returned batch is
             real rows first, then virtual rows (SB3 concatenates
             real_data, virtual_data).  Virtual goals: "future"
             t' = cur + floor(u1 * (len - cur)) (np.random.randint(cur, len)),
             "final" len - 1, "episode" floor(u1 * len); goal slot
             (t' + ep_start) % C; desired_goal of obs and next_obs := that
             transition's next_achieved_goal; reward =
             compute_reward(next_achieved_goal, new goal) in float32; dones =
             done * (1 - timeout).
"""
from __future__ import annotations

from typing import Dict

import numpy as np

FUTURE, FINAL, EPISODE = 0, 1, 2
TAG_HER = 0x48455230
_M0, _M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
_W0, _W1 = 0x9E3779B9, 0xBB67AE85
_MASK = np.uint64(0xFFFFFFFF)


def philox4x32_10(c0, c1, c2, c3, k0: int, k1: int):
    """Vectorised Philox4x32-10 (Salmon et al., SC'11), uint32 arrays in and out."""
    c = [np.asarray(x, dtype=np.uint64) & _MASK for x in (c0, c1, c2, c3)]
    k0 = np.uint64(k0 & 0xFFFFFFFF)
    k1 = np.uint64(k1 & 0xFFFFFFFF)
    for _ in range(10):
        p0 = _M0 * c[0]
        p1 = _M1 * c[2]
        hi0, lo0 = p0 >> np.uint64(32), p0 & _MASK
        hi1, lo1 = p1 >> np.uint64(32), p1 & _MASK
        c = [hi1 ^ c[1] ^ k0, lo1, hi0 ^ c[3] ^ k1, lo0]
        k0 = np.uint64((int(k0) + _W0) & 0xFFFFFFFF)
        k1 = np.uint64((int(k1) + _W1) & 0xFFFFFFFF)
    return [x.astype(np.uint32) for x in c]


def u53(lo, hi) -> np.ndarray:
    v = (hi.astype(np.uint64) << np.uint64(32)) | lo.astype(np.uint64)
    return (v >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


def distance_f32(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """utils.distance (utils.py:18-30) on float32 arrays, as numpy evaluates it."""
    a = np.asarray(a, dtype=np.float32)
    b = np.asarray(b, dtype=np.float32)
    d = np.linalg.norm(a - b, axis=-1)
    return np.round(d, 6)


def compute_reward_f32(ag, dg, reward_type: int, thr: float = 0.05) -> np.ndarray:
    """Reach.compute_reward (reach.py:84-89) on float32 batches."""
    d = distance_f32(ag, dg)
    if reward_type == 2:   # ReachAO sparse, reach_ao.py:1320 (collision term 0)
        return -1 + np.array(d < np.float32(thr), dtype=np.float32)
    if reward_type == 0:
        return -np.array(d > thr, dtype=np.float32)
    return -d.astype(np.float32)


class HerOracle:
    """Host mirror of one pgx_replay ring, same layout ([C, N, ...]) and draws."""

    def __init__(self, n_envs: int, capacity: int, obs_dim: int, action_dim: int, reward_type: int = 0,
                 strategy: int = FUTURE, her_ratio: float = 0.8, thr: float = 0.05, seed: int = 0):
        C, N = capacity, n_envs
        self.C, self.N, self.od, self.ad = C, N, obs_dim, action_dim
        self.reward_type, self.strategy, self.her_ratio, self.thr, self.seed = reward_type, strategy, her_ratio, thr, seed
        z = lambda *s: np.zeros((C, N) + s, np.float32)  # noqa: E731
        self.obs, self.next_obs = z(obs_dim), z(obs_dim)
        self.ag, self.dg, self.next_ag, self.next_dg = z(3), z(3), z(3), z(3)
        self.action, self.reward = z(action_dim), z()
        self.done = np.zeros((C, N), np.uint8)
        self.timeout = np.zeros((C, N), np.uint8)
        self.ep_start = np.zeros((C, N), np.int64)
        self.ep_length = np.zeros((C, N), np.int64)
        self.cur_ep_start = np.zeros(N, np.int64)
        self.pos = 0
        self.full = False

    def add(self, obs, ag, dg, action, reward, next_obs, next_ag, next_dg, done, timeout) -> None:
        C, pos = self.C, self.pos
        for e in range(self.N):
            start, length = self.ep_start[pos, e], self.ep_length[pos, e]
            if length > 0:
                self.ep_length[np.arange(pos, start + length) % C, e] = 0
        self.ep_start[pos] = self.cur_ep_start
        self.obs[pos], self.ag[pos], self.dg[pos] = obs, ag, dg
        self.action[pos], self.reward[pos] = action, reward
        self.next_obs[pos], self.next_ag[pos], self.next_dg[pos] = next_obs, next_ag, next_dg
        self.done[pos], self.timeout[pos] = done, timeout
        self.pos = (pos + 1) % C
        if self.pos == 0:
            self.full = True
        for e in np.flatnonzero(np.asarray(done)):
            start = self.cur_ep_start[e]
            end = self.pos if self.pos >= start else self.pos + C
            self.ep_length[np.arange(start, end) % C, e] = end - start
            self.cur_ep_start[e] = self.pos

    def draws(self, batch: int, draw: int):
        b = np.arange(batch, dtype=np.uint64)
        r = philox4x32_10(b & _MASK, b >> np.uint64(32), np.full(batch, draw & 0xFFFFFFFF, np.uint64),
                          np.full(batch, TAG_HER ^ ((draw >> 32) & 0xFFFFFFFF), np.uint64), self.seed & 0xFFFFFFFF,
                          self.seed >> 32)
        return u53(r[0], r[1]), u53(r[2], r[3])

    def sample(self, batch: int, draw: int) -> Dict[str, np.ndarray]:
        C, N = self.C, self.N
        valid = np.flatnonzero(self.ep_length > 0)
        if len(valid) == 0:
            raise RuntimeError("Unable to sample before the end of the first episode")
        u0, u1 = self.draws(batch, draw)
        j = np.minimum((u0 * len(valid)).astype(np.int64), len(valid) - 1)
        flat = valid[j]
        slot, env = flat // N, flat % N
        nbv = int(self.her_ratio * batch)
        her = np.arange(batch) < nbv
        start, length = self.ep_start[slot, env], self.ep_length[slot, env]
        cur = (slot - start) % C
        if self.strategy == FINAL:
            t_in = length - 1
        elif self.strategy == EPISODE:
            t_in = (u1 * length).astype(np.int64)
        else:
            t_in = cur + (u1 * (length - cur)).astype(np.int64)
        gslot = (t_in + start) % C
        new_goal = self.next_ag[gslot, env]
        dg = np.where(her[:, None], new_goal, self.dg[slot, env])
        ndg = np.where(her[:, None], new_goal, self.next_dg[slot, env])
        rew = np.where(her, compute_reward_f32(self.next_ag[slot, env], new_goal, self.reward_type, self.thr),
                       self.reward[slot, env]).astype(np.float32)
        out = dict(obs=self.obs[slot, env], achieved_goal=self.ag[slot, env], desired_goal=dg,
                   action=self.action[slot, env], reward=rew, next_obs=self.next_obs[slot, env],
                   next_achieved_goal=self.next_ag[slot, env], next_desired_goal=ndg,
                   done=(self.done[slot, env] * (1 - self.timeout[slot, env])).astype(np.float32),
                   slot=slot.astype(np.int32), env=env.astype(np.int32),
                   goal_slot=np.where(her, gslot, -1).astype(np.int32))
        # SB3 returns the real samples first, then the virtual ones
        order = np.concatenate([np.arange(nbv, batch), np.arange(nbv)])
        return {k: v[order] for k, v in out.items()}
