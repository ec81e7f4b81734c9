"""Diagnostic: default solve modes against PGX_PGS_MODE=2 (all rows, never speculate), same
seeds and Philox actions, at n envs: per step the envs whose observation differs."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import panda_gym_amd as pg  # noqa: E402

env_id = sys.argv[1]
n = int(sys.argv[2])
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 14
obs = {}
for mode in ("0", "2"):
    os.environ["PGX_PGS_MODE"] = mode
    v = pg.PandaVecEnv(env_id, num_envs=n, device="cuda:0", seed=5, lanes_per_env=16)
    v.reset_tensors()
    o = []
    for t in range(steps):
        v.step_tensors(v.sample_actions(t))
        o.append(v.obs.clone())
    obs[mode] = o
    v.close()
for t in range(steps):
    d = (obs["0"][t] - obs["2"][t]).abs().amax(dim=1)
    bad = torch.nonzero(d > 0).flatten()
    print(env_id, n, t, "envs differing:", bad.numel(), "max", float(d.max()), "first", bad[:8].tolist(), flush=True)
