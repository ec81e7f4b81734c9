"""Diagnostic: the two-waves-per-SIMD build (8192 envs) against two one-wave 4096-env shards,
per step: envs whose observation differs and the largest difference (PGX_PGS_MODE honoured)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import panda_gym_amd as pg  # noqa: E402

env_id = sys.argv[1] if len(sys.argv) > 1 else "PandaReach-v3"
n = 8192
big = pg.PandaVecEnv(env_id, num_envs=n, device="cuda:0", seed=5, lanes_per_env=16)
parts = [pg.PandaVecEnv(env_id, num_envs=n // 2, device="cuda:0", seed=5, lanes_per_env=16,
                        env_id_offset=k * (n // 2)) for k in range(2)]
for v in [big] + parts:
    v.reset_tensors()
for t in range(14):
    big.step_tensors(big.sample_actions(t))
    for v in parts:
        v.step_tensors(v.sample_actions(t))
    got = torch.cat([v.obs for v in parts])
    d = (got - big.obs).abs().amax(dim=1)
    bad = torch.nonzero(d > 0).flatten()
    print(t, "envs differing:", bad.numel(), "max", float(d.max()), "first", bad[:8].tolist(), flush=True)
