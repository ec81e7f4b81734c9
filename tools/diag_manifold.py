"""Robot contact points per substep under Bullet's per-pair manifold rule (<= 4 per colliding
pair, before the row budget), fp64 oracle, bench workload (random policy, auto-reset): the
share of substeps a robot budget of B points would cut, per task.
Usage: python tools/diag_manifold.py [n_envs] [steps] [budget]   (budget: the oracle's, default 16)"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402
from panda_gym_amd import abi, envs  # noqa: E402
from panda_gym_amd.model import load_model  # noqa: E402


def run(env_id, n, steps, budget):
    model = abi.make_model(load_model("panda_custom0"), ee_link=11)
    cfg = abi.make_config(envs.spec(env_id), n, model, abi.default_sim_params())
    O.set_robot_budget(budget)
    env = O.OracleVecEnv(cfg, n)
    env.reset()
    O.pair_hist(clear=True)
    for t in range(steps):
        env.step(env.sample_actions(t))
    h = O.pair_hist(clear=True)
    O.set_robot_budget(-1)
    tot = h.sum()
    return {"substeps": int(tot), "hist": {i: int(c) for i, c in enumerate(h) if c},
            **{f"over_{b}": float(h[b + 1:].sum() / tot) for b in (4, 6, 8, 12)}}


if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    budget = int(sys.argv[3]) if len(sys.argv) > 3 else 16
    for env_id in ("PandaReach-v3", "PandaPush-v3", "PandaPickAndPlace-v3", "PandaReachAO-v3"):
        print(env_id, json.dumps(run(env_id, n, steps, budget)), flush=True)
