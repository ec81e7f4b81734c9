"""Steady-state step time of one config (episode phases staggered, as bench.py times the headline),
for A/B runs of handle options: python tools/time_staggered.py ENV N [key=value ...]
(values parsed as Python literals, e.g. full_manifold=False lanes_per_env=16); prints one JSON line."""
import ast
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import panda_gym_amd as pg  # noqa: E402


def main():
    env_id, n = sys.argv[1], int(sys.argv[2])
    kw = {k: ast.literal_eval(v) for k, v in (a.split("=", 1) for a in sys.argv[3:])}
    v = pg.PandaVecEnv(env_id, num_envs=n, device="cuda:0", seed=0, **kw)
    v.reset_tensors(episode_phase="staggered")
    T = int(v.spec.max_episode_steps)
    for t in range(T + 20):
        v.step_tensors(v.sample_actions(t))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    steps = 200
    torch.cuda.synchronize()
    e0.record()
    for t in range(steps):
        v.step_tensors(v.sample_actions(T + 20 + t))
    e1.record()
    torch.cuda.synchronize()
    print(json.dumps({"env_id": env_id, "n": n, **{k: str(x) for k, x in kw.items()}, "kernel": v.step_kernel(),
                      "ms_per_step": e0.elapsed_time(e1) / steps}), flush=True)
    v.close()


if __name__ == "__main__":
    main()
