"""Step-kernel time of the task / contact variants at 4096 envs (HIP events, 200 launches each).
Usage: python tools/time_variants.py"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import panda_gym_amd as pg  # noqa: E402


def run(env_id, contacts=True, policy="random", n=4096, launches=200, warm=100):
    venv = pg.PandaVecEnv(env_id, num_envs=n, device="cuda:0", seed=0, contacts=contacts)
    venv.reset_tensors()
    up = torch.zeros((n, venv.action_dim), device="cuda:0")
    up[:, 2] = 1.0
    for t in range(warm):
        venv.step_tensors(venv.sample_actions(t) if policy == "random" else up)
    acts = venv.sample_actions(warm).clone() if policy == "random" else up
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(launches):
        venv.step_tensors(acts)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / launches
    cnt = venv.state()["contacts"].cpu().numpy()
    frac = float(((cnt[0::2] >= 0).sum(axis=0) > 0).mean())
    venv.close()
    return ms, frac


for env_id, contacts, policy in [("PandaReach-v3", False, "random"), ("PandaReach-v3", True, "up"),
                                 ("PandaReach-v3", True, "random"), ("PandaPush-v3", True, "up"),
                                 ("PandaPush-v3", True, "random"), ("PandaPickAndPlace-v3", True, "random")]:
    ms, frac = run(env_id, contacts, policy)
    print(f"{env_id:24s} contacts={int(contacts)} policy={policy:6s} {ms:.3f} ms/step  "
          f"{4096 / ms / 1e3:.2f} M env-steps/s  envs-with-contacts {frac:.2f}", flush=True)
