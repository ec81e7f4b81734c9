"""Robot contact points per env at the end of each step (the warm-start cache's live robot slots),
steady state (staggered episode phases, random policy): the distribution that sets the per-pair
budget kernels' extra rows.  python tools/point_hist.py ENV N [steps]"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import panda_gym_amd as pg  # noqa: E402
from panda_gym_amd import abi  # noqa: E402


def main():
    env_id, n = sys.argv[1], int(sys.argv[2])
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 100
    v = pg.PandaVecEnv(env_id, num_envs=n, device="cuda:0", seed=0)
    v.reset_tensors(episode_phase="staggered")
    T = int(v.spec.max_episode_steps)
    for t in range(T):
        v.step_tensors(v.sample_actions(t))
    rb = v.robot_contact_budget()
    hist = np.zeros(rb + 1, np.int64)
    wave_max = np.zeros(rb + 1, np.int64)
    launch_max = np.zeros(rb + 1, np.int64)
    for t in range(steps):
        v.step_tensors(v.sample_actions(T + t))
        c = v.state()["contacts"]
        ids = c[2 * abi.OBJECT_POINTS::2][:rb]            # robot slots' feature ids
        cnt = (ids >= 0).sum(0).cpu().numpy()
        hist += np.bincount(cnt, minlength=rb + 1)[:rb + 1]
        wm = cnt.reshape(-1, 4).max(1)                    # 16-lane layout: 4 envs per wave
        wave_max += np.bincount(wm, minlength=rb + 1)[:rb + 1]
        launch_max[cnt.max()] += 1
        torch.cuda.synchronize()
    print(json.dumps({"env_id": env_id, "n": n, "steps": steps, "budget": rb,
                      "env_steps_by_points": hist.tolist(), "wave_steps_by_max_points": wave_max.tolist(),
                      "launches_by_max_points": launch_max.tolist()}), flush=True)
    v.close()


if __name__ == "__main__":
    main()
