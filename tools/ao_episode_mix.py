"""ReachAO episode-end mix under the bench's random policy (staggered phases, steady state): the share
of env-steps that end an episode by collision (terminated without success), by success, and by the
TimeLimit, and the mean episode length -- what sets how often the in-kernel ReachAO reset runs.
python tools/ao_episode_mix.py [N] [STEPS]; prints one JSON line."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import panda_gym_amd as pg  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    v = pg.PandaVecEnv("PandaReachAO-v3", num_envs=n, device="cuda:0", seed=0)
    v.reset_tensors(episode_phase="staggered")
    T = int(v.spec.max_episode_steps)
    for t in range(T + 20):
        v.step_tensors(v.sample_actions(t))
    term = succ = trunc = 0
    for t in range(steps):
        _, _, te, tr, su = v.step_tensors(v.sample_actions(T + 20 + t))
        te, tr, su = te.bool(), tr.bool(), su.bool()
        term += int((te & ~su).sum())
        succ += int((te & su).sum())
        trunc += int((tr & ~te).sum())
    tot = n * steps
    ends = term + succ + trunc
    print(json.dumps({"n": n, "steps": steps, "collision_end_per_env_step": term / tot,
                      "success_end_per_env_step": succ / tot, "timelimit_end_per_env_step": trunc / tot,
                      "mean_episode_length": tot / max(ends, 1)}), flush=True)
    v.close()


if __name__ == "__main__":
    main()
