"""Step-kernel time of each task config in both step layouts (PGX_LANES_PER_ENV = 16 / 1) with
the product library: HIP events around `launches` steps of the device random policy.
Usage: python tools/time_layouts.py [launches]"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import panda_gym_amd as pg  # noqa: E402

CASES = [("PandaReach-v3", 4096, True), ("PandaReach-v3", 4096, False), ("PandaReach-v3", 8192, True),
         ("PandaReach-v3", 16384, True), ("PandaReach-v3", 65536, True), ("PandaPush-v3", 4096, True),
         ("PandaPickAndPlace-v3", 8192, True), ("PandaPickAndPlace-v3", 16384, True),
         ("PandaReachAO-v3", 8192, True)]


def run(env_id, n, contacts, launches):
    venv = pg.PandaVecEnv(env_id, num_envs=n, device="cuda:0", seed=0, contacts=contacts)
    venv.reset_tensors()
    for t in range(30):
        venv.step_tensors(venv.sample_actions(t))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for t in range(launches):
        venv.step_tensors(venv.sample_actions(30 + t))
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / launches
    venv.close()
    return ms


if __name__ == "__main__":
    launches = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    if os.environ.get("TL_CASES"):   # e.g. TL_CASES="PandaReach-v3:16384:1,PandaPush-v3:16384:1"
        CASES = [(a, int(b), bool(int(c))) for a, b, c in (x.split(":") for x in os.environ["TL_CASES"].split(","))]
    for env_id, n, contacts in CASES:
        row = {"env_id": env_id, "n": n, "contacts": contacts}
        for lanes in (16, 1):
            os.environ["PGX_LANES_PER_ENV"] = str(lanes)
            ms = run(env_id, n, contacts, launches)
            row[f"ms_{lanes}"] = round(ms, 4)
            row[f"Msteps_{lanes}"] = round(n / ms / 1e3, 3)
        print(json.dumps(row), flush=True)
