"""Run the same object-task rollout twice on the device and report bitwise differences and the
one-step oracle error per step (diagnostic)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import panda_gym_amd as pg  # noqa: E402
from oracle import oracle as O  # noqa: E402
from test_gpu_parity import _state_to_oracle  # noqa: E402

env_id = sys.argv[1] if len(sys.argv) > 1 else "PandaPush-v3"
O.build()
runs = []
for rep in range(2):
    venv = pg.PandaVecEnv(env_id, num_envs=256, device="cuda:0", seed=5)
    venv.reset_tensors(seed=100)
    ref = O.OracleVecEnv(venv._cfg, 256)
    hist = []
    for k in range(6):
        _state_to_oracle(venv, ref)
        a = venv.sample_actions(k).clone()
        venv.step_tensors(a)
        out = ref.step(a.cpu().numpy())
        obs = venv.obs.cpu().numpy().copy()
        e = np.abs(obs - out["obs"])
        i = int(np.argmax(e[:, :3].max(axis=1)))
        print(f"rep {rep} step {k}: ee err max {e[:, :3].max():.3e} (env {i}) obj err {e[:, 6:9].max():.3e}")
        if e[:, :3].max() > 1e-3:
            st = venv.state()
            print("   gpu", obs[i, :9]); print("   ref", out["obs"][i, :9])
            print("   q   ", st["q"].cpu().numpy()[:, i]); print("   qref", ref.q[i])
            print("   cont", st["contacts"].cpu().numpy()[:, i])
        hist.append(obs)
    runs.append(np.stack(hist))
    venv.close()
d = np.abs(runs[0] - runs[1])
print("run-to-run max diff per step:", d.reshape(6, -1).max(axis=1))
