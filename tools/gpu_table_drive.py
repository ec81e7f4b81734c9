"""GPU: the table-drive scenario of test_reach_with_table_contacts (and one Push random-policy run)
per step from the device state, device vs fp64 oracle against the fp32 oracle vs fp64 from the
same state (the restated algorithm's own fp32 envelope), at the tool bar's friction of
panda.py:69-70 (the default library) and at mu 0.25 everywhere (round 3's value, through
libpgx_rtmodel.so), in both layouts.

    python tools/gpu_table_drive.py
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import panda_gym_amd as pg  # noqa: E402
from oracle import oracle as O  # noqa: E402
from panda_gym_amd import _native  # noqa: E402
from test_gpu_parity import _state_to_oracle  # noqa: E402


def _copy(src, dst):
    for k in ("q", "qd", "qc", "goal", "obj", "elapsed", "episode"):
        getattr(dst, k)[:] = getattr(src, k)


def run(env_id, n, steps, lanes, actions=None, **kw):
    venv = pg.PandaVecEnv(env_id, num_envs=n, device="cuda:0", seed=3, lanes_per_env=lanes, **kw)
    venv.reset_tensors(seed=3)
    r64 = O.OracleVecEnv(venv._cfg, n)
    r32 = O.OracleVecEnv(venv._cfg, n, fp32=True)
    dev, f32, bad = [], [], None
    for t in range(steps):
        _state_to_oracle(venv, r64)
        _copy(r64, r32)
        a = venv.sample_actions(t).clone() if actions is None else torch.as_tensor(actions, device="cuda:0")
        venv.step_tensors(a)
        an = a.cpu().numpy()
        o64, o32 = r64.step(an), r32.step(an)
        keep = (o64["truncated"] == 0)
        obs = venv.obs.cpu().numpy()
        if bad is None and not np.isfinite(obs).all():
            bad = {"step": t, "envs": np.flatnonzero(~np.isfinite(obs).all(axis=1)).tolist()[:8]}
        dev.append(np.abs(obs[keep, :3] - o64["obs"][keep, :3]).max(axis=1))
        f32.append(np.abs(o32["obs"][keep, :3] - o64["obs"][keep, :3]).max(axis=1))
    venv.close()
    d, f = np.concatenate(dev), np.concatenate(f32)
    q = lambda x, p: float(np.percentile(x, p))  # noqa: E731
    return {"first_nonfinite": bad, "device": {"p99": q(d, 99), "p99.9": q(d, 99.9), "max": float(d.max())},
            "fp32_oracle": {"p99": q(f, 99), "p99.9": q(f, 99.9), "max": float(f.max())}}


def main():
    pg.load_native()
    rt = os.path.join(os.path.dirname(_native.LIB_PATH), "libpgx_rtmodel.so")
    rng = np.random.default_rng(3)
    off = rng.uniform(-0.2, 0.2, (64, 3)).astype(np.float32)
    off[:, 2] = 0.0
    drive = np.clip(np.array([0.3, -0.2, -1.0], np.float32) + off, -1, 1).astype(np.float32)
    # link_friction holds the combined mu of a link against the scene (abi.default_sim_params)
    cases = (("tool_mu_0.5", {}), ("mu_0.25_everywhere", {"sim_params": {"link_friction": [0.25] * 16}, "lib_path": rt}),
             ("mu_0.5_everywhere", {"sim_params": {"link_friction": [0.5] * 16}, "lib_path": rt}))
    for lanes in (16, 1):
        for name, kw in cases:
            r = run("PandaReach-v3", 64, 30, lanes, drive, **kw)
            print(json.dumps({"case": "table_drive", "lanes": lanes, "friction": name, **r}), flush=True)
            r = run("PandaPush-v3", 256, 50, lanes, None, **kw)
            print(json.dumps({"case": "push_random", "lanes": lanes, "friction": name, **r}), flush=True)


if __name__ == "__main__":
    main()
