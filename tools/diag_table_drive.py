"""The table-drive scenario of test_gpu_contacts.test_reach_with_table_contacts, in the oracle only:
how far the restated algorithm itself moves per step, from the same fp32-rounded state, when it
is evaluated in fp32 (the fp32 build) or when its input is perturbed by 1e-7 relative -- at the
tool bar's lateral friction of panda.py:69-70 (links 9, 10 at 1.0: mu 0.5 against the table) and
at the round-3 value (0.5 everywhere: mu 0.25).

    python tools/diag_table_drive.py [--envs 64] [--steps 30]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402
from panda_gym_amd import abi, envs  # noqa: E402
from panda_gym_amd.model import load_model  # noqa: E402


def make(env_id, n, tool_mu, fp32=False):
    model = abi.make_model(load_model("panda_custom0"), ee_link=11)
    params = abi.default_sim_params()
    for i in abi.FINGER_FRICTION_LINKS:
        params.link_friction[i] = tool_mu
    cfg = abi.make_config(envs.spec(env_id), n, model, params, seed=3, full_manifold=True)
    return O.OracleVecEnv(cfg, n, fp32=fp32), (model, params, cfg)


def _copy(src, dst, rel=0.0, rng=None):
    for k in ("q", "qd", "qc", "goal", "obj", "elapsed", "episode"):
        getattr(dst, k)[:] = getattr(src, k)
    if rel:
        dst.q[:] *= 1.0 + rel * rng.standard_normal(dst.q.shape)
        dst.qd[:] *= 1.0 + rel * rng.standard_normal(dst.qd.shape)


def run(n, steps, tool_mu, trials=4):
    base, k0 = make("PandaReach-v3", n, tool_mu)
    f64, k1 = make("PandaReach-v3", n, tool_mu)
    f32, k2 = make("PandaReach-v3", n, tool_mu, fp32=True)
    pert, k3 = make("PandaReach-v3", n, tool_mu)
    base.reset()
    rng = np.random.default_rng(3)
    off = rng.uniform(-0.2, 0.2, (n, 3)).astype(np.float32)
    off[:, 2] = 0.0
    a = np.clip(np.array([0.3, -0.2, -1.0], np.float32) + off, -1, 1).astype(np.float32)
    e32, epert = [], []
    prng = np.random.default_rng(0)
    for t in range(steps):
        # the device state is fp32: round the carried state first
        for k in ("q", "qd", "qc"):
            getattr(base, k)[:] = getattr(base, k).astype(np.float32)
        base.obj[:, :13] = base.obj[:, :13].astype(np.float32)
        _copy(base, f64)
        _copy(base, f32)
        o64 = f64.step(a)
        o32 = f32.step(a)
        e32.append(np.abs(o32["obs"][:, :3] - o64["obs"][:, :3]).max(axis=1))
        d = np.zeros(n)
        for _ in range(trials):
            _copy(base, pert, 1e-7, prng)
            op = pert.step(a)
            d = np.maximum(d, np.abs(op["obs"][:, :3] - o64["obs"][:, :3]).max(axis=1))
        epert.append(d)
        base.step(a)
    del k0, k1, k2, k3
    e32, epert = np.concatenate(e32), np.concatenate(epert)
    q = lambda x, p: float(np.percentile(x, p))  # noqa: E731
    return {"tool_mu_link": tool_mu, "envs": n, "steps": steps,
            "fp32_oracle_ee": {"p99": q(e32, 99), "max": float(e32.max())},
            "perturbed_1e-7_ee": {"p99": q(epert, 99), "max": float(epert.max())}}


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=64)
    ap.add_argument("--steps", type=int, default=30)
    args = ap.parse_args()
    for mu in (1.0, 0.5):
        print(json.dumps(run(args.envs, args.steps, mu)), flush=True)
