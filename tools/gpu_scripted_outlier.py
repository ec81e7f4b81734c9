"""Find and dump the per-step outliers of the scripted-push parity run (tests/test_gpu_contacts.py
test_persistent_manifold_branches_under_a_scripted_push): every env-step whose EE or achieved goal
differs from the fp64 oracle by more than --thr after one step from the same state, with the oracle
input state, the action, and the device's and oracle's outputs, into gpurun_out/scripted_outliers.npz
for the CPU analysis (tools/analyze_outlier.py).

    python tools/gpu_scripted_outlier.py [--env PandaPickAndPlace-v3] [--thr 1e-2]
"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import panda_gym_amd as pg  # noqa: E402
from oracle import oracle as O  # noqa: E402
from scripted_push import ScriptedPush  # noqa: E402
from test_gpu_parity import _state_to_oracle  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--env", default="PandaPickAndPlace-v3")
    ap.add_argument("--thr", type=float, default=1e-2)
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--steps", type=int, default=40)
    args = ap.parse_args()
    n = args.n
    venv = pg.PandaVecEnv(args.env, num_envs=n, device="cuda:0", seed=3, lanes_per_env=16, full_manifold=True)
    venv.reset_tensors(seed=3)
    ref = O.OracleVecEnv(venv._cfg, n)
    pol = ScriptedPush(n, seed=7, obj_col=6 if args.env == "PandaPush-v3" else 7)
    recs = []
    for t in range(args.steps):
        _state_to_oracle(venv, ref)
        saved = {k: getattr(ref, k).copy() for k in ("q", "qd", "qc", "goal", "obj", "elapsed", "episode")}
        a = pol(venv.obs.cpu().numpy(), t)
        if args.env != "PandaPush-v3":
            a = np.concatenate([a, np.zeros((n, 1), np.float32)], axis=1)
        at = torch.as_tensor(a, device="cuda:0")
        venv.step_tensors(at)
        out = ref.step(a)
        obs, ag = venv.obs.cpu().numpy(), venv.achieved_goal.cpu().numpy()
        err = np.maximum(np.abs(obs[:, :3] - out["obs"][:, :3]).max(1), np.abs(ag - out["ag"]).max(1))
        err[out["truncated"] != 0] = 0.0
        for i in np.flatnonzero(~(err <= args.thr)):   # NaN included
            st = venv.state()
            recs.append(dict(t=t, env=i, err=err[i], action=a[i], dev_obs=obs[i], ora_obs=out["obs"][i],
                             dev_obj=st["object"][:, i].cpu().numpy(), ora_obj=ref.obj[i, :13].copy(),
                             **{"in_" + k: v[i] for k, v in saved.items()}))
            print(f"t {t} env {i} err {err[i]:.3e} dev obj {st['object'][:3, i].cpu().numpy()} "
                  f"oracle obj {ref.obj[i, :3]} dev ee {obs[i, :3]} oracle ee {out['obs'][i, :3]}", flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.savez(os.path.join(ROOT, "gpurun_out", "scripted_outliers.npz"),
             **{f"{k}_{j}": np.asarray(v) for j, r in enumerate(recs) for k, v in r.items()}, count=len(recs))
    print(f"{len(recs)} outliers above {args.thr}")


if __name__ == "__main__":
    main()
