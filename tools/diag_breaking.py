"""How far Bullet's relative contact breaking threshold (the default since round 6: per pair the
smaller of the two shapes' angular motion disc x 0.02, oracle breaking_thresholds) moves the envs
from the global 0.02 of rounds 2-5 (oracle flag PGX_FLAG_GLOBAL_BREAKING), in the fp64 oracle: the
same reset and the same device-Philox random actions for both, free running; the divergence of the
EE and object positions per step against the chaos floor of the default rule itself (its initial
state perturbed by 1e-7 relative); the robot contact points per substep under
each rule, and the manifold pool's occupancy.

    python tools/diag_breaking.py [--envs 128] [--steps 50] [--env PandaPush-v3 ...]
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402
from panda_gym_amd import abi, envs  # noqa: E402
from panda_gym_amd.model import load_model  # noqa: E402


def make(env_id, n, flags):
    model = abi.make_model(load_model("panda_custom0"), ee_link=11)
    params = abi.default_sim_params(flags=flags)
    cfg = abi.make_config(envs.spec(env_id), n, model, params, seed=1, full_manifold=True)
    return O.OracleVecEnv(cfg, n), (model, params, cfg)


def run(env_id, n, steps):
    base, k0 = make(env_id, n, 0)
    pert, k1 = make(env_id, n, 0)
    glob, k2 = make(env_id, n, abi.FLAG_GLOBAL_BREAKING)
    for e in (base, pert, glob):
        e.reset()
    rng = np.random.default_rng(0)
    pert.q[:] *= 1.0 + 1e-7 * rng.standard_normal(pert.q.shape)
    if env_id not in ("PandaReach-v3", "PandaReachAO-v3"):
        pert.obj[:, :3] *= 1.0 + 1e-7 * rng.standard_normal((n, 3))
    O.pair_hist(clear=True)
    rows, hist = [], {"relative": None, "global": None}
    pool_max, pool_sum, pool_n = 0, 0.0, 0
    for t in range(steps):
        a = base.sample_actions(t)
        ob = base.step(a)
        h = O.pair_hist(clear=True)
        hist["relative"] = h if hist["relative"] is None else hist["relative"] + h
        op = pert.step(a)
        O.pair_hist(clear=True)
        og = glob.step(a)
        h = O.pair_hist(clear=True)
        hist["global"] = h if hist["global"] is None else hist["global"] + h
        if env_id != "PandaReach-v3":
            cnt = base.obj[:, O.OBJ_MAN]
            pool_max, pool_sum, pool_n = max(pool_max, int(cnt.max())), pool_sum + float(cnt.sum()), pool_n + n
        live = (ob["truncated"] == 0) & (og["truncated"] == 0) & (op["truncated"] == 0)
        if t + 1 in (1, 2, 5, 10, 20, 30, 49) and live.any():
            def dev(x, y, cols):
                d = np.abs(x["obs"][live][:, cols] - y["obs"][live][:, cols]).max(axis=1)
                return {"p50": float(np.percentile(d, 50)), "p99": float(np.percentile(d, 99)), "max": float(d.max())}
            row = {"step": t + 1, "ee_global_rule": dev(ob, og, [0, 1, 2]), "ee_chaos_floor": dev(ob, op, [0, 1, 2])}
            if env_id in ("PandaPush-v3", "PandaPickAndPlace-v3"):
                row.update(object_global_rule=dev(ob, og, [6, 7, 8]), object_chaos_floor=dev(ob, op, [6, 7, 8]))
            rows.append(row)
    del k0, k1, k2

    def summ(h):
        tot = h.sum()
        pts = np.arange(len(h))
        return {"substeps": int(tot), "mean_points": float((h * pts).sum() / tot), "share_gt0": float(h[1:].sum() / tot),
                "share_gt4": float(h[5:].sum() / tot), "max": int(pts[h > 0].max())}
    return {"env_id": env_id, "envs": n, "steps": steps, "divergence": rows,
            "robot_points_per_substep": {k: summ(v) for k, v in hist.items()},
            "pool": {"max_points": pool_max, "mean_points_after_step": pool_sum / max(pool_n, 1)}}


def thresholds():
    """The per-pair thresholds the default rule gives (link, scene body), in metres."""
    model = load_model("panda_custom0")
    out = {}
    for i, name in enumerate(model.link_names):
        out[name] = (np.linalg.norm(model.aabb_half[i]) + np.linalg.norm(model.aabb_center[i])) * 0.02
    m = 0.001
    box = lambda *h: float(np.linalg.norm(np.array(h) + m) * 0.02)  # noqa: E731
    out.update(table=box(0.55, 0.35, 0.2), table_reach_ao=box(1.0, 0.65, 0.2), plane=box(3.0, 3.0, 0.01),
               cube=box(0.02, 0.02, 0.02), obstacle=box(0.05, 0.05, 0.05))
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=128)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--env", nargs="*", default=["PandaReach-v3", "PandaPush-v3", "PandaPickAndPlace-v3",
                                                 "PandaReachAO-v3"])
    args = ap.parse_args()
    print(json.dumps({"thresholds_m": thresholds()}), flush=True)
    for env_id in args.env:
        print(json.dumps(run(env_id, args.envs, args.steps)), flush=True)
