"""How far Bullet's persistent manifolds (the default with the per-pair budget since round 5) move
Push / PickAndPlace / ReachAO from round 4's fresh rule (each pair's 4 deepest candidates of the
substep, oracle flag PGX_FLAG_FRESH_MANIFOLD), in the fp64 oracle: the same reset and the same
device-Philox random actions for both, free running; the divergence of the EE and object positions
per step, against the chaos floor of the default rule itself (its initial state perturbed by 1e-7
relative: contact trajectories are chaotic at rounding level); the robot
contact points per substep in each mode, the manifold pool's occupancy and its overflows
(pgxo_diag_hist[120]: points dropped because the pool was full).

    python tools/diag_persistent.py [--envs 128] [--steps 50]
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


def make(env_id, n, flags):
    model = abi.make_model(load_model("panda_custom0"), ee_link=11)
    params = abi.default_sim_params(flags=flags)
    cfg = abi.make_config(envs.spec(env_id), n, model, params, seed=1, full_manifold=True)
    return O.OracleVecEnv(cfg, n), (model, params, cfg)


def run(env_id, n, steps):
    base, k0 = make(env_id, n, 0)
    pert, k1 = make(env_id, n, 0)
    pers, k2 = make(env_id, n, abi.FLAG_FRESH_MANIFOLD)   # ("pers": the comparison rule, round 4's)
    for e in (base, pert, pers):
        e.reset()
    rng = np.random.default_rng(0)
    pert.q[:] *= 1.0 + 1e-7 * rng.standard_normal(pert.q.shape)
    pert.obj[:, :3] *= 1.0 + 1e-7 * rng.standard_normal((n, 3))
    O.pair_hist(clear=True)
    import ctypes as C
    diag = np.zeros(128, np.int64)
    O.lib().pgxo_diag_read(diag.ctypes.data_as(C.c_void_p), 1)
    rows = []
    hist = {}
    pool_max, pool_sum, pool_n = 0, 0, 0
    for t in range(steps):
        a = base.sample_actions(t)
        ob = base.step(a)
        hist.setdefault("default", np.zeros(O.ROBOT_HIST if hasattr(O, "ROBOT_HIST") else 33, np.int64))
        hist["default"] += O.pair_hist(clear=True)[:len(hist["default"])]
        op = pert.step(a)
        O.pair_hist(clear=True)
        om = pers.step(a)
        hist.setdefault("fresh", np.zeros_like(hist["default"]))
        hist["fresh"] += O.pair_hist(clear=True)[:len(hist["default"])]
        cnt = base.obj[:, O.OBJ_MAN]
        pool_max, pool_sum, pool_n = max(pool_max, int(cnt.max())), pool_sum + float(cnt.sum()), pool_n + n
        live = (ob["truncated"] == 0) & (om["truncated"] == 0) & (op["truncated"] == 0)
        if t + 1 in (1, 2, 5, 10, 20, 30, 49) and live.any():
            def dev(x, y, cols):
                d = np.abs(x["obs"][live][:, cols] - y["obs"][live][:, cols]).max(axis=1)
                return {"p50": float(np.percentile(d, 50)), "p99": float(np.percentile(d, 99)), "max": float(d.max())}
            oc = [0, 1, 2] if env_id == "PandaReachAO-v3" else [6, 7, 8]
            rows.append({"step": t + 1, "ee_fresh_rule": dev(ob, om, [0, 1, 2]), "ee_chaos_floor": dev(ob, op, [0, 1, 2]),
                         "object_fresh_rule": dev(ob, om, oc), "object_chaos_floor": dev(ob, op, oc)})
    del k0, k1, k2

    def summ(h):
        tot = h.sum()
        pts = np.arange(len(h))
        return {"substeps": int(tot), "mean_points": float((h * pts).sum() / tot), "share_gt4": float(h[5:].sum() / tot),
                "share_gt8": float(h[9:].sum() / tot), "max": int(pts[h > 0].max())}
    O.lib().pgxo_diag_read(diag.ctypes.data_as(C.c_void_p), 1)
    return {"env_id": env_id, "envs": n, "steps": steps, "divergence": rows,
            "robot_points_per_substep": {k: summ(v) for k, v in hist.items()},
            "pool": {"max_points": pool_max, "mean_points_after_step": pool_sum / max(pool_n, 1),
                     "overflow_drops": int(diag[120])}}


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=128)
    ap.add_argument("--steps", type=int, default=50)
    args = ap.parse_args()
    for env_id in ("PandaPush-v3", "PandaPickAndPlace-v3", "PandaReachAO-v3"):
        print(json.dumps(run(env_id, args.envs, args.steps)), flush=True)
