"""Distribution of the per-step GPU-vs-oracle error (from the same state) on the random-policy
contact workload of tests/test_gpu_contacts.py, and, for the worst sample, the oracle's own
sensitivity: the same oracle step from the state perturbed by 1e-7 relative (fp32 rounding
scale).  An outlier whose oracle self-sensitivity is of the same size is PGS chaos, not a bug.
Usage: [PGX_LIB=...] python tools/diag_parity_stats.py [env_id] [n] [steps] [lanes]"""
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
from test_gpu_parity import _state_to_oracle  # noqa: E402

env_id = sys.argv[1] if len(sys.argv) > 1 else "PandaPush-v3"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 256
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 50
lanes = int(sys.argv[4]) if len(sys.argv) > 4 else 16
venv = pg.PandaVecEnv(env_id, num_envs=n, device="cuda:0", seed=21, lanes_per_env=lanes)
venv.reset_tensors(seed=21)
ref = O.OracleVecEnv(venv._cfg, n)
ee_e, ag_e, worst = [], [], (0.0, None)
for t in range(steps):
    _state_to_oracle(venv, ref)
    saved = (ref.q.copy(), ref.qd.copy(), ref.goal.copy(), ref.obj.copy(), ref.elapsed.copy(), ref.episode.copy())
    a = venv.sample_actions(t).clone()
    venv.step_tensors(a)
    out = ref.step(a.cpu().numpy())
    if out["truncated"].any():
        continue
    ag = venv.achieved_goal.cpu().numpy()
    e_ag = np.abs(ag - out["ag"]).max(1)
    ee_e.append(np.abs(venv.obs.cpu().numpy()[:, :3] - out["obs"][:, :3]).max(1))
    ag_e.append(e_ag)
    i = int(e_ag.argmax())
    if e_ag[i] > worst[0]:
        worst = (float(e_ag[i]), (t, i, saved, a.cpu().numpy()[i:i + 1], out["ag"][i].copy()))
ee_e, ag_e = np.concatenate(ee_e), np.concatenate(ag_e)
res = {"lib": os.path.basename(os.environ.get("PGX_LIB", "libpgx.so")), "env_id": env_id,
       "ee": {p: float(np.percentile(ee_e, p)) for p in (50, 99, 99.9)} | {"max": float(ee_e.max())},
       "ag": {p: float(np.percentile(ag_e, p)) for p in (50, 99, 99.9)} | {"max": float(ag_e.max())}}
t, i, saved, a1, ag_ref = worst[1]
cfg1 = type(venv._cfg).from_buffer_copy(venv._cfg)
cfg1.n_envs = 1
sens = []
rng = np.random.default_rng(0)
for k in range(8):
    r1 = O.OracleVecEnv(cfg1, 1)
    q, qd, goal, obj, el, ep = (x[i:i + 1].copy() for x in saved)
    pert = lambda x: x * (1.0 + 1e-7 * rng.standard_normal(x.shape))  # noqa: E731
    r1.q[:], r1.qd[:], r1.goal[:], r1.obj[:] = pert(q), pert(qd), goal, obj
    r1.obj[:, :13] = pert(obj[:, :13])
    r1.elapsed[:], r1.episode[:] = el, ep
    o1 = r1.step(a1)
    sens.append(float(np.abs(o1["ag"][0] - ag_ref).max()))
res["worst"] = {"step": t, "env": i, "gpu_err": worst[0], "oracle_self_sensitivity_1e-7": sens}
print(json.dumps(res))
venv.close()
