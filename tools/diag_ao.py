"""Diagnostics for ReachAO obs parity: worst unit-vector / distance entries, device vs oracle."""
import sys

import numpy as np

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import panda_gym_amd as pg  # noqa: E402
from oracle import oracle as O  # noqa: E402

pg.load_native()
n = 64
venv = pg.PandaVecEnv("PandaReachAO-v3", num_envs=n, device="cuda:0", seed=3)
venv.reset_tensors(seed=100)
spec = pg.spec("PandaReachAO-v3")
dr = [pg.seeded_reset(spec, 100 + i) for i in range(n)]
ref = O.OracleVecEnv(venv._cfg, n)
out = ref.reset(inject_goal=np.array([d[0] for d in dr]), inject_obj=np.array([d[1] for d in dr]))
obs = venv.obs.cpu().numpy()
e = np.abs(obs - out["obs"])
u = e[:, 29:56].reshape(n, 9, 3).max(2)
for idx in np.argsort(u.ravel())[::-1][:6]:
    env, l = divmod(idx, 9)
    dist, pa, pb, _ = O.ao_link_distances(venv._cfg, ref.q[env], ref.obstacles[env])
    print(f"env {env} link {l} err {u[env, l]:.3g} d_gpu {obs[env, 20 + l]:.7g} d_ref {out['obs'][env, 20 + l]:.7g}")
    print("   u_gpu", obs[env, 29 + 3 * l:32 + 3 * l], "u_ref", out["obs"][env, 29 + 3 * l:32 + 3 * l])
    print("   pa", pa[l], "pb", pb[l])
    d = np.linalg.norm(ref.obstacles[env] - pb[l], axis=1)
    print("   obstacle nearest pb:", int(np.argmin(d)), ref.obstacles[env][int(np.argmin(d))])
