"""Diagnostic: GPU vs oracle error growth along a free-running trajectory (not a test)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import panda_gym_amd as pg
from oracle import oracle as O

n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
env_id = sys.argv[2] if len(sys.argv) > 2 else "PandaReach-v3"
venv = pg.PandaVecEnv(env_id, num_envs=n, device="cuda:0", seed=11)
venv.reset_tensors()
ref = O.OracleVecEnv(venv._cfg, n)
st = venv.state()
ref.q[:] = st["q"].double().cpu().numpy().T; ref.qd[:] = st["qd"].double().cpu().numpy().T
ref.qc[:] = st["qc"].double().cpu().numpy().T
ref.goal[:] = st["goal"].cpu().numpy().T
for t in range(50):
    a = venv.sample_actions(t).clone()
    venv.step_tensors(a)
    out = ref.step(a.cpu().numpy())
    o = venv.obs.cpu().numpy()
    e = np.abs(o - out["obs"])
    ep, ev = e[:, :3].max(1), e[:, 3:].max(1)
    st = venv.state()
    eq = np.abs(st["q"].double().cpu().numpy().T - ref.q).max(1)
    print(f"t={t:2d} pos max {ep.max():.2e} p99 {np.percentile(ep,99):.2e} med {np.median(ep):.2e} | "
          f"vel max {ev.max():.2e} p99 {np.percentile(ev,99):.2e} med {np.median(ev):.2e} | q max {eq.max():.2e} worst env {int(np.argmax(ev))}")
