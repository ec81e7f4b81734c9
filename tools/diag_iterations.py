"""Per-substep PGS sweep counts, contact points and IK iterations of the fp64 oracle on
the bench workload (random policy, auto-reset), grouped per 64-env wave the way the HIP
kernel runs them: the wave's cost is set by its slowest lane.
Usage: python tools/diag_iterations.py [task] [n_envs] [steps]"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402
from panda_gym_amd import abi  # noqa: E402
from panda_gym_amd.model import load_model  # noqa: E402

task = {"reach": abi.TASK_REACH, "push": abi.TASK_PUSH, "pnp": abi.TASK_PICK_AND_PLACE}[sys.argv[1] if len(sys.argv) > 1 else "reach"]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 256
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 60
model = abi.make_model(load_model("panda_custom0"), ee_link=11)
params = abi.default_sim_params()
cfg = abi.make_config(abi.EnvSpec(task=task), n, model, params, contacts=True)
env = O.OracleVecEnv(cfg, n)
env.reset()
lib = O.lib()
h = (C.c_int64 * 128)()
lib.pgxo_diag_read(h, 1)
sweeps = np.zeros(64)
cons = np.zeros(16)
ik = np.zeros(32)
for t in range(steps):
    env.step(env.sample_actions(t))
    lib.pgxo_diag_read(h, 1)
    a = np.array(h[:])
    sweeps += a[:64]; cons += a[64:80]; ik += a[80:112]
    lim = a[112:115] + (lim if t else 0)
tot = sweeps.sum()
mean = (sweeps * np.arange(64)).sum() / tot
print(f"substeps {int(tot)}: mean PGS sweeps {mean:.1f}; share at 50: {sweeps[50] / tot:.2f}")
print("sweep histogram (count>0):", {i: int(c) for i, c in enumerate(sweeps) if c})
print("contact points per substep:", {i: int(c) for i, c in enumerate(cons) if c})
print(f"IK iterations mean {(ik * np.arange(32)).sum() / ik.sum():.1f}:", {i: int(c) for i, c in enumerate(ik) if c})
print(f"substeps with a joint-limit impulse {lim[0] / tot:.4f}, with robot contacts {lim[1] / tot:.3f}, both {lim[2] / tot:.4f}")
