"""Per env and step, the device-vs-oracle deviation of the side-wall / edge scenario of
tests/test_gpu_contacts.py::test_cube_at_the_table_side_wall_and_edge, with the contact ids each
side kept after the step (the object-scene slots: vertex v against the table box is id v, against
the plane 8 + v) for the steps above --thr.

    python tools/gpu_wall_diag.py [--lanes 16] [--thr 5e-5]
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
from test_gpu_parity import _state_to_oracle  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lanes", type=int, default=16)
    ap.add_argument("--thr", type=float, default=5e-5)
    args = ap.parse_args()
    n = 16
    venv = pg.PandaVecEnv("PandaPush-v3", num_envs=n, device="cuda:0", seed=4, lanes_per_env=args.lanes)
    venv.reset_tensors()
    rng = np.random.default_rng(5)
    st = venv.state()
    obj = np.zeros((13, n), np.float32)
    for i in range(n):
        yaw = rng.uniform(-0.3, 0.3)
        obj[3:7, i] = (0.0, 0.0, np.sin(yaw / 2), np.cos(yaw / 2))
        if i < 8:
            obj[0:3, i] = (0.25 + 0.035 + 0.02 * rng.random(), rng.uniform(-0.2, 0.2), -0.38)
            obj[7:10, i] = (-0.6, 0.0, 0.0)
        else:
            obj[0:3, i] = (0.2 + 0.02 * rng.random(), rng.uniform(-0.2, 0.2), 0.02)
            obj[7:10, i] = (0.8, 0.0, 0.0)
    st["object"].copy_(torch.as_tensor(obj, device="cuda:0"))
    st["contacts"][0::2] = -1.0
    st["contacts"][1::2] = 0.0
    if "manifolds" in st:
        st["manifolds"].zero_()
    ref = O.OracleVecEnv(venv._cfg, n)
    zero = torch.zeros((n, 3), dtype=torch.float32, device="cuda:0")
    for t in range(25):
        _state_to_oracle(venv, ref)
        pre = ref.obj[:, :13].copy()
        venv.step_tensors(zero)
        ref.step(zero.cpu().numpy())
        s2 = venv.state()
        ob = s2["object"].cpu().numpy()
        dev_ids = s2["contacts"].cpu().numpy()[0:2 * O.OBJECT_POINTS:2].T
        ora_ids = ref.obj[:, O.OBJ_CACHE:O.OBJ_CACHE1:2]
        err = np.abs(ob[0:3].T - ref.obj[:, 0:3]).max(axis=1)
        for i in np.flatnonzero(err > args.thr):
            print(f"t {t} env {i} err {err[i]:.2e} pre pos {np.round(pre[i, :3], 5)} vel {np.round(pre[i, 7:10], 3)} "
                  f"w {np.round(pre[i, 10:13], 2)} | ids dev {dev_ids[i].tolist()} oracle {ora_ids[i].tolist()} | "
                  f"dev pos {ob[0:3, i]} oracle {ref.obj[i, 0:3]}", flush=True)


if __name__ == "__main__":
    main()
