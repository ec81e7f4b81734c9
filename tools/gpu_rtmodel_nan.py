"""GPU bisect: which (library, layout, contacts, substeps) combination of the Reach step produces
non-finite state on the table-drive actions of test_reach_with_table_contacts.

    python tools/gpu_rtmodel_nan.py
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import panda_gym_amd as pg  # noqa: E402
from panda_gym_amd import _native  # noqa: E402


def run(lib, lanes, contacts, n_substeps, env_id="PandaReach-v3", steps=3, sp=None):
    n = 64
    rng = np.random.default_rng(3)
    off = rng.uniform(-0.2, 0.2, (n, 3)).astype(np.float32)
    off[:, 2] = 0.0
    a = torch.as_tensor(np.clip(np.array([0.3, -0.2, -1.0], np.float32) + off, -1, 1), device="cuda:0")
    kw = {"lib_path": lib} if lib else {}
    if sp is not None:
        kw["sim_params"] = sp
    v = pg.PandaVecEnv(env_id, num_envs=n, device="cuda:0", seed=3, lanes_per_env=lanes, contacts=contacts,
                       n_substeps=n_substeps, **kw)
    v.reset_tensors(seed=3)
    res = {"lib": os.path.basename(lib) if lib else "libpgx.so", "lanes": lanes, "contacts": contacts,
           "n_substeps": n_substeps, "env": env_id, "sim_params": sp}
    for t in range(steps):
        v.step_tensors(a if env_id != "PandaReachJoints-v3" else torch.zeros((n, 7), device="cuda:0"))
        st = v.state()
        bad = {k: int((~torch.isfinite(st[k])).any(dim=0).sum().item()) for k in ("q", "qd", "qc")}
        bad["obs"] = int((~torch.isfinite(v.obs)).any(dim=1).sum().item())
        if any(bad.values()):
            res["first_bad_step"] = t
            res["bad_envs"] = bad
            break
    v.close()
    return res


def main():
    pg.load_native()
    rt = os.path.join(os.path.dirname(_native.LIB_PATH), os.environ.get("RT_LIB", "libpgx_rtmodel.so"))
    from panda_gym_amd import abi

    dflt = list(abi.default_sim_params().link_friction)
    only9 = list(dflt)
    only9[9] = 0.25
    for sp in ({"link_friction": dflt}, {"link_friction": [0.25] * 16}, {"link_friction": only9}, {"friction": 0.3},
               {"link_friction": [0.25] * 16, "n_substeps": 1}):
        for lanes in (1, 16):
            for contacts in (True, False):
                spp = dict(sp)
                ns = spp.pop("n_substeps", 20)
                print(json.dumps(run(rt, lanes, contacts, ns, sp=spp)), flush=True)
    print(json.dumps(run(rt, 1, True, 20, "PandaPush-v3", sp={"link_friction": [0.25] * 16})), flush=True)


if __name__ == "__main__":
    main()
