"""GPU probe for non-finite step outputs (round-5 investigation of profiles/r04/rtmodel_slp_nan.log).

    python tools/gpu_nan_probe.py abl/libA.so [abl/libB.so ...]

For every library (debug builds from `make -C panda-gym_amd/csrc dbg`, see its Makefile): the
table-drive Reach workload of tools/gpu_rtmodel_nan.py in the one-lane layout (the kernel that
produced non-finite q / obs), then a few random-policy steps of every task in both layouts.  Each
case runs in its own child process (device printf from PGX_NAN_TRAP builds lands in its stdout,
which is echoed), and prints one JSON line: the first step with a non-finite state or output and
the number of envs affected.
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import json, os, sys
import numpy as np
import torch
sys.path.insert(0, os.getcwd())
import ctypes
from panda_gym_amd import _native
_l = ctypes.CDLL(sys.argv[1])   # an older build may lack newer exports: check the ones it has
_native.EXPORTS = [x for x in _native.EXPORTS if hasattr(_l, x)]
import panda_gym_amd as pg
lib, env_id, lanes, steps, drive = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), sys.argv[5] == "1"
n = 64
kw = {"lib_path": lib}
if "rt" in os.path.basename(lib):
    kw["sim_params"] = {"friction": 0.25}
v = pg.PandaVecEnv(env_id, num_envs=n, device="cuda:0", seed=3, lanes_per_env=lanes, **kw)
v.reset_tensors(seed=3)
if drive:
    rng = np.random.default_rng(3)
    off = rng.uniform(-0.2, 0.2, (n, 3)).astype(np.float32)
    off[:, 2] = 0.0
    a = torch.as_tensor(np.clip(np.array([0.3, -0.2, -1.0], np.float32) + off, -1, 1), device="cuda:0")
res = {"lib": os.path.basename(lib), "env": env_id, "lanes": lanes, "drive": drive}
for t in range(steps):
    act = a if drive else v.sample_actions(t)
    v.step_tensors(act)
    torch.cuda.synchronize()
    st = v.state()
    bad = {k: int((~torch.isfinite(st[k])).any(dim=0).sum().item()) for k in ("q", "qd", "qc")}
    bad["obs"] = int((~torch.isfinite(v.obs)).any(dim=1).sum().item())
    if any(bad.values()):
        res["first_bad_step"] = t
        res["bad_envs"] = bad
        break
v.close()
print(json.dumps(res), flush=True)
'''

CASES = [("PandaReach-v3", 1, 3, True), ("PandaReach-v3", 1, 20, False), ("PandaReach-v3", 16, 20, False),
         ("PandaPush-v3", 16, 20, False), ("PandaPush-v3", 1, 10, False), ("PandaReachAO-v3", 16, 20, False),
         ("PandaReachAO-v3", 1, 10, False)]


def main():
    cases = CASES
    if os.environ.get("PROBE_CASES"):   # e.g. PROBE_CASES=0,0,0: case indices, repeats allowed
        cases = [CASES[int(k)] for k in os.environ["PROBE_CASES"].split(",")]
    for lib in sys.argv[1:]:
        path = os.path.abspath(lib)
        for env_id, lanes, steps, drive in cases:
            out = subprocess.run([sys.executable, "-c", CHILD, path, env_id, str(lanes), str(steps), "1" if drive else "0"],
                                 capture_output=True, text=True, cwd=ROOT, timeout=240)
            lines = [ln for ln in out.stdout.splitlines() if ln.strip()]
            traps = [ln for ln in lines if ln.startswith("PGX_NAN")]
            for ln in traps[:24]:
                print(ln)
            if out.returncode != 0:
                print(json.dumps({"lib": os.path.basename(lib), "env": env_id, "lanes": lanes, "rc": out.returncode,
                                  "stderr": out.stderr[-800:]}), flush=True)
                return out.returncode
            print(lines[-1] if lines else "{}", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
