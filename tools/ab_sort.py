"""A/B of the heavy-first env order (PGX_SORT_ENVS unset = auto, 0 = off, 1 = forced) on the
per-pair manifold configs; three alternating child runs per mode, the median ms per step.
Usage: python tools/ab_sort.py"""
import json
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
CHILD = open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "ab_libs.py")).read().split("CHILD = r'''")[1].split("'''")[0]
CASES = [("PandaPickAndPlace-v3", 16384), ("PandaPush-v3", 4096), ("PandaPickAndPlace-v3", 32768), ("PandaReachAO-v3", 16384)]
res = {}
for rep in range(3):
    for mode in ("auto", "0", "1"):
        for env_id, n in CASES:
            env = dict(os.environ)
            env.pop("PGX_SORT_ENVS", None)
            if mode != "auto":
                env["PGX_SORT_ENVS"] = mode
            out = subprocess.run([sys.executable, "-c", CHILD, env_id, str(n), "1", "-1", "0"], capture_output=True,
                                 text=True, env=env, timeout=200)
            try:
                v = float(out.stdout.strip().split()[-1])
            except (ValueError, IndexError):
                print(env_id, n, mode, out.stderr[-300:], file=sys.stderr)
                v = float("nan")
            res.setdefault(f"{env_id}{n}-sort_{mode}", []).append(v)
            print(f"{env_id}{n}-sort_{mode} {v:.4f}", flush=True)
print(json.dumps({k: round(sorted(v)[1], 4) for k, v in res.items()}))
