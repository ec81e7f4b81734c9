"""A/B of the heavy-first order's key: robot points past the register budget (PGX_SORT_KEY=0, the
default: most envs stay in one bin, in their original order) against all robot points (1); three
alternating child runs, the median ms per step.  Usage: python tools/ab_sort3.py"""
import json
import os
import subprocess
import sys

CHILD = open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "ab_libs.py")).read().split("CHILD = r'''")[1].split("'''")[0]
CASES = [("PandaPickAndPlace-v3", 16384), ("PandaPickAndPlace-v3", 32768), ("PandaReachAO-v3", 16384)]
res = {}
for rep in range(3):
    for key in ("0", "1"):
        for env_id, n in CASES:
            env = dict(os.environ)
            env.pop("PGX_SORT_ENVS", None)
            env["PGX_SORT_KEY"] = key
            out = subprocess.run([sys.executable, "-c", CHILD, env_id, str(n), "1", "-1", "0"], capture_output=True,
                                 text=True, env=env, timeout=200)
            try:
                v = float(out.stdout.strip().split()[-1])
            except (ValueError, IndexError):
                print(env_id, n, key, out.stderr[-300:], file=sys.stderr)
                v = float("nan")
            res.setdefault(f"{env_id}{n}-key{key}", []).append(v)
            print(f"{env_id}{n}-key{key} {v:.4f}", flush=True)
print(json.dumps({k: round(sorted(v)[1], 4) for k, v in res.items()}))
