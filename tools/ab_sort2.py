"""A/B of the heavy-first env order on ReachAO 8192 (two resident waves per SIMD: all 2048 waves fit)
and with the one-wave build (PGX_WAVES_PER_SIMD=1: two rounds of 1024); three alternating child runs,
the median ms per step.  Usage: python tools/ab_sort2.py"""
import json
import os
import subprocess
import sys

CHILD = open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "ab_libs.py")).read().split("CHILD = r'''")[1].split("'''")[0]
# (label, env id, envs, waves per SIMD (0 auto), PGX_SORT_ENVS (None: auto))
CASES = [("ao8192-auto", "PandaReachAO-v3", 8192, 0, None), ("ao8192-sort", "PandaReachAO-v3", 8192, 0, "1"),
         ("ao8192-w1", "PandaReachAO-v3", 8192, 1, "0"), ("ao8192-w1-sort", "PandaReachAO-v3", 8192, 1, "1"),
         ("pnp16384-auto", "PandaPickAndPlace-v3", 16384, 0, None)]
res = {}
for rep in range(3):
    for label, env_id, n, waves, sort in CASES:
        env = dict(os.environ)
        env.pop("PGX_SORT_ENVS", None)
        if sort is not None:
            env["PGX_SORT_ENVS"] = sort
        out = subprocess.run([sys.executable, "-c", CHILD, env_id, str(n), "1", "-1", str(waves)], capture_output=True,
                             text=True, env=env, timeout=200)
        try:
            v = float(out.stdout.strip().split()[-1])
        except (ValueError, IndexError):
            print(label, out.stderr[-300:], file=sys.stderr)
            v = float("nan")
        res.setdefault(label, []).append(v)
        print(f"{label} {v:.4f}", flush=True)
print(json.dumps({k: round(sorted(v)[1], 4) for k, v in res.items()}))
