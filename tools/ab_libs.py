"""A/B the step kernel of two builds of libpgx on one box (box-to-box clock variance is a few %):
alternates the libraries in child processes and prints the median ms per config.
Usage: python tools/ab_libs.py libA.so libB.so"""
import json
import os
import subprocess
import sys

# (env id, envs, contacts, full manifold: -1 = the library's default, waves per SIMD: 0 = auto)
CASES = [("PandaReach-v3", 4096, 1, -1, 0), ("PandaPush-v3", 4096, 1, -1, 0), ("PandaReachAO-v3", 8192, 1, -1, 0),
         ("PandaReach-v3", 4096, 0, -1, 0), ("PandaReach-v3", 8192, 1, -1, 0), ("PandaReach-v3", 16384, 1, -1, 0)]
CHILD = r'''
import os, sys, json, torch
sys.path.insert(0, os.getcwd())
import ctypes
from panda_gym_amd import _native
lib = ctypes.CDLL(_native.LIB_PATH)   # an older build may lack newer exports: check the ones it has
_native.EXPORTS = [e for e in _native.EXPORTS if hasattr(lib, e)]
import panda_gym_amd as pg
env_id, n, contacts, full = sys.argv[1], int(sys.argv[2]), bool(int(sys.argv[3])), int(sys.argv[4])
if sys.argv[5] != "0":
    os.environ["PGX_WAVES_PER_SIMD"] = sys.argv[5]   # 1 / 2: force the one- / two-wave build
kw = json.loads(os.environ.get("AB_KW", "{}"))   # e.g. AB_KW='{"lanes_per_env": 16}'
if full >= 0:
    kw["full_manifold"] = bool(full)
venv = pg.PandaVecEnv(env_id, num_envs=n, device="cuda:0", seed=0, contacts=contacts, **kw)
stagger = os.environ.get("AB_STAGGER") == "1"   # steady state: staggered episode phases, one episode of warmup
venv.reset_tensors(episode_phase="staggered" if stagger else None)
warm = 60 if stagger else 30
for t in range(warm):
    venv.step_tensors(venv.sample_actions(t))
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
torch.cuda.synchronize(); e0.record()
for t in range(100):
    venv.step_tensors(venv.sample_actions(warm + t))
e1.record(); torch.cuda.synchronize()
print(e0.elapsed_time(e1) / 100)
'''

if __name__ == "__main__":
    libs = sys.argv[1:]
    if os.environ.get("AB_CASES"):   # e.g. AB_CASES="PandaReach-v3:4096:1,PandaPush-v3:4096:1"
        # e.g. AB_CASES="PandaReach-v3:4096:1:0,PandaPush-v3:4096:1:1" (env:envs:contacts[:full[:waves]])
        CASES = [(f[0], int(f[1]), int(f[2]), int(f[3]) if len(f) > 3 else -1, int(f[4]) if len(f) > 4 else 0)
                 for f in (x.split(":") for x in os.environ["AB_CASES"].split(","))]

    def key(env_id, n, contacts, full, waves):
        return (env_id + str(n) + ("" if contacts else "-free") + {-1: "", 0: "-4pt", 1: "-full"}[full]
                + ("" if not waves else f"-w{waves}"))

    res = {lib: {key(*c): [] for c in CASES} for lib in libs}
    for rep in range(3):
        for lib in libs:
            for c in CASES:
                out = subprocess.run([sys.executable, "-c", CHILD] + [str(x) for x in c],
                                     capture_output=True, text=True,
                                     env={**os.environ, "PGX_LIB": os.path.abspath(lib)}, timeout=120)
                try:
                    res[lib][key(*c)].append(float(out.stdout.strip().split()[-1]))
                except (ValueError, IndexError):
                    print(f"{lib} {c}: {out.stderr[-400:]}", file=sys.stderr)
                    res[lib][key(*c)].append(float("nan"))
    for lib in libs:
        print(json.dumps({"lib": os.path.basename(lib), **{k: round(sorted(v)[1], 4) for k, v in res[lib].items()}}),
              flush=True)
