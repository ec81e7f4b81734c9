import os, subprocess, sys, json
CHILD = open('/root/repo/tools/ab_libs.py').read().split("CHILD = r'''")[1].split("'''")[0]
res = {}
for rep in range(3):
    for mode in ("0", "1", "2"):
        for case in (("PandaReachAO-v3", 8192, 1), ("PandaReach-v3", 8192, 1), ("PandaPickAndPlace-v3", 16384, 1)):
            out = subprocess.run([sys.executable, "-c", CHILD, case[0], str(case[1]), str(case[2])], capture_output=True, text=True,
                                 env={**os.environ, "PGX_WAVES_PER_SIMD": mode}, timeout=200)
            res.setdefault((mode,) + case, []).append(float(out.stdout.strip().split()[-1]))
for k, v in sorted(res.items()):
    print(k, round(sorted(v)[1], 4))
