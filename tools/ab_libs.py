import os, sys, json
sys.argv = [sys.argv[0], "100"]
sys.path.insert(0, os.getcwd())
import tools.time_layouts as T
T.CASES = [("PandaReach-v3", 4096, True), ("PandaReach-v3", 4096, False), ("PandaPush-v3", 4096, True)]
os.environ["PGX_LANES_PER_ENV"] = "1"
for env_id, n, c in T.CASES:
    ms = [T.run(env_id, n, c, 100) for _ in range(3)]
    print(json.dumps({"lib": os.environ.get("PGX_LIB", "new"), "env": env_id, "contacts": c, "ms": [round(x, 4) for x in ms]}), flush=True)
