import time, numpy as np, torch, sys, os
sys.path.insert(0, os.getcwd())
import panda_gym_amd as pg
venv = pg.PandaVecEnv("PandaReach-v3", num_envs=4096, device="cuda:0", seed=0)
venv.reset()
a = np.zeros((4096, 3), np.float32)
for _ in range(20): venv.step(a)
T = {}
def tick(k, t0):
    T[k] = T.get(k, 0.0) + time.perf_counter() - t0
for _ in range(100):
    t0 = time.perf_counter(); venv.step_async(a); tick("step_async", t0)
    t0 = time.perf_counter(); out = venv.step_tensors(venv._pending); venv._pending = None; tick("step_tensors(launch)", t0)
    hs = venv._host_stage(); st = torch.cuda.current_stream()
    t0 = time.perf_counter(); hs["packed"].copy_(venv._outbuf, non_blocking=True); hs["errors"].copy_(hs["errors_dev"], non_blocking=True); tick("copy launch", t0)
    t0 = time.perf_counter(); st.synchronize(); tick("sync(kernel+copy)", t0)
    t0 = time.perf_counter(); hs["errors"].item(); o = {k: hs[k].numpy().copy() for k in ("observation", "achieved_goal", "desired_goal")}; r = hs["reward"].numpy().copy(); fl = hs["flags"].numpy() != 0; tick("numpy copies", t0)
    t0 = time.perf_counter(); infos = [{"is_success": s, "is_truncated": c} for s, c in zip(fl[0].tolist(), fl[3].tolist())]; tick("infos", t0)
t0 = time.perf_counter()
for _ in range(100): venv.step(a)
T["full step"] = time.perf_counter() - t0
print({k: round(v * 10, 4) for k, v in T.items()}, "ms per step")
