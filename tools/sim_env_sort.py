"""Would grouping envs of similar solver effort into waves pay?  From the fp64 oracle's per-solve
sweep trace (pgxo_diag_trace: env-major within a vec step), the sum over 4-env waves of each
substep's max sweeps, in natural order and sorted by the previous step's total sweeps.
Usage: python tools/sim_env_sort.py [env_id]"""
import ctypes as C, sys, numpy as np
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle as O
from panda_gym_amd import abi, envs
from panda_gym_amd.model import load_model
n, steps = 1024, 40
env_id = sys.argv[1] if len(sys.argv) > 1 else "PandaPickAndPlace-v3"
model = abi.make_model(load_model("panda_custom0"), ee_link=11)
cfg = abi.make_config(envs.spec(env_id), n, model, abi.default_sim_params())
env = O.OracleVecEnv(cfg, n); env.reset()
lib = O.lib()
buf = np.zeros(n * 20 * 2, dtype=np.int32)
per = []
for t in range(steps):
    lib.pgxo_diag_trace(buf.ctypes.data_as(C.c_void_p), C.c_int64(buf.size))
    env.step(env.sample_actions(t))
    L = lib.pgxo_diag_trace_len()
    per.append(buf[:L].copy())
lens = {len(p) for p in per}
print("trace lens", sorted(lens)[:5])
# assume env-major: env e's substeps consecutive (collisions none in PnP)
S = []
for p in per:
    if len(p) != n * 20: S.append(None); continue
    S.append(p.reshape(n, 20))
tot_nat = tot_sort = tot_mean = 0
for t in range(1, steps):
    if S[t] is None or S[t-1] is None: continue
    s = S[t]
    nat = s.reshape(n // 4, 4, 20).max(1).sum()
    key = S[t-1].sum(1)
    order = np.argsort(key, kind="stable")
    srt = s[order].reshape(n // 4, 4, 20).max(1).sum()
    tot_nat += nat; tot_sort += srt; tot_mean += s.sum() / 4
print(env_id, "sum of wave maxima: natural", tot_nat, "sorted by prev-step sweeps", tot_sort, f"({tot_sort/tot_nat:.3f})", "ideal (mean)", tot_mean, f"({tot_mean/tot_nat:.3f})")
