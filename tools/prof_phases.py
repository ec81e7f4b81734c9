"""Phase breakdown of the step kernel (s_memtime per wave, libpgx_prof.so = make -C
panda-gym_amd/csrc prof).  Prints mean cycles per wave per env step by phase and the
PGS sweeps per substep the waves ran.
Usage: PGX_LIB=abl/libpgx_prof.so python tools/prof_phases.py [env_id] [n] [contacts]"""
import ctypes as C
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import panda_gym_amd as pg  # noqa: E402
from panda_gym_amd import _native  # noqa: E402

NAMES = ["prologue+IK", "FK+detect", "dynamics", "row setup", "PGS sweeps", "integrate", "epilogue"]


def run(env_id, n, contacts, launches=100, warm=26):
    lib = _native.load()
    buf = (C.c_ulonglong * 24)()
    kw = json.loads(os.environ.get("PH_KW", "{}"))   # e.g. PH_KW='{"full_manifold": true}'
    venv = pg.PandaVecEnv(env_id, num_envs=n, device="cuda:0", seed=0, contacts=contacts, **kw)
    if os.environ.get("PH_STAGGER"):   # the bench's steady state: staggered episode phases, one episode in
        venv.reset_tensors(episode_phase="staggered")
        warm = max(warm, venv.spec.max_episode_steps + 5)
    else:
        venv.reset_tensors()
    for t in range(warm):
        venv.step_tensors(venv.sample_actions(t))
    torch.cuda.synchronize()
    lib.pgx_prof_read(buf, 1)
    acts = [venv.sample_actions(warm + t).clone() for t in range(launches)]
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for a in acts:
        venv.step_tensors(a)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / launches
    lib.pgx_prof_read(buf, 1)
    # libpgx's default rule (pgx_api.cpp): 16 lanes with contacts at any batch, else up to 8192 envs
    wide = venv._cfg.lanes_per_env == 16 or (venv._cfg.lanes_per_env == 0 and (n <= 8192 or contacts))
    waves = n // (4 if wide else 64)
    wv = (C.c_ulonglong * (10 * waves))()
    lib.pgx_prof_wave_read(wv, waves)
    import numpy as np
    w = np.frombuffer(wv, dtype=np.uint64).reshape(waves, 10).astype(np.int64)
    dur = w[:, 1] - w[:, 0]
    start = w[:, 0] - w[:, 0].min()
    end = w[:, 1] - w[:, 0].min()
    top = np.argsort(dur)[-max(waves // 100, 1):]
    wave_stats = {"waves": waves, "dur_mean": float(dur.mean()), "dur_p50": float(np.median(dur)),
                  "dur_p99": float(np.percentile(dur, 99)), "dur_max": float(dur.max()),
                  "start_max": float(start.max()), "end_max": float(end.max()),
                  "sweeps_mean": float(w[:, 2].mean()), "sweeps_top1pct": float(w[top, 2].mean()),
                  "nonfar_mean": float(w[:, 3].mean()), "nonfar_top1pct": float(w[top, 3].mean()),
                  "redo_mean": float(w[:, 4].mean()), "redo_top1pct": float(w[top, 4].mean()),
                  "allrows_mean": float(w[:, 5].mean()), "allrows_top1pct": float(w[top, 5].mean()),
                  "partial_mean": float(w[:, 6].mean()), "partial_top1pct": float(w[top, 6].mean()),
                  "pgs_cyc_mean": float(w[:, 7].mean()), "pgs_cyc_top1pct": float(w[top, 7].mean()),
                  "detect_cyc_mean": float(w[:, 8].mean()), "detect_cyc_top1pct": float(w[top, 8].mean()),
                  "epilogue_cyc_mean": float(w[:, 9].mean()), "epilogue_cyc_top1pct": float(w[top, 9].mean())}
    per = [buf[k] / (waves * launches) for k in range(24)]
    tot = sum(per[:7]) + per[14] + per[15] + sum(per[19:24])
    out = {"lib": os.path.basename(_native.LIB_PATH), "staggered": bool(os.environ.get("PH_STAGGER")),
           "env_id": env_id, "n": n, "contacts": contacts, "ms_per_step": ms,
           "cycles_per_wave_step": tot, "clock_ghz_est": tot / (ms * 1e6),
           "phases": {NAMES[k]: round(per[k]) for k in range(7)},
           "share": {NAMES[k]: round(per[k] / tot, 3) for k in range(7)},
           "sweeps_per_substep": per[8] / max(per[9], 1e-9), "nonfar_frac": per[10] / max(per[9], 1e-9),
           "contact_substep_frac": per[11] / max(per[9], 1e-9),
           "speculation_redo_frac": per[12] / max(per[9], 1e-9), "partial_frac": per[7] / max(per[9], 1e-9),
           "partial_k2_frac": per[16] / max(per[7], 1e-9), "partial_contact_frac": per[18] / max(per[7], 1e-9), "all_rows_frac": per[13] / max(per[9], 1e-9),
           "cycles_per_sweep": per[4] / max(per[8], 1e-9), "last_launch_waves": wave_stats,
           "ik_iterations_per_wave_step": per[17],
           "detect_split": {"g0_vertices": round(per[19]), "fk": round(per[20]), "robot_contacts": round(per[21])},
           "row_setup_split": {"contact_points": round(per[22]), "delassus_lanes": round(per[23]),
                               "joint_rows": round(per[3])},
           "dynamics_split": {"newton_euler": round(per[14]), "crba_cholesky": round(per[15]),
                              "minv_and_rest": round(per[2])}}
    venv.close()
    return out


if __name__ == "__main__":
    cases = [("PandaReach-v3", 4096, True), ("PandaReach-v3", 4096, False), ("PandaPush-v3", 4096, True),
             ("PandaPickAndPlace-v3", 16384, True), ("PandaReachAO-v3", 8192, True)]
    if len(sys.argv) > 1:
        cases = [(sys.argv[1], int(sys.argv[2]), bool(int(sys.argv[3])))]
    for c in cases:
        print(json.dumps(run(*c)), flush=True)
