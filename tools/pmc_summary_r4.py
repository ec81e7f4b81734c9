"""Summarise the PMC passes of tools/pmc_r3.sh per kernel into profiles/pmc_*.json (read by bench.py).
Round 4: the per-pair manifold kernels (WIDE = 2) are the default; algorithmic bytes from
bench.alg_bytes_per_env_step (the state a step carries).

    python tools/pmc_summary_r4.py [gpurun_out/pmc_r4] [r04]

Kernels (told apart by name and grid size, the bench's legs): the headline step kernel (Reach
4096, table), the object kernel at Push 4096 and at PickAndPlace 16384, the ReachAO kernel at
8192, and the HER sample kernel.  HBM bytes = 2 x FETCH_SIZE + WRITE_SIZE (KB per dispatch):
FETCH_SIZE reports half the bytes read on gfx950 (MI355X_MICROARCH.md; calibrated for these
kernels' access pattern in profiles/r02/calib).  The stall split (pass 4): SQ_WAVE_CYCLES ~
SQ_WAIT_ANY + SQ_WAIT_INST_ANY + SQ_ACTIVE_INST_ANY (quad-cycles).
"""
import csv
import glob
import gzip
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

# (json name, kernel-name fragment, grid threads, envs, algorithmic bytes per launch or None)
HER_B, HER_RATIO = 1 << 20, 0.8


def her_alg():
    from bench import HER_AD, HER_OD, her_alg_bytes

    row_dim = 2 * HER_OD + HER_AD + 14
    row_stride = (row_dim + 3) // 4 * 4
    return her_alg_bytes(HER_B, int(HER_RATIO * HER_B), row_dim, row_stride)


def _alg(task, obs_dim, action_dim, points, envs):
    from bench import alg_bytes_per_env_step

    return alg_bytes_per_env_step(task, obs_dim, action_dim, points)["total"] * envs


KERNELS = [   # (name, kernel-name fragment (any step_kernel / step_kernel_o2 build), grid threads, envs, alg bytes)
    ("pmc_step_kernel", "0, 0, 1, 0, 2>", 4096 * 16, 4096, _alg("reach_table", 6, 3, 8, 4096)),
    ("pmc_object_kernel_push", "0, 1, 1, 0, 2>", 4096 * 16, 4096, _alg("push", 18, 3, 12, 4096)),
    ("pmc_object_kernel_pnp", "0, 1, 1, 0, 2>", 16384 * 16, 16384, _alg("pick_and_place", 19, 4, 12, 16384)),
    ("pmc_reach_ao_kernel", "1, 0, 1, 1, 2>", 8192 * 16, 8192, _alg("reach_ao", 56, 7, 8, 8192)),
    ("pmc_sample_kernel", "sample_kernel", None, None, None),
]


ROBOT_POINTS = {"pmc_step_kernel": 8, "pmc_object_kernel_push": 12, "pmc_object_kernel_pnp": 12,
                "pmc_reach_ao_kernel": 8}   # the per-pair manifold budgets (include/pgx.h)


# the pass script of each round's profiles (round 6 reran round 5's, tools/gpu_r6.sh PMC=1)
PASS_SCRIPT = "pmc_r5.sh"


def main(src=os.path.join(ROOT, "gpurun_out", "pmc_r4"), round_tag="r04"):
    rows = []
    for p in sorted(glob.glob(os.path.join(src, "p*", "run_counter_collection.csv"))):
        rows += list(csv.DictReader(open(p)))
    dst = os.path.join(ROOT, "profiles", round_tag, "pmc")
    os.makedirs(dst, exist_ok=True)
    for p in glob.glob(os.path.join(src, "p*", "run_counter_collection.csv")):   # kept gzipped
        with open(p, "rb") as fi, gzip.open(os.path.join(dst, os.path.basename(os.path.dirname(p)) +
                                                "_counter_collection.csv.gz"), "wb") as fo:
            shutil.copyfileobj(fi, fo)
    for name, frag, grid, envs, alg in KERNELS:
        agg = defaultdict(list)
        for r in rows:
            if frag not in r["Kernel_Name"]:
                continue
            if grid is not None and int(r["Grid_Size"]) != grid:
                continue
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
        if not agg:
            print(name, "no dispatches")
            continue
        mean = {k: sum(v) / len(v) for k, v in agg.items()}
        if name == "pmc_sample_kernel":
            alg = her_alg()
        hbm = (2.0 * mean.get("FETCH_SIZE", 0.0) + mean.get("WRITE_SIZE", 0.0)) * 1024.0
        waves = mean.get("SQ_WAVES") or 0.0
        # "void (anonymous namespace)::step_kernel<0, 0, 1, 0, 2>(PgxDevModel const*, ...)" -> the template id
        names = sorted({r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
                        for r in rows if frag in r["Kernel_Name"] and (grid is None or int(r["Grid_Size"]) == grid)})
        out = {
            "kernel": frag, "kernel_names": names, "num_envs": envs, "grid_threads": grid,
            "robot_points": ROBOT_POINTS.get(name),
            "dispatches": {k: len(v) for k, v in agg.items()}, "counters_mean_per_dispatch": mean,
            "fetch_kb": mean.get("FETCH_SIZE"), "write_kb": mean.get("WRITE_SIZE"), "fetch_correction": 2.0,
            "fetch_correction_source": "profiles/r02/calib (tools/calib/run.sh); MI355X_MICROARCH.md HBM section",
            "hbm_bytes_per_launch": hbm, "read_bytes_per_launch": 2.0 * mean.get("FETCH_SIZE", 0.0) * 1024.0,
            "write_bytes_per_launch": mean.get("WRITE_SIZE", 0.0) * 1024.0, "alg_bytes_per_launch": alg,
            "traffic_over_alg": hbm / alg if alg else None,
            "source": f"tools/{PASS_SCRIPT} + tools/pmc_summary_r4.py (rocprofv3 --pmc, one group "
                      f"per run), profiles/{round_tag}/pmc",
        }
        if "SQ_INSTS_VALU" in mean:
            out["valu_instr_per_launch"] = mean["SQ_INSTS_VALU"]
            out["valu_lane_ops_per_launch"] = mean["SQ_INSTS_VALU"] * 64
            if envs:
                out["valu_instr_per_env_step"] = mean["SQ_INSTS_VALU"] * 64 / envs
            if waves:
                out["valu_instr_per_wave"] = mean["SQ_INSTS_VALU"] / waves
        wc = mean.get("SQ_WAVE_CYCLES")
        if wc and "SQ_WAIT_ANY" in mean:
            out["stall_split"] = {k: mean.get(k, 0.0) / wc for k in
                                  ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                                   "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_SCA")}
            if waves and "SQ_INSTS_VALU" in mean:
                # quad-cycles per wave / VALU instructions per wave = cycles per VALU / 4
                out["cycles_per_valu_instr"] = 4.0 * wc / mean["SQ_INSTS_VALU"]
        with open(os.path.join(ROOT, "profiles", name + ".json"), "w") as f:
            json.dump(out, f, indent=1)
        print(name, json.dumps({k: out.get(k) for k in ("hbm_bytes_per_launch", "alg_bytes_per_launch",
                                                        "traffic_over_alg", "valu_instr_per_wave",
                                                        "cycles_per_valu_instr")}),
              json.dumps(out.get("stall_split")))


if __name__ == "__main__":
    main(*sys.argv[1:3])
