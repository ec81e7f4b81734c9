"""Summarise rocprofv3 PMC passes (tools/profile_pmc.sh) for the step kernel into profiles/.

Writes profiles/pmc_step_kernel.json (read by bench.py for roofline.traffic and
roofline_valu) and copies the per-pass CSVs under profiles/<round>/pmc/.

Units: FETCH_SIZE / WRITE_SIZE are KB per dispatch (TCC_EA0_RDREQ/WRREQ based).
MI355X_MICROARCH.md §HBM: FETCH_SIZE reads 1/2 of the bytes of 16-B-per-lane streaming
loads on gfx950 and other widths are uncalibrated there.  tools/calib (profiles/r02/calib)
calibrates the widths and the pattern of the step kernel: dword, dwordx2 and 16-B streaming
copies of 512 MiB and the step kernel's SoA pattern (4 envs per wave, one dword per row from
the lead lane, XCD block mapping, 40 rows x 4096 envs, repeated launches) all report FETCH_SIZE
= 1/2 of the bytes read and WRITE_SIZE = the bytes written, so `fetch_correction` = 2.
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(src=os.path.join(ROOT, "gpurun_out", "pmc"), round_tag="r01", num_envs=4096, kernel="step_kernel<0, 0, 1, 0, 1>"):
    agg = defaultdict(list)
    for p in sorted(glob.glob(os.path.join(src, "p*", "run_counter_collection.csv"))):
        for r in csv.DictReader(open(p)):
            if kernel in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    mean = {k: sum(v) / len(v) for k, v in agg.items()}
    waves = mean.get("SQ_WAVES", 0.0)
    out = {
        "kernel": kernel, "num_envs": num_envs, "dispatches": {k: len(v) for k, v in agg.items()},
        "counters_mean_per_dispatch": mean,
        "valu_instr_per_launch": mean.get("SQ_INSTS_VALU"),
        "valu_lane_ops_per_launch": mean.get("SQ_INSTS_VALU", 0.0) * 64,
        "valu_instr_per_env_step": mean.get("SQ_INSTS_VALU", 0.0) * 64 / num_envs,
        "salu_instr_per_wave": mean.get("SQ_INSTS_SALU", 0.0) / waves if waves else None,
        "fetch_kb": mean.get("FETCH_SIZE"), "write_kb": mean.get("WRITE_SIZE"), "fetch_correction": 2.0,
        "fetch_correction_source": "profiles/r02/calib (tools/calib/run.sh)",
        "hbm_bytes_per_launch": (2.0 * mean.get("FETCH_SIZE", 0.0) + mean.get("WRITE_SIZE", 0.0)) * 1024.0,
        "read_bytes_per_launch": 2.0 * mean.get("FETCH_SIZE", 0.0) * 1024.0,
        "write_bytes_per_launch": mean.get("WRITE_SIZE", 0.0) * 1024.0,
        "alg_bytes_per_launch": 199.0 * num_envs,
        "source": "tools/profile_pmc.sh (rocprofv3 --pmc, one counter group per run) on MI355X",
    }
    dst = os.path.join(ROOT, "profiles", round_tag, "pmc")
    os.makedirs(dst, exist_ok=True)
    for p in glob.glob(os.path.join(src, "p*", "run_counter_collection.csv")):
        shutil.copy(p, os.path.join(dst, os.path.basename(os.path.dirname(p)) + "_counter_collection.csv"))
    with open(os.path.join(ROOT, "profiles", "pmc_step_kernel.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: out[k] for k in ("valu_instr_per_env_step", "hbm_bytes_per_launch", "alg_bytes_per_launch")}))


if __name__ == "__main__":
    main(*sys.argv[1:3])
