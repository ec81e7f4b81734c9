"""Register / scratch / occupancy of the step kernels (hipcc -Rpass-analysis=kernel-resource-usage).

    python tools/regs.py [--tu 1|2] [--src panda-gym_amd/csrc/pgx_kernels.hip] [--rev GIT_REV]

--rev compiles the kernel source of a git revision instead (the headers of the work tree).
"""
import argparse
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "panda-gym_amd", "csrc")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tu", default="2")
    ap.add_argument("--src", default=os.path.join(CSRC, "pgx_kernels.hip"))
    ap.add_argument("--rev", default=None)
    ap.add_argument("--filter", default="step_kernel")
    args = ap.parse_args()
    src = args.src
    tmp = None
    if args.rev:
        txt = subprocess.run(["git", "-C", ROOT, "show", f"{args.rev}:panda-gym_amd/csrc/pgx_kernels.hip"],
                             check=True, capture_output=True, text=True).stdout
        tmp = os.path.join(CSRC, f".regs_{os.getpid()}.hip")
        with open(tmp, "w") as f:
            f.write(txt)
        src = tmp
    flags = [*os.environ.get("REGS_FLAGS", "").split(), "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-fhip-fp32-correctly-rounded-divide-sqrt",
             "-Wno-unused-function", f"-DPGX_TU={args.tu}"]
    if args.tu != "1":
        flags.append("-fno-slp-vectorize")
    try:
        with tempfile.TemporaryDirectory() as td:
            r = subprocess.run(["/opt/rocm/bin/hipcc"] + flags + ["-c", "-o", os.path.join(td, "k.o"), src,
                                                                  "-Rpass-analysis=kernel-resource-usage"],
                               capture_output=True, text=True, cwd=CSRC)
    finally:
        if tmp:
            os.unlink(tmp)
    cur, rows = None, []
    for ln in r.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", ln)
        if m:
            cur = {"name": m.group(1)}
            rows.append(cur)
            continue
        for key, pat in (("vgpr", r"VGPRs: (\d+)"), ("agpr", r"AGPRs: (\d+)"), ("scratch", r"ScratchSize \[bytes/lane\]: (\d+)"),
                         ("occ", r"Occupancy \[waves/SIMD\]: (\d+)"), ("lds", r"LDS Size \[bytes/block\]: (\d+)")):
            m = re.search(pat, ln)
            if m and cur is not None:
                cur[key] = int(m.group(1))
    if r.returncode != 0:
        sys.stderr.write(r.stderr[-3000:])
        sys.exit(1)
    for row in rows:
        if args.filter not in row["name"]:
            continue
        nm = re.sub(r"_ZN12_GLOBAL__N_1\d+", "", row["name"]).split("EEEv")[0]
        print(f"{nm:40s} vgpr {row.get('vgpr', '?'):>4} agpr {row.get('agpr', '?'):>4} scratch {row.get('scratch', '?'):>5} "
              f"occ {row.get('occ', '?')} lds {row.get('lds', '?')}")


if __name__ == "__main__":
    main()
