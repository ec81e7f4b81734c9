#!/bin/bash
# PMC passes of the calibration copies (each counter group its own run).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/calib
mkdir -p $OUT
timeout -k 10 60 tools/calib/fetch_calib > $OUT/known.jsonl || exit 1
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/f -o run -- tools/calib/fetch_calib > $OUT/f.log 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/w -o run -- tools/calib/fetch_calib > $OUT/w.log 2>&1 || exit 1
cat $OUT/known.jsonl
python3 - <<'PY'
import csv, glob, collections
for tag in ("f", "w"):
    agg = collections.defaultdict(list)
    for p in glob.glob(f"gpurun_out/calib/{tag}/run_counter_collection.csv"):
        for r in csv.DictReader(open(p)):
            agg[(r["Kernel_Name"].split("(")[0][-30:], r["Counter_Name"])].append(float(r["Counter_Value"]))
    for k, v in agg.items():
        print(k, [round(x) for x in v])
PY
