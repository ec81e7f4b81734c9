#!/bin/bash
# PMC passes for the step kernel (each counter group in its own run, --kernel-trace/--stats not mixed in).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc
mkdir -p $OUT
CMD="python3 bench.py --steps 30 --warmup 5 --kernel-launches 10 --no-cpu-baseline"
timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES" "FETCH_SIZE" "WRITE_SIZE" "SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_SMEM SQ_INSTS_VMEM"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- $CMD > $OUT/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
echo pmc done
