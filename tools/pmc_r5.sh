#!/bin/bash
# (round 5: tools/pmc_r4.sh with the output directory as a parameter) PMC passes over a short bench run (every kernel of it: the headline step kernel, the object
# kernel of the Push / PickAndPlace legs, the ReachAO kernel, HER sample/add), one counter group
# per rocprofv3 run and never mixed with tracing (MI355X_MICROARCH.md, rocprofv3 PMC slots):
#   p1 instruction mix, p2 FETCH_SIZE, p3 WRITE_SIZE, p4 the stall split
#   (WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~ WAVE_CYCLES).
# Counters this box does not list (rocprofv3 -L) are dropped from a group before it runs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${PMC_OUT:-gpurun_out/pmc_r5}
mkdir -p $OUT
CMD="python3 bench.py --steps 30 --warmup 5 --kernel-launches 10 --no-cpu-baseline --task-steps 20 --her-calls 5"
timeout -s KILL 120 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
have() { grep -qw "$1" $OUT/counters.txt; }
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM" \
           "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA"; do
  i=$((i+1))
  sel=""
  for c in $grp; do if have $c; then sel="$sel $c"; else echo "pass $i: $c not listed, dropped"; fi; done
  [ -z "$sel" ] && continue
  timeout -s KILL 240 rocprofv3 --pmc $sel --output-format csv -d $OUT/p$i -o run -- $CMD > $OUT/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
  echo "pass $i:$sel"
done
echo pmc done
