#!/bin/bash
# A/B of two library builds on one box: the GPU tests named in AB_TESTS (on the second library),
# tools/ab_libs.py on AB_CASES, and tools/time_staggered.py (steady state) on STAG_CASES for each.
#   bash tools/gpu_lib_ab.sh TAG libA.so libB.so
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; A=$2; B=$3
OUT=gpurun_out/ab_$TAG
mkdir -p $OUT
if [ -n "$AB_TESTS" ]; then
  PGX_LIB=$B timeout -k 10 600 python -u -m pytest $AB_TESTS -q -m gpu --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1
  rc=$?
  grep -E "FAILED|ERROR" $OUT/pytest.log | head -20; tail -2 $OUT/pytest.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
if [ -n "$AB_CASES" ]; then
  timeout -k 10 900 python -u tools/ab_libs.py $A $B > $OUT/ab.log 2> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
  cat $OUT/ab.log
fi
for spec in $STAG_CASES; do
  IFS=: read -r env n <<< "$spec"
  for L in $A $B $A $B; do
    PGX_LIB=$L timeout -k 10 200 python tools/time_staggered.py $env $n >> $OUT/stag.log 2>&1 || { tail -5 $OUT/stag.log; exit 1; }
    echo "  ($L)" >> $OUT/stag.log
  done
done
[ -n "$STAG_CASES" ] && cat $OUT/stag.log
exit 0
