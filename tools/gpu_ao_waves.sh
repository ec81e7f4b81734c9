#!/bin/bash
# ReachAO 8192 / Reach 4096 in steady state for two builds and both wave modes (PGX_WAVES_PER_SIMD)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/ao_waves; mkdir -p $OUT
for rep in 1 2; do
  for L in panda-gym_amd/libpgx.so ${ALT:-abl/libpgx_arm8.so}; do
    for W in ${WAVES:-0 1}; do
      PGX_LIB=$L PGX_WAVES_PER_SIMD=$W timeout -k 10 200 python tools/time_staggered.py PandaReachAO-v3 8192 >> $OUT/t.log 2>&1 || exit 1
      echo "  lib=$L waves=$W" >> $OUT/t.log
    done
    PGX_LIB=$L timeout -k 10 200 python tools/time_staggered.py PandaReach-v3 4096 >> $OUT/t.log 2>&1 || exit 1
    echo "  lib=$L" >> $OUT/t.log
  done
done
grep -v amdgpu.ids $OUT/t.log | paste - -
