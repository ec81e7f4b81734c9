#!/bin/bash
# GPU tests (current tree) + A/B timing of library builds + phase profile of a prof build.
# Usage: AB="abl/a.so abl/b.so" AB_CASES=... PH_LIB=abl/libpgx_prof_x.so PH_CASE="PandaReachAO-v3 8192 1" bash tools/gpu_ab.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-ab}
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { tail -60 gpurun_out/pytest_$TAG.log; exit 1; }
  tail -2 gpurun_out/pytest_$TAG.log
fi
if [ -n "$AB" ]; then
  timeout -k 10 600 python tools/ab_libs.py $AB > gpurun_out/ab_$TAG.log 2>&1 || { tail -20 gpurun_out/ab_$TAG.log; exit 1; }
  cat gpurun_out/ab_$TAG.log
fi
if [ -n "$PH_LIB" ]; then
  PGX_LIB=$PH_LIB timeout -k 10 300 python3 tools/prof_phases.py $PH_CASE > gpurun_out/ph_$TAG.log 2>&1 || { tail -20 gpurun_out/ph_$TAG.log; exit 1; }
  tail -1 gpurun_out/ph_$TAG.log | cut -c1-600
fi
