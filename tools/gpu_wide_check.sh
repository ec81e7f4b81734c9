#!/bin/bash
# GPU parity suite, step-kernel times of both layouts (product library), phase profile of the
# headline config.  Each GPU step has its own time limit; stop at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/time_layouts.py 100 > gpurun_out/time_layouts.json 2>&1 || { tail gpurun_out/time_layouts.json; exit 1; }
grep env_id gpurun_out/time_layouts.json
PGX_LIB=$PWD/panda-gym_amd/libpgx_prof.so timeout -k 10 300 python tools/prof_phases.py PandaReach-v3 4096 1 > gpurun_out/phases_wide.json 2>&1 || { tail gpurun_out/phases_wide.json; exit 1; }
grep env_id gpurun_out/phases_wide.json
