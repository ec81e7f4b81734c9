#!/bin/bash
# GPU A/B of libpgx builds in abl/ (first = baseline), plus the GPU tests against the candidate.
# Usage (on the box): bash tools/ab_run.sh abl/libpgx_base.so abl/libpgx_x.so [...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "$AB_TESTS" ]; then
  PGX_LIB=$PWD/$2 timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/ab_pytest.log 2>&1 || { tail -40 gpurun_out/ab_pytest.log; exit 1; }
  tail -2 gpurun_out/ab_pytest.log
fi
timeout -k 10 500 python tools/ab_libs.py "$@" 2>&1 | tee gpurun_out/ab.log
