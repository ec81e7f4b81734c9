#!/bin/bash
# Phase profile (libpgx_prof.so) of the step kernels, then the PMC passes of the headline kernel.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
PGX_LIB=panda-gym_amd/libpgx_prof.so timeout -k 10 300 python3 tools/prof_phases.py > gpurun_out/phases.jsonl 2> gpurun_out/phases.err || { tail -20 gpurun_out/phases.err; exit 1; }
cat gpurun_out/phases.jsonl
[ "${PGX_SKIP_PMC:-0}" = 1 ] || bash tools/profile_pmc.sh
