#!/bin/bash
# Round 4: phase profiles (libpgx_prof.so) of the default budget (per-pair manifolds) and the
# 4-point budget, per config; one process per case, each under its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/phases_${1:-r4}.jsonl
: > $OUT
export PGX_LIB=$PWD/panda-gym_amd/libpgx_prof.so
for c in "PandaPush-v3 4096" "PandaPickAndPlace-v3 16384" "PandaReachAO-v3 8192" "PandaReach-v3 4096"; do
  for full in true false; do
    PH_KW="{\"full_manifold\": $full}" PGX_WAVES_PER_SIMD=${WAVES:-0} timeout -k 10 240 python -u tools/prof_phases.py $c 1 >> $OUT 2> gpurun_out/phases_err.log || { tail -5 gpurun_out/phases_err.log; exit 1; }
    tail -1 $OUT | python -c "import json,sys; d=json.loads(sys.stdin.read()); w=d['last_launch_waves']; print(d['env_id'], d['n'], '$full', round(d['ms_per_step'],3), 'wave mean/p99/max', int(w['dur_mean']), int(w['dur_p99']), int(w['dur_max']), 'sweeps', round(d['sweeps_per_substep'],1), 'cyc/sweep', int(d['cycles_per_sweep']))"
  done
done
