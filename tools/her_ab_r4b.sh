#!/bin/bash
# HER sample kernel A/B: early stores of the untouched columns (default) against all stores after
# the relabelling (PGX_HER_EARLY=0), and 16 / 32 / 64 samples per block (PGX_HER_SPB); three
# alternating runs of bench.py's HER leg each; then the HER GPU tests on the default.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/her_ab_r4b.log
: > $OUT
for rep in 1 2 3; do
  for mode in e32 n32 e16 e64; do
    unset PGX_HER_EARLY PGX_HER_SPB
    case $mode in
      n32) export PGX_HER_EARLY=0 ;;
      e16) export PGX_HER_SPB=16 ;;
      e64) export PGX_HER_SPB=64 ;;
    esac
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-tasks --no-ao --no-cpu-baseline --kernel-launches 10 > gpurun_out/her_b.json 2> gpurun_out/her_b.err || { tail -5 gpurun_out/her_b.err; exit 1; }
    python -c "import json,sys; d=json.loads(open('gpurun_out/her_b.json').read().strip().splitlines()[-1])['her_relabel']; print('$mode', d['ms_per_call'], d['value'])" >> $OUT
  done
done
unset PGX_HER_EARLY PGX_HER_SPB
cat $OUT
timeout -k 10 400 python -u -m pytest -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_her.py > gpurun_out/pytest_her.log 2>&1; tail -3 gpurun_out/pytest_her.log
