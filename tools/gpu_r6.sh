#!/bin/bash
# Round 6 GPU script.  Every GPU step runs under its own time limit; the first crash, abort or
# time limit ends the script.  Steps (environment switches):
#   tests (unless NO_TESTS=1): pytest -m gpu over PGX_TESTS (default tests/), PGX_PYTEST_ARGS
#                              appended; assertion failures (rc 1) let the later steps run
#   SMOKE=1: __graft_entry__.smoke()
#   AB="abl/a.so abl/b.so" AB_CASES=...: tools/ab_libs.py timing of library builds
#   PHASES="lib:env:n ...": tools/prof_phases.py wave-time profiles (staggered phases)
#   BENCH=1: bench.py with the driver's arguments (--steps 20 --warmup 5) and with its defaults, then
#            rocprofv3 --kernel-trace --stats of the driver-argument run
#   PMC=1: tools/pmc_r5.sh (one counter group per rocprofv3 run) into gpurun_out/pmc_r5
#   RUN="cmd": any extra python command line (run with timeout 600)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r6}
TEST_RC=0
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest ${PGX_TESTS:-tests} -v -s -m gpu --timeout 240 --timeout-method thread \
    ${PGX_PYTEST_ARGS} > gpurun_out/pytest_gpu_$TAG.log 2>&1
  TEST_RC=$?
  grep -E "FAILED|ERROR|ReachAO pcg64 resets|oracle resets agree" gpurun_out/pytest_gpu_$TAG.log | head -40
  tail -3 gpurun_out/pytest_gpu_$TAG.log
  if [ $TEST_RC -ne 0 ] && [ $TEST_RC -ne 1 ]; then exit $TEST_RC; fi
fi
if [ -n "$SMOKE" ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 ||
    { tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
  cat gpurun_out/smoke_$TAG.log
fi
if [ -n "$RUN" ]; then
  timeout -k 10 600 $RUN > gpurun_out/run_$TAG.log 2>&1 || { tail -40 gpurun_out/run_$TAG.log; exit 1; }
  tail -60 gpurun_out/run_$TAG.log
fi
if [ -n "$AB" ]; then
  timeout -k 10 1100 python -u tools/ab_libs.py $AB > gpurun_out/ab_$TAG.log 2> gpurun_out/ab_$TAG.err ||
    { tail -20 gpurun_out/ab_$TAG.err; exit 1; }
  cat gpurun_out/ab_$TAG.log
fi
if [ -n "$PHASES" ]; then
  for spec in $PHASES; do
    IFS=: read -r plib penv pn <<< "$spec"
    PGX_LIB=$plib PH_STAGGER=1 timeout -k 10 300 python tools/prof_phases.py $penv $pn 1 >> gpurun_out/phases_$TAG.jsonl \
      2>> gpurun_out/phases_$TAG.err || { tail -20 gpurun_out/phases_$TAG.err; exit 1; }
  done
  cat gpurun_out/phases_$TAG.jsonl
fi
if [ -n "$BENCH" ]; then
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_drv_$TAG.json 2> gpurun_out/bench_drv_$TAG.err ||
    { tail -20 gpurun_out/bench_drv_$TAG.err; exit 1; }
  cat gpurun_out/bench_drv_$TAG.json
  timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err ||
    { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
  cat gpurun_out/bench_$TAG.json
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- \
    python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1 ||
    { tail -20 gpurun_out/prof_$TAG.log; exit 1; }
  find gpurun_out/prof_$TAG -name "*stats*"
fi
if [ -n "$PMC" ]; then
  timeout -k 10 1000 bash tools/pmc_r5.sh > gpurun_out/pmc_$TAG.log 2>&1 || { tail -20 gpurun_out/pmc_$TAG.log; exit 1; }
  tail -6 gpurun_out/pmc_$TAG.log
fi
exit $TEST_RC
