#!/bin/bash
# Round 4: GPU tests (current tree), then optional A/B timing of library builds (AB="abl/a.so abl/b.so",
# AB_CASES=env:envs:contacts:full,...), then optional bench + rocprof kernel stats (BENCH=1).
# Each GPU step under its own time limit, chained: the first failure ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r4}
TEST_RC=0
if [ -z "$NO_TESTS" ]; then
  # assertion failures (pytest rc 1) do not stop the timing steps below; anything else (a crash,
  # an abort, a time limit) ends the script here
  timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 240 --timeout-method thread ${PGX_PYTEST_ARGS} > gpurun_out/pytest_gpu_$TAG.log 2>&1
  TEST_RC=$?
  grep -E "FAILED|ERROR" gpurun_out/pytest_gpu_$TAG.log | head -40
  tail -3 gpurun_out/pytest_gpu_$TAG.log
  if [ $TEST_RC -ne 0 ] && [ $TEST_RC -ne 1 ]; then exit $TEST_RC; fi
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
  cat gpurun_out/smoke_$TAG.log
fi
if [ -n "$AB" ]; then
  timeout -k 10 1100 python -u tools/ab_libs.py $AB > gpurun_out/ab_$TAG.log 2> gpurun_out/ab_$TAG.err || { tail -20 gpurun_out/ab_$TAG.err; exit 1; }
  cat gpurun_out/ab_$TAG.log
fi
if [ -n "$BENCH" ]; then
  timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
  cat gpurun_out/bench_$TAG.json
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1 || { tail -20 gpurun_out/prof_$TAG.log; exit 1; }
  find gpurun_out/prof_$TAG -name "*stats*"
fi
exit $TEST_RC
