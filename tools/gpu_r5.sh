#!/bin/bash
# Round 5 GPU script.  Steps (each under its own time limit, chained so the first crash ends it):
#   PROBE="abl/a.so ..."  tools/gpu_nan_probe.py on debug libraries (make -C panda-gym_amd/csrc dbg)
#   NANWT=abl/<worktree> NANWT_LIBS="a.so b.so"  tools/gpu_rtmodel_nan.py inside an older source tree, per
#                         runtime-model library of that tree
#   tests (unless NO_TESTS=1): pytest -m gpu (PGX_PYTEST_ARGS appended), then smoke()
#   AB="abl/a.so abl/b.so" AB_CASES=...: tools/ab_libs.py timing of library builds
#   PMC=1: tools/pmc_r5.sh (rocprofv3 --pmc passes over a short bench run) into gpurun_out/pmc_r5
#   BENCH=1: bench.py with the driver's arguments (--steps 20 --warmup 5) and the defaults, then
#            rocprofv3 --kernel-trace --stats of the driver-argument run
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r5}
TEST_RC=0
if [ -n "$PROBE" ]; then
  timeout -k 10 900 python -u tools/gpu_nan_probe.py $PROBE > gpurun_out/probe_$TAG.log 2>&1
  rc=$?
  tail -60 gpurun_out/probe_$TAG.log
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
if [ -n "$NANWT" ]; then   # tools/gpu_rtmodel_nan.py inside an older tree (a git worktree under abl/), per library
  for lib in ${NANWT_LIBS:-libpgx_rtmodel.so}; do
    echo "# $lib" >> gpurun_out/nanwt_$TAG.log
    ( cd "$NANWT" && RT_LIB=$lib timeout -k 10 300 python -u tools/gpu_rtmodel_nan.py ) >> gpurun_out/nanwt_$TAG.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then tail -30 gpurun_out/nanwt_$TAG.log; exit $rc; fi
  done
  grep -v amdgpu.ids gpurun_out/nanwt_$TAG.log
fi
if [ -n "$REPRO" ]; then   # the round-4 sort's graph fault, restated (tools/repro_sort_graph.hip)
  timeout -k 10 120 tools/repro_sort_graph 96 > gpurun_out/repro_sort_$TAG.log 2>&1 &&
    timeout -k 10 180 python tools/repro_sort_graph_torch.py >> gpurun_out/repro_sort_$TAG.log 2>&1
  rc=$?
  cat gpurun_out/repro_sort_$TAG.log
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
if [ -z "$NO_TESTS" ]; then
  # assertion failures (pytest rc 1) do not stop the timing steps below; anything else (a crash,
  # an abort, a time limit) ends the script here
  timeout -k 10 900 python -u -m pytest ${PGX_TESTS:-tests} -v -m gpu --timeout 240 --timeout-method thread ${PGX_PYTEST_ARGS} > gpurun_out/pytest_gpu_$TAG.log 2>&1
  TEST_RC=$?
  grep -E "FAILED|ERROR" gpurun_out/pytest_gpu_$TAG.log | head -40
  tail -3 gpurun_out/pytest_gpu_$TAG.log
  if [ $TEST_RC -ne 0 ] && [ $TEST_RC -ne 1 ]; then if [ -n "$PMC" ]; then   # the PMC passes (tools/pmc_r5.sh), one counter group per rocprofv3 run
  timeout -k 10 1000 bash tools/pmc_r5.sh > gpurun_out/pmc_$TAG.log 2>&1 || { tail -20 gpurun_out/pmc_$TAG.log; exit 1; }
  tail -6 gpurun_out/pmc_$TAG.log
fi
exit $TEST_RC; fi
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
  cat gpurun_out/smoke_$TAG.log
fi
if [ -n "$PHASES" ]; then   # phase profiles: PHASES="lib:env:n ..." (tools/prof_phases.py, staggered phases)
  for spec in $PHASES; do
    IFS=: read -r plib penv pn <<< "$spec"
    PGX_LIB=$plib PH_STAGGER=1 timeout -k 10 300 python tools/prof_phases.py $penv $pn 1 >> gpurun_out/phases_$TAG.jsonl 2>> gpurun_out/phases_$TAG.err || { tail -20 gpurun_out/phases_$TAG.err; exit 1; }
  done
  cat gpurun_out/phases_$TAG.jsonl
fi
if [ -n "$AB" ]; then
  timeout -k 10 1100 python -u tools/ab_libs.py $AB > gpurun_out/ab_$TAG.log 2> gpurun_out/ab_$TAG.err || { tail -20 gpurun_out/ab_$TAG.err; exit 1; }
  cat gpurun_out/ab_$TAG.log
fi
if [ -n "$BENCH" ]; then
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_drv_$TAG.json 2> gpurun_out/bench_drv_$TAG.err || { tail -20 gpurun_out/bench_drv_$TAG.err; exit 1; }
  cat gpurun_out/bench_drv_$TAG.json
  timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
  cat gpurun_out/bench_$TAG.json
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1 || { tail -20 gpurun_out/prof_$TAG.log; exit 1; }
  find gpurun_out/prof_$TAG -name "*stats*"
fi
if [ -n "$PMC" ]; then   # the PMC passes (tools/pmc_r5.sh), one counter group per rocprofv3 run
  timeout -k 10 1000 bash tools/pmc_r5.sh > gpurun_out/pmc_$TAG.log 2>&1 || { tail -20 gpurun_out/pmc_$TAG.log; exit 1; }
  tail -6 gpurun_out/pmc_$TAG.log
fi
exit $TEST_RC
