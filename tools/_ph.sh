cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
if [ -n "$TEST_LIB" ]; then
PGX_LIB=$PWD/${TEST_LIB} timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/ab_pytest.log 2>&1 || { tail -40 gpurun_out/ab_pytest.log; exit 1; }
tail -2 gpurun_out/ab_pytest.log
fi
if [ -n "$PH_CASES" ]; then
for cs in $PH_CASES; do IFS=: read e n k <<< "$cs"; PGX_LIB=panda-gym_amd/libpgx_prof.so timeout -k 10 200 python3 tools/prof_phases.py $e $n $k || exit 1; done
fi
if [ -n "$AB_LIBS" ]; then
AB_CASES=${AB_CASES:-PandaReach-v3:4096:1,PandaReach-v3:4096:0,PandaReachAO-v3:8192:1} timeout -k 10 500 python tools/ab_libs.py $AB_LIBS 2>&1 | tee gpurun_out/ab.log
fi
