set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -30 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
PGX_LIB=$PWD/panda-gym_amd/libpgx_prof.so timeout -k 10 300 python tools/prof_phases.py > gpurun_out/phases.json 2>&1; rc=$?
cat gpurun_out/phases.json
exit $rc
