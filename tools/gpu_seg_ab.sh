set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/seg
timeout -k 10 300 python -u -m pytest tests/test_gpu_env_order.py tests/test_gpu_determinism.py -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/seg/pytest.log 2>&1; tail -2 gpurun_out/seg/pytest.log
AB_CASES="PandaPickAndPlace-v3:16384:1,PandaReachAO-v3:16384:1,PandaPickAndPlace-v3:32768:1" timeout -k 10 600 python -u tools/ab_libs.py abl/libpgx_r5i.so panda-gym_amd/libpgx.so > gpurun_out/seg/ab.log 2> gpurun_out/seg/ab.err || { tail -5 gpurun_out/seg/ab.err; exit 1; }
cat gpurun_out/seg/ab.log
for L in abl/libpgx_r5i.so panda-gym_amd/libpgx.so; do
  for C in FETCH_SIZE WRITE_SIZE; do
    PGX_LIB=$L timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d gpurun_out/seg/$(basename $L .so)_$C -o run -- python3 tools/time_staggered.py PandaPickAndPlace-v3 16384 > gpurun_out/seg/pmc_$(basename $L .so)_$C.log 2>&1 || { echo "pmc failed"; tail -5 gpurun_out/seg/pmc_$(basename $L .so)_$C.log; exit 1; }
  done
done
echo done
