set -o pipefail
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/ab_base.json 2>gpurun_out/ab.err && \
PGX_LIB=$PWD/panda-gym_amd/libpgx_gm.so timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/ab_gm.json 2>>gpurun_out/ab.err && \
python -c "
import json
for f in ['ab_base','ab_gm']:
    d=json.load(open('gpurun_out/'+f+'.json')); print(f, round(d['value']), round(d['roofline']['kernel_ms'],4))"
