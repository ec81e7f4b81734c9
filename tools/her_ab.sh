for L in libpgx_a libpgx_b libpgx_a libpgx_b; do
PGX_LIB=$PWD/panda-gym_amd/$L.so timeout -k 10 120 python -c "
import sys, os, json; sys.path.insert(0, os.getcwd())
import torch, bench
r = bench.her_leg(torch.device('cuda:0'), 50, False)
print('$L', round(r['ms_per_call'], 4), round(r['roofline']['frac'], 3))
" || exit 1
done
