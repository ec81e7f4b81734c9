#!/bin/bash
# Register / scratch report of ONE step kernel instantiation (a few seconds to a minute instead of
# the whole library's four): tools/ru_one.sh "step_kernel_o2<1, 0, 1, 1, 2>" [extra hipcc flags]
set -e
K=${1:-"step_kernel_o2<1, 0, 1, 1, 2>"}
shift || true
D=$(cd "$(dirname "$0")/../panda-gym_amd/csrc" && pwd)
T=$(mktemp -d)
cat > $T/one.hip <<EOT
#define PGX_TU 3
#include "$D/pgx_kernels.hip"
void pgx_ru_one(const PgxDevModel* m, const PgxDevEnv& e, const PgxDevState& s, const float* a, const PgxDevOut& o) {
    hipLaunchKernelGGL(($K), dim3(1), dim3(64), 0, 0, m, e, s, a, o);
}
EOT
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -fhip-fp32-correctly-rounded-divide-sqrt \
  -Wno-unused-function ${SLP:--fno-slp-vectorize} -I"$D" --cuda-device-only -c -o $T/one.o $T/one.hip \
  -Rpass-analysis=kernel-resource-usage "$@" 2>&1 | grep -A14 step_kernel | grep -E "Function Name|VGPRs:|AGPRs|ScratchSize|Occupancy|LDS Size" | sed 's/^.*remark: //'
if [ -n "$ASM" ]; then   # ASM=<file>: the device assembly too
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -fhip-fp32-correctly-rounded-divide-sqrt \
    -Wno-unused-function ${SLP:--fno-slp-vectorize} -I"$D" --cuda-device-only -S -o "$ASM" $T/one.hip "$@"
fi
rm -rf $T
