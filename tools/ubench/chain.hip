// Dependent-chain latency of the PGS row's instruction mix on one wave (s_memtime cycles per link).
#include <hip/hip_runtime.h>
#include <cstdio>
template <int CTRL> __device__ __forceinline__ float dpp(float x) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), CTRL, 0xF, 0xF, true));
}
__global__ void chains(float* out, long long* cyc, int n) {
    float g = out[threadIdx.x], a = out[64 + threadIdx.x], b = out[128 + threadIdx.x];
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; i++) {       // (0) fma chain
#pragma unroll
        for (int k = 0; k < 16; k++) g = fmaf(g, a, b);
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; i++) {       // (1) dpp-sub -> med3 -> fmac  (one PGS row)
#pragma unroll
        for (int k = 0; k < 16; k++) {
            float x = b - dpp<0x153>(g);
            float d = __builtin_amdgcn_fmed3f(x, -a, a);
            g = fmaf(a, d, g);
        }
    }
    long long t2 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; i++) {       // (2) same without dpp (register read)
#pragma unroll
        for (int k = 0; k < 16; k++) {
            float x = b - g;
            float d = __builtin_amdgcn_fmed3f(x, -a, a);
            g = fmaf(a, d, g);
        }
    }
    long long t3 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; i++) {       // (3) independent fma (issue rate): 4 chains interleaved
        float g1 = g, g2 = g + 1, g3 = g + 2;
#pragma unroll
        for (int k = 0; k < 16; k++) { g = fmaf(g, a, b); g1 = fmaf(g1, a, b); g2 = fmaf(g2, a, b); g3 = fmaf(g3, a, b); }
        g = g + g1 + g2 + g3;
    }
    long long t4 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = g;
    if (threadIdx.x == 0) { cyc[0] = t1 - t0; cyc[1] = t2 - t1; cyc[2] = t3 - t2; cyc[3] = t4 - t3; }
}
int main() {
    float* d; long long* c; hipMalloc(&d, 4096); hipMalloc(&c, 64); hipMemset(d, 0, 4096);
    const int n = 1000;
    for (int rep = 0; rep < 2; rep++) {
        hipLaunchKernelGGL(chains, dim3(1), dim3(64), 0, 0, d, c, n);
        long long h[4]; hipMemcpy(h, c, 32, hipMemcpyDeviceToHost);
        printf("cycles per link: fma chain %.2f | dpp-sub,med3,fmac row %.2f (%.2f per op) | sub,med3,fmac %.2f | 4 indep fma chains %.2f per fma\n",
               h[0] / (16.0 * n), h[1] / (16.0 * n), h[1] / (48.0 * n), h[2] / (16.0 * n), h[3] / (64.0 * n));
    }
    return 0;
}
