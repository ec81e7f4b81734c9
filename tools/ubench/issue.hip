// Issue cost of the PGS row's instruction kinds on one wave64 (s_memtime cycles per instruction):
// 8 independent streams (throughput) and 1 dependent stream (latency) per kind.
#include <hip/hip_runtime.h>
#include <cstdio>
template <int CTRL> __device__ __forceinline__ float dpp(float x) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), CTRL, 0xF, 0xF, true));
}
template <int K> __device__ __forceinline__ float op(float g, float a, float b) {
    if constexpr (K == 0) return fmaf(g, a, b);
    if constexpr (K == 1) return __builtin_amdgcn_fmed3f(g, a, b);
    if constexpr (K == 2) return b - dpp<0x153>(g);          /* v_subrev_dpp row_newbcast */
    if constexpr (K == 3) return b - dpp<0xB1>(g);           /* v_subrev_dpp quad_perm */
    if constexpr (K == 4) return -a - g;                     /* v_sub_e64 with neg */
    if constexpr (K == 5) return g + b;                      /* v_add_e32 */
    if constexpr (K == 6) return fmaxf(fmaxf(g, fabsf(a)), fabsf(b));   /* v_max3 */
    return dpp<0x153>(g);                                     /* v_mov_dpp */
}
template <int K> __global__ void kern(float* out, long long* cyc, int n) {
    float a = out[64 + threadIdx.x], b = out[128 + threadIdx.x];
    float g[8];
#pragma unroll
    for (int s = 0; s < 8; s++) g[s] = out[threadIdx.x] + s;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; i++) {
#pragma unroll
        for (int k = 0; k < 8; k++)
#pragma unroll
            for (int s = 0; s < 8; s++) g[s] = op<K>(g[s], a, b);
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    float h = g[0];
    for (int i = 0; i < n; i++) {
#pragma unroll
        for (int k = 0; k < 64; k++) h = op<K>(h, a, b);
    }
    long long t2 = __builtin_amdgcn_s_memtime();
    float acc = h;
#pragma unroll
    for (int s = 0; s < 8; s++) acc += g[s];
    out[threadIdx.x] = acc;
    if (threadIdx.x == 0) { cyc[0] = t1 - t0; cyc[1] = t2 - t1; }
}
typedef float f2 __attribute__((ext_vector_type(2)));
__global__ void kpk(float* out, long long* cyc, int n) {   /* v_pk_fma_f32: two fp32 fma per lane */
    f2 a = {out[64 + threadIdx.x], out[65 + threadIdx.x]}, b = {out[128 + threadIdx.x], out[3]};
    f2 g[8];
#pragma unroll
    for (int s = 0; s < 8; s++) g[s] = (f2){out[threadIdx.x] + s, out[threadIdx.x + 1] + s};
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; i++) {
#pragma unroll
        for (int k = 0; k < 8; k++)
#pragma unroll
            for (int s = 0; s < 8; s++) g[s] = __builtin_elementwise_fma(g[s], a, b);
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    f2 h = g[0];
    for (int i = 0; i < n; i++) {
#pragma unroll
        for (int k = 0; k < 64; k++) h = __builtin_elementwise_fma(h, a, b);
    }
    long long t2 = __builtin_amdgcn_s_memtime();
    f2 acc = h;
#pragma unroll
    for (int s = 0; s < 8; s++) acc += g[s];
    out[threadIdx.x] = acc.x + acc.y;
    if (threadIdx.x == 0) { cyc[0] = t1 - t0; cyc[1] = t2 - t1; }
}
template <int K> void run(const char* name, float* d, long long* c) {
    const int n = 500;
    for (int rep = 0; rep < 2; rep++) {
        hipLaunchKernelGGL(kern<K>, dim3(1), dim3(64), 0, 0, d, c, n);
        long long h[2]; (void)hipMemcpy(h, c, 16, hipMemcpyDeviceToHost);
        if (rep) printf("%-28s throughput %.2f  latency %.2f cycles/instr\n", name, h[0] / (64.0 * n), h[1] / (64.0 * n));
    }
}
int main() {
    float* d; long long* c; (void)hipMalloc(&d, 4096); (void)hipMalloc(&c, 64); (void)hipMemset(d, 0, 4096);
    run<0>("v_fma", d, c); run<1>("v_med3", d, c); run<2>("v_subrev_dpp row_newbcast", d, c);
    run<3>("v_subrev_dpp quad_perm", d, c); run<4>("v_sub_e64 neg", d, c); run<5>("v_add_e32", d, c);
    run<6>("v_max3 |a| |b|", d, c); run<7>("v_mov_dpp row_newbcast", d, c);
    for (int rep = 0; rep < 2; rep++) {
        hipLaunchKernelGGL(kpk, dim3(1), dim3(64), 0, 0, d, c, 500);
        long long h[2]; (void)hipMemcpy(h, c, 16, hipMemcpyDeviceToHost);
        if (rep) printf("%-28s throughput %.2f  latency %.2f cycles/instr\n", "v_pk_fma_f32", h[0] / (64.0 * 500), h[1] / (64.0 * 500));
    }
    return 0;
}
