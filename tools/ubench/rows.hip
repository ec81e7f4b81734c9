// The wide layout's motor-row sweep in isolation: 7 rows (DPP broadcast, shifted-bound clamp,
// impulse update, residual) per half-sweep + the per-lane exit test, 1 wave vs 1024 waves.
#include <hip/hip_runtime.h>
#include <cstdio>
template <int CTRL> __device__ __forceinline__ float dpp(float x) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), CTRL, 0xF, 0xF, true));
}
template <int V> struct IC { static constexpr int value = V; };
template <int B, int E, class F> __device__ __forceinline__ void sfor(F&& f) { if constexpr (B < E) { f(IC<B>{}); sfor<B + 1, E>(f); } }
template <int V>
__global__ __launch_bounds__(64) void rows(float* io, long long* cyc, int n, float thr) {
    const int t = threadIdx.x;
    float gv = io[t] * 1e-3f, rhs[7], lam[7], hi[7], mc[7];
#pragma unroll
    for (int r = 0; r < 7; r++) { rhs[r] = io[64 * (r + 1) + t]; lam[r] = 0.0f; hi[r] = 0.1f + r; mc[r] = io[64 * (r + 8) + t] * 1e-3f; }
    long long t0 = __builtin_amdgcn_s_memtime();
    int it = 0;
    for (; it < n; it++) {
        float resid = 0.0f;
        sfor<0, 7>([&](auto rc) {
            constexpr int r = decltype(rc)::value;
            if constexpr (V == 0) {   /* shifted bounds */
                const float x = rhs[r] - dpp<0x150 + r>(gv);
                const float d = __builtin_amdgcn_fmed3f(x, -hi[r] - lam[r], hi[r] - lam[r]);
                lam[r] += d;
                gv += mc[r] * d;
                resid = fmaxf(resid, fabsf(d));
            } else {                  /* lam + rhs off the chain, delta = nl - lam */
                const float x = (lam[r] + rhs[r]) - dpp<0x150 + r>(gv);
                const float nl = __builtin_amdgcn_fmed3f(x, -hi[r], hi[r]);
                const float d = nl - lam[r];
                lam[r] = nl;
                gv += mc[r] * d;
                resid = fmaxf(resid, fabsf(d));
            }
        });
        if (resid * resid <= thr) break;
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    io[t] = gv + lam[0] + lam[6];
    if (t == 0 && blockIdx.x == 0) { cyc[0] = t1 - t0; cyc[1] = it; }
}
int main() {
    float* d; long long* c;
    (void)hipMalloc(&d, 64 * 16 * 4 * 2048); (void)hipMalloc(&c, 64);
    (void)hipMemset(d, 0, 64 * 16 * 4 * 2048);
    for (int v = 0; v < 2; v++)
    for (int blocks : {1024, 1024}) {
        hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
        (void)hipEventRecord(e0);
        if (v == 0) hipLaunchKernelGGL(rows<0>, dim3(blocks), dim3(64), 0, 0, d, c, 2000, -1.0f);
        else hipLaunchKernelGGL(rows<1>, dim3(blocks), dim3(64), 0, 0, d, c, 2000, -1.0f);
        (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
        float ms; (void)hipEventElapsedTime(&ms, e0, e1);
        long long h[2]; (void)hipMemcpy(h, c, 16, hipMemcpyDeviceToHost);
        printf("variant %d %4d waves: %.1f cycles per half-sweep of 7 rows (%.1f per row), %.3f ms\n", v, blocks, h[0] / (double)h[1],
               h[0] / (7.0 * h[1]), ms);
    }
    return 0;
}
