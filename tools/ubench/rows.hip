// The wide layout's motor-row sweep in isolation: 7 rows (DPP broadcast, shifted-bound clamp,
// impulse update, residual) per half-sweep + the per-lane exit test, 1 wave vs 1024 waves.
#include <hip/hip_runtime.h>
#include <cstdio>
template <int CTRL> __device__ __forceinline__ float dpp(float x) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), CTRL, 0xF, 0xF, true));
}
template <int V> struct IC { static constexpr int value = V; };
template <int B, int E, class F> __device__ __forceinline__ void sfor(F&& f) { if constexpr (B < E) { f(IC<B>{}); sfor<B + 1, E>(f); } }
typedef float f2 __attribute__((ext_vector_type(2)));
template <int V>
__global__ __launch_bounds__(64) void rows(float* io, long long* cyc, int n, float thr) {
    const int t = threadIdx.x;
    float gv = io[t] * 1e-3f, rhs[7], lam[7], hi[7], mc[7];
#pragma unroll
    for (int r = 0; r < 7; r++) { rhs[r] = io[64 * (r + 1) + t]; lam[r] = 0.0f; hi[r] = 0.1f + r; mc[r] = io[64 * (r + 8) + t] * 1e-3f; }
    /* lane r holds -(column of row r-1) at coordinate r */
    float coefn = 0.0f, dprev = 0.0f;
#pragma unroll
    for (int r = 0; r < 7; r++) coefn = (t % 16 == r) ? -mc[(r + 6) % 7] : coefn;
    float gw = io[t + 1] * 1e-3f, wc[7];
    f2 G = {gv, gw}, C[7], hb[7];
#pragma unroll
    for (int r = 0; r < 7; r++) { wc[r] = io[64 * (r + 1) + t + 3] * 1e-3f; C[r] = (f2){mc[r], wc[r]}; hb[r] = (f2){-hi[r], hi[r]}; }
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
            } else if constexpr (V == 3) {   /* V0 + the Delassus-lane register gw */
                const float x = rhs[r] - dpp<0x150 + r>(gv);
                const float d = __builtin_amdgcn_fmed3f(x, -hi[r] - lam[r], hi[r] - lam[r]);
                lam[r] += d;
                gv += mc[r] * d;
                gw += wc[r] * d;
                resid = fmaxf(resid, fabsf(d));
            } else if constexpr (V == 4) {   /* V3 packed: {gv, gw} and the bound pair in v_pk ops */
                const float x = rhs[r] - dpp<0x150 + r>(G.x);
                const f2 b = hb[r] - (f2){lam[r], lam[r]};
                const float d = __builtin_amdgcn_fmed3f(x, b.x, b.y);
                lam[r] += d;
                G = __builtin_elementwise_fma(C[r], (f2){d, d}, G);
                resid = fmaxf(resid, fabsf(d));
            } else if constexpr (V == 2) {   /* look-ahead: the previous row's impulse enters by one fmac */
                constexpr int rp = (r + 6) % 7;
                const float xpre = rhs[r] - dpp<0x150 + r>(gv);
                gv += mc[rp] * dprev;
                const float x = fmaf(dpp<0x150 + r>(coefn), dprev, xpre);
                const float d = __builtin_amdgcn_fmed3f(x, -hi[r] - lam[r], hi[r] - lam[r]);
                lam[r] += d;
                dprev = d;
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
    gv += mc[6] * dprev;
    io[t] = gv + lam[0] + lam[6] + gw + G.x + G.y;
    if (t == 0 && blockIdx.x == 0) { cyc[0] = t1 - t0; cyc[1] = it; }
}
int main() {
    float* d; long long* c;
    (void)hipMalloc(&d, 64 * 16 * 4 * 2048); (void)hipMalloc(&c, 64);
    (void)hipMemset(d, 0, 64 * 16 * 4 * 2048);
    for (int v = 0; v < 5; v++)
    for (int blocks : {1024, 1024}) {
        hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
        (void)hipEventRecord(e0);
        if (v == 0) hipLaunchKernelGGL(rows<0>, dim3(blocks), dim3(64), 0, 0, d, c, 2000, -1.0f);
        else if (v == 3) hipLaunchKernelGGL(rows<3>, dim3(blocks), dim3(64), 0, 0, d, c, 2000, -1.0f);
        else if (v == 4) hipLaunchKernelGGL(rows<4>, dim3(blocks), dim3(64), 0, 0, d, c, 2000, -1.0f);
        else if (v == 2) hipLaunchKernelGGL(rows<2>, dim3(blocks), dim3(64), 0, 0, d, c, 2000, -1.0f);
        else hipLaunchKernelGGL(rows<1>, dim3(blocks), dim3(64), 0, 0, d, c, 2000, -1.0f);
        (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
        float ms; (void)hipEventElapsedTime(&ms, e0, e1);
        long long h[2]; (void)hipMemcpy(h, c, 16, hipMemcpyDeviceToHost);
        printf("variant %d %4d waves: %.1f cycles per half-sweep of 7 rows (%.1f per row), %.3f ms\n", v, blocks, h[0] / (double)h[1],
               h[0] / (7.0 * h[1]), ms);
    }
    return 0;
}
