/*
 * pgx_common.h -- device helpers shared by the env-step kernels and the HER ring.
 */
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

/* Philox4x32-10 (Salmon et al. 2011): counter (c0..c3), key (k0, k1). */
__device__ __forceinline__ void philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1,
                                       uint32_t* out) {
#pragma unroll
    for (int r = 0; r < 10; r++) {
        uint32_t hi0 = __umulhi(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
        uint32_t hi1 = __umulhi(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
        uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

/* top 53 bits of (hi:lo) as a double in [0, 1) */
__device__ __forceinline__ double u53(uint32_t lo, uint32_t hi) {
    return (double)((((uint64_t)hi << 32) | lo) >> 11) * (1.0 / 9007199254740992.0);
}

#pragma clang fp contract(off)
/* utils.distance (utils.py:18-30) on float32 rows, as numpy evaluates it on float32
 * arrays: d = a - b, sum of squares left to right, sqrt, np.round(d, 6) = rint(d*1e6)/1e6. */
__device__ __forceinline__ float distance_f32_f32(const float* a, const float* b) {
    float d0 = a[0] - b[0], d1 = a[1] - b[1], d2 = a[2] - b[2];
    float s = d0 * d0 + d1 * d1;
    s = s + d2 * d2;
    float d = sqrtf(s);
    float y = rintf(d * 1e6f);
    return y / 1e6f;
}
#pragma clang fp contract(on)

/* Task.compute_reward (reach.py:84-89): sparse -(d > thr) as f32 (-0.0 on success), dense -d;
 * ReachAO sparse (reach_ao.py:1320) -1 + (d < thr) (+0.0 on success) */
__device__ __forceinline__ float reward_f32(float d, int reward_type, float thr) {
    if (reward_type == 2) return d < thr ? 0.0f : -1.0f;
    return reward_type == 0 ? -((d > thr) ? 1.0f : 0.0f) : -d;
}
