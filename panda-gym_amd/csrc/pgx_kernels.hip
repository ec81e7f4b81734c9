/*
 * pgx_kernels.hip -- lockstep batched Panda env step for gfx950 (MI355X).
 *
 * One environment per lane, the whole env step (IK + 20 physics substeps +
 * observation + reward + TimeLimit/auto-reset) in one launch with the state
 * in VGPRs.  The path is FP32-VALU bound (no dense contraction: MFMA does not
 * apply); HBM traffic is the SoA state (coalesced, env-minor) plus the
 * action/obs rows.  Robot constants arrive by value in the kernarg segment
 * (scalar loads), so per-lane registers hold only per-env state.
 *
 * Reference hot path restated here (RaikoPipe/panda-gym):
 *   RobotTaskEnv.step            panda_gym/envs/core.py:352-368
 *   Panda.set_action             panda_gym/envs/robots/panda.py:120-172
 *     ee_displacement_to_target  panda.py:226-246 -> PyBullet.inverse_kinematics
 *                                pybullet.py:465-493 (Bullet DLS IK, see ik())
 *     arm_joint_ctrl_to_target   panda.py:248-262
 *     control_joints             pybullet.py:437-455 (POSITION_CONTROL motors)
 *   PyBullet.step                pybullet.py:68-71 (20 x stepSimulation, see substep())
 *   Panda.get_obs / get_ee_*     panda.py:264-312 (COM position/velocity of link 11)
 *   Reach.is_success/compute_reward reach.py:80-89, utils.distance utils.py:4-16
 */
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "../../include/pgx.h"
#include "pgx_default_model.h"
#include "pgx_common.h"
#include "pgx_dev.h"
#include "pgx_model_consts.h"
#include "pgx_rows.h"

#ifdef PGX_PROF
#define PGX_PROF_N 24
__device__ unsigned long long pgx_prof_counters[PGX_PROF_N];
/* per wave of the last launch (block id): start / end s_memtime, sweeps, non-far, redo, all-rows */
#define PGX_PROF_WAVES 16384
__device__ unsigned long long pgx_prof_wave[PGX_PROF_WAVES][10];
extern "C" int pgx_prof_wave_read(unsigned long long* out, int n) {
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(pgx_prof_wave), sizeof(unsigned long long) * 10 * (size_t)n);
}
extern "C" int pgx_prof_read(unsigned long long* out, int clear) {
    hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(pgx_prof_counters), sizeof(unsigned long long) * PGX_PROF_N);
    if (e == hipSuccess && clear) {
        unsigned long long z[PGX_PROF_N] = {0};
        e = hipMemcpyToSymbol(HIP_SYMBOL(pgx_prof_counters), z, sizeof z);
    }
    return (int)e;
}
#endif
namespace {

constexpr int NJ = PGX_NJ;

/* The constant block (PgxDevModel: the folded robot and the physics / solver parameters) is a
 * compile-time constant of the kernels: pgx_create builds the block for a handle and refuses
 * one that differs from these (the reference's defaults: pybullet's timestep, solver, motor and
 * contact constants, panda.py's forces and neutral pose; generated into pgx_default_model.h by
 * tools/gen_default_model.py from pgx_create's own folding), so every parameter folds into the
 * instruction stream -- no scalar load and wait (SQ_WAIT_ANY was 15 % of the headline's wave
 * cycles; -2.6 % kernel time).  Two blocks: the robot base of Reach / Push / PickAndPlace and
 * of ReachAO.  `fresh()` is the identity here.  `make runtime-model` builds the kernels that
 * read the handle's block instead (other parameters; the round-2 kernels). */
typedef const __attribute__((address_space(4))) PgxDevModel* MPtr;
typedef const __attribute__((address_space(4))) PgxDevModel& MRef;
#ifndef PGX_RUNTIME_MODEL
static_assert(sizeof(PgxDevModel) == 4 * PGX_DEV_MODEL_WORDS, "default model block size");
__constant__ const PgxDevModel kDefModelArm = __builtin_bit_cast(PgxDevModel, kDefModelArmWords);
__constant__ const PgxDevModel kDefModelAo = __builtin_bit_cast(PgxDevModel, kDefModelAoWords);
template <int AO>
__device__ __forceinline__ MPtr model_ptr(const PgxDevModel*) { return AO ? (MPtr)&kDefModelAo : (MPtr)&kDefModelArm; }
__device__ __forceinline__ MPtr fresh(MPtr p) { return p; }
#else
/* `make runtime-model` (libpgx_rtmodel.so): any parameters, read from the handle's device block
 * through scalar loads; the asm hides the pointer at the top of each substep / IK iteration so
 * the loads are re-issued where used rather than ~350 constants hoisted into VGPR lanes. */
__device__ __forceinline__ MPtr fresh(uint64_t addr) {
    asm volatile("; pgx fresh model pointer %0" : "+s"(addr));
    return (MPtr)addr;
}
__device__ __forceinline__ MPtr fresh(MPtr p) { return fresh((uint64_t)p); }
template <int AO>
__device__ __forceinline__ MPtr model_ptr(const PgxDevModel* mdev) { return fresh((uint64_t)mdev); }
#endif

/* Phase profile (build with -DPGX_PROF, tools/prof_phases.py): per-wave s_memtime
 * deltas accumulated in LDS by phase, summed over waves into pgx_prof_counters at the
 * end of the launch.  Compiled out of the product library. */
#ifdef PGX_PROF
__shared__ volatile unsigned long long g_prof[PGX_PROF_N];   /* volatile: never kept in per-lane registers */
__shared__ volatile unsigned long long g_prof_t;
__device__ __forceinline__ void prof_mark(int k) {
    const unsigned long long t = __builtin_amdgcn_s_memtime();
    g_prof[k] += t - g_prof_t;
    g_prof_t = t;
}
#define PGX_PROF_MARK(k) prof_mark(k)
#define PGX_PROF_COUNT(k, v) (g_prof[k] += (unsigned long long)(v))
/* sweeps: counted per lane in a register, the wave's maximum (the loop's trip count) added
 * once per substep, so the counting adds nothing to the sweep loop's LDS traffic */
#define PGX_PROF_SWEEP() (++prof_sweeps)
#define PGX_PROF_SWEEPS_DONE()                                                       \
    do {                                                                             \
        int v_ = prof_sweeps;                                                        \
        for (int o_ = 32; o_ >= 1; o_ >>= 1) v_ = max(v_, __shfl_xor(v_, o_));      \
        g_prof[8] += (unsigned long long)v_;                                         \
    } while (0)
#define PGX_PROF_SWEEPS_DECL int prof_sweeps = 0
#else
#define PGX_PROF_MARK(k) ((void)0)
#define PGX_PROF_COUNT(k, v) ((void)0)
#define PGX_PROF_SWEEP() ((void)0)
#define PGX_PROF_SWEEPS_DONE() ((void)0)
#define PGX_PROF_SWEEPS_DECL ((void)0)
#endif

/* Debug builds only (make dbg, tools/gpu_nan_probe.py): PGX_NAN_TRAP prints the first non-finite
 * value per lane at each phase of the one-lane step (IK targets, unconstrained dynamics, the
 * solve, the integration, the observation) with the model constants read at that point;
 * PGX_LDS_POISON fills the step's LDS with NaN at kernel start, so any read of LDS the kernel did
 * not write first turns into a non-finite result in every build. */
#ifdef PGX_NAN_TRAP
__device__ int pgx_nan_prints;
#define PGX_TRAP(tag, sub, arr, n, mm)                                                                          \
    do {                                                                                                   \
        bool bad_ = false;                                                                                 \
        for (int t_ = 0; t_ < (n); t_++) bad_ = bad_ || !isfinite((arr)[t_]);                            \
        if (bad_ && atomicAdd(&pgx_nan_prints, 1) < 96)                                                    \
            printf("PGX_NAN tag %d sub %d block %d lane %d v %g %g %g %g %g %g %g | dt %g kp %g kd %g "     \
                   "maxv %g res %g erp %g fr %g it %d\n",                                                 \
                   (tag), (sub), (int)blockIdx.x, (int)threadIdx.x, (arr)[0], (n) > 1 ? (arr)[1] : 0.0f,   \
                   (n) > 2 ? (arr)[2] : 0.0f, (n) > 3 ? (arr)[3] : 0.0f, (n) > 4 ? (arr)[4] : 0.0f,        \
                   (n) > 5 ? (arr)[5] : 0.0f, (n) > 6 ? (arr)[6] : 0.0f, (mm).dt, (mm).kp, (mm).kd,         \
                   (mm).max_vel, (mm).residual_abs, (mm).contact_erp, (mm).friction, (mm).num_iterations); \
    } while (0)
#else
#define PGX_TRAP(tag, sub, arr, n, mm) ((void)0)
#endif

struct V3 {
    float x, y, z;
};
__device__ __forceinline__ V3 v3(float x, float y, float z) { return V3{x, y, z}; }
__device__ __forceinline__ V3 operator+(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ V3 operator-(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ V3 operator*(float s, V3 a) { return v3(s * a.x, s * a.y, s * a.z); }
__device__ __forceinline__ float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ V3 cross(V3 a, V3 b) {
    return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
/* Hot-path reciprocal / square root: the hardware v_rcp_f32 / v_sqrt_f32 (1 ulp).  The
 * library is compiled with correctly rounded '/' and sqrtf, which the reward path needs
 * for bit-exact parity with numpy; the physics does not. */
__device__ __forceinline__ float fast_rcp(float x) { return __builtin_amdgcn_rcpf(x); }
__device__ __forceinline__ float fast_sqrt(float x) { return __builtin_amdgcn_sqrtf(x); }
__device__ __forceinline__ float norm(V3 a) { return fast_sqrt(dot(a, a)); }

/* sin/cos of a joint angle (|x| < ~1e3): Cody-Waite reduction by pi/2 in three parts and
 * the Cephes single-precision minimax polynomials on [-pi/4, pi/4] (~1 ulp).  Branch-free
 * and ~25 VALU ops, against the generic sincosf whose Payne-Hanek path is also emitted. */
__device__ __forceinline__ void joint_sincos(float x, float* s_out, float* c_out) {
    const float k = rintf(x * 0.63661977236758134f);
    float r = fmaf(k, -1.5703125f, x);
    r = fmaf(k, -4.837512969970703125e-4f, r);
    r = fmaf(k, -7.54978995489188216e-8f, r);
    const float z = r * r;
    const float s = fmaf(r * z, fmaf(z, fmaf(z, -1.9515295891e-4f, 8.3321608736e-3f), -1.6666654611e-1f), r);
    const float c = fmaf(z * z, fmaf(z, fmaf(z, 2.443315711809948e-5f, -1.388731625493765e-3f), 4.166664568298827e-2f),
                         fmaf(-0.5f, z, 1.0f));
    const int q = (int)k & 3;
    const float ss = (q & 1) ? c : s, cc = (q & 1) ? s : c;
    *s_out = (q & 2) ? -ss : ss;
    *c_out = ((q + 1) & 2) ? -cc : cc;
}

/* a V3 from three lane-minor LDS rows */
template <int W>
__device__ __forceinline__ V3 lds3(const float (*a)[W], int ln) { return v3(a[0][ln], a[1][ln], a[2][ln]); }

typedef float f2 __attribute__((ext_vector_type(2)));   /* packed fp32 pair (v_pk_*_f32) */
/* PGS rows with packed updates (pk_fma_acc): bit 0 joint rows and bit 1 contact rows pair the
 * coordinate and Delassus registers {gv, gw}; bit 2 pairs the two Delassus registers {gw, gw2}
 * (object tasks, full manifold).  Per kernel family, as measured (profiles/r05/ab_packed_rows.log):
 * ReachAO gains with its contact rows paired (0.779 -> 0.768 ms at 8192, scratch unchanged; both
 * kinds 0.766 ms but 32 B more scratch per lane); the object kernels gain with {gw, gw2} (Push 4096
 * 1.212 -> 1.199 ms, PickAndPlace 16384 2.909 -> 2.855, no scratch); {gv, gw} pairs lose 0.4-5.8 %
 * everywhere else (the pairs' aligned registers: more AGPR copies, or spills in two-wave builds) */
#ifndef PGX_PK
#define PGX_PK 4
#endif
#ifndef PGX_PK_AO
#define PGX_PK_AO 2
#endif
/* {a, b} += {ca, cb} s as one v_pk_fma_f32: each half is the fused multiply-add of the scalar
 * form, bit for bit, in one issue instead of two (two of a PGS row's register updates) */
__device__ __forceinline__ void pk_fma_acc(float& a, float& b, f2 cab, float s) {
    const f2 r = __builtin_elementwise_fma(cab, (f2){s, s}, (f2){a, b});
    a = r.x;
    b = r.y;
}
constexpr int GW = 16;          /* lanes per env: one DPP row */
constexpr int EPW = 64 / GW;    /* envs per wave */

template <int V>
struct IC {
    static constexpr int value = V;
};
/* compile-time loop (DPP controls must be constants) */
template <int B, int E, class F>
__device__ __forceinline__ void sfor(F&& f) {
    if constexpr (B < E) {
        f(IC<B>{});
        sfor<B + 1, E>(f);
    }
}
template <int CTRL>
__device__ __forceinline__ float dpp(float x) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), CTRL, 0xF, 0xF, true));
}
/* lane SRC of this lane's 16-lane row (DPP row_newbcast, gfx90a+) */
template <int SRC>
__device__ __forceinline__ float bcast16(float x) {
    return dpp<0x150 + SRC>(x);
}
/* sum over the 16-lane row, the same bits in every lane: each butterfly step adds two
 * partner sums that are already equal within their halves, and fl(a+b) = fl(b+a) */
__device__ __forceinline__ float sum16(float x) {
    x += dpp<0xB1>(x);    /* quad_perm [1,0,3,2] */
    x += dpp<0x4E>(x);    /* quad_perm [2,3,0,1] */
    x += dpp<0x141>(x);   /* row_half_mirror */
    x += dpp<0x140>(x);   /* row_mirror */
    return x;
}
/* Per-lane selection by row position K as one v_cndmask with a constant lane mask.  Plain
 * `c == k ? a[k] : v` chains get rewritten by the compiler into a dynamically indexed
 * stack array (scratch memory); the asm keeps them as selects. */
template <int K>
__device__ __forceinline__ float lane_sel(float a, float other) {   /* lanes with c == K take a */
    constexpr uint64_t mask = 0x0001000100010001ull << K;
    float r;
    asm("v_cndmask_b32 %0, %1, %2, %3" : "=v"(r) : "v"(other), "v"(a), "s"(mask));
    return r;
}
/* object coordinate of (lin, ang) for this lane: 7-9 linear, 10-12 angular, else 0 */
__device__ __forceinline__ float pick_obj(V3 lin, V3 ang) {
    float v = 0.0f;
    v = lane_sel<7>(lin.x, v); v = lane_sel<8>(lin.y, v); v = lane_sel<9>(lin.z, v);
    v = lane_sel<10>(ang.x, v); v = lane_sel<11>(ang.y, v); v = lane_sel<12>(ang.z, v);
    return v;
}
/* this lane's arm entry a[c] (c < 7), else `other` */
__device__ __forceinline__ float pick_arm(const float* a, float other) {
    float v = other;
    sfor<0, NJ>([&](auto kc) __attribute__((always_inline)) { v = lane_sel<decltype(kc)::value>(a[decltype(kc)::value], v); });
    return v;
}
/* generalized coordinate of (arm[7], lin, ang) for this lane: arm dof c < 7, object 7-12, else 0 */
__device__ __forceinline__ float pick_gen(const float* arm, V3 lin, V3 ang) { return pick_arm(arm, pick_obj(lin, ang)); }
__device__ __forceinline__ V3 pick_v3(const V3* a) {
    float x[NJ], y[NJ], zz[NJ];
#pragma unroll
    for (int k = 0; k < NJ; k++) { x[k] = a[k].x; y[k] = a[k].y; zz[k] = a[k].z; }
    return v3(pick_arm(x, 0.0f), pick_arm(y, 0.0f), pick_arm(zz, 0.0f));
}

/* the 16-lane row's mask of a predicate (bit c = lane c of this env's row) */
__device__ __forceinline__ unsigned row_ballot(bool v) {
    return (unsigned)((__ballot(v) >> (threadIdx.x & ~(unsigned)(GW - 1))) & 0xFFFFull);
}
__device__ __forceinline__ bool row_any(bool v) { return row_ballot(v) != 0u; }

/* sin/cos of the 7 joint angles.  PAR (wide layout, all 16 lanes of an env hold the same
 * q): lane c evaluates joint c and the row broadcasts, 14 DPP moves instead of 7
 * polynomial evaluations per lane. */
template <bool PAR>
__device__ __forceinline__ void joint_sincos_all(const float* q, float* s, float* c) {
    if constexpr (PAR) {
        float ls, lc;
        joint_sincos(pick_arm(q, 0.0f), &ls, &lc);
        sfor<0, PGX_NJ>([&](auto jc) __attribute__((always_inline)) {
            constexpr int j = decltype(jc)::value;
            s[j] = bcast16<j>(ls);
            c[j] = bcast16<j>(lc);
        });
    } else {
#pragma unroll
        for (int j = 0; j < PGX_NJ; j++) joint_sincos(q[j], &s[j], &c[j]);
    }
}

/* row-major 3x3 */
struct M3 {
    float m[9];
};
__device__ __forceinline__ V3 mul(const M3& A, V3 v) {
    return v3(A.m[0] * v.x + A.m[1] * v.y + A.m[2] * v.z, A.m[3] * v.x + A.m[4] * v.y + A.m[5] * v.z,
              A.m[6] * v.x + A.m[7] * v.y + A.m[8] * v.z);
}
/* x * k where k comes from the compile-time robot tables (pgx_model_consts.h):
 * after unrolling k is a literal, so 0 / +-1 factors vanish (x + -0.0f folds to x
 * exactly in IEEE) and only the genuine products remain. */
__device__ __forceinline__ float kmul(float x, float k) {
    return k == 0.0f ? -0.0f : (k == 1.0f ? x : (k == -1.0f ? -x : x * k));
}
/* A * v and A * B with v, B constant tables */
__device__ __forceinline__ V3 mulc(const M3& A, const float* v) {
    return v3(kmul(A.m[0], v[0]) + kmul(A.m[1], v[1]) + kmul(A.m[2], v[2]),
              kmul(A.m[3], v[0]) + kmul(A.m[4], v[1]) + kmul(A.m[5], v[2]),
              kmul(A.m[6], v[0]) + kmul(A.m[7], v[1]) + kmul(A.m[8], v[2]));
}
__device__ __forceinline__ M3 mulm(const M3& A, const float* B) {
    M3 C;
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++)
            C.m[i * 3 + j] = kmul(A.m[i * 3], B[j]) + kmul(A.m[i * 3 + 1], B[3 + j]) + kmul(A.m[i * 3 + 2], B[6 + j]);
    return C;
}
__device__ __forceinline__ V3 col(const M3& A, int c) { return v3(A.m[c], A.m[3 + c], A.m[6 + c]); }

/* symmetric 3x3 stored xx,yy,zz,xy,xz,yz */
struct S3 {
    float xx, yy, zz, xy, xz, yz;
};
__device__ __forceinline__ V3 mul(const S3& I, V3 v) {
    return v3(I.xx * v.x + I.xy * v.y + I.xz * v.z, I.xy * v.x + I.yy * v.y + I.yz * v.z,
              I.xz * v.x + I.yz * v.y + I.zz * v.z);
}
/* R diag(d) R^T */
__device__ __forceinline__ S3 rot_diag(const M3& R, const float* d) {
    S3 o;
    const float* r = R.m;
    o.xx = r[0] * r[0] * d[0] + r[1] * r[1] * d[1] + r[2] * r[2] * d[2];
    o.yy = r[3] * r[3] * d[0] + r[4] * r[4] * d[1] + r[5] * r[5] * d[2];
    o.zz = r[6] * r[6] * d[0] + r[7] * r[7] * d[1] + r[8] * r[8] * d[2];
    o.xy = r[0] * r[3] * d[0] + r[1] * r[4] * d[1] + r[2] * r[5] * d[2];
    o.xz = r[0] * r[6] * d[0] + r[1] * r[7] * d[1] + r[2] * r[8] * d[2];
    o.yz = r[3] * r[6] * d[0] + r[4] * r[7] * d[1] + r[5] * r[8] * d[2];
    return o;
}
/* R S R^T for a full symmetric S */
__device__ __forceinline__ S3 rot_sym(const M3& R, const float* s) {
    const float Sm[9] = {s[0], s[3], s[4], s[3], s[1], s[5], s[4], s[5], s[2]};
    float T[9];
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++)
            T[i * 3 + j] = kmul(R.m[i * 3], Sm[j]) + kmul(R.m[i * 3 + 1], Sm[3 + j]) + kmul(R.m[i * 3 + 2], Sm[6 + j]);
    auto e = [&](int i, int j) { return T[i * 3] * R.m[j * 3] + T[i * 3 + 1] * R.m[j * 3 + 1] + T[i * 3 + 2] * R.m[j * 3 + 2]; };
    S3 o;
    o.xx = e(0, 0); o.yy = e(1, 1); o.zz = e(2, 2); o.xy = e(0, 1); o.xz = e(0, 2); o.yz = e(1, 2);
    return o;
}
__device__ __forceinline__ S3 add(const S3& a, const S3& b) {
    return S3{a.xx + b.xx, a.yy + b.yy, a.zz + b.zz, a.xy + b.xy, a.xz + b.xz, a.yz + b.yz};
}
/* parallel-axis term m(|r|^2 E - r r^T) */
__device__ __forceinline__ S3 steiner(float m, V3 r) {
    float rr = dot(r, r);
    return S3{m * (rr - r.x * r.x), m * (rr - r.y * r.y), m * (rr - r.z * r.z), -m * r.x * r.y, -m * r.x * r.z,
              -m * r.y * r.z};
}

/* ------------------------------------------------------------ kinematics */
/* Chain forward kinematics: URDF frame rotation R[j] and pivot o[j] of the
 * 7 arm links (the multibody link frames sit at o[j] + R[j]*com[j]). */
struct Chain {
    M3 R[NJ];
    V3 o[NJ];
};

template <bool PAR = false>
__device__ __forceinline__ void fk_chain(MRef m, const float* q, Chain& k) {
    M3 PR = {{1, 0, 0, 0, 1, 0, 0, 0, 1}};
    V3 PO = v3(m.base[0], m.base[1], m.base[2]);
    float sj[NJ], cj[NJ];
    joint_sincos_all<PAR>(q, sj, cj);
#pragma unroll
    for (int j = 0; j < NJ; j++) {
        M3 R = mulm(PR, kJr[j]);
        V3 o = PO + mulc(PR, kJp[j]);
        const float s = sj[j], c = cj[j];
        /* R * Rz(q): rotate the first two columns */
#pragma unroll
        for (int r = 0; r < 3; r++) {
            float a = R.m[r * 3], b = R.m[r * 3 + 1];
            R.m[r * 3] = c * a + s * b;
            R.m[r * 3 + 1] = -s * a + c * b;
        }
        k.R[j] = R;
        k.o[j] = o;
        PR = R;
        PO = o;
    }
}

/* ------------------------------------------------------------------- IK */
/* btMatrix3x3::getRotation */
__device__ __forceinline__ void mat_to_quat(const M3& M, float* q) {
    const float* m = M.m;
    float tr = m[0] + m[4] + m[8];
    if (tr > 0.0f) {
        float s = fast_sqrt(tr + 1.0f);
        q[3] = s * 0.5f;
        s = 0.5f * fast_rcp(s);
        q[0] = (m[7] - m[5]) * s;
        q[1] = (m[2] - m[6]) * s;
        q[2] = (m[3] - m[1]) * s;
    } else if (!(m[0] < m[4]) && !(m[0] < m[8])) { /* i = 0, j = 1, k = 2 */
        float s = fast_sqrt(m[0] - m[4] - m[8] + 1.0f);
        q[0] = s * 0.5f;
        s = 0.5f * fast_rcp(s);
        q[3] = (m[7] - m[5]) * s;
        q[1] = (m[3] + m[1]) * s;
        q[2] = (m[6] + m[2]) * s;
    } else if (m[0] < m[4] && !(m[4] < m[8])) { /* i = 1, j = 2, k = 0 */
        float s = fast_sqrt(m[4] - m[8] - m[0] + 1.0f);
        q[1] = s * 0.5f;
        s = 0.5f * fast_rcp(s);
        q[3] = (m[2] - m[6]) * s;
        q[2] = (m[7] + m[5]) * s;
        q[0] = (m[1] + m[3]) * s;
    } else { /* i = 2, j = 0, k = 1 */
        float s = fast_sqrt(m[8] - m[0] - m[4] + 1.0f);
        q[2] = s * 0.5f;
        s = 0.5f * fast_rcp(s);
        q[3] = (m[3] - m[1]) * s;
        q[0] = (m[2] + m[6]) * s;
        q[1] = (m[5] + m[7]) * s;
    }
}

/* In-register Cholesky solve of a 7x7 SPD system (lower triangle packed). */
__device__ __forceinline__ void chol7(float A[NJ][NJ]) {
#pragma unroll
    for (int j = 0; j < NJ; j++) {
        float s = A[j][j];
#pragma unroll
        for (int k = 0; k < j; k++) s -= A[j][k] * A[j][k];
        float inv = __builtin_amdgcn_rsqf(fmaxf(s, 1e-30f));
        A[j][j] = inv; /* the factor's diagonal is stored inverted */
#pragma unroll
        for (int i = j + 1; i < NJ; i++) {
            float t = A[i][j];
#pragma unroll
            for (int k = 0; k < j; k++) t -= A[i][k] * A[j][k];
            A[i][j] = t * inv;
        }
    }
}
__device__ __forceinline__ void chol7_solve(const float L[NJ][NJ], const float* b, float* x) {
    float y[NJ];
#pragma unroll
    for (int i = 0; i < NJ; i++) {
        float s = b[i];
#pragma unroll
        for (int k = 0; k < i; k++) s -= L[i][k] * y[k];
        y[i] = s * L[i][i];
    }
#pragma unroll
    for (int i = NJ - 1; i >= 0; i--) {
        float s = y[i];
#pragma unroll
        for (int k = i + 1; k < NJ; k++) s -= L[k][i] * x[k];
        x[i] = s * L[i][i];
    }
}

/* calculateInverseKinematics(link 11, pos, orn=[1,0,0,0]) as the reference
 * calls it (pybullet.py:478-484): Bullet's damped-least-squares IK with
 * orientation, <= ik_max_iters iterations from the current q while the
 * pre-update position error exceeds ik_residual; the IK point is the EE
 * link's joint pivot; dq = (J^T J + 0.5 I)^-1 J^T e clamped to max|dq|<=pi/4.
 * The orientation error angle is taken as 2*atan2(|v|, w) (== 2*acos(w) for a
 * unit quaternion, but well conditioned in fp32 for small angles). */
template <bool PAR = false>
__device__ __forceinline__ void ik(MPtr mp, const float* q0, V3 target, const float* torn, float* qout) {
    float qs[NJ];
#pragma unroll
    for (int j = 0; j < NJ; j++) qs[j] = q0[j];
    float diff = 1e30f;
    const int max_iters = mp->ik_max_iters;
    const float residual = mp->ik_residual;
    for (int it = 0; it < max_iters; it++) {
        if (!(diff > residual)) break;
        PGX_PROF_COUNT(17, 1);
        MRef m = *fresh(mp);
        Chain k;
        fk_chain<PAR>(m, qs, k);
        V3 x = k.o[6] + mulc(k.R[6], kEePivot);
        M3 Ree = mulm(k.R[6], kEeRot);
        float cq[4], dq[4];
        mat_to_quat(Ree, cq);
        /* dq = torn * conj(cq) */
        {
            const float ax = torn[0], ay = torn[1], az = torn[2], aw = torn[3];
            const float bx = -cq[0], by = -cq[1], bz = -cq[2], bw = cq[3];
            dq[0] = aw * bx + ax * bw + ay * bz - az * by;
            dq[1] = aw * by + ay * bw + az * bx - ax * bz;
            dq[2] = aw * bz + az * bw + ax * by - ay * bx;
            dq[3] = aw * bw - ax * bx - ay * by - az * bz;
        }
        float vn = fast_sqrt(dq[0] * dq[0] + dq[1] * dq[1] + dq[2] * dq[2]);
        float angle = 2.0f * atan2f(vn, dq[3]);
        if (angle > 3.14159265358979f) angle -= 6.28318530717959f;
        V3 axis = vn > 1e-30f ? (1.0f / vn) * v3(dq[0], dq[1], dq[2]) : v3(1.0f, 0.0f, 0.0f);
        V3 ep = target - x;
        V3 er = angle * axis;
        float A[NJ][NJ], g[NJ], dth[NJ];
        if constexpr (PAR) {
            /* the normal equations across the env's row: lane c < 7 holds Jacobian column c, forms
             * row c of J^T J (column b broadcast from lane b) and g_c, and the row broadcasts the
             * lower triangle back to every lane for the (redundant) Cholesky.  The same products
             * in the same order as the per-lane form below, so the same bits. */
            V3 zs[NJ], os[NJ];
#pragma unroll
            for (int j = 0; j < NJ; j++) { zs[j] = col(k.R[j], 2); os[j] = k.o[j]; }
            const V3 jwc = pick_v3(zs), jvc = cross(jwc, x - pick_v3(os));
            const float gc = dot(jvc, ep) + dot(jwc, er);
            float Ac[NJ];
            sfor<0, NJ>([&](auto bc) __attribute__((always_inline)) {
                constexpr int b = decltype(bc)::value;
                const V3 jvb = v3(bcast16<b>(jvc.x), bcast16<b>(jvc.y), bcast16<b>(jvc.z));
                const V3 jwb = v3(bcast16<b>(jwc.x), bcast16<b>(jwc.y), bcast16<b>(jwc.z));
                Ac[b] = dot(jvc, jvb) + dot(jwc, jwb);
            });
            sfor<0, NJ>([&](auto ac) __attribute__((always_inline)) {
                constexpr int a = decltype(ac)::value;
                g[a] = bcast16<a>(gc);
                sfor<0, a + 1>([&](auto bc) __attribute__((always_inline)) {
                    constexpr int b = decltype(bc)::value;
                    A[a][b] = bcast16<a>(Ac[b]);
                });
                A[a][a] += m.ik_damping;
            });
        } else {
            V3 jv[NJ], jw[NJ];
#pragma unroll
            for (int j = 0; j < NJ; j++) {
                jw[j] = col(k.R[j], 2);
                jv[j] = cross(jw[j], x - k.o[j]);
            }
#pragma unroll
            for (int a = 0; a < NJ; a++) {
                g[a] = dot(jv[a], ep) + dot(jw[a], er);
#pragma unroll
                for (int b = 0; b <= a; b++) A[a][b] = dot(jv[a], jv[b]) + dot(jw[a], jw[b]);
                A[a][a] += m.ik_damping;
            }
        }
        chol7(A);
        chol7_solve(A, g, dth);
        float mx = 0.0f;
#pragma unroll
        for (int j = 0; j < NJ; j++) mx = fmaxf(mx, fabsf(dth[j]));
        float sc = mx > m.ik_max_angle ? m.ik_max_angle * fast_rcp(mx) : 1.0f;
#pragma unroll
        for (int j = 0; j < NJ; j++) qs[j] += dth[j] * sc;
        diff = norm(x - target);
    }
#pragma unroll
    for (int j = 0; j < NJ; j++) qout[j] = qs[j];
}

/* --------------------------------------------------------------- physics */
/* ------------------------------------------------ ReachAO geometry (shared) */
constexpr int AO_N = PGX_AO_OBSTACLES;
constexpr float kAoSize = 0.05f, kAoMargin = 0.001f;
constexpr float kAoCubeBound = 0.0866025404f;   /* 0.05 * sqrt(3): cuboid circumradius */

/* AO collision-link slot of each capsule (-1: base, hand) */
__host__ __device__ constexpr int ao_slot(int c) {
    return kCapLink[c] < 0 ? -1 : (kCapLink[c] <= 7 ? kCapLink[c] : (kCapLink[c] == 9 ? 8 : -1));
}
__device__ constexpr int kAoSlot[PGX_NCAP] = {ao_slot(0), ao_slot(1), ao_slot(2), ao_slot(3), ao_slot(4),
                                              ao_slot(5), ao_slot(6), ao_slot(7), ao_slot(8), ao_slot(9),
                                              ao_slot(10), ao_slot(11), ao_slot(12), ao_slot(13)};
static_assert(PGX_NCAP == 14, "kAoSlot table");


/* signed distance to the axis-aligned box (c, h) */
__device__ __forceinline__ float box_sd(V3 P, V3 c, V3 h) {
    const float dx = fabsf(P.x - c.x) - h.x, dy = fabsf(P.y - c.y) - h.y, dz = fabsf(P.z - c.z) - h.z;
    const float ox = fmaxf(dx, 0.0f), oy = fmaxf(dy, 0.0f), oz = fmaxf(dz, 0.0f);
    return fast_sqrt(ox * ox + oy * oy + oz * oz) + fminf(fmaxf(dx, fmaxf(dy, dz)), 0.0f);
}

/* closest point of segment AB to C */
__device__ __forceinline__ V3 seg_closest(V3 A, V3 B, V3 C) {
    const V3 ab = B - A;
    const float l2 = dot(ab, ab);
    float t = l2 > 0.0f ? dot(C - A, ab) * fast_rcp(l2) : 0.0f;   /* (1 ulp; a true division is ~10 VALU) */
    t = fminf(fmaxf(t, 0.0f), 1.0f);
    return A + t * ab;
}

/* capsule (A, B, r) vs rounded box (c, full half extents hf): a golden-section search
 * on the inner box's signed distance along the axis, the signed distance returned; with NV
 * also the closest axis point P and the unit direction n from it towards the box (into the
 * box through the nearest face when P is inside the inner box) */
/* Does segment A + t ab, t in [0, 1], meet the box [lo, hi]?  (slab clipping) */
__device__ __forceinline__ bool seg_meets_box(V3 A, V3 ab, V3 lo, V3 hi) {
    float t0 = 0.0f, t1 = 1.0f;
    bool miss = false;
    const float a[3] = {A.x, A.y, A.z}, d[3] = {ab.x, ab.y, ab.z}, l[3] = {lo.x, lo.y, lo.z}, u[3] = {hi.x, hi.y, hi.z};
#pragma unroll
    for (int i = 0; i < 3; i++) {
        if (fabsf(d[i]) < 1e-20f) {
            miss = miss || a[i] < l[i] || a[i] > u[i];
        } else {
            const float inv = fast_rcp(d[i]);
            const float ta = (l[i] - a[i]) * inv, tb = (u[i] - a[i]) * inv;
            t0 = fmaxf(t0, fminf(ta, tb));
            t1 = fminf(t1, fmaxf(ta, tb));
        }
    }
    return !miss && t0 <= t1;
}
/* Closest point P of a segment that misses the box [lo, hi] (its distance is > 0): the squared
 * distance f(t) = |e(t)|^2, e = P(t) - clamp(P(t)), is convex and piecewise quadratic in t, its
 * pieces changing where a coordinate crosses a slab face (<= 6 breakpoints), so f'(t)/2 =
 * e(t).ab is continuous, non-decreasing and linear between breakpoints.  Evaluated at 0, 1 and
 * the breakpoints, the largest point with f' <= 0 and the smallest with f' >= 0 bound the piece
 * holding the minimiser, where linear interpolation of f' is exact: 8 evaluations, no search
 * (capsule_box_pair's golden section takes 34; pinned against brute force in
 * tests/test_gpu_reach_ao.py through the observation's distances and unit vectors). */
__device__ __forceinline__ V3 seg_box_closest(V3 A, V3 ab, V3 lo, V3 hi) {
    auto fprime = [&](float t) __attribute__((always_inline)) {
        const V3 P = A + t * ab;
        const float ex = P.x - fminf(fmaxf(P.x, lo.x), hi.x), ey = P.y - fminf(fmaxf(P.y, lo.y), hi.y),
                    ez = P.z - fminf(fmaxf(P.z, lo.z), hi.z);
        return ex * ab.x + ey * ab.y + ez * ab.z;
    };
    float tl = -1.0f, gl = 0.0f, th = 2.0f, gh = 0.0f;
    auto take = [&](float b) __attribute__((always_inline)) {
        const float g = fprime(b);
        if (g <= 0.0f && b > tl) { tl = b; gl = g; }
        if (g >= 0.0f && b < th) { th = b; gh = g; }
    };
    take(0.0f);
    take(1.0f);
    const float a[3] = {A.x, A.y, A.z}, d[3] = {ab.x, ab.y, ab.z}, l[3] = {lo.x, lo.y, lo.z}, u[3] = {hi.x, hi.y, hi.z};
#pragma unroll
    for (int i = 0; i < 3; i++) {
        if (fabsf(d[i]) >= 1e-20f) {
            const float inv = fast_rcp(d[i]);
            take(fminf(fmaxf((l[i] - a[i]) * inv, 0.0f), 1.0f));
            take(fminf(fmaxf((u[i] - a[i]) * inv, 0.0f), 1.0f));
        }
    }
    float t;
    if (tl < 0.0f) t = 0.0f;          /* f'(0) > 0: the minimum is at A */
    else if (th > 1.0f) t = 1.0f;
    else t = gh - gl > 0.0f ? tl - gl * (th - tl) * fast_rcp(gh - gl) : tl;
    t = fminf(fmaxf(t, fmaxf(tl, 0.0f)), fminf(th, 1.0f));
    return A + t * ab;
}

template <bool NV>
__device__ __forceinline__ float capsule_box_pair(V3 A, V3 B, float r, V3 c, V3 hf, V3* Pout, V3* nout) {
    const V3 h = v3(hf.x - kAoMargin, hf.y - kAoMargin, hf.z - kAoMargin);
    const V3 ab = B - A;
    float lo = 0.0f, hi = 1.0f;
    const bool seg = dot(ab, ab) > 0.0f;
    if (!seg_meets_box(A, ab, c - h, c + h)) {   /* outside: the exact closest pair (seg_box_closest) */
        const V3 P = seg_box_closest(A, ab, c - h, c + h);
        const V3 q = v3(fminf(fmaxf(P.x, c.x - h.x), c.x + h.x), fminf(fmaxf(P.y, c.y - h.y), c.y + h.y),
                        fminf(fmaxf(P.z, c.z - h.z), c.z + h.z));
        const V3 v = q - P;
        const float sd = norm(v);
        if (NV) {
            *Pout = P;
            *nout = sd > 0.0f ? fast_rcp(sd) * v : v3(0.0f, 0.0f, 0.0f);
        }
        return sd - kAoMargin - r;
    }
    if (seg) {   /* the segment enters the inner box: the signed distance by the search */
        /* golden-section search of the convex box_sd along the axis: one evaluation per step,
         * 34 steps shrink [0, 1] to 0.618^34 = 8e-8 (the ternary search's 40 steps of two
         * evaluations reach 9e-8) */
        const float gr = 0.61803398875f;
        float t1 = hi - gr * (hi - lo), t2 = lo + gr * (hi - lo);
        float f1 = box_sd(A + t1 * ab, c, h), f2 = box_sd(A + t2 * ab, c, h);
        for (int it = 0; it < 34; it++) {
            if (f1 <= f2) {
                hi = t2; t2 = t1; f2 = f1;
                t1 = hi - gr * (hi - lo);
                f1 = box_sd(A + t1 * ab, c, h);
            } else {
                lo = t1; t1 = t2; f1 = f2;
                t2 = lo + gr * (hi - lo);
                f2 = box_sd(A + t2 * ab, c, h);
            }
        }
    }
    V3 P = A + (seg ? 0.5f * (lo + hi) : 0.0f) * ab;
    float sd = box_sd(P, c, h);
    if (seg && sd > 0.0f) {
        /* two alternating projections (box -> segment): the search cannot resolve t where
         * the distance is flat to second order (a segment passing an edge or a corner);
         * each can only shorten the pair and pins it */
        for (int it = 0; it < 2; it++) {
            const V3 q = v3(fminf(fmaxf(P.x, c.x - h.x), c.x + h.x), fminf(fmaxf(P.y, c.y - h.y), c.y + h.y),
                            fminf(fmaxf(P.z, c.z - h.z), c.z + h.z));
            P = seg_closest(A, B, q);
        }
        sd = box_sd(P, c, h);
    }
    const float d = sd - kAoMargin - r;
    if (NV) {
        V3 n;
        if (sd > 0.0f) {
            const V3 q = v3(fminf(fmaxf(P.x, c.x - h.x), c.x + h.x), fminf(fmaxf(P.y, c.y - h.y), c.y + h.y),
                            fminf(fmaxf(P.z, c.z - h.z), c.z + h.z));
            const V3 v = q - P;
            const float len = norm(v);
            n = len > 0.0f ? fast_rcp(len) * v : v3(0.0f, 0.0f, 0.0f);
        } else {   /* inside the inner box: out through the nearest face */
            const float bx = fabsf(P.x - c.x) - h.x, by = fabsf(P.y - c.y) - h.y, bz = fabsf(P.z - c.z) - h.z;
            const int ax = (bx >= by && bx >= bz) ? 0 : (by >= bz ? 1 : 2);
            const float sx = P.x < c.x ? 1.0f : -1.0f, sy = P.y < c.y ? 1.0f : -1.0f, sz = P.z < c.z ? 1.0f : -1.0f;
            n = v3(ax == 0 ? sx : 0.0f, ax == 1 ? sy : 0.0f, ax == 2 ? sz : 0.0f);
        }
        *Pout = P;
        *nout = n;
    }
    return d;
}
/* the distance, and with VEC the unit vector from the capsule's closest point to the box's
 * (utils.unit_vector: pb - pa = d n) */
template <bool VEC>
__device__ __forceinline__ float capsule_box(V3 A, V3 B, float r, V3 c, V3 hf, V3* u) {
    V3 P, n;
    const float d = capsule_box_pair<VEC>(A, B, r, c, hf, &P, &n);
    if (VEC) *u = d > 0.0f ? n : (d < 0.0f ? (-1.0f) * n : v3(0.0f, 0.0f, 0.0f));
    return d;
}

/* capsule_box(...) <= thr as a decision (thr >= 0) */
__device__ __forceinline__ bool capsule_box_hit(V3 A, V3 B, float r, V3 c, V3 hf, float thr = 0.0f) {
    const V3 h = v3(hf.x - kAoMargin, hf.y - kAoMargin, hf.z - kAoMargin);
    const V3 ab = B - A;
    /* thr >= 0 in every use: a segment meeting the inner box is within it; one that misses it
     * has the exact (seg_box_closest) distance */
    if (seg_meets_box(A, ab, c - h, c + h)) return true;
    const V3 P = seg_box_closest(A, ab, c - h, c + h);
    const V3 q = v3(fminf(fmaxf(P.x, c.x - h.x), c.x + h.x), fminf(fmaxf(P.y, c.y - h.y), c.y + h.y),
                    fminf(fmaxf(P.z, c.z - h.z), c.z + h.z));
    return norm(q - P) - kAoMargin - r <= thr;
}

/* ReachAO's table box (table_top is its top face) */
__device__ __forceinline__ V3 ao_table_c(const PgxDevEnv& e) { return v3(e.table_cx, e.table_cy, e.table_top - e.table_hz); }
__device__ __forceinline__ V3 ao_table_h(const PgxDevEnv& e) { return v3(e.table_hx, e.table_hy, e.table_hz); }

/* ------------------------------------------------------------- contacts */
/* Restated in oracle/pgx_oracle.c ("world: object + contacts"): Bullet's manifold rule (at
 * most 4 points per colliding pair: a capsule against the table, the plane, the object or an
 * obstacle; the object against the table or the plane), then a row budget per group -- the
 * CG deepest object-scene points and the RB deepest robot points (RB: robot_budget below) --
 * rows ordered by feature id; normal rows use ERP / speculative rhs, two friction rows per
 * point along btPlaneSpace1(n) bounded by mu * normal impulse.
 * Per-env contact data lives in LDS, lane-minor (x[...][lane]): conflict-free and
 * dynamically indexable, unlike VGPRs.  Solver rows are float4 records with a 16-B lane
 * stride, so each quad is one conflict-free ds_read_b128 (MI355X_MICROARCH.md, LDS). */
constexpr int CG = PGX_OBJECT_POINTS;   /* object-scene budget; robot points whose rows live in VGPRs */
constexpr int MANIFOLD = 4;             /* btPersistentManifold MANIFOLD_CACHE_SIZE: points per pair */
/* ReachAO's obstacle pairs through Bullet's persistent manifolds (PGX_AO_FRESH: round 4's fresh
 * per-substep candidates instead -- an A/B build only, the oracle's PGX_FLAG_FRESH_MANIFOLD) */
#ifdef PGX_AO_FRESH
constexpr bool AO_PERS = false;
#else
constexpr bool AO_PERS = true;
#endif

/* Capsule c's contact breaking threshold against the table / plane / cube / an obstacle (PgxDevModel
 * tau_*: Bullet's relative per-pair rule, pgx.h contact_distance), selected from the block by
 * compile-time index -- folded to constants in the default build, where the cube and obstacle pairs
 * take one value for every capsule (the scene body's disc is the smaller) */
enum { TAU_TABLE = 0, TAU_PLANE = 1, TAU_OBJ = 2, TAU_OBST = 3 };
template <int W>
__device__ __forceinline__ float tau_at(MRef m, int k) {
    return W == TAU_TABLE ? m.tau_table[k] : W == TAU_PLANE ? m.tau_plane[k] : W == TAU_OBJ ? m.tau_obj[k] : m.tau_obst[k];
}
template <int W>
__device__ __forceinline__ float cap_tau(MRef m, int c) {
    float v = tau_at<W>(m, 0);
    sfor<1, PGX_NCAP>([&](auto kc) __attribute__((always_inline)) {
        constexpr int K = decltype(kc)::value;
        v = c == K ? tau_at<W>(m, K) : v;
    });
    return v;
}

/* robot points kept per env: the one-lane layout holds its rows in LDS for 64 envs (4); the
 * wide layout 4 in VGPRs, and with FULL (PGX_FLAG_FULL_MANIFOLD) the rest, up to
 * PGX_ROBOT_POINTS / _ARM, in LDS (substep_g's "extra rows") */
template <int W, int OBJ, int FULL>
constexpr int robot_budget() {
    return (W == 64 || !FULL) ? PGX_ROBOT_POINTS_ONE_LANE : (OBJ ? PGX_ROBOT_POINTS : PGX_ROBOT_POINTS_ARM);
}
static_assert(PGX_ROBOT_POINTS_ONE_LANE == CG, "the one-lane solver holds CG robot points");
/* robot points whose rows live in VGPRs as Delassus lanes (the rest are substep_g's extra rows,
 * a 16-lane reduction each): CG, and PGX_CGR_OBJ for the object tasks' per-pair budget kernels,
 * whose heavy envs (fingers on the cube: 5-7 points, profiles/r05/point_hist.log) set the launch */
#ifndef PGX_CGR_OBJ
#define PGX_CGR_OBJ 6
#endif
/* the arm tasks' per-pair budget kernels (Reach, ReachAO): four -- eight measured slower (the
 * rows' build), and two too: the launches whose waves hold 3-5 points then run reduction rows
 * (Reach 4096 0.390 -> 0.400 ms, ReachAO 8192 0.777 -> 0.984 ms; profiles/r05/ab_register_points_*) */
#ifndef PGX_CGR_ARM
#define PGX_CGR_ARM 4
#endif
static_assert(PGX_CGR_ARM >= 2 && PGX_CGR_OBJ >= 2, "the sweeps' point counts are 0, 2, 4 (<= the register budget)");
template <int W, int OBJ, int FULL>
constexpr int robot_regs() {
    return (W != 64 && FULL) ? (OBJ ? PGX_CGR_OBJ : PGX_CGR_ARM) : CG;
}

constexpr int CACHE_N = 2 * PGX_CONTACT_SLOTS;
constexpr int CACHE1 = 2 * CG;           /* robot slots of the cache */
constexpr float kTableIdLimit = 32.0f;   /* robot feature ids < 32: capsule end vs table/plane */
static_assert(PGX_NCAP <= 16, "PgxDevModel.cap_mu holds 16 capsules");

/* Combined lateral friction of a robot contact point: its capsule's link against the other body
 * (PgxDevModel.cap_mu: pgx_sim_params.link_friction -- 0.25, and 0.5 for panda_ee, whose lateral
 * friction Panda.__init__ raises to 1.0, panda.py:69-70).  The capsule from the feature id: table /
 * plane 2c + end, cube 32 + 16c + sample, obstacle 32 + 6c + obstacle (AO).  In the default build
 * the table is a compile-time constant, so the chain folds to the capsules that differ from the
 * cube's pair (m.friction). */
template <int AO, int FULL = 0>
__device__ __forceinline__ float point_mu(MRef m, float id) {
    /* (FULL with AO_PERS: ReachAO's manifold points 32 + 24 c + 4 o + slot; the PGX_AO_FRESH A/B build's
     * fresh candidates and the one-lane layout 32 + 6 c + o; the cube's 32 + 16 c + slot) */
    const float cf = id < kTableIdLimit ? id * 0.5f
                   : (id - kTableIdLimit) * (AO ? ((FULL && AO_PERS) ? (1.0f / 24.0f) : (1.0f / 6.0f)) : 0.0625f);
    const int cap = (int)(cf + 1e-3f);   /* (ids are exact small integers; the margin covers 1/6's rounding) */
    float mu = m.friction;
    sfor<0, PGX_NCAP>([&](auto kc) __attribute__((always_inline)) {
        constexpr int K = decltype(kc)::value;
        mu = cap == K ? m.cap_mu[K] : mu;
    });
    return mu;
}

template <int W, int OBJ = 1, int FULL = 0>
struct ContactLdsT {
    static constexpr int RB = robot_budget<W, OBJ, FULL>();
    /* wide layout: rows 3 p + dir of point p (object-scene points first when OBJ): the
     * register rows (NQR, robot points < CG) and every row (NQX, robot points < RB) */
    static constexpr int P0 = OBJ ? CG : 0;
    static constexpr int CGR = robot_regs<W, OBJ, FULL>();   /* robot points in registers */
    static constexpr int NQR = 3 * (P0 + CGR), NQX = 3 * (P0 + RB);
    static constexpr int XR = (W == 64 || RB <= CGR) ? 1 : NQX - NQR;   /* extra rows */
    /* Bullet's persistent manifolds of the robot's cube / obstacle pairs (FULL, the wide layout): the
     * pool's capacity in points (pgx.h PGX_MANIFOLD_POOL / _AO; Reach has no such pair) */
    static constexpr int MP = (W == 64 || !FULL) ? 1 : (OBJ ? PGX_MANIFOLD_POOL : PGX_MANIFOLD_POOL_AO);
    /* the object-scene arrays exist in the object tasks' layouts only (ReachAO's two-wave kernel
     * fits its LDS budget without them) */
    static constexpr int G0 = (W == 64 || OBJ) ? CG : 1;
    /* group 0: object vertices vs the table box / the plane top (round 6: the table's side walls too) */
    float4 g0q[G0][4][W];         /* [0] = contact point - object COM; [1 + dir] = (jinv, den, rhs, lambda) */
    float g0d[G0][W], g0id[G0][W];
    float g0n[G0][3][W];          /* the contact normal, from the table / plane to the cube */
    /* group 1: robot vs table / plane / object / obstacles */
    float g1p[RB][3][W];          /* point on the robot */
    float g1n[RB][3][W];          /* normal, from the other body to the robot */
    float g1rb[RB][3][W];         /* object contacts: point on the object - object COM */
    float g1d[RB][W], g1id[RB][W];
    int g1j[RB][W];               /* arm joint carrying the robot link */
    int g1w[RB][W];               /* a manifold point's pool index (its warm start and write-back), -1 else */
    /* the manifold pool per env (pgx.h PGX_MANIFOLD_POOL): count, then per point kid (key + slot),
     * local A (the carrying joint's frame), local B (cube frame / world), normal on B (world),
     * distance (the last refresh's), applied normal impulse */
    int mcnt[W];
    float mkid[MP][W], mla[MP][3][W], mlb[MP][3][W], mn[MP][3][W], md[MP][W], mimp[MP][W];
    /* one-lane layout, per direction: (J0..3) (J4..6, jinv) (R0..3) (R4..6, den) (cl, rhs) (ca, lambda)
     * with J the robot Jacobian row, R = M^-1 J^T, (cl, ca) the object part (0 against the table) */
    float4 g1q[W == 64 ? CG : 1][3][6][W == 64 ? W : 1];
    int cnt[2][W];
    float cache[CACHE_N][W];      /* (feature id, normal impulse): CG object-scene slots, then robot slots */
    float capA[PGX_NCAP][3][W], capB[PGX_NCAP][3][W];   /* capsule end points, world */
    /* ReachAO: obstacle centres, per collision link the closest distance and unit vector */
    float aoC[PGX_AO_OBSTACLES][3][W];
    float aoD[PGX_AO_LINKS][W], aoU[PGX_AO_LINKS][3][W];
    /* wide layout: the register rows' J (13 coordinates) and M^-1 J^T (arm part) per env,
     * row-major [row q][coordinate], so lane q reads its row back with ds_read_b128 (a transpose);
     * J stays through the sweeps (the register rows' velocities after an extra-row block) */
    float4 wJ[W == 64 ? 1 : W][W == 64 ? 1 : NQR][4], wR[W == 64 ? 1 : W][W == 64 ? 1 : NQR][2];
    /* the extra rows (robot points CG..RB-1) for the whole solve: per coordinate lane c the
     * pair (J_c, (M^-1 J^T)_c jinv), one ds_read_b64; per row rhs', lambda', lambda' at the
     * solve's start, the friction bound factor fk and jinv */
    float2 xd[(W == 64 || XR == 1) ? 1 : W][XR][16];
    float xrhs[XR][W], xlam[XR][W], xlam0[XR][W], xfk[XR][W], xjinv[XR][W];
    /* wide layout, the register points' normal rows: jinv (the cache's impulse lambda' jinv)
     * and lambda' at the solve's start (a redo), kept here through the sweeps */
    float pjn[W == 64 ? 1 : P0 + CGR][W], pl0[W == 64 ? 1 : P0 + CGR][W];
    /* wide layout, object tasks: the limit rows' rhs' and lambda' of the all-rows solve (in
     * registers beside the 24 contact rows they set the kernel's register peak) */
    float lrhs[(W == 64 || !OBJ) ? 1 : PGX_N_ROWS - PGX_NJ][W], llam[(W == 64 || !OBJ) ? 1 : PGX_N_ROWS - PGX_NJ][W];
    /* wide layout: state that lives across the substep loop but is read once per substep or after
     * it, parked here instead of in registers (the motor targets; the substeps' start poses,
     * double-buffered: getLinkState's cached pose is the last completed substep's start) */
    float ltq[W == 64 ? 1 : PGX_NJ][W], lqs[W == 64 ? 1 : 2][W == 64 ? 1 : PGX_NJ][W];
    float lkc[W == 64 ? 1 : 16][W == 64 ? 1 : 16];   /* the lane constants (LaneK fields x lane c) */
    /* wide layout: what waits for the end of the constraint solve -- q, the unconstrained joint
     * velocities vu, the object's position and orientation and its unconstrained velocities
     * (27 floats, row-uniform) -- parked through the sweeps (PARK_SOLVE) */
    float psv[W == 64 ? 1 : 27][W == 64 ? 1 : W];
    /* one-lane speculative solve: the sweep's start velocities (dv, dvl, dvw) for a redo */
    float spec0[W == 64 ? NJ + 6 : 1][W == 64 ? W : 1];
};
using ContactLds = ContactLdsT<64>;   /* one env per lane */
template <int OBJ, int FULL>
using ContactLdsGT = ContactLdsT<EPW, OBJ, FULL>;

/* The warm start of feature id: factor x the impulse of the cache slot holding id among slots
 * first .. first + N - 1 (the last match, as the oracle's loop; 0 without).  Every slot is read
 * unconditionally and selected, so the reads issue together behind one wait instead of a
 * compare-branch-read chain per slot. */
template <int N, class LT>
__device__ __forceinline__ float warm_lookup(const LT& L, int ln, int first, float id, float factor) {
    float warm = 0.0f;
#pragma unroll
    for (int s = 0; s < N; s++) {
        const float sid = L.cache[first + 2 * s][ln], imp = L.cache[first + 2 * s + 1][ln];
        warm = sid == id ? factor * imp : warm;
    }
    return warm;
}

struct ObjState {
    V3 p, v, w;
    float qx, qy, qz, qw;
};

/* btPlaneSpace1 */
__device__ __forceinline__ void plane_space(V3 n, V3& p, V3& q) {
    if (fabsf(n.z) > 0.70710678f) {
        float a = n.y * n.y + n.z * n.z, k = __builtin_amdgcn_rsqf(a);
        p = v3(0.0f, -n.z * k, n.y * k);
        q = v3(a * k, -n.x * p.z, n.x * p.y);
    } else {
        float a = n.x * n.x + n.y * n.y, k = __builtin_amdgcn_rsqf(a);
        p = v3(-n.y * k, n.x * k, 0.0f);
        q = v3(-n.z * p.y, n.z * p.x, a * k);
    }
}

__device__ __forceinline__ bool on_table(const PgxDevEnv& e, float x, float y) {
    return fabsf(x - e.table_cx) <= e.table_hx && fabsf(y - e.table_cy) <= e.table_hy;
}
__device__ __forceinline__ float ground_z(const PgxDevEnv& e, float x, float y) {
    return on_table(e, x, y) ? e.table_top : e.plane_z;
}
/* A cube vertex P against the table box (oracle vertex_vs_table, the same rule in fp32): its signed
 * distance and the normal from the box to P.  Inside, the face of least penetration (the top, then
 * x, then y on a tie); outside, the closest point of the box -- one face's distance (the top:
 * exactly P.z - top) when only one coordinate lies outside the box's slab. */
__device__ __forceinline__ float vertex_vs_table(const PgxDevEnv& e, V3 P, V3& n) {
    const float bot = e.table_top - 2.0f * e.table_hz;
    const float qx = P.x - e.table_cx, qy = P.y - e.table_cy;
    const float ex = fabsf(qx) - e.table_hx, ey = fabsf(qy) - e.table_hy;
    const float up = P.z - e.table_top, dn = bot - P.z;
    const bool top = up >= dn;
    const float ez = top ? up : dn;
    const float sx = qx < 0.0f ? -1.0f : 1.0f, sy = qy < 0.0f ? -1.0f : 1.0f, sz = top ? 1.0f : -1.0f;
    if (ex <= 0.0f && ey <= 0.0f && ez <= 0.0f) {
        if (ez >= ex && ez >= ey) { n = v3(0.0f, 0.0f, sz); return ez; }
        if (ex >= ey) { n = v3(sx, 0.0f, 0.0f); return ex; }
        n = v3(0.0f, sy, 0.0f);
        return ey;
    }
    const float ox = fmaxf(ex, 0.0f), oy = fmaxf(ey, 0.0f), oz = fmaxf(ez, 0.0f);
    if (ox == 0.0f && oy == 0.0f) { n = v3(0.0f, 0.0f, sz); return oz; }
    if (oy == 0.0f && oz == 0.0f) { n = v3(sx, 0.0f, 0.0f); return ox; }
    if (ox == 0.0f && oz == 0.0f) { n = v3(0.0f, sy, 0.0f); return oy; }
    const float d = sqrtf(ox * ox + oy * oy + oz * oz);
    const float inv = 1.0f / d;
    n = v3(sx * ox * inv, sy * oy * inv, sz * oz * inv);
    return d;
}

/* keep the CG deepest candidates of group 0 (stable: an equal depth does not displace) */
template <class LT>
__device__ __forceinline__ void g0_insert(LT& L, int ln, float d, float id, V3 r, V3 n) {
    int c = L.cnt[0][ln], pos;
    if (c < CG) { pos = c; L.cnt[0][ln] = c + 1; }
    else if (d < L.g0d[CG - 1][ln]) pos = CG - 1;
    else return;
    while (pos > 0 && d < L.g0d[pos - 1][ln]) {
        L.g0d[pos][ln] = L.g0d[pos - 1][ln];
        L.g0id[pos][ln] = L.g0id[pos - 1][ln];
        L.g0q[pos][0][ln] = L.g0q[pos - 1][0][ln];
        for (int k = 0; k < 3; k++) L.g0n[pos][k][ln] = L.g0n[pos - 1][k][ln];
        pos--;
    }
    L.g0d[pos][ln] = d; L.g0id[pos][ln] = id;
    L.g0q[pos][0][ln] = make_float4(r.x, r.y, r.z, 0.0f);
    L.g0n[pos][0][ln] = n.x; L.g0n[pos][1][ln] = n.y; L.g0n[pos][2][ln] = n.z;
}
template <class LT>
__device__ __forceinline__ void g1_copy(LT& L, int ln, int to, int from) {
    L.g1d[to][ln] = L.g1d[from][ln];
    L.g1id[to][ln] = L.g1id[from][ln];
    L.g1j[to][ln] = L.g1j[from][ln];
    L.g1w[to][ln] = L.g1w[from][ln];
    for (int k = 0; k < 3; k++) {
        L.g1p[to][k][ln] = L.g1p[from][k][ln];
        L.g1n[to][k][ln] = L.g1n[from][k][ln];
        L.g1rb[to][k][ln] = L.g1rb[from][k][ln];
    }
}
template <class LT>
__device__ __forceinline__ void g1_insert(LT& L, int ln, float d, float id, int j, V3 p, V3 n, V3 rb, int w = -1) {
    constexpr int RB = LT::RB;   /* the robot group's budget: its RB deepest */
    int c = L.cnt[1][ln], pos;
    if (c < RB) { pos = c; L.cnt[1][ln] = c + 1; }
    else if (d < L.g1d[RB - 1][ln]) pos = RB - 1;
    else return;
    while (pos > 0 && d < L.g1d[pos - 1][ln]) { g1_copy(L, ln, pos, pos - 1); pos--; }
    L.g1d[pos][ln] = d; L.g1id[pos][ln] = id; L.g1j[pos][ln] = j; L.g1w[pos][ln] = w;
    L.g1p[pos][0][ln] = p.x; L.g1p[pos][1][ln] = p.y; L.g1p[pos][2][ln] = p.z;
    L.g1n[pos][0][ln] = n.x; L.g1n[pos][1][ln] = n.y; L.g1n[pos][2][ln] = n.z;
    L.g1rb[pos][0][ln] = rb.x; L.g1rb[pos][1][ln] = rb.y; L.g1rb[pos][2][ln] = rb.z;
}
/* group 1 by depth (stable insertion sort of <= RB entries) */
template <class LT>
__device__ __forceinline__ void sort_g1_by_depth(LT& L, int ln) {
    const int c1 = L.cnt[1][ln];
    for (int i = 1; i < c1; i++)
        for (int j = i; j > 0 && L.g1d[j][ln] < L.g1d[j - 1][ln]; j--) {
            float d = L.g1d[j][ln], id = L.g1id[j][ln];
            int jj = L.g1j[j][ln], ww = L.g1w[j][ln];
            float p[3], n[3], rb[3];
            for (int k = 0; k < 3; k++) { p[k] = L.g1p[j][k][ln]; n[k] = L.g1n[j][k][ln]; rb[k] = L.g1rb[j][k][ln]; }
            g1_copy(L, ln, j, j - 1);
            L.g1d[j - 1][ln] = d; L.g1id[j - 1][ln] = id; L.g1j[j - 1][ln] = jj; L.g1w[j - 1][ln] = ww;
            for (int k = 0; k < 3; k++) { L.g1p[j - 1][k][ln] = p[k]; L.g1n[j - 1][k][ln] = n[k]; L.g1rb[j - 1][k][ln] = rb[k]; }
        }
}
/* rows are ordered by feature id (insertion sort of <= CG / RB entries) */
template <class LT>
__device__ __forceinline__ void sort_groups(LT& L, int ln) {
    const int c0 = L.cnt[0][ln];
    for (int i = 1; i < c0; i++)
        for (int j = i; j > 0 && L.g0id[j][ln] < L.g0id[j - 1][ln]; j--) {
            float t = L.g0id[j][ln]; L.g0id[j][ln] = L.g0id[j - 1][ln]; L.g0id[j - 1][ln] = t;
            t = L.g0d[j][ln]; L.g0d[j][ln] = L.g0d[j - 1][ln]; L.g0d[j - 1][ln] = t;
            const float4 tq = L.g0q[j][0][ln]; L.g0q[j][0][ln] = L.g0q[j - 1][0][ln]; L.g0q[j - 1][0][ln] = tq;
            for (int k = 0; k < 3; k++) {
                const float tn = L.g0n[j][k][ln]; L.g0n[j][k][ln] = L.g0n[j - 1][k][ln]; L.g0n[j - 1][k][ln] = tn;
            }
        }
    const int c1 = L.cnt[1][ln];
    for (int i = 1; i < c1; i++)
        for (int j = i; j > 0 && L.g1id[j][ln] < L.g1id[j - 1][ln]; j--) {
            float d = L.g1d[j][ln], id = L.g1id[j][ln];
            int jj = L.g1j[j][ln], ww = L.g1w[j][ln];
            float p[3], n[3], rb[3];
            for (int k = 0; k < 3; k++) { p[k] = L.g1p[j][k][ln]; n[k] = L.g1n[j][k][ln]; rb[k] = L.g1rb[j][k][ln]; }
            g1_copy(L, ln, j, j - 1);
            L.g1d[j - 1][ln] = d; L.g1id[j - 1][ln] = id; L.g1j[j - 1][ln] = jj; L.g1w[j - 1][ln] = ww;
            for (int k = 0; k < 3; k++) { L.g1p[j - 1][k][ln] = p[k]; L.g1n[j - 1][k][ln] = n[k]; L.g1rb[j - 1][k][ln] = rb[k]; }
        }
}

/* object-frame helpers: R(q) v and R(q)^T v for the unit quaternion (x,y,z,w) */
__device__ __forceinline__ M3 quat_mat(const ObjState& o) {
    const float x = o.qx, y = o.qy, z = o.qz, w = o.qw;
    return M3{{1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w),
               2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w),
               2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)}};
}
__device__ __forceinline__ V3 mul_t(const M3& A, V3 v) {
    return v3(A.m[0] * v.x + A.m[3] * v.y + A.m[6] * v.z, A.m[1] * v.x + A.m[4] * v.y + A.m[7] * v.z,
              A.m[2] * v.x + A.m[5] * v.y + A.m[8] * v.z);
}

/* capsule c's spheres against the object (robot_contacts' object branch): the cull (segment
 * farther from the object centre than r + h sqrt(3) + tau) unless the caller already did it */
template <class LT>
__device__ __forceinline__ void object_candidates(const PgxDevEnv& e, float tau, LT& L, int ln, const ObjState& ob,
                                                  const M3& Rc, int c, bool cull) {
    const V3 A = v3(L.capA[c][0][ln], L.capA[c][1][ln], L.capA[c][2][ln]);
    const V3 B = v3(L.capB[c][0][ln], L.capB[c][1][ln], L.capB[c][2][ln]);
    const float r = kCapR[c];
    const int jc = kCapJ[c], ns = kCapNs[c];
    const float h = e.obj_half;
    const V3 ab = B - A;
    if (cull) {
        const float l2 = dot(ab, ab);
        float t = l2 > 0.0f ? dot(ob.p - A, ab) * fast_rcp(l2) : 0.0f;
        t = fminf(fmaxf(t, 0.0f), 1.0f);
        const V3 cp = A + t * ab - ob.p;
        const float reach = r + 1.7320508f * h + tau;
        if (!(dot(cp, cp) < reach * reach)) return;
    }
    const float inv_n = ns > 1 ? 1.0f / (float)(ns - 1) : 0.0f;
    /* Bullet's manifold rule: the capsule x object pair keeps at most MANIFOLD points, its
     * deepest by (depth, sample); with a robot budget above MANIFOLD that cap binds first, so
     * a depth-only pass finds the pair's MANIFOLD-th key (ds, ss) and only samples up to it
     * are inserted.  Depth here is the same expression as below (bit-identical). */
    float dcut = 3.0e38f;
    int scut = 1 << 20;
    if (LT::RB > MANIFOLD && ns > MANIFOLD) {
        float kd[MANIFOLD];
        int ks[MANIFOLD];
#pragma unroll
        for (int t = 0; t < MANIFOLD; t++) { kd[t] = 3.0e38f; ks[t] = 1 << 20; }
        for (int s = 0; s < ns; s++) {
            const V3 C = A + ((float)s * inv_n) * ab;
            const V3 cl = mul_t(Rc, C - ob.p);
            const V3 qb = v3(fminf(fmaxf(cl.x, -h), h), fminf(fmaxf(cl.y, -h), h), fminf(fmaxf(cl.z, -h), h));
            const V3 diff = cl - qb;
            const float d2 = dot(diff, diff);
            float depth;
            if (d2 > 1e-24f) depth = fast_sqrt(d2) - r;
            else depth = -fminf(fminf(h - fabsf(cl.x), h - fabsf(cl.y)), h - fabsf(cl.z)) - r;
            if (!(depth < tau)) continue;
            /* insert (depth, s) into the sorted top-MANIFOLD (a later s never displaces an equal depth) */
            float dv = depth;
            int sv = s;
#pragma unroll
            for (int t = 0; t < MANIFOLD; t++) {
                const bool lt = dv < kd[t];
                const float td = kd[t];
                const int ts = ks[t];
                kd[t] = lt ? dv : td; ks[t] = lt ? sv : ts;
                dv = lt ? td : dv; sv = lt ? ts : sv;
            }
        }
        dcut = kd[MANIFOLD - 1];
        scut = ks[MANIFOLD - 1];
    }
    for (int s = 0; s < ns; s++) {
        const V3 C = A + ((float)s * inv_n) * ab;
        const V3 cl = mul_t(Rc, C - ob.p);
        V3 qb = v3(fminf(fmaxf(cl.x, -h), h), fminf(fmaxf(cl.y, -h), h), fminf(fmaxf(cl.z, -h), h));
        const V3 diff = cl - qb;
        const float d2 = dot(diff, diff);
        V3 nl;
        float depth;
        if (d2 > 1e-24f) {
            const float dist = fast_sqrt(d2);
            nl = fast_rcp(dist) * diff;
            depth = dist - r;
        } else { /* centre inside the box: out through the nearest face */
            const float bx = h - fabsf(cl.x), by = h - fabsf(cl.y), bz = h - fabsf(cl.z);
            int ax = 0;
            float best = bx;
            if (by < best) { best = by; ax = 1; }
            if (bz < best) { best = bz; ax = 2; }
            const float sx = cl.x < 0.0f ? -1.0f : 1.0f, sy = cl.y < 0.0f ? -1.0f : 1.0f,
                        sz = cl.z < 0.0f ? -1.0f : 1.0f;
            nl = v3(ax == 0 ? sx : 0.0f, ax == 1 ? sy : 0.0f, ax == 2 ? sz : 0.0f);
            if (ax == 0) qb.x = sx * h;
            if (ax == 1) qb.y = sy * h;
            if (ax == 2) qb.z = sz * h;
            depth = -best - r;
        }
        if (depth < tau && (depth < dcut || (depth == dcut && s <= scut))) {
            const V3 n = mul(Rc, nl);
            g1_insert(L, ln, depth, (float)(32 + 16 * c + s), jc, C - r * n, n, mul(Rc, qb));
        }
    }
}

/* object_candidates in the wide layout, lane-parallel: capsule cn (wave-uniform) against the
 * object, lane s of the env's row evaluating sample s (<= 13 per capsule) -- one pass instead of
 * every lane walking every sample twice.  The same candidates and order: Bullet's manifold rule
 * keeps the pair's MANIFOLD deepest by (depth, sample), ranked by broadcast; they are inserted
 * (g1_insert) in sample order, every lane of the env reading the candidate lane's values.
 * env_near: this env's cull (robot_contacts' segment test) passed for the capsule. */
template <class LT>
__device__ __forceinline__ void object_candidates_g(const PgxDevEnv& e, float tau, LT& L, int es, const ObjState& ob,
                                                    const M3& Rc, int cn, int c, bool env_near) {
    static_assert(PGX_NCAP <= 16, "capsule table");
    const V3 A = lds3(L.capA[cn], es), B = lds3(L.capB[cn], es);
    const float r = kCapR[cn];
    const int jc = kCapJ[cn], ns = kCapNs[cn];
    const float h = e.obj_half;
    const V3 ab = B - A;
    const float inv_n = ns > 1 ? 1.0f / (float)(ns - 1) : 0.0f;
    const V3 C = A + ((float)c * inv_n) * ab;
    const V3 cl = mul_t(Rc, C - ob.p);
    V3 qb = v3(fminf(fmaxf(cl.x, -h), h), fminf(fmaxf(cl.y, -h), h), fminf(fmaxf(cl.z, -h), h));
    const V3 diff = cl - qb;
    const float d2 = dot(diff, diff);
    V3 nl;
    float depth;
    if (d2 > 1e-24f) {
        const float dist = fast_sqrt(d2);
        nl = fast_rcp(dist) * diff;
        depth = dist - r;
    } else { /* centre inside the box: out through the nearest face */
        const float bx = h - fabsf(cl.x), by = h - fabsf(cl.y), bz = h - fabsf(cl.z);
        int ax = 0;
        float best = bx;
        if (by < best) { best = by; ax = 1; }
        if (bz < best) { best = bz; ax = 2; }
        const float sx = cl.x < 0.0f ? -1.0f : 1.0f, sy = cl.y < 0.0f ? -1.0f : 1.0f, sz = cl.z < 0.0f ? -1.0f : 1.0f;
        nl = v3(ax == 0 ? sx : 0.0f, ax == 1 ? sy : 0.0f, ax == 2 ? sz : 0.0f);
        if (ax == 0) qb.x = sx * h;
        if (ax == 1) qb.y = sy * h;
        if (ax == 2) qb.z = sz * h;
        depth = -best - r;
    }
    const bool cand = env_near && c < ns && depth < tau;
    bool keep = cand;
    if constexpr (LT::RB > MANIFOLD) {   /* the pair's MANIFOLD deepest by (depth, sample) */
        const float dd = cand ? depth : 3.0e38f;
        int rank = 0;
        sfor<0, 16>([&](auto uc) __attribute__((always_inline)) {
            constexpr int U = decltype(uc)::value;
            const float du = bcast16<U>(dd);
            rank += (du < dd || (du == dd && U < c)) ? 1 : 0;
        });
        keep = cand && rank < MANIFOLD;
    }
    const uint64_t bm = __ballot(keep);
    if (bm == 0) return;
    unsigned wm = __builtin_amdgcn_readfirstlane((unsigned)((bm | (bm >> 16) | (bm >> 32) | (bm >> 48)) & 0xFFFFu));
    const V3 n = mul(Rc, nl);
    const V3 pa = C - r * n, rb = mul(Rc, qb);
    const int row0 = (int)(threadIdx.x & ~(unsigned)(GW - 1));
    while (wm) {   /* in sample order, as the sequential walk inserts them */
        const int k = __builtin_ctz(wm);
        wm &= wm - 1u;
        const int src = row0 + k;
        const bool ck = __shfl((int)keep, src) != 0;
        const float dk = __shfl(depth, src);
        const V3 pk = v3(__shfl(pa.x, src), __shfl(pa.y, src), __shfl(pa.z, src));
        const V3 nk = v3(__shfl(n.x, src), __shfl(n.y, src), __shfl(n.z, src));
        const V3 rk = v3(__shfl(rb.x, src), __shfl(rb.y, src), __shfl(rb.z, src));
        if (ck) g1_insert(L, es, dk, (float)(32 + 16 * cn + k), jc, pk, nk, rk);
    }
}

/* ---- Bullet's persistent manifolds in the wide layout (FULL kernels, the robot's pairs with the cube
 * or the obstacles): the oracle's man_add / pool_refresh (oracle/pgx_oracle.c)
 * with the same rules and order, in fp32.  The per-env steps (a merge, the insertion into the row
 * list) run on every lane of the env's row with the same values (LDS reads, identical writes); the
 * refresh runs lane-parallel, lane p of the row refreshing pool point p. */
template <int AO>
__device__ __forceinline__ int man_capsule(int key) { return AO ? (key - 32) / 24 : (key - 32) / 16; }

/* addContactPoint of the new point (la, lb, n, d) to manifold `key` of env es's pool: getCacheEntry
 * (the cached point nearest in A's frame, strictly within thr^2, first in slot order) -> its fields
 * replaced, impulse kept; else appended below 4 points (dropped when the pool is full); else
 * sortCachedPoints' slot overwritten, impulse 0 */
template <class LT>
__device__ __forceinline__ void man_add_g(LT& L, int es, int c, int key, V3 la, V3 lb, V3 n, float d, float thr2) {
    constexpr int MP = LT::MP;
    const int cnt = L.mcnt[es];
    /* lane p of the row looks at pool point p: the manifold's points by slot from the row's ballots */
    const int p = c < cnt ? c : 0;
    const int kidp = (int)L.mkid[p][es];
    const bool match = c < cnt && (kidp & ~3) == key;
    const V3 lap = lds3(L.mla[p], es);
    const float dp = L.md[p][es];
    const V3 e = lap - la;
    const float ddp = dot(e, e);
    const int row0 = (int)(threadIdx.x & ~(unsigned)(GW - 1));
    int idx[4], nk = 0;
#pragma unroll
    for (int sl = 0; sl < 4; sl++) {
        const unsigned m = row_ballot(match && (kidp & 3) == sl);
        idx[sl] = m ? __builtin_ctz(m) : 0;
        nk += m ? 1 : 0;
    }
    /* getCacheEntry: the nearest in slot order, strictly within thr^2 */
    int near = -1;
    float sh = thr2;
#pragma unroll
    for (int sl = 0; sl < 4; sl++) {
        const float dd = __shfl(ddp, row0 + idx[sl]);
        if (sl < nk && dd < sh) { sh = dd; near = sl; }
    }
    int at;
    if (near >= 0) {
        at = idx[0];
        at = near == 1 ? idx[1] : at; at = near == 2 ? idx[2] : at; at = near == 3 ? idx[3] : at;
    } else if (nk < 4) {
        if (cnt >= MP) return;   /* the pool is full: dropped (as the oracle) */
        at = cnt;
        L.mkid[at][es] = (float)(key + nk);
        L.mimp[at][es] = 0.0f;
        L.mcnt[es] = cnt + 1;
    } else {   /* sortCachedPoints: keep the deepest, else the largest area */
        V3 cla[4];
        float cd[4];
#pragma unroll
        for (int sl = 0; sl < 4; sl++) {
            const int src = row0 + idx[sl];
            cla[sl] = v3(__shfl(lap.x, src), __shfl(lap.y, src), __shfl(lap.z, src));
            cd[sl] = __shfl(dp, src);
        }
        int maxi = -1;
        float maxpen = d;
#pragma unroll
        for (int sl = 0; sl < 4; sl++)
            if (cd[sl] < maxpen) { maxi = sl; maxpen = cd[sl]; }
        float res[4];
        res[0] = maxi == 0 ? 0.0f : dot(cross(la - cla[1], cla[3] - cla[2]), cross(la - cla[1], cla[3] - cla[2]));
        res[1] = maxi == 1 ? 0.0f : dot(cross(la - cla[0], cla[3] - cla[2]), cross(la - cla[0], cla[3] - cla[2]));
        res[2] = maxi == 2 ? 0.0f : dot(cross(la - cla[0], cla[3] - cla[1]), cross(la - cla[0], cla[3] - cla[1]));
        res[3] = maxi == 3 ? 0.0f : dot(cross(la - cla[0], cla[2] - cla[1]), cross(la - cla[0], cla[2] - cla[1]));
        int best = 0;
        float bv = res[0];
#pragma unroll
        for (int sl = 1; sl < 4; sl++)
            if (res[sl] > bv) { bv = res[sl]; best = sl; }
        at = idx[0];
        at = best == 1 ? idx[1] : at; at = best == 2 ? idx[2] : at; at = best == 3 ? idx[3] : at;
        L.mimp[at][es] = 0.0f;
    }
    L.mla[at][0][es] = la.x; L.mla[at][1][es] = la.y; L.mla[at][2][es] = la.z;
    L.mlb[at][0][es] = lb.x; L.mlb[at][1][es] = lb.y; L.mlb[at][2][es] = lb.z;
    L.mn[at][0][es] = n.x; L.mn[at][1][es] = n.y; L.mn[at][2][es] = n.z;
    L.md[at][es] = d;
}

/* the joint frame j (lane j of the row holds R_j, o_j in Rl, ol) in any lane: a row bpermute */
__device__ __forceinline__ void joint_frame(const M3& Rl, V3 ol, int j, M3& R, V3& o) {
    const int src = (int)(threadIdx.x & ~(unsigned)(GW - 1)) + (j < 0 ? 0 : j);
#pragma unroll
    for (int t = 0; t < 9; t++) R.m[t] = __shfl(Rl.m[t], src);
    o = v3(__shfl(ol.x, src), __shfl(ol.y, src), __shfl(ol.z, src));
}

/* refreshContactPoints of env es's pool (lane c refreshes point c), the removals renumbered as
 * Bullet's removeContactPoint does (reverse slot order, the last slot's point fills the hole) with
 * the survivors' pool order kept, then every point inserted into the robot row list (g1_insert:
 * after the table candidates, in pool order) as its own row: id = kid, pool index in g1w.
 * OBJ: B is the cube (Rc, op), else a static obstacle (local B = world). */
template <int OBJ, int AO, class LT>
__device__ __forceinline__ void man_refresh_insert_g(MRef m, LT& L, int es, int c, const M3& Rl, V3 ol, const M3& Rc,
                                                     V3 op) {
    const int cnt = L.mcnt[es];
    const bool mine = c < cnt;
    const int p = mine ? c : 0;
    const int kid = (int)L.mkid[p][es], key = kid & ~3;
    const int cap = man_capsule<AO>(key < 32 ? 32 : key);
    const int capc = cap < 0 ? 0 : (cap >= PGX_NCAP ? PGX_NCAP - 1 : cap);
    const int j = kCapJ[capc];
    /* the point's pair's breaking threshold: its capsule against the cube / the obstacle */
    const float thr = AO ? cap_tau<TAU_OBST>(m, capc) : cap_tau<TAU_OBJ>(m, capc);
    M3 R;
    V3 o;
    joint_frame(Rl, ol, j, R, o);
    const V3 la = lds3(L.mla[p], es), lb = lds3(L.mlb[p], es), n = lds3(L.mn[p], es);
    const V3 pa = o + mul(R, la);
    const V3 pb = OBJ ? op + mul(Rc, lb) : lb;
    const float d = dot(pa - pb, n);
    const V3 e = pb - (pa - d * n);
    const bool drop = mine && (d > thr || dot(e, e) > thr * thr);
    const unsigned dm = row_ballot(drop);
    const unsigned km = row_ballot(mine && !drop);
    const int row0 = (int)(threadIdx.x & ~(unsigned)(GW - 1));
    const int newp = mine && !drop ? __builtin_popcount(km & ((1u << c) - 1u)) : -1;
    int kidn = kid;   /* this point's kid after the removals */
    if (__any(dm != 0u)) {   /* (rare) removals: this point's slot after Bullet's renumbering, compaction */
        int slot = kid & 3, dmask = 0, nk = 0;
        for (int t = 0; t < GW; t++) {
            const int kt = __shfl(kid, row0 + t);
            const bool inm = ((km | dm) >> t) & 1u;
            if (inm && (kt & ~3) == key) {
                nk++;
                if ((dm >> t) & 1u) dmask |= 1 << (kt & 3);
            }
        }
        int cur0 = 0, cur1 = 1, cur2 = 2, cur3 = 3, nn = nk;
#pragma unroll
        for (int s2 = 3; s2 >= 0; s2--) {
            const int cs = s2 == 0 ? cur0 : (s2 == 1 ? cur1 : (s2 == 2 ? cur2 : cur3));
            if (s2 < nn && ((dmask >> cs) & 1)) {
                const int last = nn - 1 == 0 ? cur0 : (nn - 1 == 1 ? cur1 : (nn - 1 == 2 ? cur2 : cur3));
                if (s2 == 0) cur0 = last; else if (s2 == 1) cur1 = last; else if (s2 == 2) cur2 = last; else cur3 = last;
                nn--;
            }
        }
        int ns = slot;
        ns = (0 < nn && cur0 == slot) ? 0 : ns;
        ns = (1 < nn && cur1 == slot) ? 1 : ns;
        ns = (2 < nn && cur2 == slot) ? 2 : ns;
        ns = (3 < nn && cur3 == slot) ? 3 : ns;
        kidn = key + ns;
        /* read every field, then write it at the compacted index with the new kid */
        const float imp = L.mimp[p][es];
        if (newp >= 0) {
            L.mkid[newp][es] = (float)kidn;
            L.mla[newp][0][es] = la.x; L.mla[newp][1][es] = la.y; L.mla[newp][2][es] = la.z;
            L.mlb[newp][0][es] = lb.x; L.mlb[newp][1][es] = lb.y; L.mlb[newp][2][es] = lb.z;
            L.mn[newp][0][es] = n.x; L.mn[newp][1][es] = n.y; L.mn[newp][2][es] = n.z;
            L.md[newp][es] = d;
            L.mimp[newp][es] = imp;
        }
        L.mcnt[es] = __builtin_popcount(km);
    } else if (mine) {
        L.md[p][es] = d;
    }
    /* the manifold points as rows.  With room for every point (the common case) each kept lane
     * writes its row straight to its id-ordered slot after the table candidates (their ids are
     * below 32, every manifold id above): its rank among the env's kept ids by row broadcasts.
     * Otherwise the budget's deepest by (depth, discovery), as g1_insert keeps them: the table
     * candidates first, then the points in pool order, then id order (oracle select_points). */
    const V3 rb = pb - op;
    const int nkeep = __builtin_popcount(km);
    const int nt = L.cnt[1][es];
    const float kf = (float)kidn;
    int rank = 0;
    sfor<0, 16>([&](auto uc) __attribute__((always_inline)) {
        constexpr int U = decltype(uc)::value;
        const float ku = bcast16<U>(kf);
        rank += (((km >> U) & 1u) && ku < kf) ? 1 : 0;
    });
    if (nt + nkeep <= LT::RB) {
        if (newp >= 0) {
            const int sl = nt + rank;
            L.g1d[sl][es] = d; L.g1id[sl][es] = kf; L.g1j[sl][es] = j; L.g1w[sl][es] = newp;
            L.g1p[sl][0][es] = pa.x; L.g1p[sl][1][es] = pa.y; L.g1p[sl][2][es] = pa.z;
            L.g1n[sl][0][es] = n.x; L.g1n[sl][1][es] = n.y; L.g1n[sl][2][es] = n.z;
            const V3 r0 = OBJ ? rb : v3(0.0f, 0.0f, 0.0f);
            L.g1rb[sl][0][es] = r0.x; L.g1rb[sl][1][es] = r0.y; L.g1rb[sl][2][es] = r0.z;
        }
        L.cnt[1][es] = nt + nkeep;
        return;
    }
    sort_g1_by_depth(L, es);
    for (int t = 0; t < GW; t++) {
        if (!__any(t < nkeep)) break;
        /* the lane holding new pool index t: the t-th set bit of km */
        unsigned mm = km;
        for (int u = 0; u < t; u++) mm &= mm - 1u;
        const int src = row0 + (mm ? __builtin_ctz(mm) : 0);
        const float dt = __shfl(d, src);
        const int kidt = __shfl(kidn, src);
        const V3 pt = v3(__shfl(pa.x, src), __shfl(pa.y, src), __shfl(pa.z, src));
        const V3 nt2 = v3(__shfl(n.x, src), __shfl(n.y, src), __shfl(n.z, src));
        const V3 rt = v3(__shfl(rb.x, src), __shfl(rb.y, src), __shfl(rb.z, src));
        const int jt = __shfl(j, src);
        if (t < nkeep) g1_insert(L, es, dt, (float)kidt, jt, pt, nt2, OBJ ? rt : v3(0.0f, 0.0f, 0.0f), t);
    }
    sort_groups(L, es);
}

/* Bullet's persistent manifold of capsule cn (wave-uniform) and the cube (FULL kernels): lane s of
 * the env's row evaluates sample s as object_candidates_g does (the same arithmetic), the pair's new
 * point is its deepest candidate (ties: the lowest sample -- GJK's closest pair of the convex
 * capsule and the box, restated), and addContactPoint merges it into the env's pool (man_add_g):
 * point on the capsule pa = C - r n in the frame of the capsule's joint, the box's closest point
 * in the cube frame, the normal from the cube, the depth. */
template <class LT>
__device__ __forceinline__ void object_new_point_g(const PgxDevEnv& e, float tau, LT& L, int es, const ObjState& ob,
                                                   const M3& Rc, int cn, int c, bool env_near, const M3& Rl, V3 ol) {
    const V3 A = lds3(L.capA[cn], es), B = lds3(L.capB[cn], es);
    const float r = kCapR[cn];
    const int jc = kCapJ[cn], ns = kCapNs[cn];
    const float h = e.obj_half;
    const V3 ab = B - A;
    const float inv_n = ns > 1 ? 1.0f / (float)(ns - 1) : 0.0f;
    const V3 C = A + ((float)c * inv_n) * ab;
    const V3 cl = mul_t(Rc, C - ob.p);
    V3 qb = v3(fminf(fmaxf(cl.x, -h), h), fminf(fmaxf(cl.y, -h), h), fminf(fmaxf(cl.z, -h), h));
    const V3 diff = cl - qb;
    const float d2 = dot(diff, diff);
    V3 nl;
    float depth;
    if (d2 > 1e-24f) {
        const float dist = fast_sqrt(d2);
        nl = fast_rcp(dist) * diff;
        depth = dist - r;
    } else { /* centre inside the box: out through the nearest face */
        const float bx = h - fabsf(cl.x), by = h - fabsf(cl.y), bz = h - fabsf(cl.z);
        int ax = 0;
        float best = bx;
        if (by < best) { best = by; ax = 1; }
        if (bz < best) { best = bz; ax = 2; }
        const float sx = cl.x < 0.0f ? -1.0f : 1.0f, sy = cl.y < 0.0f ? -1.0f : 1.0f, sz = cl.z < 0.0f ? -1.0f : 1.0f;
        nl = v3(ax == 0 ? sx : 0.0f, ax == 1 ? sy : 0.0f, ax == 2 ? sz : 0.0f);
        if (ax == 0) qb.x = sx * h;
        if (ax == 1) qb.y = sy * h;
        if (ax == 2) qb.z = sz * h;
        depth = -best - r;
    }
    const bool cand = env_near && c < ns && depth < tau;
    const float dd = cand ? depth : 3.0e38f;
    int rank = 0;
    sfor<0, 16>([&](auto uc) __attribute__((always_inline)) {
        constexpr int U = decltype(uc)::value;
        const float du = bcast16<U>(dd);
        rank += (du < dd || (du == dd && U < c)) ? 1 : 0;
    });
    const unsigned bm = row_ballot(cand && rank == 0);
    M3 Rj;
    V3 oj;
    joint_frame(Rl, ol, jc, Rj, oj);   /* (every lane: a row bpermute) */
    const int src = (int)(threadIdx.x & ~(unsigned)(GW - 1)) + (bm ? __builtin_ctz(bm) : 0);
    const V3 n = mul(Rc, nl);
    const V3 pa = C - r * n;
    const V3 pk = v3(__shfl(pa.x, src), __shfl(pa.y, src), __shfl(pa.z, src));
    const V3 nk = v3(__shfl(n.x, src), __shfl(n.y, src), __shfl(n.z, src));
    const V3 qk = v3(__shfl(qb.x, src), __shfl(qb.y, src), __shfl(qb.z, src));
    const float dk = __shfl(depth, src);
    if (bm) man_add_g(L, es, c, 32 + 16 * cn, mul_t(Rj, pk - oj), qk, nk, dk, tau * tau);
}

/* ReachAO: the obstacles are static colliders (create_obstacle_sphere / _cuboid,
 * reach_ao.py:819-860: mass 0, not ghosts), so stepSimulation resolves robot contacts with
 * them like the table's (oracle detect(), "ReachAO" branch): capsule c (wave-uniform) against
 * each obstacle, one closest pair per pair within the processing threshold tau; the contact
 * normal points from the obstacle to the robot, the point on the robot is P + r n.  The
 * capsule-to-centre distance minus the radius / circumradius bounds the pair from below, so
 * the exact query runs only for pairs that can be within tau. */
template <class LT>
__device__ __forceinline__ bool ao_capsule_near(LT& L, int ln, int c, float tau) {
    const V3 A = lds3(L.capA[c], ln), B = lds3(L.capB[c], ln);
    bool near = false;
    for (int o = 0; o < AO_N; o++) {
        const V3 C = lds3(L.aoC[o], ln);
        const float dc = norm(C - seg_closest(A, B, C)) - kCapR[c] - (o < 3 ? kAoSize : kAoCubeBound);
        near = near || dc < tau;
    }
    return near;
}
template <class LT>
__device__ __forceinline__ void ao_obstacle_candidates(LT& L, int ln, int c, float tau) {
    const V3 A = lds3(L.capA[c], ln), B = lds3(L.capB[c], ln);
    const float r = kCapR[c];
    const int jc = kCapJ[c];
    const V3 hcube = v3(kAoSize, kAoSize, kAoSize);
    for (int o = 0; o < AO_N; o++) {
        const V3 C = lds3(L.aoC[o], ln);
        const V3 P0 = seg_closest(A, B, C);
        const V3 v = C - P0;
        const float len = norm(v);
        float d;
        V3 P = P0, n;
        if (o < 3) {
            d = len - r - kAoSize;
            n = len > 0.0f ? fast_rcp(len) * v : v3(0.0f, 0.0f, 1.0f);
        } else {
            if (!(len - r - kAoCubeBound < tau)) continue;
            d = capsule_box_pair<true>(A, B, r, C, hcube, &P, &n);
        }
        if (d < tau) g1_insert(L, ln, d, (float)(32 + 6 * c + o), jc, P + r * n, (-1.0f) * n, v3(0.0f, 0.0f, 0.0f));
    }
}

/* Robot capsules against the table/plane (end spheres) and the object (spheres sampled
 * along the axis), from the world end points the FK pass left in LDS.  A runtime loop
 * over the capsule table (wave-uniform index: scalar loads) keeps the code compact. */
template <int OBJ, class LT, int AO = 0>
__device__ __forceinline__ void robot_contacts(MRef m, const PgxDevEnv& e, LT& L, int ln, const ObjState& ob,
                                            const M3& Rc) {
    for (int c = 0; c < PGX_NCAP; c++) {
        const V3 A = v3(L.capA[c][0][ln], L.capA[c][1][ln], L.capA[c][2][ln]);
        const V3 B = v3(L.capB[c][0][ln], L.capB[c][1][ln], L.capB[c][2][ln]);
        const float r = kCapR[c];
        const int flags = kCapFlags[c], jc = kCapJ[c], ns = kCapNs[c];
        if (flags & PGX_CAP_VS_TABLE) {
            for (int end = 0; end < (ns == 1 ? 1 : 2); end++) {
                const V3 P = end ? B : A;
                const bool ont = on_table(e, P.x, P.y);
                const float zt = ont ? e.table_top : e.plane_z;
                const float d = P.z - r - zt;
                if (d < (ont ? cap_tau<TAU_TABLE>(m, c) : cap_tau<TAU_PLANE>(m, c)))
                    g1_insert(L, ln, d, (float)(2 * c + end), jc, v3(P.x, P.y, P.z - r), v3(0.0f, 0.0f, 1.0f),
                              v3(0.0f, 0.0f, 0.0f));
            }
        }
        if (OBJ && (flags & PGX_CAP_VS_OBJECT)) object_candidates(e, cap_tau<TAU_OBJ>(m, c), L, ln, ob, Rc, c, true);
        /* flags 0: the base and panda_link1, whose capsule lies on the joint-1 axis and cannot
         * move towards an obstacle (the reset keeps them 0.03 clear) */
        if (AO && flags != 0) {
            const float tau = cap_tau<TAU_OBST>(m, c);
            if (ao_capsule_near(L, ln, c, tau)) ao_obstacle_candidates(L, ln, c, tau);
        }
    }
}

/* world end points of the capsules carried by arm joint j (compile-time walk) */
template <int C = 0, class LT>
__device__ __forceinline__ void link_capsules(int j, LT& L, int ln, const M3& R, V3 oj) {
    if constexpr (C < PGX_NCAP) {
        if (kCapJ[C] == j) {
            const V3 A = oj + mulc(R, kCapA[C]), B = oj + mulc(R, kCapB[C]);
            L.capA[C][0][ln] = A.x; L.capA[C][1][ln] = A.y; L.capA[C][2][ln] = A.z;
            L.capB[C][0][ln] = B.x; L.capB[C][1][ln] = B.y; L.capB[C][2][ln] = B.z;
        }
        link_capsules<C + 1, LT>(j, L, ln, R, oj);
    }
}

/* One Bullet stepSimulation() of the arm (+ object and contacts when compiled in):
 *   contacts at the current poses (CONT)
 *   qd_u = clamp(qd + dt * M^-1 (-b(q,qd)))          (ABA + applyDeltaVee)
 *   object: v_u = v + dt (g - (k + k|v|) v - w x v), w_u = w - dt (k + k|w|) w
 *   PGS over the motor/limit rows in Bullet's sorted order, reversed on even
 *   sweeps, then the contact normal rows, then the friction rows; early exit when
 *   the max squared row residual <= residual_thr
 *   qd = clamp(qd_u + M^-1 J^T lambda); q += dt*qd   (constraint pass, stepPositions)
 *   object: p += dt v, orientation by the exponential map of w dt
 * M by composite-rigid-body, b by Newton-Euler with Bullet's link damping. */
/* Capsule c's table constants for lane c of a 16-lane row (lanes >= PGX_NCAP: capsule 0's, as
 * the callers' cc = 0), selected from compile-time values: a lane-indexed read of the constant
 * tables compiles to a global load and a vmcnt wait inside the substep loop. */
struct CapLane {
    float r;
    int flags, ns, j, slot;
};
__device__ __forceinline__ CapLane cap_lane() {
    float r = kCapR[0], fl = (float)kCapFlags[0], ns = (float)kCapNs[0], j = (float)kCapJ[0];
    float sl = (float)ao_slot(0);
    sfor<1, PGX_NCAP>([&](auto kc) __attribute__((always_inline)) {
        constexpr int K = decltype(kc)::value;
        r = lane_sel<K>(kCapR[K], r);
        fl = lane_sel<K>((float)kCapFlags[K], fl);
        ns = lane_sel<K>((float)kCapNs[K], ns);
        j = lane_sel<K>((float)kCapJ[K], j);
        sl = lane_sel<K>((float)ao_slot(K), sl);
    });
    return CapLane{r, (int)fl, (int)ns, (int)j, (int)sl};
}

/* Robot capsule ends vs the table / plane in the wide layout (no object): lane c tests
 * capsule c's end spheres (the candidates of robot_contacts' table branch; at most 2 per
 * pair); the row keeps the RB deepest by (depth, discovery order) like g1_insert -- ranked by
 * broadcast only when an env has more -- and every kept candidate goes straight to its id-ordered slot
 * (ids 2c + end grow with the lane), so sort_groups has nothing left to do. */
template <class LT>
__device__ __forceinline__ void robot_table_contacts_g(MRef m, const PgxDevEnv& e, LT& L, int es, int c) {
    const int cc = c < PGX_NCAP ? c : 0;
    const CapLane cl = cap_lane();
    const bool on = c < PGX_NCAP && (cl.flags & PGX_CAP_VS_TABLE);
    const V3 A = lds3(L.capA[cc], es), B = lds3(L.capB[cc], es);
    const float r = cl.r;
    const bool two = cl.ns != 1;
    /* each end against the box under it, within the pair's breaking threshold (cap_tau) */
    const float tt = cap_tau<TAU_TABLE>(m, cc), tp = cap_tau<TAU_PLANE>(m, cc);
    const bool t0 = on_table(e, A.x, A.y), t1 = on_table(e, B.x, B.y);
    const float d0 = A.z - r - (t0 ? e.table_top : e.plane_z);
    const float d1 = B.z - r - (t1 ? e.table_top : e.plane_z);
    const bool c0 = on && d0 < (t0 ? tt : tp), c1 = on && two && d1 < (t1 ? tt : tp);
    unsigned m0 = row_ballot(c0), m1 = row_ballot(c1);
    const int total = __builtin_popcount(m0) + __builtin_popcount(m1);
    bool k0 = c0, k1 = c1;
    if (__any(total > LT::RB)) {
        /* rank = candidates strictly before in (depth, discovery = 2 lane + end) order */
        const float e0 = c0 ? d0 : 3.0e38f, e1 = c1 ? d1 : 3.0e38f;
        int r0 = 0, r1 = 0;
        sfor<0, PGX_NCAP>([&](auto kc) __attribute__((always_inline)) {
            constexpr int K = decltype(kc)::value;
            const float y0 = bcast16<K>(e0), y1 = bcast16<K>(e1);
            r0 += (y0 < e0 || (y0 == e0 && K < c)) + (y1 < e0 || (y1 == e0 && K < c));
            r1 += (y0 < e1 || (y0 == e1 && K <= c)) + (y1 < e1 || (y1 == e1 && K < c));
        });
        k0 = c0 && r0 < LT::RB;
        k1 = c1 && r1 < LT::RB;
        m0 = row_ballot(k0);
        m1 = row_ballot(k1);
    }
    const unsigned below = (1u << (c & 15)) - 1u;
    const int base = __builtin_popcount(m0 & below) + __builtin_popcount(m1 & below);
    const int jc = cl.j;
    if (k0) {
        const int sl = base;
        L.g1d[sl][es] = d0; L.g1id[sl][es] = (float)(2 * c); L.g1j[sl][es] = jc; L.g1w[sl][es] = -1;
        L.g1p[sl][0][es] = A.x; L.g1p[sl][1][es] = A.y; L.g1p[sl][2][es] = A.z - r;
        L.g1n[sl][0][es] = 0.0f; L.g1n[sl][1][es] = 0.0f; L.g1n[sl][2][es] = 1.0f;
        L.g1rb[sl][0][es] = 0.0f; L.g1rb[sl][1][es] = 0.0f; L.g1rb[sl][2][es] = 0.0f;
    }
    if (k1) {
        const int sl = base + (k0 ? 1 : 0);
        L.g1d[sl][es] = d1; L.g1id[sl][es] = (float)(2 * c + 1); L.g1j[sl][es] = jc; L.g1w[sl][es] = -1;
        L.g1p[sl][0][es] = B.x; L.g1p[sl][1][es] = B.y; L.g1p[sl][2][es] = B.z - r;
        L.g1n[sl][0][es] = 0.0f; L.g1n[sl][1][es] = 0.0f; L.g1n[sl][2][es] = 1.0f;
        L.g1rb[sl][0][es] = 0.0f; L.g1rb[sl][1][es] = 0.0f; L.g1rb[sl][2][es] = 0.0f;
    }
    L.cnt[1][es] = __builtin_popcount(m0) + __builtin_popcount(m1);
}

/* Per-substep dynamics shared by both solver layouts: contact detection at the current
 * poses (CONT), FK fused with the per-link terms, Newton-Euler bias, CRBA mass matrix,
 * Cholesky, the unconstrained velocities vu = clamp(qd + dt M^-1 (-b)) and M^-1 (lower
 * triangle); the object's unconstrained velocities (OBJ). */
struct Dyn {
    V3 z[NJ], o[NJ];
    float Mi[NJ][NJ];     /* one-lane layout: M^-1, lower triangle */
    float mcol[NJ];       /* wide layout: lane c's column of M^-1 (0 on lanes >= 7) */
    float mdiag[NJ];      /* wide layout: diag(M^-1) on every lane */
    float vu[NJ];
    V3 vcu, wcu;
    bool coll;            /* ReachAO, wide layout: check_collided at the substep's start pose */
};

template <int OBJ, int CONT, class LT, bool PAR = false, int AO = 0>
__device__ __forceinline__ void substep_dyn(MRef m, const PgxDevEnv& e, const float* q, const float* qd,
                                            const ObjState& ob, LT* Lp, int ln, Dyn& D, int lane = 0) {
    M3 Rc;
    if (OBJ) Rc = quat_mat(ob);
    if (CONT) { Lp->cnt[0][ln] = 0; Lp->cnt[1][ln] = 0; }
    if (OBJ) { /* object vertices vs the box top under them */
        const float h = e.obj_half;
        /* every vertex against the table box (ids 0-7), then against the plane's top (ids 8-15) */
#pragma unroll
        for (int k = 0; k < 16; k++) {
            const int vtx = k & 7;
            const V3 r = mul(Rc, v3((vtx & 1) ? h : -h, (vtx & 2) ? h : -h, (vtx & 4) ? h : -h));
            const V3 P = ob.p + r;
            V3 n = v3(0.0f, 0.0f, 1.0f);
            const float d = k < 8 ? vertex_vs_table(e, P, n) : P.z - e.plane_z;
            if (d < (k < 8 ? m.tau_obj_table : m.tau_obj_plane)) g0_insert(*Lp, ln, d, (float)k, r, n);
        }
    }
    /* FK fused with the per-link quantities the dynamics need, so the 3x3
     * rotations die immediately (only panda_link7's survives for its group). */
    V3 (&z)[NJ] = D.z;
    V3 (&o)[NJ] = D.o;
    V3 c[NJ];
    S3 Iw[NJ];
    M3 R6;
    {
        M3 PR = {{1, 0, 0, 0, 1, 0, 0, 0, 1}};
        V3 PO = v3(m.base[0], m.base[1], m.base[2]);
        float sjs[NJ], cjs[NJ];
        joint_sincos_all<PAR>(q, sjs, cjs);
#pragma unroll
        for (int j = 0; j < NJ; j++) {
            M3 R = mulm(PR, kJr[j]);
            V3 oj = PO + mulc(PR, kJp[j]);
            const float s = sjs[j], cs = cjs[j];
#pragma unroll
            for (int r = 0; r < 3; r++) {
                float a = R.m[r * 3], b = R.m[r * 3 + 1];
                R.m[r * 3] = cs * a + s * b;
                R.m[r * 3 + 1] = -s * a + cs * b;
            }
            z[j] = col(R, 2);
            o[j] = oj;
            c[j] = oj + mulc(R, kCom[j]);
            if (j < NJ - 1) Iw[j] = rot_diag(R, kInertia[j]);
            else { Iw[j] = rot_sym(R, kI6c); R6 = R; }
            if constexpr (CONT) link_capsules(j, *Lp, ln, R, oj);
            PR = R;
            PO = oj;
        }
    }
    if (CONT) {
        if constexpr (PAR && !OBJ && !AO) {
            robot_table_contacts_g(m, e, *Lp, ln, lane);
        } else {
            robot_contacts<OBJ, LT, AO>(m, e, *Lp, ln, ob, Rc);
            sort_groups(*Lp, ln);
        }
    }
    PGX_PROF_MARK(1);
    const V3 g = v3(m.gravity[0], m.gravity[1], m.gravity[2]);

    /* forward Newton-Euler (qdd = 0) fused with the link wrenches at the COM
     * (inertial + gravity + Bullet damping m*v*(k+k|v|), I*w*(k+k|w|)) */
    V3 F[NJ], T[NJ];
    {
        V3 wp = v3(0, 0, 0), alp = v3(0, 0, 0), vp = v3(0, 0, 0), ap = v3(0, 0, 0), pp = o[0];
#pragma unroll
        for (int j = 0; j < NJ; j++) {
            V3 r = o[j] - pp;
            V3 wr = cross(wp, r);
            V3 vo = vp + wr;
            V3 ao = ap + cross(alp, r) + cross(wp, wr);
            V3 sz = qd[j] * z[j];
            V3 w = wp + sz;
            V3 al = alp + cross(wp, sz);
            V3 rc = c[j] - o[j];
            V3 wrc = cross(w, rc);
            V3 v = vo + wrc;
            V3 a = ao + cross(al, rc) + cross(w, wrc);
            float wn = norm(w);
            V3 Iww = mul(Iw[j], w);
            F[j] = kMass[j] * (a - g);
            T[j] = mul(Iw[j], al) + cross(w, Iww);
            if (j < NJ - 1) {
                F[j] = F[j] + (kMass[j] * (m.lin_damp + m.lin_damp * norm(v))) * v;
                T[j] = T[j] + (m.ang_damp + m.ang_damp * wn) * Iww;
            } else {
                /* link-7 group: composite inertial terms, per-body damping */
                S3 Iown = rot_sym(R6, kI6own);
                T[j] = T[j] + (m.ang_damp + m.ang_damp * wn) * mul(Iown, w);
#pragma unroll
                for (int b = 0; b < PGX_NDAMP; b++) {
                    {
                        V3 rb = mulc(R6, kDpos[b]);
                        V3 vb = vo + cross(w, rb);
                        V3 fd = (kDmass[b] * (m.lin_damp + m.lin_damp * norm(vb))) * vb;
                        F[j] = F[j] + fd;
                        T[j] = T[j] + cross(o[j] + rb - c[j], fd);
                    }
                }
            }
            wp = w; alp = al; vp = v; ap = a; pp = c[j];
        }
    }

    /* backward: generalised bias b_j = z_j . (moment of subtree wrench about pivot j) */
    float nb[NJ];
    {
        V3 Fs = v3(0, 0, 0), Ns = v3(0, 0, 0), oc = o[NJ - 1];
#pragma unroll
        for (int j = NJ - 1; j >= 0; j--) {
            V3 N = T[j] + cross(c[j] - o[j], F[j]) + Ns + cross(oc - o[j], Fs);
            nb[j] = -dot(z[j], N);
            Fs = Fs + F[j];
            Ns = N;
            oc = o[j];
        }
    }

    PGX_PROF_MARK(14);
    /* composite-rigid-body mass matrix (lower triangle, row >= col) */
    float Mt[NJ][NJ];
    {
        float mc = kMass[NJ - 1];
        V3 cc = c[NJ - 1];
        S3 Ic = Iw[NJ - 1];
#pragma unroll
        for (int j = NJ - 1; j >= 0; j--) {
            if (j < NJ - 1) {
                float mj = kMass[j];
                float mt = mc + mj;
                V3 cn = fast_rcp(mt) * (mc * cc + mj * c[j]);
                Ic = add(add(Ic, steiner(mc, cc - cn)), add(Iw[j], steiner(mj, c[j] - cn)));
                mc = mt;
                cc = cn;
            }
            V3 f = mc * cross(z[j], cc - o[j]);
            V3 n0 = mul(Ic, z[j]) + cross(cc - o[j], f);
            Mt[j][j] = dot(z[j], n0);
#pragma unroll
            for (int i = 0; i < j; i++) Mt[j][i] = dot(z[i], n0 + cross(o[j] - o[i], f));
        }
    }
    chol7(Mt);
    float (&vu)[NJ] = D.vu;
    {
        float qdd[NJ];
        chol7_solve(Mt, nb, qdd);
#pragma unroll
        for (int j = 0; j < NJ; j++) vu[j] = fminf(fmaxf(qd[j] + m.dt * qdd[j], -m.max_vel), m.max_vel);
    }

    PGX_PROF_MARK(15);
    /* M^-1 = L^-T L^-1 (symmetric, lower triangle kept) */
    float (&Mi)[NJ][NJ] = D.Mi;
    {
        float X[NJ][NJ];
#pragma unroll
        for (int i = 0; i < NJ; i++) {
            float inv = Mt[i][i]; /* chol7 stores the inverted diagonal */
#pragma unroll
            for (int jj = 0; jj <= i; jj++) {
                float s = (jj == i) ? 1.0f : 0.0f;
#pragma unroll
                for (int kk = jj; kk < i; kk++) s -= Mt[i][kk] * X[kk][jj];
                X[i][jj] = s * inv;
            }
        }
#pragma unroll
        for (int i = 0; i < NJ; i++)
#pragma unroll
            for (int jj = 0; jj <= i; jj++) {
                float s = 0.0f;
#pragma unroll
                for (int l = i; l < NJ; l++) s += X[l][i] * X[l][jj];
                Mi[i][jj] = s;
            }
    }

    /* object: unconstrained velocities (btMultiBody floating base) */
    V3& vcu = D.vcu;
    V3& wcu = D.wcu;
    vcu = v3(0, 0, 0);
    wcu = v3(0, 0, 0);
    if (OBJ) {
        const float vn = norm(ob.v), wn = norm(ob.w);
        vcu = ob.v + m.dt * (g - (m.lin_damp + m.lin_damp * vn) * ob.v - cross(ob.w, ob.v));
        wcu = ob.w - (m.dt * (m.ang_damp + m.ang_damp * wn)) * ob.w;
    }
}

/* ------------------------------------------- wide layout: lane-parallel dynamics */
/* In the wide layout lane c < 7 of an env's row owns arm link c for the Newton-Euler bias
 * and the mass matrix: the recursions over the chain become prefix / suffix sums over the
 * row (three DPP adds each, row_shr / row_shl 1, 2, 4), every per-link term is evaluated
 * once instead of on all 16 lanes, and the results the redundant Cholesky needs (the
 * bias b, the lower triangle of M) are broadcast back.  Same equations as substep_dyn,
 * rearranged (below); only fp32 rounding differs. */
struct LaneK {   /* link c's constants (lanes >= 7: zero) */
    float mass, com[3];
    float I[6], Iown[6];   /* inertia about the COM in the link frame (xx,yy,zz,xy,xz,yz); the
                              one its angular damping uses (link-7 group: the bodies' own) */
};
__device__ __forceinline__ void lane_consts(LaneK& k) {
    k.mass = 0.0f;
#pragma unroll
    for (int t = 0; t < 3; t++) k.com[t] = 0.0f;
#pragma unroll
    for (int t = 0; t < 6; t++) { k.I[t] = 0.0f; k.Iown[t] = 0.0f; }
    sfor<0, NJ>([&](auto jc) __attribute__((always_inline)) {
        constexpr int j = decltype(jc)::value;
        k.mass = lane_sel<j>(kMass[j], k.mass);
#pragma unroll
        for (int t = 0; t < 3; t++) k.com[t] = lane_sel<j>(kCom[j][t], k.com[t]);
#pragma unroll
        for (int t = 0; t < 6; t++) {
            const float a = j < NJ - 1 ? (t < 3 ? kInertia[j < NJ - 1 ? j : 0][t < 3 ? t : 0] : 0.0f) : kI6c[t];
            const float b = j < NJ - 1 ? a : kI6own[t];
            if (a != 0.0f) k.I[t] = lane_sel<j>(a, k.I[t]);
            if (b != 0.0f) k.Iown[t] = lane_sel<j>(b, k.Iown[t]);
        }
    });
}
/* inclusive prefix (suffix) sum over lanes 0..c (c..15) of each 16-lane row */
__device__ __forceinline__ float row_pre(float x) {
    x += dpp<0x111>(x);   /* row_shr:1 (lane 0 reads 0) */
    x += dpp<0x112>(x);   /* row_shr:2 */
    x += dpp<0x114>(x);   /* row_shr:4 */
    return x;
}
__device__ __forceinline__ float row_suf(float x) {
    x += dpp<0x101>(x);   /* row_shl:1 */
    x += dpp<0x102>(x);   /* row_shl:2 */
    x += dpp<0x104>(x);   /* row_shl:4 */
    return x;
}
__device__ __forceinline__ V3 row_pre(V3 a) { return v3(row_pre(a.x), row_pre(a.y), row_pre(a.z)); }
__device__ __forceinline__ V3 row_suf(V3 a) { return v3(row_suf(a.x), row_suf(a.y), row_suf(a.z)); }
/* x on the link lanes 0..6 of every row, 0 elsewhere (one v_cndmask) */
__device__ __forceinline__ float link_only(float x) {
    float r;
    asm("v_cndmask_b32 %0, 0, %1, %2" : "=v"(r) : "v"(x), "s"(0x007F007F007F007Full));
    return r;
}
__device__ __forceinline__ V3 link_only(V3 a) { return v3(link_only(a.x), link_only(a.y), link_only(a.z)); }
/* R S R^T for a symmetric S held in registers */
__device__ __forceinline__ S3 rot_sym_r(const M3& R, const float* s) {
    const float Sm[9] = {s[0], s[3], s[4], s[3], s[1], s[5], s[4], s[5], s[2]};
    float T[9];
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++)
            T[i * 3 + j] = R.m[i * 3] * Sm[j] + R.m[i * 3 + 1] * Sm[3 + j] + R.m[i * 3 + 2] * Sm[6 + j];
    auto e = [&](int i, int j) { return T[i * 3] * R.m[j * 3] + T[i * 3 + 1] * R.m[j * 3 + 1] + T[i * 3 + 2] * R.m[j * 3 + 2]; };
    S3 o;
    o.xx = e(0, 0); o.yy = e(1, 1); o.zz = e(2, 2); o.xy = e(0, 1); o.xz = e(0, 2); o.yz = e(1, 2);
    return o;
}
__device__ __forceinline__ V3 mul_sym(const float* s, V3 v) {
    return v3(s[0] * v.x + s[3] * v.y + s[4] * v.z, s[3] * v.x + s[1] * v.y + s[5] * v.z,
              s[4] * v.x + s[5] * v.y + s[2] * v.z);
}

/* substep_dyn for the wide layout (16 lanes per env, lane c of the row).  Positions are
 * taken relative to the robot base.  With t_k = qd_k z_k (joint k's contribution to the
 * angular velocity) and prefix sums over the links k <= c:
 *   w_c = sum t_k,  S_c = sum t_k x o_k,  COM velocity v_c = w_c x c_c - S_c,
 *   pivot velocity u_c = w_c x o_c - S_c,  alpha_c = sum w_{k-1} x t_k   (qdd = 0),
 *   dS_c = sum (w_{k-1} x t_k) x o_k + t_k x u_k,  a_c = alpha_c x c_c + w_c x v_c - dS_c,
 * i.e. d/dt of v_c; the link wrenches at the COM are those of substep_dyn; the bias is
 *   b_c = -z_c . (sum_{k>=c} (T_k + c_k x F_k) - o_c x sum_{k>=c} F_k)   (suffix sums).
 * Mass matrix: the subtree of joint c has mass M, first moment H = sum m c and inertia
 * about the base I (suffix sums); spun about z_c through o_c its momentum is
 * f = z_c x (H - M o_c) and its angular momentum about o_c is n = I_o z_c with
 *   I_o z = I z - 2 (H.o) z + H (o.z) + o (H.z) + M (|o|^2 z - o (o.z)),
 * and M[c][i] = z_i . (n + (o_c - o_i) x f) for i <= c (CRBA), broadcast to every lane. */
template <int OBJ, int CONT, int AO = 0, int FULL = 0>
__device__ __forceinline__ void substep_dyn_g(MRef m, const PgxDevEnv& e, const float* q, const float* qd,
                                              const ObjState& ob, ContactLdsGT<OBJ, FULL>* Lp, int es, Dyn& D, int c,
                                              const LaneK& K, bool check = false) {
    M3 Rc;
    D.coll = false;
    if (OBJ) Rc = quat_mat(ob);
    if (CONT) { Lp->cnt[0][es] = 0; Lp->cnt[1][es] = 0; }
    if (OBJ) { /* object vertices vs the table box (lane c < 8: vertex c) and the plane's top (lane c >= 8:
                * vertex c - 8), the candidates' discovery order and ids as the one-lane walk's: the 4
                * deepest by (depth, id) as g0_insert keeps them, in id order as sort_groups leaves them */
        const float h = e.obj_half;
        const int vtx = c & 7;
        const V3 r = mul(Rc, v3((vtx & 1) ? h : -h, (vtx & 2) ? h : -h, (vtx & 4) ? h : -h));
        const V3 P = ob.p + r;
        V3 nrm = v3(0.0f, 0.0f, 1.0f);
        const float d = c < 8 ? vertex_vs_table(e, P, nrm) : P.z - e.plane_z;
        const bool cand = d < (c < 8 ? m.tau_obj_table : m.tau_obj_plane);
        const float dd = cand ? d : 3.0e38f;
        int rank = 0;
        sfor<0, 16>([&](auto uc) __attribute__((always_inline)) {
            constexpr int U = decltype(uc)::value;
            const float du = bcast16<U>(dd);
            rank += (du < dd || (du == dd && U < c)) ? 1 : 0;
        });
        const bool keep = cand && rank < CG;
        const unsigned mk = row_ballot(keep);
        const int sl = __builtin_popcount(mk & ((1u << (c & 15)) - 1u));
        if (keep) {
            Lp->g0d[sl][es] = d;
            Lp->g0id[sl][es] = (float)c;
            Lp->g0q[sl][0][es] = make_float4(r.x, r.y, r.z, 0.0f);
            Lp->g0n[sl][0][es] = nrm.x; Lp->g0n[sl][1][es] = nrm.y; Lp->g0n[sl][2][es] = nrm.z;
        }
        Lp->cnt[0][es] = __builtin_popcount(mk);
        PGX_PROF_MARK(19);
    }
    /* FK (redundant: constant-folded per link), capsule end points, and this lane's link */
    V3 (&z)[NJ] = D.z;
    V3 (&o)[NJ] = D.o;
    M3 Rl = {{0, 0, 0, 0, 0, 0, 0, 0, 0}};
    V3 ol = v3(0, 0, 0);
    {
        M3 PR = {{1, 0, 0, 0, 1, 0, 0, 0, 1}};
        V3 PO = v3(m.base[0], m.base[1], m.base[2]);
        float sjs[NJ], cjs[NJ];
        joint_sincos_all<true>(q, sjs, cjs);
        sfor<0, NJ>([&](auto jc) __attribute__((always_inline)) {
            constexpr int j = decltype(jc)::value;
            M3 R = mulm(PR, kJr[j]);
            V3 oj = PO + mulc(PR, kJp[j]);
            const float sn = sjs[j], cs = cjs[j];
#pragma unroll
            for (int r = 0; r < 3; r++) {
                float a = R.m[r * 3], b = R.m[r * 3 + 1];
                R.m[r * 3] = cs * a + sn * b;
                R.m[r * 3 + 1] = -sn * a + cs * b;
            }
            z[j] = col(R, 2);
            o[j] = oj;
            if constexpr (CONT) link_capsules(j, *Lp, es, R, oj);
#pragma unroll
            for (int t = 0; t < 9; t++) Rl.m[t] = lane_sel<j>(R.m[t], Rl.m[t]);
            ol = v3(lane_sel<j>(oj.x, ol.x), lane_sel<j>(oj.y, ol.y), lane_sel<j>(oj.z, ol.z));
            PR = R;
            PO = oj;
        });
    }
    if (CONT) {
        if constexpr (!OBJ) {
            robot_table_contacts_g(m, e, *Lp, es, c);
            if constexpr (AO) {
                /* obstacle contacts (ao_obstacle_candidates), lane-parallel: per obstacle, lane c
                 * measures capsule c's pair (the cull first, the exact query only where the pair
                 * can be within tau); the rare candidates are then inserted by depth (g1_insert)
                 * after the table candidates, every lane of the env reading the candidate lane's
                 * values, and finally put in id order.  Obstacle-major insertion instead of
                 * robot_contacts' capsule-major order: only an exact depth tie could order
                 * differently. */
                const int cc = c < PGX_NCAP ? c : 0;
                const float tau = cap_tau<TAU_OBST>(m, cc);   /* this lane's capsule against an obstacle */
                const CapLane cl = cap_lane();
                const bool cap_on = c < PGX_NCAP && cl.flags != 0;
                /* check (every substep but the first): the step loop's check_collided of the
                 * previous substep's end pose -- this pose -- fused in here, as ao_collided_g
                 * decides it (same pairs, same arithmetic): lane c's obstacle pairs when c is a
                 * collision link, its table distance for links 2..ee */
                const int slot = c < PGX_NCAP ? cl.slot : -1;
                const bool chk = check && slot >= 0;
                const V3 A = lds3(Lp->capA[cc], es), B = lds3(Lp->capB[cc], es);
                const float r = cl.r;
                const V3 hcube = v3(kAoSize, kAoSize, kAoSize);
                const int row0 = (int)(threadIdx.x & ~(unsigned)(GW - 1));
                bool sorted = false, hit = false;
                if (chk && slot >= 1) {
                    V3 tc = ao_table_c(e), th = ao_table_h(e);
                    /* recomputed here in every substep: hoisted out of the substep loop, the box
                     * bounds derived from them were spilled and reloaded (two-wave kernel) */
                    asm volatile("" : "+v"(tc.x), "+v"(tc.y), "+v"(tc.z), "+v"(th.x), "+v"(th.y), "+v"(th.z));
                    const V3 thi = v3(th.x - kAoMargin, th.y - kAoMargin, th.z - kAoMargin);
                    const float lb = fminf(box_sd(A, tc, thi), box_sd(B, tc, thi)) - 0.5f * norm(B - A) - kAoMargin - r;
                    if (lb <= 0.0f) hit = capsule_box_hit(A, B, r, tc, th);
                }
                unsigned cmask = 0;   /* FULL: this lane's candidate obstacles */
                int o1 = -1;          /* FULL: the first of them, its point kept (the rest recomputed) */
                V3 pa1 = v3(0.0f, 0.0f, 0.0f), pb1 = pa1, n1v = pa1;
                float d1 = 0.0f;
                V3 Cs[AO_N];   /* the obstacle centres, one LDS batch */
#pragma unroll
                for (int o = 0; o < AO_N; o++) Cs[o] = lds3(Lp->aoC[o], es);
#ifdef PGX_AB_NO_OBST   /* timing bound only (wrong results): the obstacle pairs skipped */
                if (true) {} else
#endif
#pragma unroll
                for (int o = 0; o < AO_N; o++) {
                    const V3 C = Cs[o];
                    V3 P = seg_closest(A, B, C);
                    const V3 v = C - P;
                    const float len = norm(v);
                    float d = 3.0e38f;
                    V3 n = len > 0.0f ? fast_rcp(len) * v : v3(0.0f, 0.0f, 1.0f);
                    if (cap_on || chk) {
                        if (o < 3) d = len - r - kAoSize;
                        else if (len - r - kAoCubeBound < (cap_on ? tau : 0.0f))
#ifdef PGX_AB_NO_BOXPAIR   /* timing bound only (wrong results): the bound for the box query */
                            d = len - r - kAoCubeBound;
#else
                            d = capsule_box_pair<true>(A, B, r, C, hcube, &P, &n);
#endif
                    }
                    hit = hit || (chk && d <= 0.0f);
                    const bool cand = cap_on && d < tau;
                    if constexpr (FULL && AO_PERS) {   /* the manifolds take the new points after the collision check */
                        cmask |= cand ? (1u << o) : 0u;
                        if (cand && o1 < 0) {
                            o1 = o;
                            pa1 = P + r * n;
                            pb1 = pa1 + d * n;
                            n1v = n;
                            d1 = d;
                        }
                        continue;
                    }
                    const uint64_t bm = __ballot(cand);
                    if (bm == 0) continue;
                    if (!sorted) { sort_g1_by_depth(*Lp, es); sorted = true; }
                    unsigned wm = __builtin_amdgcn_readfirstlane(
                        (unsigned)((bm | (bm >> 16) | (bm >> 32) | (bm >> 48)) & 0xFFFFu));
                    const V3 pa = P + r * n;
                    while (wm) {
                        const int k = __builtin_ctz(wm);
                        wm &= wm - 1u;
                        const int src = row0 + k;
                        const bool ck = __shfl((int)cand, src) != 0;
                        const float dk = __shfl(d, src);
                        const V3 pk = v3(__shfl(pa.x, src), __shfl(pa.y, src), __shfl(pa.z, src));
                        const V3 nk = v3(__shfl(n.x, src), __shfl(n.y, src), __shfl(n.z, src));
                        if (ck) g1_insert(*Lp, es, dk, (float)(32 + 6 * k + o), kCapJ[k], pk, (-1.0f) * nk, v3(0.0f, 0.0f, 0.0f));
                    }
                }
                if (sorted) sort_groups(*Lp, es);
                D.coll = row_any(hit);
                if (D.coll) return;   /* the step stops here: nothing of this substep runs */
                if constexpr (FULL && AO_PERS) {
                    /* Bullet's persistent manifolds of the obstacle pairs: each candidate pair's new
                     * point (the same closest-pair arithmetic as above, recomputed for the few
                     * candidates) merged obstacle-major, capsule by capsule, then the refresh and the
                     * rows (oracle detect(), the persistent branch) */
                    if (__any(cmask != 0u)) {
                        for (int o = 0; o < AO_N; o++) {
                            const bool have = (cmask >> o) & 1u;
                            const uint64_t bo = __ballot(have);
                            if (bo == 0) continue;
                            V3 pa = pa1, pb = pb1, n = n1v;   /* pa on the capsule, towards the obstacle; pb on it */
                            float d = d1;
                            if (have && o != o1) {   /* a second candidate of this capsule: the pair again */
                                const V3 C = lds3(Lp->aoC[o], es);
                                V3 P = seg_closest(A, B, C);
                                const V3 v = C - P;
                                const float len = norm(v);
                                n = len > 0.0f ? fast_rcp(len) * v : v3(0.0f, 0.0f, 1.0f);
                                if (o < 3) d = len - r - kAoSize;
                                else d = capsule_box_pair<true>(A, B, r, C, hcube, &P, &n);
                                pa = P + r * n;
                                pb = pa + d * n;   /* (static obstacle: local = world) */
                            }
                            unsigned wo = __builtin_amdgcn_readfirstlane(
                                (unsigned)((bo | (bo >> 16) | (bo >> 32) | (bo >> 48)) & 0xFFFFu));
                            while (wo) {
                                const int k = __builtin_ctz(wo);   /* wave-uniform: capsule k's joint frame */
                                wo &= wo - 1u;
                                const int src = row0 + k;
                                M3 Rj;
                                V3 oj;
                                joint_frame(Rl, ol, kCapJ[k], Rj, oj);
                                if (__shfl((int)have, src) == 0) continue;
                                const V3 pak = v3(__shfl(pa.x, src), __shfl(pa.y, src), __shfl(pa.z, src));
                                const V3 lak = mul_t(Rj, pak - oj);
                                const V3 pbk = v3(__shfl(pb.x, src), __shfl(pb.y, src), __shfl(pb.z, src));
                                const V3 nk = v3(__shfl(n.x, src), __shfl(n.y, src), __shfl(n.z, src));
                                const float dk = __shfl(d, src);
                                const float tk = cap_tau<TAU_OBST>(m, k);
                                man_add_g(*Lp, es, c, 32 + 24 * k + 4 * o, lak, pbk, (-1.0f) * nk, dk, tk * tk);
                            }
                        }
                    }
                    if (__any(Lp->mcnt[es] > 0))
                        man_refresh_insert_g<0, 1>(m, *Lp, es, c, Rl, ol, M3{{1, 0, 0, 0, 1, 0, 0, 0, 1}},
                                                   v3(0.0f, 0.0f, 0.0f));
                }
            }
        } else {
            PGX_PROF_MARK(20);
            /* robot_contacts' object cull per capsule lane; without a capsule in reach of the
             * object anywhere in the wave the robot group holds table candidates only, which
             * robot_table_contacts_g finds lane-parallel (the same candidates, order and ids) */
            const int cc = c < PGX_NCAP ? c : 0;
            const CapLane cl = cap_lane();
            bool near = false;
            if (c < PGX_NCAP && (cl.flags & PGX_CAP_VS_OBJECT)) {
                const V3 A = lds3(Lp->capA[cc], es), B = lds3(Lp->capB[cc], es);
                const V3 ab = B - A;
                const float l2 = dot(ab, ab);
                float t = l2 > 0.0f ? dot(ob.p - A, ab) * fast_rcp(l2) : 0.0f;
                t = fminf(fmaxf(t, 0.0f), 1.0f);
                const V3 cp = A + t * ab - ob.p;
                const float reach = cl.r + 1.7320508f * e.obj_half + cap_tau<TAU_OBJ>(m, cc);
                near = dot(cp, cp) < reach * reach;
            }
            /* table candidates lane-parallel (id-ordered, so re-sorted by depth: ids grow with
             * discovery among them), then the near capsules' object spheres inserted by depth
             * (g1_insert), then id order; only exact depth ties between a table and an object
             * candidate could order differently from robot_contacts' discovery order */
            robot_table_contacts_g(m, e, *Lp, es, c);
            const uint64_t bn = __ballot(near);
            unsigned wm = (unsigned)((bn | (bn >> 16) | (bn >> 32) | (bn >> 48)) & 0xFFFFu);
            if constexpr (FULL) {
                /* Bullet's persistent manifolds of the cube pairs: the near capsules' new points merged
                 * into the pool in capsule order, the pool refreshed, its points the rows after the
                 * table candidates (oracle detect(), the persistent branch) */
                const unsigned rm = row_ballot(near);
                wm = __builtin_amdgcn_readfirstlane(wm);
                while (wm) {
                    const int cn = __builtin_ctz(wm);
                    wm &= wm - 1u;
                    object_new_point_g(e, cap_tau<TAU_OBJ>(m, cn), *Lp, es, ob, Rc, cn, c, ((rm >> cn) & 1u) != 0, Rl, ol);
                }
                if (__any(Lp->mcnt[es] > 0)) man_refresh_insert_g<1, 0>(m, *Lp, es, c, Rl, ol, Rc, ob.p);
                PGX_PROF_MARK(21);
            } else if (wm) {
                const unsigned rm = row_ballot(near);
                sort_g1_by_depth(*Lp, es);
                wm = __builtin_amdgcn_readfirstlane(wm);
                while (wm) {
                    const int cn = __builtin_ctz(wm);
                    wm &= wm - 1u;
                    object_candidates_g(e, cap_tau<TAU_OBJ>(m, cn), *Lp, es, ob, Rc, cn, c, ((rm >> cn) & 1u) != 0);
                }
                PGX_PROF_MARK(21);
                sort_groups(*Lp, es);
            }
        }
    }
    PGX_PROF_MARK(1);
    const V3 g = v3(m.gravity[0], m.gravity[1], m.gravity[2]);
    const V3 base = v3(m.base[0], m.base[1], m.base[2]);
    const V3 zl = col(Rl, 2);
    const V3 ob_l = ol - base;                                   /* pivot, base-relative */
    const V3 cw = ol + mul(Rl, v3(K.com[0], K.com[1], K.com[2]));   /* COM, world */
    const V3 cb = cw - base;

    /* ---- Newton-Euler bias by prefix / suffix sums over the link lanes */
    const float qdl = pick_arm(qd, 0.0f);
    const V3 t1 = qdl * zl;
    const V3 w = row_pre(t1);
    const V3 alt = cross(w - t1, t1);
    const V3 al = row_pre(alt);
    const V3 S = row_pre(cross(t1, ob_l));
    const V3 u = cross(w, ob_l) - S;                             /* pivot velocity */
    const V3 dS = row_pre(cross(alt, ob_l) + cross(t1, u));
    const V3 v = cross(w, cb) - S;                               /* COM velocity */
    const V3 a = cross(al, cb) + cross(w, v) - dS;               /* COM acceleration */
    const S3 Iw = rot_sym_r(Rl, K.I);
    const V3 Iww = mul(Iw, w);
    const float wn = norm(w);
    const V3 Iow = mul(Rl, mul_sym(K.Iown, mul_t(Rl, w)));
    V3 F = K.mass * (a - g);
    V3 T = mul(Iw, al) + cross(w, Iww) + (m.ang_damp + m.ang_damp * wn) * Iow;
    {
        /* damping m v (k + k|v|): per link; the link-7 group per body (lane 6's values) */
        const V3 Fd = (K.mass * (m.lin_damp + m.lin_damp * norm(v))) * v;
        V3 Fg = v3(0, 0, 0), Tg = v3(0, 0, 0);
#pragma unroll
        for (int b = 0; b < PGX_NDAMP; b++) {
            const V3 rb = mulc(Rl, kDpos[b]);
            const V3 vb = u + cross(w, rb);
            const V3 fd = (kDmass[b] * (m.lin_damp + m.lin_damp * norm(vb))) * vb;
            Fg = Fg + fd;
            Tg = Tg + cross(ol + rb - cw, fd);
        }
        F = F + v3(lane_sel<NJ - 1>(Fg.x, Fd.x), lane_sel<NJ - 1>(Fg.y, Fd.y), lane_sel<NJ - 1>(Fg.z, Fd.z));
        T = T + v3(lane_sel<NJ - 1>(Tg.x, 0.0f), lane_sel<NJ - 1>(Tg.y, 0.0f), lane_sel<NJ - 1>(Tg.z, 0.0f));
    }
    const V3 Fs = row_suf(link_only(F));
    const V3 Ms = row_suf(link_only(T + cross(cb, F)));
    const float nbl = -dot(zl, Ms - cross(ob_l, Fs));
    float nb[NJ];
    sfor<0, NJ>([&](auto jc) __attribute__((always_inline)) {
        constexpr int j = decltype(jc)::value;
        nb[j] = bcast16<j>(nbl);
    });
    PGX_PROF_MARK(14);

    /* ---- mass matrix (CRBA) by suffix sums of mass, first moment and base-referred inertia */
    float Mt[NJ][NJ];
    {
        const float ml = link_only(K.mass);
        const S3 st = steiner(ml, cb);
        const float Mc = row_suf(ml);
        const V3 H = row_suf(ml * cb);
        const float Ixx = row_suf(link_only(Iw.xx + st.xx)), Iyy = row_suf(link_only(Iw.yy + st.yy));
        const float Izz = row_suf(link_only(Iw.zz + st.zz)), Ixy = row_suf(link_only(Iw.xy + st.xy));
        const float Ixz = row_suf(link_only(Iw.xz + st.xz)), Iyz = row_suf(link_only(Iw.yz + st.yz));
        const S3 Is = {Ixx, Iyy, Izz, Ixy, Ixz, Iyz};
        const V3 f = cross(zl, H - Mc * ob_l);
        const float Ho = dot(H, ob_l), oz = dot(ob_l, zl), Hz = dot(H, zl), oo = dot(ob_l, ob_l);
        const V3 n = mul(Is, zl) + (Mc * oo - 2.0f * Ho) * zl + oz * H + Hz * ob_l - (Mc * oz) * ob_l;
        float colv[NJ];
#pragma unroll
        for (int i = 0; i < NJ; i++) colv[i] = dot(z[i], n + cross(ol - o[i], f));   /* M[c][i], i <= c */
        sfor<0, NJ>([&](auto jc) __attribute__((always_inline)) {
            constexpr int j = decltype(jc)::value;
            sfor<0, j + 1>([&](auto ic) __attribute__((always_inline)) {
                constexpr int i = decltype(ic)::value;
                Mt[j][i] = bcast16<j>(colv[i]);
            });
        });
    }
    chol7(Mt);
    float (&vu)[NJ] = D.vu;
    {
        float qdd[NJ];
        chol7_solve(Mt, nb, qdd);
#pragma unroll
        for (int j = 0; j < NJ; j++) vu[j] = fminf(fmaxf(qd[j] + m.dt * qdd[j], -m.max_vel), m.max_vel);
    }

    PGX_PROF_MARK(15);
    /* M^-1 lane-parallel: lane c solves L L^T x = e_c (its column; e = 0 on lanes >= 7), the
     * diagonal is broadcast from the lanes that own it */
    {
        float y[NJ], x[NJ];
        sfor<0, NJ>([&](auto ic) __attribute__((always_inline)) {
            constexpr int i = decltype(ic)::value;
            float sacc = lane_sel<i>(1.0f, 0.0f);
#pragma unroll
            for (int k = 0; k < i; k++) sacc -= Mt[i][k] * y[k];
            y[i] = sacc * Mt[i][i];   /* chol7 stores the inverted diagonal */
        });
#pragma unroll
        for (int i = NJ - 1; i >= 0; i--) {
            float sacc = y[i];
#pragma unroll
            for (int k = i + 1; k < NJ; k++) sacc -= Mt[k][i] * x[k];
            x[i] = sacc * Mt[i][i];
        }
#pragma unroll
        for (int k = 0; k < NJ; k++) D.mcol[k] = x[k];
        sfor<0, NJ>([&](auto dc) __attribute__((always_inline)) {
            constexpr int d = decltype(dc)::value;
            D.mdiag[d] = bcast16<d>(x[d]);
        });
    }
    V3& vcu = D.vcu;
    V3& wcu = D.wcu;
    vcu = v3(0, 0, 0);
    wcu = v3(0, 0, 0);
    if (OBJ) {
        const float vn = norm(ob.v), wn2 = norm(ob.w);
        vcu = ob.v + m.dt * (g - (m.lin_damp + m.lin_damp * vn) * ob.v - cross(ob.w, ob.v));
        wcu = ob.w - (m.dt * (m.ang_damp + m.ang_damp * wn2)) * ob.w;
    }
}

/* floating-base object: v, w after the constraint pass; p += dt v, orientation by the
 * exponential map (btMultiBody::stepPositionsMultiDof) */
__device__ __forceinline__ void object_integrate(MRef m, ObjState& ob, V3 v, V3 w) {
    ob.v = v;
    ob.w = w;
    ob.p = ob.p + m.dt * ob.v;
    /* btMultiBody::stepPositionsMultiDof, base: exponential map of w dt */
    float ang = norm(ob.w);
    if (ang * m.dt > 0.39269908f) ang = 0.39269908f * m.inv_dt;
    const float hdt = 0.5f * m.dt;
    const float f = ang < 0.001f ? (hdt - m.dt * m.dt * m.dt * 0.020833333333f * ang * ang)
                                 : __sinf(ang * hdt) * fast_rcp(ang);
    const float ax = ob.w.x * f, ay = ob.w.y * f, az = ob.w.z * f, aw = __cosf(ang * hdt);
    /* dq * q (Hamilton, (x,y,z,w)) */
    const float nx = aw * ob.qx + ax * ob.qw + ay * ob.qz - az * ob.qy;
    const float ny = aw * ob.qy + ay * ob.qw + az * ob.qx - ax * ob.qz;
    const float nz = aw * ob.qz + az * ob.qw + ax * ob.qy - ay * ob.qx;
    const float nw = aw * ob.qw - ax * ob.qx - ay * ob.qy - az * ob.qz;
    const float inn = __builtin_amdgcn_rsqf(nx * nx + ny * ny + nz * nz + nw * nw);
    ob.qx = nx * inn; ob.qy = ny * inn; ob.qz = nz * inn; ob.qw = nw * inn;
}

template <int OBJ, int CONT, int AO = 0>
__device__ __forceinline__ void substep(MPtr mp, const PgxDevEnv& e, float* q, float* qd, const float* tq,
                                        ObjState& ob, ContactLds* Lp, int ln) {
    MRef m = *fresh(mp);
    Dyn D;
    substep_dyn<OBJ, CONT, ContactLds, false, AO>(m, e, q, qd, ob, Lp, ln, D);
    const V3 (&z)[NJ] = D.z;
    const V3 (&o)[NJ] = D.o;
    const float (&Mi)[NJ][NJ] = D.Mi;
    const float (&vu)[NJ] = D.vu;
    const V3 vcu = D.vcu, wcu = D.wcu;
#define MINV(a, b) ((a) >= (b) ? Mi[a][b] : Mi[b][a])
    PGX_PROF_MARK(2);
#ifdef PGX_NAN_TRAP
    {
        float mid[NJ];
        for (int j = 0; j < NJ; j++) mid[j] = Mi[j][j];
        PGX_TRAP(1, 0, vu, NJ, m);
        PGX_TRAP(2, 0, mid, NJ, m);
    }
#endif
    float dv[NJ];
#pragma unroll
    for (int j = 0; j < NJ; j++) dv[j] = 0.0f;
    V3 dvl = v3(0, 0, 0), dvw = v3(0, 0, 0);   /* object velocity deltas */
    const float inv_m = e.obj_inv_mass, inv_i = e.obj_inv_inertia;

    /* ---- contact rows (setup + warm start) */
    int n0 = 0, n1 = 0;
    float mu1[CG];   /* the robot points' combined friction (point_mu) */
#pragma unroll
    for (int k = 0; k < CG; k++) mu1[k] = m.friction;
    if (CONT) {
        ContactLds& L = *Lp;
        n0 = L.cnt[0][ln];
        n1 = L.cnt[1][ln];
        const float erp_dt = m.contact_erp * m.inv_dt;
        for (int k = 0; k < CG; k++) {
            if (OBJ && k < n0) {
                const float4 r4 = L.g0q[k][0][ln];
                const V3 r = v3(r4.x, r4.y, r4.z);
                const float id = L.g0id[k][ln];
                const float warm = warm_lookup<CG>(L, ln, 0, id, m.warmstart);
                V3 t1, t2;
                const V3 nk = lds3(L.g0n[k], ln);
                plane_space(nk, t1, t2);
#pragma unroll
                for (int dir = 0; dir < 3; dir++) {
                    /* u = n, then btPlaneSpace1(n); ang = r x u */
                    const V3 lin = dir == 0 ? nk : (dir == 1 ? t1 : t2);
                    const V3 ang = cross(r, lin);
                    const float den = inv_m + dot(ang, ang) * inv_i;
                    const float jinv = den > 2.220446e-16f ? fast_rcp(den) : 0.0f;
                    const float rel = dot(lin, vcu) + dot(ang, wcu);
                    float rhs;
                    if (dir == 0) {
                        const float pen = L.g0d[k][ln];
                        rhs = (pen > 0.0f ? (-rel - pen * m.inv_dt) : (-pen * erp_dt - rel)) * jinv;
                    } else {
                        rhs = -rel * jinv;
                    }
                    const float lam = dir == 0 ? warm : 0.0f;
                    L.g0q[k][1 + dir][ln] = make_float4(jinv, den, rhs, lam);
                    if (dir == 0) { dvl = dvl + (lam * inv_m) * lin; dvw = dvw + (lam * inv_i) * ang; }
                }
            }
            if (k < n1) {
                const V3 P = v3(L.g1p[k][0][ln], L.g1p[k][1][ln], L.g1p[k][2][ln]);
                const V3 n = v3(L.g1n[k][0][ln], L.g1n[k][1][ln], L.g1n[k][2][ln]);
                const V3 rb = v3(L.g1rb[k][0][ln], L.g1rb[k][1][ln], L.g1rb[k][2][ln]);
                const int jl = L.g1j[k][ln];
                const float id = L.g1id[k][ln];
                mu1[k] = point_mu<AO>(m, id);
                const bool vs_obj = OBJ && id >= kTableIdLimit;
                const float warm = warm_lookup<CG>(L, ln, CACHE1, id, m.warmstart);
                V3 t1, t2;
                plane_space(n, t1, t2);
                V3 Jv[NJ];
#pragma unroll
                for (int a = 0; a < NJ; a++) Jv[a] = a <= jl ? cross(z[a], P - o[a]) : v3(0, 0, 0);
#pragma unroll
                for (int dir = 0; dir < 3; dir++) {
                    const V3 u = dir == 0 ? n : (dir == 1 ? t1 : t2);
                    float J[NJ], Rs[NJ];
                    float den = 0.0f, rel = 0.0f;
#pragma unroll
                    for (int a = 0; a < NJ; a++) { J[a] = dot(u, Jv[a]); rel += J[a] * vu[a]; }
#pragma unroll
                    for (int a = 0; a < NJ; a++) {
                        float s = 0.0f;
#pragma unroll
                        for (int b = 0; b < NJ; b++) s += MINV(a, b) * J[b];
                        Rs[a] = s;
                        den += J[a] * s;
                    }
                    V3 cl = v3(0, 0, 0), ca = v3(0, 0, 0);
                    if (vs_obj) {
                        cl = -1.0f * u;
                        ca = -1.0f * cross(rb, u);
                        den += inv_m * dot(cl, cl) + inv_i * dot(ca, ca);
                        rel += dot(cl, vcu) + dot(ca, wcu);
                    }
                    const float jinv = den > 2.220446e-16f ? fast_rcp(den) : 0.0f;
                    float rhs;
                    if (dir == 0) {
                        const float pen = L.g1d[k][ln];
                        rhs = (pen > 0.0f ? (-rel - pen * m.inv_dt) : (-pen * erp_dt - rel)) * jinv;
                    } else {
                        rhs = -rel * jinv;
                    }
                    const float lam = dir == 0 ? warm : 0.0f;
                    L.g1q[k][dir][0][ln] = make_float4(J[0], J[1], J[2], J[3]);
                    L.g1q[k][dir][1][ln] = make_float4(J[4], J[5], J[6], jinv);
                    L.g1q[k][dir][2][ln] = make_float4(Rs[0], Rs[1], Rs[2], Rs[3]);
                    L.g1q[k][dir][3][ln] = make_float4(Rs[4], Rs[5], Rs[6], den);
                    L.g1q[k][dir][4][ln] = make_float4(cl.x, cl.y, cl.z, rhs);
                    L.g1q[k][dir][5][ln] = make_float4(ca.x, ca.y, ca.z, lam);
                    if (dir == 0) {
#pragma unroll
                        for (int a = 0; a < NJ; a++) dv[a] += Rs[a] * lam;
                        if (OBJ) { dvl = dvl + (lam * inv_m) * cl; dvw = dvw + (lam * inv_i) * ca; }
                    }
                }
            }
        }
    }
    /* accumulated contact impulses live in VGPRs during the sweeps, so the LDS row
     * records stay read-only and their loads can be issued ahead of the dependent math */
    float lam0[CG][3], lam1[CG][3];
#pragma unroll
    for (int k = 0; k < CG; k++)
#pragma unroll
        for (int dir = 0; dir < 3; dir++) {
            lam0[k][dir] = (CONT && OBJ && k < n0) ? Lp->g0q[k][1 + dir][ln].w : 0.0f;
            lam1[k][dir] = (CONT && k < n1) ? Lp->g1q[k][dir][5][ln].w : 0.0f;
        }

    /* rows (btMultiBodyJointMotor / btMultiBodyJointLimitConstraint::createConstraintRows):
     * jinv depends only on the dof, bounds are constants, so per row only rhs and
     * the accumulated impulse live in registers. */
    float den[NJ], jinv[NJ];
#pragma unroll
    for (int d = 0; d < NJ; d++) {
        den[d] = Mi[d][d];
        jinv[d] = den[d] > 2.220446e-16f ? fast_rcp(den[d]) : 0.0f; /* SIMD_EPSILON guard */
    }
    float rhs[PGX_N_ROWS], lam[PGX_N_ROWS];
#pragma unroll
    for (int r = 0; r < PGX_N_ROWS; r++) {
        const int kind = kPgxRowCode[r] >> 4, d = kPgxRowCode[r] & 15;
        const float rel = kind == 2 ? -vu[d] : vu[d];
        lam[r] = 0.0f;
        if (kind == 0) {
            float pos_term = (tq[d] - q[d]) * m.inv_dt;
            float desired = m.kp * pos_term + vu[d] + m.kd * (0.0f - vu[d]);
            rhs[r] = (desired - rel) * jinv[d];
        }
    }
    auto init_limit_rows = [&]() {
#pragma unroll
        for (int r = 0; r < PGX_N_ROWS; r++) {
            const int kind = kPgxRowCode[r] >> 4, d = kPgxRowCode[r] & 15;
            if (kind == 0) continue;
            const float rel = kind == 2 ? -vu[d] : vu[d];
            float pen = kind == 1 ? (q[d] - kLower[d]) : (kUpper[d] - q[d]);
            float verr = -rel, perr = 0.0f;
            if (pen > 0.0f) verr -= pen * m.inv_dt;
            else perr = -pen * m.erp * m.inv_dt;
            rhs[r] = (perr + verr) * jinv[d];
        }
    };
    /* Exact skip of the joint-limit rows.  With only motor impulses |lambda_k| <= F_k dt
     * applied, |dv_d| <= B_d = sum_k |Minv_dk| F_k dt.  A not-violated limit row of dof d
     * can only get a positive impulse once vu_d + dv_d crosses -pen/dt (lower) or
     * +pen/dt (upper); if that is impossible for every limit row, none ever leaves 0
     * during the sweep (by induction), every evaluation of them clamps to delta = 0,
     * and dropping them changes no bit of the result or of the exit iteration.  Robot
     * contact impulses are unbounded, so the skip needs an env without robot contacts. */
    bool far_nc = true;   /* the motor-impulse bound alone keeps every limit row idle */
#pragma unroll
    for (int d = 0; d < NJ; d++) {
        float B = 0.0f;
#pragma unroll
        for (int k = 0; k < NJ; k++) B += fabsf(MINV(d, k)) * m.max_impulse[k];
        B = B * 1.001f + 1e-6f;
        const float penl = q[d] - kLower[d], penu = kUpper[d] - q[d];
        far_nc = far_nc && penl > 0.0f && penu > 0.0f && (vu[d] - B) > -penl * m.inv_dt &&
                 (vu[d] + B) < penu * m.inv_dt;
    }
    const bool far = far_nc && n1 == 0;
    /* resolveSingleConstraintRowGeneric, branch-free: clamp the accumulated impulse,
     * apply the clamped delta through the unit response M^-1 J^T (a column of M^-1). */
    auto row = [&](const int r, float& resid) {
        const int kind = kPgxRowCode[r] >> 4, d = kPgxRowCode[r] & 15;
        const float lo = kind == 0 ? -m.max_impulse[d] : 0.0f;
        const float hi = kind == 0 ? m.max_impulse[d] : m.limit_max_imp;
        const float vd = kind == 2 ? -dv[d] : dv[d];
        float delta = fmaf(-vd, jinv[d], rhs[r]);
        /* v_med3 with the bounds straight from SGPRs (lo <= hi always holds) */
        const float nl = __builtin_amdgcn_fmed3f(lam[r] + delta, lo, hi);
        delta = nl - lam[r];
        lam[r] = nl;
        const float sd = kind == 2 ? -delta : delta;
        /* No branch around the column update: a wave-uniform skip of zero-delta rows
         * (__any) measured 1.46x slower (it splits the sweep into basic blocks). */
#pragma unroll
        for (int cc = 0; cc < NJ; cc++) dv[cc] += MINV(cc, d) * sd;
        /* track max |row residual|; fl(x^2) is monotone in |x|, so squaring the max
         * once per sweep equals the max of the squares */
        resid = fmaxf(resid, fabsf(delta * den[d]));
    };
    /* contact rows: normal rows of both groups, then friction rows (bounds from the
     * current normal impulse, skipped while it is 0) */
    /* friction coefficient in a register: a model load inside the bound selects makes the
     * compiler branch around it (a scalar load + wait per friction row) */
    float mu = m.friction;
    asm("" : "+s"(mu));
    const bool g0_any = CONT && OBJ && __any(n0 > 0);
    const bool g1_any = CONT && __any(n1 > 0);
    auto contact_rows = [&](float& resid) {
        const ContactLds& L = *Lp;
#pragma unroll
        for (int fr = 0; fr < 2; fr++) {
            if (OBJ && g0_any) {   /* wave-uniform; inside, inactive points are predicated off */
#pragma unroll
                for (int k = 0; k < CG; k++) {
                    const bool act = k < n0;   /* a resting cube has 4: predicate, no branch */
                    {
                        const float4 r4 = L.g0q[k][0][ln];
                        const V3 r = v3(r4.x, r4.y, r4.z);
                        const float ln_n = lam0[k][0];
                        /* the point's normal (a side wall's since round 6) and btPlaneSpace1 of it */
                        V3 nk = lds3(L.g0n[k], ln), t1, t2;
                        nk = act ? nk : v3(0.0f, 0.0f, 1.0f);
                        plane_space(nk, t1, t2);
#pragma unroll
                        for (int dir = fr ? 1 : 0; dir < (fr ? 3 : 1); dir++) {
                            const V3 u = dir == 0 ? nk : (dir == 1 ? t1 : t2);
                            const V3 a = cross(r, u);
                            const float4 rw = L.g0q[k][1 + dir][ln];
                            const float jv = rw.x, dn = rw.y, rh = rw.z, lm = lam0[k][dir];
                            const float lo = fr ? -mu * ln_n : 0.0f;
                            const float hi = fr ? mu * ln_n : 1e10f;
                            const float jdv = dot(u, dvl) + dot(a, dvw);
                            float delta = rh - jdv * jv;
                            const float nl = __builtin_amdgcn_fmed3f(lm + delta, lo, hi);
                            /* a friction row waits for a positive normal impulse */
                            delta = (!act || (fr && !(ln_n > 0.0f))) ? 0.0f : nl - lm;
                            lam0[k][dir] = lm + delta;
                            const float sm = delta * inv_m, si = delta * inv_i;
                            dvl = dvl + sm * u;
                            dvw = dvw + si * a;
                            resid = fmaxf(resid, fabsf(delta * dn));
                        }
                    }
                }
            }
            if (!g1_any) continue;
#pragma unroll
            for (int k = 0; k < CG; k++) {
                const bool act = k < n1;   /* robot points are sparse: skip idle slots */
                if (__any(act) && act) {
                    const float ln_n = lam1[k][0];
#pragma unroll
                    for (int dir = fr ? 1 : 0; dir < (fr ? 3 : 1); dir++) {
                        const float4 q0 = L.g1q[k][dir][0][ln], q1 = L.g1q[k][dir][1][ln];
                        const float4 q2 = L.g1q[k][dir][2][ln], q3 = L.g1q[k][dir][3][ln];
                        const float4 q4 = L.g1q[k][dir][4][ln], q5 = L.g1q[k][dir][5][ln];
                        const float jv = q1.w, dn = q3.w, rh = q4.w, lm = lam1[k][dir];
                        const float lo = fr ? -mu1[k] * ln_n : 0.0f;
                        const float hi = fr ? mu1[k] * ln_n : 1e10f;
                        /* two partial sums: half the dependent-FMA chain */
                        float ja = q0.x * dv[0] + q0.z * dv[2] + q1.x * dv[4] + q1.z * dv[6];
                        float jb = q0.y * dv[1] + q0.w * dv[3] + q1.y * dv[5];
                        V3 cl = v3(0, 0, 0), ca = v3(0, 0, 0);
                        if (OBJ) {
                            cl = v3(q4.x, q4.y, q4.z);
                            ca = v3(q5.x, q5.y, q5.z);
                            jb += dot(cl, dvl) + dot(ca, dvw);
                        }
                        const float jdv = ja + jb;
                        float delta = rh - jdv * jv;
                        const float nl = __builtin_amdgcn_fmed3f(lm + delta, lo, hi);
                        delta = (!act || (fr && !(ln_n > 0.0f))) ? 0.0f : nl - lm;
                        lam1[k][dir] = lm + delta;
                        dv[0] += q2.x * delta; dv[1] += q2.y * delta; dv[2] += q2.z * delta; dv[3] += q2.w * delta;
                        dv[4] += q3.x * delta; dv[5] += q3.y * delta; dv[6] += q3.z * delta;
                        if (OBJ) { dvl = dvl + (delta * inv_m) * cl; dvw = dvw + (delta * inv_i) * ca; }
                        resid = fmaxf(resid, fabsf(delta * dn));
                    }
                }
            }
        }
    };
    const bool any_contact = CONT && __any(n0 > 0 || n1 > 0);
    /* Sweeps alternate direction (Bullet reverses the row order on even iterations); the
     * loop body holds one even (reverse) and one odd (forward) sweep, so no value has to
     * be merged from two branch arms (that cost ~35 v_mov per sweep). */
    const int n_it = m.num_iterations;
    /* the exit threshold in an SGPR before the sweeps: read from the model inside the loop it
     * costs a scalar load and its s_waitcnt on every sweep */
    float res_thr = m.residual_abs;
    asm("" : "+s"(res_thr));
    PGX_TRAP(3, n1, dv, NJ, m);
    PGX_TRAP(8, n1, rhs, NJ, m);
    PGX_PROF_MARK(3);
    PGX_PROF_COUNT(9, 1);
    PGX_PROF_SWEEPS_DECL;
    if (__all(far)) {
        for (int it = 0; it < n_it; it += 2) {
            float resid = 0.0f;
#pragma unroll
            for (int r = PGX_N_ROWS - 1; r >= 0; r--)
                if ((kPgxRowCode[r] >> 4) == 0) row(r, resid);
            if (CONT && any_contact) contact_rows(resid);
            PGX_PROF_SWEEP();
            if (resid <= res_thr || it + 1 >= n_it) break;
            resid = 0.0f;
#pragma unroll
            for (int r = 0; r < PGX_N_ROWS; r++)
                if ((kPgxRowCode[r] >> 4) == 0) row(r, resid);
            if (CONT && any_contact) contact_rows(resid);
            PGX_PROF_SWEEP();
            if (resid <= res_thr) break;
        }
    } else {
        PGX_PROF_COUNT(10, 1);
        init_limit_rows();
        /* Speculative solve (as substep_g's MODE 1): when the motor-impulse bound alone keeps
         * every limit row idle in every env of the wave (only robot-contact impulses, which
         * are unbounded, stand in the way of the far solve), sweep without the 14 limit rows
         * and check, at each position the limit block takes in the order (the head of the
         * reversed sweep, after the motor rows of the forward one), that each of them would
         * compute delta = fma(-v, jinv, rhs) <= 0 there: with lambda = 0 that row clamps to
         * 0 and leaves dv, lambda and the residual bit for bit unchanged, and a block of
         * no-ops leaves dv constant across it, so one check per position covers all 14.  A
         * wave where any env fails is solved again from the same start with every row. */
        bool redo = true;
        if (CONT && e.pgs_mode != 2 && __all(far_nc)) {
            float rl[NJ], ru[NJ];
#pragma unroll
            for (int r = NJ; r < PGX_N_ROWS; r++) {
                const int kind = kPgxRowCode[r] >> 4, d = kPgxRowCode[r] & 15;
                if (kind == 1) rl[d] = rhs[r];
                else ru[d] = rhs[r];
            }
            ContactLds& L = *Lp;
#pragma unroll
            for (int j = 0; j < NJ; j++) L.spec0[j][ln] = dv[j];
            L.spec0[NJ][ln] = dvl.x; L.spec0[NJ + 1][ln] = dvl.y; L.spec0[NJ + 2][ln] = dvl.z;
            L.spec0[NJ + 3][ln] = dvw.x; L.spec0[NJ + 4][ln] = dvw.y; L.spec0[NJ + 5][ln] = dvw.z;
            /* the smallest -delta seen: a limit row would act exactly when it is negative */
            float lmargin = 3.0e38f;
            auto limit_check = [&]() {
#pragma unroll
                for (int d = 0; d < NJ; d++)
                    lmargin = fminf(lmargin, fminf(-fmaf(-dv[d], jinv[d], rl[d]), -fmaf(dv[d], jinv[d], ru[d])));
            };
            for (int it = 0; it < n_it; it += 2) {
                float resid = 0.0f;
                limit_check();
#pragma unroll
                for (int r = PGX_N_ROWS - 1; r >= 0; r--)
                    if ((kPgxRowCode[r] >> 4) == 0) row(r, resid);
                if (CONT && any_contact) contact_rows(resid);
                PGX_PROF_SWEEP();
                if (resid <= res_thr || it + 1 >= n_it) break;
                resid = 0.0f;
#pragma unroll
                for (int r = 0; r < PGX_N_ROWS; r++)
                    if ((kPgxRowCode[r] >> 4) == 0) row(r, resid);
                limit_check();
                if (CONT && any_contact) contact_rows(resid);
                PGX_PROF_SWEEP();
                if (resid <= res_thr) break;
            }
            redo = __any(lmargin < 0.0f) || e.pgs_mode == 3;
            if (redo) {   /* back to the start: velocities, impulses (warm starts from the records) */
                PGX_PROF_COUNT(12, 1);
#pragma unroll
                for (int j = 0; j < NJ; j++) dv[j] = L.spec0[j][ln];
                dvl = v3(L.spec0[NJ][ln], L.spec0[NJ + 1][ln], L.spec0[NJ + 2][ln]);
                dvw = v3(L.spec0[NJ + 3][ln], L.spec0[NJ + 4][ln], L.spec0[NJ + 5][ln]);
#pragma unroll
                for (int r = 0; r < PGX_N_ROWS; r++) lam[r] = 0.0f;
#pragma unroll
                for (int k = 0; k < CG; k++)
#pragma unroll
                    for (int dir = 0; dir < 3; dir++) {
                        lam0[k][dir] = (CONT && OBJ && k < n0) ? L.g0q[k][1 + dir][ln].w : 0.0f;
                        lam1[k][dir] = (CONT && k < n1) ? L.g1q[k][dir][5][ln].w : 0.0f;
                    }
            }
        } else {
            PGX_PROF_COUNT(13, 1);
        }
        for (int it = 0; redo && it < n_it; it += 2) {
            float resid = 0.0f;
#pragma unroll
            for (int r = PGX_N_ROWS - 1; r >= 0; r--) row(r, resid);
            if (CONT && any_contact) contact_rows(resid);
            PGX_PROF_SWEEP();
            if (resid <= res_thr || it + 1 >= n_it) break;
            resid = 0.0f;
#pragma unroll
            for (int r = 0; r < PGX_N_ROWS; r++) row(r, resid);
            if (CONT && any_contact) contact_rows(resid);
            PGX_PROF_SWEEP();
            if (resid <= res_thr) break;
        }
    }
#undef MINV
    PGX_PROF_SWEEPS_DONE();
    PGX_TRAP(4, n1, dv, NJ, m);
    PGX_PROF_MARK(4);
    PGX_PROF_COUNT(11, any_contact ? 1 : 0);
#pragma unroll
    for (int j = 0; j < NJ; j++) {
        float vn = fminf(fmaxf(vu[j] + dv[j], -m.max_vel), m.max_vel);
        qd[j] = vn;
        q[j] += m.dt * vn;
    }
    PGX_TRAP(5, n1, q, NJ, m);
    PGX_TRAP(6, n1, qd, NJ, m);
    if (CONT) { /* contact cache: this step's features and normal impulses */
        ContactLds& L = *Lp;
#pragma unroll
        for (int s = 0; s < CG; s++) {
            L.cache[2 * s][ln] = s < n0 ? L.g0id[s][ln] : -1.0f;
            L.cache[2 * s + 1][ln] = s < n0 ? lam0[s][0] : 0.0f;
            L.cache[8 + 2 * s][ln] = s < n1 ? L.g1id[s][ln] : -1.0f;
            L.cache[8 + 2 * s + 1][ln] = s < n1 ? lam1[s][0] : 0.0f;
        }
    }
    if (OBJ) object_integrate(m, ob, vcu + dvl, wcu + dvw);
    PGX_PROF_MARK(5);
}

/* ======================================================= wide layout: 16 lanes per env */
/* At the headline batch (4096 envs = 64 waves in the one-lane layout, 6 % of the chip's
 * 1024 SIMDs) the step is bound by one wave's dependent instruction stream, 77 % of it
 * the PGS sweeps (tools/prof_phases.py).  The wide layout gives each env one 16-lane DPP
 * row and splits the solver's coordinates over it: lanes 0-6 own the arm dofs'
 * velocity deltas, lanes 7-9 / 10-12 the object's linear / angular ones.  A motor row
 * broadcasts its dof's delta (row_newbcast), a contact row reduces J.dv with a 4-step
 * DPP butterfly, and every lane applies the impulse to its own coordinate, so a row
 * costs ~8 instructions on the critical path instead of ~13 + 14 for the 7-wide column
 * updates and dot products.  Everything else (FK, dynamics, detection, IK, epilogue)
 * runs redundantly and bit-identically on the 16 lanes, so all lanes of an env take the
 * same branches; only the lead lane stores. */
/* One stepSimulation() in the wide layout: the same restatement as substep() (dynamics
 * shared through substep_dyn), rows solved in the same order with the same exit rule. */
/* the row table's limit block: (lower, upper) pairs of one dof each, after the 7 motor rows */
constexpr bool limit_rows_paired() {
    for (int r = 0; r < NJ; r++)
        if ((kPgxRowCode[r] >> 4) != 0) return false;
    for (int r = NJ; r + 1 < PGX_N_ROWS; r += 2)
        if ((kPgxRowCode[r] >> 4) != 1 || (kPgxRowCode[r + 1] >> 4) != 2 ||
            (kPgxRowCode[r] & 15) != (kPgxRowCode[r + 1] & 15))
            return false;
    return (PGX_N_ROWS - NJ) % 2 == 0;
}

template <int OBJ, int CONT, int PART = 1, int AO = 0, int FULL = 0>
__device__ __forceinline__ bool substep_g(MPtr mp, const PgxDevEnv& e, float* q, float* qd, const float* tq,
                                          ObjState& ob, ContactLdsGT<OBJ, FULL>* Lp, int es, int c, const LaneK& K,
                                          bool check = false) {
    MRef m = *fresh(mp);
    /* The object tasks keep the limit rows of the all-rows solve (a failed speculation, limit
     * pairs near two or more dofs) in LDS, and the two-waves-per-SIMD kernel (PART 2, 256
     * registers, taken above 4096 envs) takes that solve instead of the partial one: in
     * registers, those rows beside the 24 contact rows set the kernel's register peak (256 VGPR
     * + 172 AGPR; squeezed into 256 they spilled inside every sweep, PickAndPlace 16384 6.5 ms).
     * PickAndPlace 16384: 2.93 -> 2.59 ms (profiles/r03/ab_lds_limit_rows.log). */
    constexpr bool LDS_LIM = OBJ;
    constexpr bool NO_PART = OBJ && PART == 2;
    constexpr bool PERS = CONT && FULL && (OBJ || (AO && AO_PERS));   /* Bullet's persistent manifolds (the pool) */
    Dyn D;
    substep_dyn_g<OBJ, CONT, AO, FULL>(m, e, q, qd, ob, Lp, es, D, c, K, check);
    if constexpr (AO) {
        if (D.coll) return true;   /* collided at the start pose: this substep does not run */
    }
    const V3 (&z)[NJ] = D.z;
    const V3 (&o)[NJ] = D.o;
    float vu[NJ];
#pragma unroll
    for (int j = 0; j < NJ; j++) vu[j] = D.vu[j];
    V3 vcu = D.vcu, wcu = D.wcu;
    PGX_PROF_MARK(2);
    const bool arm = c < NJ;
    const float inv_m = e.obj_inv_mass, inv_i = e.obj_inv_inertia;
    /* this lane's coordinate: M^-1 row (arm), object inverse mass / inertia, velocity */
    float mcol[NJ];
#pragma unroll
    for (int d = 0; d < NJ; d++) mcol[d] = D.mcol[d];
    const float kobj = OBJ ? ((c >= 7 && c < 10) ? inv_m : ((c >= 10 && c < 13) ? inv_i : 0.0f)) : 0.0f;
    const float vu_c = pick_gen(vu, vcu, wcu);
    float gv = 0.0f;   /* this lane's velocity delta */

    /* ---- contact rows: per lane J_c and (M^-1 J^T)_c, per row rhs / jinv / den / lambda */
    constexpr int P0 = OBJ ? CG : 0;            /* group-1 rows follow group 0's */
    constexpr int CGR = ContactLdsGT<OBJ, FULL>::CGR;   /* robot points with register (Delassus) rows */
    constexpr int NP = P0 + (CONT ? CGR : 0);
    constexpr int RB = CONT ? ContactLdsGT<OBJ, FULL>::RB : CGR;   /* robot budget: points CGR.. are the extra rows */
    constexpr int NQR = ContactLdsGT<OBJ, FULL>::NQR;
    constexpr int NC_ = OBJ ? 13 : NJ;          /* generalized coordinates in lanes */
    /* extra points run in the sweep: multiples of XSTEP, one sweep copy per multiple (round 4:
     * 4 -> 2 -> 1, Push 2.29 -> 2.04 -> 2.02 ms, ReachAO 8192 0.93 -> 0.82 -> 0.77 ms; the
     * waves with extra points are the launch's tail, and their envs rarely use all of them;
     * a runtime loop over the points instead, row data in LDS: Push 3.0 ms,
     * profiles/r04/ab_extra_rows_*.log) */
    constexpr int XSTEP = 1;
    int n1x = 0;                                /* the wave's largest robot point count, when above CGR */
    int nxr = 0;                                /* extra points the sweep runs: n1x - CGR rounded up to XSTEP */
    float cJ[NP > 0 ? NP : 1][3], cR[NP > 0 ? NP : 1][3], crhs[NP > 0 ? NP : 1][3], cjinv[NP > 0 ? NP : 1][3];
    float cden[NP > 0 ? NP : 1][3], clam[NP > 0 ? NP : 1][3];
    float pmu[NP > 0 ? NP : 1];   /* the points' combined lateral friction (object scene: m.friction) */
    bool act[NP > 0 ? NP : 1];
    int n0 = 0, n1 = 0;
    if (CONT) {
        ContactLdsGT<OBJ, FULL>& L = *Lp;
        n0 = L.cnt[0][es];
        n1 = L.cnt[1][es];
        const float erp_dt = m.contact_erp * m.inv_dt;
        /* the warm-start cache slots, read once for every point (ids, impulses) */
        float cid0[CG], cim0[CG], cid1[CGR], cim1[CGR];
#pragma unroll
        for (int s2 = 0; s2 < CG; s2++) {
            cid0[s2] = OBJ ? L.cache[2 * s2][es] : -1.0f;
            cim0[s2] = OBJ ? L.cache[2 * s2 + 1][es] : 0.0f;
        }
#pragma unroll
        for (int s2 = 0; s2 < CGR; s2++) {
            cid1[s2] = L.cache[CACHE1 + 2 * s2][es];
            cim1[s2] = L.cache[CACHE1 + 2 * s2 + 1][es];
        }
        auto warm_of = [&](const float* ids, const float* ims, auto n_c, float id) __attribute__((always_inline)) {
            float w = 0.0f;
#pragma unroll
            for (int s2 = 0; s2 < decltype(n_c)::value; s2++) w = ids[s2] == id ? m.warmstart * ims[s2] : w;
            return w;
        };
#pragma unroll
        for (int p = 0; p < NP; p++) pmu[p] = m.friction;
#pragma unroll
        for (int k = 0; k < P0; k++) { /* object vertices vs the table / plane: object coordinates only */
            act[k] = k < n0;
            const float4 r4 = L.g0q[k][0][es];
            const V3 r = v3(r4.x, r4.y, r4.z);
            const float id = L.g0id[k][es];
            const float warm = warm_of(cid0, cim0, IC<CG>{}, id);
            /* the point's normal (+z on the table top and the plane; a side wall's, round 6) and
             * btPlaneSpace1 of it */
            V3 nk = lds3(L.g0n[k], es), t1, t2;
            nk = act[k] ? nk : v3(0.0f, 0.0f, 1.0f);
            plane_space(nk, t1, t2);
#pragma unroll
            for (int dir = 0; dir < 3; dir++) {
                const V3 lin = dir == 0 ? nk : (dir == 1 ? t1 : t2);
                const V3 ang = cross(r, lin);
                const float den = inv_m + dot(ang, ang) * inv_i;
                const float jinv = den > 2.220446e-16f ? fast_rcp(den) : 0.0f;
                const float rel = dot(lin, vcu) + dot(ang, wcu);
                float rhs;
                if (dir == 0) {
                    const float pen = L.g0d[k][es];
                    rhs = (pen > 0.0f ? (-rel - pen * m.inv_dt) : (-pen * erp_dt - rel)) * jinv;
                } else {
                    rhs = -rel * jinv;
                }
                const float J = pick_obj(lin, ang);
                cJ[k][dir] = act[k] ? J : 0.0f;
                cR[k][dir] = act[k] ? J * kobj : 0.0f;
                crhs[k][dir] = act[k] ? rhs : 0.0f;
                cjinv[k][dir] = act[k] ? jinv : 0.0f;
                cden[k][dir] = act[k] ? den : 0.0f;
                clam[k][dir] = (act[k] && dir == 0) ? warm : 0.0f;
                gv += cR[k][dir] * clam[k][dir];
            }
        }
        /* robot vs table / plane / object: this lane's joint axis and pivot */
        const V3 zc = pick_v3(z), oc = pick_v3(o);
        /* the points' records read up front, one batch behind one wait (read inside each point's
         * branch they cost a wait per point) */
        V3 gP[CGR], gN[CGR], gRb[CGR];
        int gJ[CGR], gW[CGR];
        float gId[CGR], gD[CGR];
        auto read_point = [&](int k) __attribute__((always_inline)) {
            gP[k] = v3(L.g1p[k][0][es], L.g1p[k][1][es], L.g1p[k][2][es]);
            gN[k] = v3(L.g1n[k][0][es], L.g1n[k][1][es], L.g1n[k][2][es]);
            gRb[k] = OBJ ? v3(L.g1rb[k][0][es], L.g1rb[k][1][es], L.g1rb[k][2][es]) : v3(0.0f, 0.0f, 0.0f);
            gJ[k] = L.g1j[k][es];
            gW[k] = PERS ? L.g1w[k][es] : -1;
            gId[k] = L.g1id[k][es];
            gD[k] = L.g1d[k][es];
        };
        /* a manifold point's warm start is its own applied impulse (btManifoldPoint::m_appliedImpulse
         * x the warm-starting factor), a fresh table point's its feature's cached one */
        auto warm_pt = [&](int w, float id) __attribute__((always_inline)) {
            return (PERS && w >= 0) ? m.warmstart * L.mimp[w < 0 ? 0 : w][es] : warm_of(cid1, cim1, IC<CGR>{}, id);
        };
        /* (ReachAO: points are rare and the o2 kernel's registers scarce: read per point) */
        if (!AO && __any(n1 > 0)) {
#pragma unroll
            for (int k = 0; k < CGR; k++) read_point(k);
        }
#pragma unroll
        for (int k = 0; k < (CONT ? CGR : 0); k++) {
            const int p = P0 + k;
            act[p] = k < n1;
#pragma unroll
            for (int dir = 0; dir < 3; dir++) {
                cJ[p][dir] = 0.0f; cR[p][dir] = 0.0f; crhs[p][dir] = 0.0f;
                cjinv[p][dir] = 0.0f; cden[p][dir] = 0.0f; clam[p][dir] = 0.0f;
            }
            if (__any(act[p])) {   /* wave-uniform; robot points are sparse */
                if (AO) read_point(k);
                const V3 P = gP[k];
                const V3 n = gN[k];
                const V3 rb = gRb[k];
                const int jl = gJ[k];
                const float id = gId[k];
                pmu[p] = point_mu<AO, FULL>(m, id);
                const bool vs_obj = OBJ && id >= kTableIdLimit;
                const float warm = warm_pt(gW[k], id);
                V3 t1, t2;
                plane_space(n, t1, t2);
                const V3 Jv = (arm && c <= jl) ? cross(zc, P - oc) : v3(0, 0, 0);
#pragma unroll
                for (int dir = 0; dir < 3; dir++) {
                    const V3 u = dir == 0 ? n : (dir == 1 ? t1 : t2);
                    float J = dot(u, Jv);
                    if (OBJ) {
                        const V3 ca = cross(rb, u);
                        const float oj = pick_obj(-1.0f * u, -1.0f * ca);
                        J = (!arm && vs_obj) ? oj : J;
                    }
                    float R = kobj * J;
                    sfor<0, NJ>([&](auto bc) __attribute__((always_inline)) {
                        constexpr int b = decltype(bc)::value;
                        R += mcol[b] * bcast16<b>(J);
                    });
                    const float den = sum16(J * R);
                    const float rel = sum16(J * vu_c);
                    const float jinv = den > 2.220446e-16f ? fast_rcp(den) : 0.0f;
                    float rhs;
                    if (dir == 0) {
                        const float pen = gD[k];
                        rhs = (pen > 0.0f ? (-rel - pen * m.inv_dt) : (-pen * erp_dt - rel)) * jinv;
                    } else {
                        rhs = -rel * jinv;
                    }
                    cJ[p][dir] = act[p] ? J : 0.0f;
                    cR[p][dir] = act[p] ? R : 0.0f;
                    crhs[p][dir] = act[p] ? rhs : 0.0f;
                    cjinv[p][dir] = act[p] ? jinv : 0.0f;
                    cden[p][dir] = act[p] ? den : 0.0f;
                    clam[p][dir] = (act[p] && dir == 0) ? warm : 0.0f;
                    gv += cR[p][dir] * clam[p][dir];
                }
            }
        }
        /* ---- robot points CGR..RB-1 (an env with more than CGR robot points: fp64 oracle under
         * the random policy, Push / PickAndPlace 1.2 % of substeps, Reach 1e-5): the same row
         * setup, kept in LDS for the solve -- (J, M^-1 J^T jinv) per coordinate lane in xd, the
         * row scalars per env -- and solved after the register rows of each half-sweep
         * (extra_rows below).  The sweep runs a compile-time number of extra points, the wave's
         * count rounded up to XSTEP: the rows past an env's own count are zero rows (bounds 0,
         * delta' = 0 exactly), so the points the wave lacks are written as zero rows too. */
        if constexpr (RB > CGR) {
            for (int k = CGR; k < RB && __any(k < n1); k++) n1x = k + 1;
            n1x = __builtin_amdgcn_readfirstlane(n1x);
            nxr = n1x > CGR ? (n1x - CGR + XSTEP - 1) / XSTEP * XSTEP : 0;
            for (int k = CGR; k < CGR + nxr; k++) {   /* wave-uniform */
                if (k >= n1x) {
#pragma unroll
                    for (int dir = 0; dir < 3; dir++) {
                        const int xq = 3 * (P0 + k) + dir - NQR;
                        L.xd[es][xq][c] = make_float2(0.0f, 0.0f);
                        L.xrhs[xq][es] = 0.0f;
                        L.xlam[xq][es] = L.xlam0[xq][es] = 0.0f;
                        L.xfk[xq][es] = 0.0f;
                        L.xjinv[xq][es] = 0.0f;
                    }
                    continue;
                }
                const bool a = k < n1;
                const V3 P = v3(L.g1p[k][0][es], L.g1p[k][1][es], L.g1p[k][2][es]);
                const V3 n = v3(L.g1n[k][0][es], L.g1n[k][1][es], L.g1n[k][2][es]);
                const V3 rb = v3(L.g1rb[k][0][es], L.g1rb[k][1][es], L.g1rb[k][2][es]);
                const int jl = L.g1j[k][es];
                const float id = L.g1id[k][es];
                const bool vs_obj = OBJ && id >= kTableIdLimit;
                const int wk = PERS ? L.g1w[k][es] : -1;
                const float warm = (PERS && wk >= 0) ? m.warmstart * L.mimp[wk < 0 ? 0 : wk][es]
                                                     : warm_lookup<RB>(L, es, CACHE1, id, m.warmstart);
                V3 t1, t2;
                plane_space(n, t1, t2);
                const V3 Jv = (arm && c <= jl) ? cross(zc, P - oc) : v3(0, 0, 0);
                float jinv_n = 0.0f;
#pragma unroll
                for (int dir = 0; dir < 3; dir++) {
                    const V3 u = dir == 0 ? n : (dir == 1 ? t1 : t2);
                    float J = dot(u, Jv);
                    if (OBJ) {
                        const V3 ca = cross(rb, u);
                        const float oj = pick_obj(-1.0f * u, -1.0f * ca);
                        J = (!arm && vs_obj) ? oj : J;
                    }
                    float R = kobj * J;
                    sfor<0, NJ>([&](auto bc) __attribute__((always_inline)) {
                        constexpr int b = decltype(bc)::value;
                        R += mcol[b] * bcast16<b>(J);
                    });
                    const float den = sum16(J * R);
                    const float rel = sum16(J * vu_c);
                    const float jinv = den > 2.220446e-16f ? fast_rcp(den) : 0.0f;
                    float rhs;
                    if (dir == 0) {
                        const float pen = L.g1d[k][es];
                        rhs = (pen > 0.0f ? (-rel - pen * m.inv_dt) : (-pen * erp_dt - rel)) * jinv;
                    } else {
                        rhs = -rel * jinv;
                    }
                    /* as the register rows: inactive -> zero row; scaled units; an unusable row
                     * (jinv = 0) is inert (bounds 0, its warm start already in gv) */
                    const float Ja = a ? J : 0.0f, Ra = a ? R : 0.0f, ja = a ? jinv : 0.0f, da = a ? den : 0.0f;
                    const float lam = (a && dir == 0) ? warm : 0.0f;
                    gv += Ra * lam;
                    if (dir == 0) jinv_n = ja;
                    const bool rok = a && ja != 0.0f;
                    const bool rok_n = a && jinv_n != 0.0f;
                    const int q = 3 * (P0 + k) + dir, xq = q - NQR;
                    L.xd[es][xq][c] = make_float2(c < NC_ ? Ja : 0.0f, Ra * ja);
                    /* every lane of the env writes the same (row-uniform) values */
                    L.xrhs[xq][es] = (a ? rhs : 0.0f) * da;
                    L.xlam[xq][es] = L.xlam0[xq][es] = rok_n && dir == 0 ? lam * da : 0.0f;
                    L.xfk[xq][es] = dir == 0 ? (rok ? 3.0e38f : 0.0f) : (rok ? point_mu<AO, FULL>(m, id) * jinv_n * da : 0.0f);
                    L.xjinv[xq][es] = ja;
                }
            }
        }
    }

    PGX_PROF_MARK(22);
    /* ---- contact-row velocities in lanes.  Lane q = 3 point + dir holds w_q = J_q.dv (register
     * gw; the object tasks' rows 16..23 in a second register gw2, lanes 0..7) and the Delassus
     * entries W[q][s] = J_q M^-1 J_s^T of every row s (Wm: motor / limit rows of dof d,
     * = (M^-1 J_q^T)_d; Wc: contact rows), so a contact row reads its velocity with one
     * broadcast, like a motor row, instead of a 16-lane reduction; every row's impulse also
     * updates gw (one more off-chain fma; {gw, gw2} as one packed pair). */
    constexpr bool WROWS = CONT;
    constexpr int NQ = WROWS ? 3 * NP : 1;      /* 12 (Reach), 24 (object tasks) */
    constexpr bool TWO = NQ > GW;
    constexpr int NC = OBJ ? 13 : NJ;           /* generalized coordinates in lanes */
    bool g1k_any[CGR], g0k_any[CG];
#pragma unroll
    for (int k = 0; k < CGR; k++) g1k_any[k] = CONT && __any(k < n1);
#pragma unroll
    for (int k = 0; k < CG; k++) g0k_any[k] = CONT && OBJ && __any(k < n0);
    /* rows of point p live in the wave (slots fill from 0) */
    auto row_live = [&](int pp) __attribute__((always_inline)) { return pp < P0 ? g0k_any[pp] : g1k_any[pp - P0]; };
    float gw = 0.0f, gw2 = 0.0f, Wm[NJ], Wm2[NJ], Wc[NQ], Wc2[NQ];
#pragma unroll
    for (int d = 0; d < NJ; d++) { Wm[d] = 0.0f; Wm2[d] = 0.0f; }
#pragma unroll
    for (int s2 = 0; s2 < NQ; s2++) { Wc[s2] = 0.0f; Wc2[s2] = 0.0f; }
    if constexpr (WROWS) {
        if (g1k_any[0] || (OBJ && g0k_any[0])) {   /* any contact point in the wave (slots fill from 0) */
            /* transpose through LDS: lane c < NC holds J_q[c], (M^-1 J_q^T)[c] of every row q; lane
             * q reads row q back (and row 16 + q into the second register).  Rows of idle points
             * are zero (their J and R are), so every row is written.  One wave per workgroup: LDS
             * ops of the wave complete in order. */
            ContactLdsGT<OBJ, FULL>& L = *Lp;
            if (c < NC) {
                float* wj = &L.wJ[es][0][0].x;
                float* wr = &L.wR[es][0][0].x;
                sfor<0, NQ>([&](auto qc) __attribute__((always_inline)) {
                    constexpr int q = decltype(qc)::value;
                    wj[16 * q + c] = cJ[q / 3][q % 3];
                    if (c < NJ) wr[8 * q + c] = cR[q / 3][q % 3];
                });
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            auto build = [&](auto reg_c, float* Wmr, float* Wcr, float& gwr) __attribute__((always_inline)) {
                constexpr int R0 = decltype(reg_c)::value * GW;   /* first row of this register */
                const int qr = R0 + c < NQ ? R0 + c : NQ - 1;
                const bool rl = R0 + c < NQ;
                float Jq[NC];
                const float4* jrow = &L.wJ[es][qr][0];
#pragma unroll
                for (int v4 = 0; v4 < (NC + 3) / 4; v4++) {
                    const float4 t = jrow[v4];
                    const float tv[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
                    for (int u = 0; u < 4; u++)
                        if (4 * v4 + u < NC) Jq[4 * v4 + u] = rl ? tv[u] : 0.0f;
                }
                const float4 ra = L.wR[es][qr][0], rb = L.wR[es][qr][1];
                Wmr[0] = rl ? ra.x : 0.0f; Wmr[1] = rl ? ra.y : 0.0f; Wmr[2] = rl ? ra.z : 0.0f;
                Wmr[3] = rl ? ra.w : 0.0f; Wmr[4] = rl ? rb.x : 0.0f; Wmr[5] = rl ? rb.y : 0.0f;
                Wmr[6] = rl ? rb.z : 0.0f;
                /* W[q][s] = J_q . (M^-1 J_s^T): lane q against the row broadcasts of column s
                 * (object-scene rows have object coordinates only) */
                sfor<0, NQ>([&](auto sc) __attribute__((always_inline)) {
                    constexpr int s2 = decltype(sc)::value;
                    constexpr int C0 = (s2 / 3 < P0) ? NJ : 0;
                    if (row_live(s2 / 3)) {
                        float w = Jq[C0] * bcast16<C0>(cR[s2 / 3][s2 % 3]);
                        sfor<C0 + 1, NC>([&](auto lc) __attribute__((always_inline)) {
                            constexpr int l = decltype(lc)::value;
                            w = fmaf(Jq[l], bcast16<l>(cR[s2 / 3][s2 % 3]), w);
                        });
                        Wcr[s2] = w;
                    }
                });
                float w = Jq[0] * bcast16<0>(gv);
                sfor<1, NC>([&](auto lc) __attribute__((always_inline)) {
                    constexpr int l = decltype(lc)::value;
                    w = fmaf(Jq[l], bcast16<l>(gv), w);
                });
                gwr = w;
            };
            build(IC<0>{}, Wm, Wc, gw);
            /* rows 16..23 belong to robot points 1..3 (slots fill from 0): idle in every env of
             * the wave while point 1 is, and an idle row reads 0 (bounds [0, 0]) */
            if constexpr (TWO) { if (g1k_any[1]) build(IC<1>{}, Wm2, Wc2, gw2); }
        }
    }
    /* the extra rows' scalars into lanes (row x: lane x % 16 of register x / 16) */
    constexpr int XB = (RB > CGR) ? (3 * (RB - CGR) + GW - 1) / GW : 1;
    float xs_rhs[XB], xs_lam[XB], xs_fk[XB], xs_jinv[XB];
    auto load_xs = [&](bool start) __attribute__((always_inline)) {
        if constexpr (RB > CGR) {
            ContactLdsGT<OBJ, FULL>& L = *Lp;
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
#pragma unroll
            for (int b = 0; b < XB; b++) {
                const int xq = GW * b + c;
                const bool ok = xq < 3 * nxr;
                const int xr = ok ? xq : 0;
                xs_lam[b] = ok ? L.xlam0[xr][es] : 0.0f;
                if (start) {
                    xs_rhs[b] = ok ? L.xrhs[xr][es] : 0.0f;
                    xs_fk[b] = ok ? L.xfk[xr][es] : 0.0f;
                    xs_jinv[b] = ok ? L.xjinv[xr][es] : 0.0f;
                }
            }
        }
    };
#pragma unroll
    for (int b = 0; b < XB; b++) { xs_rhs[b] = 0.0f; xs_lam[b] = 0.0f; xs_fk[b] = 0.0f; xs_jinv[b] = 0.0f; }
    if (RB > CGR && nxr > 0) load_xs(true);
    PGX_PROF_MARK(23);

    /* ---- motor / limit rows (as substep()): per row rhs and lambda, per dof jinv / den */
    float den[NJ], jinv[NJ];
#pragma unroll
    for (int d = 0; d < NJ; d++) {
        den[d] = D.mdiag[d];
        jinv[d] = den[d] > 2.220446e-16f ? fast_rcp(den[d]) : 0.0f;
    }
    float rhs[PGX_N_ROWS];
#pragma unroll
    for (int r = 0; r < PGX_N_ROWS; r++) {
        const int kind = kPgxRowCode[r] >> 4, d = kPgxRowCode[r] & 15;
        rhs[r] = 0.0f;
        if (kind == 0) {
            const float pos_term = (tq[d] - q[d]) * m.inv_dt;
            const float desired = m.kp * pos_term + vu[d] + m.kd * (0.0f - vu[d]);
            rhs[r] = desired - vu[d];   /* scaled units: rhs * den */
        }
    }
    auto init_limit_rows = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int r = 0; r < PGX_N_ROWS; r++) {
            const int kind = kPgxRowCode[r] >> 4, d = kPgxRowCode[r] & 15;
            if (kind == 0) continue;
            const float rel = kind == 2 ? -vu[d] : vu[d];
            const float pen = kind == 1 ? (q[d] - kLower[d]) : (kUpper[d] - q[d]);
            float verr = -rel, perr = 0.0f;
            if (pen > 0.0f) verr -= pen * m.inv_dt;
            else perr = -pen * m.erp * m.inv_dt;
            rhs[r] = perr + verr;   /* scaled units */
        }
    };
    /* exact limit-row skip (see substep()); lane c < 7 tests dof c (its M^-1 row is mcol, the
     * same terms in the same order as the redundant loop), the row's ballot ANDs them */
    bool ok_c = true;
    bool far_nc = true;
    if (arm) {
        float B = 0.0f;
#pragma unroll
        for (int k = 0; k < NJ; k++) B += fabsf(mcol[k]) * m.max_impulse[k];
        B = B * 1.001f + 1e-6f;
        float lo_a[NJ], up_a[NJ];
#pragma unroll
        for (int d = 0; d < NJ; d++) { lo_a[d] = kLower[d]; up_a[d] = kUpper[d]; }
        const float qc = pick_arm(q, 0.0f);
        const float penl = qc - pick_arm(lo_a, 0.0f), penu = pick_arm(up_a, 0.0f) - qc;
        ok_c = penl > 0.0f && penu > 0.0f && (vu_c - B) > -penl * m.inv_dt && (vu_c + B) < penu * m.inv_dt;
    }
    far_nc = !row_any(!ok_c);   /* the motor-impulse bound alone keeps every limit row idle */
    const bool far = far_nc && n1 == 0;
    /* Rows in scaled units: each row equation multiplied by its den (= J M^-1 J^T), so
     * lambda' = lambda den, rhs' = rhs den and the unclamped update is
     *   lambda' + delta' = (lambda' + rhs') - s v_d        (jinv den = 1)
     * with v_d the row's velocity: one DPP-sourced v_sub/v_add of the broadcast delta-v off
     * a sum formed off the chain; delta' = delta den is the residual Bullet tracks, and the
     * coordinate updates take the columns pre-multiplied by jinv.  Chain per row:
     * v_sub_dpp -> med3 -> fmac (the next broadcast's source). */
    float mcs[NJ], wms[NJ], wms2[NJ];
    /* PKM / PKC (WROWS): a joint (contact) row's coordinate and Delassus coefficients as one pair,
     * {mcs, wms} ({cR, Wc}), so that the row's gv / gw updates are one pk_fma_acc.  Per kernel:
     * the pairs' aligned registers raise the register peak, which costs more than the issue
     * saved except in the ReachAO kernels (PGX_PK / PGX_PK_AO, above) */
    constexpr int PK = AO ? PGX_PK_AO : PGX_PK;
    constexpr bool PKM = WROWS && (PK & 1) != 0, PKC = WROWS && (PK & 2) != 0;
    /* PKD (bit 2; the object tasks' full-manifold kernels, two Delassus registers, neither PKM nor
     * PKC): the pair is {gw, gw2} instead, coefficients {wms, wms2} / {Wc, Wc2} */
    constexpr bool PKD = TWO && FULL && !PKM && !PKC && (PK & 4) != 0;
    f2 mw[NJ], crw[NQ], mw2[NJ], cw2[NQ];
    /* motor rows: the shifted bound pair (lo' - lambda', hi' - lambda') tracked instead of
     * lambda', one v_pk_add_f32 per row update (lambda' itself is not needed after the solve:
     * joint rows are not warm-started); limit rows keep lambda' (fewer live registers) */
    f2 bnd[NJ];
    float lam[PGX_N_ROWS], lhi[NJ];
#pragma unroll
    for (int d = 0; d < NJ; d++) {
        mcs[d] = mcol[d] * jinv[d];
        wms[d] = Wm[d] * jinv[d];
        wms2[d] = Wm2[d] * jinv[d];
        lhi[d] = m.limit_max_imp * den[d];
    }
    auto init_bounds = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int r = 0; r < PGX_N_ROWS; r++) {
            const int kind = kPgxRowCode[r] >> 4, d = kPgxRowCode[r] & 15;
            lam[r] = 0.0f;
            if (kind == 0) bnd[d] = (f2){-m.max_impulse[d] * den[d], m.max_impulse[d] * den[d]};
            else if (LDS_LIM) __hip_atomic_store(&Lp->llam[r - NJ][es], 0.0f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        }
    };
    init_bounds();
    /* G2 (g2_c): the second Delassus register holds live rows in this solve (rows 16.. exist:
     * robot points past the first in the object tasks); without them its updates are skipped */
    auto mrow = [&](auto rc, auto g2_c, float& resid) __attribute__((always_inline)) {
        constexpr int r = decltype(rc)::value;
        constexpr int kind = kPgxRowCode[r] >> 4, d = kPgxRowCode[r] & 15;
        /* delta' = clamp(rhs' - s v_d, lo' - lambda', hi' - lambda'): the shifted bounds are
         * formed off the chain, so the clamp yields the impulse increment directly */
        const float x = kind == 2 ? rhs[r] + bcast16<d>(gv) : rhs[r] - bcast16<d>(gv);
        float delta;
        if constexpr (kind == 0) {
            delta = __builtin_amdgcn_fmed3f(x, bnd[d].x, bnd[d].y);
            bnd[d] -= (f2){delta, delta};
        } else if constexpr (LDS_LIM) {
            /* the object tasks' limit rows (the all-rows solve only) in LDS: relaxed atomics so
             * they are neither hoisted out of the sweep loop nor promoted back to registers */
            float* lr = &Lp->lrhs[r - NJ][es];
            float* ll = &Lp->llam[r - NJ][es];
            const float rr = __hip_atomic_load(lr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
            const float lm = __hip_atomic_load(ll, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
            const float xl = kind == 2 ? rr + bcast16<d>(gv) : rr - bcast16<d>(gv);
            delta = __builtin_amdgcn_fmed3f(xl, -lm, lhi[d] - lm);
            __hip_atomic_store(ll, lm + delta, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        } else {
            delta = __builtin_amdgcn_fmed3f(x, -lam[r], lhi[d] - lam[r]);
            lam[r] += delta;
        }
        const float sd = kind == 2 ? -delta : delta;
        if constexpr (PKD) {
            gv += mcs[d] * sd;
            if constexpr (decltype(g2_c)::value) pk_fma_acc(gw, gw2, mw2[d], sd);
            else gw += mw2[d].x * sd;
        } else {
            if constexpr (PKM) {
                pk_fma_acc(gv, gw, mw[d], sd);
            } else {
                gv += mcs[d] * sd;
                if constexpr (WROWS) gw += wms[d] * sd;
            }
            if constexpr (TWO && decltype(g2_c)::value) gw2 += wms2[d] * sd;
        }
        resid = fmaxf(resid, fabsf(delta));
    };
    /* contact rows in scaled units too: lambda' = lambda den, friction bounds
     * +-mu lambda_n den_f = +-lambda'_n (mu jinv_n den_f); an idle row (inactive point, no
     * usable den, or a friction row while the normal impulse is 0) gets the bounds
     * [lambda', lambda']: delta' = 0 without a select on the chain */
    constexpr int NPP = NP > 0 ? NP : 1;
    float fk[NPP][3];
    bool rok[NPP][3];   /* row usable: den above SIMD_EPSILON (else jinv = 0 and the row is inert) */
#pragma unroll
    for (int p = 0; p < NP; p++)
#pragma unroll
        for (int dir = 0; dir < 3; dir++) {
            rok[p][dir] = act[p] && cjinv[p][dir] != 0.0f;
            fk[p][dir] = rok[p][dir] ? pmu[p] * cjinv[p][0] * cden[p][dir] : 0.0f;   /* unusable row: bounds 0 */
            crhs[p][dir] *= cden[p][dir];
            clam[p][dir] *= cden[p][dir];
            cR[p][dir] *= cjinv[p][dir];
        }
    if constexpr (WROWS) {
#pragma unroll
        for (int q = 0; q < NQ; q++) {
            Wc[q] *= cjinv[q / 3][q % 3];
            if (TWO) Wc2[q] *= cjinv[q / 3][q % 3];
        }
        /* from here lane q of gw (gw2) holds x_q = rhs'_q - w_q, what its row clamps: a contact row
         * reads it with one broadcast and every impulse updates it with the negated coupling, so
         * the rows' rhs' leave the registers (24 per lane in the object tasks) */
        float r0 = 0.0f, r1 = 0.0f;
        sfor<0, NQ>([&](auto qc) __attribute__((always_inline)) {
            constexpr int q = decltype(qc)::value;
            if constexpr (q < GW) r0 = lane_sel<q>(crhs[q / 3][q % 3], r0);
            else r1 = lane_sel<q - GW>(crhs[q / 3][q % 3], r1);
        });
        gw = r0 - gw;
        if (TWO) gw2 = r1 - gw2;
        /* object tasks: an unusable normal row (inactive point, den <= SIMD_EPSILON: lambda' = 0)
         * holds x = -3e38 in its lane, so med3(x, -0, +3e38) = 0 with the one upper bound of every
         * normal row -- 8 bound registers fewer at the register peak (PickAndPlace 16384 -4 %,
         * Reach +0.8 %: there the per-point bound stays); other rows' impulses move that x by
         * finite amounts only */
        if constexpr (OBJ) {
            sfor<0, NQ / 3>([&](auto pc) __attribute__((always_inline)) {
                constexpr int p = decltype(pc)::value, q = 3 * p;
                const bool usable = act[p] && cjinv[p][0] != 0.0f;
                if constexpr (q < GW) gw = usable ? gw : lane_sel<q>(-3.0e38f, gw);
                else gw2 = usable ? gw2 : lane_sel<q - GW>(-3.0e38f, gw2);
            });
        }
#pragma unroll
        for (int q = 0; q < NQ; q++) { Wc[q] = -Wc[q]; Wc2[q] = -Wc2[q]; }
#pragma unroll
        for (int d = 0; d < NJ; d++) { wms[d] = -wms[d]; wms2[d] = -wms2[d]; }
        if constexpr (PKM) {
#pragma unroll
            for (int d = 0; d < NJ; d++) mw[d] = (f2){mcs[d], wms[d]};
        }
        if constexpr (PKC) {
#pragma unroll
            for (int q = 0; q < NQ; q++) crw[q] = (f2){cR[q / 3][q % 3], Wc[q]};
        }
        if constexpr (PKD) {
#pragma unroll
            for (int d = 0; d < NJ; d++) mw2[d] = (f2){wms[d], wms2[d]};
#pragma unroll
            for (int q = 0; q < NQ; q++) cw2[q] = (f2){Wc[q], Wc2[q]};
        }
    }
    /* shifted bounds as for the joint rows: delta' = clamp(rhs' - w, lo' - lambda', hi' - lambda').
     * A normal row's upper bound is +inf (0 with lambda' = 0 for an unusable row; in the object
     * tasks such a row is inert through its x, above); a friction row is idle (bounds 0) while
     * its normal impulse is 0. */
    float chi[NPP];
    if constexpr (CONT) {   /* the normal rows' jinv for the cache: in LDS through the sweeps */
#pragma unroll
        for (int p = 0; p < NP; p++) Lp->pjn[p][es] = cjinv[p][0];
    }
#pragma unroll
    for (int p = 0; p < NP; p++) {
        chi[p] = rok[p][0] ? 3.0e38f : 0.0f;
        if (WROWS && !rok[p][0]) clam[p][0] = 0.0f;   /* already applied to gv; the cache stores lambda' jinv = 0 */
    }
    auto crow = [&](auto pc, auto dc, const bool fr, auto g2_c, float& resid) __attribute__((always_inline)) {
        constexpr int p = decltype(pc)::value, dir = decltype(dc)::value, q = 3 * p + dir;
        const float ln_n = clam[p][0], lm = clam[p][dir];
        float lo, hi;
        if (fr) {   /* idle while the normal impulse is 0: the bound pair times 0 (an unusable
                     * row has fk = 0 and lambda' = 0, so its bounds are 0 as well) */
            const float mk = ln_n > 0.0f ? 1.0f : 0.0f;
            const float fkv = fk[p][dir];
            const f2 b = ((f2){-fkv, fkv} * ln_n - lm) * mk;
            lo = b.x;
            hi = b.y;
        } else {
            lo = -lm;
            hi = OBJ ? 3.0e38f : chi[p];
        }
        const float x = q < GW ? bcast16<q % GW>(gw) : bcast16<q % GW>(gw2);   /* rhs' - w */
        const float delta = __builtin_amdgcn_fmed3f(x, lo, hi);
        clam[p][dir] = lm + delta;
        if constexpr (PKD) {
            gv += cR[p][dir] * delta;
            if constexpr (decltype(g2_c)::value) pk_fma_acc(gw, gw2, cw2[q], delta);
            else gw += cw2[q].x * delta;
        } else {
            if constexpr (PKC) {
                pk_fma_acc(gv, gw, crw[q], delta);
            } else {
                gv += cR[p][dir] * delta;
                gw += Wc[q] * delta;
            }
            if constexpr (TWO && decltype(g2_c)::value) gw2 += Wc2[q] * delta;
        }
        resid = fmaxf(resid, fabsf(delta));
    };
    /* the wave's largest robot-point count, a scalar: the per-point branches in the sweep
     * are s_cmp on it (a per-point bool there turns into a VALU mask round trip per row) */
    int n1w = 0;
#pragma unroll
    for (int k = 0; k < CGR; k++) n1w = g1k_any[k] ? k + 1 : n1w;
    n1w = __builtin_amdgcn_readfirstlane(n1w);
    const bool g0_any = CONT && OBJ && __any(n0 > 0);
    const bool g1_any = CONT && __any(n1 > 0);
    /* NW: the robot points the sweep runs, a compile-time count chosen per wave outside the
     * sweep loop (0, 2 or 4, n1w rounded up): the rows of points n1w..NW-1 are idle (bounds
     * [lambda', lambda'] with lambda' = 0 -> delta' = 0, bit for bit), so no per-point branch
     * sits inside the sweep.  The object-scene rows (P0 points, a resting cube has 4) run in
     * every sweep of the object tasks, idle points predicated the same way. */
    /* the extra rows (robot points CGR..CGR+NX-1) of one half-sweep, after the register rows in the
     * same order as the oracle's (normal rows, then friction rows; points by id): the row
     * velocity by a 16-lane reduction (no Delassus lane), (J, M^-1 J^T jinv) per coordinate lane
     * from LDS (one ds_read_b64, independent of the chain: straight-line code, no branch, so the
     * reads issue ahead), the row scalars in lanes of registers (row x: lane x % 16 of
     * xs_*[x / 16]), read by broadcast.  The register rows' Delassus lanes are not updated per
     * extra row: after the block, every register row's x' = rhs' - J_q.dv drops by J_q . (the
     * block's change of dv) -- one 13-term dot product per lane and Delassus register, with J_q
     * from the transpose rows (wJ) -- instead of an LDS coupling and an fma per extra row. */
    int rcol = c;   /* the coordinate of lane c's R entry (MODE 3 slot lanes: their dof's) */
    auto extra_rows = [&](auto fr_c, auto nx_c, auto g2_c, float& resid) __attribute__((always_inline)) {
        constexpr int FR = decltype(fr_c)::value, NX = decltype(nx_c)::value;
        if constexpr (WROWS && RB > CGR && NX > 0) {
            ContactLdsGT<OBJ, FULL>& L = *Lp;
            const float gvb = gv;
            sfor<0, NX>([&](auto kc) __attribute__((always_inline)) {
                constexpr int kx = decltype(kc)::value;
                sfor<FR ? 1 : 0, FR ? 3 : 1>([&](auto dc) __attribute__((always_inline)) {
                    constexpr int dir = decltype(dc)::value, xq = 3 * kx + dir;
                    constexpr int b = xq / GW, l = xq % GW, bn = (3 * kx) / GW, ln_ = (3 * kx) % GW;
                    const float J = L.xd[es][xq][c].x;
                    const float Rs = L.xd[es][xq][rcol].y;
                    const float w = sum16(J * gv);
                    const float lm = bcast16<l>(xs_lam[b]), fkv = bcast16<l>(xs_fk[b]);
                    float lo, hi;
                    if constexpr (dir != 0) {
                        const float ln_n = bcast16<ln_>(xs_lam[bn]);
                        const float mk = ln_n > 0.0f ? 1.0f : 0.0f;
                        const f2 bb = ((f2){-fkv, fkv} * ln_n - lm) * mk;
                        lo = bb.x;
                        hi = bb.y;
                    } else {
                        lo = -lm;
                        hi = fkv;
                    }
                    const float delta = __builtin_amdgcn_fmed3f(bcast16<l>(xs_rhs[b]) - w, lo, hi);
                    xs_lam[b] = lane_sel<l>(lm + delta, xs_lam[b]);
                    gv += Rs * delta;
                    resid = fmaxf(resid, fabsf(delta));
                });
            });
            /* the register rows' velocities: x'_q -= J_q . (gv - gvb) */
            const float dgv = gv - gvb;
            auto correct = [&](auto reg_c, float& gwr) __attribute__((always_inline)) {
                constexpr int R0 = decltype(reg_c)::value * GW;
                const int qr = R0 + c < NQR ? R0 + c : NQR - 1;
                const float4* jrow = &L.wJ[es][qr][0];
                float Jq[NC];
#pragma unroll
                for (int v4 = 0; v4 < (NC + 3) / 4; v4++) {
                    const float4 t = jrow[v4];
                    const float tv[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
                    for (int u = 0; u < 4; u++)
                        if (4 * v4 + u < NC) Jq[4 * v4 + u] = tv[u];
                }
                float d = Jq[0] * bcast16<0>(dgv);
                sfor<1, NC>([&](auto lc) __attribute__((always_inline)) {
                    constexpr int l2 = decltype(lc)::value;
                    d = fmaf(Jq[l2], bcast16<l2>(dgv), d);
                });
                gwr -= R0 + c < NQR ? d : 0.0f;
            };
            correct(IC<0>{}, gw);
            if constexpr (TWO && decltype(g2_c)::value) correct(IC<1>{}, gw2);
        }
    };
    auto contact_rows = [&](auto nw_c, auto nx_c, auto g2_c, float& resid) __attribute__((always_inline)) {
        constexpr int NW = decltype(nw_c)::value;
#pragma unroll
        for (int fr = 0; fr < 2; fr++) {
            if (OBJ && g0_any) {
                sfor<0, P0>([&](auto kc) __attribute__((always_inline)) {
                    if (fr) { crow(kc, IC<1>{}, true, g2_c, resid); crow(kc, IC<2>{}, true, g2_c, resid); }
                    else crow(kc, IC<0>{}, false, g2_c, resid);
                });
            }
            if (NW < 0 && !g1_any) continue;
            sfor<0, (CONT ? (NW >= 0 ? NW : CGR) : 0)>([&](auto kc) __attribute__((always_inline)) {
                constexpr int k = decltype(kc)::value;
                if (NW >= 0 || k < n1w) {
                    if (fr) {
                        crow(IC<P0 + k>{}, IC<1>{}, true, g2_c, resid);
                        crow(IC<P0 + k>{}, IC<2>{}, true, g2_c, resid);
                    } else {
                        crow(IC<P0 + k>{}, IC<0>{}, false, g2_c, resid);
                    }
                }
            });
            if (fr) extra_rows(IC<1>{}, nx_c, g2_c, resid);
            else extra_rows(IC<0>{}, nx_c, g2_c, resid);
        }
    };
    const bool any_contact = CONT && __any(n0 > 0 || n1 > 0);
    const int n_it = m.num_iterations;
    /* the exit threshold in an SGPR before the sweeps: read from the model inside the loop it
     * costs a scalar load and its s_waitcnt on every sweep */
    float res_thr = m.residual_abs;
    asm("" : "+s"(res_thr));
    PGX_PROF_MARK(3);
    PGX_PROF_COUNT(9, 1);
    PGX_PROF_SWEEPS_DECL;
    /* Three solves, chosen per wave.  far: the motor-impulse bound proves every limit row
     * idle and there are no robot contacts -> motor (+ object contact) rows only.  Else, if
     * the motor-impulse bound alone holds (only robot-contact impulses, unbounded, stand in
     * the way), the sweeps run speculatively without the limit rows and every lane checks,
     * at each position the limit block would take in the order, that its dof's two limit
     * rows would compute x' <= 0 there (delta' = 0: the block would be a no-op, bit for
     * bit); a wave in which any env fails that check (0.05 % of contact substeps, fp64
     * oracle under the random policy) is solved again from the same start with the limit
     * rows.  Otherwise all 21 joint rows run. */
    float rl_c = -1.0f, ru_c = -1.0f;
    /* the smallest margin seen, min(gv - rl, -(ru + gv)): a row would compute x' > 0 (a
     * violation) exactly when its margin is negative; one v_min3 per check, no compare */
    float lmargin = 3.0e38f;
    auto limit_check = [&]() __attribute__((always_inline)) {
        lmargin = fminf(lmargin, fminf(gv - rl_c, -(ru_c + gv)));
    };
    /* MODE 3 (partial, arm tasks): the limit pairs of the dofs the motor-impulse bound cannot
     * clear in some env of the wave (dmask, at most 2 of them) run, the others are checked as in
     * MODE 1 -- at the block's start and after every pair that runs, i.e. once per stretch of
     * constant velocity, which covers each skipped pair's own position.  The running pairs sit
     * in slots: lane SL0 + S (the first idle lane past the coordinates) mirrors dof d_S -- it gets
     * lane d_S's coefficients, so its velocity delta evolves bit for bit as lane d_S's -- and a
     * slot row reads it with a compile-time broadcast, so the sweep has no runtime branch (a
     * branch per pair measured slower than all 21 rows).  Same arithmetic as mrow: the result is
     * bitwise the all-rows solve's. */
    constexpr int KMAX = CONT ? 1 : 2;   /* two slots measured -1.2 % without the table, +1 % with it */
    constexpr int SL0 = OBJ ? 13 : NJ;   /* first slot lane: the first lane past the coordinates */
    unsigned dmask = 0u;
    float smcs[KMAX], swms[KMAX], swms2[KMAX], srh[KMAX][2], slhi[KMAX], slam[KMAX][2];
    f2 smw[KMAX];   /* PKM: {smcs, swms} */
    auto srow = [&](auto sc, auto kc, auto g2_c, float& resid) __attribute__((always_inline)) {
        constexpr int S = decltype(sc)::value, KIND = decltype(kc)::value;   /* 1 lower, 2 upper */
        const float x = KIND == 2 ? srh[S][1] + bcast16<SL0 + S>(gv) : srh[S][0] - bcast16<SL0 + S>(gv);
        const float delta = __builtin_amdgcn_fmed3f(x, -slam[S][KIND - 1], slhi[S] - slam[S][KIND - 1]);
        slam[S][KIND - 1] += delta;
        const float sd = KIND == 2 ? -delta : delta;
        if constexpr (PKM) {
            pk_fma_acc(gv, gw, smw[S], sd);
        } else {
            gv += smcs[S] * sd;
            if constexpr (WROWS) gw += swms[S] * sd;
        }
        if constexpr (TWO && decltype(g2_c)::value) gw2 += swms2[S] * sd;
        resid = fmaxf(resid, fabsf(delta));
    };
    static_assert(limit_rows_paired(), "limit rows come as (lower, upper) pairs of one dof after the motor rows");
    auto solve = [&](auto mode_c, auto nw_c, auto k_c, auto nx_c) __attribute__((always_inline)) {
        constexpr int MODE = decltype(mode_c)::value;   /* 0 far, 1 speculative, 2 all rows, 3 partial */
        constexpr int NW = decltype(nw_c)::value;
        constexpr int K = decltype(k_c)::value;         /* MODE 3: slots in use */
        /* NX: extra robot points (past CGR) the sweep runs, 0 or a multiple of XSTEP */
        constexpr bool G2 = TWO && (NW < 0 || 3 * (P0 + NW) > GW);
        const IC<G2 ? 1 : 0> g2_c{};
        for (int it = 0; it < n_it; it += 2) {
            float resid = 0.0f;
            if constexpr (MODE == 1 || MODE == 3) limit_check();
            if constexpr (MODE == 3) {   /* the limit block leads the reversed sweep */
                sfor<0, K>([&](auto i) __attribute__((always_inline)) {
                    constexpr int S = K - 1 - decltype(i)::value;
                    srow(IC<S>{}, IC<2>{}, g2_c, resid);
                    srow(IC<S>{}, IC<1>{}, g2_c, resid);
                    limit_check();
                });
            }
            sfor<0, PGX_N_ROWS>([&](auto i) __attribute__((always_inline)) {
                constexpr int r = PGX_N_ROWS - 1 - decltype(i)::value;
                if constexpr (MODE == 2 || (kPgxRowCode[r] >> 4) == 0) mrow(IC<r>{}, g2_c, resid);
            });
            if (CONT && (OBJ || NW > 0 || (NW < 0 && any_contact))) contact_rows(nw_c, nx_c, g2_c, resid);
            PGX_PROF_SWEEP();
            if (resid <= res_thr || it + 1 >= n_it) break;
            resid = 0.0f;
            sfor<0, PGX_N_ROWS>([&](auto i) __attribute__((always_inline)) {
                constexpr int r = decltype(i)::value;
                if constexpr (MODE == 2 || (kPgxRowCode[r] >> 4) == 0) mrow(IC<r>{}, g2_c, resid);
            });
            if constexpr (MODE == 1 || MODE == 3) limit_check();
            if constexpr (MODE == 3) {
                sfor<0, K>([&](auto sc) __attribute__((always_inline)) {
                    srow(sc, IC<1>{}, g2_c, resid);
                    srow(sc, IC<2>{}, g2_c, resid);
                    limit_check();
                });
            }
            if (CONT && (OBJ || NW > 0 || (NW < 0 && any_contact))) contact_rows(nw_c, nx_c, g2_c, resid);
            PGX_PROF_SWEEP();
            if (resid <= res_thr) break;
        }
    };
    /* the robot point count fixed at compile time (above) for every mode but far; the extra
     * points (past CGR) only in the speculative and all-rows solves (the partial one hands a wave
     * with extra points to the all-rows solve) */
    auto solve_w = [&](auto mode_c, auto k_c) __attribute__((always_inline)) {
        constexpr int MODE = decltype(mode_c)::value;
        if constexpr (WROWS) {
            /* (n1w counts register points only: a wave with extra points has n1w = CGR, which is 2
             * for the arm tasks, so the extra-point copies are chosen by nxr first) */
            if (n1w == 0) solve(mode_c, IC<0>{}, k_c, IC<0>{});
            else if (nxr == 0 && n1w <= 2) solve(mode_c, IC<2>{}, k_c, IC<0>{});
            else if (CGR > 4 && nxr == 0 && n1w <= 4) solve(mode_c, IC<(CGR > 4 ? 4 : CGR)>{}, k_c, IC<0>{});
            else if constexpr (RB > CGR && MODE != 3) {
                if (nxr == 0) {
                    solve(mode_c, IC<CGR>{}, k_c, IC<0>{});
                } else {   /* one sweep copy per multiple of XSTEP (the wave's count rounded up) */
                    sfor<1, (RB - CGR) / XSTEP + 1>([&](auto ic) __attribute__((always_inline)) {
                        constexpr int NXC = decltype(ic)::value * XSTEP;
                        if (nxr == NXC) solve(mode_c, IC<CGR>{}, k_c, IC<NXC>{});
                    });
                }
            } else {
                solve(mode_c, IC<CGR>{}, k_c, IC<0>{});
            }
        } else {
            solve(mode_c, IC<-1>{}, k_c, IC<0>{});
        }
    };
    /* PARK_SOLVE: the state read only after the solve waits in LDS through the sweeps (relaxed
     * atomics: neither kept in registers nor hoisted) -- 27 registers fewer at the sweeps' peak,
     * where the two-waves-per-SIMD object kernel spills to scratch */
#ifndef PGX_NO_PARK_SOLVE
    constexpr bool PARK_SOLVE = CONT && (OBJ || AO || PART == 2);
#else
    constexpr bool PARK_SOLVE = false;
#endif
    auto park = [&](int k, float v) __attribute__((always_inline)) {
        __hip_atomic_store(&Lp->psv[k][es], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    };
    auto unpark = [&](int k) __attribute__((always_inline)) {
        return __hip_atomic_load(&Lp->psv[k][es], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    };
    if constexpr (PARK_SOLVE) {
#pragma unroll
        for (int j = 0; j < NJ; j++) { park(j, q[j]); park(NJ + j, vu[j]); }
        if constexpr (OBJ) {
            park(14, ob.p.x); park(15, ob.p.y); park(16, ob.p.z);
            park(17, ob.qx); park(18, ob.qy); park(19, ob.qz); park(20, ob.qw);
            park(21, vcu.x); park(22, vcu.y); park(23, vcu.z);
            park(24, wcu.x); park(25, wcu.y); park(26, wcu.z);
        }
    }
    if (__all(far)) {   /* (far implies no robot point in the wave) */
        solve(IC<0>{}, IC<0>{}, IC<0>{}, IC<0>{});
    } else {
        PGX_PROF_COUNT(10, 1);
        init_limit_rows();
        if constexpr (LDS_LIM) {   /* the limit rows' rhs' for an all-rows solve: in LDS */
#pragma unroll
            for (int r = NJ; r < PGX_N_ROWS; r++)
                __hip_atomic_store(&Lp->lrhs[r - NJ][es], rhs[r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        }
        if (e.pgs_mode != 2) {
            float rl[NJ], ru[NJ];
#pragma unroll
            for (int r = NJ; r < PGX_N_ROWS; r++) {
                const int kind = kPgxRowCode[r] >> 4, d = kPgxRowCode[r] & 15;
                if (kind == 1) rl[d] = rhs[r];
                else ru[d] = rhs[r];
            }
            rl_c = pick_arm(rl, -3.0e38f);   /* other lanes never flag (object coordinates) */
            ru_c = pick_arm(ru, -3.0e38f);
            const bool spec_all = __all(far_nc);
            int nk = 0;
            if (!spec_all) {   /* partial: the dofs the motor bound cannot clear, in any env */
                const uint64_t bm = __ballot(arm && !ok_c);
                dmask = __builtin_amdgcn_readfirstlane((unsigned)((bm | (bm >> 16) | (bm >> 32) | (bm >> 48)) & 0x7Fu));
                nk = __builtin_popcount(dmask);
            }
            const float gv0 = gv, gw0 = gw, gw20 = gw2;
            if constexpr (CONT) {   /* the start lambda'_n for a redo: in LDS through the sweeps */
#pragma unroll
                for (int p = 0; p < NP; p++) Lp->pl0[p][es] = clam[p][0];
            }
            if (PART && !NO_PART && !spec_all && nk <= KMAX && nxr == 0) {   /* (NO_PART: all rows instead, fewer registers) */
                PGX_PROF_COUNT(7, 1);
                /* slots in the pairs' table order; slot lane SL0 + S mirrors dof d_S */
                int ds[2] = {0, 0};
                int k = 0;
                sfor<0, (PGX_N_ROWS - NJ) / 2>([&](auto pc) __attribute__((always_inline)) {
                    constexpr int d = kPgxRowCode[NJ + 2 * decltype(pc)::value] & 15;
                    if ((dmask >> d) & 1u) { if (k == 0) ds[0] = d; else ds[1] = d; k++; }
                });
                ds[0] = __builtin_amdgcn_readfirstlane(ds[0]);
                ds[1] = __builtin_amdgcn_readfirstlane(ds[1]);
                const int src = (int)(threadIdx.x & ~(unsigned)(GW - 1));
                auto mirror = [&](float& x) __attribute__((always_inline)) {
                    x = lane_sel<SL0>(__shfl(x, src + ds[0]), x);
                    if (KMAX > 1 && nk > 1) x = lane_sel<SL0 + 1>(__shfl(x, src + ds[1]), x);
                };
#pragma unroll
                for (int d = 0; d < NJ; d++) {
                    if constexpr (PKM) {   /* (mcs / cR live on only as the pairs' halves) */
                        float t = mw[d].x;
                        mirror(t);
                        mw[d].x = t;
                    } else {
                        mirror(mcs[d]);
                    }
                }
                mirror(gv);
                if (g1_any) {
#pragma unroll
                    for (int p = 0; p < NP; p++)
#pragma unroll
                        for (int dir = 0; dir < 3; dir++) {
                            if constexpr (PKC) {
                                float t = crw[3 * p + dir].x;
                                mirror(t);
                                crw[3 * p + dir].x = t;
                            } else {
                                mirror(cR[p][dir]);
                            }
                        }
                }
                /* the slots' row data: dof d_S's entries, selected with uniform masks */
#pragma unroll
                for (int S = 0; S < KMAX; S++) {
                    if constexpr (PKM) smw[S] = mw[0];
                    else { smcs[S] = mcs[0]; swms[S] = PKD ? mw2[0].x : wms[0]; }
                    swms2[S] = PKD ? mw2[0].y : wms2[0]; slhi[S] = lhi[0];
                    srh[S][0] = rl[0]; srh[S][1] = ru[0];
                    slam[S][0] = 0.0f; slam[S][1] = 0.0f;
                    sfor<1, NJ>([&](auto dc) __attribute__((always_inline)) {
                        constexpr int d = decltype(dc)::value;
                        const bool hit = ds[S] == d;   /* wave-uniform */
                        auto sel = [&](float a, float o) __attribute__((always_inline)) { return hit ? a : o; };
                        if constexpr (PKM) smw[S] = hit ? mw[d] : smw[S];
                        else { smcs[S] = sel(mcs[d], smcs[S]); swms[S] = sel(PKD ? mw2[d].x : wms[d], swms[S]); }
                        swms2[S] = sel(PKD ? mw2[d].y : wms2[d], swms2[S]);
                        slhi[S] = sel(lhi[d], slhi[S]);
                        srh[S][0] = sel(rl[d], srh[S][0]); srh[S][1] = sel(ru[d], srh[S][1]);
                    });
                }
                /* the checks skip the running dofs and the slot lanes */
                if ((dmask >> c) & 1u) { rl_c = -3.0e38f; ru_c = -3.0e38f; }
                if (c == SL0) rcol = ds[0];
                if (KMAX > 1 && nk > 1 && c == SL0 + 1) rcol = ds[1];
                PGX_PROF_COUNT(16, nk == 2 ? 1 : 0);
                PGX_PROF_COUNT(18, any_contact ? 1 : 0);
                if (KMAX == 1 || nk == 1) solve_w(IC<3>{}, IC<1>{});
                else solve_w(IC<3>{}, IC<KMAX>{});
            } else if (spec_all) {
                solve_w(IC<1>{}, IC<0>{});
            } else {
                lmargin = -1.0f;   /* more than KMAX dofs: all rows */
            }
            const bool viol = lmargin < 0.0f;
            if (__any(row_any(viol)) || e.pgs_mode == 3) {
                PGX_PROF_COUNT(12, 1);
                gv = gv0;
                gw = gw0;
                gw2 = gw20;
#pragma unroll
                for (int p = 0; p < NP; p++) {
                    clam[p][0] = CONT ? Lp->pl0[p][es] : 0.0f;
                    clam[p][1] = 0.0f;
                    clam[p][2] = 0.0f;
                }
                if (RB > CGR && nxr > 0) load_xs(false);
                init_bounds();
                solve_w(IC<2>{}, IC<0>{});
            }
        } else {
            PGX_PROF_COUNT(13, 1);
            solve_w(IC<2>{}, IC<0>{});
        }
    }
    PGX_PROF_SWEEPS_DONE();
    PGX_PROF_MARK(4);
    PGX_PROF_COUNT(11, any_contact ? 1 : 0);
    if constexpr (PARK_SOLVE) {
#pragma unroll
        for (int j = 0; j < NJ; j++) { q[j] = unpark(j); vu[j] = unpark(NJ + j); }
        if constexpr (OBJ) {
            ob.p = v3(unpark(14), unpark(15), unpark(16));
            ob.qx = unpark(17); ob.qy = unpark(18); ob.qz = unpark(19); ob.qw = unpark(20);
            vcu = v3(unpark(21), unpark(22), unpark(23));
            wcu = v3(unpark(24), unpark(25), unpark(26));
        }
    }
    sfor<0, NJ>([&](auto jc) __attribute__((always_inline)) {
        constexpr int j = decltype(jc)::value;
        const float vn = fminf(fmaxf(vu[j] + bcast16<j>(gv), -m.max_vel), m.max_vel);
        qd[j] = vn;
        q[j] += m.dt * vn;
    });
    if (CONT) { /* contact cache: this step's features and normal impulses */
        ContactLdsGT<OBJ, FULL>& L = *Lp;
        /* every slot's id and jinv read unconditionally (one batch, one wait), then selected */
        float gid0[CG], pj0[CG], gid1[CGR], pj1[CGR];
#pragma unroll
        for (int s = 0; s < CG; s++) {
            gid0[s] = OBJ ? L.g0id[s][es] : -1.0f;
            pj0[s] = OBJ ? L.pjn[s][es] : 0.0f;
        }
#pragma unroll
        for (int s = 0; s < CGR; s++) {
            gid1[s] = L.g1id[s][es];
            pj1[s] = L.pjn[P0 + s][es];
        }
#pragma unroll
        for (int s = 0; s < CG; s++) {
            L.cache[2 * s][es] = (OBJ && s < n0) ? gid0[s] : -1.0f;
            L.cache[2 * s + 1][es] = (OBJ && s < n0) ? clam[s][0] * pj0[s] : 0.0f;
        }
#pragma unroll
        for (int s = 0; s < CGR; s++) {
            L.cache[CACHE1 + 2 * s][es] = s < n1 ? gid1[s] : -1.0f;
            L.cache[CACHE1 + 2 * s + 1][es] = s < n1 ? clam[P0 + s][0] * pj1[s] : 0.0f;
        }
        if constexpr (RB > CGR) {
            if (n1x > CGR) {   /* the extra normal rows' impulses: lane x % 16 of xs_lam[x / 16] to LDS */
#pragma unroll
                for (int b = 0; b < XB; b++)
                    if (GW * b + c < 3 * (n1x - CGR)) L.xlam[GW * b + c][es] = xs_lam[b];
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            }
            for (int s = CGR; s < RB; s++) {
                const int xq = 3 * (s - CGR);
                L.cache[CACHE1 + 2 * s][es] = s < n1 ? L.g1id[s][es] : -1.0f;
                L.cache[CACHE1 + 2 * s + 1][es] = s < n1 ? L.xlam[xq][es] * L.xjinv[xq][es] : 0.0f;
            }
        }
        if constexpr (PERS) {   /* the solved normal impulse back to its manifold point (writeBackContacts):
                                 * lane c takes slot c (each point feeds one slot, so no two lanes write
                                 * the same word) */
            static_assert(RB <= GW, "one lane per robot slot");
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            if (c < n1) {
                const int w = L.g1w[c][es];
                if (w >= 0) L.mimp[w][es] = L.cache[CACHE1 + 2 * c + 1][es];
            }
        }
    }
    if (OBJ) {
        const V3 dvl = v3(bcast16<7>(gv), bcast16<8>(gv), bcast16<9>(gv));
        const V3 dvw = v3(bcast16<10>(gv), bcast16<11>(gv), bcast16<12>(gv));
        object_integrate(m, ob, vcu + dvl, wcu + dvw);
    }
    PGX_PROF_MARK(5);
    return false;
}

/* EE (link 11) COM position and velocity: getLinkState(11)[0] and [6] */
__device__ __forceinline__ void ee_state(MRef m, const float* q, const float* qd, V3& pos, V3& vel) {
    Chain k;
    fk_chain(m, q, k);
    pos = k.o[NJ - 1] + mulc(k.R[NJ - 1], kEeCom);
    V3 vv = v3(0, 0, 0);
#pragma unroll
    for (int j = 0; j < NJ; j++) vv = vv + qd[j] * cross(col(k.R[j], 2), pos - k.o[j]);
    vel = vv;
}

/* getLinkState(11) as the reference reads it (oracle link_state_cached): Bullet's cached link
 * transform is the pose qc the last substep was solved at, and the local velocity (current q,
 * qd) is turned to world with the cached rotation: pos = COM(qc), vel = R7(qc) R7(q)^T v(q, qd)
 * (the EE link is rigid on link 7, so its rotation cancels in R_ee(qc) R_ee(q)^T). */
__device__ __forceinline__ void ee_state_cached(MRef m, const float* qc, const float* q, const float* qd, V3& pos,
                                                V3& vel) {
    Chain k;
    fk_chain(m, q, k);
    const V3 p = k.o[NJ - 1] + mulc(k.R[NJ - 1], kEeCom);
    V3 vv = v3(0, 0, 0);
#pragma unroll
    for (int j = 0; j < NJ; j++) vv = vv + qd[j] * cross(col(k.R[j], 2), p - k.o[j]);
    const V3 vl = mul_t(k.R[NJ - 1], vv);
    Chain kc;
    fk_chain(m, qc, kc);
    pos = kc.o[NJ - 1] + mulc(kc.R[NJ - 1], kEeCom);
    vel = mul(kc.R[NJ - 1], vl);
}

/* -------------------------------------------------------------- RNG */
/* philox(): pgx_common.h */
constexpr uint32_t TAG_RESET = 0x52455345u;
constexpr uint32_t TAG_ACTION = 0x41435430u;

__device__ __forceinline__ double reset_uniform_s(uint64_t seed, uint64_t env, uint32_t episode, int kidx) {
    uint32_t o[4];
    philox((uint32_t)env, (uint32_t)(env >> 32), episode, TAG_RESET + (uint32_t)(kidx >> 1), (uint32_t)seed,
           (uint32_t)(seed >> 32), o);
    uint64_t u = (kidx & 1) ? ((uint64_t)o[2] | ((uint64_t)o[3] << 32)) : ((uint64_t)o[0] | ((uint64_t)o[1] << 32));
    return (double)(u >> 11) * (1.0 / 9007199254740992.0);
}
__device__ __forceinline__ double reset_uniform(const PgxDevEnv& e, uint64_t env, uint32_t episode, int kidx) {
    return reset_uniform_s(e.seed, env, episode, kidx);
}

/* numpy's PCG64 (XSL-RR 128/64, the generator gymnasium's seeding.np_random builds,
 * core.py:302): state <- state * M + inc (mod 2^128), then the output of the new state:
 * rotr64(hi ^ lo, hi >> 58).  next_double = (u >> 11) * 2^-53 as in the reset draws above.
 * next_uint32 (numpy pcg64_next32) hands out a 64-bit output's low half and keeps the high half
 * for the next call (has_uint32 / uinteger); next_uint64 and next_double leave that half alone.
 * numpy leaves a spent uinteger in its state; the record holds 0 there (pcg64_record does too).
 * Record per env (pgx_set_rng_streams, PGX_PCG64_WORDS): state_lo, state_hi, inc_lo, inc_hi,
 * has_uint32, uinteger -- numpy's bit_generator.state. */
struct Pcg64 {
    uint64_t lo, hi, ilo, ihi;
    uint32_t has, u32;
};
__device__ __forceinline__ Pcg64 pcg64_load(const uint64_t* r) {
    return Pcg64{r[0], r[1], r[2], r[3], (uint32_t)r[4], (uint32_t)r[5]};
}
__device__ __forceinline__ void pcg64_store(const Pcg64& g, uint64_t* r) {
    r[0] = g.lo; r[1] = g.hi; r[2] = g.ilo; r[3] = g.ihi; r[4] = g.has; r[5] = g.u32;
}
__device__ __forceinline__ uint64_t pcg64_next64(Pcg64& g) {
    constexpr uint64_t MLO = 0x4385DF649FCCF645ull, MHI = 0x2360ED051FC65DA4ull;
    const uint64_t plo = g.lo * MLO;
    uint64_t hi = __umul64hi(g.lo, MLO) + g.lo * MHI + g.hi * MLO;
    const uint64_t lo = plo + g.ilo;
    hi += g.ihi + (uint64_t)(lo < plo);
    g.lo = lo;
    g.hi = hi;
    const uint64_t x = hi ^ lo;
    const uint32_t rot = (uint32_t)(hi >> 58);
    return (x >> rot) | (x << ((64u - rot) & 63u));
}
__device__ __forceinline__ double pcg64_next_double(Pcg64& g) {
    return (double)(pcg64_next64(g) >> 11) * (1.0 / 9007199254740992.0);
}
__device__ __forceinline__ uint32_t pcg64_next32(Pcg64& g) {
    if (g.has) {   /* (the spent half is cleared: a record's uinteger is 0 unless has_uint32) */
        const uint32_t v = g.u32;
        g.has = 0;
        g.u32 = 0;
        return v;
    }
    const uint64_t n = pcg64_next64(g);
    g.has = 1;
    g.u32 = (uint32_t)(n >> 32);
    return (uint32_t)n;
}
/* Generator.integers(off, off + rng + 1) for rng < 2^32 - 1 (int64 default: Lemire's bounded
 * draw on next_uint32, numpy buffered_bounded_lemire_uint32) */
__device__ __forceinline__ uint32_t pcg64_bounded(Pcg64& g, uint32_t rng) {
    const uint32_t excl = rng + 1u;
    uint64_t m = (uint64_t)pcg64_next32(g) * excl;
    uint32_t left = (uint32_t)m;
    if (left < excl) {
        const uint32_t thr = (0xFFFFFFFFu - rng) % excl;
        while (left < thr) {
            m = (uint64_t)pcg64_next32(g) * excl;
            left = (uint32_t)m;
        }
    }
    return (uint32_t)(m >> 32);
}
/* random_interval(max) for max < 2^32 (Generator.shuffle of a list): masked rejection on next_uint32 */
__device__ __forceinline__ uint32_t pcg64_interval(Pcg64& g, uint32_t max) {
    if (max == 0) return 0;
    uint32_t mask = max;
    mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16;
    uint32_t v;
    while ((v = (pcg64_next32(g) & mask)) > max) {}
    return v;
}

/* --------------------------------------------------------- env epilogue */
#pragma clang fp contract(off)
/* utils.distance on (float32 achieved, float64 goal) -> float64, rounded to 1e-6 */
__device__ double distance_f32_f64(V3 ag, const double* gl) {
    double d0 = (double)ag.x - gl[0], d1 = (double)ag.y - gl[1], d2 = (double)ag.z - gl[2];
    double s = d0 * d0 + d1 * d1;
    s = s + d2 * d2;
    double d = sqrt(s);
    return rint(d * 1e6) / 1e6;
}
/* goal = offset + noise (push.py:77-79), unfused */
__device__ double goal_add(double a, double b) { return a + b; }
/* numpy Generator.uniform: low + (high - low) * u, unfused */
__device__ double uniform_draw(double low, double high, double u) {
    double r = high - low;
    double t = r * u;
    return low + t;
}
#pragma clang fp contract(on)

/* pybullet getEulerFromQuaternion (PyBullet.get_base_rotation, pybullet.py:216-219) */
__device__ __forceinline__ V3 quat_euler(const ObjState& o) {
    const float x = o.qx, y = o.qy, z = o.qz, w = o.qw;
    const float sqx = x * x, sqy = y * y, sqz = z * z, squ = w * w;
    const float sarg = -2.0f * (x * z - w * y);
    const float pitch = sarg <= -1.0f ? -0.5f * 3.141592538f : (sarg >= 1.0f ? 0.5f * 3.141592538f : asinf(sarg));
    const float roll = atan2f(2.0f * (y * z + w * x), squ - sqx - sqy + sqz);
    const float yaw = atan2f(2.0f * (x * y + w * z), squ + sqx - sqy - sqz);
    return v3(roll, pitch, yaw);
}

/* RobotTaskEnv._get_obs (core.py:286-296): robot obs (panda.py:264-288), then the task
 * obs of Push / PickAndPlace (push.py:49-63): object position, euler, velocity, angular
 * velocity. */
template <int OBJ>
__device__ __forceinline__ void write_obs(const PgxDevEnv& e, float* dst, V3 pos, V3 vel, const ObjState& ob) {
    dst[0] = pos.x; dst[1] = pos.y; dst[2] = pos.z;
    dst[3] = vel.x; dst[4] = vel.y; dst[5] = vel.z;
    int n = 6;
    if (!e.block_gripper) dst[n++] = 0.0f; /* custom_0 fingers are fixed joints: width 0 */
    if (OBJ) {
        const V3 rpy = quat_euler(ob);
        dst[n] = ob.p.x; dst[n + 1] = ob.p.y; dst[n + 2] = ob.p.z;
        dst[n + 3] = rpy.x; dst[n + 4] = rpy.y; dst[n + 5] = rpy.z;
        dst[n + 6] = ob.v.x; dst[n + 7] = ob.v.y; dst[n + 8] = ob.v.z;
        dst[n + 9] = ob.w.x; dst[n + 10] = ob.w.y; dst[n + 11] = ob.w.z;
    }
}

/* Panda.reset + Task.reset (reach.py:63-78, push.py:69-87, pick_and_place.py:65-85): draws
 * in the reference's order (goal noise 0-2, PickAndPlace's z coin 3, object noise); the
 * object is re-posed upright, its velocity kept (resetBasePositionAndOrientation). */
template <int OBJ>
__device__ __forceinline__ void reset_env(MRef m, const PgxDevEnv& e, int i, uint32_t& episode, const double* inject,
                                          const double* inject_obj, float* q, float* qd, double* goal,
                                          ObjState& ob, bool lead = true) {
#pragma unroll
    for (int j = 0; j < NJ; j++) { q[j] = m.neutral_q[j]; qd[j] = 0.0f; }
    uint64_t env = e.env_id_offset + (uint64_t)i;
    /* the draw source: the env's numpy PCG64 stream (pgx_set_rng_streams) advanced in draw order,
     * or the Philox counter (env, episode, draw index) */
    const bool pcg = e.pcg_on != nullptr && *e.pcg_on != 0;
    Pcg64 g{0, 0, 0, 0, 0, 0};
    if (pcg) g = pcg64_load(e.pcg + PGX_PCG64_WORDS * (size_t)i);
    auto draw = [&](int k) -> double { return pcg ? pcg64_next_double(g) : reset_uniform(e, env, episode, k); };
    double noise[3];
#pragma unroll
    for (int c = 0; c < 3; c++) noise[c] = uniform_draw(e.goal_low[c], e.goal_high[c], draw(c));
    int k = 3;
    if (OBJ && e.goal_z_zero_prob > 0.0) {
        if (draw(k) < e.goal_z_zero_prob) noise[2] = 0.0;
        k++;
    }
#pragma unroll
    for (int c = 0; c < 3; c++) goal[c] = inject ? inject[c] : goal_add(e.goal_offset[c], noise[c]);
    if (OBJ) {
        double p[3];
#pragma unroll
        for (int c = 0; c < 3; c++) {
            const double u = draw(k + c);
            p[c] = inject_obj ? inject_obj[c] : goal_add(e.obj_offset[c], uniform_draw(e.obj_low[c], e.obj_high[c], u));
        }
        ob.p = v3((float)p[0], (float)p[1], (float)p[2]);
        ob.qx = 0.0f; ob.qy = 0.0f; ob.qz = 0.0f; ob.qw = 1.0f;
    }
    /* an injected reset replaces the task's draws: its stream stays where it was */
    if (pcg && lead && !inject && !inject_obj) pcg64_store(g, e.pcg + PGX_PCG64_WORDS * (size_t)i);
    episode += 1;
}

__device__ __forceinline__ void load_obj(const PgxDevState& s, int N, int i, ObjState& ob) {
    const float* o = s.object;
    ob.p = v3(o[0 * N + i], o[1 * N + i], o[2 * N + i]);
    ob.qx = o[3 * N + i]; ob.qy = o[4 * N + i]; ob.qz = o[5 * N + i]; ob.qw = o[6 * N + i];
    ob.v = v3(o[7 * N + i], o[8 * N + i], o[9 * N + i]);
    ob.w = v3(o[10 * N + i], o[11 * N + i], o[12 * N + i]);
}
__device__ __forceinline__ void store_obj(const PgxDevState& s, int N, int i, const ObjState& ob) {
    float* o = s.object;
    o[0 * N + i] = ob.p.x; o[1 * N + i] = ob.p.y; o[2 * N + i] = ob.p.z;
    o[3 * N + i] = ob.qx; o[4 * N + i] = ob.qy; o[5 * N + i] = ob.qz; o[6 * N + i] = ob.qw;
    o[7 * N + i] = ob.v.x; o[8 * N + i] = ob.v.y; o[9 * N + i] = ob.v.z;
    o[10 * N + i] = ob.w.x; o[11 * N + i] = ob.w.y; o[12 * N + i] = ob.w.z;
}


/* ------------------------------------------------------------- ReachAO */
/* PandaReachAO-v3 "reachao_rand" (reach_ao.py; restated in oracle/pgx_oracle.c "ReachAO"):
 * 3 spheres (r 0.05) then 3 cuboids (half 0.05, rounded by the 1 mm box margin) per env,
 * centres in LDS; the robot's 9 collision links (panda_link1..8, panda_ee: every capsule
 * but the base and the hand) against them after every substep (step_check_collision
 * :182-188, early exit), and against the table for links 2..ee (check_collided
 * :896-900); the observation's closest distance + unit vector per link (get_obs
 * "vectors+closest_per_link" :902-959).  Exact distances are evaluated only for pairs a
 * cheap bound cannot rule out: the capsule axis against the obstacle's bounding sphere. */
/* world end points of every capsule at q (base capsule included) into LDS */
template <int C = 0, class LT>
__device__ __forceinline__ void ao_caps_walk(const Chain& k, MRef m, LT& L, int ln) {
    if constexpr (C < PGX_NCAP) {
        V3 A, B;
        if constexpr (kCapJ[C] < 0) {
            const V3 b = v3(m.base[0], m.base[1], m.base[2]);
            A = b + v3(kCapA[C][0], kCapA[C][1], kCapA[C][2]);
            B = b + v3(kCapB[C][0], kCapB[C][1], kCapB[C][2]);
        } else {
            A = k.o[kCapJ[C]] + mulc(k.R[kCapJ[C]], kCapA[C]);
            B = k.o[kCapJ[C]] + mulc(k.R[kCapJ[C]], kCapB[C]);
        }
        L.capA[C][0][ln] = A.x; L.capA[C][1][ln] = A.y; L.capA[C][2][ln] = A.z;
        L.capB[C][0][ln] = B.x; L.capB[C][1][ln] = B.y; L.capB[C][2][ln] = B.z;
        ao_caps_walk<C + 1, LT>(k, m, L, ln);
    }
}
template <class LT>
__device__ __forceinline__ void ao_caps(MRef m, const float* q, LT& L, int ln) {
    Chain k;
    fk_chain(m, q, k);
    ao_caps_walk(k, m, L, ln);
}


/* check_collided: any collision link within 0 of an obstacle, or links 2..ee of the table */
template <class LT>
__device__ __forceinline__ bool ao_collided(const PgxDevEnv& e, LT& L, int ln) {
    const V3 tc = ao_table_c(e), th = ao_table_h(e);
    const V3 thi = v3(th.x - kAoMargin, th.y - kAoMargin, th.z - kAoMargin);
    const V3 hcube = v3(kAoSize, kAoSize, kAoSize);
    bool hit = false;
    for (int c = 0; c < PGX_NCAP && !hit; c++) {
        const int slot = kAoSlot[c];
        if (slot < 0) continue;
        const V3 A = lds3(L.capA[c], ln), B = lds3(L.capB[c], ln);
        const float r = kCapR[c];
        for (int o = 0; o < AO_N; o++) {
            const V3 C = lds3(L.aoC[o], ln);
            const V3 P = seg_closest(A, B, C);
            const float dc = norm(C - P) - r;
            if (o < 3) hit = hit || dc - kAoSize <= 0.0f;
            else if (dc - kAoCubeBound <= 0.0f) hit = hit || capsule_box_hit(A, B, r, C, hcube);
        }
        if (slot >= 1) {
            /* box_sd is 1-Lipschitz: min over the segment >= min(ends) - |AB| / 2 */
            const float lb = fminf(box_sd(A, tc, thi), box_sd(B, tc, thi)) - 0.5f * norm(B - A) - kAoMargin - r;
            if (lb <= 0.0f) hit = hit || capsule_box_hit(A, B, r, tc, th);
        }
    }
    return hit;
}

/* per collision link: the closest obstacle's distance and unit vector into LDS */
template <class LT>
__device__ __forceinline__ void ao_link_obs(LT& L, int ln) {
    for (int l = 0; l < PGX_AO_LINKS; l++) L.aoD[l][ln] = 3.0e38f;
    const V3 hcube = v3(kAoSize, kAoSize, kAoSize);
    for (int c = 0; c < PGX_NCAP; c++) {
        const int slot = kAoSlot[c];
        if (slot < 0) continue;
        const V3 A = lds3(L.capA[c], ln), B = lds3(L.capB[c], ln);
        const float r = kCapR[c];
        float best = L.aoD[slot][ln];
        V3 bu = v3(0.0f, 0.0f, 0.0f);
        bool upd = false;
        for (int o = 0; o < AO_N; o++) {
            const V3 C = lds3(L.aoC[o], ln);
            const V3 P = seg_closest(A, B, C);
            const V3 v = C - P;
            const float len = norm(v);
            if (o < 3) {
                const float d = len - r - kAoSize;
                if (d < best) {
                    best = d;
                    const V3 n = len > 0.0f ? fast_rcp(len) * v : v3(0.0f, 0.0f, 1.0f);
                    bu = d > 0.0f ? n : (d < 0.0f ? (-1.0f) * n : v3(0.0f, 0.0f, 0.0f));
                    upd = true;
                }
            } else if (len - r - kAoCubeBound < best) {
                V3 u;
                const float d = capsule_box<true>(A, B, r, C, hcube, &u);
                if (d < best) { best = d; bu = u; upd = true; }
            }
        }
        if (upd) {
            L.aoD[slot][ln] = best;
            L.aoU[slot][0][ln] = bu.x; L.aoU[slot][1][ln] = bu.y; L.aoU[slot][2][ln] = bu.z;
        }
    }
}

/* Wide layout (16 lanes per env): lane c evaluates capsule c (14 capsules) against the six
 * obstacles and the table, the same per-pair arithmetic as ao_collided / ao_link_obs; the env's
 * decision is the OR over its row (ballot), the per-link minimum is combined across the
 * capsules of one link in capsule order with the sequential code's strict '<' (the earlier
 * capsule keeps a tie). */
template <class LT>
__device__ __forceinline__ bool ao_collided_g(const PgxDevEnv& e, LT& L, int es, int c) {
    const V3 tc = ao_table_c(e), th = ao_table_h(e);
    const V3 thi = v3(th.x - kAoMargin, th.y - kAoMargin, th.z - kAoMargin);
    const V3 hcube = v3(kAoSize, kAoSize, kAoSize);
    const int cc = c < PGX_NCAP ? c : 0;
    const CapLane cl = cap_lane();
    const int slot = c < PGX_NCAP ? cl.slot : -1;
    bool hit = false;
    if (slot >= 0) {
        const V3 A = lds3(L.capA[cc], es), B = lds3(L.capB[cc], es);
        const float r = cl.r;
        for (int o = 0; o < AO_N; o++) {
            const V3 C = lds3(L.aoC[o], es);
            const V3 P = seg_closest(A, B, C);
            const float dc = norm(C - P) - r;
            if (o < 3) hit = hit || dc - kAoSize <= 0.0f;
            else if (dc - kAoCubeBound <= 0.0f) hit = hit || capsule_box_hit(A, B, r, C, hcube);
        }
        if (slot >= 1) {
            const float lb = fminf(box_sd(A, tc, thi), box_sd(B, tc, thi)) - 0.5f * norm(B - A) - kAoMargin - r;
            if (lb <= 0.0f) hit = hit || capsule_box_hit(A, B, r, tc, th);
        }
    }
    return row_any(hit);
}
__host__ __device__ constexpr bool ao_first_of_slot(int c) {
    for (int k = 0; k < c; k++)
        if (ao_slot(k) == ao_slot(c)) return false;
    return true;
}
template <class LT>
__device__ __forceinline__ void ao_link_obs_g(LT& L, int es, int c) {
    const V3 hcube = v3(kAoSize, kAoSize, kAoSize);
    const int cc = c < PGX_NCAP ? c : 0;
    const CapLane cl = cap_lane();
    const int slot = c < PGX_NCAP ? cl.slot : -1;
    float best = 3.0e38f;
    V3 bu = v3(0.0f, 0.0f, 0.0f);
    if (slot >= 0) {
        const V3 A = lds3(L.capA[cc], es), B = lds3(L.capB[cc], es);
        const float r = cl.r;
        for (int o = 0; o < AO_N; o++) {
            const V3 C = lds3(L.aoC[o], es);
            const V3 P = seg_closest(A, B, C);
            const V3 v = C - P;
            const float len = norm(v);
            if (o < 3) {
                const float d = len - r - kAoSize;
                if (d < best) {
                    best = d;
                    const V3 n = len > 0.0f ? fast_rcp(len) * v : v3(0.0f, 0.0f, 1.0f);
                    bu = d > 0.0f ? n : (d < 0.0f ? (-1.0f) * n : v3(0.0f, 0.0f, 0.0f));
                }
            } else if (len - r - kAoCubeBound < best) {
                V3 u;
                const float d = capsule_box<true>(A, B, r, C, hcube, &u);
                if (d < best) { best = d; bu = u; }
            }
        }
    }
    float D[PGX_AO_LINKS], Ux[PGX_AO_LINKS], Uy[PGX_AO_LINKS], Uz[PGX_AO_LINKS];
    sfor<0, PGX_NCAP>([&](auto kc) __attribute__((always_inline)) {
        constexpr int C = decltype(kc)::value, sl = ao_slot(C);
        if constexpr (sl >= 0) {
            const float b = bcast16<C>(best), x = bcast16<C>(bu.x), y = bcast16<C>(bu.y), z = bcast16<C>(bu.z);
            if constexpr (ao_first_of_slot(C)) {
                D[sl] = b; Ux[sl] = x; Uy[sl] = y; Uz[sl] = z;
            } else {
                const bool take = b < D[sl];
                D[sl] = take ? b : D[sl]; Ux[sl] = take ? x : Ux[sl]; Uy[sl] = take ? y : Uy[sl];
                Uz[sl] = take ? z : Uz[sl];
            }
        }
    });
#pragma unroll
    for (int l = 0; l < PGX_AO_LINKS; l++) {
        L.aoD[l][es] = D[l];
        L.aoU[l][0][es] = Ux[l]; L.aoU[l][1][es] = Uy[l]; L.aoU[l][2][es] = Uz[l];
    }
}

/* robot obs ("ee","js": panda.py:264-288) + 9 distances + 9 unit vectors */
template <class LT>
__device__ __forceinline__ void ao_write_obs(float* dst, V3 pos, V3 vel, const float* q, const float* qd,
                                             const LT& L, int ln) {
    dst[0] = pos.x; dst[1] = pos.y; dst[2] = pos.z;
    dst[3] = vel.x; dst[4] = vel.y; dst[5] = vel.z;
#pragma unroll
    for (int j = 0; j < NJ; j++) { dst[6 + j] = q[j]; dst[13 + j] = qd[j]; }
#pragma unroll
    for (int l = 0; l < PGX_AO_LINKS; l++) dst[20 + l] = L.aoD[l][ln];
#pragma unroll
    for (int l = 0; l < PGX_AO_LINKS; l++)
#pragma unroll
        for (int k = 0; k < 3; k++) dst[29 + 3 * l + k] = L.aoU[l][k][ln];
}

/* ---- The reset's accept / reject geometry in fp64 (round 6).  Every test restates the host
 * sampler's numpy arithmetic (panda-gym_amd/reach_ao.py: box_sd, rbox_sd, capsule_sphere_dist,
 * capsule_box_dist) operation for operation, unfused, on the host's own fp64 capsules at the
 * neutral pose (pgx_config.ao_capsules_neutral, PgxDevEnv.ao_geo), so a device-drawn reset takes
 * the host restatement's branch at every test and consumes numpy's stream draw for draw.  Round 5
 * ran these tests on the kernel's fp32 capsules, and a seed whose test sat within fp32 rounding of
 * its threshold took the other branch.  Only resets run this code. */
/* The reset code is inlined (round 6): as __noinline__ calls its frames -- the by-reference
 * arguments, the callees' stacks -- put 164 B per lane of scratch under ReachAO's step kernels.
 * Inlined at the end of the step, where little else is live, it costs the substep loop nothing.
 * -DPGX_AO_CALL=__noinline__ builds the calls for an A/B. */
#ifndef PGX_AO_CALL
#define PGX_AO_CALL __forceinline__
#endif
constexpr double kAo64Size = 0.05, kAo64Margin = 0.001, kAo64DummyR = 0.05;   /* reach_ao.py AO_SIZE, MARGIN, DUMMY_R */
constexpr double kAo64GoalMargin = 0.1, kAo64ObstMargin = 0.03;                 /* GOAL_MARGIN, OBST_MARGIN */
/* decisions the early exits below take only with this much room: the host's value of a capsule-box
 * distance lies within |AB| (2/3)^40 < 1e-7 of the exact minimum (convex search + projections) */
constexpr double kAo64Slack = 1e-6;
struct D3 { double x, y, z; };
__device__ __forceinline__ D3 d3(double x, double y, double z) { return D3{x, y, z}; }

/* box_sd: |P - c| - h, sqrt of the positive parts' squares + the inner part */
__device__ __forceinline__ double ao64_box_sd(D3 P, D3 c, D3 h) {
#pragma clang fp contract(off)
    const double dx = fabs(P.x - c.x) - h.x, dy = fabs(P.y - c.y) - h.y, dz = fabs(P.z - c.z) - h.z;
    const double px = dx > 0.0 ? dx : 0.0, py = dy > 0.0 ? dy : 0.0, pz = dz > 0.0 ? dz : 0.0;
    const double o = px * px + py * py + pz * pz;
    const double inner = fmax(fmax(dx, dy), dz);
    return sqrt(o) + (inner < 0.0 ? inner : 0.0);
}
/* rbox_sd: the box rounded by MARGIN */
__device__ __forceinline__ double ao64_rbox_sd(D3 P, D3 c, D3 h) {
#pragma clang fp contract(off)
    return ao64_box_sd(P, c, d3(h.x - kAo64Margin, h.y - kAo64Margin, h.z - kAo64Margin)) - kAo64Margin;
}
__device__ __forceinline__ double ao64_clip01(double x) { return fmin(fmax(x, 0.0), 1.0); }

/* capsule (A, B, r) against a sphere (C, R): capsule_sphere_dist */
__device__ __forceinline__ double ao64_capsule_sphere(D3 A, D3 B, double r, D3 C, double R) {
#pragma clang fp contract(off)
    const D3 ab = d3(B.x - A.x, B.y - A.y, B.z - A.z);
    const double l2 = ab.x * ab.x + ab.y * ab.y + ab.z * ab.z;
    const double num = (C.x - A.x) * ab.x + (C.y - A.y) * ab.y + (C.z - A.z) * ab.z;
    const double t = l2 > 0.0 ? ao64_clip01(num / l2) : 0.0;
    const D3 P = d3(A.x + t * ab.x, A.y + t * ab.y, A.z + t * ab.z);
    const D3 v = d3(C.x - P.x, C.y - P.y, C.z - P.z);
    return sqrt(v.x * v.x + v.y * v.y + v.z * v.z) - r - R;
}

/* Is capsule (A, B, r)'s capsule_box_dist to the rounded cube (c, half size s) <= thr?
 * capsule_box_dist: 40 ternary-search steps on the inner box's signed distance along the axis, two
 * alternating projections (box -> segment) where the point is outside, box_sd - MARGIN - r.  The
 * search's samples decide early where they leave room: a sample within thr - kAo64Slack (the final
 * value is at most the best sample + 1e-7, the projections only lower it) is a hit, and the best
 * sample minus |AB| times the bracket (the exact minimum of the convex box distance is no lower)
 * beyond thr + kAo64Slack is clear; otherwise the full computation decides, as the host's. */
__device__ PGX_AO_CALL bool ao64_capsule_box_within(D3 A, D3 B, double r, D3 c, double s, double thr) {
#pragma clang fp contract(off)
    const D3 hb = d3(s - kAo64Margin, s - kAo64Margin, s - kAo64Margin);
    const D3 ab = d3(B.x - A.x, B.y - A.y, B.z - A.z);
    const double l2 = ab.x * ab.x + ab.y * ab.y + ab.z * ab.z;
    const bool nz = l2 > 0.0;
    const double len = sqrt(l2);
    double lo = 0.0, hi = 1.0;
    for (int it = 0; it < 40; it++) {
        const double w = hi - lo;
        const double m1 = lo + w / 3.0, m2 = hi - w / 3.0;
        const double f1 = ao64_box_sd(d3(A.x + m1 * ab.x, A.y + m1 * ab.y, A.z + m1 * ab.z), c, hb);
        const double f2 = ao64_box_sd(d3(A.x + m2 * ab.x, A.y + m2 * ab.y, A.z + m2 * ab.z), c, hb);
        const double fb = fmin(f1, f2) - kAo64Margin - r;
        if (fb <= thr - kAo64Slack) return true;
        if (fb - len * w > thr + kAo64Slack) return false;
        const bool left = f1 <= f2;
        hi = left ? m2 : hi;
        lo = left ? lo : m1;
    }
    const double t = nz ? 0.5 * (lo + hi) : 0.0;
    D3 P = d3(A.x + t * ab.x, A.y + t * ab.y, A.z + t * ab.z);
    const bool outside = ao64_box_sd(P, c, hb) > 0.0 && nz;
    const double den = nz ? l2 : 1.0;
    for (int it = 0; it < 2; it++) {
        const D3 q = d3(fmin(fmax(P.x, c.x - hb.x), c.x + hb.x), fmin(fmax(P.y, c.y - hb.y), c.y + hb.y),
                        fmin(fmax(P.z, c.z - hb.z), c.z + hb.z));
        const double num = (q.x - A.x) * ab.x + (q.y - A.y) * ab.y + (q.z - A.z) * ab.z;
        const double tq = ao64_clip01(num / den);
        if (outside) P = d3(A.x + tq * ab.x, A.y + tq * ab.y, A.z + tq * ab.z);
    }
    return ao64_box_sd(P, c, hb) - kAo64Margin - r <= thr;
}

/* Does the robot come within thr of a sphere (kind 0, radius s) or a rounded cube (kind 1, half
 * size s) at C?  RobotGeometry.distance(kind, C, s) - thr <= 0 with the minimum over the capsules:
 * rounding is monotone, so that is "some capsule's value <= thr", which the first such capsule
 * decides.  A capsule whose axis keeps more than r + circumradius + thr + kAo64Slack from the
 * cube's centre is clear without the search.  geo: [PGX_NCAP][7] (A, B, r) at the neutral pose.
 * PAR (wide layout): lane c tests capsule c, the row ballot ORs them. */
template <bool PAR>
__device__ PGX_AO_CALL bool ao_robot_hit64(const double* __restrict__ geo, int lane, int kind, D3 C, double s,
                                            double thr) {
    auto test = [&](int cp) __attribute__((always_inline)) {
        const double* g = geo + 7 * cp;
        const D3 A = d3(g[0], g[1], g[2]), B = d3(g[3], g[4], g[5]);
        const double r = g[6];
        if (kind == 0) return ao64_capsule_sphere(A, B, r, C, s) <= thr;
        if (ao64_capsule_sphere(A, B, r, C, 1.7320508075688772 * s) > thr + kAo64Slack) return false;
        return ao64_capsule_box_within(A, B, r, C, s, thr);
    };
    if constexpr (PAR) {
        return row_any(lane < PGX_NCAP && test(lane < PGX_NCAP ? lane : 0));
    } else {
        for (int cp = 0; cp < PGX_NCAP; cp++)
            if (test(cp)) return true;
        return false;
    }
}

/* the reset's draw source: the env's numpy PCG64 stream (g, pgx_set_rng_streams) or the Philox
 * counter (env, episode, draw index) */
struct AoDraw {
    uint64_t seed;
    uint64_t env;
    uint32_t episode;
    int k;
    bool pcg;   /* draw from g (held here by value: no pointer, so it stays in registers) */
    Pcg64 g;
};
__device__ __forceinline__ double ao_draw(AoDraw& d) {
    return d.pcg ? pcg64_next_double(d.g) : reset_uniform_s(d.seed, d.env, d.episode, d.k++);
}
__device__ __forceinline__ double ao_uniform(AoDraw& d, double lo, double hi) {
    return uniform_draw(lo, hi, ao_draw(d));
}
/* sample_within_hollow_sphere (reach_ao.py:1188-1211) */
__device__ PGX_AO_CALL void ao_hollow_sphere(AoDraw& d, double rmin, double rmax, bool upper, double* out) {
    const double pi = 3.14159265358979323846;
    const double phi = ao_uniform(d, 0.0, 2.0 * pi);
    const double theta = upper ? ao_uniform(d, 0.0, 0.5 * pi) : ao_uniform(d, 0.0, pi);
    const double r = cbrt(ao_uniform(d, pow(rmin, 3.0), pow(rmax, 3.0)));
    out[0] = r * sin(theta) * cos(phi);
    out[1] = r * sin(theta) * sin(phi);
    out[2] = r * cos(theta);
}

/* ReachAO.reset for reachao_rand (reach_ao.py:965-1082; oracle ao_reset_task): goal,
 * obstacles by rejection against robot / table / dummy sphere, 4-5 active.  Needs the
 * neutral-pose capsules in LDS; leaves the centres in L.aoC.  rec: the env's PCG64 record
 * (pgx_set_rng_streams; nullptr: Philox), drawn as numpy's Generator draws (uniform / random:
 * next_double; integers(4, 6): Lemire on next_uint32; shuffle of the 6 names: random_interval on
 * next_uint32) and written back by the lead lane unless the reset is injected. */
/* What ao_reset reads of the env, by value: a reference to the kernel's PgxDevEnv argument would
 * make every lane copy the whole struct to scratch at kernel start (368 B per lane) for this
 * rarely taken call. */
struct AoResetIn {
    uint64_t seed;
    const double* geo;   /* PgxDevEnv.ao_geo: fp64 capsules at the neutral pose, then the table box */
    double ex, ey, ez;   /* get_ee_position after Panda.reset (pgx_config.ao_ee_neutral, or the fp32 FK) */
};
__device__ __forceinline__ AoResetIn ao_reset_in(const PgxDevEnv& e, V3 ee) {
    return AoResetIn{e.seed, e.ao_geo, e.ao_ee_set ? e.ao_ee[0] : (double)ee.x,
                     e.ao_ee_set ? e.ao_ee[1] : (double)ee.y, e.ao_ee_set ? e.ao_ee[2] : (double)ee.z};
}
template <bool PAR, class LT>
__device__ PGX_AO_CALL bool ao_reset(const AoResetIn& in, LT& L, int ln, int lane, uint64_t env, uint32_t episode,
                                      const double* inject_goal, const double* inject_obst, double* goal,
                                      uint64_t* rec, bool lead) {
#pragma clang fp contract(off)
    bool failed = false;   /* set_coll_free_obs gave up: the reference raises StopIteration */
    const double ex = in.ex, ey = in.ey, ez = in.ez;
    AoDraw d{in.seed, env, episode, 0, rec != nullptr, Pcg64{0, 0, 0, 0, 0, 0}};
    if (rec) d.g = pcg64_load(rec);
    const double* geo = in.geo;
    const D3 tc = d3(geo[7 * PGX_NCAP], geo[7 * PGX_NCAP + 1], geo[7 * PGX_NCAP + 2]);
    const D3 th = d3(geo[7 * PGX_NCAP + 3], geo[7 * PGX_NCAP + 4], geo[7 * PGX_NCAP + 5]);
    D3 dummy = d3(0.0, 0.0, 0.0);
    for (int i = 0;; i++) {
        ao_hollow_sphere(d, 0.5, 0.8, true, goal);
        if (i > 9999) { goal[0] = ex; goal[1] = ey; goal[2] = ez; break; }
        dummy = d3(goal[0], goal[1], goal[2]);
        /* set_coll_free_goal (reach_ao.py:1101-1123; host reset_draws): the dummy sphere keeps more
         * than GOAL_MARGIN from the table and from the robot */
        const bool coll = ao64_rbox_sd(dummy, tc, th) - kAo64DummyR <= kAo64GoalMargin ||
                          ao_robot_hit64<PAR>(geo, lane, 0, dummy, kAo64DummyR, kAo64GoalMargin);
        if (!coll) break;
    }
    const D3 hcube = d3(kAo64Size, kAo64Size, kAo64Size);
    const D3 tgrow = d3(th.x + kAo64Size - 2.0 * kAo64Margin, th.y + kAo64Size - 2.0 * kAo64Margin,
                        th.z + kAo64Size - 2.0 * kAo64Margin);
    for (int o = 0; o < AO_N; o++) {
        double P[3];
        bool placed = false;
        for (int it = 0; it < 10000; it++) {
            const double rnd = ao_draw(d);
            double sm[3];
            ao_hollow_sphere(d, 0.1, 0.5, false, sm);
            if (rnd > 0.5) { P[0] = sm[0] + goal[0]; P[1] = sm[1] + goal[1]; P[2] = sm[2] + goal[2]; }
            else { P[0] = ex + sm[0]; P[1] = ey + sm[1]; P[2] = ez + sm[2]; }
            /* set_coll_free_obs (reach_ao.py:1137-1161; host reset_draws): more than OBST_MARGIN
             * from the table, the dummy sphere and the robot */
            const D3 Pd = d3(P[0], P[1], P[2]);
            double dtab, ddum;
            if (o < 3) {
                dtab = ao64_rbox_sd(Pd, tc, th) - kAo64Size;
                const D3 v = d3(Pd.x - dummy.x, Pd.y - dummy.y, Pd.z - dummy.z);
                ddum = sqrt(v.x * v.x + v.y * v.y + v.z * v.z) - kAo64Size - kAo64DummyR;
            } else {
                dtab = ao64_box_sd(Pd, tc, tgrow) - 2.0 * kAo64Margin;
                ddum = ao64_rbox_sd(dummy, Pd, hcube) - kAo64DummyR;
            }
            const bool coll = dtab <= kAo64ObstMargin || ddum <= kAo64ObstMargin ||
                              ao_robot_hit64<PAR>(geo, lane, o < 3 ? 0 : 1, Pd, kAo64Size, kAo64ObstMargin);
            if (!coll) { placed = true; break; }
        }
        failed = failed || !placed;
        L.aoC[o][0][ln] = (float)P[0]; L.aoC[o][1][ln] = (float)P[1]; L.aoC[o][2][ln] = (float)P[2];
    }
    const int n_active = 4 + (rec ? (int)pcg64_bounded(d.g, 1u) : (int)(ao_draw(d) * 2.0));
    int perm[AO_N] = {0, 1, 2, 3, 4, 5};
    for (int j = AO_N - 1; j > 0; j--) {   /* Fisher-Yates, unrolled so perm stays in VGPRs */
        int r = rec ? (int)pcg64_interval(d.g, (uint32_t)j) : (int)(ao_draw(d) * (double)(j + 1));
        r = r > j ? j : r;
        int pj = 0, pr = 0;
#pragma unroll
        for (int t = 0; t < AO_N; t++) { pj = t == j ? perm[t] : pj; pr = t == r ? perm[t] : pr; }
#pragma unroll
        for (int t = 0; t < AO_N; t++) perm[t] = t == j ? pr : (t == r ? pj : perm[t]);
    }
#pragma unroll
    for (int t = 0; t < AO_N; t++) {
        int pt = perm[t];
        if (t < AO_N - n_active) { L.aoC[pt][0][ln] = 99.9f; L.aoC[pt][1][ln] = 99.9f; L.aoC[pt][2][ln] = -99.9f; }
    }
    if (inject_goal) { goal[0] = inject_goal[0]; goal[1] = inject_goal[1]; goal[2] = inject_goal[2]; }
    if (inject_obst)
        for (int o = 0; o < AO_N; o++)
            for (int k = 0; k < 3; k++) L.aoC[o][k][ln] = (float)inject_obst[3 * o + k];
    if (rec && lead && !inject_goal && !inject_obst) pcg64_store(d.g, rec);
    return failed && !inject_obst;
}

template <class LT>
__device__ __forceinline__ void ao_load(const PgxDevState& s, int N, int i, LT& L, int ln) {
#pragma unroll
    for (int o = 0; o < AO_N; o++)
#pragma unroll
        for (int k = 0; k < 3; k++) L.aoC[o][k][ln] = s.obstacles[(3 * o + k) * N + i];
}
template <class LT>
__device__ __forceinline__ void ao_store(const PgxDevState& s, int N, int i, const LT& L, int ln) {
#pragma unroll
    for (int o = 0; o < AO_N; o++) {
#pragma unroll
        for (int k = 0; k < 3; k++) s.obstacles[(3 * o + k) * N + i] = L.aoC[o][k][ln];
        s.obstacles[(3 * AO_N + o) * N + i] = L.aoC[o][0][ln] < 50.0f ? 1.0f : 0.0f;
    }
}

/* Workgroups are dealt to the 8 XCDs round-robin (block b -> XCD b % 8), each with its own
 * L2: give every XCD a contiguous range of blocks, so the env-minor state rows one wave
 * touches share cache lines with its neighbours' on the same L2 instead of being fetched
 * once per XCD (PMC: 4.3 MB of HBM traffic per 4096-env launch for 0.8 MB of state). */
__device__ __forceinline__ int xcd_block() {
    const int nb = gridDim.x, b = blockIdx.x;
    if (nb % 8) return b;
    return (b % 8) * (nb / 8) + b / 8;
}

/* WIDE = 0: one env per lane (64 per wave); WIDE = 1: 16 lanes per env (4 per wave,
 * substep_g), the redundant lanes compute the same values and only the lead lane stores. */
template <int CONTROL, int OBJ, int CONT, int AO, int WIDE, int PART = 1>
__device__ __forceinline__ void step_body(const PgxDevModel* __restrict__ mdev, const PgxDevEnv& e,
                                          const PgxDevState& s, const float* __restrict__ action, const PgxDevOut& o) {
    /* WIDE: 0 one lane per env, 1 sixteen, 2 sixteen with the full manifold budget */
    constexpr int FULL = WIDE == 2 ? 1 : 0;
    using LT = ContactLdsT<WIDE ? EPW : 64, WIDE ? OBJ : 1, FULL>;
    /* the cache slots this layout uses (the rest stay empty: the reset kernel clears them) */
    constexpr int CACHE_K = 2 * (CG + LT::RB);
    const int ln = WIDE ? (int)threadIdx.x / GW : (int)threadIdx.x;   /* env slot in the wave (LDS index) */
    const int c = WIDE ? (int)threadIdx.x % GW : 0;                   /* lane within the env's row */
    const bool lead = c == 0;
    const int N = e.n_envs;
    /* heavy-first order (e.perm, pgx_launch_step): dispatch order = block order, so the blocks are
     * not dealt out per XCD there; an env's result does not depend on its wave mates */
    const int slot = ((e.perm && e.perm_segs == 1) ? (int)blockIdx.x : xcd_block()) * (WIDE ? EPW : 64) + ln;
    if (slot >= N) return;
    const int i = e.perm ? e.perm[slot] : slot;
#ifdef PGX_CHECK_PERM
    /* debug builds (make dbg DBG=-DPGX_CHECK_PERM): the heavy-first permutation is a bijection of
     * [0, N) (env_sort_scatter_kernel); an entry outside it would index every state row out of range */
    if ((unsigned)i >= (unsigned)N) {
        printf("pgx: perm[%d] = %d outside [0, %d)\n", slot, i, N);
        __builtin_trap();
    }
#endif
    /* the prologue loads index by a laundered copy of i: the compiler cannot reuse their
     * 64-bit addresses for the epilogue stores and keep ~17 address pairs live across the
     * whole step (recomputing them at the end is a few adds) */
    int ii = i;
    asm volatile("" : "+v"(ii));
    LT* L = nullptr;
    if constexpr (CONT) {
        __shared__ LT lds_buf;   /* one-lane: ~126 KB, one wave per CU; wide: ~9 KB */
        L = &lds_buf;
#ifdef PGX_LDS_POISON
        {
            float* w = reinterpret_cast<float*>(L);
            for (size_t t = threadIdx.x; t < sizeof(LT) / 4; t += blockDim.x) w[t] = __builtin_nanf("");
            __syncthreads();
        }
#endif
        /* every row slot starts finite: the sweeps run unused slots predicated off, and an
         * inactive slot later only holds an earlier substep's (finite) row */
#pragma unroll
        for (int k = 0; k < (WIDE ? 0 : CG); k++) {
#pragma unroll
            for (int qq = 0; qq < 4; qq++) L->g0q[k][qq][ln] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            L->g0n[k][0][ln] = 0.0f; L->g0n[k][1][ln] = 0.0f; L->g0n[k][2][ln] = 1.0f;
#pragma unroll
            for (int dir = 0; dir < 3; dir++)
#pragma unroll
                for (int qq = 0; qq < 6; qq++) L->g1q[k][dir][qq][ln] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        }
    }
#ifdef PGX_PROF
    if (threadIdx.x < PGX_PROF_N) g_prof[threadIdx.x] = 0;
    g_prof_t = __builtin_amdgcn_s_memtime();
    const unsigned long long prof_t0 = g_prof_t;
#endif
    const MPtr mp = model_ptr<AO>(mdev);   /* the compiled block == *mdev (pgx_create checks) */
    MRef m = *mp;
    float q[NJ], qd[NJ], tq[NJ];
#pragma unroll
    for (int j = 0; j < NJ; j++) {
        q[j] = s.q[j * N + ii];
        qd[j] = s.qd[j * N + ii];
    }
    ObjState ob;
    if (OBJ) load_obj(s, N, ii, ob);
    if (CONT) {
#pragma unroll
        for (int k = 0; k < CACHE_K; k++) L->cache[k][ln] = s.contacts[k * N + ii];
    }
    /* Bullet's persistent manifolds (the wide FULL kernels of the object tasks and ReachAO): the
     * pool, point p loaded by lane p of the env's row */
    constexpr bool PERS = WIDE == 2 && CONT && (OBJ || (AO && AO_PERS));
    if constexpr (PERS) {
        const int mc = (int)s.man[ii];
        L->mcnt[ln] = mc;
        if (c < mc) {
            const float* b = s.man + (size_t)(1 + PGX_MANIFOLD_POINT * c) * N + ii;
            L->mkid[c][ln] = b[0];
#pragma unroll
            for (int t = 0; t < 3; t++) {
                L->mla[c][t][ln] = b[(size_t)(1 + t) * N];
                L->mlb[c][t][ln] = b[(size_t)(4 + t) * N];
                L->mn[c][t][ln] = b[(size_t)(7 + t) * N];
            }
            L->md[c][ln] = b[(size_t)10 * N];
            L->mimp[c][ln] = b[(size_t)11 * N];
        }
    }
    if constexpr (AO) ao_load(s, N, ii, *L, ln);

    /* Panda.set_action: clip to Box(-1,1) in float32 */
    const int A = e.action_dim;
    if (CONTROL == 0) {
        float a[3];
#pragma unroll
        for (int c = 0; c < 3; c++) a[c] = fminf(fmaxf(action[(size_t)ii * A + c], -1.0f), 1.0f);
        /* get_ee_position() (panda.py:235) is getLinkState's cached pose (ee_state_cached) */
        float qcl[NJ];
#pragma unroll
        for (int j = 0; j < NJ; j++) qcl[j] = s.qc[j * N + ii];
        Chain k;
        fk_chain<WIDE != 0>(m, qcl, k);
        V3 pos = k.o[NJ - 1] + mulc(k.R[NJ - 1], kEeCom);
        V3 tgt = pos + v3(a[0] * m.ee_step, a[1] * m.ee_step, a[2] * m.ee_step);
        tgt.z = fmaxf(0.0f, tgt.z);
        const float torn[4] = {1.0f, 0.0f, 0.0f, 0.0f};
        ik<WIDE != 0>(mp, q, tgt, torn, tq);
        if constexpr (!WIDE) PGX_TRAP(0, 0, tq, NJ, m);
    } else {
#pragma unroll
        for (int j = 0; j < NJ; j++) {
            float a = fminf(fmaxf(action[(size_t)ii * A + j], -1.0f), 1.0f);
            tq[j] = q[j] + a * m.joint_step;
        }
    }

    PGX_PROF_MARK(0);
    LaneK lk;
    if constexpr (WIDE) lane_consts(lk);
    const int n_substeps = e.n_substeps;
    bool collided = false;
    /* the pose the last substep starts from: getLinkState's cached pose (defined before the loop:
     * with no substep it is the pose itself, and no path reads an uninitialised value -- the
     * round-4 runtime-model SLP build's non-finite outputs) */
    float qprev[NJ];
#pragma unroll
    for (int j = 0; j < NJ; j++) qprev[j] = q[j];
    /* PARK (wide layout with contacts, an LDS buffer): the motor targets and the substeps' start
     * poses wait in LDS (relaxed atomics: not promoted back into registers) -- ~14 registers
     * fewer across the substep loop, which the two-waves-per-SIMD kernels otherwise spill to
     * scratch and reload from memory in every substep */
    constexpr bool PARK = WIDE && CONT && (OBJ || AO || PART == 2);   /* (the headline kernel, one wave
                                                                      * and no spills: +0.4 %, not parked) */
    auto lds_st = [&](float* a, float v) __attribute__((always_inline)) { __hip_atomic_store(a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT); };
    auto lds_ld = [&](float* a) __attribute__((always_inline)) { return __hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT); };
    float* lkf = &lk.mass;   /* LaneK: 16 floats */
    static_assert(sizeof(LaneK) == 16 * sizeof(float), "LaneK layout");
    if constexpr (PARK) {
#pragma unroll
        for (int j = 0; j < NJ; j++) lds_st(&L->ltq[j][ln], tq[j]);
#pragma unroll
        for (int f = 0; f < 16; f++) lds_st(&L->lkc[f][c], lkf[f]);   /* (every env's lane c writes the same) */
    }
    int qslot = 0;   /* PARK: the buffer holding the last completed substep's start pose */
    for (int st = 0; st < n_substeps; st++) {
        float qstart[NJ];
        if constexpr (PARK) {
#pragma unroll
            for (int j = 0; j < NJ; j++) {
                lds_st(&L->lqs[st & 1][j][ln], q[j]);
                tq[j] = lds_ld(&L->ltq[j][ln]);
            }
#pragma unroll
            for (int f = 0; f < 16; f++) lkf[f] = lds_ld(&L->lkc[f][c]);
        } else {
#pragma unroll
            for (int j = 0; j < NJ; j++) qstart[j] = q[j];
        }
        if constexpr (WIDE) {
            /* ReachAO step_check_collision (reach_ao.py:182-188): the check after substep st - 1
             * runs inside substep st's contact detection (the same pose); a hit stops the loop
             * before anything of substep st happens */
            /* ReachAO (two waves per SIMD, 256 registers): the lane's row slot and lane index made opaque
             * in every substep, so what derives from them (LDS addresses, lane masks) is recomputed
             * there instead of hoisted out of the loop, spilled and reloaded in every substep
             * (scratch 632 -> 280 B per lane with the reset's inputs passed by value and the
             * collision check's table box opaque; PMC 93 -> 22 MB per ReachAO 8192 launch) */
            int cl = c, esl = ln;
            if constexpr (AO) asm volatile("" : "+v"(cl), "+v"(esl));
            if (substep_g<OBJ, CONT, PART, AO, FULL>(mp, e, q, qd, tq, ob, L, esl, cl, lk, AO && st > 0)) {
                collided = true;
                break;
            }
        } else {
            substep<OBJ, CONT, AO>(mp, e, q, qd, tq, ob, L, ln);
        }
        if constexpr (PARK) qslot = st & 1;
        else {
#pragma unroll
            for (int j = 0; j < NJ; j++) qprev[j] = qstart[j];
        }
        if constexpr (AO && !WIDE) {   /* ReachAO step_check_collision: check after every substep */
            ao_caps(*fresh(mp), q, *L, ln);
            if (ao_collided(e, *L, ln)) { collided = true; break; }
        }
    }
    if constexpr (AO && WIDE) {   /* the check after the last substep */
        if (!collided) {
            ao_caps(*fresh(mp), q, *L, ln);
            collided = ao_collided_g(e, *L, ln, c);
        }
    }

    if constexpr (PARK) {
#pragma unroll
        for (int j = 0; j < NJ; j++) qprev[j] = lds_ld(&L->lqs[qslot][j][ln]);
    }
    /* the env's row again after the substep loop, from the block and the lane (laundered) and the
     * heavy-first permutation (an atomic load, never merged with the prologue's): neither i nor
     * the prologue's row addresses stay live through the loop (ReachAO's two-wave kernel spilled
     * them to scratch, a dirty line per wave written back at every launch) */
    int ie = i;
    if constexpr (AO) {   /* (ReachAO only: the headline kernel measured +0.9 % with it, profiles/r06/ab_v19.log) */
        int lnx = ln;
        asm volatile("" : "+v"(lnx));
        const int sl = ((e.perm && e.perm_segs == 1) ? (int)blockIdx.x : xcd_block()) * (WIDE ? EPW : 64) + lnx;
        ie = e.perm ? __hip_atomic_load(&e.perm[sl], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : sl;
    }
    double goal[3];   /* read after the substep loop: not live across it */
#pragma unroll
    for (int c = 0; c < 3; c++) goal[c] = s.goal[c * N + (AO ? ie : ii)];
    V3 pos, vel;
    ee_state_cached(*fresh(mp), qprev, q, qd, pos, vel);
#ifdef PGX_NAN_TRAP
    if constexpr (!WIDE) {
        const float pv[6] = {pos.x, pos.y, pos.z, vel.x, vel.y, vel.z};
        PGX_TRAP(7, 0, pv, 6, m);
    }
#endif
    const int od = e.obs_dim;
    const V3 ag = OBJ ? ob.p : pos;
    double d = distance_f32_f64(ag, goal);
    bool succ = d < e.distance_threshold;
    float rew;
    if (AO) {   /* ReachAO.compute_reward sparse + collision_reward (reach_ao.py:1317-1320, 1376-1377) */
        rew = -1.0f + ((d + (collided ? 1.0 : 0.0)) < e.distance_threshold ? 1.0f : 0.0f);
        if (collided) rew += (float)e.collision_reward;
    } else {
        rew = e.reward == 0 ? -((d > e.distance_threshold) ? 1.0f : 0.0f) : -(float)d;
    }
    int el = s.elapsed[ie] + 1;
    uint32_t episode = s.episode[ie];
    /* TimeLimit, ReachAO.is_truncated (collision); terminate_on_success (core.py:359-361) */
    const bool trunc = (e.max_episode_steps > 0 && el >= e.max_episode_steps) || collided;
    const bool term = e.terminate_on_success && succ;
    if (lead) {
        if (o.reward) o.reward[ie] = rew;
        if (o.success) o.success[ie] = succ;
        if (o.terminated) o.terminated[ie] = term;
        if (o.truncated) o.truncated[ie] = trunc;
        if (o.task_truncated) o.task_truncated[ie] = collided;
    }
    if constexpr (AO) {
        if constexpr (WIDE) ao_link_obs_g(*L, ln, c);
        else ao_link_obs(*L, ln);
    }
    if (trunc || term) {
        if (o.terminal_obs && lead) {
            if constexpr (AO) ao_write_obs(o.terminal_obs + (size_t)ie * od, pos, vel, q, qd, *L, ln);
            else write_obs<OBJ>(e, o.terminal_obs + (size_t)ie * od, pos, vel, ob);
        }
        if (o.terminal_ag && lead) {
            o.terminal_ag[3 * (size_t)ie] = ag.x; o.terminal_ag[3 * (size_t)ie + 1] = ag.y;
            o.terminal_ag[3 * (size_t)ie + 2] = ag.z;
        }
        if (o.terminal_dg && lead) {
            o.terminal_dg[3 * (size_t)ie] = (float)goal[0]; o.terminal_dg[3 * (size_t)ie + 1] = (float)goal[1];
            o.terminal_dg[3 * (size_t)ie + 2] = (float)goal[2];
        }
    }
    /* SB3 VecEnv auto-reset of a finished env (off for a single gymnasium env: no_auto_reset) */
    if ((trunc || term) && !e.no_auto_reset) {
        if constexpr (AO) {
            MRef mr = *fresh(mp);
#pragma unroll
            for (int j = 0; j < NJ; j++) { q[j] = mr.neutral_q[j]; qd[j] = 0.0f; qprev[j] = q[j]; }
            ee_state(mr, q, qd, pos, vel);
            ao_caps(mr, q, *L, ln);
            uint64_t* rec = (e.pcg_on != nullptr && *e.pcg_on != 0) ? e.pcg + PGX_PCG64_WORDS * (size_t)ie : nullptr;
            const AoResetIn rin = ao_reset_in(e, pos);
            if (ao_reset<WIDE != 0>(rin, *L, ln, c, e.env_id_offset + (uint64_t)ie, episode, nullptr, nullptr, goal, rec,
                                    lead) &&
                lead)
                atomicOr(s.errors, PGX_ERR_AO_OBSTACLE);
            episode += 1;
            if constexpr (WIDE) ao_link_obs_g(*L, ln, c);
            else ao_link_obs(*L, ln);
        } else {
            reset_env<OBJ>(m, e, ie, episode, nullptr, nullptr, q, qd, goal, ob, lead);
            ee_state(m, q, qd, pos, vel);
#pragma unroll
            for (int j = 0; j < NJ; j++) qprev[j] = q[j];   /* resetJointState refreshes the link cache */
        }
        el = 0;
        if (CONT) {
#pragma unroll
            for (int k = 0; k < CACHE_K; k++) L->cache[k][ln] = (k & 1) ? 0.0f : -1.0f;
        }
        /* the reset teleports the bodies: Bullet's broadphase drops the pairs that no longer
         * overlap and the next refresh any other point (oracle pgxo_vec_step / reset) */
        if constexpr (PERS) L->mcnt[ln] = 0;
    }
    if constexpr (PERS) {   /* the pool back, point p by lane p */
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        const int mc = L->mcnt[ln];
        if (lead) s.man[ie] = (float)mc;
        if (c < mc) {
            float* b = s.man + (size_t)(1 + PGX_MANIFOLD_POINT * c) * N + ie;
            b[0] = L->mkid[c][ln];
#pragma unroll
            for (int t = 0; t < 3; t++) {
                b[(size_t)(1 + t) * N] = L->mla[c][t][ln];
                b[(size_t)(4 + t) * N] = L->mlb[c][t][ln];
                b[(size_t)(7 + t) * N] = L->mn[c][t][ln];
            }
            b[(size_t)10 * N] = L->md[c][ln];
            b[(size_t)11 * N] = L->mimp[c][ln];
        }
    }
    const V3 ag2 = OBJ ? ob.p : pos;
    if (!lead) return;
    if (o.obs) {
        if constexpr (AO) ao_write_obs(o.obs + (size_t)ie * od, pos, vel, q, qd, *L, ln);
        else write_obs<OBJ>(e, o.obs + (size_t)ie * od, pos, vel, ob);
    }
    if (o.ag) { o.ag[3 * (size_t)ie] = ag2.x; o.ag[3 * (size_t)ie + 1] = ag2.y; o.ag[3 * (size_t)ie + 2] = ag2.z; }
    if (o.dg) {
        o.dg[3 * (size_t)ie] = (float)goal[0]; o.dg[3 * (size_t)ie + 1] = (float)goal[1];
        o.dg[3 * (size_t)ie + 2] = (float)goal[2];
    }
#pragma unroll
    for (int j = 0; j < NJ; j++) {
        s.q[j * N + ie] = q[j];
        s.qd[j * N + ie] = qd[j];
        s.qc[j * N + ie] = qprev[j];
    }
#pragma unroll
    for (int c = 0; c < 3; c++) s.goal[c * N + ie] = goal[c];
    if (OBJ) store_obj(s, N, ie, ob);
    if constexpr (AO) ao_store(s, N, ie, *L, ln);
    if (CONT) {
#pragma unroll
        for (int k = 0; k < CACHE_K; k++) s.contacts[k * N + ie] = L->cache[k][ln];
    }
    s.elapsed[ie] = el;
    s.episode[ie] = episode;
#ifdef PGX_PROF
    PGX_PROF_MARK(6);
    if (threadIdx.x == 0) {
        for (int k = 0; k < PGX_PROF_N; k++) atomicAdd(&pgx_prof_counters[k], g_prof[k]);
        if (blockIdx.x < PGX_PROF_WAVES) {
            unsigned long long* w = pgx_prof_wave[blockIdx.x];
            w[0] = prof_t0; w[1] = g_prof_t; w[2] = g_prof[8]; w[3] = g_prof[10]; w[4] = g_prof[12]; w[5] = g_prof[13];
            w[6] = g_prof[7]; w[7] = g_prof[4]; w[8] = g_prof[1]; w[9] = g_prof[6];
        }
    }
#endif
}

/* the ReachAO step kernels take the table / plane geometry from the constant block (equal to the
 * env's, pgx_create): compile-time constants in the default build rather than kernel arguments the
 * register allocator holds in VGPRs through the substep loop (its two-wave kernel spilled three) */
template <int AO>
__device__ __forceinline__ void scene_from_model(PgxDevEnv& e, const PgxDevModel* mdev) {
    if constexpr (!AO) return;   /* (the arm / object kernels: +0.4 % on the headline, profiles/r06/ab_v19.log) */
    MRef m = *model_ptr<AO>(mdev);
    e.table_cx = m.table_cx; e.table_cy = m.table_cy; e.table_hx = m.table_hx; e.table_hy = m.table_hy;
    e.table_top = m.table_top; e.plane_z = m.plane_z; e.table_hz = m.table_hz;
}
/* The step kernel at one wave per SIMD (all of the register file: no spills; the batch
 * fills the chip only to one wave per SIMD, 4096 envs in the wide layout) and at two
 * (register budget 256, some spilled to scratch): beyond 1024 waves a second wave per
 * SIMD hides the first one's dependent latency -- ReachAO at 8192 envs 1.00 -> 0.78 ms,
 * Reach 1.11 -> 1.07 ms (joint-control Reach, fewer contacts, 0.57 -> 0.75: not used
 * there), while at 4096 envs the spills would cost 0.63 -> 0.89 ms. */
template <int CONTROL, int OBJ, int CONT, int AO, int WIDE>
__global__ __launch_bounds__(64) void step_kernel(const PgxDevModel* __restrict__ mdev, PgxDevEnv e, PgxDevState s,
                                                  const float* __restrict__ action, PgxDevOut o) {
    scene_from_model<AO>(e, mdev);
    step_body<CONTROL, OBJ, CONT, AO, WIDE>(mdev, e, s, action, o);
}
template <int CONTROL, int OBJ, int CONT, int AO, int WIDE>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2, 2))) void step_kernel_o2(
    const PgxDevModel* __restrict__ mdev, PgxDevEnv e, PgxDevState s, const float* __restrict__ action, PgxDevOut o) {
    scene_from_model<AO>(e, mdev);
    step_body<CONTROL, OBJ, CONT, AO, WIDE, AO ? 0 : 2>(mdev, e, s, action, o);
}

template <int OBJ, int AO>
__global__ __launch_bounds__(64) void reset_kernel(const PgxDevModel* __restrict__ mdev, PgxDevEnv e, PgxDevState s,
                                                   const uint8_t* mask, const double* inject_goal,
                                                   const double* inject_obj, PgxDevOut o) {
    const int ln = threadIdx.x;
    const int i = blockIdx.x * blockDim.x + ln;
    const int N = e.n_envs;
    if (i >= N) return;
    ContactLds* L = nullptr;
    if constexpr (AO) {
        __shared__ ContactLds lds_buf;
        L = &lds_buf;
    }
    MRef m = *model_ptr<AO>(mdev);
    if (mask && !mask[i]) return;
    float q[NJ], qd[NJ];
    double goal[3];
    ObjState ob;
    if (OBJ) load_obj(s, N, i, ob);
    uint32_t episode = s.episode[i];
    V3 pos, vel;
    if constexpr (AO) {
#pragma unroll
        for (int j = 0; j < NJ; j++) { q[j] = m.neutral_q[j]; qd[j] = 0.0f; }
        ee_state(m, q, qd, pos, vel);
        ao_caps(m, q, *L, ln);
        uint64_t* rec = (e.pcg_on != nullptr && *e.pcg_on != 0) ? e.pcg + PGX_PCG64_WORDS * (size_t)i : nullptr;
        const AoResetIn rin = ao_reset_in(e, pos);
        if (ao_reset<false>(rin, *L, ln, 0, e.env_id_offset + (uint64_t)i, episode,
                            inject_goal ? inject_goal + 3 * (size_t)i : nullptr,
                            inject_obj ? inject_obj + 3 * AO_N * (size_t)i : nullptr, goal, rec, true))
            atomicOr(s.errors, PGX_ERR_AO_OBSTACLE);
        episode += 1;
        ao_link_obs(*L, ln);
    } else {
        reset_env<OBJ>(m, e, i, episode, inject_goal ? inject_goal + 3 * (size_t)i : nullptr,
                       inject_obj ? inject_obj + 3 * (size_t)i : nullptr, q, qd, goal, ob);
        ee_state(m, q, qd, pos, vel);
    }
    const V3 ag = OBJ ? ob.p : pos;
    if (o.obs) {
        if constexpr (AO) ao_write_obs(o.obs + (size_t)i * e.obs_dim, pos, vel, q, qd, *L, ln);
        else write_obs<OBJ>(e, o.obs + (size_t)i * e.obs_dim, pos, vel, ob);
    }
    if (o.ag) { o.ag[3 * (size_t)i] = ag.x; o.ag[3 * (size_t)i + 1] = ag.y; o.ag[3 * (size_t)i + 2] = ag.z; }
    if (o.dg) {
        o.dg[3 * (size_t)i] = (float)goal[0]; o.dg[3 * (size_t)i + 1] = (float)goal[1];
        o.dg[3 * (size_t)i + 2] = (float)goal[2];
    }
    if (o.success) o.success[i] = distance_f32_f64(ag, goal) < e.distance_threshold;
#pragma unroll
    for (int j = 0; j < NJ; j++) {
        s.q[j * N + i] = q[j];
        s.qd[j * N + i] = qd[j];
        s.qc[j * N + i] = q[j];   /* resetJointState refreshes the link cache */
    }
#pragma unroll
    for (int c = 0; c < 3; c++) s.goal[c * N + i] = goal[c];
    if (OBJ) store_obj(s, N, i, ob);
    if constexpr (AO) ao_store(s, N, i, *L, ln);
#pragma unroll
    for (int k = 0; k < CACHE_N; k++) s.contacts[k * N + i] = (k & 1) ? 0.0f : -1.0f;
    if (s.man) s.man[i] = 0.0f;   /* the persistent manifold pool: empty after a reset */
    s.elapsed[i] = 0;
    s.episode[i] = episode;
}

__global__ __launch_bounds__(256) void sample_actions_kernel(PgxDevEnv e, float* action, uint64_t step) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= e.n_envs) return;
    const int A = e.action_dim;
    const uint64_t env = e.env_id_offset + (uint64_t)i;
    uint32_t o[4];
    for (int a = 0; a < A; a++) {
        if ((a & 3) == 0)
            philox((uint32_t)env, (uint32_t)(env >> 32), (uint32_t)step,
                   TAG_ACTION + ((uint32_t)(step >> 32) << 4) + (uint32_t)(a >> 2), (uint32_t)e.seed,
                   (uint32_t)(e.seed >> 32), o);
        uint32_t u = o[a & 3];
        action[(size_t)i * A + a] = (float)(u >> 8) * (1.0f / 16777216.0f) * 2.0f - 1.0f;
    }
}

__global__ __launch_bounds__(256) void compute_reward_kernel(const float* __restrict__ ag, const float* __restrict__ dg,
                                                             int64_t n, int32_t reward_type, float thr,
                                                             float* __restrict__ out) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        out[i] = reward_f32(distance_f32_f32(ag + 3 * i, dg + 3 * i), reward_type, thr);
    }
}

/* Heavy-first env order for the per-pair manifold kernels.  A wave costs what its heaviest env
 * costs (the robot-point rows past the register budget dominate), and when a
 * launch has more waves than the chip holds at once the dispatcher hands them out in block order:
 * grouping the envs by the robot contact points they held at the end of the previous step, most
 * first, puts the heavy envs into fewer waves and starts those first (longest-first scheduling).
 * Key = active robot slots of the warm-start cache.  A stable counting sort (13 bins, descending)
 * in two launches of 256-env blocks and no atomics (nothing to clear between launches): 1. each
 * block's keys and its per-bin counts; 2. each block sums the counts of the bins above and of the
 * blocks before it, ranks its envs inside each bin by ballot, and writes the permutation.  (Order
 * does not matter for the results -- the step kernels give every env the same bits whatever its
 * wave mates, test_gpu_env_order -- but a stable sort keeps every launch reproducible.) */
constexpr int SORT_BINS = PGX_ROBOT_POINTS + 1;
constexpr int SORT_BLOCK = 256;
__global__ __launch_bounds__(SORT_BLOCK) void env_sort_keys_kernel(PgxDevState s, int N, int rb, int all, uint8_t* keys,
                                                                   int32_t* blk) {
    __shared__ int32_t wc[SORT_BLOCK / 64][SORT_BINS];
    const int i = blockIdx.x * SORT_BLOCK + threadIdx.x, lane = (int)__lane_id(), w = (int)threadIdx.x / 64;
    int key = -1;
    if (i < N) {
        key = 0;
        for (int r = 0; r < rb; r++) key += s.contacts[(size_t)(CACHE1 + 2 * r) * N + i] >= 0.0f ? 1 : 0;
        if (!all) key = key > CG ? key - CG : 0;
        keys[i] = (uint8_t)key;
    }
    for (int k = 0; k < SORT_BINS; k++) {
        const int c = __popcll(__ballot(key == k));
        if (lane == 0) wc[w][k] = c;
    }
    __syncthreads();
    if (threadIdx.x < SORT_BINS) {
        int c = 0;
        for (int ww = 0; ww < SORT_BLOCK / 64; ww++) c += wc[ww][threadIdx.x];
        blk[(size_t)blockIdx.x * SORT_BINS + threadIdx.x] = c;
    }
}
__global__ __launch_bounds__(SORT_BLOCK) void env_sort_scatter_kernel(int N, const uint8_t* keys, const int32_t* blk,
                                                                      int32_t* perm, int segs) {
    __shared__ int32_t base[SORT_BINS];
    __shared__ int32_t wc[SORT_BLOCK / 64][SORT_BINS];
    /* segs > 1 (N a multiple of segs x SORT_BLOCK): the envs sort within segs equal contiguous
     * segments (segment x = the env range XCD x steps unsorted, xcd_block), each heavy-first */
    const int bps = (int)gridDim.x / segs, me = (int)blockIdx.x, sg = me / bps;
    const int b0 = sg * bps, nb = b0 + bps;
    const int i = me * SORT_BLOCK + threadIdx.x, lane = (int)__lane_id(), w = (int)threadIdx.x / 64;
    /* per bin: the total over all blocks and over the blocks before this one; thread t reads the
     * counts of blocks t, t + 256, ... (independent loads), then a wave and a block reduction */
    __shared__ int32_t red[SORT_BLOCK / 64][2][SORT_BINS];
    int tot[SORT_BINS], pre[SORT_BINS];
#pragma unroll
    for (int k = 0; k < SORT_BINS; k++) { tot[k] = 0; pre[k] = 0; }
    for (int bb = b0 + threadIdx.x; bb < nb; bb += SORT_BLOCK) {
#pragma unroll
        for (int k = 0; k < SORT_BINS; k++) {
            const int c = blk[(size_t)bb * SORT_BINS + k];
            tot[k] += c;
            pre[k] += bb < me ? c : 0;
        }
    }
#pragma unroll
    for (int k = 0; k < SORT_BINS; k++) {
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
            tot[k] += __shfl_xor(tot[k], d);
            pre[k] += __shfl_xor(pre[k], d);
        }
        if (lane == 0) { red[w][0][k] = tot[k]; red[w][1][k] = pre[k]; }
    }
    __syncthreads();
    if (threadIdx.x < SORT_BINS) {   /* bins above k in every block, then bin k in the blocks before */
        const int k = threadIdx.x;
        int off = 0;
        for (int kk = SORT_BINS - 1; kk > k; kk--)
            for (int ww = 0; ww < SORT_BLOCK / 64; ww++) off += red[ww][0][kk];
        for (int ww = 0; ww < SORT_BLOCK / 64; ww++) off += red[ww][1][k];
        base[k] = off + sg * (N / segs);
    }
    const int key = i < N ? (int)keys[i] : -1;
    uint64_t mine_k = 0ull;
    for (int k = 0; k < SORT_BINS; k++) {
        const uint64_t m = __ballot(key == k);
        if (key == k) mine_k = m;
        if (lane == 0) wc[w][k] = __popcll(m);
    }
    __syncthreads();
    if (key >= 0) {
        int r = base[key] + __popcll(mine_k & ((1ull << lane) - 1ull));
        for (int ww = 0; ww < w; ww++) r += wc[ww][key];
        perm[r] = i;
    }
}

/* The same order in one launch when a segment fits one workgroup (<= 1024 envs: every batch up to
 * 8192 in eight per-XCD segments, or up to 1024 in one): block x sorts segment x -- keys, per-wave
 * ballot counts in LDS, then each env's place -- instead of the two launches above (the headline's
 * 4096 envs: one ≈ 4 µs launch for two of 4.8 + 6.3 µs). */
constexpr int SORT_SEG_MAX = 1024;
__global__ __launch_bounds__(SORT_SEG_MAX) void env_sort_segment_kernel(PgxDevState s, int N, int rb, int all,
                                                                        int32_t* perm) {
    __shared__ int32_t wc[SORT_SEG_MAX / 64][SORT_BINS];
    __shared__ int32_t base[SORT_BINS];
    const int S = (int)blockDim.x, t = (int)threadIdx.x, lane = (int)__lane_id(), w = t / 64, nw = (S + 63) / 64;
    const int i = (int)blockIdx.x * S + t;   /* (the launcher gives S = N / segments: i < N) */
    int key = 0;
    for (int r = 0; r < rb; r++) key += s.contacts[(size_t)(CACHE1 + 2 * r) * N + i] >= 0.0f ? 1 : 0;
    if (!all) key = key > CG ? key - CG : 0;
    uint64_t mine_k = 0ull;
    for (int k = 0; k < SORT_BINS; k++) {
        const uint64_t m = __ballot(key == k);
        if (key == k) mine_k = m;
        if (lane == 0) wc[w][k] = __popcll(m);
    }
    __syncthreads();
    if (t < SORT_BINS) {   /* the segment's envs in the bins above k */
        int off = 0;
        for (int kk = SORT_BINS - 1; kk > t; kk--)
            for (int ww = 0; ww < nw; ww++) off += wc[ww][kk];
        base[t] = off;
    }
    __syncthreads();
    int r = base[key] + __popcll(mine_k & ((1ull << lane) - 1ull));
    for (int ww = 0; ww < w; ww++) r += wc[ww][key];
    perm[(int)blockIdx.x * S + r] = i;
}

}  // namespace

/* PGX_TU splits the library into translation units (Makefile): 1 holds the arm-only
 * step kernels (Reach, both control modes), compiled with SLP vectorisation -- packed
 * fp32 (v_pk_fma/add/mul_f32) in the redundant per-lane kinematics and dynamics, -2 % on the
 * headline kernel; 4 the ReachAO step kernels, with the scheduler's alternative register
 * pressure trackers (its two-wave build spills less: DESIGN.md section 4); 2 everything else,
 * compiled without SLP (the object tasks' register pressure turns the packed pairs into scratch
 * spills).  0 = one unit (the profiling build); 3 = no launcher (tools/ru_one.sh instantiates one
 * kernel for a register / scratch report). */
#ifndef PGX_TU
#define PGX_TU 0
#endif
/* every launch names its kernel (rocprof's spelling) in *name: the label bench.py reports */
#define PGX_KNAME(K, C, O, T, A, W) #K "<" #C ", " #O ", " #T ", " #A ", " #W ">"
#define PGX_STEP(C, O, K, A, W)                                                                   \
    do {                                                                                          \
        hipLaunchKernelGGL((step_kernel<C, O, K, A, W>), grid, block, 0, st, m, e, s, action, o); \
        if (name) *name = PGX_KNAME(step_kernel, C, O, K, A, W);                                  \
    } while (0)
#define PGX_STEP2(C, O, K, A, W)                                                                      \
    do {                                                                                              \
        if (two) {                                                                                    \
            hipLaunchKernelGGL((step_kernel_o2<C, O, K, A, W>), grid, block, 0, st, m, e, s, action, o); \
            if (name) *name = PGX_KNAME(step_kernel_o2, C, O, K, A, W);                                \
        } else {                                                                                      \
            PGX_STEP(C, O, K, A, W);                                                                  \
        }                                                                                             \
    } while (0)
#if PGX_TU != 3 && PGX_TU != 4
/* The heavy-first env order of the per-pair manifold launches (wide layout), from 256 waves (1024
 * envs) on.  Rounds 4-5 sorted only beyond the waves the chip holds at once (longest-first
 * scheduling); round 6 measured it faster at every batch from 1024 envs, the two sort kernels
 * (≈ 10 µs) included: Reach 4096 0.380 -> 0.369 ms, Reach 2048 0.376 -> 0.366, Reach 8192 0.587 ->
 * 0.566, Push 4096 0.935 -> 0.924, PickAndPlace 4096 0.933 -> 0.930, ReachAO 8192 0.514 -> 0.501
 * (profiles/r06/ab_*sort*.log).  A wave costs its heaviest env's rows times the most sweeps any of
 * its envs needs; envs of one weight sharing waves leave fewer waves that pay for both. */
constexpr unsigned kSortMinWaves = 256u;
/* the heavy-first env order (env_sort_keys_kernel / env_sort_scatter_kernel) into e.perm_buf;
 * returns the env the step launch reads (perm set) */
static PgxDevEnv sort_envs(const PgxDevEnv& e, const PgxDevState& s, hipStream_t st) {
    PgxDevEnv es = e;
    const int rb = e.has_object ? PGX_ROBOT_POINTS : PGX_ROBOT_POINTS_ARM;
    {   /* one launch when a segment fits a workgroup */
        const int segs = (e.sort_segs != 1 && e.n_envs % (8 * SORT_BLOCK) == 0) ? 8 : 1;
        const int S = e.n_envs / segs;
        if (S <= SORT_SEG_MAX && S > 0) {
            hipLaunchKernelGGL(env_sort_segment_kernel, dim3(segs), dim3(S), 0, st, s, e.n_envs, rb, e.sort_key,
                               e.perm_buf);
            es.perm = e.perm_buf;
            es.perm_segs = segs;
            return es;
        }
    }
    const int nb = (e.n_envs + SORT_BLOCK - 1) / SORT_BLOCK;
    uint8_t* keys = reinterpret_cast<uint8_t*>(e.perm_buf + e.n_envs);
    int32_t* blk = e.perm_buf + e.n_envs + (e.n_envs + 3) / 4;
    hipLaunchKernelGGL(env_sort_keys_kernel, dim3(nb), dim3(SORT_BLOCK), 0, st, s, e.n_envs, rb, e.sort_key, keys, blk);
    /* per-XCD segments when the batch divides: a wave's env rows then stay in one L2's range */
    const int segs = (e.sort_segs != 1 && e.n_envs % (8 * SORT_BLOCK) == 0) ? 8 : 1;
    hipLaunchKernelGGL(env_sort_scatter_kernel, dim3(nb), dim3(SORT_BLOCK), 0, st, e.n_envs, (const uint8_t*)keys,
                       (const int32_t*)blk, e.perm_buf, segs);
    es.perm = e.perm_buf;
    es.perm_segs = segs;
    return es;
}
#endif
#if PGX_TU == 4 || PGX_TU == 0
int pgx_launch_step_ao(const PgxDevModel* m, const PgxDevEnv& e, const PgxDevState& s, const float* action,
                       const PgxDevOut& o, void* stream, const char** name, bool two, bool wide) {
    hipStream_t st = (hipStream_t)stream;
    const int per_block = wide ? EPW : 64;
    dim3 block(64), grid((e.n_envs + per_block - 1) / per_block);
    if (wide && e.full_manifold) PGX_STEP2(1, 0, 1, 1, 2);
    else if (wide) PGX_STEP2(1, 0, 1, 1, 1);
    else PGX_STEP(1, 0, 1, 1, 0);
    return (int)hipGetLastError();
}
#endif
#if PGX_TU != 2 && PGX_TU != 3 && PGX_TU != 4
int pgx_launch_step_arm(const PgxDevModel* m, const PgxDevEnv& e, const PgxDevState& s, const float* action,
                        const PgxDevOut& o, void* stream, const char** name) {
    hipStream_t st = (hipStream_t)stream;
    const int wide = e.lanes_per_env == GW;
    const int per_block = wide ? EPW : 64;
    dim3 block(64), grid((e.n_envs + per_block - 1) / per_block);
    const bool two = e.wave_mode == 2 || (e.wave_mode == 0 && wide && grid.x > 1024);   /* more waves than SIMDs */
    if (wide && e.contacts && e.full_manifold) {   /* Bullet's per-pair manifolds (the default budget) */
        /* the heavy-first order from 1024 envs (kSortMinWaves), as the object / ReachAO launches */
        PgxDevEnv es = e;
        es.perm = nullptr;
        if (e.perm_buf && (e.sort_mode == 1 || (e.sort_mode == 0 && grid.x >= kSortMinWaves))) es = sort_envs(e, s, st);
        const PgxDevEnv& e = es;
        if (e.control) PGX_STEP(1, 0, 1, 0, 2);
        else PGX_STEP2(0, 0, 1, 0, 2);
        return (int)hipGetLastError();
    }
    switch ((e.control * 4 + (e.contacts ? 1 : 0)) * 2 + wide) {
        case 0: PGX_STEP(0, 0, 0, 0, 0); break;
        case 1: PGX_STEP(0, 0, 0, 0, 1); break;
        case 2: PGX_STEP(0, 0, 1, 0, 0); break;
        case 3: PGX_STEP2(0, 0, 1, 0, 1); break;
        case 8: PGX_STEP(1, 0, 0, 0, 0); break;
        case 9: PGX_STEP(1, 0, 0, 0, 1); break;
        case 10: PGX_STEP(1, 0, 1, 0, 0); break;
        case 11: PGX_STEP(1, 0, 1, 0, 1); break;   /* (joint-control Reach at 8192: 0.57 -> 0.75 ms with two) */
        default: return (int)hipErrorInvalidValue;
    }
    return (int)hipGetLastError();
}
#endif
#if PGX_TU != 1 && PGX_TU != 3 && PGX_TU != 4
int pgx_launch_step(const PgxDevModel* m, const PgxDevEnv& e, const PgxDevState& s, const float* action,
                    const PgxDevOut& o, void* stream, const char** name) {
    if (!e.ao && !e.has_object) return pgx_launch_step_arm(m, e, s, action, o, stream, name);
    hipStream_t st = (hipStream_t)stream;
    const int wide = e.lanes_per_env == GW;
    const int per_block = wide ? EPW : 64;
    dim3 block(64), grid((e.n_envs + per_block - 1) / per_block);
    const bool two = e.wave_mode == 2 || (e.wave_mode == 0 && wide && grid.x > 1024);   /* more waves than SIMDs */
    const int variant = e.control * 4 + (e.has_object ? 2 : 0) + (e.contacts ? 1 : 0);
    if (wide && e.full_manifold) {
        const bool sort = e.perm_buf && (e.sort_mode == 1 || (e.sort_mode == 0 && grid.x >= kSortMinWaves));
        PgxDevEnv es = e;
        es.perm = nullptr;
        if (sort) es = sort_envs(e, s, st);
        const PgxDevEnv& e = es;
        /* the object tasks' per-pair manifold kernels run one wave per SIMD at every batch: their
         * 32 KB of LDS per wave lets only 5 of the two-wave build's 8 waves per CU in, and at 256
         * registers it spills 676 B per lane (PickAndPlace 16384: 8.54 ms two-wave, 4.51 ms one
         * wave, profiles/r04/ab_full_waves_start.log) */
        if (e.ao) return pgx_launch_step_ao(m, e, s, action, o, stream, name, two, true);
        switch (variant) {
            case 3: PGX_STEP(0, 1, 1, 0, 2); break;
            case 7: PGX_STEP(1, 1, 1, 0, 2); break;
            default: return (int)hipErrorInvalidValue;
        }
        return (int)hipGetLastError();
    }
    if (e.ao) return pgx_launch_step_ao(m, e, s, action, o, stream, name, two, wide);
    switch (variant * 2 + wide) {
        case 6: PGX_STEP(0, 1, 1, 0, 0); break;
        case 7: PGX_STEP2(0, 1, 1, 0, 1); break;
        case 14: PGX_STEP(1, 1, 1, 0, 0); break;
        case 15: PGX_STEP2(1, 1, 1, 0, 1); break;
        default: return (int)hipErrorInvalidValue;   /* object without contacts: rejected at create */
    }
    return (int)hipGetLastError();
}

int pgx_launch_reset(const PgxDevModel* m, const PgxDevEnv& e, const PgxDevState& s, const uint8_t* mask,
                     const double* inject_goal, const double* inject_obj, const PgxDevOut& o, void* stream) {
    dim3 block(64), grid((e.n_envs + 63) / 64);
    if (e.ao)
        hipLaunchKernelGGL((reset_kernel<0, 1>), grid, block, 0, (hipStream_t)stream, m, e, s, mask, inject_goal, inject_obj, o);
    else if (e.has_object)
        hipLaunchKernelGGL((reset_kernel<1, 0>), grid, block, 0, (hipStream_t)stream, m, e, s, mask, inject_goal, inject_obj, o);
    else
        hipLaunchKernelGGL((reset_kernel<0, 0>), grid, block, 0, (hipStream_t)stream, m, e, s, mask, inject_goal, inject_obj, o);
    return (int)hipGetLastError();
}

int pgx_launch_sample_actions(const PgxDevEnv& e, float* action, uint64_t step, void* stream) {
    dim3 block(256), grid((e.n_envs + 255) / 256);
    hipLaunchKernelGGL(sample_actions_kernel, grid, block, 0, (hipStream_t)stream, e, action, step);
    return (int)hipGetLastError();
}

int pgx_launch_compute_reward(const float* ag, const float* dg, int64_t n, int32_t reward_type, double thr, float* out,
                              void* stream) {
    if (n <= 0) return 0;
    int64_t blocks = (n + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(compute_reward_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, ag, dg, n,
                       reward_type, (float)thr, out);
    return (int)hipGetLastError();
}
/* one device word written on the stream (the PCG64 mode word): a kernel node, not a memset node,
 * when a caller captures it -- a memset node of a graph destroyed after instantiation (torch's
 * default capture) replays garbage from its second launch on, DESIGN.md section 4 */
__global__ void set_word_kernel(int32_t* p, int32_t v) { *p = v; }
int pgx_launch_set_word(int32_t* p, int32_t v, void* stream) {
    hipLaunchKernelGGL(set_word_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, p, v);
    return (int)hipGetLastError();
}
#endif  /* PGX_TU 0 or 2 */
#undef PGX_STEP
#undef PGX_STEP2
#undef PGX_KNAME
