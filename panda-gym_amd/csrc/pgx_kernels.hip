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

#include "pgx_common.h"
#include "pgx_dev.h"
#include "pgx_model_consts.h"
#include "pgx_rows.h"

namespace {

constexpr int NJ = PGX_NJ;

/* The robot constants (PgxDevModel, ~1.4 KB) live in a device buffer read
 * through the constant address space, so every access is a scalar load
 * (s_load_dwordx16 into SGPRs).  `fresh()` hides the pointer behind an empty
 * asm at the top of each substep / IK iteration: the compiler then re-issues
 * the scalar loads where the values are used instead of hoisting ~350
 * constants out of the loops and spilling them to VGPR lanes (which cost one
 * v_readlane VALU instruction per use). */
typedef const __attribute__((address_space(4))) PgxDevModel* MPtr;
typedef const __attribute__((address_space(4))) PgxDevModel& MRef;
__device__ __forceinline__ MPtr fresh(uint64_t addr) {
    asm volatile("; pgx fresh model pointer %0" : "+s"(addr));
    return (MPtr)addr;
}
__device__ __forceinline__ MPtr fresh(MPtr p) { return fresh((uint64_t)p); }

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

__device__ __forceinline__ void fk_chain(MRef m, const float* q, Chain& k) {
    M3 PR = {{1, 0, 0, 0, 1, 0, 0, 0, 1}};
    V3 PO = v3(m.base[0], m.base[1], m.base[2]);
#pragma unroll
    for (int j = 0; j < NJ; j++) {
        M3 R = mulm(PR, kJr[j]);
        V3 o = PO + mulc(PR, kJp[j]);
        float s, c;
        joint_sincos(q[j], &s, &c);
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
__device__ __forceinline__ void ik(MPtr mp, const float* q0, V3 target, const float* torn, float* qout) {
    float qs[NJ];
#pragma unroll
    for (int j = 0; j < NJ; j++) qs[j] = q0[j];
    float diff = 1e30f;
    const int max_iters = mp->ik_max_iters;
    const float residual = mp->ik_residual;
    for (int it = 0; it < max_iters; it++) {
        if (!(diff > residual)) break;
        MRef m = *fresh(mp);
        Chain k;
        fk_chain(m, qs, k);
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
        V3 jv[NJ], jw[NJ];
#pragma unroll
        for (int j = 0; j < NJ; j++) {
            jw[j] = col(k.R[j], 2);
            jv[j] = cross(jw[j], x - k.o[j]);
        }
        float A[NJ][NJ], g[NJ], dth[NJ];
#pragma unroll
        for (int a = 0; a < NJ; a++) {
            g[a] = dot(jv[a], ep) + dot(jw[a], er);
#pragma unroll
            for (int b = 0; b <= a; b++) A[a][b] = dot(jv[a], jv[b]) + dot(jw[a], jw[b]);
            A[a][a] += m.ik_damping;
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
/* One Bullet stepSimulation() of the fixed-base arm (no contacts):
 *   qd_u = clamp(qd + dt * M^-1 (-b(q,qd)))          (ABA + applyDeltaVee)
 *   PGS over the motor/limit rows in Bullet's sorted order, reversed on even
 *   sweeps, early exit when max squared row residual <= residual_thr
 *   qd = clamp(qd_u + M^-1 J^T lambda); q += dt*qd   (constraint pass, stepPositions)
 * M by composite-rigid-body, b by Newton-Euler with Bullet's link damping. */
__device__ __forceinline__ void substep(MPtr mp, float* q, float* qd, const float* tq) {
    MRef m = *fresh(mp);
    /* FK fused with the per-link quantities the dynamics need, so the 3x3
     * rotations die immediately (only panda_link7's survives for its group). */
    V3 z[NJ], o[NJ], c[NJ];
    S3 Iw[NJ];
    M3 R6;
    {
        M3 PR = {{1, 0, 0, 0, 1, 0, 0, 0, 1}};
        V3 PO = v3(m.base[0], m.base[1], m.base[2]);
#pragma unroll
        for (int j = 0; j < NJ; j++) {
            M3 R = mulm(PR, kJr[j]);
            V3 oj = PO + mulc(PR, kJp[j]);
            float s, cs;
            joint_sincos(q[j], &s, &cs);
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
            PR = R;
            PO = oj;
        }
    }
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
    float vu[NJ];
    {
        float qdd[NJ];
        chol7_solve(Mt, nb, qdd);
#pragma unroll
        for (int j = 0; j < NJ; j++) vu[j] = fminf(fmaxf(qd[j] + m.dt * qdd[j], -m.max_vel), m.max_vel);
    }

    /* M^-1 = L^-T L^-1 (symmetric, lower triangle kept) */
    float Mi[NJ][NJ];
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
#define MINV(a, b) ((a) >= (b) ? Mi[a][b] : Mi[b][a])

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
     * and dropping them changes no bit of the result or of the exit iteration. */
    bool far = true;
#pragma unroll
    for (int d = 0; d < NJ; d++) {
        float B = 0.0f;
#pragma unroll
        for (int k = 0; k < NJ; k++) B += fabsf(MINV(d, k)) * m.max_impulse[k];
        B = B * 1.001f + 1e-6f;
        const float penl = q[d] - kLower[d], penu = kUpper[d] - q[d];
        far = far && penl > 0.0f && penu > 0.0f && (vu[d] - B) > -penl * m.inv_dt && (vu[d] + B) < penu * m.inv_dt;
    }
    float dv[NJ];
#pragma unroll
    for (int j = 0; j < NJ; j++) dv[j] = 0.0f;
    /* resolveSingleConstraintRowGeneric, branch-free: clamp the accumulated impulse,
     * apply the clamped delta through the unit response M^-1 J^T (a column of M^-1). */
    auto row = [&](const int r, float& resid) {
        const int kind = kPgxRowCode[r] >> 4, d = kPgxRowCode[r] & 15;
        const float lo = kind == 0 ? -m.max_impulse[d] : 0.0f;
        const float hi = kind == 0 ? m.max_impulse[d] : m.limit_max_imp;
        const float vd = kind == 2 ? -dv[d] : dv[d];
        float delta = rhs[r] - vd * jinv[d];
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
    if (__all(far)) {
        for (int it = 0; it < m.num_iterations; it++) {
            float resid = 0.0f;
            if (it & 1) {
#pragma unroll
                for (int r = 0; r < PGX_N_ROWS; r++)
                    if ((kPgxRowCode[r] >> 4) == 0) row(r, resid);
            } else {
#pragma unroll
                for (int r = PGX_N_ROWS - 1; r >= 0; r--)
                    if ((kPgxRowCode[r] >> 4) == 0) row(r, resid);
            }
            if (resid * resid <= m.residual_thr) break;
        }
    } else {
        init_limit_rows();
        for (int it = 0; it < m.num_iterations; it++) {
            float resid = 0.0f;
            if (it & 1) {
#pragma unroll
                for (int r = 0; r < PGX_N_ROWS; r++) row(r, resid);
            } else {
#pragma unroll
                for (int r = PGX_N_ROWS - 1; r >= 0; r--) row(r, resid);
            }
            if (resid * resid <= m.residual_thr) break;
        }
    }
#undef MINV
#pragma unroll
    for (int j = 0; j < NJ; j++) {
        float vn = fminf(fmaxf(vu[j] + dv[j], -m.max_vel), m.max_vel);
        qd[j] = vn;
        q[j] += m.dt * vn;
    }
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

/* -------------------------------------------------------------- RNG */
/* philox(): pgx_common.h */
constexpr uint32_t TAG_RESET = 0x52455345u;
constexpr uint32_t TAG_ACTION = 0x41435430u;

__device__ __forceinline__ double reset_uniform(const PgxDevEnv& e, uint64_t env, uint32_t episode, int kidx) {
    uint32_t o[4];
    philox((uint32_t)env, (uint32_t)(env >> 32), episode, TAG_RESET + (uint32_t)(kidx >> 1), (uint32_t)e.seed,
           (uint32_t)(e.seed >> 32), o);
    uint64_t u = (kidx & 1) ? ((uint64_t)o[2] | ((uint64_t)o[3] << 32)) : ((uint64_t)o[0] | ((uint64_t)o[1] << 32));
    return (double)(u >> 11) * (1.0 / 9007199254740992.0);
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
/* numpy Generator.uniform: low + (high - low) * u, unfused */
__device__ double uniform_draw(double low, double high, double u) {
    double r = high - low;
    double t = r * u;
    return low + t;
}
#pragma clang fp contract(on)

__device__ __forceinline__ void write_obs(const PgxDevEnv& e, float* dst, V3 pos, V3 vel) {
    dst[0] = pos.x; dst[1] = pos.y; dst[2] = pos.z;
    dst[3] = vel.x; dst[4] = vel.y; dst[5] = vel.z;
    if (!e.block_gripper) dst[6] = 0.0f; /* custom_0 fingers are fixed joints: width 0 */
}

__device__ __forceinline__ void reset_env(MRef m, const PgxDevEnv& e, int i, uint32_t& episode,
                                          const double* inject, float* q, float* qd, double* goal) {
#pragma unroll
    for (int j = 0; j < NJ; j++) { q[j] = m.neutral_q[j]; qd[j] = 0.0f; }
    uint64_t env = e.env_id_offset + (uint64_t)i;
#pragma unroll
    for (int c = 0; c < 3; c++)
        goal[c] = inject ? inject[c] : uniform_draw(e.goal_low[c], e.goal_high[c], reset_uniform(e, env, episode, c));
    episode += 1;
}

template <int CONTROL>
__global__ __launch_bounds__(64) void step_kernel(const PgxDevModel* __restrict__ mdev, PgxDevEnv e, PgxDevState s,
                                                  const float* __restrict__ action, PgxDevOut o) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int N = e.n_envs;
    if (i >= N) return;
    const MPtr mp = fresh((uint64_t)mdev);
    MRef m = *mp;
    float q[NJ], qd[NJ], tq[NJ];
#pragma unroll
    for (int j = 0; j < NJ; j++) {
        q[j] = s.q[j * N + i];
        qd[j] = s.qd[j * N + i];
    }
    double goal[3];
#pragma unroll
    for (int c = 0; c < 3; c++) goal[c] = s.goal[c * N + i];

    /* Panda.set_action: clip to Box(-1,1) in float32 */
    const int A = e.action_dim;
    if (CONTROL == 0) {
        float a[3];
#pragma unroll
        for (int c = 0; c < 3; c++) a[c] = fminf(fmaxf(action[(size_t)i * A + c], -1.0f), 1.0f);
        V3 pos, vel;
        Chain k;
        fk_chain(m, q, k);
        pos = k.o[NJ - 1] + mulc(k.R[NJ - 1], kEeCom);
        V3 tgt = pos + v3(a[0] * m.ee_step, a[1] * m.ee_step, a[2] * m.ee_step);
        tgt.z = fmaxf(0.0f, tgt.z);
        const float torn[4] = {1.0f, 0.0f, 0.0f, 0.0f};
        ik(mp, q, tgt, torn, tq);
        (void)vel;
    } else {
#pragma unroll
        for (int j = 0; j < NJ; j++) {
            float a = fminf(fmaxf(action[(size_t)i * A + j], -1.0f), 1.0f);
            tq[j] = q[j] + a * m.joint_step;
        }
    }

    const int n_substeps = m.n_substeps;
    for (int st = 0; st < n_substeps; st++) substep(mp, q, qd, tq);

    V3 pos, vel;
    ee_state(*fresh(mp), q, qd, pos, vel);
    const int od = e.obs_dim;
    double d = distance_f32_f64(pos, goal);
    bool succ = d < e.distance_threshold;
    float rew = e.reward == 0 ? -((d > e.distance_threshold) ? 1.0f : 0.0f) : -(float)d;
    int el = s.elapsed[i] + 1;
    uint32_t episode = s.episode[i];
    bool trunc = e.max_episode_steps > 0 && el >= e.max_episode_steps;
    if (o.reward) o.reward[i] = rew;
    if (o.success) o.success[i] = succ;
    if (o.terminated) o.terminated[i] = 0;
    if (o.truncated) o.truncated[i] = trunc;
    if (trunc) {
        if (o.terminal_obs) write_obs(e, o.terminal_obs + (size_t)i * od, pos, vel);
        if (o.terminal_ag) {
            o.terminal_ag[3 * (size_t)i] = pos.x; o.terminal_ag[3 * (size_t)i + 1] = pos.y;
            o.terminal_ag[3 * (size_t)i + 2] = pos.z;
        }
        if (o.terminal_dg) {
            o.terminal_dg[3 * (size_t)i] = (float)goal[0]; o.terminal_dg[3 * (size_t)i + 1] = (float)goal[1];
            o.terminal_dg[3 * (size_t)i + 2] = (float)goal[2];
        }
        reset_env(m, e, i, episode, nullptr, q, qd, goal);
        el = 0;
        ee_state(m, q, qd, pos, vel);
    }
    if (o.obs) write_obs(e, o.obs + (size_t)i * od, pos, vel);
    if (o.ag) { o.ag[3 * (size_t)i] = pos.x; o.ag[3 * (size_t)i + 1] = pos.y; o.ag[3 * (size_t)i + 2] = pos.z; }
    if (o.dg) {
        o.dg[3 * (size_t)i] = (float)goal[0]; o.dg[3 * (size_t)i + 1] = (float)goal[1];
        o.dg[3 * (size_t)i + 2] = (float)goal[2];
    }
#pragma unroll
    for (int j = 0; j < NJ; j++) {
        s.q[j * N + i] = q[j];
        s.qd[j * N + i] = qd[j];
    }
#pragma unroll
    for (int c = 0; c < 3; c++) s.goal[c * N + i] = goal[c];
    s.elapsed[i] = el;
    s.episode[i] = episode;
}

__global__ __launch_bounds__(64) void reset_kernel(const PgxDevModel* __restrict__ mdev, PgxDevEnv e, PgxDevState s,
                                                   const uint8_t* mask, const double* inject_goal, PgxDevOut o) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int N = e.n_envs;
    if (i >= N) return;
    MRef m = *fresh((uint64_t)mdev);
    if (mask && !mask[i]) return;
    float q[NJ], qd[NJ];
    double goal[3];
    uint32_t episode = s.episode[i];
    reset_env(m, e, i, episode, inject_goal ? inject_goal + 3 * (size_t)i : nullptr, q, qd, goal);
    V3 pos, vel;
    ee_state(m, q, qd, pos, vel);
    if (o.obs) write_obs(e, o.obs + (size_t)i * e.obs_dim, pos, vel);
    if (o.ag) { o.ag[3 * (size_t)i] = pos.x; o.ag[3 * (size_t)i + 1] = pos.y; o.ag[3 * (size_t)i + 2] = pos.z; }
    if (o.dg) {
        o.dg[3 * (size_t)i] = (float)goal[0]; o.dg[3 * (size_t)i + 1] = (float)goal[1];
        o.dg[3 * (size_t)i + 2] = (float)goal[2];
    }
    if (o.success) o.success[i] = distance_f32_f64(pos, goal) < e.distance_threshold;
#pragma unroll
    for (int j = 0; j < NJ; j++) {
        s.q[j * N + i] = q[j];
        s.qd[j * N + i] = qd[j];
    }
#pragma unroll
    for (int c = 0; c < 3; c++) s.goal[c * N + i] = goal[c];
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

}  // namespace

int pgx_launch_step(const PgxDevModel* m, const PgxDevEnv& e, const PgxDevState& s, const float* action,
                    const PgxDevOut& o, void* stream) {
    dim3 block(64), grid((e.n_envs + 63) / 64);
    hipStream_t st = (hipStream_t)stream;
    if (e.control == 0)
        hipLaunchKernelGGL(step_kernel<0>, grid, block, 0, st, m, e, s, action, o);
    else
        hipLaunchKernelGGL(step_kernel<1>, grid, block, 0, st, m, e, s, action, o);
    return (int)hipGetLastError();
}

int pgx_launch_reset(const PgxDevModel* m, const PgxDevEnv& e, const PgxDevState& s, const uint8_t* mask,
                     const double* inject_goal, const PgxDevOut& o, void* stream) {
    dim3 block(64), grid((e.n_envs + 63) / 64);
    hipLaunchKernelGGL(reset_kernel, grid, block, 0, (hipStream_t)stream, m, e, s, mask, inject_goal, o);
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
