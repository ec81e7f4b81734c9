/*
 * pgx_oracle.c -- TEST INFRASTRUCTURE ONLY (checker, never the measured path).
 *
 * fp64 CPU restatement of the reference's per-step hot path.  The reference's
 * arithmetic lives in pybullet 3.2.6 (Bullet3, requirements.txt:108), which is
 * not vendored and not installed here, so each function below restates the
 * published Bullet algorithm the reference's call sites rely on and names the
 * reference call site.  It is pinned against the reference's own known-answer
 * tests (test/pybullet_test.py:124-266, atol 1e-3) in tests/test_oracle_known_answers.py
 * and against golden vectors produced from the reference's numpy code
 * (panda_gym/utils.py) in tests/golden/.
 *
 * Deliberately written differently from the HIP kernel (generic tree, Jacobian-
 * based mass matrix and bias, fp64) so that parity is a real cross-check.
 */
#include "pgx_oracle.h"

#include <math.h>
#include <string.h>

#define L PGX_MAX_LINKS
#define D PGX_MAX_DOFS

/* phase marks for the operation-counting build (oracle/flops_count.cpp); no-ops here:
 * 0 action + IK, 1 contact detection, 2 dynamics (FK, M, bias, Cholesky, M^-1, free
 * velocities), 3 constraint-row setup, 4 PGS sweeps, 5 integration + contact cache,
 * 6 observation / success / reward, 7 reset (draws, rejection sampling, reset obs),
 * 8 ReachAO per-substep collision check */
#ifndef PGXO_PHASE
#define PGXO_PHASE(k) ((void)0)
#endif

/* ----------------------------------------------------------------- small vec */
/* diagnostics (tools/diag_iterations.py): histograms of PGS sweeps [0,64), contact
 * points per substep [64,80), IK iterations [80,112), substeps ending with a joint-limit
 * impulse [112], with robot contacts [113], both [114]; the persistent manifolds' branches:
 * a point dropped because the pool was full [120], addContactPoint merging into a cached point
 * (replaceContactPoint) [121], appending (addManifoldPoint) [122], replacing sortCachedPoints' slot
 * [123], refreshContactPoints removing a point past the threshold [124] or slid off [125]; not part
 * of the restatement */
int64_t pgxo_diag_hist[128];
/* the histograms are bumped with relaxed atomics: bench.py's cpu_baseline steps oracle shards in threads */
#define PGXO_HIST_ADD(h, i, v) __atomic_fetch_add(&(h)[(i)], (int64_t)(v), __ATOMIC_RELAXED)
void pgxo_diag_read(int64_t* out, int clear) {
    for (int i = 0; i < 128; i++)
        out[i] = clear ? __atomic_exchange_n(&pgxo_diag_hist[i], 0, __ATOMIC_RELAXED)
                       : __atomic_load_n(&pgxo_diag_hist[i], __ATOMIC_RELAXED);
}
/* optional trace of every solve's sweep count, in call order (env-major within a vec step) */
static int32_t* diag_trace;
static int64_t diag_trace_cap, diag_trace_pos;
void pgxo_diag_trace(int32_t* buf, int64_t cap) { diag_trace = buf; diag_trace_cap = cap; diag_trace_pos = 0; }
int64_t pgxo_diag_trace_len(void) { return diag_trace_pos; }

static void v3_cross(const double* a, const double* b, double* o) {
    double x = a[1] * b[2] - a[2] * b[1];
    double y = a[2] * b[0] - a[0] * b[2];
    double z = a[0] * b[1] - a[1] * b[0];
    o[0] = x; o[1] = y; o[2] = z;
}
static double v3_dot(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
static double v3_norm(const double* a) { return sqrt(v3_dot(a, a)); }
static void m3_mul(const double* A, const double* B, double* C) {
    double t[9];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++)
            t[i * 3 + j] = A[i * 3] * B[j] + A[i * 3 + 1] * B[3 + j] + A[i * 3 + 2] * B[6 + j];
    memcpy(C, t, sizeof t);
}
static void m3_v(const double* A, const double* v, double* o) {
    double x = A[0] * v[0] + A[1] * v[1] + A[2] * v[2];
    double y = A[3] * v[0] + A[4] * v[1] + A[5] * v[2];
    double z = A[6] * v[0] + A[7] * v[1] + A[8] * v[2];
    o[0] = x; o[1] = y; o[2] = z;
}
static void axis_angle(const double* ax, double ang, double* R) {
    double c = cos(ang), s = sin(ang), t = 1.0 - c;
    double x = ax[0], y = ax[1], z = ax[2];
    R[0] = t * x * x + c;     R[1] = t * x * y - s * z; R[2] = t * x * z + s * y;
    R[3] = t * x * y + s * z; R[4] = t * y * y + c;     R[5] = t * y * z - s * x;
    R[6] = t * x * z - s * y; R[7] = t * y * z + s * x; R[8] = t * z * z + c;
}

/* ------------------------------------------------------------- kinematics */
typedef struct {
    double R[L][9];   /* URDF link frame rotation (== COM frame rotation) */
    double o[L][3];   /* URDF link frame origin */
    double p[L][3];   /* COM (multibody link frame origin; getLinkState()[0]) */
    double z[L][3];   /* joint axis, world */
} kin_t;

/* Forward kinematics of the multibody (Bullet link order; links at COM).
 * Used by getLinkState (panda_gym/pybullet.py:249-273). */
static void fk(const pgx_model* m, const double* base, const double* q, kin_t* k) {
    for (int i = 0; i < m->n_links; i++) {
        int par = m->parent[i];
        double PR[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
        double PO[3] = {base[0], base[1], base[2]};
        if (par >= 0) {
            memcpy(PR, k->R[par], sizeof PR);
            memcpy(PO, k->o[par], sizeof PO);
        }
        double R[9], o[3];
        m3_mul(PR, m->jrot[i], R);
        m3_v(PR, m->jpos[i], o);
        o[0] += PO[0]; o[1] += PO[1]; o[2] += PO[2];
        m3_v(R, m->axis[i], k->z[i]);
        int d = m->dof_of_link[i];
        if (d >= 0 && m->jtype[i] == PGX_JOINT_REVOLUTE) {
            double Rq[9];
            axis_angle(m->axis[i], q[d], Rq);
            m3_mul(R, Rq, R);
        } else if (d >= 0 && m->jtype[i] == PGX_JOINT_PRISMATIC) {
            o[0] += k->z[i][0] * q[d]; o[1] += k->z[i][1] * q[d]; o[2] += k->z[i][2] * q[d];
        }
        memcpy(k->R[i], R, sizeof R);
        memcpy(k->o[i], o, sizeof o);
        double c[3];
        m3_v(R, m->com[i], c);
        k->p[i][0] = o[0] + c[0]; k->p[i][1] = o[1] + c[1]; k->p[i][2] = o[2] + c[2];
    }
}

void pgxo_fk(const pgx_model* m, const double base[3], const double* q, double* com_pos, double* rot,
             double* origin) {
    kin_t k;
    fk(m, base, q, &k);
    for (int i = 0; i < m->n_links; i++) {
        if (com_pos) memcpy(com_pos + 3 * i, k.p[i], 3 * sizeof(double));
        if (rot) memcpy(rot + 9 * i, k.R[i], 9 * sizeof(double));
        if (origin) memcpy(origin + 3 * i, k.o[i], 3 * sizeof(double));
    }
}

/* is dof d an ancestor-or-self joint of link i */
static int on_path(const pgx_model* m, int i, int d) {
    int lk = m->link_of_dof[d];
    for (int j = i; j >= 0; j = m->parent[j])
        if (j == lk) return 1;
    return 0;
}

/* Jacobian (world) of point x rigidly attached to link i: Jv[3][nd], Jw[3][nd] */
static void jacobian(const pgx_model* m, const kin_t* k, int i, const double* x, double* Jv, double* Jw) {
    int nd = m->n_dofs;
    for (int d = 0; d < nd; d++) {
        double cv[3] = {0, 0, 0}, cw[3] = {0, 0, 0};
        if (on_path(m, i, d)) {
            int lk = m->link_of_dof[d];
            if (m->jtype[lk] == PGX_JOINT_REVOLUTE) {
                double r[3] = {x[0] - k->o[lk][0], x[1] - k->o[lk][1], x[2] - k->o[lk][2]};
                v3_cross(k->z[lk], r, cv);
                memcpy(cw, k->z[lk], sizeof cw);
            } else {
                memcpy(cv, k->z[lk], sizeof cv);
            }
        }
        for (int r = 0; r < 3; r++) {
            Jv[r * nd + d] = cv[r];
            Jw[r * nd + d] = cw[r];
        }
    }
}

/* world inertia R diag(I) R^T */
static void world_inertia(const double* R, const double* I, double* Iw) {
    for (int a = 0; a < 3; a++)
        for (int b = 0; b < 3; b++)
            Iw[a * 3 + b] = R[a * 3] * I[0] * R[b * 3] + R[a * 3 + 1] * I[1] * R[b * 3 + 1] +
                            R[a * 3 + 2] * I[2] * R[b * 3 + 2];
}

/* COM link velocities: compTreeLinkVelocities as used by getLinkState(computeLinkVelocity=1)
 * (panda_gym/pybullet.py:275-299). */
static void link_vel(const pgx_model* m, const kin_t* k, const double* qd, int i, double* v, double* w) {
    double Jv[3 * D], Jw[3 * D];
    jacobian(m, k, i, k->p[i], Jv, Jw);
    int nd = m->n_dofs;
    for (int r = 0; r < 3; r++) {
        v[r] = 0; w[r] = 0;
        for (int d = 0; d < nd; d++) {
            v[r] += Jv[r * nd + d] * qd[d];
            w[r] += Jw[r * nd + d] * qd[d];
        }
    }
}

void pgxo_link_velocity(const pgx_model* m, const double base[3], const double* q, const double* qd, int link,
                        double lin[3], double ang[3]) {
    kin_t k;
    fk(m, base, q, &k);
    link_vel(m, &k, qd, link, lin, ang);
}

/* --------------------------------------------------------------- dynamics */
/* Joint-space inertia sum_i m J_v^T J_v + J_w^T I_w J_w: the matrix Bullet's
 * ABA (btMultiBody::computeAccelerationsArticulatedBodyAlgorithmMultiDof)
 * inverts implicitly. */
static void mass_matrix(const pgx_model* m, const kin_t* k, double* M) {
    int nd = m->n_dofs;
    memset(M, 0, sizeof(double) * nd * nd);
    for (int i = 0; i < m->n_links; i++) {
        if (m->mass[i] == 0.0) continue;
        double Jv[3 * D], Jw[3 * D], Iw[9];
        jacobian(m, k, i, k->p[i], Jv, Jw);
        world_inertia(k->R[i], m->inertia[i], Iw);
        for (int a = 0; a < nd; a++)
            for (int b = 0; b < nd; b++) {
                double s = 0;
                for (int r = 0; r < 3; r++) s += m->mass[i] * Jv[r * nd + a] * Jv[r * nd + b];
                for (int r = 0; r < 3; r++)
                    for (int c = 0; c < 3; c++) s += Jw[r * nd + a] * Iw[r * 3 + c] * Jw[c * nd + b];
                M[a * nd + b] += s;
            }
    }
}

void pgxo_mass_matrix(const pgx_model* m, const double base[3], const double* q, double* M) {
    kin_t k;
    fk(m, base, q, &k);
    mass_matrix(m, &k, M);
}

/* Generalised bias b(q,qd): Coriolis/centrifugal + gyroscopic + Bullet's link
 * damping m*v*(k1+k2|v|), I*w*(k1+k2|w|) (btMultiBody DAMPING_K1/K2 = 0.04)
 * - gravity (btMultiBodyDynamicsWorld adds m*g to every link).  qdd = -M^-1 b. */
static void bias(const pgx_model* m, const pgx_sim_params* p, const kin_t* k, const double* qd, int with_gravity,
                 int with_velocity, double* b) {
    double w[L][3], al[L][3], v[L][3], acc[L][3];
    int nd = m->n_dofs;
    for (int d = 0; d < nd; d++) b[d] = 0;
    for (int i = 0; i < m->n_links; i++) {
        int par = m->parent[i];
        double wp[3] = {0, 0, 0}, alp[3] = {0, 0, 0}, vp[3] = {0, 0, 0}, ap[3] = {0, 0, 0}, pp[3];
        if (par >= 0) {
            memcpy(wp, w[par], sizeof wp); memcpy(alp, al[par], sizeof alp);
            memcpy(vp, v[par], sizeof vp); memcpy(ap, acc[par], sizeof ap);
            memcpy(pp, k->p[par], sizeof pp);
        } else {
            memcpy(pp, k->o[i], sizeof pp);
        }
        double r[3] = {k->o[i][0] - pp[0], k->o[i][1] - pp[1], k->o[i][2] - pp[2]};
        double vo[3], ao[3], t1[3], t2[3];
        v3_cross(wp, r, t1);
        for (int c = 0; c < 3; c++) vo[c] = vp[c] + t1[c];
        v3_cross(alp, r, t1);
        v3_cross(wp, r, t2);
        v3_cross(wp, t2, t2);
        for (int c = 0; c < 3; c++) ao[c] = ap[c] + t1[c] + t2[c];
        int d = m->dof_of_link[i];
        double qdi = (d >= 0 && with_velocity) ? qd[d] : 0.0;
        double sz[3] = {k->z[i][0] * qdi, k->z[i][1] * qdi, k->z[i][2] * qdi};
        memcpy(w[i], wp, sizeof wp);
        memcpy(al[i], alp, sizeof alp);
        if (d >= 0 && m->jtype[i] == PGX_JOINT_REVOLUTE) {
            for (int c = 0; c < 3; c++) w[i][c] += sz[c];
            v3_cross(wp, sz, t1);
            for (int c = 0; c < 3; c++) al[i][c] += t1[c];
        } else if (d >= 0 && m->jtype[i] == PGX_JOINT_PRISMATIC) {
            v3_cross(wp, sz, t1);
            for (int c = 0; c < 3; c++) { vo[c] += sz[c]; ao[c] += 2.0 * t1[c]; }
        }
        double rc[3] = {k->p[i][0] - k->o[i][0], k->p[i][1] - k->o[i][1], k->p[i][2] - k->o[i][2]};
        v3_cross(w[i], rc, t1);
        for (int c = 0; c < 3; c++) v[i][c] = vo[c] + t1[c];
        v3_cross(al[i], rc, t1);
        v3_cross(w[i], rc, t2);
        v3_cross(w[i], t2, t2);
        for (int c = 0; c < 3; c++) acc[i][c] = ao[c] + t1[c] + t2[c];
    }
    for (int i = 0; i < m->n_links; i++) {
        double mi = m->mass[i];
        if (mi == 0.0) continue;
        double F[3], T[3], Iw[9], Iww[3], Ial[3], t1[3];
        double vn = v3_norm(v[i]), wn = v3_norm(w[i]);
        for (int c = 0; c < 3; c++) {
            F[c] = mi * acc[i][c];
            if (with_gravity) F[c] -= mi * p->gravity[c];
            F[c] += mi * v[i][c] * (p->lin_damping + p->lin_damping * vn);
        }
        world_inertia(k->R[i], m->inertia[i], Iw);
        m3_v(Iw, w[i], Iww);
        m3_v(Iw, al[i], Ial);
        v3_cross(w[i], Iww, t1);
        for (int c = 0; c < 3; c++) T[c] = Ial[c] + t1[c] + Iww[c] * (p->ang_damping + p->ang_damping * wn);
        double Jv[3 * D], Jw[3 * D];
        jacobian(m, k, i, k->p[i], Jv, Jw);
        for (int dd = 0; dd < nd; dd++)
            for (int r = 0; r < 3; r++) b[dd] += Jv[r * nd + dd] * F[r] + Jw[r * nd + dd] * T[r];
    }
}

void pgxo_bias(const pgx_model* m, const pgx_sim_params* p, const double base[3], const double* q,
               const double* qd, int with_gravity, double* b) {
    kin_t k;
    fk(m, base, q, &k);
    bias(m, p, &k, qd, with_gravity, 1, b);
}

/* The same M and b in the recursive form the HIP kernel computes them in (composite rigid
 * bodies for M, Newton-Euler for b; SURVEY.md section 8d's "CRBA + RNEA + 7x7 Cholesky"), for the
 * operation count of that formulation (oracle flag PGX_FLAG_DYN_RECURSIVE, oracle/count_flops.py
 * key "recursive"); equal to mass_matrix / bias to rounding (tests/test_flops.py).  Links are in
 * Bullet order, parents first.
 *   b: forward pass as bias() (velocities / accelerations at the COM with qdd = 0), per link
 *      the wrench at its COM (F, T), then one backward pass accumulating the subtree's force Fs
 *      and moment Ns about the link's pivot: b_d = z . Ns of the dof's link.
 *   M: backward pass of the subtree's mass Mc, first moment H = sum m p and inertia about the
 *      world origin Io; spun about z_j through o_j the composite has momentum f = z_j x (H - Mc o_j)
 *      and angular momentum about o_j n = Io z_j - o_j x (H x z_j) ... written as below; then
 *      M[i][j] = z_i . (n + (o_j - o_i) x f) for every dof i on the path to the root. */
static void dyn_recursive(const pgx_model* m, const pgx_sim_params* p, const kin_t* k, const double* qd,
                          int with_gravity, double* M, double* b) {
    const int nl = m->n_links, nd = m->n_dofs;
    double w[L][3], al[L][3], v[L][3], acc[L][3];
    for (int i = 0; i < nl; i++) {   /* forward: as bias() */
        int par = m->parent[i];
        double wp[3] = {0, 0, 0}, alp[3] = {0, 0, 0}, vp[3] = {0, 0, 0}, ap[3] = {0, 0, 0}, pp[3];
        if (par >= 0) {
            memcpy(wp, w[par], sizeof wp); memcpy(alp, al[par], sizeof alp);
            memcpy(vp, v[par], sizeof vp); memcpy(ap, acc[par], sizeof ap);
            memcpy(pp, k->p[par], sizeof pp);
        } else {
            memcpy(pp, k->o[i], sizeof pp);
        }
        double r[3] = {k->o[i][0] - pp[0], k->o[i][1] - pp[1], k->o[i][2] - pp[2]};
        double vo[3], ao[3], t1[3], t2[3];
        v3_cross(wp, r, t1);
        for (int c = 0; c < 3; c++) vo[c] = vp[c] + t1[c];
        v3_cross(alp, r, t1);
        v3_cross(wp, r, t2);
        v3_cross(wp, t2, t2);
        for (int c = 0; c < 3; c++) ao[c] = ap[c] + t1[c] + t2[c];
        int d = m->dof_of_link[i];
        double qdi = d >= 0 ? qd[d] : 0.0;
        double sz[3] = {k->z[i][0] * qdi, k->z[i][1] * qdi, k->z[i][2] * qdi};
        memcpy(w[i], wp, sizeof wp);
        memcpy(al[i], alp, sizeof alp);
        if (d >= 0 && m->jtype[i] == PGX_JOINT_REVOLUTE) {
            for (int c = 0; c < 3; c++) w[i][c] += sz[c];
            v3_cross(wp, sz, t1);
            for (int c = 0; c < 3; c++) al[i][c] += t1[c];
        } else if (d >= 0 && m->jtype[i] == PGX_JOINT_PRISMATIC) {
            v3_cross(wp, sz, t1);
            for (int c = 0; c < 3; c++) { vo[c] += sz[c]; ao[c] += 2.0 * t1[c]; }
        }
        double rc[3] = {k->p[i][0] - k->o[i][0], k->p[i][1] - k->o[i][1], k->p[i][2] - k->o[i][2]};
        v3_cross(w[i], rc, t1);
        for (int c = 0; c < 3; c++) v[i][c] = vo[c] + t1[c];
        v3_cross(al[i], rc, t1);
        v3_cross(w[i], rc, t2);
        v3_cross(w[i], t2, t2);
        for (int c = 0; c < 3; c++) acc[i][c] = ao[c] + t1[c] + t2[c];
    }
    /* backward: subtree force Fs and moment Ns about the pivot o_i; composite Mc, H, Io */
    double Fs[L][3], Ns[L][3], Mc[L], H[L][3], Io[L][9];
    for (int i = 0; i < nl; i++) {
        Mc[i] = 0.0;
        for (int c = 0; c < 3; c++) { Fs[i][c] = 0.0; Ns[i][c] = 0.0; H[i][c] = 0.0; }
        for (int c = 0; c < 9; c++) Io[i][c] = 0.0;
    }
    for (int i = nl - 1; i >= 0; i--) {
        const double mi = m->mass[i];
        if (mi != 0.0) {
            double F[3], T[3], Iw[9], Iww[3], Ial[3], t1[3], rc[3];
            double vn = v3_norm(v[i]), wn = v3_norm(w[i]);
            for (int c = 0; c < 3; c++) {
                F[c] = mi * acc[i][c];
                if (with_gravity) F[c] -= mi * p->gravity[c];
                F[c] += mi * v[i][c] * (p->lin_damping + p->lin_damping * vn);
            }
            world_inertia(k->R[i], m->inertia[i], Iw);
            m3_v(Iw, w[i], Iww);
            m3_v(Iw, al[i], Ial);
            v3_cross(w[i], Iww, t1);
            for (int c = 0; c < 3; c++) T[c] = Ial[c] + t1[c] + Iww[c] * (p->ang_damping + p->ang_damping * wn);
            for (int c = 0; c < 3; c++) rc[c] = k->p[i][c] - k->o[i][c];
            v3_cross(rc, F, t1);
            for (int c = 0; c < 3; c++) { Fs[i][c] += F[c]; Ns[i][c] += T[c] + t1[c]; }
            /* composite: mass, first moment, inertia about the world origin (Steiner) */
            const double* pc = k->p[i];
            const double pp = v3_dot(pc, pc);
            Mc[i] += mi;
            for (int c = 0; c < 3; c++) H[i][c] += mi * pc[c];
            for (int a = 0; a < 3; a++)
                for (int c = 0; c < 3; c++) Io[i][a * 3 + c] += Iw[a * 3 + c] + mi * ((a == c ? pp : 0.0) - pc[a] * pc[c]);
        }
        const int par = m->parent[i];
        if (par >= 0) {   /* hand the subtree to the parent: the moment moves from o_i to o_par */
            double r[3] = {k->o[i][0] - k->o[par][0], k->o[i][1] - k->o[par][1], k->o[i][2] - k->o[par][2]}, t1[3];
            v3_cross(r, Fs[i], t1);
            for (int c = 0; c < 3; c++) { Fs[par][c] += Fs[i][c]; Ns[par][c] += Ns[i][c] + t1[c]; H[par][c] += H[i][c]; }
            Mc[par] += Mc[i];
            for (int c = 0; c < 9; c++) Io[par][c] += Io[i][c];
        }
    }
    for (int d = 0; d < nd; d++) {
        const int i = m->link_of_dof[d];
        b[d] = m->jtype[i] == PGX_JOINT_REVOLUTE ? v3_dot(k->z[i], Ns[i]) : v3_dot(k->z[i], Fs[i]);
    }
    /* M by composite rigid bodies (revolute dofs; a prismatic dof's column is f alone) */
    memset(M, 0, sizeof(double) * nd * nd);
    for (int dj = 0; dj < nd; dj++) {
        const int j = m->link_of_dof[dj];
        const double* z = k->z[j];
        const double* o = k->o[j];
        double f[3], n[3], t1[3], t2[3];
        if (m->jtype[j] == PGX_JOINT_REVOLUTE) {
            /* f = z x (H - Mc o); angular momentum about o: Io z - o x (z x H) - H x (z x o)
             *   + Mc o x (z x o)  (the composite's inertia moved from the origin to o) */
            double hm[3] = {H[j][0] - Mc[j] * o[0], H[j][1] - Mc[j] * o[1], H[j][2] - Mc[j] * o[2]};
            v3_cross(z, hm, f);
            m3_v(Io[j], z, n);
            double zh[3], zo[3];
            v3_cross(z, H[j], zh);
            v3_cross(z, o, zo);
            v3_cross(o, zh, t1);
            v3_cross(H[j], zo, t2);
            double t3[3];
            v3_cross(o, zo, t3);
            for (int c = 0; c < 3; c++) n[c] = n[c] - t1[c] - t2[c] + Mc[j] * t3[c];
        } else {
            for (int c = 0; c < 3; c++) { f[c] = Mc[j] * z[c]; n[c] = 0.0; }
            double t3[3];
            v3_cross(H[j], z, t3);   /* moment about o of the translating composite: (c - o) x Mc z */
            v3_cross(o, f, t1);
            for (int c = 0; c < 3; c++) n[c] = t3[c] - t1[c];
        }
        /* up the chain: dof i on the path from link j to the root */
        for (int a = j; a >= 0; a = m->parent[a]) {
            const int di = m->dof_of_link[a];
            if (di < 0) continue;
            double r[3] = {o[0] - k->o[a][0], o[1] - k->o[a][1], o[2] - k->o[a][2]};
            v3_cross(r, f, t1);
            double val = m->jtype[a] == PGX_JOINT_REVOLUTE
                             ? k->z[a][0] * (n[0] + t1[0]) + k->z[a][1] * (n[1] + t1[1]) + k->z[a][2] * (n[2] + t1[2])
                             : v3_dot(k->z[a], f);
            M[di * nd + dj] = val;
            M[dj * nd + di] = val;
        }
    }
}

void pgxo_dyn_recursive(const pgx_model* m, const pgx_sim_params* p, const double base[3], const double* q,
                        const double* qd, int with_gravity, double* M, double* b) {
    kin_t k;
    fk(m, base, q, &k);
    dyn_recursive(m, p, &k, qd, with_gravity, M, b);
}

/* SPD solve / inverse via Cholesky (fp64) */
static int chol(int n, const double* A, double* Lm) {
    for (int i = 0; i < n; i++)
        for (int j = 0; j <= i; j++) {
            double s = A[i * n + j];
            for (int kk = 0; kk < j; kk++) s -= Lm[i * n + kk] * Lm[j * n + kk];
            if (i == j) {
                if (s <= 0) return -1;
                Lm[i * n + i] = sqrt(s);
            } else {
                Lm[i * n + j] = s / Lm[j * n + j];
            }
        }
    return 0;
}
static void chol_solve(int n, const double* Lm, const double* b, double* x) {
    double y[D * 2];
    for (int i = 0; i < n; i++) {
        double s = b[i];
        for (int kk = 0; kk < i; kk++) s -= Lm[i * n + kk] * y[kk];
        y[i] = s / Lm[i * n + i];
    }
    for (int i = n - 1; i >= 0; i--) {
        double s = y[i];
        for (int kk = i + 1; kk < n; kk++) s -= Lm[kk * n + i] * x[kk];
        x[i] = s / Lm[i * n + i];
    }
}

static double clampd(double x, double lo, double hi) { return x < lo ? lo : (x > hi ? hi : x); }

/* ======================================================= world: object + contacts
 * The scene of Reach/Push/PickAndPlace (Task._create_scene, push.py:31-47;
 * PyBullet.create_table / create_plane pybullet.py:759-817): a static table box
 * (top z = 0), a static plane box (top z = -0.4) and, for Push/PickAndPlace, a
 * free 4 cm cube (a zero-link btMultiBody with a floating base).
 *
 * Contacts restated from Bullet 3.2.x (btMultiBodyDynamicsWorld +
 * btMultiBodyConstraintSolver) -- unpinned: no known answer exists:
 *  - detection at the start of the step, points with separation < contact_distance
 *    (0.02, speculative); Bullet's manifold rule: one btPersistentManifold of at most
 *    MANIFOLD_CACHE_SIZE = 4 points per colliding pair (a capsule -- a child shape of its
 *    link's compound, btCompoundCollisionAlgorithm keeps a manifold per child -- against
 *    the table, the plane, the cube or an obstacle; the cube against the table or the
 *    plane), restated as the pair's 4 deepest candidates; then an explicit per-env row
 *    budget per group (object vs table/plane: PGX_OBJECT_POINTS, robot vs anything:
 *    robot_budget, the kernel's PGX_ROBOT_POINTS unless a test sets it), the deepest
 *    first; depth ties: discovery order (capsule, then ends / samples / obstacles), as
 *    the kernel ranks; rows ordered by feature id.  Features with a fixed identity (cube
 *    vertex, capsule end, capsule sample sphere, capsule x obstacle) carry the normal
 *    impulse to the next step (warm start x 0.85) like a manifold point does;
 *  - cube vs table / plane: cube vertices against the top face of the box under them;
 *    robot capsules (model.capsules) vs table / plane: the end spheres; robot capsules
 *    vs cube: spheres sampled along the capsule axis at <= r/2 spacing vs the box;
 *  - rows per point: normal (impulse >= 0; rhs from ERP 0.2 when penetrating, from
 *    -distance/dt when separated), two friction rows along btPlaneSpace1(normal) with
 *    |impulse| <= mu * normal impulse (mu: the two bodies' lateral frictions multiplied, 0.5 * 0.5,
 *    but 1.0 * 0.5 for panda_ee's capsules -- panda.py:69-70); solved after the joint rows in
 *    every sweep (normal rows, then friction rows; a friction row is skipped while its
 *    normal impulse is 0), same residual exit;
 *  - body A is the robot (or the cube against the table), B the table (or the cube):
 *    the normal points from B to A, A's Jacobian is taken at the point on A, B's at
 *    the point on B.
 * Cube dynamics: btMultiBody floating base -- gravity, damping m v (k + k|v|),
 * I w (k + k|w|), the base bias term m (w x v) (computeAccelerations...MultiDof:
 * "zeroAccSpatFrc[0].addLinear(m_baseMass * omega.cross(vel))"), gyroscopic w x I w
 * (zero for a cube); orientation by the exponential map (stepPositionsMultiDof). */
/* obj[]: pos3 quat4 (x,y,z,w) linvel3 angvel3, the contact cache (id, impulse) x
 * (PGX_OBJECT_POINTS + PGXO_ROBOT_MAX), ReachAO obstacles (centres 6 x 3, active flags 6),
 * the cached link pose qc[7] (below) */
#define OBJ_CACHE 13
#define OBJ_CACHE1 (OBJ_CACHE + 2 * PGX_OBJECT_POINTS)
#define OBJ_AO (OBJ_CACHE1 + 2 * PGXO_ROBOT_MAX)
#define OBJ_QC (OBJ_AO + 4 * PGX_AO_OBSTACLES)
/* the persistent manifold pool (pgx.h PGX_MANIFOLD_POOL): count, then PGXO_POOL_MAX points of
 * MAN_PT doubles (kid, local A [3], local B [3], normal on B [3], distance, impulse) */
#define MAN_PT PGX_MANIFOLD_POINT
#define OBJ_MAN (OBJ_QC + 7)
#define OBJ_N (OBJ_MAN + 1 + PGXO_POOL_MAX * MAN_PT)
#define N_CACHE (PGX_OBJECT_POINTS + PGXO_ROBOT_MAX)
typedef char obj_layout_check[(OBJ_N == PGXO_OBJ_N) ? 1 : -1];
static void quat_mul(const double* a, const double* b, double* o);
#define NC_MAX (PGX_OBJECT_POINTS + PGXO_ROBOT_MAX)

/* the robot group's row budget: -1 = the configuration's (pgx_config.contacts: 4, or with
 * PGX_CONTACTS_FULL PGX_ROBOT_POINTS with an object, else PGX_ROBOT_POINTS_ARM); tests set
 * others (PGXO_ROBOT_MAX = no budget in practice).  Per substep, the robot points the per-pair
 * rule keeps before it. */
static int robot_budget = -1;
int64_t pgxo_pair_hist[PGXO_ROBOT_HIST];
void pgxo_set_robot_budget(int b) { robot_budget = b < 0 ? -1 : (b > PGXO_ROBOT_MAX ? PGXO_ROBOT_MAX : b); }
void pgxo_pair_hist_read(int64_t* out, int clear) {
    for (int i = 0; i < PGXO_ROBOT_HIST; i++)
        out[i] = clear ? __atomic_exchange_n(&pgxo_pair_hist[i], 0, __ATOMIC_RELAXED)
                       : __atomic_load_n(&pgxo_pair_hist[i], __ATOMIC_RELAXED);
}
/* per-thread scratch: bench.py's cpu_baseline steps one env shard per host thread */
#ifdef __cplusplus
#define PGXO_TLS thread_local
#else
#define PGXO_TLS _Thread_local
#endif
/* the last detection's points (tests): group, feature id, link, separation */
static PGXO_TLS int last_n;
static PGXO_TLS int last_grp[PGX_OBJECT_POINTS + PGXO_ROBOT_MAX], last_id[PGX_OBJECT_POINTS + PGXO_ROBOT_MAX],
    last_link[PGX_OBJECT_POINTS + PGXO_ROBOT_MAX];
static PGXO_TLS double last_dist[PGX_OBJECT_POINTS + PGXO_ROBOT_MAX];
int pgxo_last_contacts(int32_t* grp, int32_t* id, int32_t* link, double* dist) {
    for (int i = 0; i < last_n; i++) { grp[i] = last_grp[i]; id[i] = last_id[i]; link[i] = last_link[i]; dist[i] = last_dist[i]; }
    return last_n;
}

typedef struct {
    int grp, id, link;
    double n[3], pa[3], pb[3], dist;
    double* mp;   /* a manifold point: where the solved impulse goes back to, else NULL */
    double imp;   /* a manifold point: its applied impulse (warm start) */
    int sub;      /* row order after id (the study mode's table manifolds: the slot) */
} contact_t;

typedef struct {
    int contacts, has_object;
    double half, mass, inertia;
    double tc[3], th[3], plane_z;
    const double* obst;   /* ReachAO: obstacle centres [6][3] (static colliders), else NULL */
    int robot_points;     /* the robot group's budget (pgx_config.contacts: 4, or PGX_CONTACTS_FULL's) */
    /* the pairs' contact breaking thresholds (world_of, breaking_thresholds): capsule ci's link against
     * the table / plane / cube / an obstacle, and the cube against the table / plane */
    double tau_table[PGX_MAX_CAPSULES], tau_plane[PGX_MAX_CAPSULES], tau_cube[PGX_MAX_CAPSULES],
        tau_obst[PGX_MAX_CAPSULES];
    double tau_cube_table, tau_cube_plane;
} world_t;

/* closest pair of a capsule and an obstacle (ReachAO section below): signed distance d,
 * point on the capsule pa, on the obstacle pb, n the unit direction from the capsule axis
 * towards the obstacle (pb - pa = d n away from contact) */
typedef struct { double d, pa[3], pb[3], n[3]; } cdist_t;
static cdist_t ao_capsule_obstacle(const double* A, const double* B, double r, int o, const double* obst);
static double ao_pair_lower_bound(const double* A, const double* B, double r, int o, const double* obst);

static void quat_to_mat(const double* q, double* R) {
    double x = q[0], y = q[1], z = q[2], w = q[3];
    R[0] = 1 - 2 * (y * y + z * z); R[1] = 2 * (x * y - z * w);     R[2] = 2 * (x * z + y * w);
    R[3] = 2 * (x * y + z * w);     R[4] = 1 - 2 * (x * x + z * z); R[5] = 2 * (y * z - x * w);
    R[6] = 2 * (x * z - y * w);     R[7] = 2 * (y * z + x * w);     R[8] = 1 - 2 * (x * x + y * y);
}

/* A cube vertex P against the table box (top z = tc + th): its signed distance, the contact normal
 * from the box to P and the point on the box.  Inside the box, the face of least penetration (the top
 * first, then x, then y on a tie); outside, the closest point of the box -- one face's distance when
 * only one coordinate lies outside the box's slab (the top face: exactly P.z - top, as rounds 2-5). */
static double vertex_vs_table(const world_t* W, const double* P, double* n, double* pb) {
    const double top = W->tc[2] + W->th[2], bot = W->tc[2] - W->th[2];
    const double qx = P[0] - W->tc[0], qy = P[1] - W->tc[1];
    const double ex = fabs(qx) - W->th[0], ey = fabs(qy) - W->th[1];
    const double up = P[2] - top, dn = bot - P[2];
    const double ez = up >= dn ? up : dn;
    const double sx = qx < 0 ? -1.0 : 1.0, sy = qy < 0 ? -1.0 : 1.0, sz = up >= dn ? 1.0 : -1.0;
    pb[0] = P[0]; pb[1] = P[1]; pb[2] = P[2];
    n[0] = n[1] = n[2] = 0.0;
    if (ex <= 0 && ey <= 0 && ez <= 0) {   /* inside: the face of least penetration */
        if (ez >= ex && ez >= ey) { n[2] = sz; pb[2] = sz > 0 ? top : bot; return ez; }
        if (ex >= ey) { n[0] = sx; pb[0] = W->tc[0] + sx * W->th[0]; return ex; }
        n[1] = sy; pb[1] = W->tc[1] + sy * W->th[1];
        return ey;
    }
    const double ox = ex > 0 ? ex : 0.0, oy = ey > 0 ? ey : 0.0, oz = ez > 0 ? ez : 0.0;
    if (ox > 0) pb[0] = W->tc[0] + sx * W->th[0];
    if (oy > 0) pb[1] = W->tc[1] + sy * W->th[1];
    if (oz > 0) pb[2] = sz > 0 ? top : bot;
    if (ox == 0 && oy == 0) { n[2] = sz; return oz; }
    if (oy == 0 && oz == 0) { n[0] = sx; return ox; }
    if (ox == 0 && oz == 0) { n[1] = sy; return oy; }
    const double d = sqrt(ox * ox + oy * oy + oz * oz);
    n[0] = sx * ox / d; n[1] = sy * oy / d; n[2] = sz * oz / d;
    return d;
}

/* top of the static box under (x, y): the table top inside its footprint, else the plane */
static double ground_z(const world_t* W, const double* P) {
    if (fabs(P[0] - W->tc[0]) <= W->th[0] && fabs(P[1] - W->tc[1]) <= W->th[1]) return W->tc[2] + W->th[2];
    return W->plane_z;
}

/* candidates of one group in discovery order, each with its colliding pair */
#define CAND_MAX (32 * PGX_MAX_CAPSULES + 8)
typedef struct {
    contact_t c[CAND_MAX];
    int pair[CAND_MAX];
    int n;
} cands_t;
static void cand_add(cands_t* s, const contact_t* c, int pair) {
    if (s->n < CAND_MAX) { s->c[s->n] = *c; s->pair[s->n] = pair; s->n++; }
}
/* candidate j before candidate i: deeper, or as deep and discovered first */
static int before(const cands_t* s, int j, int i) {
    return s->c[j].dist < s->c[i].dist || (s->c[j].dist == s->c[i].dist && j < i);
}
/* Bullet's manifold rule (<= 4 points per pair: the pair's 4 deepest), then the group's budget
 * (its `budget` deepest); returns the kept count, *n_pair = the points before the budget */
static int select_points(const cands_t* s, int budget, contact_t* out, int* n_pair) {
    int keep[CAND_MAX], np = 0, n = 0;
    for (int i = 0; i < s->n; i++) {
        int rank = 0;
        for (int j = 0; j < s->n; j++) rank += j != i && s->pair[j] == s->pair[i] && before(s, j, i);
        keep[i] = rank < 4;
        np += keep[i];
    }
    for (int i = 0; i < s->n; i++) {
        if (!keep[i]) continue;
        int rank = 0;
        for (int j = 0; j < s->n; j++) rank += j != i && keep[j] && before(s, j, i);
        if (rank < budget) out[n++] = s->c[i];
    }
    if (n_pair) *n_pair = np;
    return n;
}
static void sort_by_id(contact_t* s, int n) {   /* by (id, sub) */
    for (int i = 1; i < n; i++)
        for (int j = i; j > 0 && (s[j].id < s[j - 1].id || (s[j].id == s[j - 1].id && s[j].sub < s[j - 1].sub)); j--) {
            contact_t t = s[j]; s[j] = s[j - 1]; s[j - 1] = t;
        }
}

/* number of sample spheres along a capsule (spacing <= r/2) */
static int capsule_samples(const double* a, const double* b, double r) {
    double d[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]};
    double len = v3_norm(d);
    if (len <= 0.0) return 1;
    return (int)ceil(len / (0.5 * r) - 1e-9) + 1;
}

enum { PAIR_TABLE = 0, PAIR_PLANE = 1, PAIR_CUBE = 2, PAIR_OBSTACLE = 3 };   /* + 16 x capsule */

/* ---- Bullet's persistent contact manifold (btPersistentManifold / btManifoldResult, Bullet 3 as
 * pybullet 3.2.6 runs it; not vendored).  The default with PGX_CONTACTS_FULL for the robot's pairs
 * with the cube and with the obstacles: per pair (a capsule against the cube or an obstacle) the
 * narrow phase reports one new point per stepSimulation -- GJK's closest pair of the convex
 * capsule and the box, restated as the pair's deepest sample (ties: the lowest sample); the exact
 * closest pair for an obstacle -- and addContactPoint (btManifoldResult) merges it:
 *   getCacheEntry: the cached point nearest to it in A's local frame, strictly within the breaking
 *     threshold squared (0.02^2), first in slot order -> replaceContactPoint: the new point's
 *     positions, normal and distance, the cached applied impulse kept (MAINTAIN_PERSISTENCY);
 *   else addManifoldPoint: appended below MANIFOLD_CACHE_SIZE = 4, else sortCachedPoints picks
 *     the slot to overwrite (impulse 0): the slot whose replacement leaves the largest
 *     |(pt - c_a) x (c_b - c_c)|^2 ("gContactCalcArea3Points"), never the point deeper than the
 *     new one and every other (KEEP_DEEPEST_POINT), the first on ties (maxAxis4);
 * then refreshContactPoints moves every cached point with its bodies (local -> world), recomputes
 * its distance along the stored normal, and in reverse slot order removes a point past the
 * breaking threshold (validContactDistance) or whose B point slid more than the threshold off A's
 * projection (removeContactPoint: the last slot's point fills the hole).  Every manifold point is
 * a solver row warm-started from its own applied impulse (x 0.85) and written back after the solve.
 * The robot's end spheres against the table / plane keep the fresh rule: each is a child shape with
 * a manifold of its own whose one point is re-reported every substep (merged into itself, impulse
 * kept), i.e. the fresh candidate with its feature's warm start -- PGX_FLAG_PERSISTENT_MANIFOLD runs
 * them through manifolds too, and a test pins the two to rounding.  Cube vs table / plane: the box-box
 * detector re-reports all (<= 4) points every substep, restated as its 4 deepest vertices.
 * Kept per env in a pool of at most PGX_MANIFOLD_POOL (PGX_MANIFOLD_POOL_AO) points, the kernel's
 * layout (pgx.h): a point that would need a new pool entry when the pool is full is dropped and
 * counted (pgxo_diag_hist[120]; not reached in the configs' random-policy runs).  Merge order:
 * the cube pairs by capsule, the obstacle pairs obstacle-major (the kernels' lane-parallel order);
 * a new point's pool entry goes last, removals keep the others' order. */
enum { MP_KID = 0, MP_LA = 1, MP_LB = 4, MP_N = 7, MP_D = 10, MP_IMP = 11 };
#define KEY_TABLE 1024   /* study mode: 1024 + 64 c + 8 (table 0 / plane 1) + 4 end */

static double* pool_pt(double* P, int i) { return P + 1 + MAN_PT * i; }
/* the arm link whose frame carries capsule ci (its own or the nearest ancestor with a moving joint:
 * the fixed links past panda_link7 ride on it) -- the kernels' kCapJ joint frame */
static int cap_frame_link(const pgx_model* m, int ci) {
    int l = m->cap_link[ci];
    while (l >= 0 && m->dof_of_link[l] < 0) l = m->parent[l];
    return l;
}
/* manifold key -> capsule; its B body is the cube (has_object), an obstacle or the table */
static int key_capsule(int key, int has_object) {
    if (key >= KEY_TABLE) return (key - KEY_TABLE) / 64;
    return has_object ? (key - 32) / 16 : (key - 32) / 24;
}
/* the points of manifold `key` by slot (idx[slot] = pool index); their count */
static int man_points(double* P, int key, int idx[4]) {
    int n = 0;
    const int cnt = (int)P[0];
    for (int i = 0; i < cnt; i++) {
        const int kid = (int)pool_pt(P, i)[MP_KID];
        if ((kid & ~3) == key) { idx[kid & 3] = i; n++; }
    }
    return n;
}
static int man_sort_cached(double* P, const int idx[4], const double* np) {   /* sortCachedPoints */
    const double* c[4];
    for (int i = 0; i < 4; i++) c[i] = pool_pt(P, idx[i]);
    int maxi = -1;
    double maxpen = np[MP_D];
    for (int i = 0; i < 4; i++)
        if (c[i][MP_D] < maxpen) { maxi = i; maxpen = c[i][MP_D]; }
    double res[4] = {0, 0, 0, 0};
    static const int ia[4] = {1, 0, 0, 0}, ib[4] = {3, 3, 3, 2}, ic[4] = {2, 2, 1, 1};
    for (int i = 0; i < 4; i++) {
        if (i == maxi) continue;
        double a[3], b[3], x[3];
        for (int j = 0; j < 3; j++) {
            a[j] = np[MP_LA + j] - c[ia[i]][MP_LA + j];
            b[j] = c[ib[i]][MP_LA + j] - c[ic[i]][MP_LA + j];
        }
        v3_cross(a, b, x);
        res[i] = v3_dot(x, x);
    }
    int best = 0;
    for (int i = 1; i < 4; i++)
        if (res[i] > res[best]) best = i;
    return best;
}
/* addContactPoint of np (MP layout; kid and impulse ignored) to manifold `key`; returns the slot
 * it went to, -1 when the pool was full */
static int man_add(double* P, int cap, int key, const double* np, double thr2) {
    int idx[4];
    const int n = man_points(P, key, idx);
    int near = -1;
    double sh = thr2;
    for (int i = 0; i < n; i++) {   /* getCacheEntry */
        const double* c = pool_pt(P, idx[i]);
        double e[3] = {c[MP_LA] - np[MP_LA], c[MP_LA + 1] - np[MP_LA + 1], c[MP_LA + 2] - np[MP_LA + 2]};
        const double dd = v3_dot(e, e);
        if (dd < sh) { sh = dd; near = i; }
    }
    if (near >= 0) {   /* replaceContactPoint: the cached impulse stays */
        double* c = pool_pt(P, idx[near]);
        memcpy(c + MP_LA, np + MP_LA, (MP_IMP - MP_LA) * sizeof(double));
        PGXO_HIST_ADD(pgxo_diag_hist, 121, 1);
        return near;
    }
    if (n < 4) {
        const int cnt = (int)P[0];
        if (cnt >= cap) { PGXO_HIST_ADD(pgxo_diag_hist, 120, 1); return -1; }
        PGXO_HIST_ADD(pgxo_diag_hist, 122, 1);
        double* c = pool_pt(P, cnt);
        memcpy(c, np, MAN_PT * sizeof(double));
        c[MP_KID] = key + n;
        c[MP_IMP] = 0.0;
        P[0] = cnt + 1;
        return n;
    }
    const int slot = man_sort_cached(P, idx, np);
    PGXO_HIST_ADD(pgxo_diag_hist, 123, 1);
    double* c = pool_pt(P, idx[slot]);
    memcpy(c + MP_LA, np + MP_LA, (MP_IMP - MP_LA) * sizeof(double));
    c[MP_IMP] = 0.0;
    return slot;
}
/* refreshContactPoints of every manifold in the pool, from the points' world positions pa, pb:
 * distance along the stored normal, then per manifold in reverse slot order the removals (the
 * last slot's point takes a removed point's slot); the pool keeps the survivors' order */
static void pool_refresh(double* P, const double (*pa)[3], const double (*pb)[3], const double* thr) {
    const int cnt = (int)P[0];
    int drop[PGXO_POOL_MAX];
    for (int i = 0; i < cnt; i++) {
        double* c = pool_pt(P, i);
        const double* n = c + MP_N;
        const double d = (pa[i][0] - pb[i][0]) * n[0] + (pa[i][1] - pb[i][1]) * n[1] + (pa[i][2] - pb[i][2]) * n[2];
        c[MP_D] = d;
        drop[i] = d > thr[i];
        if (drop[i]) PGXO_HIST_ADD(pgxo_diag_hist, 124, 1);
        else {
            double e[3];
            for (int j = 0; j < 3; j++) e[j] = pb[i][j] - (pa[i][j] - n[j] * d);
            drop[i] = v3_dot(e, e) > thr[i] * thr[i];
            if (drop[i]) PGXO_HIST_ADD(pgxo_diag_hist, 125, 1);
        }
    }
    int seen[PGXO_POOL_MAX] = {0};
    for (int i = 0; i < cnt; i++) {
        const int key = (int)pool_pt(P, i)[MP_KID] & ~3;
        if (seen[i]) continue;
        int cur[4];
        int n = man_points(P, key, cur);
        for (int s2 = 0; s2 < n; s2++) seen[cur[s2]] = 1;
        for (int s2 = n - 1; s2 >= 0; s2--)
            if (drop[cur[s2]]) { cur[s2] = cur[n - 1]; n--; }
        for (int s2 = 0; s2 < n; s2++) pool_pt(P, cur[s2])[MP_KID] = key + s2;
    }
    int k = 0;
    for (int i = 0; i < cnt; i++) {
        if (drop[i]) continue;
        if (k != i) memcpy(pool_pt(P, k), pool_pt(P, i), MAN_PT * sizeof(double));
        k++;
    }
    P[0] = k;
}
/* world positions of pool point i's A (robot) and B points */
static void man_world(const pgx_model* m, const kin_t* k, const double* obj, int has_object, const double* c,
                      double* pa, double* pb) {
    const int key = (int)c[MP_KID] & ~3, fl = cap_frame_link(m, key_capsule(key, has_object));
    m3_v(k->R[fl], c + MP_LA, pa);
    for (int i = 0; i < 3; i++) pa[i] += k->o[fl][i];
    if (key < KEY_TABLE && has_object) {   /* the cube: B's local frame moves with it */
        double Rc[9];
        quat_to_mat(obj + 3, Rc);
        m3_v(Rc, c + MP_LB, pb);
        for (int i = 0; i < 3; i++) pb[i] += obj[i];
    } else {                                /* table / plane / obstacle: static, local = world */
        memcpy(pb, c + MP_LB, 3 * sizeof(double));
    }
}
/* test entry points: a pool whose bodies do not move (local = world) */
int pgxo_manifold_add(double* P, int cap, int key, const double* point, double thr) {
    return man_add(P, cap, key, point, thr * thr);
}
void pgxo_manifold_refresh_static(double* P, double thr) {
    double pa[PGXO_POOL_MAX][3], pb[PGXO_POOL_MAX][3], th[PGXO_POOL_MAX];
    for (int i = 0; i < (int)P[0]; i++) {
        for (int j = 0; j < 3; j++) { pa[i][j] = pool_pt(P, i)[MP_LA + j]; pb[i][j] = pool_pt(P, i)[MP_LB + j]; }
        th[i] = thr;
    }
    pool_refresh(P, pa, pb, th);
}

/* a pair's new point: the contact, its manifold key and its merge order */
typedef struct { contact_t c; int key, order; } newpt_t;
#define NEWPT_MAX (4 * PGX_MAX_CAPSULES + PGX_MAX_CAPSULES * PGX_AO_OBSTACLES)

/* contact detection; returns the number of contacts (grouped, each group sorted by id) */
/* the breaking threshold of manifold `key`'s pair: capsule vs cube / obstacle, or (study mode) a table /
 * plane end sphere -- for a table key of a new point `c` gives its box, else the key's code */
static double key_threshold(const world_t* W, int key, const contact_t* c) {
    (void)c;
    if (key >= KEY_TABLE) {
        const int ci = (key - KEY_TABLE) / 64, code = ((key - KEY_TABLE) >> 3) & 7;
        return code == PAIR_PLANE ? W->tau_plane[ci] : W->tau_table[ci];
    }
    const int ci = key_capsule(key, W->has_object);
    return W->has_object ? W->tau_cube[ci] : W->tau_obst[ci];
}

static int detect(const pgx_model* m, const pgx_sim_params* p, const world_t* W, const kin_t* k, double* obj,
                  contact_t* out) {
    static PGXO_TLS cands_t s0, s1;   /* per thread (cpu_baseline runs shards in threads) */
    s0.n = 0; s1.n = 0;
    /* Bullet's persistent manifolds for the cube / obstacle pairs (the default budget), and with the
     * study flag for the table / plane pairs as well */
    const int pers = W->contacts == PGX_CONTACTS_FULL && !(p->flags & PGX_FLAG_FRESH_MANIFOLD);
    const int pers_table = pers && (p->flags & PGX_FLAG_PERSISTENT_MANIFOLD);
    static PGXO_TLS newpt_t np[NEWPT_MAX];
    int nnp = 0;
    double Rc[9];
    if (W->has_object) {
        /* round 6: the cube's vertices against the whole table box -- its top and its side walls --
         * and against the plane's top (candidates: the table's for every vertex, ids 0-7, then the
         * plane's, ids 8-15).  Rounds 2-5 took each vertex against the top face of the box under it,
         * so a vertex that crossed the table's edge below the top met the top face from inside, its
         * whole depth as penetration (a cube knocked over the edge was thrown back up: DESIGN.md
         * section 2). */
        quat_to_mat(obj + 3, Rc);
        const double h = W->half;
        double P8[8][3];
        for (int v = 0; v < 8; v++) {
            double lc[3] = {(v & 1) ? h : -h, (v & 2) ? h : -h, (v & 4) ? h : -h};
            m3_v(Rc, lc, P8[v]);
            for (int i = 0; i < 3; i++) P8[v][i] += obj[i];
        }
        for (int v = 0; v < 8; v++) {
            const double* P = P8[v];
            double n[3], pb[3];
            const double d = vertex_vs_table(W, P, n, pb);
            if (d < W->tau_cube_table) {
                contact_t c = {0, v, -1, {n[0], n[1], n[2]}, {P[0], P[1], P[2]}, {pb[0], pb[1], pb[2]}, d, NULL, 0.0, 0};
                cand_add(&s0, &c, PAIR_TABLE);
            }
        }
        for (int v = 0; v < 8; v++) {
            const double* P = P8[v];
            const double d = P[2] - W->plane_z;
            if (d < W->tau_cube_plane) {
                contact_t c = {0, 8 + v, -1, {0, 0, 1}, {P[0], P[1], P[2]}, {P[0], P[1], W->plane_z}, d, NULL, 0.0, 0};
                cand_add(&s0, &c, PAIR_PLANE);
            }
        }
    }
    for (int ci = 0; ci < m->n_capsules; ci++) {
        int li = m->cap_link[ci];
        if (m->cap_flags[ci] == 0) continue;   /* base / panda_link1: no contacts */
        double A[3], B[3];
        m3_v(k->R[li], m->cap_a[ci], A);
        m3_v(k->R[li], m->cap_b[ci], B);
        for (int i = 0; i < 3; i++) { A[i] += k->o[li][i]; B[i] += k->o[li][i]; }
        const double r = m->cap_radius[ci];
        int same = m->cap_a[ci][0] == m->cap_b[ci][0] && m->cap_a[ci][1] == m->cap_b[ci][1] &&
                   m->cap_a[ci][2] == m->cap_b[ci][2];
        if (W->contacts && (m->cap_flags[ci] & PGX_CAP_VS_TABLE)) {
            for (int e = 0; e < (same ? 1 : 2); e++) {
                const double* P = e ? B : A;
                double zt = ground_z(W, P);
                double d = P[2] - r - zt;
                if (d < (zt == W->plane_z ? W->tau_plane[ci] : W->tau_table[ci])) {
                    contact_t c = {1, 2 * ci + e, li, {0, 0, 1}, {P[0], P[1], P[2] - r}, {P[0], P[1], zt}, d, NULL,
                                   0.0, 0};
                    const int code = zt == W->plane_z ? PAIR_PLANE : PAIR_TABLE;
                    if (pers_table) {
                        np[nnp].c = c;
                        np[nnp].key = KEY_TABLE + 64 * ci + 8 * code + 4 * e;
                        np[nnp].order = 2 * ci + e;
                        nnp++;
                    } else {
                        cand_add(&s1, &c, 16 * ci + code);
                    }
                }
            }
        }
        if (W->has_object && (m->cap_flags[ci] & PGX_CAP_VS_OBJECT)) {
            const double h = W->half;
            int ns = capsule_samples(m->cap_a[ci], m->cap_b[ci], r);
            int best = -1;
            for (int s = 0; s < ns; s++) {
                double t = ns > 1 ? (double)s / (double)(ns - 1) : 0.0, C[3], rel[3], cl[3];
                for (int i = 0; i < 3; i++) { C[i] = A[i] + t * (B[i] - A[i]); rel[i] = C[i] - obj[i]; }
                /* box frame: R^T (C - p) */
                for (int i = 0; i < 3; i++) cl[i] = Rc[i] * rel[0] + Rc[3 + i] * rel[1] + Rc[6 + i] * rel[2];
                double qb[3], diff[3], nl[3], depth;
                for (int i = 0; i < 3; i++) { qb[i] = clampd(cl[i], -h, h); diff[i] = cl[i] - qb[i]; }
                double dist = v3_norm(diff);
                if (dist > 1e-12) {
                    for (int i = 0; i < 3; i++) nl[i] = diff[i] / dist;
                    depth = dist - r;
                } else { /* sphere centre inside the box: push out through the nearest face */
                    int ax = 0;
                    double bst = h - fabs(cl[0]);
                    for (int i = 1; i < 3; i++)
                        if (h - fabs(cl[i]) < bst) { bst = h - fabs(cl[i]); ax = i; }
                    double sg = cl[ax] < 0 ? -1.0 : 1.0;
                    nl[0] = nl[1] = nl[2] = 0.0;
                    nl[ax] = sg;
                    qb[ax] = sg * h;
                    depth = -bst - r;
                }
                if (depth < W->tau_cube[ci]) {
                    contact_t c;
                    c.grp = 2; c.id = 32 + ci * 16 + s; c.link = li; c.dist = depth;
                    c.mp = NULL; c.imp = 0.0; c.sub = 0;
                    m3_v(Rc, nl, c.n);
                    m3_v(Rc, qb, c.pb);
                    for (int i = 0; i < 3; i++) { c.pb[i] += obj[i]; c.pa[i] = C[i] - r * c.n[i]; }
                    if (pers) {   /* the pair's one new point: its deepest sample (the first on a tie) */
                        if (best < 0 || depth < np[best].c.dist) {
                            if (best < 0) { best = nnp++; np[best].key = 32 + 16 * ci; np[best].order = 1000 + ci; }
                            np[best].c = c;
                        }
                    } else {
                        cand_add(&s1, &c, 16 * ci + PAIR_CUBE);
                    }
                }
            }
        }
        /* ReachAO: the obstacles are static colliders (create_obstacle_sphere / _cuboid,
         * reach_ao.py:819-860: mass 0, not ghosts), so Bullet resolves robot contacts with
         * them inside stepSimulation like the table's: per capsule and obstacle the closest
         * pair (one point, as the convex-convex query returns it) within the processing
         * threshold, the normal from the obstacle to the robot, a static body B */
        if (W->obst) {
            for (int o = 0; o < PGX_AO_OBSTACLES; o++) {
                /* the axis-to-centre distance minus the radii bounds the pair from below: a pair
                 * that cannot be within tau is not measured (the same candidates) */
                if (ao_pair_lower_bound(A, B, r, o, W->obst) >= W->tau_obst[ci]) continue;
                const cdist_t cd = ao_capsule_obstacle(A, B, r, o, W->obst);
                if (cd.d < W->tau_obst[ci]) {
                    contact_t c = {1, 32 + 6 * ci + o, li, {-cd.n[0], -cd.n[1], -cd.n[2]},
                                   {cd.pa[0], cd.pa[1], cd.pa[2]}, {cd.pb[0], cd.pb[1], cd.pb[2]}, cd.d, NULL, 0.0, 0};
                    if (pers) {
                        np[nnp].c = c;
                        np[nnp].key = 32 + 24 * ci + 4 * o;
                        np[nnp].order = 2000 + 16 * o + ci;
                        nnp++;
                    } else {
                        cand_add(&s1, &c, 16 * ci + PAIR_OBSTACLE + o);
                    }
                }
            }
        }
    }
    if (pers) {
        double* P = obj + OBJ_MAN;
        const int cap = pers_table ? PGXO_POOL_MAX : (W->has_object ? PGX_MANIFOLD_POOL : PGX_MANIFOLD_POOL_AO);
        /* 1. addContactPoint in merge order (insertion sort by order), within the pair's breaking
         * threshold */
        for (int i = 1; i < nnp; i++)
            for (int j = i; j > 0 && np[j].order < np[j - 1].order; j--) { newpt_t t = np[j]; np[j] = np[j - 1]; np[j - 1] = t; }
        for (int j = 0; j < nnp; j++) {
            const contact_t* c = &np[j].c;
            const int fl = cap_frame_link(m, key_capsule(np[j].key, W->has_object));
            double pt[MAN_PT], d[3];
            for (int i = 0; i < 3; i++) d[i] = c->pa[i] - k->o[fl][i];
            for (int i = 0; i < 3; i++)
                pt[MP_LA + i] = k->R[fl][i] * d[0] + k->R[fl][3 + i] * d[1] + k->R[fl][6 + i] * d[2];
            if (np[j].key < KEY_TABLE && W->has_object) {
                double e[3] = {c->pb[0] - obj[0], c->pb[1] - obj[1], c->pb[2] - obj[2]};
                for (int i = 0; i < 3; i++) pt[MP_LB + i] = Rc[i] * e[0] + Rc[3 + i] * e[1] + Rc[6 + i] * e[2];
            } else {
                memcpy(pt + MP_LB, c->pb, 3 * sizeof(double));
            }
            memcpy(pt + MP_N, c->n, 3 * sizeof(double));
            pt[MP_D] = c->dist;
            pt[MP_KID] = 0.0;
            pt[MP_IMP] = 0.0;
            const double thr = key_threshold(W, np[j].key, &np[j].c);
            man_add(P, cap, np[j].key, pt, thr * thr);
        }
        /* 2. refreshContactPoints: move the points with their bodies, drop the broken ones (each
         * against its pair's threshold) */
        const int cnt = (int)P[0];
        double pa[PGXO_POOL_MAX][3], pb[PGXO_POOL_MAX][3], thr[PGXO_POOL_MAX];
        for (int i = 0; i < cnt; i++) {
            man_world(m, k, obj, W->has_object, pool_pt(P, i), pa[i], pb[i]);
            thr[i] = key_threshold(W, (int)pool_pt(P, i)[MP_KID] & ~3, NULL);
        }
        pool_refresh(P, pa, pb, thr);
        /* 3. the manifold points are the group's candidates after the fresh table ones, in pool order,
         * each its own pair (a manifold holds <= 4 already) */
        for (int i = 0; i < (int)P[0]; i++) {
            double* c = pool_pt(P, i);
            const int kid = (int)c[MP_KID], key = kid & ~3, ci = key_capsule(key, W->has_object);
            contact_t ct;
            ct.grp = (key < KEY_TABLE && W->has_object) ? 2 : 1;
            ct.id = key >= KEY_TABLE ? 2 * ci + ((key >> 2) & 1) : kid;
            ct.sub = key >= KEY_TABLE ? (kid & 3) : 0;
            ct.link = m->cap_link[ci];
            man_world(m, k, obj, W->has_object, c, ct.pa, ct.pb);
            memcpy(ct.n, c + MP_N, sizeof ct.n);
            ct.dist = c[MP_D];
            ct.mp = c;
            ct.imp = c[MP_IMP];
            cand_add(&s1, &ct, 100000 + i);
        }
    }
    int np1;
    const int n0 = select_points(&s0, PGX_OBJECT_POINTS, out, NULL);
    const int budget = robot_budget >= 0 ? robot_budget : W->robot_points;
    const int n1 = select_points(&s1, budget, out + n0, &np1);
    PGXO_HIST_ADD(pgxo_pair_hist, np1 < PGXO_ROBOT_HIST - 1 ? np1 : PGXO_ROBOT_HIST - 1, 1);
    sort_by_id(out, n0);
    sort_by_id(out + n0, n1);
    last_n = n0 + n1;
    for (int i = 0; i < last_n; i++) {
        last_grp[i] = out[i].grp; last_id[i] = out[i].id; last_link[i] = out[i].link; last_dist[i] = out[i].dist;
    }
    return n0 + n1;
}

/* btPlaneSpace1 */
static void plane_space(const double* n, double* p, double* q) {
    if (fabs(n[2]) > 0.7071067811865476) {
        double a = n[1] * n[1] + n[2] * n[2], k = 1.0 / sqrt(a);
        p[0] = 0; p[1] = -n[2] * k; p[2] = n[1] * k;
        q[0] = a * k; q[1] = -n[0] * p[2]; q[2] = n[0] * p[1];
    } else {
        double a = n[0] * n[0] + n[1] * n[1], k = 1.0 / sqrt(a);
        p[0] = -n[1] * k; p[1] = n[0] * k; p[2] = 0;
        q[0] = -n[2] * p[1]; q[1] = n[2] * p[0]; q[2] = a * k;
    }
}

typedef struct {
    double Jr[D], Rr[D];   /* robot Jacobian row and M^-1 J^T */
    double Jc[6], Rc[6];   /* object (linvel, angvel) row and its response */
    double jinv, rhs, lam, lo, hi;
} crow_t;

/* One stepSimulation() (PyBullet.step pybullet.py:68-71 calls this 20x):
 *  1. contacts at the current poses (world only)
 *  2. unconstrained: qd += dt*qdd(q,qd), clamp |qd| <= maxCoordinateVelocity
 *     (btMultiBodyDynamicsWorld::solveExternalForces -> ABA + applyDeltaVeeMultiDof);
 *     object: v += dt (g - (k + k|v|) v - w x v), w += dt (-(k + k|w|) w)
 *  3. constraint rows (btMultiBodyJointMotor / btMultiBodyJointLimitConstraint ::
 *     createConstraintRows, contact rows above) solved by projected Gauss-Seidel
 *     (btMultiBodyConstraintSolver::resolveSingleConstraintRowGeneric): joint rows in
 *     the world's sorted order, reversed on even iterations, then normal rows, then
 *     friction rows; stop when the max squared row residual <= residual_threshold
 *  4. qd += M^-1 J^T lambda (constraint pass), q += dt*qd (stepPositionsMultiDof);
 *     object: p += dt v, orientation by the exponential map of w dt. */
static void substep_impl(const pgx_model* m, const pgx_sim_params* p, const double base[3], double* q, double* qd,
                         const pgxo_motor* motors, pgxo_stats* st, const world_t* W, double* obj) {
    int nd = m->n_dofs;
    double dt = p->dt;
    kin_t k;
    PGXO_PHASE(2);
    fk(m, base, q, &k);
    contact_t con[NC_MAX];
    PGXO_PHASE(1);
    int ncon = W ? detect(m, p, W, &k, obj, con) : 0;
    PGXO_PHASE(2);
    double M[D * D], Lm[D * D], b[D], qdd[D], Minv[D * D];
    if (p->flags & PGX_FLAG_DYN_RECURSIVE) {
        dyn_recursive(m, p, &k, qd, 1, M, b);
    } else {
        mass_matrix(m, &k, M);
        bias(m, p, &k, qd, 1, 1, b);
    }
    memset(Lm, 0, sizeof Lm);
    chol(nd, M, Lm);
    double nb[D] = {0};
    for (int d = 0; d < nd; d++) nb[d] = -b[d];
    chol_solve(nd, Lm, nb, qdd);
    for (int c = 0; c < nd; c++) {
        double e[D] = {0}, x[D];
        e[c] = 1.0;
        chol_solve(nd, Lm, e, x);
        for (int r = 0; r < nd; r++) Minv[r * nd + c] = x[r];
    }
    double vu[D];
    for (int d = 0; d < nd; d++) vu[d] = clampd(qd[d] + dt * qdd[d], -p->max_coord_vel, p->max_coord_vel);
    double vcu[3] = {0, 0, 0}, wcu[3] = {0, 0, 0};
    const int has_obj = W && W->has_object;
    if (has_obj) {
        const double* v = obj + 7;
        const double* w = obj + 10;
        double vn = v3_norm(v), wn = v3_norm(w), wxv[3];
        v3_cross(w, v, wxv);
        for (int i = 0; i < 3; i++) {
            vcu[i] = v[i] + dt * (p->gravity[i] - (p->lin_damping + p->lin_damping * vn) * v[i] - wxv[i]);
            wcu[i] = w[i] + dt * (-(p->ang_damping + p->ang_damping * wn) * w[i]);
        }
    }

    /* --- joint rows */
    PGXO_PHASE(3);
    int nr = 0;
    double rhs[PGX_MAX_ROWS], lo[PGX_MAX_ROWS], hi[PGX_MAX_ROWS], inv[PGX_MAX_ROWS], sgn[PGX_MAX_ROWS],
        lam[PGX_MAX_ROWS];
    int rdof[PGX_MAX_ROWS];
    for (int r = 0; r < m->n_rows; r++) {
        int kind = m->row_kind[r], d = m->row_dof[r];
        double s = (kind == PGX_ROW_LIMIT_UPPER) ? -1.0 : 1.0;
        double denom = Minv[d * nd + d];
        double jinv = denom > 2.220446049250313e-16 ? 1.0 / denom : 0.0;
        double rel_vel = s * vu[d];
        double r_rhs, r_lo, r_hi;
        if (kind == PGX_ROW_MOTOR) {
            const pgxo_motor* mo = &motors[d];
            if (mo->max_impulse == 0.0) continue;   /* createConstraintRows returns early */
            double pos_term = 1.0 * (mo->target_q - q[d]) / dt; /* m_erp = 1 */
            double desired = mo->kp * pos_term + vu[d] + mo->kd * (mo->target_qd - vu[d]);
            r_rhs = (desired - rel_vel) * jinv;
            r_lo = -mo->max_impulse;
            r_hi = mo->max_impulse;
        } else {
            double pen = (kind == PGX_ROW_LIMIT_LOWER) ? (q[d] - m->lower[d]) : (m->upper[d] - q[d]);
            double verr = -rel_vel, perr = 0.0;
            if (pen > 0) verr -= pen / dt;        /* speculative: may approach, not cross */
            else perr = -pen * p->erp / dt;
            r_rhs = (perr + verr) * jinv;
            r_lo = 0.0;
            r_hi = p->limit_max_impulse;
        }
        rhs[nr] = r_rhs; lo[nr] = r_lo; hi[nr] = r_hi; inv[nr] = jinv; sgn[nr] = s; rdof[nr] = d; lam[nr] = 0.0;
        nr++;
    }
    if (st) { /* diagnostics only: the HIP kernel's limit-row skip criterion */
        int far = 1;
        for (int d = 0; d < nd; d++) {
            double B = 0;
            for (int kk = 0; kk < nd; kk++) B += fabs(Minv[d * nd + kk]) * (motors[kk].max_impulse);
            B = B * 1.001 + 1e-6;
            double penl = q[d] - m->lower[d], penu = m->upper[d] - q[d];
            far = far && penl > 0 && penu > 0 && (vu[d] - B) > -penl / dt && (vu[d] + B) < penu / dt;
        }
        st->limits_far = far;
        st->n_contacts = ncon;
    }
    double dv[D] = {0}, dvc[6] = {0, 0, 0, 0, 0, 0};

    /* --- contact rows: [3 * k] normal, [3 * k + 1 + j] friction j */
    crow_t cr[3 * NC_MAX];
    for (int c = 0; c < ncon; c++) {
        const contact_t* ct = &con[c];
        double dirs[3][3];
        memcpy(dirs[0], ct->n, sizeof dirs[0]);
        plane_space(ct->n, dirs[1], dirs[2]);
        double Jv[3 * D], Jw[3 * D];
        if (ct->grp != 0) jacobian(m, &k, ct->link, ct->pa, Jv, Jw);
        for (int j = 0; j < 3; j++) {
            crow_t* R = &cr[3 * c + j];
            const double* u = dirs[j];
            memset(R, 0, sizeof *R);
            if (ct->grp != 0)
                for (int d = 0; d < nd; d++) R->Jr[d] = Jv[d] * u[0] + Jv[nd + d] * u[1] + Jv[2 * nd + d] * u[2];
            if (ct->grp == 0 || ct->grp == 2) {
                const double* pt = ct->grp == 0 ? ct->pa : ct->pb;
                double rr[3] = {pt[0] - obj[0], pt[1] - obj[1], pt[2] - obj[2]}, rxu[3];
                v3_cross(rr, u, rxu);
                double sg = ct->grp == 0 ? 1.0 : -1.0;
                for (int i = 0; i < 3; i++) { R->Jc[i] = sg * u[i]; R->Jc[3 + i] = sg * rxu[i]; }
            }
            for (int a = 0; a < nd; a++) {
                double s = 0;
                for (int d = 0; d < nd; d++) s += Minv[a * nd + d] * R->Jr[d];
                R->Rr[a] = s;
            }
            for (int i = 0; i < 3; i++) { R->Rc[i] = R->Jc[i] / W->mass; R->Rc[3 + i] = R->Jc[3 + i] / W->inertia; }
            double den = 0, rel = 0;
            for (int d = 0; d < nd; d++) { den += R->Jr[d] * R->Rr[d]; rel += R->Jr[d] * vu[d]; }
            for (int i = 0; i < 6; i++) den += R->Jc[i] * R->Rc[i];
            for (int i = 0; i < 3; i++) rel += R->Jc[i] * vcu[i] + R->Jc[3 + i] * wcu[i];
            R->jinv = den > 2.220446049250313e-16 ? 1.0 / den : 0.0;
            if (j == 0) {
                double pen = ct->dist, perr = 0.0, verr = -rel;
                if (pen > 0) verr -= pen / dt;
                else perr = -pen * p->contact_erp / dt;
                R->rhs = (perr + verr) * R->jinv;
                R->lo = 0.0;
                R->hi = 1e10;
                /* warm start from the same feature's impulse of the previous step (persistent
                 * manifold: the point's own applied impulse) */
                const double* cache = obj + (ct->grp != 0 ? OBJ_CACHE1 : OBJ_CACHE);
                if (ct->mp) R->lam = p->warmstart * ct->imp;
                else
                    for (int s = 0; s < (ct->grp != 0 ? PGXO_ROBOT_MAX : PGX_OBJECT_POINTS); s++)
                        if ((int)cache[2 * s] == ct->id) R->lam = p->warmstart * cache[2 * s + 1];
                if (R->lam != 0.0) {
                    for (int d = 0; d < nd; d++) dv[d] += R->Rr[d] * R->lam;
                    for (int i = 0; i < 6; i++) dvc[i] += R->Rc[i] * R->lam;
                }
            } else {
                R->rhs = -rel * R->jinv;
            }
        }
    }

    int it_used = 0;
    PGXO_PHASE(4);
    for (int it = 0; it < p->num_iterations; it++) {
        double resid = 0.0;
        for (int j = 0; j < nr; j++) {
            int r = (it & 1) ? j : nr - 1 - j;
            int d = rdof[r];
            double delta = rhs[r] - sgn[r] * dv[d] * inv[r];
            double sum = lam[r] + delta;
            if (sum < lo[r]) { delta = lo[r] - lam[r]; lam[r] = lo[r]; }
            else if (sum > hi[r]) { delta = hi[r] - lam[r]; lam[r] = hi[r]; }
            else lam[r] = sum;
            for (int c = 0; c < nd; c++) dv[c] += Minv[c * nd + d] * sgn[r] * delta;
            double res = inv[r] != 0.0 ? delta / inv[r] : 0.0;
            if (res * res > resid) resid = res * res;
        }
        for (int pass = 0; pass < 2; pass++) {
            for (int c = 0; c < ncon; c++) {
                for (int j = (pass ? 1 : 0); j < (pass ? 3 : 1); j++) {
                    crow_t* R = &cr[3 * c + j];
                    if (pass) { /* friction: bounds from the normal impulse, skipped while it is 0 */
                        double ln = cr[3 * c].lam;
                        if (!(ln > 0.0)) continue;
                        /* combined lateral friction (btManifoldResult: the product): the cube
                         * against the table / plane, or the robot link against any body */
                        const double mu = con[c].grp == 0 ? p->friction : p->link_friction[con[c].link];
                        R->lo = -mu * ln;
                        R->hi = mu * ln;
                    }
                    double jdv = 0;
                    for (int d = 0; d < nd; d++) jdv += R->Jr[d] * dv[d];
                    for (int i = 0; i < 6; i++) jdv += R->Jc[i] * dvc[i];
                    double delta = R->rhs - jdv * R->jinv;
                    double sum = R->lam + delta;
                    if (sum < R->lo) { delta = R->lo - R->lam; R->lam = R->lo; }
                    else if (sum > R->hi) { delta = R->hi - R->lam; R->lam = R->hi; }
                    else R->lam = sum;
                    for (int d = 0; d < nd; d++) dv[d] += R->Rr[d] * delta;
                    for (int i = 0; i < 6; i++) dvc[i] += R->Rc[i] * delta;
                    double res = R->jinv != 0.0 ? delta / R->jinv : 0.0;
                    if (res * res > resid) resid = res * res;
                }
            }
        }
        it_used = it + 1;
        if (!(p->flags & PGX_FLAG_NO_RESIDUAL_EXIT) && resid <= p->residual_threshold) break;
    }
    if (st) st->solver_iterations = it_used;
    PGXO_HIST_ADD(pgxo_diag_hist, it_used < 63 ? it_used : 63, 1);
    if (diag_trace && diag_trace_pos < diag_trace_cap) diag_trace[diag_trace_pos++] = it_used;
    PGXO_HIST_ADD(pgxo_diag_hist, 64 + (ncon < 15 ? ncon : 15), 1);
    {
        int lim = 0, rob = 0;
        for (int r = 0; r < nr; r++) lim |= m->row_kind[r] != PGX_ROW_MOTOR && lam[r] != 0.0;
        for (int c2 = 0; c2 < ncon; c2++) rob |= con[c2].grp != 0;
        PGXO_HIST_ADD(pgxo_diag_hist, 112, lim); PGXO_HIST_ADD(pgxo_diag_hist, 113, rob); PGXO_HIST_ADD(pgxo_diag_hist, 114, lim && rob);
    }
    PGXO_PHASE(5);
    double vn[D];
    for (int d = 0; d < nd; d++) vn[d] = clampd(vu[d] + dv[d], -p->max_coord_vel, p->max_coord_vel);
    if (p->flags & PGX_FLAG_CONSTRAINT_PASS_BIAS) {
        double bv[D], x[D];
        bias(m, p, &k, vu, 0, 1, bv);
        for (int d = 0; d < nd; d++) bv[d] = -bv[d];
        chol_solve(nd, Lm, bv, x);
        for (int d = 0; d < nd; d++) vn[d] = clampd(vn[d] + dt * x[d], -p->max_coord_vel, p->max_coord_vel);
    }
    for (int d = 0; d < nd; d++) {
        qd[d] = vn[d];
        q[d] += dt * vn[d];
    }
    for (int c = 0; c < ncon; c++)   /* persistent manifold: the applied impulse back to its point */
        if (con[c].mp) con[c].mp[MP_IMP] = cr[3 * c].lam;
    if (W) { /* contact cache: this step's features and normal impulses, per group */
        double* cache = obj + OBJ_CACHE;
        for (int s = 0; s < N_CACHE; s++) { cache[2 * s] = -1.0; cache[2 * s + 1] = 0.0; }
        int used[2] = {0, 0};
        for (int c = 0; c < ncon; c++) {
            int g = con[c].grp != 0, s = used[g]++;
            cache[2 * PGX_OBJECT_POINTS * g + 2 * s] = con[c].id;
            cache[2 * PGX_OBJECT_POINTS * g + 2 * s + 1] = cr[3 * c].lam;
        }
    }
    if (has_obj) {
        double* pos = obj;
        double* qt = obj + 3;
        double* v = obj + 7;
        double* w = obj + 10;
        for (int i = 0; i < 3; i++) {
            v[i] = vcu[i] + dvc[i];
            w[i] = wcu[i] + dvc[3 + i];
            pos[i] += dt * v[i];
        }
        /* btMultiBody::stepPositionsMultiDof, base: exponential map of w dt */
        double ang = v3_norm(w), ax[3];
        if (ang * dt > 0.25 * 1.5707963267948966) ang = 0.25 * 1.5707963267948966 / dt;
        double f = ang < 0.001 ? (0.5 * dt - dt * dt * dt * 0.020833333333 * ang * ang) : sin(0.5 * ang * dt) / ang;
        for (int i = 0; i < 3; i++) ax[i] = w[i] * f;
        double dq[4] = {ax[0], ax[1], ax[2], cos(ang * dt * 0.5)}, nq[4];
        quat_mul(dq, qt, nq);
        double nn = sqrt(nq[0] * nq[0] + nq[1] * nq[1] + nq[2] * nq[2] + nq[3] * nq[3]);
        for (int i = 0; i < 4; i++) qt[i] = nq[i] / nn;
    }
}

void pgxo_substep(const pgx_model* m, const pgx_sim_params* p, const double base[3], double* q, double* qd,
                  const pgxo_motor* motors, pgxo_stats* st) {
    substep_impl(m, p, base, q, qd, motors, st, NULL, NULL);
}

/* Bullet's contact breaking threshold per pair (btCollisionDispatcher::getNewManifold: with
 * CD_USE_RELATIVE_CONTACT_BREAKING_THRESHOLD, which btCollisionDispatcher's constructor sets and
 * pybullet keeps, the smaller of the two collision shapes' getContactBreakingThreshold(
 * gContactBreakingThreshold); btCollisionShape::getContactBreakingThreshold = getAngularMotionDisc()
 * x that, getAngularMotionDisc = the bounding sphere of the shape's AABB at the identity, radius
 * |max - min| / 2, plus |its centre|).  The shapes: a robot link's compound (pgx_model.link_aabb_*,
 * child and compound margins included), and the scene's createMultiBody boxes and spheres, each a
 * URDF-importer compound of one child at its origin (AABB half extents + the compound margin 0.001):
 * the table and the plane (create_plane: half extents 3 x 3 x 0.01, pybullet.py:759-778), the cube
 * (object_half), the obstacles (sphere radius / cuboid half extent 0.05, reach_ao.py:819-860).
 * PGX_FLAG_GLOBAL_BREAKING: the global contact_distance for every pair (rounds 2-5). */
#define URDF_COMPOUND_MARGIN 0.001
static double box_disc(double hx, double hy, double hz) {
    const double a = hx + URDF_COMPOUND_MARGIN, b = hy + URDF_COMPOUND_MARGIN, c = hz + URDF_COMPOUND_MARGIN;
    return sqrt(a * a + b * b + c * c);
}
static double dmin2(double a, double b) { return a < b ? a : b; }
/* (model constants, not per-step work: the operation-counting build leaves them out of the count) */
#ifndef PGXO_CONST_BEGIN
#define PGXO_CONST_BEGIN ((void)0)
#define PGXO_CONST_END ((void)0)
#endif
static void breaking_thresholds(const pgx_config* c, world_t* W) {
    PGXO_CONST_BEGIN;
    const pgx_model* m = c->model;
    const double tau = c->params->contact_distance;
    const int rel = !(c->params->flags & PGX_FLAG_GLOBAL_BREAKING);
    const double t_table = rel ? box_disc(c->table_half[0], c->table_half[1], c->table_half[2]) * tau : tau;
    const double t_plane = rel ? box_disc(3.0, 3.0, 0.01) * tau : tau;
    const double t_cube = rel ? box_disc(c->object_half, c->object_half, c->object_half) * tau : tau;
    const double t_obst = rel ? box_disc(0.05, 0.05, 0.05) * tau : tau;
    for (int ci = 0; ci < m->n_capsules; ci++) {
        const int li = m->cap_link[ci];
        double t_link = tau;
        if (rel && li >= 0) t_link = (v3_norm(m->link_aabb_half[li]) + v3_norm(m->link_aabb_center[li])) * tau;
        W->tau_table[ci] = dmin2(t_link, t_table);
        W->tau_plane[ci] = dmin2(t_link, t_plane);
        W->tau_cube[ci] = dmin2(t_link, t_cube);
        W->tau_obst[ci] = dmin2(t_link, t_obst);
    }
    W->tau_cube_table = dmin2(t_cube, t_table);
    W->tau_cube_plane = dmin2(t_cube, t_plane);
    PGXO_CONST_END;
}

/* test entry point: out[4 * PGX_MAX_CAPSULES + 2] = the table, plane, cube and obstacle thresholds per
 * capsule, then the cube's against the table and the plane */
void pgxo_breaking_thresholds(const pgx_config* c, double* out) {
    world_t W;
    memset(&W, 0, sizeof W);
    breaking_thresholds(c, &W);
    for (int i = 0; i < PGX_MAX_CAPSULES; i++) {
        out[i] = W.tau_table[i];
        out[PGX_MAX_CAPSULES + i] = W.tau_plane[i];
        out[2 * PGX_MAX_CAPSULES + i] = W.tau_cube[i];
        out[3 * PGX_MAX_CAPSULES + i] = W.tau_obst[i];
    }
    out[4 * PGX_MAX_CAPSULES] = W.tau_cube_table;
    out[4 * PGX_MAX_CAPSULES + 1] = W.tau_cube_plane;
}

static void world_of(const pgx_config* c, world_t* W) {
    breaking_thresholds(c, W);
    W->contacts = c->contacts;
    W->has_object = c->task == PGX_TASK_PUSH || c->task == PGX_TASK_PICK_AND_PLACE;
    W->half = c->object_half;
    W->mass = c->object_mass;
    W->inertia = c->object_inertia;
    for (int i = 0; i < 3; i++) { W->tc[i] = c->table_center[i]; W->th[i] = c->table_half[i]; }
    W->plane_z = c->plane_z;
    W->obst = NULL;
    W->robot_points = c->contacts != PGX_CONTACTS_FULL ? PGX_ROBOT_POINTS_ONE_LANE
                    : (W->has_object ? PGX_ROBOT_POINTS : PGX_ROBOT_POINTS_ARM);
}

void pgxo_world_substep(const pgx_config* c, double* q, double* qd, double* obj, const pgxo_motor* motors,
                        pgxo_stats* st) {
    world_t W;
    world_of(c, &W);
    W.obst = c->task == PGX_TASK_REACH_AO ? obj + OBJ_AO : NULL;
    substep_impl(c->model, c->params, c->base_pos, q, qd, motors, st, &W, obj);
}

/* ------------------------------------------------------------------- IK */
/* btMatrix3x3::getRotation */
static void mat_to_quat(const double* m, double* qo) {
    double tr = m[0] + m[4] + m[8];
    double t[4];
    if (tr > 0.0) {
        double s = sqrt(tr + 1.0);
        t[3] = s * 0.5;
        s = 0.5 / s;
        t[0] = (m[7] - m[5]) * s;
        t[1] = (m[2] - m[6]) * s;
        t[2] = (m[3] - m[1]) * s;
    } else {
        int i = m[0] < m[4] ? (m[4] < m[8] ? 2 : 1) : (m[0] < m[8] ? 2 : 0);
        int j = (i + 1) % 3, kk = (i + 2) % 3;
        double s = sqrt(m[i * 3 + i] - m[j * 3 + j] - m[kk * 3 + kk] + 1.0);
        t[i] = s * 0.5;
        s = 0.5 / s;
        t[3] = (m[kk * 3 + j] - m[j * 3 + kk]) * s;
        t[j] = (m[j * 3 + i] + m[i * 3 + j]) * s;
        t[kk] = (m[kk * 3 + i] + m[i * 3 + kk]) * s;
    }
    memcpy(qo, t, sizeof t);
}
static void quat_mul(const double* a, const double* b, double* o) { /* (x,y,z,w) Hamilton */
    double x = a[3] * b[0] + a[0] * b[3] + a[1] * b[2] - a[2] * b[1];
    double y = a[3] * b[1] + a[1] * b[3] + a[2] * b[0] - a[0] * b[2];
    double z = a[3] * b[2] + a[2] * b[3] + a[0] * b[1] - a[1] * b[0];
    double w = a[3] * b[3] - a[0] * b[0] - a[1] * b[1] - a[2] * b[2];
    o[0] = x; o[1] = y; o[2] = z; o[3] = w;
}

/* PyBullet.inverse_kinematics (panda_gym/pybullet.py:465-493) ->
 * calculateInverseKinematics with a target orientation: Bullet's
 * IKTrajectoryHelper::computeIK, IK2_VEL_DLS_WITH_ORIENTATION, iterated
 * maxNumIterations=20 times from the current joint positions while the
 * end-effector position error (measured before each update) exceeds
 * residualThreshold=1e-4.  The IK point is the link's joint pivot (the
 * inverse-dynamics tree body origin = URDF link frame origin), not the COM
 * that getLinkState reports.  Each iteration: 6xn Jacobian of that point,
 * e = [target - pos; angle*axis of target*current^-1] (angle kept in float),
 * dq = (J^T J + 0.5 I)^-1 J^T e, scaled to max|dq| <= pi/4, q += dq. */
int pgxo_ik(const pgx_model* m, const pgx_sim_params* p, const double base[3], const double* q_start, int link,
            const double target_pos[3], const double target_orn[4], double* q_out, pgxo_stats* st) {
    int nd = m->n_dofs;
    double qs[D];
    memcpy(qs, q_start, sizeof(double) * nd);
    double diff = 1e30;
    int it = 0;
    /* the target orientation goes through a btTransform (normalising it) */
    double tn = sqrt(target_orn[0] * target_orn[0] + target_orn[1] * target_orn[1] + target_orn[2] * target_orn[2] +
                     target_orn[3] * target_orn[3]);
    double torn[4] = {target_orn[0] / tn, target_orn[1] / tn, target_orn[2] / tn, target_orn[3] / tn};
    const double PI_ = 3.1415926535897932384626433832795028841972;
    for (it = 0; it < p->ik_max_iters && diff > p->ik_residual; it++) {
        kin_t k;
        fk(m, base, qs, &k);
        const double* pt = (p->flags & PGX_FLAG_IK_COM) ? k.p[link] : k.o[link];
        double Jv[3 * D], Jw[3 * D];
        jacobian(m, &k, link, pt, Jv, Jw);
        /* base frame (base rotation is identity in every reference env) */
        double pos[3] = {pt[0] - base[0], pt[1] - base[1], pt[2] - base[2]};
        double tgt[3] = {target_pos[0] - base[0], target_pos[1] - base[1], target_pos[2] - base[2]};
        double cur_q[4], dq4[4], inv_cur[4];
        mat_to_quat(k.R[link], cur_q);
        inv_cur[0] = -cur_q[0]; inv_cur[1] = -cur_q[1]; inv_cur[2] = -cur_q[2]; inv_cur[3] = cur_q[3];
        quat_mul(torn, inv_cur, dq4);
        double wq = clampd(dq4[3], -1.0, 1.0);
        float angle = (float)(2.0 * acos(wq));
        double ax[3];
        double s2 = 1.0 - dq4[3] * dq4[3];
        if (s2 < 10.0 * 2.220446049250313e-16) {
            ax[0] = 1; ax[1] = 0; ax[2] = 0;
        } else {
            double s = 1.0 / sqrt(s2);
            ax[0] = dq4[0] * s; ax[1] = dq4[1] * s; ax[2] = dq4[2] * s;
        }
        double an = v3_norm(ax);
        ax[0] /= an; ax[1] /= an; ax[2] /= an;
        if (angle > PI_) angle = (float)(angle - 2.0 * PI_);
        else if (angle < -PI_) angle = (float)(angle + 2.0 * PI_);
        double e[6] = {tgt[0] - pos[0], tgt[1] - pos[1], tgt[2] - pos[2],
                       (double)angle * ax[0], (double)angle * ax[1], (double)angle * ax[2]};
        /* U = J^T J + damping; dT1 = J^T e; U dtheta = dT1 (Jacobian::CalcDeltaThetasDLS2) */
        double U[D * D], rhs_[D], Lm[D * D], dth[D];
        for (int a = 0; a < nd; a++) {
            double s = 0;
            for (int r = 0; r < 3; r++) s += Jv[r * nd + a] * e[r] + Jw[r * nd + a] * e[3 + r];
            rhs_[a] = s;
            for (int bb = 0; bb < nd; bb++) {
                double u = 0;
                for (int r = 0; r < 3; r++) u += Jv[r * nd + a] * Jv[r * nd + bb] + Jw[r * nd + a] * Jw[r * nd + bb];
                U[a * nd + bb] = u + (a == bb ? p->ik_damping : 0.0);
            }
        }
        memset(Lm, 0, sizeof Lm);
        chol(nd, U, Lm);
        chol_solve(nd, Lm, rhs_, dth);
        double mx = 0;
        for (int a = 0; a < nd; a++) mx = fabs(dth[a]) > mx ? fabs(dth[a]) : mx;
        if (mx > p->ik_max_angle)
            for (int a = 0; a < nd; a++) dth[a] *= p->ik_max_angle / mx;
        for (int a = 0; a < nd; a++) q_out[a] = qs[a] + dth[a];
        const double res3[3] = {pos[0] - tgt[0], pos[1] - tgt[1], pos[2] - tgt[2]};
        diff = v3_norm(res3);
        memcpy(qs, q_out, sizeof(double) * nd);
    }
    if (it == 0) memcpy(q_out, q_start, sizeof(double) * nd);
    if (st) { st->ik_iterations = it; st->ik_residual = diff; }
    PGXO_HIST_ADD(pgxo_diag_hist, 80 + (it < 31 ? it : 31), 1);
    return it;
}

/* ---------------------------------------------------------------- reward */
/* utils.distance (panda_gym/utils.py:4-16): norm then np.round(d, 6), computed
 * in float64 when the goal is float64 (RobotTaskEnv.step passes the f64 goal,
 * core.py:358,366). np.round = rint(x*1e6)/1e6. */
double pgxo_distance_f32_f64(const float ag[3], const double g[3]) {
    double d0 = (double)ag[0] - g[0], d1 = (double)ag[1] - g[1], d2 = (double)ag[2] - g[2];
    double d = sqrt(d0 * d0 + d1 * d1 + d2 * d2);
    return rint(d * 1e6) / 1e6;
}
/* Same on two float32 arrays (HER relabel: compute_reward(ag_f32, dg_f32)):
 * numpy keeps float32 throughout (norm = sqrt of pairwise-summed squares). */
float pgxo_distance_f32_f32(const float ag[3], const float g[3]) {
    float d0 = ag[0] - g[0], d1 = ag[1] - g[1], d2 = ag[2] - g[2];
    float s = (d0 * d0 + d1 * d1) + d2 * d2;
    float d = sqrtf(s);
    float y = rintf(d * 1e6f);
    return y / 1e6f;
}
void pgxo_compute_reward_f32(const float* ag, const float* dg, int64_t n, int reward_type, double thr, float* out) {
    for (int64_t i = 0; i < n; i++) {
        float d = pgxo_distance_f32_f32(ag + 3 * i, dg + 3 * i);
        /* numpy compares a float32 array with a Python float in float32 */
        if (reward_type == PGX_REWARD_SPARSE_AO) out[i] = -1.0f + (d < (float)thr ? 1.0f : 0.0f);
        else if (reward_type == PGX_REWARD_SPARSE) out[i] = -(d > (float)thr ? 1.0f : 0.0f);
        else out[i] = -d;
    }
}

static int obs_dim(const pgx_config* c);
static int action_dim(const pgx_config* c);

/* ------------------------------------------------------------------ RNG */
void pgxo_philox(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
    uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3], k0 = key[0], k1 = key[1];
    for (int r = 0; r < 10; r++) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0, hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        c0 = hi1 ^ c1 ^ k0; c1 = lo1; c2 = hi0 ^ c3 ^ k1; c3 = lo0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

#define TAG_RESET 0x52455345u
#define TAG_ACTION 0x41435430u

/* k-th uniform double of the reset draws of (env, episode): (u64 >> 11) * 2^-53
 * like numpy's random_standard_uniform, so goal = low + (high-low)*u. */
static double reset_uniform(const pgx_config* c, uint64_t env, uint32_t episode, int kidx) {
    uint32_t ctr[4] = {(uint32_t)env, (uint32_t)(env >> 32), episode, TAG_RESET + (uint32_t)(kidx >> 1)};
    uint32_t key[2] = {(uint32_t)c->seed, (uint32_t)(c->seed >> 32)};
    uint32_t o[4];
    pgxo_philox(ctr, key, o);
    uint64_t u = (kidx & 1) ? ((uint64_t)o[2] | ((uint64_t)o[3] << 32)) : ((uint64_t)o[0] | ((uint64_t)o[1] << 32));
    return (double)(u >> 11) * (1.0 / 9007199254740992.0);
}

void pgxo_sample_actions(const pgx_config* c, int64_t n, uint64_t step, float* action) {
    int A = action_dim(c);
    uint32_t key[2] = {(uint32_t)c->seed, (uint32_t)(c->seed >> 32)};
    for (int64_t e = 0; e < n; e++) {
        uint64_t env = c->env_id_offset + (uint64_t)e;
        for (int a = 0; a < A; a++) {
            uint32_t ctr[4] = {(uint32_t)env, (uint32_t)(env >> 32), (uint32_t)step,
                               TAG_ACTION + ((uint32_t)(step >> 32) << 4) + (uint32_t)(a >> 2)};
            uint32_t o[4];
            pgxo_philox(ctr, key, o);
            uint32_t u = o[a & 3];
            action[e * A + a] = (float)(u >> 8) * (1.0f / 16777216.0f) * 2.0f - 1.0f;
        }
    }
}

/* --------------------------------------------------------- env semantics */
static int obs_dim(const pgx_config* c) {
    if (c->task == PGX_TASK_REACH_AO) return 20 + 4 * PGX_AO_LINKS;   /* obs_type ("ee","js") + 36 */
    int robot = 6 + (c->block_gripper ? 0 : 1);
    int task = (c->task == PGX_TASK_REACH) ? 0 : 12;
    return robot + task;
}
static int action_dim(const pgx_config* c) {
    int a = (c->control == PGX_CONTROL_EE) ? 3 : 7;
    return a + (c->block_gripper ? 0 : 1);
}

/* pybullet getEulerFromQuaternion (PyBullet.get_base_rotation, pybullet.py:216-219) */
static void quat_to_euler(const double* q, double* rpy) {
    double sqx = q[0] * q[0], sqy = q[1] * q[1], sqz = q[2] * q[2], squ = q[3] * q[3];
    double sarg = -2.0 * (q[0] * q[2] - q[3] * q[1]);
    rpy[1] = sarg <= -1.0 ? -0.5 * 3.141592538 : (sarg >= 1.0 ? 0.5 * 3.141592538 : asin(sarg));
    rpy[0] = atan2(2.0 * (q[1] * q[2] + q[3] * q[0]), squ - sqx - sqy + sqz);
    rpy[2] = atan2(2.0 * (q[0] * q[1] + q[3] * q[2]), squ + sqx - sqy - sqz);
}

/* RobotTaskEnv._get_obs (core.py:286-296): robot obs (panda.py:264-288) + task obs
 * (push.py:49-63 / pick_and_place.py:52-59: object position, euler, velocity, angular
 * velocity); achieved goal = EE position (Reach) or object position (Push/PnP). */
static void ao_obs(const pgx_config* c, const double* q, const double* qd, const double* qc, const double* goal,
                   const double* obst, float* obs, float* ag, float* dg);
static void ao_reset_one(const pgx_config* c, int64_t e, const double* inject_goal, const double* inject_obst,
                         double* q, double* qd, double* goal, double* obj, int32_t* elapsed, uint32_t* episode);
static int ao_collided(const pgx_config* c, const double* q, const double* obst);

/* getLinkState(ee_link, computeLinkVelocity=1) (PyBullet.get_link_position / _velocity,
 * pybullet.py:249-286; Panda.get_ee_position / _velocity, panda.py:306-312) without
 * computeForwardKinematics reads the link's cached world transform, which Bullet refreshes
 * (btMultiBodyDynamicsWorld::forwardKinematics) before the constraint solve of each
 * stepSimulation -- i.e. at the pose qc *before* the last substep's position update -- and
 * turns the link's local velocity (compTreeLinkVelocities: the current q and qd) into world
 * coordinates with that cached rotation.  resetJointState refreshes it (qc = q).  So:
 *   position = COM of the link at qc,  velocity = R(qc) R(q)^T v(q, qd).
 * Pinned by the reference's own known answers (test/pybullet_test.py:139-170): after one
 * env step of joint 6, link 5's orientation [0.707, -0.02, 0.02, 0.707] and COM velocity
 * [-0.0068, 0, 0.1186] are those of the cached pose (q of substep 19: y = -0.02005,
 * v_x = -0.00677), while the joint angle (:190-204, getJointState: current) is 0.063 --
 * the three answers are inconsistent with link states at the current pose (y -0.0222,
 * v_x -0.0075).  tests/test_oracle_known_answers.py. */
static void link_state_cached(const pgx_config* c, const double* q, const double* qd, const double* qc, int link,
                              double pos[3], double vel[3]) {
    const pgx_model* m = c->model;
    if (c->params->flags & PGX_FLAG_LINKSTATE_CURRENT) qc = q;
    kin_t k, kc;
    fk(m, c->base_pos, q, &k);
    fk(m, c->base_pos, qc, &kc);
    double v[3], w[3], vl[3];
    link_vel(m, &k, qd, link, v, w);
    for (int i = 0; i < 3; i++)   /* R(q)^T v: the local velocity */
        vl[i] = k.R[link][i] * v[0] + k.R[link][3 + i] * v[1] + k.R[link][6 + i] * v[2];
    m3_v(kc.R[link], vl, vel);
    memcpy(pos, kc.p[link], 3 * sizeof(double));
}

static void env_obs(const pgx_config* c, const double* q, const double* qd, const double* goal, const double* obj,
                    float* obs, float* ag, float* dg) {
    if (c->task == PGX_TASK_REACH_AO) { ao_obs(c, q, qd, obj ? obj + OBJ_QC : q, goal, obj + OBJ_AO, obs, ag, dg); return; }
    const pgx_model* m = c->model;
    double ee[3], v[3];
    link_state_cached(c, q, qd, obj ? obj + OBJ_QC : q, m->ee_link, ee, v);
    float o[32];
    int n = 0;
    for (int i = 0; i < 3; i++) o[n++] = (float)ee[i];
    for (int i = 0; i < 3; i++) o[n++] = (float)v[i];
    if (!c->block_gripper) o[n++] = 0.0f; /* fixed finger joints in custom_0: width 0 */
    const int has_obj = c->task != PGX_TASK_REACH;
    if (has_obj) {
        double rpy[3];
        quat_to_euler(obj + 3, rpy);
        for (int i = 0; i < 3; i++) o[n++] = (float)obj[i];
        for (int i = 0; i < 3; i++) o[n++] = (float)rpy[i];
        for (int i = 0; i < 3; i++) o[n++] = (float)obj[7 + i];
        for (int i = 0; i < 3; i++) o[n++] = (float)obj[10 + i];
    }
    if (obs) memcpy(obs, o, sizeof(float) * n);
    if (ag) for (int i = 0; i < 3; i++) ag[i] = (float)(has_obj ? obj[i] : ee[i]);
    if (dg) for (int i = 0; i < 3; i++) dg[i] = (float)goal[i];
}

/* Panda.reset (panda.py:290-298) + Task.reset: Reach reach.py:63-78, Push push.py:69-87,
 * PickAndPlace pick_and_place.py:65-85 -- draws in the reference's order: goal noise
 * (3), PickAndPlace's random() < 0.3 (1), object noise (3).  The object is re-posed
 * with identity orientation; its velocity is kept (resetBasePositionAndOrientation). */
static void reset_one(const pgx_config* c, int64_t e, const double* inject_goal, const double* inject_obj, double* q,
                      double* qd, double* goal, double* obj, int32_t* elapsed, uint32_t* episode) {
    if (c->task == PGX_TASK_REACH_AO) {
        ao_reset_one(c, e, inject_goal, inject_obj, q, qd, goal, obj, elapsed, episode);
        return;
    }
    int nd = c->model->n_dofs;
    for (int d = 0; d < nd; d++) { q[d] = c->neutral_q[d]; qd[d] = 0.0; }
    uint64_t env = c->env_id_offset + (uint64_t)e;
    double noise[3];
    for (int i = 0; i < 3; i++)
        noise[i] = c->goal_low[i] + (c->goal_high[i] - c->goal_low[i]) * reset_uniform(c, env, *episode, i);
    int kk = 3;
    if (c->task == PGX_TASK_PICK_AND_PLACE) {
        if (reset_uniform(c, env, *episode, kk) < c->goal_z_zero_prob) noise[2] = 0.0;
        kk++;
    }
    for (int i = 0; i < 3; i++) goal[i] = inject_goal ? inject_goal[i] : c->goal_offset[i] + noise[i];
    if (c->task != PGX_TASK_REACH && obj) {
        for (int i = 0; i < 3; i++) {
            double nz = c->obj_low[i] + (c->obj_high[i] - c->obj_low[i]) * reset_uniform(c, env, *episode, kk + i);
            obj[i] = inject_obj ? inject_obj[i] : c->obj_offset[i] + nz;
        }
        obj[3] = 0.0; obj[4] = 0.0; obj[5] = 0.0; obj[6] = 1.0;
    }
    if (obj) {
        for (int s = 0; s < N_CACHE; s++) { obj[OBJ_CACHE + 2 * s] = -1.0; obj[OBJ_CACHE + 2 * s + 1] = 0.0; }
        memcpy(obj + OBJ_QC, q, 7 * sizeof(double));   /* resetJointState refreshes the link cache */
        /* a reset teleports the bodies: Bullet's broadphase drops the pairs that stop overlapping, and
         * the next refresh the points of any other (they separate far beyond the 0.02 threshold) */
        memset(obj + OBJ_MAN, 0, (1 + PGXO_POOL_MAX * MAN_PT) * sizeof(double));
    }
    *elapsed = 0;
    *episode += 1;
}

int pgxo_vec_reset(const pgx_config* c, int64_t n, const uint8_t* mask, const double* inject_goal,
                   const double* inject_obj, double* q, double* qd, double* goal, double* obj, int32_t* elapsed,
                   uint32_t* episode, float* obs, float* ag, float* dg) {
    int nd = c->model->n_dofs, od = obs_dim(c);
    PGXO_PHASE(7);
    for (int64_t e = 0; e < n; e++) {
        if (mask && !mask[e]) continue;
        double* oe = obj ? obj + OBJ_N * e : NULL;
        const int io = c->task == PGX_TASK_REACH_AO ? 3 * PGX_AO_OBSTACLES : 3;
        reset_one(c, e, inject_goal ? inject_goal + 3 * e : NULL, inject_obj ? inject_obj + io * e : NULL, q + nd * e,
                  qd + nd * e, goal + 3 * e, oe, elapsed + e, episode + e);
        env_obs(c, q + nd * e, qd + nd * e, goal + 3 * e, oe, obs ? obs + od * e : NULL, ag ? ag + 3 * e : NULL,
                dg ? dg + 3 * e : NULL);
    }
    return PGX_OK;
}

/* ======================================================== ReachAO ("reachao_rand")
 * reach_ao.py with TrainConfig defaults (classes/train_config.py): joint control,
 * obs_type ("ee","js"), task obs "vectors+closest_per_link", truncate on collision,
 * terminate on success, sparse reward with collision_reward -100, 20 substeps with a
 * collision check after each (step_check_collision :182-188).  Distances restate
 * pyb_utils' CollisionDetector (a fork, absent here) on the capsule geometry
 * (Model.capsules, the URDF's cylinder+sphere unions) against sphere / box
 * obstacles: signed distances (negative when penetrating), closest point pairs. */
static const int kAoKind[PGX_AO_OBSTACLES] = {0, 0, 0, 1, 1, 1};   /* 3 spheres, then 3 cuboids */
static uint32_t pgxo_errors;   /* PGX_ERR_* of the device errors word, set by the resets */
uint32_t pgxo_take_errors(void) {
    uint32_t e = pgxo_errors;
    pgxo_errors = 0;
    return e;
}
#define AO_SIZE 0.05          /* sphere radius / cuboid half extent (create_scenario_reachao3/_rand) */
#define AO_DUMMY_R 0.05       /* the goal's dummy sphere (reach_ao.py:281-287) */
#define AO_MARGIN 0.001       /* btBoxShape collision margin of createCollisionShape boxes: the
                                 box is its inner box (h - m) swept by a sphere of radius m */
#define AO_PI 3.14159265358979323846
static const int kAoLinks[PGX_AO_LINKS] = {0, 1, 2, 3, 4, 5, 6, 7, 9};  /* link1..8, panda_ee */

/* signed distance of P to the axis-aligned box (c, h): negative inside */
static double box_sd(const double* P, const double* c, const double* h) {
    double o = 0.0, in = -1e300;
    for (int i = 0; i < 3; i++) {
        double di = fabs(P[i] - c[i]) - h[i];
        if (di > 0) o += di * di;
        if (di > in) in = di;
    }
    return sqrt(o) + (in < 0 ? in : 0.0);
}

static cdist_t capsule_sphere(const double* A, const double* B, double r, const double* C, double R) {
    double ab[3] = {B[0] - A[0], B[1] - A[1], B[2] - A[2]}, l2 = v3_dot(ab, ab), t = 0.0, P[3], v[3];
    if (l2 > 0) t = clampd(((C[0] - A[0]) * ab[0] + (C[1] - A[1]) * ab[1] + (C[2] - A[2]) * ab[2]) / l2, 0.0, 1.0);
    for (int i = 0; i < 3; i++) { P[i] = A[i] + t * ab[i]; v[i] = C[i] - P[i]; }
    double len = v3_norm(v), n[3] = {0, 0, 1};
    if (len > 0) for (int i = 0; i < 3; i++) n[i] = v[i] / len;
    cdist_t o;
    o.d = len - r - R;
    for (int i = 0; i < 3; i++) { o.pa[i] = P[i] + r * n[i]; o.pb[i] = C[i] - R * n[i]; o.n[i] = n[i]; }
    return o;
}

/* signed distance to the rounded box (c, h) with margin AO_MARGIN */
static double rbox_sd(const double* P, const double* c, const double* h) {
    const double hi[3] = {h[0] - AO_MARGIN, h[1] - AO_MARGIN, h[2] - AO_MARGIN};
    return box_sd(P, c, hi) - AO_MARGIN;
}

/* capsule vs rounded axis-aligned box: the signed distance to the inner box is convex
 * along the segment, minimised by 40 ternary-search steps ((2/3)^40 ~ 1e-7 of the
 * segment); the margin and the capsule radius are then subtracted */
static cdist_t capsule_box(const double* A, const double* B, double r, const double* c, const double* hfull) {
    const double h[3] = {hfull[0] - AO_MARGIN, hfull[1] - AO_MARGIN, hfull[2] - AO_MARGIN};
    double ab[3] = {B[0] - A[0], B[1] - A[1], B[2] - A[2]}, lo = 0.0, hi = 1.0, P[3];
    if (v3_dot(ab, ab) > 0) {
        for (int it = 0; it < 40; it++) {
            double m1 = lo + (hi - lo) / 3.0, m2 = hi - (hi - lo) / 3.0, P1[3], P2[3];
            for (int i = 0; i < 3; i++) { P1[i] = A[i] + m1 * ab[i]; P2[i] = A[i] + m2 * ab[i]; }
            if (box_sd(P1, c, h) <= box_sd(P2, c, h)) hi = m2;
            else lo = m1;
        }
    }
    double t = 0.5 * (lo + hi);
    if (!(v3_dot(ab, ab) > 0)) t = 0.0;
    for (int i = 0; i < 3; i++) P[i] = A[i] + t * ab[i];
    double sd = box_sd(P, c, h), q[3], n[3];
    if (sd > 0) {
        /* two alternating projections (box -> segment): the search cannot resolve t where
         * the distance is flat to second order (a segment passing an edge or a corner);
         * each projection can only shorten the pair (|P' - q| <= |P - q|) and pins it */
        for (int it = 0; it < 2 && v3_dot(ab, ab) > 0; it++) {
            for (int i = 0; i < 3; i++) q[i] = clampd(P[i], c[i] - h[i], c[i] + h[i]);
            double tq = clampd(((q[0] - A[0]) * ab[0] + (q[1] - A[1]) * ab[1] + (q[2] - A[2]) * ab[2]) / v3_dot(ab, ab),
                               0.0, 1.0);
            for (int i = 0; i < 3; i++) P[i] = A[i] + tq * ab[i];
        }
        sd = box_sd(P, c, h);
        for (int i = 0; i < 3; i++) q[i] = clampd(P[i], c[i] - h[i], c[i] + h[i]);
        double v[3] = {q[0] - P[0], q[1] - P[1], q[2] - P[2]}, len = v3_norm(v);
        for (int i = 0; i < 3; i++) n[i] = len > 0 ? v[i] / len : 0.0;
    } else { /* inside: through the nearest face */
        int ax = 0;
        double best = -1e300;
        for (int i = 0; i < 3; i++) {
            double di = fabs(P[i] - c[i]) - h[i];
            if (di > best) { best = di; ax = i; }
        }
        memcpy(q, P, sizeof q);
        double sg = P[ax] < c[ax] ? -1.0 : 1.0;
        q[ax] = c[ax] + sg * h[ax];
        n[0] = n[1] = n[2] = 0.0;
        n[ax] = -sg;   /* from the capsule axis towards the box interior */
    }
    cdist_t o;
    o.d = sd - AO_MARGIN - r;
    for (int i = 0; i < 3; i++) { o.pa[i] = P[i] + r * n[i]; o.pb[i] = q[i] - AO_MARGIN * n[i]; o.n[i] = n[i]; }
    return o;
}

static void capsule_world(const pgx_model* m, const kin_t* k, const double* base, int ci, double* A, double* B) {
    int li = m->cap_link[ci];
    if (li < 0) {
        for (int i = 0; i < 3; i++) { A[i] = base[i] + m->cap_a[ci][i]; B[i] = base[i] + m->cap_b[ci][i]; }
        return;
    }
    m3_v(k->R[li], m->cap_a[ci], A);
    m3_v(k->R[li], m->cap_b[ci], B);
    for (int i = 0; i < 3; i++) { A[i] += k->o[li][i]; B[i] += k->o[li][i]; }
}

static cdist_t capsule_obstacle(const double* A, const double* B, double r, int kind, const double* C) {
    if (kind == 0) return capsule_sphere(A, B, r, C, AO_SIZE);
    const double h[3] = {AO_SIZE, AO_SIZE, AO_SIZE};
    return capsule_box(A, B, r, C, h);
}

static cdist_t ao_capsule_obstacle(const double* A, const double* B, double r, int o, const double* obst) {
    return capsule_obstacle(A, B, r, kAoKind[o], obst + 3 * o);
}
/* capsule axis to obstacle centre, minus the capsule radius and the sphere radius / the
 * rounded cube's circumradius: <= the pair's distance */
static double ao_pair_lower_bound(const double* A, const double* B, double r, int o, const double* obst) {
    const cdist_t axis = capsule_sphere(A, B, 0.0, obst + 3 * o, 0.0);
    return axis.d - r - (kAoKind[o] == 0 ? AO_SIZE : AO_SIZE * 1.7320508075688772);
}

static void table_box(const pgx_config* c, double* tc, double* th) {
    for (int i = 0; i < 3; i++) { tc[i] = c->table_center[i]; th[i] = c->table_half[i]; }
}

/* CollisionDetector.compute_distances_per_link: per collision link, the closest obstacle
 * (distance, point pair); returns the table distance of links 2..ee (check_collided) */
static double ao_link_distances(const pgx_config* c, const kin_t* k, const double* obst, double* dist,
                                double (*pa)[3], double (*pb)[3]) {
    const pgx_model* m = c->model;
    double tc[3], th[3], dtable = 1e300;
    table_box(c, tc, th);
    for (int l = 0; l < PGX_AO_LINKS; l++) {
        dist[l] = 1e300;
        for (int ci = 0; ci < m->n_capsules; ci++) {
            if (m->cap_link[ci] != kAoLinks[l]) continue;
            double A[3], B[3];
            capsule_world(m, k, c->base_pos, ci, A, B);
            for (int o = 0; o < PGX_AO_OBSTACLES; o++) {
                cdist_t cd = capsule_obstacle(A, B, m->cap_radius[ci], kAoKind[o], obst + 3 * o);
                if (cd.d < dist[l]) {
                    dist[l] = cd.d;
                    memcpy(pa[l], cd.pa, sizeof cd.pa);
                    memcpy(pb[l], cd.pb, sizeof cd.pb);
                }
            }
            if (kAoLinks[l] >= 1) {   /* get_link_object_distance(table, ignore link0, link1) */
                cdist_t ct = capsule_box(A, B, m->cap_radius[ci], tc, th);
                if (ct.d < dtable) dtable = ct.d;
            }
        }
    }
    return dtable;
}

/* check_collided (reach_ao.py:896-900): min over the collision links of the obstacle
 * distance <= 0, or of the table distance of links 2..ee.  Only the decision is needed, so a
 * pair whose lower bound is already > 0 is not measured (the decision is the same as with
 * every distance computed, which ao_obs does): capsule vs obstacle -- the distance from the
 * capsule axis to the obstacle centre minus the radius / the rounded cube's circumradius and
 * the capsule radius; capsule vs table -- the signed distance of the rounded box is
 * 1-Lipschitz, so along the axis it is >= min(sd(A), sd(B)) - |AB| / 2. */
static int ao_collided(const pgx_config* c, const double* q, const double* obst) {
    const pgx_model* m = c->model;
    kin_t k;
    fk(m, c->base_pos, q, &k);
    double tc[3], th[3];
    table_box(c, tc, th);
    const double circum = AO_SIZE * 1.7320508075688772;   /* sqrt(3) * half extent */
    for (int l = 0; l < PGX_AO_LINKS; l++) {
        for (int ci = 0; ci < m->n_capsules; ci++) {
            if (m->cap_link[ci] != kAoLinks[l]) continue;
            double A[3], B[3];
            capsule_world(m, &k, c->base_pos, ci, A, B);
            const double r = m->cap_radius[ci];
            for (int o = 0; o < PGX_AO_OBSTACLES; o++) {
                const double* C = obst + 3 * o;
                const cdist_t axis = capsule_sphere(A, B, 0.0, C, 0.0);   /* axis to centre */
                if (axis.d - r - (kAoKind[o] == 0 ? AO_SIZE : circum) > 0.0) continue;
                if (capsule_obstacle(A, B, r, kAoKind[o], C).d <= 0.0) return 1;
            }
            if (kAoLinks[l] >= 1) {
                double ab[3] = {B[0] - A[0], B[1] - A[1], B[2] - A[2]};
                double sa = rbox_sd(A, tc, th), sb = rbox_sd(B, tc, th);
                if ((sa < sb ? sa : sb) - 0.5 * v3_norm(ab) - r > 0.0) continue;
                if (capsule_box(A, B, r, tc, th).d <= 0.0) return 1;
            }
        }
    }
    return 0;
}

/* whole-robot (every capsule incl. base and hand) distance to a sphere (kind 0) / box (1) */
static double ao_robot_distance(const pgx_config* c, const kin_t* k, int kind, const double* C, double size) {
    const pgx_model* m = c->model;
    double best = 1e300;
    for (int ci = 0; ci < m->n_capsules; ci++) {
        double A[3], B[3];
        capsule_world(m, k, c->base_pos, ci, A, B);
        cdist_t cd;
        if (kind == 0) cd = capsule_sphere(A, B, m->cap_radius[ci], C, size);
        else {
            const double h[3] = {size, size, size};
            cd = capsule_box(A, B, m->cap_radius[ci], C, h);
        }
        if (cd.d < best) best = cd.d;
    }
    return best;
}

/* sample_within_hollow_sphere (reach_ao.py:1188-1211): phi, theta, r = cbrt(U(rmin^3, rmax^3)) */
typedef struct { const pgx_config* c; uint64_t env; uint32_t episode; int k; } draw_t;
static double ao_draw(draw_t* d) { return reset_uniform(d->c, d->env, d->episode, d->k++); }
static double ao_uniform(draw_t* d, double lo, double hi) { return lo + (hi - lo) * ao_draw(d); }
static void hollow_sphere(draw_t* d, double rmin, double rmax, int upper_half_only, double* out) {
    double phi = ao_uniform(d, 0.0, 2.0 * AO_PI);
    double theta = upper_half_only ? ao_uniform(d, 0.0, 0.5 * AO_PI) : ao_uniform(d, 0.0, AO_PI);
    double r = cbrt(ao_uniform(d, pow(rmin, 3.0), pow(rmax, 3.0)));   /* Python's radius ** 3 */
    out[0] = r * sin(theta) * cos(phi);
    out[1] = r * sin(theta) * sin(phi);
    out[2] = r * cos(theta);
}

/* ReachAO.reset for "reachao_rand" (reach_ao.py:965-1033): collision-free goal
 * (set_coll_free_goal(["table","robot"]), margin 0.1), collision-free obstacles
 * (set_coll_free_obs(0.03), sample_obstacle_experimental), then 4 or 5 active obstacles
 * (set_random_num_obs: integers(4, 6), shuffle, the first ones moved to (99.9,99.9,-99.9)).
 * Device-stream draws (the host reproduces the numpy stream for seeded resets). */
static void ao_reset_task(const pgx_config* c, int64_t e, uint32_t episode, const double* q, double* goal,
                          double* obst, double* active) {
    draw_t d = {c, c->env_id_offset + (uint64_t)e, episode, 0};
    kin_t k;
    fk(c->model, c->base_pos, q, &k);
    double tc[3], th[3];
    table_box(c, tc, th);
    const double* ee = k.p[c->model->ee_link];
    double dummy[3];   /* the dummy sphere stays at the last tested sample */
    for (int i = 0;; i++) {
        hollow_sphere(&d, 0.5, 0.8, 1, goal);
        if (i > 9999) { memcpy(goal, ee, 3 * sizeof(double)); break; }   /* the 10001st draw is discarded */
        memcpy(dummy, goal, sizeof dummy);
        int coll = rbox_sd(goal, tc, th) - AO_DUMMY_R <= 0.1 ||
                   ao_robot_distance(c, &k, 0, goal, AO_DUMMY_R) <= 0.1;
        if (!coll) break;
    }
    for (int o = 0; o < PGX_AO_OBSTACLES; o++) {
        double* P = obst + 3 * o;
        int placed = 0;
        for (int it = 0; it < 10000; it++) {
            double rnd = ao_draw(&d), s[3];
            hollow_sphere(&d, 0.1, 0.5, 0, s);
            const double* ctr = rnd > 0.5 ? goal : ee;
            for (int j = 0; j < 3; j++) P[j] = s[j] + ctr[j];
            double dtab, ddum;
            if (kAoKind[o] == 0) {
                dtab = rbox_sd(P, tc, th) - AO_SIZE;
                double v[3] = {P[0] - dummy[0], P[1] - dummy[1], P[2] - dummy[2]};
                ddum = v3_norm(v) - AO_SIZE - AO_DUMMY_R;
            } else {
                /* rounded box vs rounded box: inner AABBs' gap minus both margins */
                double hs[3] = {th[0] + AO_SIZE - 2 * AO_MARGIN, th[1] + AO_SIZE - 2 * AO_MARGIN,
                                th[2] + AO_SIZE - 2 * AO_MARGIN};
                const double h[3] = {AO_SIZE, AO_SIZE, AO_SIZE};
                dtab = box_sd(P, tc, hs) - 2 * AO_MARGIN;
                ddum = rbox_sd(dummy, P, h) - AO_DUMMY_R;
            }
            int coll = ao_robot_distance(c, &k, kAoKind[o], P, AO_SIZE) <= 0.03 || dtab <= 0.03 || ddum <= 0.03;
            if (!coll) { placed = 1; break; }
        }
        /* set_coll_free_obs raises StopIteration on the 10001st attempt (reach_ao.py:1143-1145):
         * the last draw stays, the sticky error word records it (pgxo_take_errors) */
        if (!placed) pgxo_errors |= PGX_ERR_AO_OBSTACLE;
        active[o] = 1.0;
    }
    int n_active = 4 + (int)(ao_draw(&d) * 2.0);           /* integers(4, 6) */
    int perm[PGX_AO_OBSTACLES];
    for (int o = 0; o < PGX_AO_OBSTACLES; o++) perm[o] = o;
    for (int j = PGX_AO_OBSTACLES - 1; j > 0; j--) {        /* Fisher-Yates */
        int r = (int)(ao_draw(&d) * (double)(j + 1));
        if (r > j) r = j;
        int t = perm[j]; perm[j] = perm[r]; perm[r] = t;
    }
    for (int j = 0; j < PGX_AO_OBSTACLES - n_active; j++) {
        double* P = obst + 3 * perm[j];
        P[0] = 99.9; P[1] = 99.9; P[2] = -99.9;
        active[perm[j]] = 0.0;
    }
}

/* robot obs (ee pos, ee vel, q, qd) + closest distance per link (9) + unit vectors (27) */
static void ao_obs(const pgx_config* c, const double* q, const double* qd, const double* qc, const double* goal,
                   const double* obst, float* obs, float* ag, float* dg) {
    const pgx_model* m = c->model;
    kin_t k;
    fk(m, c->base_pos, q, &k);
    double ee[3], v[3];   /* "ee" obs from getLinkState (cached pose); distances at the current pose */
    link_state_cached(c, q, qd, qc, m->ee_link, ee, v);
    float o[64];
    int n = 0;
    for (int i = 0; i < 3; i++) o[n++] = (float)ee[i];
    for (int i = 0; i < 3; i++) o[n++] = (float)v[i];
    for (int i = 0; i < 7; i++) o[n++] = (float)q[i];
    for (int i = 0; i < 7; i++) o[n++] = (float)qd[i];
    double dist[PGX_AO_LINKS], pa[PGX_AO_LINKS][3], pb[PGX_AO_LINKS][3];
    ao_link_distances(c, &k, obst, dist, pa, pb);
    for (int l = 0; l < PGX_AO_LINKS; l++) o[n++] = (float)dist[l];
    for (int l = 0; l < PGX_AO_LINKS; l++) {   /* utils.unit_vector(point on link, point on obstacle) */
        double u[3] = {pb[l][0] - pa[l][0], pb[l][1] - pa[l][1], pb[l][2] - pa[l][2]}, len = v3_norm(u);
        for (int i = 0; i < 3; i++) o[n++] = (float)(len > 0 ? u[i] / len : 0.0);
    }
    if (obs) memcpy(obs, o, sizeof(float) * n);
    if (ag) for (int i = 0; i < 3; i++) ag[i] = (float)ee[i];
    if (dg) for (int i = 0; i < 3; i++) dg[i] = (float)goal[i];
}

static void ao_reset_one(const pgx_config* c, int64_t e, const double* inject_goal, const double* inject_obst,
                         double* q, double* qd, double* goal, double* obj, int32_t* elapsed, uint32_t* episode) {
    int nd = c->model->n_dofs;
    for (int d = 0; d < nd; d++) { q[d] = c->neutral_q[d]; qd[d] = 0.0; }
    double* obst = obj + OBJ_AO;
    double* active = obj + OBJ_AO + 3 * PGX_AO_OBSTACLES;
    ao_reset_task(c, e, *episode, q, goal, obst, active);
    if (inject_goal) memcpy(goal, inject_goal, 3 * sizeof(double));
    if (inject_obst)
        for (int o = 0; o < PGX_AO_OBSTACLES; o++) {
            memcpy(obst + 3 * o, inject_obst + 3 * o, 3 * sizeof(double));
            active[o] = inject_obst[3 * o] < 50.0 ? 1.0 : 0.0;
        }
    for (int s = 0; s < N_CACHE; s++) { obj[OBJ_CACHE + 2 * s] = -1.0; obj[OBJ_CACHE + 2 * s + 1] = 0.0; }
    memcpy(obj + OBJ_QC, q, 7 * sizeof(double));
    memset(obj + OBJ_MAN, 0, (1 + PGXO_POOL_MAX * MAN_PT) * sizeof(double));
    *elapsed = 0;
    *episode += 1;
}

double pgxo_ao_capsule_sphere(const double* A, const double* B, double r, const double* C, double R, double* pa,
                              double* pb) {
    cdist_t o = capsule_sphere(A, B, r, C, R);
    memcpy(pa, o.pa, sizeof o.pa);
    memcpy(pb, o.pb, sizeof o.pb);
    return o.d;
}
double pgxo_ao_capsule_box(const double* A, const double* B, double r, const double* c, const double* h, double* pa,
                           double* pb) {
    cdist_t o = capsule_box(A, B, r, c, h);
    memcpy(pa, o.pa, sizeof o.pa);
    memcpy(pb, o.pb, sizeof o.pb);
    return o.d;
}
double pgxo_ao_link_distances(const pgx_config* c, const double* q, const double* obst, double* dist, double* pa,
                              double* pb) {
    kin_t k;
    fk(c->model, c->base_pos, q, &k);
    return ao_link_distances(c, &k, obst, dist, (double(*)[3])pa, (double(*)[3])pb);
}
int pgxo_ao_collided(const pgx_config* c, const double* q, const double* obst) { return ao_collided(c, q, obst); }

/* check_collided's margin at q: min over the collision links of the obstacle distance and over
 * links 2..ee of the table distance (collided <=> margin <= 0), every distance measured */
static double ao_margin(const pgx_config* c, const double* q, const double* obst) {
    kin_t k;
    fk(c->model, c->base_pos, q, &k);
    double dist[PGX_AO_LINKS], pa[PGX_AO_LINKS][3], pb[PGX_AO_LINKS][3];
    double mg = ao_link_distances(c, &k, obst, dist, pa, pb);
    for (int l = 0; l < PGX_AO_LINKS; l++) mg = dist[l] < mg ? dist[l] : mg;
    return mg;
}
/* Diagnostics (tests): with a buffer set, pgxo_vec_step records per ReachAO env the collision
 * margin of every substep check that ran, as the smallest |margin| of the step -- how close the
 * step's collision decisions came to their threshold -- and the margin at the last check. */
static double* diag_margin_abs;
static double* diag_margin_last;
static int64_t diag_margin_n;
void pgxo_diag_collision_margin(double* min_abs, double* last, int64_t n) {
    diag_margin_abs = min_abs;
    diag_margin_last = last;
    diag_margin_n = n;
}

/* RobotTaskEnv.step (core.py:352-368) for one env + TimeLimit + VecEnv auto-reset */
int pgxo_vec_step(const pgx_config* c, int64_t n, double* q, double* qd, double* goal, double* obj, int32_t* elapsed,
                  uint32_t* episode, const float* action, float* obs, float* ag, float* dg, float* reward,
                  uint8_t* success, uint8_t* terminated, uint8_t* truncated, float* terminal_obs) {
    const pgx_model* m = c->model;
    const pgx_sim_params* p = c->params;
    int nd = m->n_dofs, A = action_dim(c), od = obs_dim(c);
    for (int64_t e = 0; e < n; e++) {
        double* qe = q + nd * e;
        double* qde = qd + nd * e;
        double* ge = goal + 3 * e;
        double* oe = obj + OBJ_N * e;
        PGXO_PHASE(0);
        /* Panda.set_action (panda.py:120-172): clip to the action space (float32) */
        float a[8];
        for (int i = 0; i < A; i++) {
            float x = action[e * A + i];
            a[i] = x < -1.0f ? -1.0f : (x > 1.0f ? 1.0f : x);
        }
        double tq[D];
        if (c->control == PGX_CONTROL_EE) {
            /* ee_displacement_to_target_arm_angles (panda.py:226-246): get_ee_position() is
             * getLinkState's cached pose (link_state_cached) */
            kin_t k;
            fk(m, c->base_pos, (p->flags & PGX_FLAG_LINKSTATE_CURRENT) ? qe : oe + OBJ_QC, &k);
            float step32 = (float)c->ee_step;
            double tgt[3];
            for (int i = 0; i < 3; i++) tgt[i] = k.p[m->ee_link][i] + (double)(a[i] * step32);
            tgt[2] = tgt[2] > 0.0 ? tgt[2] : 0.0;
            const double orn[4] = {1.0, 0.0, 0.0, 0.0};
            pgxo_ik(m, p, c->base_pos, qe, m->ee_link, tgt, orn, tq, NULL);
        } else {
            /* arm_joint_ctrl_to_target_arm_angles (panda.py:248-262) */
            float step32 = (float)c->joint_step;
            for (int i = 0; i < 7; i++) tq[i] = qe[i] + (double)(a[i] * step32);
        }
        /* control_joints POSITION_CONTROL (pybullet.py:437-455), forces panda.py:63 */
        pgxo_motor mot[D];
        for (int d = 0; d < nd; d++) {
            mot[d].target_q = tq[d];
            mot[d].target_qd = 0.0;
            mot[d].kp = p->motor_kp;
            mot[d].kd = p->motor_kd;
            mot[d].max_impulse = c->joint_forces[d] * p->dt;
        }
        const int ao = c->task == PGX_TASK_REACH_AO;
        int collided = 0;
        const int diag_m = ao && diag_margin_abs && e < diag_margin_n;
        if (diag_m) diag_margin_abs[e] = diag_margin_last[e] = 1e300;
        for (int s = 0; s < p->n_substeps; s++) {
            memcpy(oe + OBJ_QC, qe, 7 * sizeof(double));   /* the link cache: the pose this substep solves at */
            pgxo_world_substep(c, qe, qde, oe, mot, NULL);
            /* ReachAO step_check_collision (reach_ao.py:182-188) */
            PGXO_PHASE(8);
            if (diag_m) {
                const double mg = ao_margin(c, qe, oe + OBJ_AO);
                diag_margin_last[e] = mg;
                if (fabs(mg) < diag_margin_abs[e]) diag_margin_abs[e] = fabs(mg);
            }
            if (ao && ao_collided(c, qe, oe + OBJ_AO)) { collided = 1; break; }
        }
        PGXO_PHASE(6);

        float o[64], agv[3], dgv[3];
        env_obs(c, qe, qde, ge, oe, o, agv, dgv);
        double d = pgxo_distance_f32_f64(agv, ge);
        uint8_t succ = d < c->distance_threshold;
        float rew;
        if (ao) {
            /* ReachAO.compute_reward "sparse"/"reach" + collision_reward (reach_ao.py:1317-1377) */
            rew = -1.0f + ((d + (double)collided) < c->distance_threshold ? 1.0f : 0.0f);
            rew += (float)(collided * c->collision_reward);
        } else {
            rew = (c->reward == PGX_REWARD_SPARSE) ? -(d > c->distance_threshold ? 1.0f : 0.0f) : -(float)d;
        }
        elapsed[e] += 1;
        uint8_t trunc = (c->max_episode_steps > 0 && elapsed[e] >= c->max_episode_steps) || collided;
        /* terminate_on_success (core.py:359-361): False for Reach/Push/PnP, True in ReachAO's config */
        uint8_t term = c->terminate_on_success ? succ : 0;
        if (reward) reward[e] = rew;
        if (success) success[e] = succ;
        if (terminated) terminated[e] = term;
        if (truncated) truncated[e] = trunc;
        if (trunc || term) {
            if (terminal_obs) memcpy(terminal_obs + od * e, o, sizeof(float) * od);
        }
        if ((trunc || term) && !c->no_auto_reset) {
            PGXO_PHASE(7);
            reset_one(c, e, NULL, NULL, qe, qde, ge, oe, elapsed + e, episode + e);
            env_obs(c, qe, qde, ge, oe, o, agv, dgv);
        }
        if (obs) memcpy(obs + od * e, o, sizeof(float) * od);
        if (ag) memcpy(ag + 3 * e, agv, sizeof agv);
        if (dg) memcpy(dg + 3 * e, dgv, sizeof dgv);
    }
    return PGX_OK;
}
