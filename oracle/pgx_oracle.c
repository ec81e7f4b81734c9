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

/* ----------------------------------------------------------------- small vec */
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

/* One stepSimulation() of a fixed-base multibody with joint motors and joint
 * limits, no contacts (PyBullet.step pybullet.py:68-71 calls this 20x):
 *  1. unconstrained: qd += dt*qdd(q,qd), clamp |qd| <= maxCoordinateVelocity
 *     (btMultiBodyDynamicsWorld::solveExternalForces -> ABA + applyDeltaVeeMultiDof)
 *  2. constraint rows (btMultiBodyJointMotor / btMultiBodyJointLimitConstraint ::
 *     createConstraintRows) solved by projected Gauss-Seidel
 *     (btMultiBodyConstraintSolver::resolveSingleConstraintRowGeneric), rows in the
 *     world's sorted order, reversed on even iterations, stop when the max squared
 *     row residual <= residual_threshold or after num_iterations
 *  3. qd += M^-1 J^T lambda (constraint pass), q += dt*qd (stepPositionsMultiDof). */
void pgxo_substep(const pgx_model* m, const pgx_sim_params* p, const double base[3], double* q, double* qd,
                  const pgxo_motor* motors, pgxo_stats* st) {
    int nd = m->n_dofs;
    double dt = p->dt;
    kin_t k;
    fk(m, base, q, &k);
    double M[D * D], Lm[D * D], b[D], qdd[D], Minv[D * D];
    mass_matrix(m, &k, M);
    bias(m, p, &k, qd, 1, 1, b);
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

    /* --- constraint rows */
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
            for (int k = 0; k < nd; k++) B += fabs(Minv[d * nd + k]) * (motors[k].max_impulse);
            B = B * 1.001 + 1e-6;
            double penl = q[d] - m->lower[d], penu = m->upper[d] - q[d];
            far = far && penl > 0 && penu > 0 && (vu[d] - B) > -penl / dt && (vu[d] + B) < penu / dt;
        }
        st->limits_far = far;
    }
    double dv[D] = {0};
    int it_used = 0;
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
        it_used = it + 1;
        if (!(p->flags & PGX_FLAG_NO_RESIDUAL_EXIT) && resid <= p->residual_threshold) break;
    }
    if (st) st->solver_iterations = it_used;
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
        diff = v3_norm((double[3]){pos[0] - tgt[0], pos[1] - tgt[1], pos[2] - tgt[2]});
        memcpy(qs, q_out, sizeof(double) * nd);
    }
    if (it == 0) memcpy(q_out, q_start, sizeof(double) * nd);
    if (st) { st->ik_iterations = it; st->ik_residual = diff; }
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
        if (reward_type == PGX_REWARD_SPARSE) out[i] = -(d > (float)thr ? 1.0f : 0.0f);
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
    int robot = 6 + (c->block_gripper ? 0 : 1);
    int task = (c->task == PGX_TASK_REACH) ? 0 : 12;
    return robot + task;
}
static int action_dim(const pgx_config* c) {
    int a = (c->control == PGX_CONTROL_EE) ? 3 : 7;
    return a + (c->block_gripper ? 0 : 1);
}

static void env_obs(const pgx_config* c, const double* q, const double* qd, const double* goal, float* obs, float* ag,
                    float* dg) {
    const pgx_model* m = c->model;
    kin_t k;
    fk(m, c->base_pos, q, &k);
    double v[3], w[3];
    link_vel(m, &k, qd, m->ee_link, v, w);
    float o[32];
    int n = 0;
    for (int i = 0; i < 3; i++) o[n++] = (float)k.p[m->ee_link][i];
    for (int i = 0; i < 3; i++) o[n++] = (float)v[i];
    if (!c->block_gripper) o[n++] = 0.0f; /* fixed finger joints in custom_0: width 0 */
    if (obs) memcpy(obs, o, sizeof(float) * n);
    if (ag) for (int i = 0; i < 3; i++) ag[i] = (float)k.p[m->ee_link][i];
    if (dg) for (int i = 0; i < 3; i++) dg[i] = (float)goal[i];
}

static void reset_one(const pgx_config* c, int64_t e, const double* inject_goal, double* q, double* qd, double* goal,
                      int32_t* elapsed, uint32_t* episode) {
    int nd = c->model->n_dofs;
    for (int d = 0; d < nd; d++) { q[d] = c->neutral_q[d]; qd[d] = 0.0; }
    uint64_t env = c->env_id_offset + (uint64_t)e;
    for (int i = 0; i < 3; i++) {
        if (inject_goal) goal[i] = inject_goal[i];
        else goal[i] = c->goal_low[i] + (c->goal_high[i] - c->goal_low[i]) * reset_uniform(c, env, *episode, i);
    }
    *elapsed = 0;
    *episode += 1;
}

int pgxo_vec_reset(const pgx_config* c, int64_t n, const uint8_t* mask, const double* inject_goal,
                   const double* inject_obj, double* q, double* qd, double* goal, double* obj, int32_t* elapsed,
                   uint32_t* episode, float* obs, float* ag, float* dg) {
    (void)inject_obj; (void)obj;
    if (c->task != PGX_TASK_REACH) return PGX_E_UNSUPPORTED;
    int nd = c->model->n_dofs, od = obs_dim(c);
    for (int64_t e = 0; e < n; e++) {
        if (mask && !mask[e]) continue;
        reset_one(c, e, inject_goal ? inject_goal + 3 * e : NULL, q + nd * e, qd + nd * e, goal + 3 * e, elapsed + e,
                  episode + e);
        env_obs(c, q + nd * e, qd + nd * e, goal + 3 * e, obs ? obs + od * e : NULL, ag ? ag + 3 * e : NULL,
                dg ? dg + 3 * e : NULL);
    }
    return PGX_OK;
}

/* RobotTaskEnv.step (core.py:352-368) for one env + TimeLimit + VecEnv auto-reset */
int pgxo_vec_step(const pgx_config* c, int64_t n, double* q, double* qd, double* goal, double* obj, int32_t* elapsed,
                  uint32_t* episode, const float* action, float* obs, float* ag, float* dg, float* reward,
                  uint8_t* success, uint8_t* terminated, uint8_t* truncated, float* terminal_obs) {
    (void)obj;
    if (c->task != PGX_TASK_REACH) return PGX_E_UNSUPPORTED;
    const pgx_model* m = c->model;
    const pgx_sim_params* p = c->params;
    int nd = m->n_dofs, A = action_dim(c), od = obs_dim(c);
    for (int64_t e = 0; e < n; e++) {
        double* qe = q + nd * e;
        double* qde = qd + nd * e;
        double* ge = goal + 3 * e;
        /* Panda.set_action (panda.py:120-172): clip to the action space (float32) */
        float a[8];
        for (int i = 0; i < A; i++) {
            float x = action[e * A + i];
            a[i] = x < -1.0f ? -1.0f : (x > 1.0f ? 1.0f : x);
        }
        double tq[D];
        if (c->control == PGX_CONTROL_EE) {
            /* ee_displacement_to_target_arm_angles (panda.py:226-246) */
            kin_t k;
            fk(m, c->base_pos, qe, &k);
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
        for (int s = 0; s < p->n_substeps; s++) pgxo_substep(m, p, c->base_pos, qe, qde, mot, NULL);

        float o[32], agv[3], dgv[3];
        env_obs(c, qe, qde, ge, o, agv, dgv);
        double d = pgxo_distance_f32_f64(agv, ge);
        uint8_t succ = d < c->distance_threshold;
        float rew = (c->reward == PGX_REWARD_SPARSE) ? -(d > c->distance_threshold ? 1.0f : 0.0f) : -(float)d;
        elapsed[e] += 1;
        uint8_t trunc = (c->max_episode_steps > 0 && elapsed[e] >= c->max_episode_steps);
        uint8_t term = 0; /* terminate_on_success=False for Reach/Push/PnP (core.py:265) */
        if (reward) reward[e] = rew;
        if (success) success[e] = succ;
        if (terminated) terminated[e] = term;
        if (truncated) truncated[e] = trunc;
        if (trunc || term) {
            if (terminal_obs) memcpy(terminal_obs + od * e, o, sizeof(float) * od);
            reset_one(c, e, NULL, qe, qde, ge, elapsed + e, episode + e);
            env_obs(c, qe, qde, ge, o, agv, dgv);
        }
        if (obs) memcpy(obs + od * e, o, sizeof(float) * od);
        if (ag) memcpy(ag + 3 * e, agv, sizeof agv);
        if (dg) memcpy(dg + 3 * e, dgv, sizeof dgv);
    }
    return PGX_OK;
}
