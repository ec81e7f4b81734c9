/*
 * pgx_api.cpp -- C-ABI of libpgx.so (declared in include/pgx.h).
 *
 * Host side of the drop-in boundary: validates the robot model against the
 * topology the kernels are compiled for, folds the fixed links rigidly
 * attached to panda_link7 into one composite body (exact for inertia; their
 * COM offsets are kept for Bullet's per-link damping), owns one device
 * allocation holding the SoA state of all N envs, and launches the kernels on
 * the caller's stream.  Nothing here allocates or synchronises on the step path.
 */
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/pgx.h"
#include "pgx_default_model.h"
#include "pgx_dev.h"
#include "pgx_model_consts.h"
#include "pgx_rows.h"

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

int hip_check(hipError_t e, const char* what) {
    if (e != hipSuccess) return fail(PGX_E_HIP, "%s: %s", what, hipGetErrorString(e));
    return PGX_OK;
}

/* 3x3 helpers in double for model preprocessing */
void m3mul(const double* A, const double* B, double* C) {
    double t[9];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) t[i * 3 + j] = A[i * 3] * B[j] + A[i * 3 + 1] * B[3 + j] + A[i * 3 + 2] * B[6 + j];
    std::memcpy(C, t, sizeof t);
}
void m3v(const double* A, const double* v, double* o) {
    double t[3];
    for (int i = 0; i < 3; i++) t[i] = A[i * 3] * v[0] + A[i * 3 + 1] * v[1] + A[i * 3 + 2] * v[2];
    std::memcpy(o, t, sizeof t);
}

}  // namespace

int pgx_set_error(int code, const char* msg) {
    g_err = msg;
    return code;
}

struct pgx_env {
    int device;
    PgxDevModel dm;      /* host copy */
    PgxDevModel* dm_dev; /* device copy at the start of the state blob */
    PgxDevEnv de;
    PgxDevState ds;
    void* blob;
    size_t blob_bytes;
    /* device snapshots by id (pgx_snapshot): slot i holds state id i, nullptr = free */
    std::vector<void*> snaps;
    /* [N][PGX_PCG64_WORDS] numpy PCG64 streams of the reset draws (pgx_set_rng_streams) and, after them, the
     * device mode word (PgxDevEnv.pcg_on): allocated by pgx_create, freed by pgx_destroy, so a
     * graph captured in either mode never reads freed memory */
    uint64_t* pcg = nullptr;
    bool pcg_set = false;   /* host mirror of the mode word */
    int man_pool = 0;       /* persistent manifold pool capacity (0: none) */
    /* the step kernel the last pgx_step launched (pgx_step_kernel) */
    const char* step_kernel = nullptr;
};

extern "C" {

const char* pgx_version(void) { return "pgx 0.1.0 (gfx950)"; }
const char* pgx_last_error(void) { return g_err.c_str(); }

int pgx_obs_dim(const pgx_config* c) {
    if (!c) return PGX_E_INVALID;
    if (c->task == PGX_TASK_REACH_AO) return 20 + 4 * PGX_AO_LINKS;   /* ("ee","js") + vectors+closest_per_link */
    return 6 + (c->block_gripper ? 0 : 1) + (c->task == PGX_TASK_REACH ? 0 : 12);
}
int pgx_action_dim(const pgx_config* c) {
    if (!c) return PGX_E_INVALID;
    return (c->control == PGX_CONTROL_EE ? 3 : 7) + (c->block_gripper ? 0 : 1);
}

/* The kernel is specialised to the env robot at compile time (pgx_model_consts.h);
 * refuse a runtime model whose folded tables differ from the compiled ones. */
static int check_compiled_tables(const PgxDevModel& dm) {
    auto same = [](const float* a, const float* b, int n, const char* what) -> int {
        for (int i = 0; i < n; i++)
            if (std::fabs(a[i] - b[i]) > 1e-6f * std::fmax(1.0f, std::fabs(b[i])))
                return fail(PGX_E_UNSUPPORTED, "model table %s[%d] = %g differs from the compiled robot (%g)", what,
                            i, (double)a[i], (double)b[i]);
        return PGX_OK;
    };
    int rc = 0;
    rc = rc ? rc : same(&dm.jp[0][0], &kJp[0][0], 21, "jp");
    rc = rc ? rc : same(&dm.jr[0][0], &kJr[0][0], 63, "jr");
    rc = rc ? rc : same(&dm.com[0][0], &kCom[0][0], 21, "com");
    rc = rc ? rc : same(dm.mass, kMass, 7, "mass");
    rc = rc ? rc : same(&dm.inertia[0][0], &kInertia[0][0], 18, "inertia");
    rc = rc ? rc : same(dm.i6c, kI6c, 6, "i6c");
    rc = rc ? rc : same(dm.i6own, kI6own, 6, "i6own");
    if (!rc && dm.ndamp != PGX_NDAMP) rc = fail(PGX_E_UNSUPPORTED, "damped body count %d != %d", dm.ndamp, PGX_NDAMP);
    rc = rc ? rc : same(&dm.dpos[0][0], &kDpos[0][0], 3 * PGX_NDAMP, "dpos");
    rc = rc ? rc : same(dm.dmass, kDmass, PGX_NDAMP, "dmass");
    rc = rc ? rc : same(dm.ee_pivot, kEePivot, 3, "ee_pivot");
    rc = rc ? rc : same(dm.ee_rot, kEeRot, 9, "ee_rot");
    rc = rc ? rc : same(dm.ee_com, kEeCom, 3, "ee_com");
    rc = rc ? rc : same(dm.lower, kLower, 7, "lower");
    rc = rc ? rc : same(dm.upper, kUpper, 7, "upper");
    return rc;
}

/* The contact capsules folded onto the arm joints (link-7 group in link 7's frame)
 * must equal the compiled kCap* tables. */
static int check_capsules(const pgx_model* m, const double (*R)[9], const double (*O)[3]) {
    if (m->n_capsules != PGX_NCAP)
        return fail(PGX_E_UNSUPPORTED, "model has %d contact capsules, kernel %d", m->n_capsules, PGX_NCAP);
    const int last = PGX_NJ - 1;
    for (int c = 0; c < PGX_NCAP; c++) {
        int li = m->cap_link[c];
        int j = li < last ? li : last;
        double a[3], b[3];
        if (li > last) {
            m3v(R[li], m->cap_a[c], a);
            m3v(R[li], m->cap_b[c], b);
            for (int k = 0; k < 3; k++) { a[k] += O[li][k]; b[k] += O[li][k]; }
        } else {
            for (int k = 0; k < 3; k++) { a[k] = m->cap_a[c][k]; b[k] = m->cap_b[c][k]; }
        }
        bool ok = j == kCapJ[c] && m->cap_flags[c] == kCapFlags[c] &&
                  std::fabs(m->cap_radius[c] - kCapR[c]) <= 1e-6;
        for (int k = 0; k < 3; k++)
            ok = ok && std::fabs(a[k] - kCapA[c][k]) <= 1e-6 && std::fabs(b[k] - kCapB[c][k]) <= 1e-6;
        if (!ok) return fail(PGX_E_UNSUPPORTED, "contact capsule %d differs from the compiled robot", c);
    }
    return PGX_OK;
}

/* Fold the model into the kernel's constant tables. */
static int build_dev_model(const pgx_config* cfg, PgxDevModel* dm) {
    const pgx_model* m = cfg->model;
    const pgx_sim_params* p = cfg->params;
    std::memset(dm, 0, sizeof *dm);
    if (m->n_dofs != PGX_NJ) return fail(PGX_E_UNSUPPORTED, "kernel is built for 7 arm dofs, model has %d", m->n_dofs);
    for (int j = 0; j < PGX_NJ; j++) {
        if (m->parent[j] != j - 1 || m->jtype[j] != PGX_JOINT_REVOLUTE || m->dof_of_link[j] != j)
            return fail(PGX_E_UNSUPPORTED, "link %d is not the %d-th revolute joint of a serial chain", j, j);
        if (m->axis[j][0] != 0.0 || m->axis[j][1] != 0.0 || m->axis[j][2] != 1.0)
            return fail(PGX_E_UNSUPPORTED, "joint %d axis is not URDF z", j);
        if (!m->has_limit[j]) return fail(PGX_E_UNSUPPORTED, "joint %d has no limit constraint", j);
    }
    if (m->n_rows != PGX_N_ROWS) return fail(PGX_E_UNSUPPORTED, "model has %d solver rows, kernel %d", m->n_rows, PGX_N_ROWS);
    for (int r = 0; r < PGX_N_ROWS; r++)
        if (((m->row_kind[r] << 4) | m->row_dof[r]) != kPgxRowCode[r])
            return fail(PGX_E_UNSUPPORTED, "solver row %d differs from the compiled row order", r);
    if (m->ee_link < PGX_NJ || m->ee_link >= m->n_links) return fail(PGX_E_INVALID, "ee_link %d", m->ee_link);

    /* transforms of every fixed link relative to panda_link7's URDF frame */
    double R[PGX_MAX_LINKS][9], O[PGX_MAX_LINKS][3];
    const int last = PGX_NJ - 1;
    const double I9[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    std::memcpy(R[last], I9, sizeof I9);
    std::memset(O[last], 0, sizeof O[last]);
    for (int i = PGX_NJ; i < m->n_links; i++) {
        int par = m->parent[i];
        if (m->jtype[i] != PGX_JOINT_FIXED || par < last || par >= i)
            return fail(PGX_E_UNSUPPORTED, "link %d is not a fixed descendant of link %d", i, last);
        m3mul(R[par], m->jrot[i], R[i]);
        m3v(R[par], m->jpos[i], O[i]);
        for (int c = 0; c < 3; c++) O[i][c] += O[par][c];
    }
    /* composite of the link-7 group: mass, COM, inertia about COM, sum of own inertias */
    double mt = 0, cm[3] = {0, 0, 0};
    double comp[PGX_MAX_LINKS][3];
    for (int i = last; i < m->n_links; i++) {
        m3v(R[i], m->com[i], comp[i]);
        for (int c = 0; c < 3; c++) comp[i][c] += O[i][c];
        mt += m->mass[i];
        for (int c = 0; c < 3; c++) cm[c] += m->mass[i] * comp[i][c];
    }
    if (mt <= 0) return fail(PGX_E_INVALID, "link-7 group has no mass");
    for (int c = 0; c < 3; c++) cm[c] /= mt;
    double Ic[9] = {0}, Io[9] = {0};
    int nd = 0;
    for (int i = last; i < m->n_links; i++) {
        double mi = m->mass[i];
        if (mi == 0.0) continue;
        double Iw[9];
        for (int a = 0; a < 3; a++)
            for (int b = 0; b < 3; b++)
                Iw[a * 3 + b] = R[i][a * 3] * m->inertia[i][0] * R[i][b * 3] +
                                R[i][a * 3 + 1] * m->inertia[i][1] * R[i][b * 3 + 1] +
                                R[i][a * 3 + 2] * m->inertia[i][2] * R[i][b * 3 + 2];
        double r[3] = {comp[i][0] - cm[0], comp[i][1] - cm[1], comp[i][2] - cm[2]};
        double rr = r[0] * r[0] + r[1] * r[1] + r[2] * r[2];
        for (int a = 0; a < 3; a++)
            for (int b = 0; b < 3; b++) {
                Io[a * 3 + b] += Iw[a * 3 + b];
                Ic[a * 3 + b] += Iw[a * 3 + b] + mi * ((a == b ? rr : 0.0) - r[a] * r[b]);
            }
        if (nd >= PGX_MAX_DAMP) return fail(PGX_E_UNSUPPORTED, "too many massive bodies on link 7");
        for (int c = 0; c < 3; c++) dm->dpos[nd][c] = (float)comp[i][c];
        dm->dmass[nd] = (float)mi;
        nd++;
    }
    dm->ndamp = nd;
    auto pack = [](const double* S, float* o) {
        o[0] = (float)S[0]; o[1] = (float)S[4]; o[2] = (float)S[8];
        o[3] = (float)S[1]; o[4] = (float)S[2]; o[5] = (float)S[5];
    };
    pack(Ic, dm->i6c);
    pack(Io, dm->i6own);
    for (int j = 0; j < PGX_NJ; j++) {
        for (int c = 0; c < 3; c++) dm->jp[j][c] = (float)m->jpos[j][c];
        for (int c = 0; c < 9; c++) dm->jr[j][c] = (float)m->jrot[j][c];
        if (j < last) {
            for (int c = 0; c < 3; c++) dm->com[j][c] = (float)m->com[j][c];
            for (int c = 0; c < 3; c++) dm->inertia[j][c] = (float)m->inertia[j][c];
            dm->mass[j] = (float)m->mass[j];
        }
        dm->lower[j] = (float)m->lower[j];
        dm->upper[j] = (float)m->upper[j];
        dm->max_impulse[j] = (float)(cfg->joint_forces[j] * p->dt);
        dm->neutral_q[j] = (float)cfg->neutral_q[j];
    }
    for (int c = 0; c < 3; c++) dm->com[last][c] = (float)cm[c];
    dm->mass[last] = (float)mt;
    const int ee = m->ee_link;
    for (int c = 0; c < 3; c++) {
        dm->ee_pivot[c] = (float)O[ee][c];
        dm->ee_com[c] = (float)comp[ee][c];
        dm->base[c] = (float)cfg->base_pos[c];
        dm->gravity[c] = (float)p->gravity[c];
    }
    for (int c = 0; c < 9; c++) dm->ee_rot[c] = (float)R[ee][c];
    dm->dt = (float)p->dt;
    dm->inv_dt = (float)(1.0 / p->dt);
    dm->lin_damp = (float)p->lin_damping;
    dm->ang_damp = (float)p->ang_damping;
    dm->max_vel = (float)p->max_coord_vel;
    if (std::isnan(p->residual_threshold))
        return fail(PGX_E_INVALID, "residual_threshold is NaN");
    dm->residual_thr = (float)p->residual_threshold;
    if (!(dm->residual_thr > 0.0f)) {
        dm->residual_abs = 0.0f;           /* thr <= 0: only an exact zero residual exits */
    } else if (!std::isfinite(dm->residual_thr)) {
        dm->residual_abs = INFINITY;       /* +inf (or > FLT_MAX): every sweep exits */
    } else {
        /* fl(t * t) is monotone in t, so {t >= 0 : fl(t * t) <= thr} = [0, residual_abs];
         * sqrtf is within an ulp or two of that bound, so a bounded walk settles it */
        volatile float thr = dm->residual_thr, t = std::sqrt(thr);
        for (int i = 0; i < 8 && t > 0.0f && (float)(t * t) > thr; i++) t = std::nextafter((float)t, 0.0f);
        for (int i = 0; i < 8; i++) {
            volatile float u = std::nextafter((float)t, INFINITY);
            if (!((float)(u * u) <= thr)) break;
            t = u;
        }
        if ((float)(t * t) > thr) return fail(PGX_E_INVALID, "residual_threshold %g: no float bound", (double)thr);
        dm->residual_abs = t;
    }
    dm->erp = (float)p->erp;
    dm->limit_max_imp = (float)p->limit_max_impulse;
    dm->kp = (float)p->motor_kp;
    dm->kd = (float)p->motor_kd;
    dm->ik_residual = (float)p->ik_residual;
    dm->ik_damping = (float)p->ik_damping;
    dm->ik_max_angle = (float)p->ik_max_angle;
    dm->num_iterations = p->num_iterations;
    dm->ik_max_iters = p->ik_max_iters;
    dm->ee_step = (float)cfg->ee_step;
    dm->joint_step = (float)cfg->joint_step;
    dm->contact_dist = (float)p->contact_distance;
    dm->contact_erp = (float)p->contact_erp;
    dm->friction = (float)p->friction;
    dm->warmstart = (float)p->warmstart;
    for (int c = 0; c < m->n_capsules && c < 16; c++) {
        const int li = m->cap_link[c];
        dm->cap_mu[c] = (float)(li >= 0 && li < PGX_MAX_LINKS ? p->link_friction[li] : p->friction);
    }
    /* Bullet's contact breaking threshold per pair (btCollisionDispatcher::getNewManifold with its
     * default CD_USE_RELATIVE_CONTACT_BREAKING_THRESHOLD): the smaller of the two collision shapes'
     * angular motion disc (|AABB half extents| + |AABB centre|) x contact_distance.  The robot links'
     * compounds from the model (link_aabb_*); the scene's createMultiBody shapes are URDF-importer
     * compounds of one child at the origin (+ the compound margin 0.001): the table, the plane (half
     * extents 3 x 3 x 0.01, panda_gym/pybullet.py:759-778), the cube, the obstacles (0.05,
     * reach_ao.py:819-860).  The oracle restates the same (oracle/pgx_oracle.c breaking_thresholds). */
    {
        const double tau = p->contact_distance, mg = 0.001;
        auto box_disc = [&](double hx, double hy, double hz) {
            return std::sqrt((hx + mg) * (hx + mg) + (hy + mg) * (hy + mg) + (hz + mg) * (hz + mg));
        };
        auto nrm = [](const double* v) { return std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]); };
        const double t_table = box_disc(cfg->table_half[0], cfg->table_half[1], cfg->table_half[2]) * tau;
        const double t_plane = box_disc(3.0, 3.0, 0.01) * tau;
        const double t_obj = box_disc(cfg->object_half, cfg->object_half, cfg->object_half) * tau;
        const double t_obst = box_disc(0.05, 0.05, 0.05) * tau;
        for (int c = 0; c < 16; c++) {
            const int li = c < m->n_capsules ? m->cap_link[c] : -1;
            const double t_link = (li >= 0 && li < PGX_MAX_LINKS)
                                      ? (nrm(m->link_aabb_half[li]) + nrm(m->link_aabb_center[li])) * tau : tau;
            dm->tau_table[c] = (float)std::fmin(t_link, t_table);
            dm->tau_plane[c] = (float)std::fmin(t_link, t_plane);
            dm->tau_obj[c] = (float)std::fmin(t_link, t_obj);
            dm->tau_obst[c] = (float)std::fmin(t_link, t_obst);
        }
        dm->tau_obj_table = (float)std::fmin(t_obj, t_table);
        dm->tau_obj_plane = (float)std::fmin(t_obj, t_plane);
    }
    dm->table_cx = (float)cfg->table_center[0];   /* (the same values as PgxDevEnv's, pgx_create) */
    dm->table_cy = (float)cfg->table_center[1];
    dm->table_hx = (float)cfg->table_half[0];
    dm->table_hy = (float)cfg->table_half[1];
    dm->table_top = (float)(cfg->table_center[2] + cfg->table_half[2]);
    dm->plane_z = (float)cfg->plane_z;
    dm->table_hz = (float)cfg->table_half[2];
    dm->scene_pad = 0.0f;
    if (p->flags != 0) return fail(PGX_E_UNSUPPORTED, "modelling flags are oracle-only");
    int rc = check_compiled_tables(*dm);
    if (!rc) rc = check_capsules(m, R, O);
    return rc;
}

/* ReachAO reset geometry (PgxDevEnv.ao_geo): [PGX_NCAP][7] capsules (A, B, r) at the neutral pose,
 * then the table centre and half extents, fp64.  The capsules are the host's
 * (pgx_config.ao_capsules_neutral, the Python host's RobotGeometry) or, when those are all zero, an
 * fp64 FK of neutral_q here (panda-gym_amd/model.py forward_kinematics restated). */
static void ao_reset_geometry(const pgx_config* cfg, double* out) {
    const pgx_model* m = cfg->model;
    bool given = false;
    for (int c = 0; c < PGX_MAX_CAPSULES; c++)
        for (int k = 0; k < 7; k++) given = given || cfg->ao_capsules_neutral[c][k] != 0.0;
    if (given) {
        for (int c = 0; c < PGX_NCAP; c++)
            for (int k = 0; k < 7; k++) out[7 * c + k] = cfg->ao_capsules_neutral[c][k];
    } else {
        double R[PGX_MAX_LINKS][9], P[PGX_MAX_LINKS][3];
        const double I[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
        auto mul = [](const double* a, const double* b, double* o) {
            for (int i = 0; i < 3; i++)
                for (int j = 0; j < 3; j++) o[3 * i + j] = a[3 * i] * b[j] + a[3 * i + 1] * b[3 + j] + a[3 * i + 2] * b[6 + j];
        };
        for (int i = 0; i < m->n_links; i++) {
            const int p = m->parent[i];
            const double* pr = p < 0 ? I : R[p];
            const double* pp = p < 0 ? cfg->base_pos : P[p];
            double r[9];
            mul(pr, m->jrot[i], r);
            for (int k = 0; k < 3; k++)
                P[i][k] = pp[k] + pr[3 * k] * m->jpos[i][0] + pr[3 * k + 1] * m->jpos[i][1] + pr[3 * k + 2] * m->jpos[i][2];
            const int d = m->dof_of_link[i];
            if (d >= 0 && m->jtype[i] == PGX_JOINT_REVOLUTE) {
                const double* ax = m->axis[i];
                const double cq = std::cos(cfg->neutral_q[d]), sq = std::sin(cfg->neutral_q[d]);
                const double K[9] = {0, -ax[2], ax[1], ax[2], 0, -ax[0], -ax[1], ax[0], 0};
                double KK[9], rot[9];
                mul(K, K, KK);
                for (int k = 0; k < 9; k++) rot[k] = I[k] + sq * K[k] + (1.0 - cq) * KK[k];
                mul(r, rot, R[i]);
            } else {
                std::memcpy(R[i], r, sizeof r);
            }
        }
        for (int c = 0; c < PGX_NCAP; c++) {
            const int li = m->cap_link[c];
            for (int e = 0; e < 2; e++) {
                const double* a = e ? m->cap_b[c] : m->cap_a[c];
                for (int k = 0; k < 3; k++)
                    out[7 * c + 3 * e + k] = li < 0 ? cfg->base_pos[k] + a[k]
                                                    : R[li][3 * k] * a[0] + R[li][3 * k + 1] * a[1] + R[li][3 * k + 2] * a[2] + P[li][k];
            }
            out[7 * c + 6] = m->cap_radius[c];
        }
    }
    for (int k = 0; k < 3; k++) {
        out[7 * PGX_NCAP + k] = cfg->table_center[k];
        out[7 * PGX_NCAP + 3 + k] = cfg->table_half[k];
    }
}
#define PGX_AO_GEO_DOUBLES (7 * PGX_NCAP + 6)

/* Host only (no HIP call): the constant block pgx_create would upload for cfg, into out
 * (tools/gen_default_model.py generates the kernels' compile-time default blocks from it). */
int pgx_dev_model_bytes(const pgx_config* cfg, void* out, int64_t nbytes) {
    if (!cfg || !out || !cfg->model || !cfg->params) return fail(PGX_E_INVALID, "null argument");
    if (nbytes != (int64_t)sizeof(PgxDevModel))
        return fail(PGX_E_INVALID, "device model is %d bytes, got %lld", (int)sizeof(PgxDevModel), (long long)nbytes);
    PgxDevModel dm;
    const int rc = build_dev_model(cfg, &dm);
    if (rc) return rc;
    std::memcpy(out, &dm, sizeof dm);
    return PGX_OK;
}

int pgx_create(const pgx_config* cfg, int device, pgx_handle* out) {
    if (!cfg || !out || !cfg->model || !cfg->params) return fail(PGX_E_INVALID, "null argument");
    *out = nullptr;
    if (cfg->n_envs <= 0) return fail(PGX_E_INVALID, "n_envs must be > 0 (got %d)", cfg->n_envs);
    if (cfg->task != PGX_TASK_REACH && cfg->task != PGX_TASK_PUSH && cfg->task != PGX_TASK_PICK_AND_PLACE &&
        cfg->task != PGX_TASK_REACH_AO)
        return fail(PGX_E_UNSUPPORTED, "task %d is not implemented by this build", cfg->task);
    const bool has_object = cfg->task == PGX_TASK_PUSH || cfg->task == PGX_TASK_PICK_AND_PLACE;
    if (cfg->task == PGX_TASK_REACH_AO &&
        (cfg->control != PGX_CONTROL_JOINTS || !cfg->block_gripper || !cfg->contacts))
        return fail(PGX_E_UNSUPPORTED, "ReachAO is built for joint control, blocked gripper and the table scene");
    if (has_object && !cfg->contacts)
        return fail(PGX_E_INVALID, "object tasks need contacts");
    if (cfg->contacts < 0 || cfg->contacts > PGX_CONTACTS_FULL)
        return fail(PGX_E_INVALID, "contacts must be 0, 1 or PGX_CONTACTS_FULL, got %d", cfg->contacts);
    if (has_object && (cfg->object_half <= 0 || cfg->object_mass <= 0 || cfg->object_inertia <= 0))
        return fail(PGX_E_INVALID, "object size, mass and inertia must be > 0");
    if (cfg->control != PGX_CONTROL_EE && cfg->control != PGX_CONTROL_JOINTS)
        return fail(PGX_E_INVALID, "control %d", cfg->control);
    if (cfg->reward != PGX_REWARD_SPARSE && cfg->reward != PGX_REWARD_DENSE)
        return fail(PGX_E_INVALID, "reward %d", cfg->reward);
    if (cfg->params->n_substeps < 1 || cfg->params->n_substeps > 1000)
        return fail(PGX_E_INVALID, "n_substeps must be in [1, 1000], got %d", cfg->params->n_substeps);
    pgx_env* h = new pgx_env();
    h->device = device;
    int rc = build_dev_model(cfg, &h->dm);
    if (rc) { delete h; return rc; }
#ifndef PGX_RUNTIME_MODEL
    {   /* the kernels carry the constant block as a compile-time constant (pgx_default_model.h) */
        static_assert(sizeof(PgxDevModel) == 4 * PGX_DEV_MODEL_WORDS, "default model block size");
        const PgxDevModelWords& def = cfg->task == PGX_TASK_REACH_AO ? kDefModelAoWords : kDefModelArmWords;
        uint32_t got[PGX_DEV_MODEL_WORDS];
        std::memcpy(got, &h->dm, sizeof got);
        for (int i = 0; i < PGX_DEV_MODEL_WORDS; i++)
            if (got[i] != def.w[i]) {
                delete h;
                return fail(PGX_E_UNSUPPORTED,
                            "physics / robot parameters differ from the ones the kernels are compiled for "
                            "(constant block word %d: 0x%08x, compiled 0x%08x; tools/gen_default_model.py)",
                            i, got[i], def.w[i]);
            }
    }
#endif
    PgxDevEnv& e = h->de;
    e.pcg = nullptr;
    e.pcg_on = nullptr;
    e.perm_buf = nullptr;
    e.perm = nullptr;
    e.sort_mode = 0;   /* PGX_SORT_ENVS: 1 always, 0 never (A/B and test hook); unset: auto */
    if (const char* so = std::getenv("PGX_SORT_ENVS")) e.sort_mode = std::atoi(so) ? 1 : -1;
    e.sort_key = 1;    /* PGX_SORT_KEY=0: only the points past the register budget (A/B hook: PickAndPlace
                          16384 3.11 -> 3.73 ms, profiles/r04/ab_env_order_key.log) */
    if (const char* sk = std::getenv("PGX_SORT_KEY")) e.sort_key = std::atoi(sk) ? 1 : 0;
    e.sort_segs = 0;   /* PGX_SORT_SEGS=1: one global heavy-first order (A/B hook; default: per-XCD segments) */
    if (const char* sg = std::getenv("PGX_SORT_SEGS")) e.sort_segs = std::atoi(sg) == 1 ? 1 : 0;
    e.perm_segs = 1;
    e.task = cfg->task;
    e.control = cfg->control;
    e.reward = cfg->reward;
    e.n_envs = cfg->n_envs;
    e.max_episode_steps = cfg->max_episode_steps;
    e.block_gripper = cfg->block_gripper;
    e.obs_dim = pgx_obs_dim(cfg);
    e.action_dim = pgx_action_dim(cfg);
    e.seed = cfg->seed;
    e.env_id_offset = cfg->env_id_offset;
    e.distance_threshold = cfg->distance_threshold;
    for (int c = 0; c < 3; c++) { e.goal_low[c] = cfg->goal_low[c]; e.goal_high[c] = cfg->goal_high[c]; }
    for (int c = 0; c < 3; c++) {
        e.goal_offset[c] = cfg->goal_offset[c];
        e.obj_low[c] = cfg->obj_low[c];
        e.obj_high[c] = cfg->obj_high[c];
        e.obj_offset[c] = cfg->obj_offset[c];
    }
    e.goal_z_zero_prob = cfg->goal_z_zero_prob;
    e.contacts = cfg->contacts ? 1 : 0;
    e.full_manifold = cfg->contacts == PGX_CONTACTS_FULL ? 1 : 0;
    e.has_object = has_object;
    e.obj_half = (float)cfg->object_half;
    e.obj_inv_mass = e.has_object ? (float)(1.0 / cfg->object_mass) : 0.0f;
    e.obj_inv_inertia = e.has_object ? (float)(1.0 / cfg->object_inertia) : 0.0f;
    e.table_cx = (float)cfg->table_center[0];
    e.table_cy = (float)cfg->table_center[1];
    e.table_hx = (float)cfg->table_half[0];
    e.table_hy = (float)cfg->table_half[1];
    e.table_top = (float)(cfg->table_center[2] + cfg->table_half[2]);
    e.plane_z = (float)cfg->plane_z;
    e.table_hz = (float)cfg->table_half[2];
    e.ao = cfg->task == PGX_TASK_REACH_AO;
    e.terminate_on_success = cfg->terminate_on_success ? 1 : 0;
    e.no_auto_reset = cfg->no_auto_reset ? 1 : 0;
    e.collision_reward = cfg->collision_reward;
    for (int k = 0; k < 3; k++) e.ao_ee[k] = cfg->ao_ee_neutral[k];
    e.ao_ee_set = (cfg->ao_ee_neutral[0] != 0.0 || cfg->ao_ee_neutral[1] != 0.0 || cfg->ao_ee_neutral[2] != 0.0) ? 1 : 0;
    /* Step layout (pgx_kernels.hip): 16 lanes per env (4096 x 16 lanes = 1024 waves = one per
     * SIMD; beyond, several per SIMD) or one lane per env.  Round 1 measured the one-lane layout
     * ahead at 16384 envs (profiles/r01/time_layouts_v11.json: 1.33 vs 2.27 ms Reach, 3.54 vs
     * 5.49 PickAndPlace); the round-2 wide kernels reversed that for the contact tasks (below).
     * cfg->lanes_per_env (0 = this rule, 1, 16) chooses; PGX_LANES_PER_ENV=1|16 overrides both
     * (A/B timing). */
    if (cfg->lanes_per_env != 0 && cfg->lanes_per_env != 1 && cfg->lanes_per_env != 16) {
        delete h;
        return fail(PGX_E_INVALID, "lanes_per_env must be 0, 1 or 16, got %d", cfg->lanes_per_env);
    }
    /* test hook for the exactness of the speculative limit-row skip (substep_g) */
    e.pgs_mode = 0;
    if (const char* pm = std::getenv("PGX_PGS_MODE")) e.pgs_mode = std::atoi(pm);
    e.n_substeps = cfg->params->n_substeps;
    e.wave_mode = 0;
    if (const char* wm = std::getenv("PGX_WAVES_PER_SIMD")) e.wave_mode = std::atoi(wm);
    /* Round-2 measurements (tools/time_layouts.py, profiles/r02/time_layouts_r02.json): with
     * contacts the wide layout now wins at every batch -- Reach 16384 0.99 vs 1.29 ms, 65536
     * 3.43 vs 4.78; ReachAO 16384 0.78 vs 1.19; PickAndPlace 16384 3.10 vs 3.29 -- so it is
     * the default there; without contacts (Reach's contact-free kernel) the two layouts tie
     * beyond 8192 envs (16384: 0.56 vs 0.54 ms) and the one-lane layout stays. */
    const int wide_max = 8192;
    e.lanes_per_env = cfg->lanes_per_env ? cfg->lanes_per_env
                                         : ((cfg->n_envs <= wide_max || cfg->contacts) ? 16 : 1);
    if (const char* lpe = std::getenv("PGX_LANES_PER_ENV")) {
        const int v = std::atoi(lpe);
        if (v != 1 && v != 16) { delete h; return fail(PGX_E_INVALID, "PGX_LANES_PER_ENV must be 1 or 16, got %s", lpe); }
        e.lanes_per_env = v;
    }
    if (e.full_manifold && e.lanes_per_env != 16) {
        delete h;
        return fail(PGX_E_UNSUPPORTED, "PGX_CONTACTS_FULL needs the 16-lane layout (the one-lane kernels keep 4 robot points)");
    }

    rc = hip_check(hipSetDevice(device), "hipSetDevice");
    if (rc) { delete h; return rc; }
    const size_t N = (size_t)cfg->n_envs;
    auto align = [](size_t x) { return (x + 255) & ~(size_t)255; };
    /* Bullet's persistent manifolds of the robot's cube / obstacle pairs (the per-pair budget's
     * kernels): the pool, count + points (pgx.h PGX_MANIFOLD_POOL) */
    const int man_pool = (e.full_manifold && (e.has_object || e.ao)) ? (e.has_object ? PGX_MANIFOLD_POOL
                                                                                     : PGX_MANIFOLD_POOL_AO) : 0;
    const size_t man_rows = man_pool ? 1 + (size_t)man_pool * PGX_MANIFOLD_POINT : 0;
    h->man_pool = man_pool;
    size_t off_goal = align(sizeof(PgxDevModel)), off_q = align(off_goal + 3 * N * 8), off_qd = align(off_q + PGX_NJ * N * 4),
           off_qc = align(off_qd + PGX_NJ * N * 4), off_obj = align(off_qc + PGX_NJ * N * 4), off_ct = align(off_obj + 13 * N * 4),
           off_ao = align(off_ct + 2 * PGX_CONTACT_SLOTS * N * 4),
           off_man = align(off_ao + (e.ao ? 4 * PGX_AO_OBSTACLES * N * 4 : 0)),
           off_el = align(off_man + man_rows * N * 4), off_ep = align(off_el + N * 4),
           off_err = align(off_ep + N * 4), off_perm = align(off_err + 4),
           total = align(off_perm + (e.full_manifold ? N * 4 + (N + 3) / 4 * 4 + (N / 256 + 1) * 13 * 4 : 0));
    rc = hip_check(hipMalloc(&h->blob, total), "hipMalloc(state)");
    if (rc) { delete h; return rc; }
    h->blob_bytes = total;
    char* b = (char*)h->blob;
    h->ds.goal = (double*)(b + off_goal);
    h->ds.q = (float*)(b + off_q);
    h->ds.qd = (float*)(b + off_qd);
    h->ds.qc = (float*)(b + off_qc);
    h->ds.object = (float*)(b + off_obj);
    h->ds.contacts = (float*)(b + off_ct);
    h->ds.obstacles = e.ao ? (float*)(b + off_ao) : nullptr;
    h->ds.man = man_pool ? (float*)(b + off_man) : nullptr;
    h->ds.elapsed = (int32_t*)(b + off_el);
    h->ds.episode = (uint32_t*)(b + off_ep);
    h->ds.errors = (uint32_t*)(b + off_err);
    if (e.full_manifold) e.perm_buf = (int32_t*)(b + off_perm);   /* heavy-first env order (not state) */
    h->dm_dev = (PgxDevModel*)b;
    /* the PCG64 reset streams and their mode word: not part of the saved state (restoreState leaves
     * np_random alone), so outside the blob */
    const size_t pcg_bytes = align(8 * PGX_PCG64_WORDS * N);
    /* after them the mode word (256 B) and ReachAO's fp64 reset geometry (constants, not state) */
    const size_t geo_bytes = e.ao ? align(8 * PGX_AO_GEO_DOUBLES) : 0;
    rc = hip_check(hipMalloc((void**)&h->pcg, pcg_bytes + 256 + geo_bytes), "hipMalloc(rng streams)");
    if (rc) { h->pcg = nullptr; (void)hipFree(h->blob); delete h; return rc; }
    e.pcg = h->pcg;
    e.pcg_on = (const int32_t*)((char*)h->pcg + pcg_bytes);
    e.ao_geo = e.ao ? (const double*)((char*)h->pcg + pcg_bytes + 256) : nullptr;
    rc = hip_check(hipMemset(h->pcg, 0, pcg_bytes + 256), "hipMemset(rng streams)");
    if (!rc && e.ao) {
        double geo[PGX_AO_GEO_DOUBLES];
        ao_reset_geometry(cfg, geo);
        rc = hip_check(hipMemcpy((void*)e.ao_geo, geo, sizeof geo, hipMemcpyHostToDevice), "ReachAO geometry copy");
    }
    if (!rc) rc = hip_check(hipMemset(h->blob, 0, total), "hipMemset(state)");
    if (!rc) rc = hip_check(hipMemcpy(h->dm_dev, &h->dm, sizeof(PgxDevModel), hipMemcpyHostToDevice), "model copy");
    if (!rc && e.perm_buf) {   /* env_order reads as the identity until a launch sorts the envs */
        std::vector<int32_t> ident(N);
        for (size_t k = 0; k < N; k++) ident[k] = (int32_t)k;
        rc = hip_check(hipMemcpy(e.perm_buf, ident.data(), N * 4, hipMemcpyHostToDevice), "env order init");
    }
    if (!rc) {
        PgxDevOut none;
        std::memset(&none, 0, sizeof none);
        rc = hip_check((hipError_t)pgx_launch_reset(h->dm_dev, h->de, h->ds, nullptr, nullptr, nullptr, none, nullptr),
                       "reset launch");
        /* episodes count resets; the construction reset (core.py:270) is not counted */
        if (!rc) rc = hip_check(hipMemset(h->ds.episode, 0, N * 4), "hipMemset(episode)");
        if (!rc) rc = hip_check(hipDeviceSynchronize(), "create sync");
    }
    if (rc) { (void)hipFree(h->pcg); (void)hipFree(h->blob); delete h; return rc; }
    *out = h;
    return PGX_OK;
}

void pgx_destroy(pgx_handle h) {
    if (!h) return;
    (void)hipSetDevice(h->device);
    for (void* p : h->snaps)
        if (p) (void)hipFree(p);
    if (h->pcg) (void)hipFree(h->pcg);
    (void)hipFree(h->blob);
    delete h;
}

int pgx_get_state(pgx_handle h, pgx_state_view* out) {
    if (!h || !out) return fail(PGX_E_INVALID, "null argument");
    out->q = h->ds.q;
    out->qd = h->ds.qd;
    out->qc = h->ds.qc;
    out->goal = h->ds.goal;
    out->object = h->ds.object;
    out->contacts = h->ds.contacts;
    out->obstacles = h->ds.obstacles;
    out->elapsed = h->ds.elapsed;
    out->episode = h->ds.episode;
    out->errors = h->ds.errors;
    out->robot_points = !h->de.contacts ? 0
                      : !h->de.full_manifold ? PGX_ROBOT_POINTS_ONE_LANE
                      : h->de.has_object ? PGX_ROBOT_POINTS : PGX_ROBOT_POINTS_ARM;
    out->env_order = h->de.perm_buf;
    out->manifolds = h->ds.man;
    out->manifold_pool = h->man_pool;
    return PGX_OK;
}

static PgxDevOut to_dev_out(const pgx_step_out* o) {
    PgxDevOut d;
    std::memset(&d, 0, sizeof d);
    if (!o) return d;
    d.obs = o->obs;
    d.ag = o->achieved_goal;
    d.dg = o->desired_goal;
    d.reward = o->reward;
    d.success = o->success;
    d.terminated = o->terminated;
    d.truncated = o->truncated;
    d.terminal_obs = o->terminal_obs;
    d.terminal_ag = o->terminal_achieved_goal;
    d.terminal_dg = o->terminal_desired_goal;
    d.task_truncated = o->task_truncated;
    return d;
}

int pgx_reset(pgx_handle h, const uint8_t* env_mask, const double* inject_goal, const double* inject_object,
              pgx_step_out* out, void* stream) {
    if (!h) return fail(PGX_E_INVALID, "null handle");
    if (inject_object && !h->de.has_object && !h->de.ao)
        return fail(PGX_E_INVALID, "object injection needs an object task (or ReachAO obstacles)");
    return hip_check((hipError_t)pgx_launch_reset(h->dm_dev, h->de, h->ds, env_mask, inject_goal, inject_object,
                                                  to_dev_out(out), stream),
                     "reset launch");
}

int pgx_step(pgx_handle h, const float* action, pgx_step_out* out, void* stream) {
    if (!h || !action) return fail(PGX_E_INVALID, "null argument");
    return hip_check((hipError_t)pgx_launch_step(h->dm_dev, h->de, h->ds, action, to_dev_out(out), stream,
                                                 &h->step_kernel),
                     "step launch");
}

const char* pgx_step_kernel(pgx_handle h) { return h ? h->step_kernel : nullptr; }

int pgx_sample_actions(pgx_handle h, float* action, uint64_t step, void* stream) {
    if (!h || !action) return fail(PGX_E_INVALID, "null argument");
    return hip_check((hipError_t)pgx_launch_sample_actions(h->de, action, step, stream), "sample launch");
}

int pgx_compute_reward(const float* ag, const float* dg, int64_t batch, int32_t reward_type, double thr, float* out,
                       void* stream) {
    if (batch < 0 || (batch > 0 && (!ag || !dg || !out))) return fail(PGX_E_INVALID, "bad arguments");
    if (reward_type != PGX_REWARD_SPARSE && reward_type != PGX_REWARD_DENSE && reward_type != PGX_REWARD_SPARSE_AO)
        return fail(PGX_E_INVALID, "reward_type %d", reward_type);
    return hip_check((hipError_t)pgx_launch_compute_reward(ag, dg, batch, reward_type, thr, out, stream),
                     "compute_reward launch");
}

int pgx_state_bytes(pgx_handle h, int64_t* nbytes) {
    if (!h || !nbytes) return fail(PGX_E_INVALID, "null argument");
    *nbytes = (int64_t)h->blob_bytes;
    return PGX_OK;
}

int pgx_save_state(pgx_handle h, void* dst, void* stream) {
    if (!h || !dst) return fail(PGX_E_INVALID, "null argument");
    return hip_check(hipMemcpyAsync(dst, h->blob, h->blob_bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream),
                     "save_state copy");
}

int pgx_restore_state(pgx_handle h, const void* src, void* stream) {
    if (!h || !src) return fail(PGX_E_INVALID, "null argument");
    return hip_check(hipMemcpyAsync(h->blob, src, h->blob_bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream),
                     "restore_state copy");
}

/* Snapshot ids (PyBullet.save_state / restore_state / remove_state, pybullet.py:79-102): an id
 * is the first non-negative integer not in use, restoring or removing an id that is not in use
 * fails (pybullet raises pybullet.error, test/save_and_restore_test.py:30-36).  The snapshot is
 * a device copy of the whole state blob on the caller's stream; the buffer is allocated here
 * (hipMalloc: not a step-path call) and freed by pgx_release or pgx_destroy. */
int pgx_snapshot(pgx_handle h, int32_t* state_id, void* stream) {
    if (!h || !state_id) return fail(PGX_E_INVALID, "null argument");
    *state_id = -1;
    size_t id = 0;
    while (id < h->snaps.size() && h->snaps[id]) id++;
    int rc = hip_check(hipSetDevice(h->device), "hipSetDevice");
    void* buf = nullptr;
    if (!rc) rc = hip_check(hipMalloc(&buf, h->blob_bytes), "hipMalloc(snapshot)");
    if (rc) return rc;
    rc = hip_check(hipMemcpyAsync(buf, h->blob, h->blob_bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream),
                   "snapshot copy");
    if (rc) { (void)hipFree(buf); return rc; }
    if (id == h->snaps.size()) h->snaps.push_back(buf);
    else h->snaps[id] = buf;
    *state_id = (int32_t)id;
    return PGX_OK;
}

static bool snap_valid(pgx_handle h, int32_t id) {
    return id >= 0 && (size_t)id < h->snaps.size() && h->snaps[id] != nullptr;
}

int pgx_restore(pgx_handle h, int32_t state_id, void* stream) {
    if (!h) return fail(PGX_E_INVALID, "null handle");
    if (!snap_valid(h, state_id)) return fail(PGX_E_INVALID, "Couldn't restore state %d: no such saved state", state_id);
    return hip_check(hipMemcpyAsync(h->blob, h->snaps[state_id], h->blob_bytes, hipMemcpyDeviceToDevice,
                                    (hipStream_t)stream),
                     "restore copy");
}

int pgx_release(pgx_handle h, int32_t state_id) {
    if (!h) return fail(PGX_E_INVALID, "null handle");
    if (!snap_valid(h, state_id)) return fail(PGX_E_INVALID, "Couldn't remove state %d: no such saved state", state_id);
    /* the copies that read or write the buffer were queued on a stream: wait for them */
    int rc = hip_check(hipSetDevice(h->device), "hipSetDevice");
    if (!rc) rc = hip_check(hipDeviceSynchronize(), "release sync");
    if (!rc) rc = hip_check(hipFree(h->snaps[state_id]), "hipFree(snapshot)");
    h->snaps[state_id] = nullptr;
    return rc;
}

/* Reset draws from numpy PCG64 streams instead of the Philox counter: a copy of the caller's
 * [N][PGX_PCG64_WORDS] records (numpy's whole bit_generator.state: state, inc, has_uint32,
 * uinteger) on `stream`, then the device mode word set on the same stream; NULL clears the word
 * (back to Philox) and keeps the buffer, which lives as long as the handle -- a HIP graph captured
 * in either mode keeps valid pointers and draws in the mode of replay time.  Every task draws from
 * them, ReachAO's rejection sampler included (reach_ao.py:1101-1161: uniforms, random, integers(4, 6)
 * and the shuffle of the six names, as numpy's Generator draws them; its accept / reject tests in
 * fp64 on the host's capsules, pgx_config.ao_capsules_neutral). */
int pgx_set_rng_streams(pgx_handle h, const uint64_t* states, void* stream) {
    if (!h) return fail(PGX_E_INVALID, "null handle");
    int rc = hip_check(hipSetDevice(h->device), "hipSetDevice");
    if (rc) return rc;
    int32_t* on = const_cast<int32_t*>(h->de.pcg_on);
    if (states)
        rc = hip_check(hipMemcpyAsync(h->pcg, states, 8 * PGX_PCG64_WORDS * (size_t)h->de.n_envs, hipMemcpyDefault, (hipStream_t)stream),
                       "rng streams copy");
    if (!rc) rc = hip_check((hipError_t)pgx_launch_set_word(on, states ? 1 : 0, stream), "rng mode word");
    if (!rc) h->pcg_set = states != nullptr;
    return rc;
}

int pgx_get_rng_streams(pgx_handle h, uint64_t* states, void* stream) {
    if (!h || !states) return fail(PGX_E_INVALID, "null argument");
    if (!h->pcg_set) return fail(PGX_E_INVALID, "no PCG64 reset streams set (pgx_set_rng_streams)");
    return hip_check(hipMemcpyAsync(states, h->pcg, 8 * PGX_PCG64_WORDS * (size_t)h->de.n_envs, hipMemcpyDefault, (hipStream_t)stream),
                     "rng streams copy");
}

}  // extern "C"
