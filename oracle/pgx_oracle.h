/*
 * pgx_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * fp64 CPU restatement of the reference's per-step hot path, used as the
 * checker for the HIP kernels (tests/, __graft_entry__.smoke(), bench.py's
 * cpu_baseline leg).  Never linked into libpgx.so.  See oracle/pgx_oracle.c
 * for the per-function reference citations and DESIGN.md for how it is pinned.
 */
#ifndef PGX_ORACLE_H
#define PGX_ORACLE_H

#include <stdint.h>
#include "../include/pgx.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct pgxo_motor {
    double target_q;
    double target_qd;
    double kp;
    double kd;
    double max_impulse;   /* 0 = motor disabled */
} pgxo_motor;

/* diagnostics of the last substep (optional) */
typedef struct pgxo_stats {
    int32_t solver_iterations;
    int32_t ik_iterations;
    double ik_residual;
    int32_t limits_far;   /* diagnostics: the kernel's exact limit-row skip test holds */
    int32_t n_contacts;   /* contact points of the last substep */
} pgxo_stats;

void pgxo_fk(const pgx_model* m, const double base[3], const double* q, double* com_pos,
             double* rot, double* origin);
void pgxo_link_velocity(const pgx_model* m, const double base[3], const double* q, const double* qd,
                        int link, double lin[3], double ang[3]);
void pgxo_mass_matrix(const pgx_model* m, const double base[3], const double* q, double* M);
void pgxo_bias(const pgx_model* m, const pgx_sim_params* p, const double base[3], const double* q,
               const double* qd, int with_gravity, double* b);
/* M and b in the recursive form (CRBA + Newton-Euler), the formulation the kernel computes; the
 * substeps use it with the oracle flag PGX_FLAG_DYN_RECURSIVE (operation count) */
void pgxo_dyn_recursive(const pgx_model* m, const pgx_sim_params* p, const double base[3], const double* q,
                        const double* qd, int with_gravity, double* M, double* b);
int pgxo_ik(const pgx_model* m, const pgx_sim_params* p, const double base[3], const double* q_start,
            int link, const double target_pos[3], const double target_orn[4], double* q_out,
            pgxo_stats* st);
void pgxo_substep(const pgx_model* m, const pgx_sim_params* p, const double base[3], double* q,
                  double* qd, const pgxo_motor* motors, pgxo_stats* st);
/* One substep of the task's scene (table, plane, object, contacts): obj[PGXO_OBJ_N] = pos3,
 * quat4 (x,y,z,w), linvel3, angvel3, the contact cache (feature id, normal impulse) x
 * (PGX_OBJECT_POINTS object-scene slots + PGXO_ROBOT_MAX robot slots), then ReachAO's
 * obstacles and the cached link pose. */
void pgxo_world_substep(const pgx_config* cfg, double* q, double* qd, double* obj,
                        const pgxo_motor* motors, pgxo_stats* st);
#define PGXO_ROBOT_MAX 16   /* robot contact slots of the oracle's cache (its largest budget) */
#define PGXO_POOL_MAX 48     /* manifold pool points per env: PGX_MANIFOLD_POOL(_AO) in the default
                                mode, all of it with the study flag PGX_FLAG_PERSISTENT_MANIFOLD */
#define PGXO_OBJ_N (13 + 2 * (PGX_OBJECT_POINTS + PGXO_ROBOT_MAX) + 4 * PGX_AO_OBSTACLES + 7 + \
                    1 + PGXO_POOL_MAX * PGX_MANIFOLD_POINT)
/* the robot group's row budget (default / -1: the configuration's, pgx_config.contacts) and
 * the histogram of robot points Bullet's per-pair rule keeps before the budget, per substep */
#define PGXO_ROBOT_HIST 33
void pgxo_set_robot_budget(int budget);
/* a manifold pool [1 + cap x PGX_MANIFOLD_POINT] (pgx.h): add a point (kid, local A, local B, normal
 * on B, distance, impulse; kid and impulse ignored) to manifold `key` -- returns its slot, -1 when
 * the pool is full -- / refresh every manifold with the bodies at rest (the btPersistentManifold
 * restatement; tests) */
int pgxo_manifold_add(double* pool, int cap, int key, const double* point, double thr);
void pgxo_manifold_refresh_static(double* pool, double thr);
void pgxo_pair_hist_read(int64_t* out, int clear);
void pgxo_breaking_thresholds(const pgx_config* c, double* out);
/* the last contact detection's points (group 0 object-scene / 1 robot-table / 2 robot-object,
 * feature id, robot link or -1, separation); returns their number */
int pgxo_last_contacts(int32_t* grp, int32_t* id, int32_t* link, double* dist);

/* ReachAO geometry (test helpers): capsule (A, B, r) vs sphere (C, R) / rounded box
 * (c, h); per-link closest obstacle of the 9 collision links at q, returning the
 * table distance of links 2..ee; whole-robot collision predicate. */
double pgxo_ao_capsule_sphere(const double* A, const double* B, double r, const double* C, double R, double* pa,
                              double* pb);
double pgxo_ao_capsule_box(const double* A, const double* B, double r, const double* c, const double* h, double* pa,
                           double* pb);
double pgxo_ao_link_distances(const pgx_config* cfg, const double* q, const double* obst, double* dist, double* pa,
                              double* pb);
int pgxo_ao_collided(const pgx_config* cfg, const double* q, const double* obst);
/* diagnostics: per env of the following pgxo_vec_step calls (ReachAO), the smallest |margin| of
 * check_collided over the substep checks that ran and the margin at the last one (collided <=>
 * margin <= 0); NULL buffers switch it off */
void pgxo_diag_collision_margin(double* min_abs, double* last, int64_t n);

/* reward / success, reference utils.distance + Reach.is_success / compute_reward */
double pgxo_distance_f32_f64(const float ag[3], const double g[3]);
float pgxo_distance_f32_f32(const float ag[3], const float g[3]);
void pgxo_compute_reward_f32(const float* ag, const float* dg, int64_t n, int reward_type,
                             double thr, float* out);

/* Philox4x32-10 (device RNG restated for parity of auto-reset draws) */
void pgxo_philox(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);

/* Batched env step with the kernel's vec-env semantics (TimeLimit + auto-reset).
 * State arrays are AoS per env here: q[N*nd], qd[N*nd], goal[N*3], obj[N*PGXO_OBJ_N]. */
int pgxo_vec_step(const pgx_config* cfg, int64_t n, double* q, double* qd, double* goal,
                  double* obj, int32_t* elapsed, uint32_t* episode, const float* action,
                  float* obs, float* ag, float* dg, float* reward, uint8_t* success,
                  uint8_t* terminated, uint8_t* truncated, float* terminal_obs);
int pgxo_vec_reset(const pgx_config* cfg, int64_t n, const uint8_t* mask, const double* inject_goal,
                   const double* inject_obj, double* q, double* qd, double* goal, double* obj,
                   int32_t* elapsed, uint32_t* episode, float* obs, float* ag, float* dg);
void pgxo_sample_actions(const pgx_config* cfg, int64_t n, uint64_t step, float* action);
/* sticky PGX_ERR_* bits set by the resets since the last call (cleared by it) */
uint32_t pgxo_take_errors(void);

#ifdef __cplusplus
}
#endif
#endif
