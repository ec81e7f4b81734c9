/*
 * pgx_dev.h -- device-side constant tables and launch interface of libpgx.
 *
 * The env robot (franka_panda_custom_0, panda.py:54) is a 7-revolute-joint
 * chain whose joint axes are all URDF z, followed by six links rigidly fixed
 * to panda_link7 (link8, hand, ee, fingers, grasptarget: Bullet links 7-12).
 * The kernel hard-codes that topology (checked on the host at pgx_create) and
 * takes every numeric constant from PgxDevModel, copied once to a device
 * buffer and read through the constant address space (scalar loads, SGPRs).
 */
#pragma once
#include <stdint.h>

#define PGX_NJ 7          /* arm joints */
#define PGX_MAX_DAMP 4    /* bodies of the link-7 group with mass (linear damping) */

struct PgxDevModel {
    float jp[PGX_NJ][3];      /* joint origin in parent URDF frame */
    float jr[PGX_NJ][9];      /* joint origin rotation (row-major) */
    float com[PGX_NJ][3];     /* COM in URDF link frame; [6] = composite COM of the link-7 group */
    float mass[PGX_NJ];       /* [6] = composite mass */
    float inertia[PGX_NJ - 1][3]; /* principal inertia of links 1..6 (COM frame == URDF frame) */
    float i6c[6];             /* composite inertia of the link-7 group about its COM (xx,yy,zz,xy,xz,yz) */
    float i6own[6];           /* sum of the group bodies' own inertias (angular damping) */
    float dpos[PGX_MAX_DAMP][3]; /* COMs of group bodies with mass (link-7 frame) */
    float dmass[PGX_MAX_DAMP];
    int32_t ndamp;
    float ee_pivot[3];        /* EE link URDF origin in link-7 frame (IK point) */
    float ee_rot[9];          /* EE link rotation relative to link 7 */
    float ee_com[3];          /* EE link COM in link-7 frame (getLinkState()[0]) */
    float lower[PGX_NJ], upper[PGX_NJ];
    float max_impulse[PGX_NJ];  /* joint_forces * dt */
    float dt, inv_dt;
    float gravity[3];
    float lin_damp, ang_damp, max_vel, residual_thr, erp, limit_max_imp, kp, kd;
    float ik_residual, ik_damping, ik_max_angle;
    int32_t num_iterations, ik_max_iters;
    float base[3];
    float ee_step, joint_step;
    float neutral_q[PGX_NJ];
    /* contacts (pgx_sim_params) */
    float contact_dist, contact_erp, friction, warmstart;
    float residual_abs;       /* largest t >= 0 with fl(t * t) <= residual_thr: the sweep exit
                                 test resid * resid <= residual_thr as one compare, resid <= t */
    float cap_mu[16];         /* combined lateral friction of capsule c's link against the scene
                                 (pgx_sim_params.link_friction of its link; PGX_NCAP used) */
    /* contact breaking thresholds per pair (Bullet's relative rule, pgx.h contact_distance): capsule
     * c's link against the table, the plane, the cube and an obstacle; the cube against the table
     * and the plane -- the distance within which a point is reported, merged and kept */
    float tau_table[16], tau_plane[16], tau_obj[16], tau_obst[16];
    float tau_obj_table, tau_obj_plane;
    /* the scene's table box and plane top (pgx_config table_center / table_half / plane_z, as
     * PgxDevEnv's fields): in the block, the step kernels' table tests fold to constants in the
     * default build instead of holding kernel-argument values in registers */
    float table_cx, table_cy, table_hx, table_hy, table_top, plane_z, table_hz, scene_pad;
};

struct PgxDevEnv {
    int32_t task, control, reward, n_envs;
    int32_t max_episode_steps, block_gripper, obs_dim, action_dim;
    uint64_t seed, env_id_offset;
    double distance_threshold;
    double goal_low[3], goal_high[3];
    /* scene (pgx_config): reset draws and the static boxes / object */
    double goal_offset[3], goal_z_zero_prob;
    double obj_low[3], obj_high[3], obj_offset[3];
    int32_t contacts, has_object;
    float obj_half, obj_inv_mass, obj_inv_inertia;
    float table_cx, table_cy, table_hx, table_hy, table_top, plane_z;
    float table_hz;
    int32_t ao;                    /* ReachAO (obstacles, per-substep collision check) */
    int32_t terminate_on_success;
    int32_t no_auto_reset;         /* pgx_config.no_auto_reset: finished envs keep their state */
    double collision_reward;
    double ao_ee[3];               /* pgx_config.ao_ee_neutral: the reset sampler's EE centre, fp64 */
    int32_t ao_ee_set;             /* 0: the kernel's fp32 FK of the neutral pose instead */
    const double* ao_geo;          /* ReachAO reset geometry, fp64, device (allocated with the handle):
                                      [PGX_NCAP][7] capsules A, B, r at the neutral pose
                                      (pgx_config.ao_capsules_neutral), then the table centre [3] and
                                      half extents [3]; nullptr for the other tasks */
    int32_t lanes_per_env;         /* step layout: 1 (env per lane) or 16 (env per DPP row) */
    int32_t pgs_mode;              /* test hook (PGX_PGS_MODE): 0 auto, 2 never speculate on the limit
                                      rows, 3 always redo the speculative solve with them */
    int32_t n_substeps;            /* stepSimulation calls per env step (a runtime loop count) */
    int32_t full_manifold;         /* contacts == PGX_CONTACTS_FULL: robot budget PGX_ROBOT_POINTS(_ARM) */
    int32_t wave_mode;             /* A/B hook (PGX_WAVES_PER_SIMD): 0 auto (two resident waves per SIMD
                                      beyond 1024 waves), 1 the one-wave build, 2 the two-wave build */
    uint64_t* pcg;                 /* [N][PGX_PCG64_WORDS] numpy PCG64 streams of the reset draws (pgx_set_rng_streams),
                                      allocated with the handle and freed with it */
    const int32_t* pcg_on;         /* device word: 1 = resets draw from pcg, 0 = the Philox counter.  In
                                      device memory and switched on the caller's stream, so a step loop
                                      captured in a HIP graph draws in the mode of replay time */
    /* heavy-first env order of the per-pair manifold kernels (pgx_launch_step): perm_buf device
     * buffer (permutation [N] i32, keys [N] u8 padded to 4 B, per-block bin counts [N/256 + 1][13]); sort_mode (PGX_SORT_ENVS) 0 auto (more waves than fit at once), 1 always, -1 never;
     * perm: the order a launch uses (nullptr: identity), set by the launcher */
    int32_t* perm_buf;
    int32_t sort_mode;
    int32_t sort_key;              /* PGX_SORT_KEY: 1 all robot points (default), 0 only those past CG */
    int32_t sort_segs;             /* PGX_SORT_SEGS: 0 auto (8 per-XCD segments when N divides), 1 one global order */
    const int32_t* perm;
    int32_t perm_segs;             /* the launch's segments: 8 = perm is heavy-first within each XCD's env range */
};

struct PgxDevState {
    float* q;          /* [7][N] */
    float* qd;         /* [7][N] */
    float* qc;         /* [7][N] the link cache's pose (getLinkState: before the last substep) */
    double* goal;      /* [3][N] */
    float* object;     /* [13][N] pos3 quat4 (x,y,z,w) linvel3 angvel3 */
    float* contacts;   /* [2*PGX_CONTACT_SLOTS][N] warm-start cache (feature id, normal impulse) */
    float* obstacles;  /* [4*PGX_AO_OBSTACLES][N] ReachAO centres (o, xyz) then active flags */
    float* man;        /* [1 + pool * PGX_MANIFOLD_POINT][N] persistent manifold pool (pgx.h), or nullptr */
    int32_t* elapsed;  /* [N] */
    uint32_t* episode; /* [N] */
    uint32_t* errors;  /* [1] sticky PGX_ERR_* bits (pgx_state_view.errors) */
};

struct PgxDevOut {
    float* obs;
    float* ag;
    float* dg;
    float* reward;
    uint8_t* success;
    uint8_t* terminated;
    uint8_t* truncated;
    float* terminal_obs;
    float* terminal_ag;
    float* terminal_dg;
    uint8_t* task_truncated;   /* ReachAO is_collided (pgx_step_out.task_truncated) */
};

/* launchers (pgx_kernels.hip); return hipError_t as int */
/* the arm-only (Reach) step kernels: their own translation unit (pgx_kernels.hip, PGX_TU) */
/* name (may be NULL): set to the launched step kernel's name, as rocprof spells it */
int pgx_launch_step_arm(const PgxDevModel* m_device, const PgxDevEnv& e, const PgxDevState& s, const float* action,
                        const PgxDevOut& o, void* stream, const char** name);
int pgx_launch_step(const PgxDevModel* m_device, const PgxDevEnv& e, const PgxDevState& s, const float* action,
                    const PgxDevOut& o, void* stream, const char** name);
/* the ReachAO step kernels: their own translation unit too (PGX_TU 4, scheduler flags of its own);
 * e as pgx_launch_step hands it on (perm set), two: the two-wave build, wide: the 16-lane layout */
int pgx_launch_step_ao(const PgxDevModel* m_device, const PgxDevEnv& e, const PgxDevState& s, const float* action,
                       const PgxDevOut& o, void* stream, const char** name, bool two, bool wide);
int pgx_launch_reset(const PgxDevModel* m_device, const PgxDevEnv& e, const PgxDevState& s, const uint8_t* mask,
                     const double* inject_goal, const double* inject_object, const PgxDevOut& o, void* stream);
int pgx_launch_sample_actions(const PgxDevEnv& e, float* action, uint64_t step, void* stream);
int pgx_launch_set_word(int32_t* p, int32_t v, void* stream);
int pgx_launch_compute_reward(const float* ag, const float* dg, int64_t n, int32_t reward_type, double thr,
                              float* out, void* stream);
