/*
 * pgx.h -- C-ABI of the MI355X-native batched Panda environment (libpgx.so).
 *
 * One handle owns the structure-of-arrays state of N lockstep environments on
 * one GPU.  Every call is asynchronous on the caller's HIP stream (passed as
 * void*, NULL = default stream) and takes plain device pointers into
 * caller-owned buffers (torch tensors on the Python side).  No call allocates,
 * frees or synchronises on the step path, so a step can be captured in a
 * hipGraph.
 *
 * Reference interfaces each entry point replaces (paths relative to
 * RaikoPipe/panda-gym):
 *   pgx_create          PandaReachEnv/PandaPushEnv/PandaPickAndPlaceEnv.__init__
 *                       panda_gym/envs/panda_tasks.py:37-88, RobotTaskEnv.__init__
 *                       panda_gym/envs/core.py:264-284, gym registration
 *                       panda_gym/__init__.py:23-91 (max_episode_steps)
 *   pgx_reset           RobotTaskEnv.reset core.py:298-308 -> Panda.reset
 *                       panda.py:290-298, Reach.reset reach.py:63-78,
 *                       Push.reset push.py:69-87, PickAndPlace.reset
 *                       pick_and_place.py:65-85
 *   pgx_step            RobotTaskEnv.step core.py:352-368 -> Panda.set_action
 *                       panda.py:120-172 (IK: pybullet.py:465-493), PyBullet.step
 *                       pybullet.py:68-71 (20 x stepSimulation), _get_obs
 *                       core.py:286-296, Task.is_success / compute_reward
 *                       reach.py:80-89, + gymnasium TimeLimit and SB3 VecEnv
 *                       auto-reset (terminal_observation)
 *   pgx_compute_reward  Task.compute_reward bound as env.compute_reward
 *                       (core.py:282; reach.py:84-89, push.py:93-98,
 *                       pick_and_place.py:91-96) over a batch (HER relabel)
 *   pgx_get_state       PyBullet.get_joint_angles / get_joint_velocities
 *                       pybullet.py:313-348 (device views of the SoA state)
 *   pgx_snapshot /      RobotTaskEnv.save_state / restore_state / remove_state
 *   pgx_restore /       core.py:310-336 -> PyBullet.save_state / restore_state /
 *   pgx_release         remove_state pybullet.py:79-102 (state ids)
 *   pgx_save_state /    the same snapshot into / out of a caller-owned device
 *   pgx_restore_state   buffer (no id)
 *
 * Error convention: every call returns PGX_OK (0) or a negative PGX_E_* code;
 * pgx_last_error() returns a thread-local message for the last failure.
 */
#ifndef PGX_H
#define PGX_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PGX_MAX_LINKS 16
#define PGX_MAX_DOFS 9
#define PGX_MAX_ROWS 27
#define PGX_MAX_CAPSULES 16
/* Contact row budgets per env (Bullet keeps <= 4 points per colliding pair; the kernels keep
 * the deepest of those up to a fixed budget per group -- DESIGN.md section 4):
 * object vs table / plane, and robot vs table / plane / object / obstacles, the latter
 * PGX_ROBOT_POINTS_ONE_LANE by default and with pgx_config.contacts = PGX_CONTACTS_FULL
 * PGX_ROBOT_POINTS in Push / PickAndPlace and PGX_ROBOT_POINTS_ARM in Reach / ReachAO. */
#define PGX_OBJECT_POINTS 4
#define PGX_ROBOT_POINTS 12
#define PGX_ROBOT_POINTS_ARM 8
#define PGX_ROBOT_POINTS_ONE_LANE 4
#define PGX_CONTACT_SLOTS (PGX_OBJECT_POINTS + PGX_ROBOT_POINTS)
#define PGX_CONTACTS_FULL 2
/* Bullet's persistent contact manifolds of the robot's pairs with the cube and with the obstacles
 * (PGX_CONTACTS_FULL; btPersistentManifold): a pool of at most
 * PGX_MANIFOLD_POOL (Push / PickAndPlace) or PGX_MANIFOLD_POOL_AO (ReachAO) points per env, kept
 * across substeps and steps -- the point count, then per point in pool order PGX_MANIFOLD_POINT
 * values: kid = key + slot (key 32 + 16 c for capsule c against the cube, 32 + 24 c + 4 o against
 * obstacle o; slot = the point's index in its manifold, < 4), local A [3] (in the frame of the arm
 * joint that carries the capsule), local B [3] (cube frame; world for a static obstacle), normal on
 * B [3] (world, from B to the robot), distance, applied normal impulse.  The row id of a point is
 * its kid. */
#define PGX_MANIFOLD_POOL 16
#define PGX_MANIFOLD_POOL_AO 8
#define PGX_MANIFOLD_POINT 12

#define PGX_OK 0
#define PGX_E_INVALID -1
#define PGX_E_HIP -2
#define PGX_E_UNSUPPORTED -3
#define PGX_E_NOMEM -4

#define PGX_JOINT_REVOLUTE 0
#define PGX_JOINT_PRISMATIC 1
#define PGX_JOINT_FIXED 4

#define PGX_TASK_REACH 0
#define PGX_TASK_PUSH 1
#define PGX_TASK_PICK_AND_PLACE 2
#define PGX_TASK_REACH_AO 3        /* ReachAO, scenario "reachao_rand" (reach_ao.py:587-599) */

/* ReachAO "reachao_rand" scene (reach_ao.py:268-290, 573-599, 819-860): 3 spheres of
 * radius 0.05 and 3 cuboids of half extent 0.05, 4-5 of them active per episode. */
#define PGX_AO_OBSTACLES 6
#define PGX_AO_LINKS 9             /* collision links: panda_link1..8, panda_ee */

#define PGX_CONTROL_EE 0
#define PGX_CONTROL_JOINTS 1

#define PGX_REWARD_SPARSE 0
#define PGX_REWARD_DENSE 1
#define PGX_REWARD_SPARSE_AO 2   /* ReachAO relabel reward: -1 + (d < thr) (reach_ao.py:1320), collision term 0 */

/* solver row kinds (pgx_model.row_kind) */
#define PGX_ROW_MOTOR 0
#define PGX_ROW_LIMIT_LOWER 1
#define PGX_ROW_LIMIT_UPPER 2

/* Multibody description in Bullet link order (built from the URDF by
 * panda-gym_amd/model.py).  All frames are URDF frames except that link
 * state is reported at the inertial origin (COM), like getLinkState()[0]. */
typedef struct pgx_model {
    int32_t n_links;                       /* links excluding the fixed base */
    int32_t n_dofs;
    int32_t ee_link;                       /* Panda.ee_link = 11 (panda.py:68) */
    int32_t n_rows;                        /* solver rows in Bullet order */
    int32_t parent[PGX_MAX_LINKS];         /* -1 = base */
    int32_t jtype[PGX_MAX_LINKS];
    int32_t dof_of_link[PGX_MAX_LINKS];    /* -1 for fixed joints */
    int32_t link_of_dof[PGX_MAX_DOFS];
    int32_t has_limit[PGX_MAX_DOFS];
    int32_t row_kind[PGX_MAX_ROWS];
    int32_t row_dof[PGX_MAX_ROWS];
    int32_t pad0;
    double jpos[PGX_MAX_LINKS][3];         /* joint origin in parent URDF frame */
    double jrot[PGX_MAX_LINKS][9];         /* row-major */
    double axis[PGX_MAX_LINKS][3];         /* joint axis in joint frame */
    double com[PGX_MAX_LINKS][3];          /* inertial origin in URDF link frame */
    double mass[PGX_MAX_LINKS];
    double inertia[PGX_MAX_LINKS][3];      /* principal inertia (Bullet AABB rule) */
    double lower[PGX_MAX_DOFS];
    double upper[PGX_MAX_DOFS];
    /* Collision geometry for contacts: the URDF's <collision> cylinders with their
     * end spheres fused into capsules (segment a-b in the URDF frame of link
     * cap_link, radius), lone spheres as zero-length capsules. */
    int32_t n_capsules;
    int32_t pad1;
    int32_t cap_link[PGX_MAX_CAPSULES];
    int32_t cap_flags[PGX_MAX_CAPSULES];   /* PGX_CAP_* */
    double cap_a[PGX_MAX_CAPSULES][3];
    double cap_b[PGX_MAX_CAPSULES][3];
    double cap_radius[PGX_MAX_CAPSULES];
    /* Bullet's link compound AABB (btCompoundShape::getAabb with the identity) in the link's COM
     * frame, child and compound margins included: centre and half extents.  The link's angular
     * motion disc |half| + |centre| scales its contact breaking threshold
     * (pgx_sim_params.contact_distance, btCollisionShape::getContactBreakingThreshold). */
    double link_aabb_center[PGX_MAX_LINKS][3];
    double link_aabb_half[PGX_MAX_LINKS][3];
} pgx_model;

#define PGX_CAP_VS_TABLE 1                 /* capsule end spheres collide with table / plane */
#define PGX_CAP_VS_OBJECT 2                /* capsule collides with the object (cube) */

/* Physics / solver constants (pybullet defaults as used by the reference). */
typedef struct pgx_sim_params {
    double dt;                    /* 1/500 (pybullet.py:50) */
    double gravity[3];            /* (0,0,-9.81) (pybullet.py:54) */
    double lin_damping;           /* btMultiBody default 0.04 */
    double ang_damping;           /* btMultiBody default 0.04 */
    double max_coord_vel;         /* btMultiBody::m_maxCoordinateVelocity 100 */
    double residual_threshold;    /* solver least-squares residual 1e-7 */
    double erp;                   /* joint-limit violation ERP 0.2 */
    double limit_max_impulse;     /* btMultiBodyConstraint default 100 */
    double motor_kp;              /* POSITION_CONTROL default positionGain 0.1 */
    double motor_kd;              /* POSITION_CONTROL default velocityGain 1.0 */
    double ik_residual;           /* calculateInverseKinematics residual 1e-4 */
    double ik_damping;            /* per-joint DLS damping 0.5 */
    double ik_max_angle;          /* BussIK MaxAngleDLS = pi/4 */
    int32_t n_substeps;           /* 20 (pybullet.py:25) */
    int32_t num_iterations;       /* numSolverIterations 50 */
    int32_t ik_max_iters;         /* maxNumIterations 20 */
    int32_t flags;                /* PGX_FLAG_* hypotheses (oracle only) */
    double contact_distance;      /* gContactBreakingThreshold 0.02.  Bullet's dispatcher scales it per
                                     pair (btCollisionDispatcher::getNewManifold with its default flag
                                     CD_USE_RELATIVE_CONTACT_BREAKING_THRESHOLD): the pair's manifold
                                     breaking threshold is the smaller of the two shapes'
                                     getContactBreakingThreshold(0.02) = angular motion disc x 0.02 --
                                     the distance within which the narrow phase reports a point
                                     (btManifoldResult::addContactPoint), merges it into a cached one
                                     (getCacheEntry) and keeps it (refreshContactPoints).  DESIGN.md
                                     section 2 "Contact breaking threshold". */
    double contact_erp;           /* ERP of multibody contact rows (m_erp 0.2) */
    double friction;              /* combined lateral friction of the cube against the table / plane:
                                     0.5 * 0.5 (each body's pybullet default; btManifoldResult
                                     multiplies the two) */
    double warmstart;             /* m_warmstartingFactor 0.85 (normal impulses) */
    /* combined lateral friction of robot link i (Bullet link index) against the scene's bodies --
     * table, plane, cube, obstacles, each at the default 0.5: 0.5 x the link's own, 0.5 x 0.5
     * except panda_ee and panda_leftfinger (links 9, 10), which Panda.__init__ raises to 1.0
     * (panda.py:69-70: set_lateral_friction(fingers_indices), pybullet.py:880-892 changeDynamics).
     * Their spinning friction 0.001 (panda.py:71-72) combines with the others' 0 to 0: no row. */
    double link_friction[PGX_MAX_LINKS];
} pgx_sim_params;

/* oracle-only modelling switches (documented in DESIGN.md) */
#define PGX_FLAG_CONSTRAINT_PASS_BIAS 1   /* re-apply velocity bias in the constraint pass */
#define PGX_FLAG_IK_COM 2                 /* IK targets the link COM instead of the joint pivot */
#define PGX_FLAG_NO_RESIDUAL_EXIT 4       /* run all solver iterations */
#define PGX_FLAG_LINKSTATE_CURRENT 8      /* getLinkState reports the pose after the last substep
                                             instead of Bullet's cached pose (rejected hypothesis) */
#define PGX_FLAG_DYN_RECURSIVE 16         /* M and b by composite rigid bodies + Newton-Euler (the
                                             kernel's formulation; same dynamics) instead of the
                                             Jacobian form: for the operation count */
#define PGX_FLAG_PERSISTENT_MANIFOLD 32   /* study: with PGX_CONTACTS_FULL, the robot's table / plane
                                             pairs through persistent manifolds too (each end sphere's
                                             manifold holds its one re-reported point, so it equals
                                             the fresh table rule to rounding: a test pins that) */
#define PGX_FLAG_FRESH_MANIFOLD 64        /* study: with PGX_CONTACTS_FULL, round 4's rule for the cube /
                                             obstacle pairs -- each pair's 4 deepest candidates of the
                                             substep -- instead of Bullet's persistent manifolds */
#define PGX_FLAG_GLOBAL_BREAKING 128      /* study: every pair's breaking threshold the global
                                             contact_distance (rounds 2-5) instead of Bullet's relative
                                             per-pair threshold */

typedef struct pgx_config {
    int32_t task;                 /* PGX_TASK_* */
    int32_t control;              /* PGX_CONTROL_* */
    int32_t reward;               /* PGX_REWARD_* */
    int32_t n_envs;
    int32_t max_episode_steps;    /* TimeLimit; 0 = never truncate */
    int32_t block_gripper;        /* Reach/Push: 1 */
    int32_t no_auto_reset;        /* 0: a finished env (terminated or truncated) is reset inside
                                     pgx_step, SB3 VecEnv style (terminal_* outputs hold the
                                     finished episode); 1: it keeps its final state until
                                     pgx_reset, like one gymnasium env (RobotTaskEnv + TimeLimit,
                                     core.py:352-368) */
    int32_t pad1;
    uint64_t seed;                /* device Philox key for auto-reset draws */
    uint64_t env_id_offset;       /* global id of env 0 (multi-GPU sharding) */
    double base_pos[3];           /* robot base (-0.6,0,0) (panda_tasks.py:85) */
    double distance_threshold;    /* 0.05 (reach.py:15) */
    double goal_low[3];
    double goal_high[3];
    double joint_forces[PGX_MAX_DOFS]; /* panda.py:63 */
    double neutral_q[PGX_MAX_DOFS];    /* panda.py:67 */
    double ee_step;               /* 0.05 (panda.py:235) */
    double joint_step;            /* 0.05 (panda.py:74) */
    const pgx_model* model;       /* host pointers, copied at create */
    const pgx_sim_params* params;
    /* scene (Task._create_scene, push.py:31-47; pybullet.py:759-817) */
    int32_t contacts;             /* 1: robot/table/object contacts (the reference's scene), the robot
                                     group's rows budgeted at PGX_ROBOT_POINTS_ONE_LANE (4) points;
                                     PGX_CONTACTS_FULL: Bullet's per-pair manifolds kept up to
                                     PGX_ROBOT_POINTS (object tasks) / _ARM points (16-lane layout) */
    int32_t lanes_per_env;        /* step layout: 0 auto (16 with contacts -- every object task
                                     and ReachAO -- at any batch, and up to 8192 envs without),
                                     1 = one env per lane, 16 = one env per 16-lane DPP row */
    double goal_offset[3];        /* goal = offset + uniform(goal_low, goal_high): (0,0,0.02) Push/PnP */
    double goal_z_zero_prob;      /* PickAndPlace: noise z = 0 with probability 0.3 */
    double obj_low[3];            /* object = obj_offset + uniform(obj_low, obj_high) */
    double obj_high[3];
    double obj_offset[3];
    double object_half;           /* cube half extent 0.02 */
    double object_mass;           /* 1.0 */
    double object_inertia;        /* principal inertia (Bullet compound-AABB rule) */
    double table_center[3];       /* (-0.3, 0, -0.2) */
    double table_half[3];         /* (0.55, 0.35, 0.2) */
    double plane_z;               /* top of the plane box: -0.4 */
    /* ReachAO (TrainConfig defaults, classes/train_config.py:24-35) */
    int32_t terminate_on_success; /* RobotTaskEnv(terminate_on_success): 1 for ReachAO */
    int32_t pad3;
    double collision_reward;      /* -100: added to the sparse reward on collision */
    double ao_ee_neutral[3];      /* ReachAO: the EE (panda_ee COM) at the neutral pose, fp64 -- the
                                     reset sampler's obstacle centre (reach_ao.py:635-644, the
                                     get_ee_position it reads after Panda.reset) and its goal
                                     fallback, a model constant computed once on the host; all zero:
                                     the kernel's own fp32 FK of that pose */
    /* ReachAO: the robot's capsules at the neutral pose in world coordinates, fp64, per capsule of
     * the model (model.n_capsules, the base's included) end A [3], end B [3], radius -- the geometry
     * of the reset sampler's accept / reject tests (reach_ao.py:1101-1161, get_distances against the
     * robot; host restatement panda-gym_amd/reach_ao.py RobotGeometry), which the device evaluates in
     * fp64 on exactly these values so that a reset drawn on the device decides every test as the
     * host's does.  All zero: pgx_create computes them by an fp64 FK of neutral_q from the model
     * (the same values to rounding). */
    double ao_capsules_neutral[PGX_MAX_CAPSULES][7];
} pgx_config;

typedef struct pgx_env* pgx_handle;

/* Output buffers of one batched step (device pointers; any may be NULL to skip).
 * obs [N,obs_dim] f32, achieved/desired [N,3] f32, reward [N] f32,
 * success/terminated/truncated [N] u8, terminal_obs [N,obs_dim] f32 (obs of the
 * finished episode, written only for envs that were auto-reset),
 * terminal_ag / terminal_dg [N,3] f32 (achieved / desired goal of the finished
 * episode: SB3 stores next_obs = infos["terminal_observation"] for them). */
typedef struct pgx_step_out {
    float* obs;
    float* achieved_goal;
    float* desired_goal;
    float* reward;
    uint8_t* success;
    uint8_t* terminated;
    uint8_t* truncated;
    float* terminal_obs;
    float* terminal_achieved_goal;
    float* terminal_desired_goal;
    uint8_t* task_truncated;      /* [N] u8 Task.is_truncated of the step (ReachAO: is_collided,
                                     reach_ao.py:1263-1264; 0 for the other tasks, reach.py:53-54),
                                     i.e. info["is_truncated"], without the TimeLimit part */
} pgx_step_out;

/* Device-resident state views (SoA, env-minor: x[k*N + env]). */
typedef struct pgx_state_view {
    float* q;           /* [n_dofs][N] */
    float* qd;          /* [n_dofs][N] */
    float* qc;          /* [n_dofs][N] pose of Bullet's cached link transforms, which getLinkState
                           reports (EE obs, IK target): the pose the last substep started from */
    double* goal;       /* [3][N] */
    float* object;      /* [13][N] pos3, quat4 (x,y,z,w), linvel3, angvel3 */
    float* contacts;    /* [2*PGX_CONTACT_SLOTS][N] warm-start cache: (id, normal impulse) per slot */
    float* obstacles;   /* [4*PGX_AO_OBSTACLES][N] ReachAO obstacle centres (x,y,z) then active flags */
    int32_t* elapsed;   /* [N] steps in the current episode */
    uint32_t* episode;  /* [N] episodes finished (RNG counter) */
    uint32_t* errors;   /* [1] sticky PGX_ERR_* bits set by the kernels; the host clears them */
    int32_t robot_points;  /* the robot contact budget of this handle's kernels (0: no contacts) */
    int32_t* env_order;    /* [N] the env order of the last step launch that sorted its envs heavy-first
                              (per-pair manifold kernels; position -> env id), the identity before
                              the first such launch, NULL for handles without the per-pair budget;
                              not state (the next sorted launch rewrites it) */
    float* manifolds;      /* [1 + manifold_pool * PGX_MANIFOLD_POINT][N] the persistent manifold pool
                              (PGX_MANIFOLD_POOL above), NULL without one */
    int32_t manifold_pool; /* its capacity in points (0: none) */
} pgx_state_view;

/* errors word (pgx_state_view.errors): a device-side reset that cannot complete the way the
 * reference's would.  PGX_ERR_AO_OBSTACLE: ReachAO.set_coll_free_obs drew 10000 obstacle
 * positions without a collision-free one, where the reference raises StopIteration
 * ("Couldn't find collision free obstacle!", reach_ao.py:1143-1145); the env keeps the last
 * draw and the host raises PgxError when it reads the bit. */
#define PGX_ERR_AO_OBSTACLE 1u

const char* pgx_version(void);
const char* pgx_last_error(void);
int pgx_obs_dim(const pgx_config* cfg);
int pgx_action_dim(const pgx_config* cfg);

/* libpgx.so compiles the device constant block in (the robot, pgx_sim_params, the scene's table
 * box and plane): a cfg that folds to another block fails with PGX_E_UNSUPPORTED, and
 * libpgx_rtmodel.so (the same kernels reading the handle's block) takes any. */
int pgx_create(const pgx_config* cfg, int device, pgx_handle* out);
/* Host only: the device constant block (PgxDevModel, nbytes = its size) pgx_create folds from cfg;
 * the build's generator of the kernels' compile-time defaults uses it. */
int pgx_dev_model_bytes(const pgx_config* cfg, void* out, int64_t nbytes);
void pgx_destroy(pgx_handle h);
int pgx_get_state(pgx_handle h, pgx_state_view* out);

/* Reset envs whose mask byte is non-zero (mask NULL = all).  inject_goal
 * [N,3] f64 (host-computed PCG64 draws for seeded resets) and inject_object
 * [N,3] f64 (Push/PickAndPlace object position) or [N,PGX_AO_OBSTACLES,3] f64 (ReachAO
 * obstacle centres, parked ones at (99.9, 99.9, -99.9)) override the device draws
 * where given.  Writes the reset obs. */
int pgx_reset(pgx_handle h, const uint8_t* env_mask, const double* inject_goal,
              const double* inject_object, pgx_step_out* out, void* stream);

/* One lockstep env step for all N envs: action [N,A] f32 (device). */
int pgx_step(pgx_handle h, const float* action, pgx_step_out* out, void* stream);
/* The step kernel the last pgx_step on h launched, as rocprof names it (e.g.
 * "step_kernel<0, 0, 1, 0, 2>"; NULL before the first step): the label a benchmark reports beside
 * its kernel time and profiles. */
const char* pgx_step_kernel(pgx_handle h);

/* Fill action [N,A] with U[-1,1) from the device Philox stream (benchmark
 * random policy; counter = (global env id, step)). */
int pgx_sample_actions(pgx_handle h, float* action, uint64_t step, void* stream);

/* Batched reward for relabelled goals: ag, dg [B,3] f32 device, out [B] f32.
 * Follows utils.distance (round to 1e-6) in float32 like the reference does
 * for float32 inputs. */
int pgx_compute_reward(const float* achieved_goal, const float* desired_goal, int64_t batch,
                       int32_t reward_type, double distance_threshold, float* out, void* stream);

/* Single-kernel copies of the whole SoA state into / out of a caller-owned device buffer. */
int pgx_state_bytes(pgx_handle h, int64_t* nbytes);
int pgx_save_state(pgx_handle h, void* dst_device, void* stream);
int pgx_restore_state(pgx_handle h, const void* src_device, void* stream);

/* State ids (PyBullet.save_state / restore_state / remove_state, pybullet.py:79-102; reached
 * through RobotTaskEnv.save_state / restore_state / remove_state, core.py:310-336).
 * pgx_snapshot copies the whole state into a buffer the handle owns and returns its id: the
 * first non-negative integer not in use (pybullet's saveState rule, so a released id is handed
 * out again).  pgx_restore copies it back; pgx_release frees it (it synchronises the device:
 * queued copies may still read the buffer).  Restoring or releasing an id that is not in use
 * returns PGX_E_INVALID ("no such saved state"), as restoreState after removeState raises
 * pybullet.error (test/save_and_restore_test.py:30-36).  pgx_destroy frees every snapshot. */
int pgx_snapshot(pgx_handle h, int32_t* state_id, void* stream);
int pgx_restore(pgx_handle h, int32_t state_id, void* stream);
int pgx_release(pgx_handle h, int32_t state_id);

/* Reset draws from numpy PCG64 streams instead of the device Philox counter (a
 * seeded reset drawn on the device, no host injection).  RobotTaskEnv.reset reseeds the task's
 * generator on EVERY reset, task.np_random = seeding.np_random(seed) (core.py:302): a reset with
 * seed s draws from PCG64(SeedSequence(s)), which is what a record set from s reproduces bit for bit
 * (goal / object in the task's order, reach.py:75-78, push.py:75-87, pick_and_place.py:71-85;
 * ReachAO's rejection sampler, reach_ao.py:965-1082, with Generator.uniform / random / integers /
 * shuffle as numpy draws them, and every accept / reject test decided in fp64 on the host's
 * capsules, pgx_config.ao_capsules_neutral -- the draws and the record bit for bit, ReachAO's goal
 * to a few ulp: the device's sin / cos / cbrt are not the host libm's).  A reset without a seed -- the step's auto-reset included -- gets a
 * fresh OS-entropy generator in the reference, so no reference value exists for it: here it
 * continues stream i, a reproducible stand-in with the same distribution, not the reference's
 * draws.  states: [N][PGX_PCG64_WORDS] uint64 per env {state_lo, state_hi, inc_lo, inc_hi,
 * has_uint32, uinteger} -- numpy's PCG64 bit_generator.state -- host or device memory, copied on
 * `stream`; NULL returns to Philox.  The mode is a device word switched on `stream` and the stream
 * buffer lives as long as the handle, so a step loop captured in a HIP graph draws in the mode of
 * replay time.  An injected reset leaves its env's stream untouched.  Streams are not part of the
 * saved state (restoreState keeps np_random as it is).  pgx_get_rng_streams copies the current
 * records out (same layout, host or device memory). */
#define PGX_PCG64_WORDS 6
int pgx_set_rng_streams(pgx_handle h, const uint64_t* states, void* stream);
int pgx_get_rng_streams(pgx_handle h, uint64_t* states, void* stream);

/* ------------------------------------------------------------------------
 * Device HER replay ring: the goal-relabelling replay buffer the reference's
 * training uses (SB3 HerReplayBuffer / the fork's VecHerReplayBuffer,
 * training/utils/setup_training.py:176-179; classes/train_config.py:15),
 * "future" strategy, relabelled rewards from Task.compute_reward
 * (reach.py:84-89 / pick_and_place.py:91-96) in float32.
 *
 * Storage is [capacity][n_envs] slot-major like SB3's (buffer_size, n_envs)
 * arrays, one padded record per transition so a sampled transition is one
 * contiguous gather; add() writes one transition per env at the shared ring
 * position, keeps SB3's episode bookkeeping (ep_start / ep_length,
 * invalidation of an overwritten episode) and refreshes the list of valid
 * transitions (ep_length > 0); sample() draws uniformly over that list,
 * relabels the first int(her_ratio*B) draws with the next_achieved_goal of a
 * transition t' of the same episode (strategy below) and recomputes their
 * rewards.  Draws come from the device Philox stream.
 *
 * Batch row layout (floats), row_dim = 2*obs_dim + action_dim + 14, rows
 * row_stride = round_up(row_dim, 4) apart:
 *   obs[obs_dim] | achieved_goal[3] | desired_goal[3] | action[action_dim] |
 *   reward | next_obs[obs_dim] | next_achieved_goal[3] | next_desired_goal[3] | done
 * SB3 order: the B - int(her_ratio*B) real rows first, then the relabelled rows.
 * ---------------------------------------------------------------------- */
typedef struct pgx_replay* pgx_replay_handle;

#define PGX_HER_FUTURE 0   /* t' uniform in [t, episode end) */
#define PGX_HER_FINAL 1    /* t' = last transition of the episode */
#define PGX_HER_EPISODE 2  /* t' uniform in [episode start, episode end) */

typedef struct pgx_replay_config {
    int32_t n_envs;
    int32_t capacity;             /* transitions per env (SB3 buffer_size) */
    int32_t obs_dim;
    int32_t action_dim;
    int32_t reward_type;          /* PGX_REWARD_* */
    int32_t strategy;             /* PGX_HER_* goal selection (SB3 GoalSelectionStrategy) */
    double distance_threshold;    /* 0.05 */
    double her_ratio;             /* 1 - 1/(n_sampled_goal+1) = 0.8 */
    uint64_t seed;
} pgx_replay_config;

/* One transition per env (device pointers): obs/next_obs [N,obs_dim], ag/dg/next_ag/next_dg
 * [N,3], action [N,A] f32, reward [N] f32, done [N] u8, timeout [N] u8 (TimeLimit.truncated). */
typedef struct pgx_transition {
    const float* obs;
    const float* achieved_goal;
    const float* desired_goal;
    const float* action;
    const float* reward;
    const float* next_obs;
    const float* next_achieved_goal;
    const float* next_desired_goal;
    const uint8_t* done;
    const uint8_t* timeout;
} pgx_transition;

/* Sampled, relabelled batch (device pointers).  rows [B, row_stride] f32 in the layout
 * above; done = done * (1 - timeout).  slot/env/goal_slot [B] i32 (optional, may be NULL):
 * the drawn indices, goal_slot -1 for real rows.  When no episode has completed yet (SB3
 * raises), every row is zero and slot = -1. */
typedef struct pgx_replay_batch {
    float* rows;
    int32_t* slot;
    int32_t* env;
    int32_t* goal_slot;
} pgx_replay_batch;

/* row_dim / row_stride of a batch row for this config (floats). */
int pgx_replay_row_dim(const pgx_replay_config* cfg);
int pgx_replay_row_stride(const pgx_replay_config* cfg);
int pgx_replay_create(const pgx_replay_config* cfg, int device, pgx_replay_handle* out);
void pgx_replay_destroy(pgx_replay_handle h);
int pgx_replay_add(pgx_replay_handle h, const pgx_transition* t, void* stream);
/* Number of transitions added per env so far (host-side counter, no sync). */
int64_t pgx_replay_size(pgx_replay_handle h);
int pgx_replay_sample(pgx_replay_handle h, int64_t batch, uint64_t draw, pgx_replay_batch* out, void* stream);
/* Device views of the bookkeeping arrays [capacity][n_envs] i32 and of the number of valid
 * transitions after the last add() (i32 scalar), for tests / checkpoint / the host guard. */
int pgx_replay_episode_arrays(pgx_replay_handle h, int32_t** ep_start, int32_t** ep_length, int32_t** n_valid);

#ifdef __cplusplus
}
#endif

#endif /* PGX_H */
