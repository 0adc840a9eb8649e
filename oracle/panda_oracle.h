/*
 * panda_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU fp64 restatement of the PandaReach/Push/PickAndPlace-v3 step()/reset()
 * path of the reference (panda_gym/envs/core.py:240-289, robots/panda.py,
 * tasks/{reach,push,pick_and_place}.py, pybullet.py) and of the subset of the
 * third-party PyBullet 3.2.5 engine those files call (pinned version:
 * env.yml:107; not vendored in /root/reference, so its published algorithm is
 * restated: btMultiBody forward dynamics, btMultiBodyJointMotor,
 * btMultiBodyJointLimitConstraint, btMultiBodyConstraintSolver PGS,
 * IKTrajectoryHelper DLS inverse kinematics, getEulerFromQuaternion) and of
 * numpy's SeedSequence/PCG64/Generator.uniform used by gymnasium.seeding.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
 * this library, and only as the checker.  The product path
 * (panda-lang-manip_amd/) never links or calls it.
 *
 * Parity pins: tests/golden/ (task layer, generated from the reference's own
 * task classes) and the known-answer tests of test/pybullet_test.py.
 */
#ifndef PANDA_ORACLE_H
#define PANDA_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
    PO_TASK_REACH = 0,
    PO_TASK_PUSH = 1,
    PO_TASK_PICK_AND_PLACE = 2,
    PO_TASK_SLIDE = 3,
    PO_TASK_STACK = 4,
    PO_TASK_FLIP = 5
};
enum { PO_CONTROL_EE = 0, PO_CONTROL_JOINTS = 1 };
enum { PO_REWARD_SPARSE = 0, PO_REWARD_DENSE = 1 };
enum { PO_SHAPE_BOX = 0, PO_SHAPE_CYLINDER = 1 };
#define PO_MAX_OBJECTS 2
#define PO_MAX_GOAL 6

/* mirrors ps_config (include/pandasim.h) in fp64, plus has_robot for the
 * engine-level KAT scenes that have no robot */
typedef struct {
    int32_t task, control, reward, block_gripper;
    int32_t has_table, has_plane, n_objects, object_shape;
    int32_t has_robot, reserved;
    double base[3];
    double object_half[3];
    double object_mass, object2_mass, object_friction;
    double table_cx, table_hx, table_hy;
} po_config;

typedef struct {
    double pos[3], quat[4], vel[3], omg[3]; /* quat (x,y,z,w) body->world */
} po_body;

/* Contact cache of the warm-started solver (Bullet's persistent manifolds,
 * btPersistentManifold + btContactSolverInfo::m_warmstartingFactor): the
 * contacts of the previous substep, slot by slot in generation order, with
 * their final normal impulses.  Ids are 1 + the contact's feature (0 = empty):
 * ground slots of object b: 1 + support-point index; gripper slots:
 * 1 + sphere + 8 * (0 object 1, 1 object 2, 2 ground).  Object-object (Stack)
 * contacts have no fixed feature: they keep the contact point in object 1's
 * frame and are matched by distance, as btPersistentManifold::getCacheEntry. */
#define PO_CACHE_SLOTS 4
typedef struct {
    double ground_lam[PO_MAX_OBJECTS][PO_CACHE_SLOTS];
    double robot_lam[PO_CACHE_SLOTS];
    double pair_lam[PO_CACHE_SLOTS];
    double pair_pt[PO_CACHE_SLOTS][3];
    int32_t ground_id[PO_MAX_OBJECTS][PO_CACHE_SLOTS];
    int32_t robot_id[PO_CACHE_SLOTS];
    int32_t pair_n, reserved;
} po_cache;

typedef struct {
    double q[9], qd[9];
    double m_target[9], m_kp[9], m_kd[9], m_vel[9], m_maximp[9];
    po_body obj[PO_MAX_OBJECTS];
    double goal[PO_MAX_GOAL];
    int64_t elapsed;
    uint64_t rng[5]; /* PCG64 state hi, lo, inc hi, lo; splitmix64 state of Flip's goal stream */
    po_cache cache;
    /* test bookkeeping, not physics: signature of the last substep's discrete
     * state (contact features and the arm's joint-limit rows, 0 = none yet)
     * and how many substeps changed it; the same for the two finger joints'
     * limit rows (po_substep; the event-onset parity tests) */
    uint64_t event_sig;
    int64_t event_changes;
    uint64_t finger_sig;
    int64_t finger_changes;
    /* which parts of event_sig have changed so far: bit 0 the contact
     * features, bit 1 the arm's joint-limit rows */
    uint64_t contact_sig, limit_sig;
    int64_t event_kinds;
} po_env;

/* Work counters (bench.py's FLOP roofline): substeps, PGS
 * iterations, rows and contacts summed over substeps; row visits = rows of a
 * kind x the substep's PGS iterations (one visit = one row update; friction
 * pairs count once); IK iterations per env step. */
typedef struct {
    int64_t substeps, pgs_iterations, rows, contacts;
    int64_t motor_rows, limit_rows, ground_contacts, robot_contacts, pair_contacts;
    int64_t motor_visits, limit_visits, ground_visits, robot_visits, pair_visits;
    int64_t steps, ik_iterations;
} po_stats;

void po_default_config(po_config *cfg, int task, int control, int reward);
void po_init_env(const po_config *cfg, po_env *env);

/* --- engine-level primitives (pybullet.py wrapper semantics) --- */
void po_link_state(const po_config *cfg, const po_env *env, int link, double pos[3], double quat[4],
                   double lin_vel[3], double ang_vel[3]);
void po_inverse_kinematics(const po_config *cfg, const double q_start[9], int link, const double pos[3],
                           const double orn[4], double q_out[9]);
void po_control_joints(po_env *env, int n, const int32_t *joints, const double *targets, const double *forces);
void po_link_frames(const po_config *cfg, const po_env *env, double R[][9], double o[][3]);
int po_num_spheres(void);
void po_gripper_spheres(const po_config *cfg, const po_env *env, double c[][3], double r[]);
void po_substep(const po_config *cfg, po_env *env, po_stats *stats);
void po_sim_step(const po_config *cfg, po_env *env, po_stats *stats);
void po_euler_from_quaternion(const double q[4], double rpy[3]);

/* --- env-level (core.py) --- */
int po_obs_dim(const po_config *cfg);
int po_action_dim(const po_config *cfg);
int po_goal_dim(const po_config *cfg);
int po_max_episode_steps(const po_config *cfg);
void po_reset(const po_config *cfg, po_env *env, int has_seed, uint64_t seed, float *obs, float *ag, float *dg);
void po_get_obs(const po_config *cfg, const po_env *env, float *obs, float *ag, float *dg);
void po_step(const po_config *cfg, po_env *env, const float *action, float *obs, float *ag, float *dg,
             float *reward, uint8_t *terminated, uint8_t *truncated, int autoreset, float *final_obs,
             float *final_ag, po_stats *stats);
int po_set_threads(int n);
void po_step_batch(const po_config *cfg, po_env *envs, int n, const float *actions, float *obs, float *ag,
                   float *dg, float *reward, uint8_t *terminated, uint8_t *truncated, int autoreset,
                   po_stats *stats);
/* Task.compute_reward / is_success of one (float32 achieved, float64 desired)
 * goal pair of `task` (goal_dim values each) */
float po_compute_reward(int task, int reward_type, const float *ag, const double *dg);
uint8_t po_is_success(int task, const float *ag, const double *dg);

/* --- numpy SeedSequence / PCG64; splitmix64 + Box-Muller for Flip's goal --- */
void po_flip_goal(uint64_t *aux_state, double quat[4]);
void po_pcg64_seed(uint64_t seed, uint64_t rng[4]);
uint64_t po_pcg64_next(uint64_t rng[4]);
double po_pcg64_double(uint64_t rng[4]);

/* --- introspection used by the tests --- */
void po_mass_matrix(const po_config *cfg, const double q[9], double M[81]);
void po_bias_forces(const po_config *cfg, const double q[9], const double qd[9], double h[9]);
void po_link_inertia(int link, double inertia[3]);
void po_set_link_aabb(int link, double lx, double ly, double lz);
/* test hook: deliberate model errors for the parity classifier's power test
 * (tests/test_judge_power.py); PO_MUT_NONE restores the model, not thread-safe */
/* test hook: the PGS exits k iterations after its stopping rule is met (k > 0) or
 * one iteration before (k < 0): parity_judge's stopping-rule probe; not thread-safe */
void po_set_pgs_shift(int k);
/* test hook: the box-box clip lines moved outward by m metres (parity_judge's
 * pair-order probe); not thread-safe */
void po_set_clip_bias(double m);
#define PO_MUT_NONE 0
#define PO_MUT_MOTOR_KP 1     /* kp := PM_MOTOR_KP x value */
#define PO_MUT_LINK_DAMPING 2 /* btMultiBody damping k1 = k2 of every body := value */
#define PO_MUT_FINGER_BOX 3   /* finger boxes' half extents += value (m) */
#define PO_MUT_PAIR_FRICTION 4 /* cube-cube friction coefficient (Stack) := its default x value */
void po_set_model_mutation(int kind, double value);
/* test hook: per-substep finger-position noise of +-amplitude (0 = off), not thread-safe */
void po_set_finger_noise(double amplitude, uint64_t seed);
/* test hook: after every substep each state component x (q, qd, object pose
 * and velocities) moves by u * ulp32(x), u uniform in [-ulps, ulps] -- the
 * fp32 resolution of the state (0 = off), not thread-safe */
void po_set_state_noise(double ulps, uint64_t seed);
/* test hook: while buf != NULL every substep appends its PGS iteration count
 * (up to cap entries); returns the entries the previous buffer received */
int64_t po_set_pgs_log(int32_t *buf, int64_t cap);

#ifdef __cplusplus
}
#endif
#endif
