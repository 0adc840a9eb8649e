/*
 * pandasim.h — C ABI of the MI355X-native batched Panda simulator
 * (libpandasim.so, built from panda-lang-manip_amd/csrc/pandasim.hip).
 *
 * Drop-in boundary for the reference's step()/reset() path.  Each entry point
 * replaces one call site of /root/reference (cited per function); see
 * INTEGRATION.md for the host-side binding (ctypes) a maintainer adds.
 *
 * Conventions
 *   - Every buffer argument is a DEVICE pointer owned by the caller (PyTorch
 *     tensors in panda-lang-manip_amd/pandasim); the library never allocates
 *     per call and holds no host-language objects.
 *   - Calls are asynchronous on the given HIP stream (hipStream_t passed as
 *     void*; NULL = default stream).  One ps_ctx per (process, device); a
 *     context is not re-entrant.
 *   - Every call returns PS_OK (0) or a negative PS_ERR_* code; no C++
 *     exception crosses the ABI.  ps_last_error() gives the message.
 *   - Batched state lives in one caller-owned device buffer of
 *     ps_layout.total_bytes bytes, structure-of-arrays, described by ps_layout.
 *     save_state/restore_state (core.py:252-278) are copies of that buffer.
 */
#ifndef PANDASIM_H
#define PANDASIM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PS_ABI_VERSION 6

/* the six registered tasks (panda_gym/__init__.py:8-54) */
enum {
    PS_TASK_REACH = 0,
    PS_TASK_PUSH = 1,
    PS_TASK_PICK_AND_PLACE = 2,
    PS_TASK_SLIDE = 3,
    PS_TASK_STACK = 4,
    PS_TASK_FLIP = 5,
    PS_NUM_TASKS = 6
};
enum { PS_CONTROL_EE = 0, PS_CONTROL_JOINTS = 1 };
enum { PS_REWARD_SPARSE = 0, PS_REWARD_DENSE = 1 };
enum { PS_SHAPE_BOX = 0, PS_SHAPE_CYLINDER = 1 };
#define PS_VISUAL_SPHERE 2 /* ps_visual.target_shape only: create_sphere ghost (reach.py:31-38) */
enum { PS_OK = 0, PS_ERR_ARG = -1, PS_ERR_HIP = -2, PS_ERR_UNSUPPORTED = -3 };

/* Largest batch one context holds (2^28 envs, ~260 GB of state): the kernels
 * address an env's state rows by a 32-bit byte offset.  ps_state_layout and
 * ps_create return PS_ERR_ARG above it. */
#define PS_MAX_ENVS (1LL << 28)

/* Scene/env configuration.  ps_default_config() fills the registered env
 * (panda_gym/__init__.py:8-54 + envs/panda_tasks.py:14-113 + the task's
 * _create_scene); the scene fields let tests build the reference's
 * engine-level KAT scenes (test/pybullet_test.py).
 *   n_objects      dynamic objects: 0 (Reach), 1, or 2 (Stack)
 *   object_shape   PS_SHAPE_BOX (half extents object_half) or
 *                  PS_SHAPE_CYLINDER (radius object_half[0], half height
 *                  object_half[2], axis z; slide.py:33-42)
 *   object_mass    mass of object 1; object2_mass of object 2 (stack.py:33-55)
 *   object_friction lateral friction of the objects (default 0.5; Slide 0.04)
 *   table_cx/hx/hy table centre x and half extents (top at z = 0;
 *                  pybullet.py:741-771) */
typedef struct {
    int32_t task, control, reward, block_gripper;
    int32_t has_table, has_plane, n_objects, object_shape;
    float base[3];
    float object_half[3];
    float object_mass, object2_mass, object_friction;
    float table_cx, table_hx, table_hy;
} ps_config;

/* State layout: byte offsets from the state pointer.  Float fields are rows
 * of `stride` floats (env i at [row*stride + i]); goal is PS_MAX_GOAL_DIM
 * rows of doubles, rng is 5 rows of uint64 (PCG64 state hi, lo, inc hi, lo of
 * the task's np_random, then the splitmix64 state of Flip's goal stream),
 * elapsed one row of int32 (TimeLimit counter). */
#define PS_MAX_GOAL_DIM 6
enum {
    PS_F_Q = 0,        /* 9 joint positions (DoF order: joints 0..6, 9, 10) */
    PS_F_QD = 9,       /* 9 joint velocities */
    PS_F_MTARGET = 18, /* 9 motor target positions */
    PS_F_MKP = 27,     /* 9 motor position gains */
    PS_F_MKD = 36,     /* 9 motor velocity gains */
    PS_F_MVEL = 45,    /* 9 motor target velocities */
    PS_F_MIMP = 54,    /* 9 motor max impulses (force * 1/500 s) */
    PS_F_CPOS = 63,    /* 3 object position (world) */
    PS_F_CQUAT = 66,   /* 4 object orientation quaternion x,y,z,w */
    PS_F_CVEL = 70,    /* 3 object linear velocity */
    PS_F_COMG = 73,    /* 3 object angular velocity */
    PS_F_C2POS = 76,   /* object 2 (Stack): position, */
    PS_F_C2QUAT = 79,  /*   orientation, */
    PS_F_C2VEL = 83,   /*   linear velocity, */
    PS_F_C2OMG = 86,   /*   angular velocity */
    /* contact cache of the warm-started solver (Bullet's persistent contact
     * manifolds): the previous substep's contacts per group,
     * slot by slot, with their final normal impulses.  Id rows pack the four
     * slots' ids as sum_k id_k * 32^k (exact in f32), id = 1 + feature, 0 =
     * empty: ground slots 1 + support point, gripper slots 1 + sphere +
     * 8 * (0 object 1, 1 object 2, 2 ground). */
    PS_F_WG0 = 89,     /* 4 ground-contact normal impulses of object 1 */
    PS_F_WG0ID = 93,   /*   their packed ids */
    PS_F_WG1 = 94,     /* object 2 (Stack) */
    PS_F_WG1ID = 98,
    PS_F_WR = 99,      /* 4 gripper-contact normal impulses */
    PS_F_WRID = 103,   /*   their packed ids */
    PS_F_WP = 104,     /* 4 object-object (Stack) normal impulses, */
    PS_F_WPPT = 108,   /*   their points in object 1's frame (x, y, z per slot), */
    PS_F_WPN = 120,    /*   and how many slots are in use */
    PS_NUM_FLOAT_ROWS = 121,
    PS_NUM_RNG_ROWS = 5
};

typedef struct {
    int64_t num_envs, stride;
    int64_t float_offset, goal_offset, rng_offset, elapsed_offset;
    int64_t total_bytes;
} ps_layout;

typedef struct ps_ctx ps_ctx;

int ps_abi_version(void);
int ps_default_config(int task, int control, int reward, ps_config *out);
int ps_state_layout(int64_t num_envs, ps_layout *out);

/* gym.make(id) -> RobotTaskEnv.__init__ (core.py:209-227), minus the initial
 * reset, which the caller issues with ps_reset. */
int ps_create(const ps_config *cfg, int64_t num_envs, int device, ps_ctx **out);
void ps_destroy(ps_ctx *ctx);
const char *ps_last_error(const ps_ctx *ctx);
int ps_obs_dim(const ps_ctx *ctx);
int ps_action_dim(const ps_ctx *ctx);
int ps_goal_dim(const ps_ctx *ctx);        /* 3, 4 (Flip quaternion) or 6 (Stack) */
int ps_max_episode_steps(const ps_ctx *ctx); /* TimeLimit: 50, Stack 100 (__init__.py:18-46) */

/* Zero state, identity object orientation and PyBullet's default joint
 * velocity motors (loadURDF, core.py:40-52). */
int ps_init_state(ps_ctx *ctx, void *state, void *stream);

/* RobotTaskEnv.reset(seed) (core.py:240-250) for every env with mask[i] != 0
 * (mask == NULL: all).  seeds != NULL: env i is re-seeded with
 * Generator(PCG64(SeedSequence(seeds[i]))) (core.py:244); seeds == NULL: the
 * env's current generator continues.  obs/ag/dg may be NULL. */
int ps_reset(ps_ctx *ctx, void *state, const uint8_t *mask, const uint64_t *seeds, float *obs, float *ag,
             float *dg, void *stream);

/* RobotTaskEnv.step(action) (core.py:280-289) + TimeLimit(50), fused:
 * Panda.set_action (panda.py:52-107, incl. calculateInverseKinematics) ->
 * PyBullet.step (pybullet.py:52-55, 20 substeps) -> _get_obs -> is_success /
 * compute_reward.  actions: [B, action_dim] f32.  obs [B, obs_dim], ag/dg
 * [B, goal_dim], reward [B] f32, terminated/truncated [B] u8.  autoreset != 0:
 * finished envs are reset in-kernel (generator continues) and obs/ag/dg hold
 * the reset observation; final_obs/final_ag (may be NULL) receive the
 * pre-reset observation of every env. */
int ps_step(ps_ctx *ctx, void *state, const float *actions, float *obs, float *ag, float *dg, float *reward,
            uint8_t *terminated, uint8_t *truncated, int autoreset, float *final_obs, float *final_ag,
            void *stream);

/* Lanes per env of ps_step's kernel: 1 (one env per lane, the large-batch
 * kernel), 16 or 8 (a group of 16 or 8 lanes shares each env's constraint
 * solve -- the small-batch kernels, one object at most: not Stack); 0
 * (default) picks 16 for batches of at most PS_GROUP16_AUTO_MAX_ENVS envs, 8
 * up to PS_GROUP8_AUTO_MAX_ENVS and 1 above.  The kernels sum in different
 * orders, so their results agree to fp32 rounding, not bit for bit: fix the
 * value to compare runs of different batch sizes bit for bit. */
#define PS_GROUP16_AUTO_MAX_ENVS 4096
#define PS_GROUP8_AUTO_MAX_ENVS 8192
int ps_set_lanes_per_env(ps_ctx *ctx, int lanes);
int ps_step_lanes(const ps_ctx *ctx); /* the value ps_step uses */

/* gymnasium's RecordEpisodeStatistics, fused into ps_step (no reference
 * counterpart: the training loop's wrapper around gym.make).  stats != NULL:
 * device [4, B] f32, caller-owned, must outlive the steps: row 0 the running
 * return of each env's current episode, row 1 the return of its last finished
 * episode, row 2 that episode's success (terminated: 1, truncated: 0), row 3
 * the number of finished episodes.  Every following ps_step adds its reward
 * to row 0 and, when the episode ends, moves it to row 1 and clears it.
 * stats == NULL turns it off. */
int ps_set_episode_stats(ps_ctx *ctx, float *stats);

/* NaN/Inf guard of ps_step (no reference counterpart; SURVEY.md §5 failure
 * detection): with flags != NULL (device [B] u8, caller-owned, must outlive
 * the steps) every following ps_step writes flags[i] = 1 when env i's joint
 * or object state is not finite after the step, else 0; with
 * reset_nonfinite != 0 such an env is also reset in-kernel (its generator
 * continues, as in auto-reset) and reported truncated, even when ps_step's
 * autoreset is 0.  flags == NULL and reset_nonfinite == 0 turn it off. */
int ps_set_nonfinite_guard(ps_ctx *ctx, uint8_t *flags, int reset_nonfinite);

/* The fused step sets POSITION_CONTROL on all nine joints (panda.py:52-107 ->
 * control_joints, pybullet.py:462-477), as env.step does.  It stores the
 * motor targets and max impulses every step but the gain rows (kp, kd,
 * target velocity) only when they may differ from its own: on the first
 * ps_step after ps_create, ps_init_state or ps_reset, and after this call
 * (a step of a buffer at another address than the last step's also writes
 * them, but a caching allocator can hand a new buffer the old address, so
 * callers must not rely on that).  A caller that swaps buffers without a
 * ps_reset, or writes motor rows itself (the plugin path's control_joints,
 * a raw write into the state, a snapshot copied into it), calls it first. */
int ps_mark_motor_rows_dirty(ps_ctx *ctx);

/* Engine level: PyBullet.step() (pybullet.py:52-55) with the motors already in
 * the state (n_substeps of 1/500 s). */
int ps_sim_step(ps_ctx *ctx, void *state, int n_substeps, void *stream);

/* getLinkState(computeLinkVelocity=1) (pybullet.py:351-400) for all envs:
 * pos/lin_vel/ang_vel [B,3], quat [B,4]; any output may be NULL. */
int ps_link_state(ps_ctx *ctx, const void *state, int link, float *pos, float *quat, float *lin_vel,
                  float *ang_vel, void *stream);

/* calculateInverseKinematics (pybullet.py:479-497) from the current joint
 * positions: pos [B,3] world, orn [B,4] (x,y,z,w), q_out [B,9]. */
int ps_inverse_kinematics(ps_ctx *ctx, const void *state, int link, const float *pos, const float *orn,
                          float *q_out, void *stream);

/* --- pieces of the unfused (Robot/Task plugin) path, pandasim/core.py --- */

#define PS_MAX_UNIFORM 8

/* gymnasium.utils.seeding.np_random(seed) (core.py:244) for every env with
 * mask[i] != 0 (mask == NULL: all): env i's generator becomes
 * Generator(PCG64(SeedSequence(seeds[i]))).  seeds: device [B] uint64. */
int ps_rng_seed(ps_ctx *ctx, void *state, const uint8_t *mask, const uint64_t *seeds, void *stream);

/* np_random.uniform(low, high) with n = len(low) <= PS_MAX_UNIFORM
 * (reach.py:52, push.py:78,85, pick_and_place.py:75-76; random() is
 * uniform(0, 1)): n consecutive draws from each masked env's stream into
 * out [B, n] f64 (device).  low/high are HOST arrays of n doubles. */
int ps_rng_uniform(ps_ctx *ctx, void *state, const uint8_t *mask, int n, const double *low, const double *high,
                   double *out, void *stream);

/* Flip's goal, scipy Rotation.random().as_quat() (flip.py:70-72): the
 * reference draws it from numpy's unseeded global RandomState; here from each
 * masked env's splitmix64 goal stream (seeded with the env seed by ps_reset /
 * ps_rng_seed), four Box-Muller normals normalised, into out [B, 4] f64. */
int ps_rng_rotation(ps_ctx *ctx, void *state, const uint8_t *mask, double *out, void *stream);

/* getBasePositionAndOrientation / getEulerFromQuaternion / getBaseVelocity of
 * object `object` (0 or 1) (pybullet.py:284-349): pos, euler, lin_vel, ang_vel
 * [B,3], quat [B,4] (x,y,z,w); any output may be NULL.  PS_ERR_UNSUPPORTED if
 * the scene has no such object. */
int ps_base_state(ps_ctx *ctx, const void *state, int object, float *pos, float *quat, float *euler,
                  float *lin_vel, float *ang_vel, void *stream);

/* Task.compute_reward / is_success of `task` (reach.py:56-65, push.py:89-98,
 * stack.py:118-131, flip.py:80-91), vectorised for HER (core.py:226): n goal
 * pairs [n, goal_dim(task)], each f64 when its *_is_double flag is set, else
 * f32.  Goal-distance tasks use utils.distance (threshold 0.05, Stack 0.1),
 * Flip uses utils.angle_distance = 1 - <a, b>^2 (threshold 0.2).  As numpy
 * does, the arithmetic is f64 when either side is f64 and f32 (threshold
 * rounded to f32) when both are f32.  reward and success may be NULL. */
int ps_compute_reward(int task, int reward_type, const void *ag, int ag_is_double, const void *dg,
                      int dg_is_double, float *reward, uint8_t *success, int64_t n, void *stream);


/* --- camera images (pybullet.py:69-264; §8(f) rank 4) --- */

/* Visual description of the scene for ps_render: flat colours (r, g, b, a in
 * [0, 1]) by role -- 0 plane, 1 table, 2 object 1, 3 object 2, 4 target 1,
 * 5 target 2, 6 robot, 7 background -- and the ghost targets' shapes
 * (PS_SHAPE_BOX, PS_SHAPE_CYLINDER, PS_VISUAL_SPHERE; -1 = none) with box half
 * extents / cylinder (radius, radius, half height) / sphere (radius, ...). */
typedef struct {
    float rgba[8][4];
    int32_t target_shape[2];
    float target_half[2][3];
} ps_visual;

/* computeViewMatrixFromYawPitchRoll(target, distance, yaw, pitch, roll,
 * upAxisIndex=2) and computeProjectionMatrixFOV(fov=60, aspect=width/height,
 * near=0.1, far=100) as column-major float[16] (pybullet.py:69-107), and
 * tran_pix_world = inv(P V) of the order='F' matrices, row-major double[16]
 * (may be NULL).  Host arithmetic only: no context, no GPU. */
int ps_camera(const float target[3], float distance, float yaw, float pitch, float roll, int width, int height,
              float view[16], float proj[16], double tran_pix_world[16]);

/* getCameraImage(width, height, view, proj) of every env (pybullet.py:186-192):
 * depth [B, height, width] f32 (OpenGL window depth, 1 = nothing hit) and rgb
 * [B, height, width, 3] u8, either may be NULL.  targets: device [B, 2, 7] f32
 * ghost-target poses (position, quaternion x,y,z,w), NULL = no targets.  The
 * arm is drawn as capsules between its joint frames plus the gripper spheres
 * (the URDF meshes are not available); the rest of the scene is exact. */
int ps_render(ps_ctx *ctx, const void *state, const float view[16], const float proj[16], int width, int height,
              const ps_visual *vis, const float *targets, float *depth, uint8_t *rgb, void *stream);

/* render()'s deprojection (pybullet.py:203-262) of depth [B, h, w]: per pixel
 * the world point [B, h*w, 3] f64, valid [B, h*w] u8 (depth < 0.99 and
 * 0 < z < 0.67 and -0.5 < x < 0.2) and pixels_2d [B, h*w, 2] f64; outputs may
 * be NULL.  tran_pix_world: HOST row-major double[16]. */
int ps_deproject_image(ps_ctx *ctx, const float *depth, const double tran_pix_world[16], int width, int height,
                       double *points, uint8_t *valid, double *pixels_2d, void *stream);

/* PyBullet.deproject(depth, pixels, tran_pix_world) (pybullet.py:109-146):
 * n pixels (column, row) int32 per env [B, n, 2] -> points [B, n, 3] f64;
 * a pixel outside the image reads nothing and yields a NaN point. */
int ps_deproject_pixels(ps_ctx *ctx, const float *depth, const int32_t *pixels, int n,
                        const double tran_pix_world[16], int width, int height, double *points, void *stream);

#ifdef __cplusplus
}
#endif
#endif
