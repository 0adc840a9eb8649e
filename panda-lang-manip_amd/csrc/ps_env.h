// ps_env.h — the env layer shared by the kernel translation units of
// libpandasim.so: the state view, task-layer device code (set_action, obs,
// reward, reset) and the fused step / plugin-path substep kernels.  Each
// step_kernels.hip object instantiates the step kernels of one (task,
// control) pair and sim_kernels.hip those of one scene, so the library
// builds as parallel hipcc jobs (pandasim/build.py); pandasim.hip holds the
// C ABI and the small kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

#include "pandasim.h"
#include "ps_physics.h"
#include "ps_task.h"

using namespace ps;

struct ps_ctx {
    ps_config cfg;
    int64_t num_envs;
    ps_layout lay;
    int device;
    char err[256];
    float *render_prims;  // [B][RENDER_PRIM_FLOATS] scratch of ps_render, allocated on first use
    float *gstash;        // Stack: GSTASH_FLOATS x stride substep stash and pair rows, allocated on first step
    uint8_t *nonfinite;   // ps_set_nonfinite_guard: per-env flag output of ps_step (caller-owned), or NULL
    int reset_nonfinite;  // ... and reset such envs in-kernel
    int lanes_per_env;    // ps_set_lanes_per_env: 0 auto, 1 or 16
    int gains_dirty;      // the state's motor gain rows may differ from the fused step's (store_motor_gains)
    const void *gains_state;  // the state buffer whose gain rows the last successful ps_step wrote
    float *epstats;       // ps_set_episode_stats: caller-owned [4][num_envs] f32, or NULL
};

// arguments of ps_step that the step launchers pass through
struct ps_step_io {
    const float *actions;
    float *obs, *ag, *dg, *reward;
    uint8_t *terminated, *truncated;
    float *final_obs, *final_ag;
    int autoreset;
};

// one launcher per (task, control) pair (step_kernels.hip) and per scene
// (sim_kernels.hip); each lives in its own object
#define PS_STEP_LAUNCHER_NAME_(T, C) ps_launch_step_##T##_##C
#define PS_STEP_LAUNCHER_NAME(T, C) PS_STEP_LAUNCHER_NAME_(T, C)
#define PS_DECLARE_STEP_LAUNCHER(T, C) \
    int PS_STEP_LAUNCHER_NAME(T, C)(ps_ctx * c, void *state, const ps_step_io &io, int lanes, hipStream_t st);
PS_DECLARE_STEP_LAUNCHER(0, 0) PS_DECLARE_STEP_LAUNCHER(0, 1) PS_DECLARE_STEP_LAUNCHER(1, 0)
PS_DECLARE_STEP_LAUNCHER(1, 1) PS_DECLARE_STEP_LAUNCHER(2, 0) PS_DECLARE_STEP_LAUNCHER(2, 1)
PS_DECLARE_STEP_LAUNCHER(3, 0) PS_DECLARE_STEP_LAUNCHER(3, 1) PS_DECLARE_STEP_LAUNCHER(4, 0)
PS_DECLARE_STEP_LAUNCHER(4, 1) PS_DECLARE_STEP_LAUNCHER(5, 0) PS_DECLARE_STEP_LAUNCHER(5, 1)
// the 16- and 8-lane group kernels of a pair (not Stack) live in an object of
// their own (step_kernels.hip with -DPS_STEP_GROUPS=1), called by the pair's
// launcher
#define PS_STEP_GROUP_LAUNCHER_NAME_(T, C) ps_launch_step_groups_##T##_##C
#define PS_STEP_GROUP_LAUNCHER_NAME(T, C) PS_STEP_GROUP_LAUNCHER_NAME_(T, C)
#define PS_DECLARE_STEP_GROUP_LAUNCHER(T, C) \
    int PS_STEP_GROUP_LAUNCHER_NAME(T, C)(ps_ctx * c, const void *params, const ps_step_io &io, int lanes, hipStream_t st);
PS_DECLARE_STEP_GROUP_LAUNCHER(0, 0) PS_DECLARE_STEP_GROUP_LAUNCHER(0, 1) PS_DECLARE_STEP_GROUP_LAUNCHER(1, 0)
PS_DECLARE_STEP_GROUP_LAUNCHER(1, 1) PS_DECLARE_STEP_GROUP_LAUNCHER(2, 0) PS_DECLARE_STEP_GROUP_LAUNCHER(2, 1)
PS_DECLARE_STEP_GROUP_LAUNCHER(3, 0) PS_DECLARE_STEP_GROUP_LAUNCHER(3, 1) PS_DECLARE_STEP_GROUP_LAUNCHER(5, 0)
PS_DECLARE_STEP_GROUP_LAUNCHER(5, 1)
#define PS_SIM_LAUNCHER_NAME_(NOBJ, SHAPE) ps_launch_sim_step_##NOBJ##_##SHAPE
#define PS_SIM_LAUNCHER_NAME(NOBJ, SHAPE) PS_SIM_LAUNCHER_NAME_(NOBJ, SHAPE)
#define PS_DECLARE_SIM_LAUNCHER(NOBJ, SHAPE) \
    int PS_SIM_LAUNCHER_NAME(NOBJ, SHAPE)(ps_ctx * c, void *state, int n_substeps, hipStream_t st);
PS_DECLARE_SIM_LAUNCHER(0, 0) PS_DECLARE_SIM_LAUNCHER(1, 0) PS_DECLARE_SIM_LAUNCHER(1, 1)
PS_DECLARE_SIM_LAUNCHER(2, 0)

// the phase-counter buffer of the diagnostic build (pandasim.hip)
#ifdef PS_PROFILE_PHASES
unsigned long long *ps_prof_buffer();
#define PS_ITER_DUMP_ENVS 131072
uint32_t *ps_iter_dump_buffer();
#endif
#ifdef PS_DEBUG_ROW_DUMP
float *ps_row_dump_buffer();
#endif

// minimum waves per SIMD the step kernels are register-allocated for
#ifndef PS_STEP_MIN_WAVES
#define PS_STEP_MIN_WAVES 1
#endif

namespace {


constexpr int kBlock = 64;
static_assert(kBlock == CW_LANES, "robot_candidates: the work lists' output rows are kBlock lanes wide");

// Per-task constants (panda_gym/__init__.py:8-54, envs/panda_tasks.py:14-113,
// tasks/*.py): objects, shape, goal size, TimeLimit and success threshold.
template <int TASK>
struct TaskTraits {
    static constexpr int NOBJ = TASK == PS_TASK_REACH ? 0 : (TASK == PS_TASK_STACK ? 2 : 1);
    static constexpr int SHAPE = TASK == PS_TASK_SLIDE ? PS_SHAPE_CYLINDER : PS_SHAPE_BOX;
    static constexpr int GOAL = TASK == PS_TASK_STACK ? 6 : (TASK == PS_TASK_FLIP ? 4 : 3);
    static constexpr int STEPS = TASK == PS_TASK_STACK ? PM_STACK_MAX_EPISODE_STEPS : PM_MAX_EPISODE_STEPS;
    static constexpr double THRESHOLD = TASK == PS_TASK_STACK ? PM_STACK_DISTANCE_THRESHOLD
                                        : TASK == PS_TASK_FLIP ? PM_FLIP_DISTANCE_THRESHOLD
                                                               : PM_DISTANCE_THRESHOLD;
};

inline int task_nobj(int task) { return task == PS_TASK_REACH ? 0 : (task == PS_TASK_STACK ? 2 : 1); }
inline int task_goal_dim(int task) { return task == PS_TASK_STACK ? 6 : (task == PS_TASK_FLIP ? 4 : 3); }
inline int task_obs_dim(int task) {
    return task == PS_TASK_REACH ? 0 : (task == PS_TASK_STACK ? 24 : (task == PS_TASK_FLIP ? 13 : 12));
}

struct StateView {
    float *f;  // [PS_NUM_FLOAT_ROWS][stride]
    double *goal;
    uint64_t *rng;
    int32_t *elapsed;
    int64_t stride;
    // Row r of env i = a wave-uniform row base (SGPRs, rebuilt from the kernel
    // arguments by two scalar ops) plus the lane's 32-bit byte offset, which
    // the loads and stores take as `global_* v_off, s[base]`.  With a 64-bit
    // per-lane address per row the compiler kept 26 of them live from the
    // state loads at entry to the stores at exit: 208 B per lane of scratch
    // (spilled and written back to HBM every step) and AGPR copies through the
    // solver.  ps_create caps num_envs at PS_MAX_ENVS so i * 8 fits 32 bits.
    // The row base goes through an empty asm pinned to SGPRs: otherwise the
    // compiler reassociates (f + off) + row * stride back into one 64-bit
    // per-lane pointer per row.
    PS_D static uint32_t off(int64_t i, uint32_t size) { return (uint32_t)i * size; }
    // (readfirstlane first: the group kernels' divergence analysis does not
    // always see the base as uniform, and an SGPR operand needs one)
    template <class T>
    PS_D static T *pin(T *p) {
        const uint64_t u = (uint64_t)p;
        uint64_t r = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(u >> 32)) << 32) |
                     (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)u);
        asm("" : "+s"(r));
        return (T *)r;
    }
    template <class T>
    PS_D static T &at(T *row_base, int64_t i) {
        return *(T *)((char *)pin(row_base) + off(i, sizeof(T)));
    }
    PS_D float &F(int row, int64_t i) const { return at(f + row * stride, i); }
    PS_D double &G(int k, int64_t i) const { return at(goal + k * stride, i); }
    PS_D uint64_t &R(int k, int64_t i) const { return at(rng + k * stride, i); }
    PS_D int32_t &E(int64_t i) const { return at(elapsed, i); }
};

inline StateView view_of(const ps_ctx *c, void *state) {
    char *b = (char *)state;
    StateView v;
    v.f = (float *)(b + c->lay.float_offset);
    v.goal = (double *)(b + c->lay.goal_offset);
    v.rng = (uint64_t *)(b + c->lay.rng_offset);
    v.elapsed = (int32_t *)(b + c->lay.elapsed_offset);
    v.stride = c->lay.stride;
    return v;
}

struct KParams {
    StateView s;
    int64_t n;
    Scene sc;
    int reward_type, block_gripper, obs_dim, action_dim, autoreset;
    uint8_t *nonfinite;  // NaN/Inf guard output (ps_set_nonfinite_guard), NULL = off
    int reset_nonfinite;
    float *gstash;  // Stack: GSTASH_FLOATS x stride per-substep stash and pair rows (ctx scratch)
    int write_gains;  // k_step also stores the motor gain rows (ps_ctx::gains_dirty)
    float *epstats;   // ps_set_episode_stats: [4][epstride] running return, last return, last success, episodes
    int64_t epstride;
#ifdef PS_PROFILE_PHASES
    unsigned long long *prof;  // phase counters (ps_prof_buffer)
    uint32_t *itdump;          // per-env PGS iterations of the last step (ps_iter_dump_buffer)
#endif
#ifdef PS_DEBUG_ROW_DUMP
    float *dbg;  // row dump (ps_row_dump_buffer)
#endif
};

inline Scene scene_of(const ps_config &c) {
    Scene s;
    s.base = mk(c.base[0], c.base[1], c.base[2]);
    s.half = mk(c.object_half[0], c.object_half[1], c.object_half[2]);
    s.mass = c.object_mass;
    s.mass2 = c.object2_mass;
    s.fric = c.object_friction;
    s.table_cx = c.table_cx;
    s.table_hx = c.table_hx;
    s.table_hy = c.table_hy;
    s.has_table = c.has_table;
    s.has_plane = c.has_plane;
    return s;
}

// ------------------------------------------------------------ state I/O
PS_D void load_robot(const StateView &s, int64_t i, float q[9], float qd[9]) {
#pragma unroll
    for (int d = 0; d < 9; d++) {
        q[d] = s.F(PS_F_Q + d, i);
        qd[d] = s.F(PS_F_QD + d, i);
    }
}
PS_D void store_robot(const StateView &s, int64_t i, const float q[9], const float qd[9]) {
#pragma unroll
    for (int d = 0; d < 9; d++) {
        s.F(PS_F_Q + d, i) = q[d];
        s.F(PS_F_QD + d, i) = qd[d];
    }
}
PS_D void load_motors(const StateView &s, int64_t i, Motors &m) {
#pragma unroll
    for (int d = 0; d < 9; d++) {
        m.target[d] = s.F(PS_F_MTARGET + d, i);
        m.kp[d] = s.F(PS_F_MKP + d, i);
        m.kd[d] = s.F(PS_F_MKD + d, i);
        m.vel[d] = s.F(PS_F_MVEL + d, i);
        m.imp[d] = s.F(PS_F_MIMP + d, i);
    }
}
// The fused step's motors are POSITION_CONTROL with PyBullet's gains (kp 0.1,
// kd 1, target velocity 0) on all nine joints.  It stores the targets and max
// impulses every step (72 B per env) and the three gain rows (108 B) only when
// they may hold something else: on the first step after ps_create /
// ps_init_state, or after ps_mark_motor_rows_dirty (the plugin path's
// control_joints, a restored snapshot).  Until then they hold PyBullet's
// default velocity motors (kp 0, kd 1, k_init_state).
PS_D void store_motor_targets(const StateView &s, int64_t i, const Motors &m) {
#pragma unroll
    for (int d = 0; d < 9; d++) {
        s.F(PS_F_MTARGET + d, i) = m.target[d];
        s.F(PS_F_MIMP + d, i) = m.imp[d];
    }
}
PS_D void store_motor_gains(const StateView &s, int64_t i, const Motors &m) {
#pragma unroll
    for (int d = 0; d < 9; d++) {
        s.F(PS_F_MKP + d, i) = m.kp[d];
        s.F(PS_F_MKD + d, i) = m.kd[d];
        s.F(PS_F_MVEL + d, i) = m.vel[d];
    }
}
PS_D int body_row(int b) { return b == 0 ? PS_F_CPOS : PS_F_C2POS; }
PS_D void load_body(const StateView &s, int64_t i, int b, Body &c) {
    int r = body_row(b);
    c.pos = mk(s.F(r, i), s.F(r + 1, i), s.F(r + 2, i));
    c.quat = Q4{s.F(r + 3, i), s.F(r + 4, i), s.F(r + 5, i), s.F(r + 6, i)};
    c.vel = mk(s.F(r + 7, i), s.F(r + 8, i), s.F(r + 9, i));
    c.omg = mk(s.F(r + 10, i), s.F(r + 11, i), s.F(r + 12, i));
}
PS_D void store_body(const StateView &s, int64_t i, int b, const Body &c) {
    int r = body_row(b);
    s.F(r, i) = c.pos.x; s.F(r + 1, i) = c.pos.y; s.F(r + 2, i) = c.pos.z;
    s.F(r + 3, i) = c.quat.x; s.F(r + 4, i) = c.quat.y; s.F(r + 5, i) = c.quat.z; s.F(r + 6, i) = c.quat.w;
    s.F(r + 7, i) = c.vel.x; s.F(r + 8, i) = c.vel.y; s.F(r + 9, i) = c.vel.z;
    s.F(r + 10, i) = c.omg.x; s.F(r + 11, i) = c.omg.y; s.F(r + 12, i) = c.omg.z;
}
PS_D Pcg load_rng(const StateView &s, int64_t i) {
    return Pcg{s.R(0, i), s.R(1, i), s.R(2, i), s.R(3, i)};
}
PS_D void store_rng(const StateView &s, int64_t i, const Pcg &r) {
    s.R(0, i) = r.sh; s.R(1, i) = r.sl; s.R(2, i) = r.ih; s.R(3, i) = r.il;
}
PS_D uint64_t &aux_rng(const StateView &s, int64_t i) { return s.R(4, i); }

// The motor rows are constant over a control step.  The fused step's targets
// (its gains are PyBullet's defaults, STD_MOTORS) stay in 9 registers across
// the substeps; the plugin path's full rows (45 floats) are re-read from the
// state at every substep instead of occupying registers through the solver
// (the index goes through an empty asm so the loads stay in the loop).
// STD_MOTORS: `tgt` holds the targets set_action computed in this lane.
template <int NOBJ, int SHAPE, bool STD_MOTORS, int G = 1>
PS_D void run_substeps(const KParams &P, int64_t i, int n, float q[9], float qd[9], Body *bd,
                       const MJStore &lds, bool live, const float *tgt PS_PROF_PARAM) {
    static_assert(kBlock == 64, "WarmCache: one wave per workgroup");
    const WarmCache<G, NOBJ> wc{P.s.f + PS_F_WG0 * P.s.stride, P.s.stride, live, lds};
    wc.to_lds();
    // G > 1: the targets come back from the state rows, which every lane of
    // the group wrote with the same values (k_step); held in registers across
    // the substeps the 8-lane Slide kernel drifted from the one-lane kernel by
    // 2 cm (the lanes' dumped targets were identical: a codegen effect, not a
    // per-lane difference), through memory it is bit-identical to it
    float tgt_mem[9];
    if constexpr (G > 1) {
#pragma unroll
        for (int d = 0; d < 9; d++) tgt_mem[d] = STD_MOTORS ? P.s.F(PS_F_MTARGET + d, i) : 0.0f;
        tgt = tgt_mem;
    }
    for (int st = 0; st < n; st++) {
        int64_t ii = i;
        asm volatile("" : "+v"(ii));
        Motors m;
        if constexpr (STD_MOTORS) {
#pragma unroll
            for (int d = 0; d < 9; d++) m.target[d] = tgt[d];
        } else {
            load_motors(P.s, ii, m);
        }
#ifdef PS_DEBUG_ROW_DUMP
        float *dump = (P.dbg && st < 2 && ((uint64_t)blockIdx.x * 64 + __lane_id()) < PS_DUMP_LANES)
                          ? P.dbg + (((uint64_t)blockIdx.x * 64 + __lane_id()) * 2 + st) * PS_DUMP_ROWS
                          : nullptr;
#endif
        substep<NOBJ, SHAPE, STD_MOTORS, G>(P.sc, q, qd, m, bd, lds, wc PS_PROF_ARG PS_DUMP_ARG);
    }
    wc.from_lds();
}

// ------------------------------------------------------- task layer pieces
// ee = grasptarget (link 11; COM == link frame): position and COM velocity
PS_D void ee_state(const Scene &sc, const float q[9], const float qd[9], V3 &pos, V3 &vel) {
    Kin k;
    fk(q, k);
    V3 p = k.f[11].o;
    V3 v = mk(0, 0, 0);
#pragma unroll
    for (int d = 0; d < 7; d++) v = v + cross(col(k.f[d].R, 2), p - k.f[d].o) * qd[d];
    pos = p + sc.base;
    vel = v;
}

// RobotTaskEnv._get_obs (core.py:229-238): robot obs (panda.py:109-119), the
// task obs (push.py:49-63; stack.py:65-91 both objects; flip.py:53-60 with the
// quaternion in place of Euler angles) and the achieved goal
template <int TASK>
PS_D void write_obs(const KParams &P, int64_t i, const float q[9], const float qd[9], const Body *bd,
                    const double g[6], float *obs, float *ag, float *dg) {
    using T = TaskTraits<TASK>;
    V3 p, v;
    ee_state(P.sc, q, qd, p, v);
    float o[31];
    o[0] = p.x; o[1] = p.y; o[2] = p.z;
    o[3] = v.x; o[4] = v.y; o[5] = v.z;
    int k = 6;
    if (!P.block_gripper) o[k++] = q[7] + q[8];
#pragma unroll
    for (int b = 0; b < T::NOBJ; b++) {
        const Body &cb = bd[b];
        o[k] = cb.pos.x; o[k + 1] = cb.pos.y; o[k + 2] = cb.pos.z;
        k += 3;
        if constexpr (TASK == PS_TASK_FLIP) {
            o[k] = cb.quat.x; o[k + 1] = cb.quat.y; o[k + 2] = cb.quat.z; o[k + 3] = cb.quat.w;
            k += 4;
        } else {
            V3 e = euler_from_quat(cb.quat);
            o[k] = e.x; o[k + 1] = e.y; o[k + 2] = e.z;
            k += 3;
        }
        o[k] = cb.vel.x; o[k + 1] = cb.vel.y; o[k + 2] = cb.vel.z;
        o[k + 3] = cb.omg.x; o[k + 4] = cb.omg.y; o[k + 5] = cb.omg.z;
        k += 6;
    }
    float a[6];
    if constexpr (TASK == PS_TASK_REACH) {
        a[0] = p.x; a[1] = p.y; a[2] = p.z;
    } else if constexpr (TASK == PS_TASK_FLIP) {
        a[0] = bd[0].quat.x; a[1] = bd[0].quat.y; a[2] = bd[0].quat.z; a[3] = bd[0].quat.w;
    } else {
        a[0] = bd[0].pos.x; a[1] = bd[0].pos.y; a[2] = bd[0].pos.z;
        if constexpr (T::NOBJ == 2) { a[3] = bd[1].pos.x; a[4] = bd[1].pos.y; a[5] = bd[1].pos.z; }
    }
    if (obs) {
#pragma unroll
        for (int j = 0; j < 31; j++)
            if (j < P.obs_dim) obs[i * P.obs_dim + j] = o[j];
    }
    if (ag) {
#pragma unroll
        for (int j = 0; j < T::GOAL; j++) ag[i * T::GOAL + j] = a[j];
    }
    if (dg) {
#pragma unroll
        for (int j = 0; j < T::GOAL; j++) dg[i * T::GOAL + j] = __double2float_rn(g[j]);
    }
}

// achieved goal of the stepped state (float32, as _get_obs casts it)
template <int TASK>
PS_D void achieved(const KParams &P, const float q[9], const float qd[9], const Body *bd, float a[6]) {
    if constexpr (TASK == PS_TASK_REACH) {
        V3 p, v;
        ee_state(P.sc, q, qd, p, v);
        a[0] = p.x; a[1] = p.y; a[2] = p.z;
    } else if constexpr (TASK == PS_TASK_FLIP) {
        a[0] = bd[0].quat.x; a[1] = bd[0].quat.y; a[2] = bd[0].quat.z; a[3] = bd[0].quat.w;
    } else {
        a[0] = bd[0].pos.x; a[1] = bd[0].pos.y; a[2] = bd[0].pos.z;
        if constexpr (TaskTraits<TASK>::NOBJ == 2) { a[3] = bd[1].pos.x; a[4] = bd[1].pos.y; a[5] = bd[1].pos.z; }
    }
}

// utils.distance (3 or 6 values) / utils.angle_distance (Flip) of float32
// achieved vs float64 desired, in float64 as numpy promotes
template <int TASK>
PS_D double goal_metric(const float a[6], const double g[6]) {
#pragma clang fp contract(off)
    if constexpr (TASK == PS_TASK_FLIP) {
        double dot = opaque(__dmul_rn((double)a[0], g[0]));
#pragma unroll
        for (int k = 1; k < 4; k++) dot = __dadd_rn(dot, opaque(__dmul_rn((double)a[k], g[k])));
        return __dsub_rn(1.0, opaque(__dmul_rn(dot, dot)));
    } else {
        constexpr int N = TaskTraits<TASK>::GOAL;
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < N; k++) {
            double e = __dsub_rn((double)a[k], g[k]);
            double e2 = opaque(__dmul_rn(e, e));
            s = k == 0 ? e2 : __dadd_rn(s, e2);
        }
        return __dsqrt_rn(s);
    }
}

PS_D float reward_for(int reward_type, double d, double thr) {
    if (reward_type == 0) return d > thr ? -1.0f : -0.0f;
    return -__double2float_rn(d);
}

// splitmix64 stream of Flip's goal (oracle po_flip_goal): R.random()
// (flip.py:70-72) as a uniform unit quaternion by Marsaglia's method -- two
// rejection-sampled points of the unit disc, q = (x1, x2, x3 t, x4 t),
// t = sqrt((1 - s1) / s2).  Only correctly rounded +, *, / and sqrt, kept
// uncontracted, so the oracle's draws are reproduced bit for bit.
PS_D uint64_t splitmix64(uint64_t &st) {
    uint64_t z = (st += 0x9E3779B97F4A7C15ULL);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
PS_D uint64_t aux_seed(uint64_t seed) { return seed ^ 0x5851F42D4C957F2DULL; }
PS_D double aux_signed_unit(uint64_t &st) {
#pragma clang fp contract(off)
    return __dsub_rn(opaque(__dmul_rn((double)(splitmix64(st) >> 11), 2.0 / 9007199254740992.0)), 1.0);
}
PS_D double disc_point(uint64_t &st, double &x, double &y) {
#pragma clang fp contract(off)
    for (;;) {
        x = aux_signed_unit(st);
        y = aux_signed_unit(st);
        double s = __dadd_rn(opaque(__dmul_rn(x, x)), opaque(__dmul_rn(y, y)));
        if (s < 1.0 && s > 0.0) return s;
    }
}
PS_D void random_rotation(uint64_t &st, double q[4]) {
#pragma clang fp contract(off)
    double x1, x2, x3, x4;
    double s1 = disc_point(st, x1, x2);
    double s2 = disc_point(st, x3, x4);
    double t = __dsqrt_rn(__ddiv_rn(__dsub_rn(1.0, s1), s2));
    q[0] = x1;
    q[1] = x2;
    q[2] = __dmul_rn(x3, t);
    q[3] = __dmul_rn(x4, t);
}

// set_base_pose -> resetBasePositionAndOrientation (pybullet.py:427-439):
// PyBullet's init-pose command sets the base pose and, with it, zero base
// linear and angular velocity
PS_D void place(Body &b, double x, double y, double z) {
    b.pos = mk((float)x, (float)y, (float)z);
    b.quat = Q4{0.0f, 0.0f, 0.0f, 1.0f};
    b.vel = mk(0.0f, 0.0f, 0.0f);
    b.omg = mk(0.0f, 0.0f, 0.0f);
}

// a reset teleports the robot and the objects: every cached contact breaks
// (its points drift beyond the breaking threshold)
PS_D void clear_contact_cache(const StateView &s, int64_t i) {
#pragma unroll
    for (int r = PS_F_WG0; r < PS_NUM_FLOAT_ROWS; r++) s.F(r, i) = 0.0f;
}

// Panda.reset + Task.reset (core.py:245-247): goal then object draws in the
// reference's order (reach.py:47-54, push.py:69-87, pick_and_place.py:65-85,
// slide.py:69-87, stack.py:103-116, flip.py:66-78)
template <int TASK>
PS_D void reset_env(float q[9], float qd[9], Body *bd, double g[6], Pcg &r, uint64_t &aux) {
#pragma unroll
    for (int d = 0; d < 9; d++) {
        q[d] = (float)neutral_q(d);
        qd[d] = 0.0f;
    }
    constexpr double xy = 0.3 / 2;  // goal_xy_range / 2 = obj_xy_range / 2
    if constexpr (TASK == PS_TASK_REACH) {
        g[0] = uniform(r, -xy, xy);
        g[1] = uniform(r, -xy, xy);
        g[2] = uniform(r, 0.0, 0.3);
    } else if constexpr (TASK == PS_TASK_STACK) {
        constexpr double size = PM_OBJECT_SIZE;
        double n0 = uniform(r, -xy, xy), n1 = uniform(r, -xy, xy), n2 = uniform(r, 0.0, 0.0);
        g[0] = __dadd_rn(0.0, n0);
        g[1] = __dadd_rn(0.0, n1);
        g[2] = __dadd_rn(size / 2, n2);
        g[3] = __dadd_rn(0.0, n0);
        g[4] = __dadd_rn(0.0, n1);
        g[5] = __dadd_rn(3 * size / 2, n2);
        double a0 = uniform(r, -xy, xy), a1 = uniform(r, -xy, xy), a2 = uniform(r, 0.0, 0.0);
        double b0 = uniform(r, -xy, xy), b1 = uniform(r, -xy, xy), b2 = uniform(r, 0.0, 0.0);
        place(bd[0], __dadd_rn(0.0, a0), __dadd_rn(0.0, a1), __dadd_rn(size / 2, a2));
        place(bd[1], __dadd_rn(0.0, b0), __dadd_rn(0.0, b1), __dadd_rn(3 * size / 2, b2));
    } else if constexpr (TASK == PS_TASK_FLIP) {
        random_rotation(aux, g);
        double o0 = uniform(r, -xy, xy), o1 = uniform(r, -xy, xy), o2 = uniform(r, 0.0, 0.0);
        place(bd[0], __dadd_rn(0.0, o0), __dadd_rn(0.0, o1), __dadd_rn(PM_OBJECT_SIZE / 2, o2));
    } else {
        // Push, PickAndPlace, Slide
        constexpr double size = TASK == PS_TASK_SLIDE ? PM_SLIDE_OBJECT_SIZE : PM_OBJECT_SIZE;
        constexpr double gx = TASK == PS_TASK_SLIDE ? PM_SLIDE_GOAL_X_OFFSET : 0.0;
        constexpr double zr = TASK == PS_TASK_PICK_AND_PLACE ? 0.2 : 0.0;
        double n0 = uniform(r, -xy + gx, xy + gx), n1 = uniform(r, -xy, xy), n2 = uniform(r, 0.0, zr);
        if (TASK == PS_TASK_PICK_AND_PLACE && pcg_double(r) < 0.3) n2 = 0.0;
        g[0] = __dadd_rn(0.0, n0);
        g[1] = __dadd_rn(0.0, n1);
        g[2] = __dadd_rn(size / 2, n2);
        double o0 = uniform(r, -xy, xy), o1 = uniform(r, -xy, xy), o2 = uniform(r, 0.0, 0.0);
        place(bd[0], __dadd_rn(0.0, o0), __dadd_rn(0.0, o1), __dadd_rn(size / 2, o2));
    }
}

// Panda.set_action (panda.py:52-107) -> motor targets (control_joints)
template <int CONTROL>
PS_D void set_action(const KParams &P, const float *act, const float q[9], Motors &m) {
    float a[8];
#pragma unroll
    for (int j = 0; j < 8; j++) a[j] = j < P.action_dim ? fminf(fmaxf(act[j], -1.0f), 1.0f) : 0.0f;
    float tq[9];
    if constexpr (CONTROL == PS_CONTROL_EE) {
        V3 p, v;
        float zero[9];
#pragma unroll
        for (int d = 0; d < 9; d++) zero[d] = 0.0f;
        ee_state(P.sc, q, zero, p, v);
        V3 t = p + mk(a[0] * 0.05f, a[1] * 0.05f, a[2] * 0.05f);
        t.z = fmaxf(0.0f, t.z);
        float qik[9];
        inverse_kinematics<11>(q, t - P.sc.base, Q4{1.0f, 0.0f, 0.0f, 0.0f}, qik);
#pragma unroll
        for (int d = 0; d < 7; d++) tq[d] = qik[d];
    } else {
#pragma unroll
        for (int d = 0; d < 7; d++) tq[d] = q[d] + a[d] * 0.05f;
    }
    float width = 0.0f;
    if (!P.block_gripper) width = (q[7] + q[8]) + a[P.action_dim - 1] * 0.2f;
    tq[7] = tq[8] = width * 0.5f;
#pragma unroll
    for (int d = 0; d < 9; d++) {
        m.target[d] = tq[d];
        m.kp[d] = (float)PM_MOTOR_KP;
        m.kd[d] = (float)PM_MOTOR_KD;
        m.vel[d] = 0.0f;
        m.imp[d] = (float)(joint_force(d) * PM_TIMESTEP);
    }
}


// ----------------------------------------------------------- host helpers
inline int fail(ps_ctx *c, int code, const char *msg) {
    if (c) snprintf(c->err, sizeof c->err, "%s", msg);
    return code;
}

inline int check_launch(ps_ctx *c) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        if (c) snprintf(c->err, sizeof c->err, "HIP launch failed: %s", hipGetErrorString(e));
        return PS_ERR_HIP;
    }
    return PS_OK;
}

inline KParams params_of(ps_ctx *c, void *state) {
    KParams P;
    P.s = view_of(c, state);
    P.n = c->num_envs;
    P.sc = scene_of(c->cfg);
    P.reward_type = c->cfg.reward;
    P.block_gripper = c->cfg.block_gripper;
    P.obs_dim = ps_obs_dim(c);
    P.action_dim = ps_action_dim(c);
    P.autoreset = 0;
    P.gstash = c->gstash;
    P.nonfinite = nullptr;
    P.reset_nonfinite = 0;
    P.write_gains = 0;
    P.epstats = c->epstats;
    P.epstride = c->num_envs;
#ifdef PS_PROFILE_PHASES
    P.prof = ps_prof_buffer();
    P.itdump = ps_iter_dump_buffer();
#endif
#ifdef PS_DEBUG_ROW_DUMP
    P.dbg = ps_row_dump_buffer();
#endif
    return P;
}

// Stack's global stash (the LDS it would use holds its ground rows): one
// allocation on the first step of a two-object context, never per step
inline int ensure_stash(ps_ctx *c, hipStream_t st) {
#ifdef PS_EXPERIMENT_TWO_WAVES
    const int64_t floats = c->cfg.n_objects == 2 ? GSTASH_FLOATS : GX_FLOATS;
#else
    if (c->cfg.n_objects != 2) return PS_OK;
    const int64_t floats = GSTASH_FLOATS;
#endif
    if (c->gstash) return PS_OK;
    const size_t bytes = sizeof(float) * (floats * c->lay.stride + GSTASH_ZERO_FLOATS);
    if (hipMalloc((void **)&c->gstash, bytes) != hipSuccess) {
        c->gstash = nullptr;
        return PS_ERR_HIP;
    }
    // all-zero (the solver's zero block after the stash, GSTASH_ZERO_FLOATS),
    // on the stream the steps run on
    if (hipMemsetAsync(c->gstash, 0, bytes, st) != hipSuccess) return PS_ERR_HIP;
    return PS_OK;
}

inline dim3 grid_of(int64_t n, int block) { return dim3((unsigned)((n + block - 1) / block)); }


// the registered scene of each task (its _create_scene + panda_tasks.py)
inline bool scene_matches_task(const ps_config &c) {
    return c.n_objects == task_nobj(c.task) &&
           (c.n_objects == 0 || c.object_shape == (c.task == PS_TASK_SLIDE ? PS_SHAPE_CYLINDER : PS_SHAPE_BOX));
}


// The fused env step: G lanes = one env = one full RobotTaskEnv.step().
// G = 1: one env per lane (large batches).  G = 16 (small batches, NOBJ <= 1):
// the 16 lanes of a group run the same setup and share the solver
// (group_pgs); lane 0 of the group writes the env's results, and the groups
// of the last wave past the batch end compute a copy of the last env and
// write nothing.
template <int TASK, int CONTROL, int G = 1>
__global__ __launch_bounds__(kBlock, PS_STEP_MIN_WAVES) void k_step(KParams P, const float *actions, float *obs, float *ag, float *dg,
                                                 float *reward, uint8_t *terminated, uint8_t *truncated,
                                                 float *final_obs, float *final_ag) {
    using T = TaskTraits<TASK>;
    const int64_t gi = ((int64_t)step_block<G>() * blockDim.x + threadIdx.x) / G;
    if (G == 1 && gi >= P.n) return;
    const bool live = gi < P.n;
    const int64_t i = live ? gi : P.n - 1;
    const bool writer = G == 1 || (live && (threadIdx.x % G) == 0);
    const StateView &s = P.s;
#ifdef PS_PROFILE_PHASES
    PhaseTimer pt;
    pt.last = (uint32_t)__builtin_amdgcn_s_memtime();
    for (int k = 0; k < PS_NUM_PROF_SLOTS; k++) pt.acc[k] = 0;
    for (int k = 0; k < PS_ITP_WORDS; k++) pt.itp[k] = 0;
#endif
    float q[9], qd[9];
    load_robot(s, i, q, qd);
    Body bd[T::NOBJ > 0 ? T::NOBJ : 1];
#pragma unroll
    for (int b = 0; b < T::NOBJ; b++) load_body(s, i, b, bd[b]);
    float tgt[9];
    {
        Motors m;
        set_action<CONTROL>(P, actions + i * P.action_dim, q, m);
        // every lane of a group stores the same targets (no lane reads a value
        // only another lane wrote; run_substeps reads them back for G > 1)
        if (G > 1 || writer) store_motor_targets(s, i, m);
        if (writer && P.write_gains) store_motor_gains(s, i, m);
#pragma unroll
        for (int d = 0; d < 9; d++) tgt[d] = m.target[d];
    }
    PS_PHASE(6);
    // LDS columns: one per lane, or one per env when the group's lanes share it
    // (shared_lds<G>, then the work lists' per-lane output rows after them)
    constexpr bool SHARED = shared_lds<G>();
    constexpr int NCOL = SHARED ? kBlock / G : kBlock;
    __shared__ float smem[lds_floats<T::NOBJ>() * NCOL + (SHARED ? CW_OUT_FLOATS * kBlock : 0)];
    MJStore lds{(lds_float *)(smem + (SHARED ? threadIdx.x / G : threadIdx.x)), NCOL};
    lds.cwo = SHARED ? (lds_float *)(smem + lds_floats<T::NOBJ>() * NCOL + threadIdx.x) : lds.base + CW_OUT * kBlock;
    if constexpr (T::NOBJ == 2) {
        lds.gst = P.gstash;
        lds.gst_stride = s.stride;
        lds.goff = StateView::off(i, 4);
        lds.gpair = (__attribute__((address_space(1))) float *)(P.gstash + (int64_t)GSTASH_PAIR_OFFSET * s.stride +
                                                                 i * (NP * PAIR_FLOATS));
        lds.ggrip = (__attribute__((address_space(1))) float *)(P.gstash + (int64_t)GSTASH_GRIP_OFFSET * s.stride +
                                                                 i * GRIP_FLOATS);
        lds.gzero = (__attribute__((address_space(1))) float *)(P.gstash + (int64_t)GSTASH_FLOATS * s.stride);
    }
#ifdef PS_EXPERIMENT_TWO_WAVES
    if constexpr (T::NOBJ < 2) {
        lds.gx = (__attribute__((address_space(1))) float *)P.gstash;
        lds.gxl = (uint32_t)(((i >> 6) * (GX_FLOATS * 64) + (i & 63)) * 4);
    }
#endif
    run_substeps<T::NOBJ, T::SHAPE, true, G>(P, i, PM_SUBSTEPS, q, qd, bd, lds, live, tgt PS_PROF_ARG);
    double g[6] = {0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int d = 0; d < T::GOAL; d++) g[d] = s.G(d, i);
    float a[6];
    achieved<TASK>(P, q, qd, bd, a);
    double dist = goal_metric<TASK>(a, g);
    bool term = dist < T::THRESHOLD;
    int el = s.E(i) + 1;
    bool trunc = el >= T::STEPS;
    const float rew = reward_for(P.reward_type, dist, T::THRESHOLD);
    if (writer) {
        reward[i] = rew;
        terminated[i] = term;
        truncated[i] = trunc;
    }
    // NaN/Inf guard: a non-finite joint or object state is
    // flagged, and with reset_nonfinite the env is reset and reported truncated
    bool reset_bad = false;
    if (P.nonfinite || P.reset_nonfinite) {
        bool ok = true;
#pragma unroll
        for (int d = 0; d < 9; d++) ok = ok && isfinite(q[d]) && isfinite(qd[d]);
#pragma unroll
        for (int b = 0; b < T::NOBJ; b++)
            ok = ok && isfinite(bd[b].pos.x + bd[b].pos.y + bd[b].pos.z + bd[b].quat.x + bd[b].quat.y + bd[b].quat.z +
                                bd[b].quat.w + bd[b].vel.x + bd[b].vel.y + bd[b].vel.z + bd[b].omg.x + bd[b].omg.y +
                                bd[b].omg.z);
        if (P.nonfinite && writer) P.nonfinite[i] = !ok;
        if (!ok && P.reset_nonfinite) {
            trunc = true;
            if (writer) truncated[i] = 1;
            reset_bad = true;
        }
    }
    if ((P.autoreset && (term || trunc)) || reset_bad) {
        if (writer && (final_obs || final_ag)) write_obs<TASK>(P, i, q, qd, bd, g, final_obs, final_ag, nullptr);
        Pcg r = load_rng(s, i);
        uint64_t aux = aux_rng(s, i);
        reset_env<TASK>(q, qd, bd, g, r, aux);
        if (writer) {
            store_rng(s, i, r);
            aux_rng(s, i) = aux;
            for (int d = 0; d < T::GOAL; d++) s.G(d, i) = g[d];
            clear_contact_cache(s, i);
        }
        el = 0;
    } else if (writer && (final_obs || final_ag)) {
        write_obs<TASK>(P, i, q, qd, bd, g, final_obs, final_ag, nullptr);
    }
    if (writer && P.epstats) {
        // RecordEpisodeStatistics, fused (ps_set_episode_stats): the running
        // return of the episode, and at its end (terminated or truncated,
        // incl. the guard's reset) the finished episode's return and success
        float *e = P.epstats + i;
        const int64_t w = P.epstride;
        const float run = e[0] + rew;
        if (term || trunc) {
            e[w] = run;
            e[2 * w] = term ? 1.0f : 0.0f;
            e[3 * w] += 1.0f;
            e[0] = 0.0f;
        } else {
            e[0] = run;
        }
    }
    if (writer) {
        s.E(i) = el;
        store_robot(s, i, q, qd);
#pragma unroll
        for (int b = 0; b < T::NOBJ; b++) store_body(s, i, b, bd[b]);
        write_obs<TASK>(P, i, q, qd, bd, g, obs, ag, dg);
    }
#ifdef PS_PROFILE_PHASES
    PS_PHASE(7);
    if ((threadIdx.x & 63) == 0)
        for (int k = 0; k < PS_NUM_PROF_SLOTS; k++)
            atomicAdd(&P.prof[k], (unsigned long long)pt.acc[k]);
    if (G == 1 && P.itdump && i < PS_ITER_DUMP_ENVS)
        for (int k = 0; k < PS_ITP_WORDS; k++) P.itdump[(int64_t)k * PS_ITER_DUMP_ENVS + i] = pt.itp[k];
#endif
}

template <int NOBJ, int SHAPE>
__global__ __launch_bounds__(kBlock) void k_sim_step(KParams P, int n_substeps) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P.n) return;
    const StateView &s = P.s;
    float q[9], qd[9];
    load_robot(s, i, q, qd);
    Body bd[NOBJ > 0 ? NOBJ : 1];
#pragma unroll
    for (int b = 0; b < NOBJ; b++) load_body(s, i, b, bd[b]);
    __shared__ float smem[lds_floats<NOBJ>() * kBlock];
    MJStore lds{(lds_float *)(smem + threadIdx.x), kBlock};
    lds.cwo = lds.base + CW_OUT * kBlock;
    if constexpr (NOBJ == 2) {
        lds.gst = P.gstash;
        lds.gst_stride = s.stride;
        lds.goff = StateView::off(i, 4);
        lds.gpair = (__attribute__((address_space(1))) float *)(P.gstash + (int64_t)GSTASH_PAIR_OFFSET * s.stride +
                                                                 i * (NP * PAIR_FLOATS));
        lds.ggrip = (__attribute__((address_space(1))) float *)(P.gstash + (int64_t)GSTASH_GRIP_OFFSET * s.stride +
                                                                 i * GRIP_FLOATS);
        lds.gzero = (__attribute__((address_space(1))) float *)(P.gstash + (int64_t)GSTASH_FLOATS * s.stride);
    }
#ifdef PS_EXPERIMENT_TWO_WAVES
    if constexpr (NOBJ < 2) {
        lds.gx = (__attribute__((address_space(1))) float *)P.gstash;
        lds.gxl = (uint32_t)(((i >> 6) * (GX_FLOATS * 64) + (i & 63)) * 4);
    }
#endif
#ifdef PS_PROFILE_PHASES
    PhaseTimer pt;
    pt.last = (uint32_t)__builtin_amdgcn_s_memtime();
    for (int k = 0; k < PS_NUM_PROF_SLOTS; k++) pt.acc[k] = 0;
#endif
    run_substeps<NOBJ, SHAPE, false>(P, i, n_substeps, q, qd, bd, lds, true, nullptr PS_PROF_ARG);
    store_robot(s, i, q, qd);
#pragma unroll
    for (int b = 0; b < NOBJ; b++) store_body(s, i, b, bd[b]);
}

}  // namespace
