// pandasim.hip — gfx950 kernels and the C ABI (include/pandasim.h) of the
// batched Panda simulator.  One env per lane; every kernel reads/writes the
// structure-of-arrays state with coalesced row accesses.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

#include <new>

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
};

#ifdef PS_PROFILE_PHASES
__device__ unsigned long long ps_phase_cycles[PS_NUM_PHASES];
extern "C" int ps_debug_phase_cycles(unsigned long long *out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(ps_phase_cycles), sizeof(unsigned long long) * PS_NUM_PHASES) != hipSuccess)
        return PS_ERR_HIP;
    if (reset) {
        unsigned long long z[PS_NUM_PHASES] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(ps_phase_cycles), z, sizeof z) != hipSuccess) return PS_ERR_HIP;
    }
    return PS_OK;
}
#endif

namespace {

constexpr int kBlock = 64;

struct StateView {
    float *f;  // [76][stride]
    double *goal;
    uint64_t *rng;
    int32_t *elapsed;
    int64_t stride;
    PS_D float &F(int row, int64_t i) const { return f[row * stride + i]; }
};

StateView view_of(const ps_ctx *c, void *state) {
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
};

Scene scene_of(const ps_config &c) {
    Scene s;
    s.base = mk(c.base[0], c.base[1], c.base[2]);
    s.half = c.cube_half;
    s.mass = c.cube_mass;
    s.has_table = c.has_table;
    s.has_plane = c.has_plane;
    s.has_cube = c.has_cube;
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
PS_D void store_motors(const StateView &s, int64_t i, const Motors &m) {
#pragma unroll
    for (int d = 0; d < 9; d++) {
        s.F(PS_F_MTARGET + d, i) = m.target[d];
        s.F(PS_F_MKP + d, i) = m.kp[d];
        s.F(PS_F_MKD + d, i) = m.kd[d];
        s.F(PS_F_MVEL + d, i) = m.vel[d];
        s.F(PS_F_MIMP + d, i) = m.imp[d];
    }
}

// The motor rows' targets/gains are constant over a control step: they are
// re-read from the (L2-resident) state buffer at every substep instead of
// occupying 45 registers through the solver.  The index goes through an empty
// asm so the loads cannot be hoisted out of the substep loop.
template <bool HAS_CUBE, bool STD_MOTORS>
PS_D void run_substeps(const KParams &P, int64_t i, int n, float q[9], float qd[9], Cube &cb,
                       const MJStore &lds PS_PROF_PARAM) {
    for (int st = 0; st < n; st++) {
        int64_t ii = i;
        asm volatile("" : "+v"(ii));
        Motors m;
        if constexpr (STD_MOTORS) {
#pragma unroll
            for (int d = 0; d < 9; d++) m.target[d] = P.s.F(PS_F_MTARGET + d, ii);
        } else {
            load_motors(P.s, ii, m);
        }
        substep<HAS_CUBE, STD_MOTORS>(P.sc, q, qd, m, cb, lds PS_PROF_ARG);
    }
}
PS_D void load_cube(const StateView &s, int64_t i, Cube &c) {
    c.pos = mk(s.F(PS_F_CPOS, i), s.F(PS_F_CPOS + 1, i), s.F(PS_F_CPOS + 2, i));
    c.quat = Q4{s.F(PS_F_CQUAT, i), s.F(PS_F_CQUAT + 1, i), s.F(PS_F_CQUAT + 2, i), s.F(PS_F_CQUAT + 3, i)};
    c.vel = mk(s.F(PS_F_CVEL, i), s.F(PS_F_CVEL + 1, i), s.F(PS_F_CVEL + 2, i));
    c.omg = mk(s.F(PS_F_COMG, i), s.F(PS_F_COMG + 1, i), s.F(PS_F_COMG + 2, i));
}
PS_D void store_cube(const StateView &s, int64_t i, const Cube &c) {
    s.F(PS_F_CPOS, i) = c.pos.x; s.F(PS_F_CPOS + 1, i) = c.pos.y; s.F(PS_F_CPOS + 2, i) = c.pos.z;
    s.F(PS_F_CQUAT, i) = c.quat.x; s.F(PS_F_CQUAT + 1, i) = c.quat.y;
    s.F(PS_F_CQUAT + 2, i) = c.quat.z; s.F(PS_F_CQUAT + 3, i) = c.quat.w;
    s.F(PS_F_CVEL, i) = c.vel.x; s.F(PS_F_CVEL + 1, i) = c.vel.y; s.F(PS_F_CVEL + 2, i) = c.vel.z;
    s.F(PS_F_COMG, i) = c.omg.x; s.F(PS_F_COMG + 1, i) = c.omg.y; s.F(PS_F_COMG + 2, i) = c.omg.z;
}
PS_D Pcg load_rng(const StateView &s, int64_t i) {
    return Pcg{s.rng[i], s.rng[s.stride + i], s.rng[2 * s.stride + i], s.rng[3 * s.stride + i]};
}
PS_D void store_rng(const StateView &s, int64_t i, const Pcg &r) {
    s.rng[i] = r.sh; s.rng[s.stride + i] = r.sl; s.rng[2 * s.stride + i] = r.ih; s.rng[3 * s.stride + i] = r.il;
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

// RobotTaskEnv._get_obs (core.py:229-238)
template <int TASK>
PS_D void write_obs(const KParams &P, int64_t i, const float q[9], const float qd[9], const Cube &cb,
                    const double g[3], float *obs, float *ag, float *dg) {
    V3 p, v;
    ee_state(P.sc, q, qd, p, v);
    float o[19];
    o[0] = p.x; o[1] = p.y; o[2] = p.z;
    o[3] = v.x; o[4] = v.y; o[5] = v.z;
    int k = 6;
    if (!P.block_gripper) o[k++] = q[7] + q[8];
    float a0 = p.x, a1 = p.y, a2 = p.z;
    if constexpr (TASK != PS_TASK_REACH) {
        V3 e = euler_from_quat(cb.quat);
        o[k] = cb.pos.x; o[k + 1] = cb.pos.y; o[k + 2] = cb.pos.z;
        o[k + 3] = e.x; o[k + 4] = e.y; o[k + 5] = e.z;
        o[k + 6] = cb.vel.x; o[k + 7] = cb.vel.y; o[k + 8] = cb.vel.z;
        o[k + 9] = cb.omg.x; o[k + 10] = cb.omg.y; o[k + 11] = cb.omg.z;
        a0 = cb.pos.x; a1 = cb.pos.y; a2 = cb.pos.z;
    }
    if (obs) {
#pragma unroll
        for (int j = 0; j < 19; j++)
            if (j < P.obs_dim) obs[i * P.obs_dim + j] = o[j];
    }
    if (ag) { ag[i * 3] = a0; ag[i * 3 + 1] = a1; ag[i * 3 + 2] = a2; }
    if (dg) {
        dg[i * 3] = __double2float_rn(g[0]);
        dg[i * 3 + 1] = __double2float_rn(g[1]);
        dg[i * 3 + 2] = __double2float_rn(g[2]);
    }
}

// Panda.reset + Task.reset (core.py:245-247)
template <int TASK>
PS_D void reset_env(const KParams &P, int64_t i, float q[9], float qd[9], Cube &cb, double g[3], Pcg &r) {
#pragma unroll
    for (int d = 0; d < 9; d++) {
        q[d] = (float)neutral_q(d);
        qd[d] = 0.0f;
    }
    if constexpr (TASK == PS_TASK_REACH) {
        g[0] = uniform(r, -0.15, 0.15);
        g[1] = uniform(r, -0.15, 0.15);
        g[2] = uniform(r, 0.0, 0.3);
    } else {
        const double zr = TASK == PS_TASK_PICK_AND_PLACE ? 0.2 : 0.0;
        double n0 = uniform(r, -0.15, 0.15), n1 = uniform(r, -0.15, 0.15), n2 = uniform(r, 0.0, zr);
        if (TASK == PS_TASK_PICK_AND_PLACE && pcg_double(r) < 0.3) n2 = 0.0;
        const double half = PM_CUBE_HALF;  // object_size / 2 in fp64 (push.py:19, 75-80)
        g[0] = __dadd_rn(0.0, n0);
        g[1] = __dadd_rn(0.0, n1);
        g[2] = __dadd_rn(half, n2);
        double o0 = uniform(r, -0.15, 0.15), o1 = uniform(r, -0.15, 0.15), o2 = uniform(r, 0.0, 0.0);
        cb.pos = mk((float)__dadd_rn(0.0, o0), (float)__dadd_rn(0.0, o1), (float)__dadd_rn(half, o2));
        cb.quat = Q4{0.0f, 0.0f, 0.0f, 1.0f};
        // object velocity is not reset (resetBasePositionAndOrientation only)
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
#ifndef PS_DBG_NO_IK
        inverse_kinematics<11>(q, t - P.sc.base, Q4{1.0f, 0.0f, 0.0f, 0.0f}, qik);
#else
        for (int d = 0; d < 9; d++) qik[d] = q[d] + t.x;
#endif
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

// ---------------------------------------------------------------- kernels
__global__ __launch_bounds__(kBlock) void k_init_state(KParams P) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P.n) return;
    const StateView &s = P.s;
    for (int r = 0; r < PS_NUM_FLOAT_ROWS; r++) s.F(r, i) = 0.0f;
    s.F(PS_F_CQUAT + 3, i) = 1.0f;
    for (int d = 0; d < 9; d++) {
        s.F(PS_F_MKD + d, i) = 1.0f;
        s.F(PS_F_MIMP + d, i) = (float)PM_DEFAULT_MOTOR_MAX_IMPULSE;
    }
    for (int d = 0; d < 3; d++) s.goal[d * s.stride + i] = 0.0;
    store_rng(s, i, pcg_seed(0));
    s.elapsed[i] = 0;
}

template <int TASK>
__global__ __launch_bounds__(kBlock) void k_reset(KParams P, const uint8_t *mask, const uint64_t *seeds, float *obs,
                                                  float *ag, float *dg) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P.n) return;
    if (mask && !mask[i]) return;
    const StateView &s = P.s;
    Pcg r = seeds ? pcg_seed(seeds[i]) : load_rng(s, i);
    float q[9], qd[9];
    Cube cb;
    load_cube(s, i, cb);
    double g[3];
    reset_env<TASK>(P, i, q, qd, cb, g, r);
    store_robot(s, i, q, qd);
    if constexpr (TASK != PS_TASK_REACH) store_cube(s, i, cb);
    for (int d = 0; d < 3; d++) s.goal[d * s.stride + i] = g[d];
    store_rng(s, i, r);
    s.elapsed[i] = 0;
    write_obs<TASK>(P, i, q, qd, cb, g, obs, ag, dg);
}

// The fused env step: one lane = one env = one full RobotTaskEnv.step().
template <int TASK, int CONTROL>
__global__ __launch_bounds__(kBlock) void k_step(KParams P, const float *actions, float *obs, float *ag, float *dg,
                                                 float *reward, uint8_t *terminated, uint8_t *truncated,
                                                 float *final_obs, float *final_ag) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P.n) return;
    const StateView &s = P.s;
    constexpr bool HAS_CUBE = TASK != PS_TASK_REACH;
#ifdef PS_PROFILE_PHASES
    PhaseTimer pt;
    pt.last = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < PS_NUM_PHASES; k++) pt.acc[k] = 0;
#endif
    float q[9], qd[9];
    load_robot(s, i, q, qd);
    Cube cb;
    if constexpr (HAS_CUBE) load_cube(s, i, cb);
    {
        Motors m;
        set_action<CONTROL>(P, actions + i * P.action_dim, q, m);
        store_motors(s, i, m);
    }
    PS_PHASE(6);
    __shared__ float smem[LDS_FLOATS * kBlock];
    MJStore lds{(lds_float *)(smem + threadIdx.x), kBlock};
    run_substeps<HAS_CUBE, true>(P, i, PM_SUBSTEPS, q, qd, cb, lds PS_PROF_ARG);
    double g[3] = {s.goal[i], s.goal[s.stride + i], s.goal[2 * s.stride + i]};
    // obs of the stepped state
    float a0, a1, a2;
    {
        V3 p, v;
        ee_state(P.sc, q, qd, p, v);
        a0 = HAS_CUBE ? cb.pos.x : p.x;
        a1 = HAS_CUBE ? cb.pos.y : p.y;
        a2 = HAS_CUBE ? cb.pos.z : p.z;
    }
    double dist = goal_distance(a0, a1, a2, g[0], g[1], g[2]);
    bool term = dist < PM_DISTANCE_THRESHOLD;
    int el = s.elapsed[i] + 1;
    bool trunc = el >= PM_MAX_EPISODE_STEPS;
    reward[i] = reward_of(P.reward_type, dist);
    terminated[i] = term;
    truncated[i] = trunc;
    if (P.autoreset && (term || trunc)) {
        if (final_obs || final_ag) write_obs<TASK>(P, i, q, qd, cb, g, final_obs, final_ag, nullptr);
        Pcg r = load_rng(s, i);
        reset_env<TASK>(P, i, q, qd, cb, g, r);
        store_rng(s, i, r);
        for (int d = 0; d < 3; d++) s.goal[d * s.stride + i] = g[d];
        el = 0;
    } else if (final_obs || final_ag) {
        write_obs<TASK>(P, i, q, qd, cb, g, final_obs, final_ag, nullptr);
    }
    s.elapsed[i] = el;
    store_robot(s, i, q, qd);
    if constexpr (HAS_CUBE) store_cube(s, i, cb);
    write_obs<TASK>(P, i, q, qd, cb, g, obs, ag, dg);
#ifdef PS_PROFILE_PHASES
    PS_PHASE(7);
    if ((threadIdx.x & 63) == 0)
        for (int k = 0; k < PS_NUM_PHASES; k++) atomicAdd((unsigned long long *)&ps_phase_cycles[k], (unsigned long long)pt.acc[k]);
#endif
}

template <bool HAS_CUBE>
__global__ __launch_bounds__(kBlock) void k_sim_step(KParams P, int n_substeps) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P.n) return;
    const StateView &s = P.s;
    float q[9], qd[9];
    load_robot(s, i, q, qd);
    Cube cb;
    if constexpr (HAS_CUBE) load_cube(s, i, cb);
    __shared__ float smem[LDS_FLOATS * kBlock];
    MJStore lds{(lds_float *)(smem + threadIdx.x), kBlock};
#ifdef PS_PROFILE_PHASES
    PhaseTimer pt;
    pt.last = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < PS_NUM_PHASES; k++) pt.acc[k] = 0;
#endif
    run_substeps<HAS_CUBE, false>(P, i, n_substeps, q, qd, cb, lds PS_PROF_ARG);
    store_robot(s, i, q, qd);
    if constexpr (HAS_CUBE) store_cube(s, i, cb);
}

__global__ __launch_bounds__(kBlock) void k_link_state(KParams P, int link, float *pos, float *quat, float *lv,
                                                       float *av) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P.n) return;
    float q[9], qd[9];
    load_robot(P.s, i, q, qd);
    Kin k;
    fk(q, k);
    // COM frame of `link` (getLinkState [0], [1], [6], [7])
    M3 R = k.f[0].R;
    V3 o = k.f[0].o;
    V3 c = mk(0, 0, 0);
    static_for<0, PM_NUM_LINKS>([&](auto L) {
        constexpr int l = decltype(L)::value;
        if (l == link) {
            R = k.f[l].R;
            o = k.f[l].o;
            c = com_pos<l>(k);
        }
    });
    V3 v = mk(0, 0, 0), w = mk(0, 0, 0);
    static_for<0, 9>([&](auto D) {
        constexpr int d = decltype(D)::value;
        constexpr int jl = dof_def(d).link;
        // ancestor-or-self test on the fixed tree: arm joints precede every
        // later link; finger joints only move their own finger
        bool anc = (jl <= 6) ? (jl <= link) : (jl == link);
        if (anc) {
            V3 a = dof_axis<d>(k);
            if (link_def(jl).type == PM_JOINT_REVOLUTE) {
                v = v + cross(a, c - k.f[jl].o) * qd[d];
                w = w + a * qd[d];
            } else {
                v = v + a * qd[d];
            }
        }
    });
    (void)o;
    if (pos) { V3 p = c + P.sc.base; pos[i * 3] = p.x; pos[i * 3 + 1] = p.y; pos[i * 3 + 2] = p.z; }
    if (quat) { Q4 qq = mat_to_quat(R); quat[i * 4] = qq.x; quat[i * 4 + 1] = qq.y; quat[i * 4 + 2] = qq.z; quat[i * 4 + 3] = qq.w; }
    if (lv) { lv[i * 3] = v.x; lv[i * 3 + 1] = v.y; lv[i * 3 + 2] = v.z; }
    if (av) { av[i * 3] = w.x; av[i * 3 + 1] = w.y; av[i * 3 + 2] = w.z; }
}

template <int LINK>
__global__ __launch_bounds__(kBlock) void k_ik(KParams P, const float *pos, const float *orn, float *q_out) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P.n) return;
    float q[9], qd[9];
    load_robot(P.s, i, q, qd);
    V3 t = mk(pos[i * 3], pos[i * 3 + 1], pos[i * 3 + 2]) - P.sc.base;
    Q4 o = Q4{orn[i * 4], orn[i * 4 + 1], orn[i * 4 + 2], orn[i * 4 + 3]};
    float out[9];
    inverse_kinematics<LINK>(q, t, o, out);
    for (int d = 0; d < 9; d++) q_out[i * 9 + d] = out[d];
}

// gymnasium.utils.seeding.np_random(seed) per env (core.py:244): the env's
// generator becomes Generator(PCG64(SeedSequence(seeds[i])))
__global__ __launch_bounds__(kBlock) void k_rng_seed(KParams P, const uint8_t *mask, const uint64_t *seeds) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P.n || (mask && !mask[i])) return;
    store_rng(P.s, i, pcg_seed(seeds[i]));
}

// Generator.uniform(low[n], high[n]) per env: n consecutive draws from the
// env's own stream (push.py:75-80 draws a 3-vector in one call)
struct UniformArgs {
    int n;
    double lo[PS_MAX_UNIFORM], hi[PS_MAX_UNIFORM];
};
__global__ __launch_bounds__(kBlock) void k_rng_uniform(KParams P, const uint8_t *mask, UniformArgs u, double *out) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P.n || (mask && !mask[i])) return;
    Pcg r = load_rng(P.s, i);
    for (int k = 0; k < u.n; k++) out[i * u.n + k] = uniform(r, u.lo[k], u.hi[k]);
    store_rng(P.s, i, r);
}

// getBasePositionAndOrientation + getEulerFromQuaternion + getBaseVelocity of
// the object (pybullet.py:284-349)
__global__ __launch_bounds__(kBlock) void k_base_state(KParams P, float *pos, float *quat, float *euler, float *vel,
                                                       float *avel) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P.n) return;
    Cube c;
    load_cube(P.s, i, c);
    if (pos) { pos[i * 3] = c.pos.x; pos[i * 3 + 1] = c.pos.y; pos[i * 3 + 2] = c.pos.z; }
    if (quat) { quat[i * 4] = c.quat.x; quat[i * 4 + 1] = c.quat.y; quat[i * 4 + 2] = c.quat.z; quat[i * 4 + 3] = c.quat.w; }
    if (euler) { V3 e = euler_from_quat(c.quat); euler[i * 3] = e.x; euler[i * 3 + 1] = e.y; euler[i * 3 + 2] = e.z; }
    if (vel) { vel[i * 3] = c.vel.x; vel[i * 3 + 1] = c.vel.y; vel[i * 3 + 2] = c.vel.z; }
    if (avel) { avel[i * 3] = c.omg.x; avel[i * 3 + 1] = c.omg.y; avel[i * 3 + 2] = c.omg.z; }
}

__global__ __launch_bounds__(256) void k_compute_reward(int reward_type, const void *ag, int ag_dbl, const void *dg,
                                                        int dg_dbl, float *reward, uint8_t *success, int64_t n) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (ag_dbl || dg_dbl) {
        // numpy promotes the mixed pair to float64 (utils.py:15)
        double a[3], g[3];
        for (int k = 0; k < 3; k++) {
            a[k] = ag_dbl ? ((const double *)ag)[i * 3 + k] : (double)((const float *)ag)[i * 3 + k];
            g[k] = dg_dbl ? ((const double *)dg)[i * 3 + k] : (double)((const float *)dg)[i * 3 + k];
        }
        double dist = goal_distance_f64(a[0], a[1], a[2], g[0], g[1], g[2]);
        if (reward) reward[i] = reward_of(reward_type, dist);
        if (success) success[i] = dist < PM_DISTANCE_THRESHOLD;
    } else {
        const float *a = (const float *)ag, *g = (const float *)dg;
        float dist = goal_distance_f32(a[i * 3], a[i * 3 + 1], a[i * 3 + 2], g[i * 3], g[i * 3 + 1], g[i * 3 + 2]);
        if (reward) reward[i] = reward_of_f32(reward_type, dist);
        if (success) success[i] = dist < (float)PM_DISTANCE_THRESHOLD;
    }
}

// ----------------------------------------------------------- host helpers
int fail(ps_ctx *c, int code, const char *msg) {
    if (c) snprintf(c->err, sizeof c->err, "%s", msg);
    return code;
}

int check_launch(ps_ctx *c) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        if (c) snprintf(c->err, sizeof c->err, "HIP launch failed: %s", hipGetErrorString(e));
        return PS_ERR_HIP;
    }
    return PS_OK;
}

KParams params_of(ps_ctx *c, void *state) {
    KParams P;
    P.s = view_of(c, state);
    P.n = c->num_envs;
    P.sc = scene_of(c->cfg);
    P.reward_type = c->cfg.reward;
    P.block_gripper = c->cfg.block_gripper;
    P.obs_dim = ps_obs_dim(c);
    P.action_dim = ps_action_dim(c);
    P.autoreset = 0;
    return P;
}

dim3 grid_of(int64_t n, int block) { return dim3((unsigned)((n + block - 1) / block)); }

}  // namespace

// ------------------------------------------------------------------- C ABI
extern "C" {

int ps_abi_version(void) { return PS_ABI_VERSION; }

int ps_default_config(int task, int control, int reward, ps_config *out) {
    if (!out || task < 0 || task > 2 || control < 0 || control > 1 || reward < 0 || reward > 1) return PS_ERR_ARG;
    memset(out, 0, sizeof *out);
    out->task = task;
    out->control = control;
    out->reward = reward;
    out->block_gripper = task != PS_TASK_PICK_AND_PLACE;
    out->has_table = 1;
    out->has_plane = 1;
    out->has_cube = task != PS_TASK_REACH;
    out->base[0] = (float)PM_BASE_X;
    out->cube_half = (float)PM_CUBE_HALF;
    out->cube_mass = (float)PM_CUBE_MASS;
    return PS_OK;
}

int ps_state_layout(int64_t num_envs, ps_layout *out) {
    if (!out || num_envs <= 0) return PS_ERR_ARG;
    int64_t stride = (num_envs + 63) & ~(int64_t)63;
    out->num_envs = num_envs;
    out->stride = stride;
    out->float_offset = 0;
    out->goal_offset = out->float_offset + (int64_t)PS_NUM_FLOAT_ROWS * stride * 4;
    out->rng_offset = out->goal_offset + 3 * stride * 8;
    out->elapsed_offset = out->rng_offset + 4 * stride * 8;
    out->total_bytes = out->elapsed_offset + stride * 4;
    return PS_OK;
}

int ps_create(const ps_config *cfg, int64_t num_envs, int device, ps_ctx **out) {
    if (!cfg || !out || num_envs <= 0) return PS_ERR_ARG;
    if (cfg->task < 0 || cfg->task > 2 || cfg->control < 0 || cfg->control > 1 || cfg->reward < 0 || cfg->reward > 1)
        return PS_ERR_ARG;
    if ((cfg->task == PS_TASK_REACH) == (cfg->has_cube != 0)) return PS_ERR_UNSUPPORTED;
    ps_ctx *c = new (std::nothrow) ps_ctx;
    if (!c) return PS_ERR_ARG;
    memset(c, 0, sizeof *c);
    c->cfg = *cfg;
    c->num_envs = num_envs;
    c->device = device;
    ps_state_layout(num_envs, &c->lay);
    *out = c;
    return PS_OK;
}

void ps_destroy(ps_ctx *ctx) { delete ctx; }

const char *ps_last_error(const ps_ctx *ctx) { return ctx ? ctx->err : "null context"; }

int ps_obs_dim(const ps_ctx *c) {
    int robot = c->cfg.block_gripper ? 6 : 7;
    return robot + (c->cfg.task == PS_TASK_REACH ? 0 : 12);
}

int ps_action_dim(const ps_ctx *c) {
    return (c->cfg.control == PS_CONTROL_EE ? 3 : 7) + (c->cfg.block_gripper ? 0 : 1);
}

int ps_init_state(ps_ctx *c, void *state, void *stream) {
    if (!c || !state) return fail(c, PS_ERR_ARG, "null argument");
    KParams P = params_of(c, state);
    hipLaunchKernelGGL(k_init_state, grid_of(P.n, kBlock), dim3(kBlock), 0, (hipStream_t)stream, P);
    return check_launch(c);
}

int ps_reset(ps_ctx *c, void *state, const uint8_t *mask, const uint64_t *seeds, float *obs, float *ag, float *dg,
             void *stream) {
    if (!c || !state) return fail(c, PS_ERR_ARG, "null argument");
    KParams P = params_of(c, state);
    dim3 g = grid_of(P.n, kBlock), b(kBlock);
    hipStream_t st = (hipStream_t)stream;
    switch (c->cfg.task) {
        case PS_TASK_REACH: hipLaunchKernelGGL(k_reset<PS_TASK_REACH>, g, b, 0, st, P, mask, seeds, obs, ag, dg); break;
        case PS_TASK_PUSH: hipLaunchKernelGGL(k_reset<PS_TASK_PUSH>, g, b, 0, st, P, mask, seeds, obs, ag, dg); break;
        default: hipLaunchKernelGGL(k_reset<PS_TASK_PICK_AND_PLACE>, g, b, 0, st, P, mask, seeds, obs, ag, dg); break;
    }
    return check_launch(c);
}

int ps_step(ps_ctx *c, void *state, const float *actions, float *obs, float *ag, float *dg, float *reward,
            uint8_t *terminated, uint8_t *truncated, int autoreset, float *final_obs, float *final_ag,
            void *stream) {
    if (!c || !state || !actions || !reward || !terminated || !truncated)
        return fail(c, PS_ERR_ARG, "null argument");
    KParams P = params_of(c, state);
    P.autoreset = autoreset;
    dim3 g = grid_of(P.n, kBlock), b(kBlock);
    hipStream_t st = (hipStream_t)stream;
#define PS_LAUNCH_STEP(T, C) \
    hipLaunchKernelGGL((k_step<T, C>), g, b, 0, st, P, actions, obs, ag, dg, reward, terminated, truncated, final_obs, final_ag)
    int ee = c->cfg.control == PS_CONTROL_EE;
    switch (c->cfg.task) {
        case PS_TASK_REACH:
            if (ee) PS_LAUNCH_STEP(PS_TASK_REACH, PS_CONTROL_EE); else PS_LAUNCH_STEP(PS_TASK_REACH, PS_CONTROL_JOINTS);
            break;
        case PS_TASK_PUSH:
            if (ee) PS_LAUNCH_STEP(PS_TASK_PUSH, PS_CONTROL_EE); else PS_LAUNCH_STEP(PS_TASK_PUSH, PS_CONTROL_JOINTS);
            break;
        default:
            if (ee) PS_LAUNCH_STEP(PS_TASK_PICK_AND_PLACE, PS_CONTROL_EE);
            else PS_LAUNCH_STEP(PS_TASK_PICK_AND_PLACE, PS_CONTROL_JOINTS);
            break;
    }
#undef PS_LAUNCH_STEP
    return check_launch(c);
}

int ps_sim_step(ps_ctx *c, void *state, int n_substeps, void *stream) {
    if (!c || !state || n_substeps < 0) return fail(c, PS_ERR_ARG, "bad argument");
    KParams P = params_of(c, state);
    dim3 g = grid_of(P.n, kBlock), b(kBlock);
    if (c->cfg.has_cube) hipLaunchKernelGGL(k_sim_step<true>, g, b, 0, (hipStream_t)stream, P, n_substeps);
    else hipLaunchKernelGGL(k_sim_step<false>, g, b, 0, (hipStream_t)stream, P, n_substeps);
    return check_launch(c);
}

int ps_link_state(ps_ctx *c, const void *state, int link, float *pos, float *quat, float *lin_vel, float *ang_vel,
                  void *stream) {
    if (!c || !state || link < 0 || link >= PM_NUM_LINKS) return fail(c, PS_ERR_ARG, "bad argument");
    KParams P = params_of(c, (void *)state);
    hipLaunchKernelGGL(k_link_state, grid_of(P.n, kBlock), dim3(kBlock), 0, (hipStream_t)stream, P, link, pos, quat,
                       lin_vel, ang_vel);
    return check_launch(c);
}

int ps_inverse_kinematics(ps_ctx *c, const void *state, int link, const float *pos, const float *orn, float *q_out,
                          void *stream) {
    if (!c || !state || !pos || !orn || !q_out || link < 0 || link >= PM_NUM_LINKS)
        return fail(c, PS_ERR_ARG, "bad argument");
    KParams P = params_of(c, (void *)state);
    dim3 g = grid_of(P.n, kBlock), b(kBlock);
    hipStream_t st = (hipStream_t)stream;
    switch (link) {
#define PS_IK_CASE(L) \
    case L: hipLaunchKernelGGL(k_ik<L>, g, b, 0, st, P, pos, orn, q_out); break;
        PS_IK_CASE(0) PS_IK_CASE(1) PS_IK_CASE(2) PS_IK_CASE(3) PS_IK_CASE(4) PS_IK_CASE(5)
        PS_IK_CASE(6) PS_IK_CASE(7) PS_IK_CASE(8) PS_IK_CASE(9) PS_IK_CASE(10) PS_IK_CASE(11)
#undef PS_IK_CASE
    }
    return check_launch(c);
}

int ps_rng_seed(ps_ctx *c, void *state, const uint8_t *mask, const uint64_t *seeds, void *stream) {
    if (!c || !state || !seeds) return fail(c, PS_ERR_ARG, "null argument");
    KParams P = params_of(c, state);
    hipLaunchKernelGGL(k_rng_seed, grid_of(P.n, kBlock), dim3(kBlock), 0, (hipStream_t)stream, P, mask, seeds);
    return check_launch(c);
}

int ps_rng_uniform(ps_ctx *c, void *state, const uint8_t *mask, int n, const double *low, const double *high,
                   double *out, void *stream) {
    if (!c || !state || !out || !low || !high || n < 1 || n > PS_MAX_UNIFORM)
        return fail(c, PS_ERR_ARG, "bad argument");
    KParams P = params_of(c, state);
    UniformArgs u;
    u.n = n;
    for (int k = 0; k < PS_MAX_UNIFORM; k++) {
        u.lo[k] = k < n ? low[k] : 0.0;
        u.hi[k] = k < n ? high[k] : 0.0;
    }
    hipLaunchKernelGGL(k_rng_uniform, grid_of(P.n, kBlock), dim3(kBlock), 0, (hipStream_t)stream, P, mask, u, out);
    return check_launch(c);
}

int ps_base_state(ps_ctx *c, const void *state, float *pos, float *quat, float *euler, float *lin_vel,
                  float *ang_vel, void *stream) {
    if (!c || !state) return fail(c, PS_ERR_ARG, "null argument");
    if (!c->cfg.has_cube) return fail(c, PS_ERR_UNSUPPORTED, "scene has no object");
    KParams P = params_of(c, (void *)state);
    hipLaunchKernelGGL(k_base_state, grid_of(P.n, kBlock), dim3(kBlock), 0, (hipStream_t)stream, P, pos, quat, euler,
                       lin_vel, ang_vel);
    return check_launch(c);
}

int ps_compute_reward(int reward_type, const void *ag, int ag_is_double, const void *dg, int dg_is_double,
                      float *reward, uint8_t *success, int64_t n, void *stream) {
    if (!ag || !dg || n < 0 || reward_type < 0 || reward_type > 1) return PS_ERR_ARG;
    if (n == 0) return PS_OK;
    hipLaunchKernelGGL(k_compute_reward, grid_of(n, 256), dim3(256), 0, (hipStream_t)stream, reward_type, ag,
                       ag_is_double, dg, dg_is_double, reward, success, n);
    return hipGetLastError() == hipSuccess ? PS_OK : PS_ERR_HIP;
}

}  // extern "C"
