// pandasim.hip — gfx950 kernels and the C ABI (include/pandasim.h) of the
// batched Panda simulator.  One env per lane; every kernel reads/writes the
// structure-of-arrays state with coalesced row accesses.
#include <new>

#include "ps_env.h"
#include "ps_render.h"

#ifdef PS_PROFILE_PHASES
// phase counters of the diagnostic build: one device buffer that every
// step object's kernels add to (KParams::prof)
static unsigned long long *g_prof = nullptr;
unsigned long long *ps_prof_buffer() {
    if (!g_prof && hipMalloc((void **)&g_prof, sizeof(unsigned long long) * PS_NUM_PROF_SLOTS) == hipSuccess)
        (void)hipMemset(g_prof, 0, sizeof(unsigned long long) * PS_NUM_PROF_SLOTS);
    return g_prof;
}
// per-env PGS iterations and contact slots of each one-lane kernel launch's 20
// substeps: PS_ITP_WORDS words x PS_ITER_DUMP_ENVS, 16 bits per substep
// (PhaseTimer::itp)
static uint32_t *g_itdump = nullptr;
uint32_t *ps_iter_dump_buffer() {
    if (!g_itdump && hipMalloc((void **)&g_itdump, sizeof(uint32_t) * PS_ITP_WORDS * PS_ITER_DUMP_ENVS) == hipSuccess)
        (void)hipMemset(g_itdump, 0, sizeof(uint32_t) * PS_ITP_WORDS * PS_ITER_DUMP_ENVS);
    return g_itdump;
}
extern "C" int ps_debug_env_iters(uint32_t *out) {
    uint32_t *b = ps_iter_dump_buffer();
    if (!b || hipDeviceSynchronize() != hipSuccess) return PS_ERR_HIP;
    if (hipMemcpy(out, b, sizeof(uint32_t) * PS_ITP_WORDS * PS_ITER_DUMP_ENVS, hipMemcpyDeviceToHost) != hipSuccess)
        return PS_ERR_HIP;
    return PS_OK;
}
extern "C" int ps_debug_phase_cycles(unsigned long long *out, int reset) {
    unsigned long long *b = ps_prof_buffer();
    if (!b || hipDeviceSynchronize() != hipSuccess) return PS_ERR_HIP;
    if (hipMemcpy(out, b, sizeof(unsigned long long) * PS_NUM_PROF_SLOTS, hipMemcpyDeviceToHost) != hipSuccess)
        return PS_ERR_HIP;
    if (reset && hipMemset(b, 0, sizeof(unsigned long long) * PS_NUM_PROF_SLOTS) != hipSuccess) return PS_ERR_HIP;
    return PS_OK;
}
#endif

#ifdef PS_DEBUG_ROW_DUMP
// row dump of the diagnostic build (KParams::dbg): PS_DUMP_LANES lanes x 2
// substeps x PS_DUMP_ROWS floats, NaN where nothing was recorded
static float *g_dump = nullptr;
static const size_t kDumpFloats = (size_t)PS_DUMP_LANES * 2 * PS_DUMP_ROWS;
float *ps_row_dump_buffer() {
    if (!g_dump && hipMalloc((void **)&g_dump, sizeof(float) * kDumpFloats) == hipSuccess)
        (void)hipMemset(g_dump, 0xFF, sizeof(float) * kDumpFloats);
    return g_dump;
}
extern "C" int ps_debug_row_dump(float *out, int reset) {
    float *b = ps_row_dump_buffer();
    if (!b || hipDeviceSynchronize() != hipSuccess) return PS_ERR_HIP;
    if (hipMemcpy(out, b, sizeof(float) * kDumpFloats, hipMemcpyDeviceToHost) != hipSuccess) return PS_ERR_HIP;
    if (reset && hipMemset(b, 0xFF, sizeof(float) * kDumpFloats) != hipSuccess) return PS_ERR_HIP;
    return PS_OK;
}
#endif

namespace {

// ---------------------------------------------------------------- kernels
__global__ __launch_bounds__(kBlock) void k_init_state(KParams P) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P.n) return;
    const StateView &s = P.s;
    for (int r = 0; r < PS_NUM_FLOAT_ROWS; r++) s.F(r, i) = 0.0f;
    s.F(PS_F_CQUAT + 3, i) = 1.0f;
    s.F(PS_F_C2QUAT + 3, i) = 1.0f;
    for (int d = 0; d < 9; d++) {
        s.F(PS_F_MKD + d, i) = 1.0f;
        s.F(PS_F_MIMP + d, i) = (float)PM_DEFAULT_MOTOR_MAX_IMPULSE;
    }
    for (int d = 0; d < PS_MAX_GOAL_DIM; d++) s.G(d, i) = 0.0;
    store_rng(s, i, pcg_seed(0));
    aux_rng(s, i) = aux_seed(0);
    s.E(i) = 0;
}

template <int TASK>
__global__ __launch_bounds__(kBlock) void k_reset(KParams P, const uint8_t *mask, const uint64_t *seeds, float *obs,
                                                  float *ag, float *dg) {
    using T = TaskTraits<TASK>;
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P.n) return;
    if (mask && !mask[i]) return;
    const StateView &s = P.s;
    Pcg r = seeds ? pcg_seed(seeds[i]) : load_rng(s, i);
    uint64_t aux = seeds ? aux_seed(seeds[i]) : aux_rng(s, i);
    float q[9], qd[9];
    Body bd[T::NOBJ > 0 ? T::NOBJ : 1];
#pragma unroll
    for (int b = 0; b < T::NOBJ; b++) load_body(s, i, b, bd[b]);
    double g[6] = {0, 0, 0, 0, 0, 0};
    reset_env<TASK>(q, qd, bd, g, r, aux);
    store_robot(s, i, q, qd);
#pragma unroll
    for (int b = 0; b < T::NOBJ; b++) store_body(s, i, b, bd[b]);
    for (int d = 0; d < T::GOAL; d++) s.G(d, i) = g[d];
    store_rng(s, i, r);
    aux_rng(s, i) = aux;
    s.E(i) = 0;
    clear_contact_cache(s, i);
    // RecordEpisodeStatistics (ps_set_episode_stats) zeroes the running
    // return on reset(): an abandoned episode's partial return does not carry
    // into the next one
    if (P.epstats) P.epstats[i] = 0.0f;
    write_obs<TASK>(P, i, q, qd, bd, g, obs, ag, dg);
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
    V3 c = mk(0, 0, 0);
    static_for<0, PM_NUM_LINKS>([&](auto L) {
        constexpr int l = decltype(L)::value;
        if (l == link) {
            R = k.f[l].R;
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
// generator becomes Generator(PCG64(SeedSequence(seeds[i]))), and Flip's goal
// stream restarts from the same seed
__global__ __launch_bounds__(kBlock) void k_rng_seed(KParams P, const uint8_t *mask, const uint64_t *seeds) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P.n || (mask && !mask[i])) return;
    store_rng(P.s, i, pcg_seed(seeds[i]));
    aux_rng(P.s, i) = aux_seed(seeds[i]);
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

// Flip's goal (Rotation.random(), flip.py:70-72) from each env's goal stream
__global__ __launch_bounds__(kBlock) void k_rng_rotation(KParams P, const uint8_t *mask, double *out) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P.n || (mask && !mask[i])) return;
    uint64_t st = aux_rng(P.s, i);
    double q[4];
    random_rotation(st, q);
    aux_rng(P.s, i) = st;
    for (int k = 0; k < 4; k++) out[i * 4 + k] = q[k];
}

// getBasePositionAndOrientation + getEulerFromQuaternion + getBaseVelocity of
// object `b` (pybullet.py:284-349)
__global__ __launch_bounds__(kBlock) void k_base_state(KParams P, int b, float *pos, float *quat, float *euler,
                                                       float *vel, float *avel) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P.n) return;
    Body c;
    load_body(P.s, i, b, c);
    if (pos) { pos[i * 3] = c.pos.x; pos[i * 3 + 1] = c.pos.y; pos[i * 3 + 2] = c.pos.z; }
    if (quat) { quat[i * 4] = c.quat.x; quat[i * 4 + 1] = c.quat.y; quat[i * 4 + 2] = c.quat.z; quat[i * 4 + 3] = c.quat.w; }
    if (euler) { V3 e = euler_from_quat(c.quat); euler[i * 3] = e.x; euler[i * 3 + 1] = e.y; euler[i * 3 + 2] = e.z; }
    if (vel) { vel[i * 3] = c.vel.x; vel[i * 3 + 1] = c.vel.y; vel[i * 3 + 2] = c.vel.z; }
    if (avel) { avel[i * 3] = c.omg.x; avel[i * 3 + 1] = c.omg.y; avel[i * 3 + 2] = c.omg.z; }
}

// compute_reward / is_success for HER (core.py:226): goal pairs of `gd`
// values; f64 arithmetic when either side is f64 (numpy promotion), f32
// otherwise (threshold rounded to f32)
__global__ __launch_bounds__(256) void k_compute_reward(int task, int reward_type, const void *ag, int ag_dbl,
                                                        const void *dg, int dg_dbl, float *reward, uint8_t *success,
                                                        int64_t n) {
#pragma clang fp contract(off)
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int gd = task == PS_TASK_STACK ? 6 : (task == PS_TASK_FLIP ? 4 : 3);
    const bool angle = task == PS_TASK_FLIP;
    const double thr = task == PS_TASK_STACK ? PM_STACK_DISTANCE_THRESHOLD
                       : angle                ? PM_FLIP_DISTANCE_THRESHOLD
                                              : PM_DISTANCE_THRESHOLD;
    if (ag_dbl || dg_dbl) {
        double m = 0.0;
        for (int k = 0; k < gd; k++) {
            double a = ag_dbl ? ((const double *)ag)[i * gd + k] : (double)((const float *)ag)[i * gd + k];
            double g = dg_dbl ? ((const double *)dg)[i * gd + k] : (double)((const float *)dg)[i * gd + k];
            double e = __dsub_rn(a, g);
            double t = angle ? opaque(__dmul_rn(a, g)) : opaque(__dmul_rn(e, e));
            m = k == 0 ? t : __dadd_rn(m, t);
        }
        double d = angle ? __dsub_rn(1.0, opaque(__dmul_rn(m, m))) : __dsqrt_rn(m);
        if (reward) reward[i] = reward_for(reward_type, d, thr);
        if (success) success[i] = d < thr;
    } else {
        const float *a = (const float *)ag, *g = (const float *)dg;
        float m = 0.0f;
        for (int k = 0; k < gd; k++) {
            float av = a[i * gd + k], gv = g[i * gd + k];
            float e = __fsub_rn(av, gv);
            float t = angle ? opaque(__fmul_rn(av, gv)) : opaque(__fmul_rn(e, e));
            m = k == 0 ? t : __fadd_rn(m, t);
        }
        // correctly rounded f32 root: the f64 root rounded once
        float d = angle ? __fsub_rn(1.0f, opaque(__fmul_rn(m, m))) : __double2float_rn(__dsqrt_rn((double)m));
        float tf = (float)thr;
        if (reward) reward[i] = reward_type == 0 ? (d > tf ? -1.0f : -0.0f) : -d;
        if (success) success[i] = d < tf;
    }
}


// ------------------------------------------------------------- rendering
// Camera of a view/projection pair (column-major float[16], as getCameraImage
// takes them): eye, the view axes (s, u, -f rows of the rotation) and the
// projection terms a pixel ray and the depth buffer need.
struct Cam {
    V3 eye, s, u, f;
    float p00, p11, p22, p23, nearv, farv;
    float light[3];
};

Cam cam_of(const float view[16], const float proj[16]) {
    Cam c;
    // V = [R | t] (row r, col k = view[k*4 + r]); eye = -R^T t
    c.s = mk(view[0], view[4], view[8]);
    c.u = mk(view[1], view[5], view[9]);
    c.f = mk(-view[2], -view[6], -view[10]);
    V3 t = mk(view[12], view[13], view[14]);
    c.eye = mk(-(c.s.x * t.x + c.u.x * t.y - c.f.x * t.z), -(c.s.y * t.x + c.u.y * t.y - c.f.y * t.z),
               -(c.s.z * t.x + c.u.z * t.y - c.f.z * t.z));
    c.p00 = proj[0];
    c.p11 = proj[5];
    c.p22 = proj[10];
    c.p23 = proj[14];
    // clip planes of the perspective matrix: z_ndc = -1 / +1
    c.nearv = proj[14] / (proj[10] - 1.0f);
    c.farv = proj[14] / (proj[10] + 1.0f);
    // a fixed key light from above and behind the camera
    V3 l = c.u * 0.6f - c.f * 0.3f + mk(0.0f, 0.0f, 0.7f);
    float ln = 1.0f / sqrtf(dot(l, l));
    c.light[0] = l.x * ln;
    c.light[1] = l.y * ln;
    c.light[2] = l.z * ln;
    return c;
}

// Per-env primitives: the arm's capsules (joint frame to joint frame), the
// gripper spheres, object and target poses.  One lane per env.
__global__ __launch_bounds__(kBlock) void k_render_prep(KParams P, int n_objects, const float *targets, float *prims) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P.n) return;
    const StateView &s = P.s;
    float q[9], qd[9];
    load_robot(s, i, q, qd);
    Kin k;
    fk(q, k);
    float *o = prims + i * RENDER_PRIM_FLOATS;
    const V3 b = P.sc.base;
    auto put3 = [&](int at, V3 v) { o[at] = v.x; o[at + 1] = v.y; o[at + 2] = v.z; };
    // link0 column, upper arm, elbow offsets, forearm, wrist, flange, hand bar
    const V3 hand_a = k.f[8].o + mul(k.f[8].R, mk(0.0f, -0.09f, 0.03f));
    const V3 hand_b = k.f[8].o + mul(k.f[8].R, mk(0.0f, 0.09f, 0.03f));
    const V3 wrist = k.f[8].o + mul(k.f[8].R, mk(0.0f, 0.0f, 0.04f));  // flange -> palm (hand origin = flange)
    const V3 A[RENDER_CAPSULES] = {mk(0, 0, 0), k.f[1].o, k.f[2].o, k.f[3].o, k.f[5].o, k.f[6].o, k.f[7].o, hand_a};
    const V3 Bp[RENDER_CAPSULES] = {k.f[0].o, k.f[2].o, k.f[3].o, k.f[4].o, k.f[6].o, k.f[7].o, wrist, hand_b};
    const float R[RENDER_CAPSULES] = {0.07f, 0.065f, 0.06f, 0.06f, 0.055f, 0.05f, 0.045f, 0.03f};
#pragma unroll
    for (int c = 0; c < RENDER_CAPSULES; c++) {
        put3(RP_CAPS + c * 7, A[c] + b);
        put3(RP_CAPS + c * 7 + 3, Bp[c] + b);
        o[RP_CAPS + c * 7 + 6] = R[c];
    }
    static_for<0, PM_NUM_SPHERES>([&](auto SS) {
        constexpr int S = decltype(SS)::value;
        constexpr SphereDef d = sphere_def(S);
        V3 c = k.f[d.link].o + mul(k.f[d.link].R, mk((float)d.c[0], (float)d.c[1], (float)d.c[2])) + b;
        put3(RP_SPH + S * 4, c);
        o[RP_SPH + S * 4 + 3] = (float)d.r;
    });
    {
        // bounding sphere of the arm's primitives: k_render skips them for rays that miss it
        V3 lo = mk(3e38f, 3e38f, 3e38f), hi = mk(-3e38f, -3e38f, -3e38f);
        auto grow = [&](V3 p) {
            lo = mk(fminf(lo.x, p.x), fminf(lo.y, p.y), fminf(lo.z, p.z));
            hi = mk(fmaxf(hi.x, p.x), fmaxf(hi.y, p.y), fmaxf(hi.z, p.z));
        };
        float rmax = 0.0f;
        for (int c = 0; c < RENDER_CAPSULES; c++) {
            grow(mk(o[RP_CAPS + c * 7], o[RP_CAPS + c * 7 + 1], o[RP_CAPS + c * 7 + 2]));
            grow(mk(o[RP_CAPS + c * 7 + 3], o[RP_CAPS + c * 7 + 4], o[RP_CAPS + c * 7 + 5]));
            rmax = fmaxf(rmax, o[RP_CAPS + c * 7 + 6]);
        }
        for (int c = 0; c < PM_NUM_SPHERES; c++) {
            grow(mk(o[RP_SPH + c * 4], o[RP_SPH + c * 4 + 1], o[RP_SPH + c * 4 + 2]));
            rmax = fmaxf(rmax, o[RP_SPH + c * 4 + 3]);
        }
        V3 ctr = (lo + hi) * 0.5f, half = (hi - lo) * 0.5f;
        put3(RP_ARM_BOUND, ctr);
        o[RP_ARM_BOUND + 3] = sqrtf(dot(half, half)) * 1.0001f + rmax + 1e-4f;
    }
    for (int ob = 0; ob < 2; ob++) {
        Body bd;
        if (ob < n_objects) load_body(s, i, ob, bd);
        else bd = Body{mk(0, 0, -100.0f), Q4{0, 0, 0, 1}, mk(0, 0, 0), mk(0, 0, 0)};
        M3 Rm = quat_to_mat(bd.quat);
        put3(RP_OBJ + ob * 12, bd.pos);
        for (int e = 0; e < 9; e++) o[RP_OBJ + ob * 12 + 3 + e] = Rm.m[e];
        V3 tp = mk(0, 0, -100.0f);
        Q4 tq = Q4{0, 0, 0, 1};
        if (targets) {
            const float *t = targets + (i * 2 + ob) * 7;
            tp = mk(t[0], t[1], t[2]);
            tq = Q4{t[3], t[4], t[5], t[6]};
        }
        M3 Rt = quat_to_mat(tq);
        put3(RP_TGT + ob * 12, tp);
        for (int e = 0; e < 9; e++) o[RP_TGT + ob * 12 + 3 + e] = Rt.m[e];
    }
}

struct RenderArgs {
    Cam cam;
    int width, height, n_objects, object_shape;
    V3 object_half, table_c, table_h;
    int has_table, has_plane;
    ps_visual vis;
};

PS_D M3 m3_at(const float *p) {
    M3 R;
#pragma unroll
    for (int e = 0; e < 9; e++) R.m[e] = p[e];
    return R;
}

// getCameraImage (pybullet.py:186-192) by ray casting: one lane per pixel,
// blockIdx.x = env.  Pixel (row r, col c) is sampled at its centre, as a
// rasteriser does; depth is OpenGL window depth of the projection matrix.
constexpr int kRenderBlock = 256;
constexpr int kRenderPix = 1;  // pixels per lane (strided by the block)

// (256, 4): four waves per SIMD at <= 128 VGPRs -- a lone wave per SIMD leaves the
// ray tests' dependent chains exposed
__global__ __launch_bounds__(kRenderBlock, 4) void k_render(RenderArgs a, const float *prims, float *depth,
                                                            uint8_t *rgb) {
    __shared__ float pr[RENDER_PRIM_FLOATS];
    __shared__ float rgba[8 * 4];  // colours by role, indexed per pixel (a kernarg array would go to scratch)
    __shared__ unsigned arm_mask;
    const int64_t env = blockIdx.x;  // x: envs (up to 2^31), y: pixel tiles (<= 65 535)
    for (int k = threadIdx.x; k < RENDER_PRIM_FLOATS; k += kRenderBlock) pr[k] = prims[env * RENDER_PRIM_FLOATS + k];
    if (threadIdx.x < 32) rgba[threadIdx.x] = a.vis.rgba[threadIdx.x >> 2][threadIdx.x & 3];
    if (threadIdx.x == 0) arm_mask = 0u;
    __syncthreads();
    const Cam &cm = a.cam;
    const int64_t npix = (int64_t)a.width * a.height;
    // Row culling of the arm primitives: this block's pixels span image rows
    // [r0, r1]; primitive k (capsules, then spheres) joins the mask when its
    // bounding sphere's conservative projected row range meets them.
    if (threadIdx.x < RENDER_CAPSULES + PM_NUM_SPHERES) {
        const int k = threadIdx.x;
        V3 c;
        float rad;
        if (k < RENDER_CAPSULES) {
            const float *q = pr + RP_CAPS + k * 7;
            V3 pa = mk(q[0], q[1], q[2]), pb = mk(q[3], q[4], q[5]);
            c = (pa + pb) * 0.5f;
            rad = 0.5f * norm(pb - pa) + q[6];
        } else {
            const float *q = pr + RP_SPH + (k - RENDER_CAPSULES) * 4;
            c = mk(q[0], q[1], q[2]);
            rad = q[3];
        }
        rad = rad * 1.001f + 1e-4f;
        int64_t p0 = (int64_t)blockIdx.y * kRenderPix * kRenderBlock;
        int64_t p1 = p0 + kRenderPix * kRenderBlock - 1;
        if (p1 >= npix) p1 = npix - 1;
        const float r0 = (float)(p0 / a.width), r1 = (float)(p1 / a.width);
        V3 v = c - cm.eye;
        float ze = dot(v, cm.f), yu = dot(v, cm.u);
        bool hit = true;
        if (ze - rad > cm.nearv) {
            float dmin = ze - rad, dmax = ze + rad;
            float nhi = yu + rad, nlo = yu - rad;
            float yhi = cm.p11 * (nhi >= 0.0f ? nhi / dmin : nhi / dmax);
            float ylo = cm.p11 * (nlo <= 0.0f ? nlo / dmin : nlo / dmax);
            // pixel-centre rows: y = 1 - (2 r + 1) / H
            float rlo = ((1.0f - yhi) * a.height - 1.0f) * 0.5f - 1.0f;
            float rhi = ((1.0f - ylo) * a.height - 1.0f) * 0.5f + 1.0f;
            hit = rlo <= r1 && rhi >= r0;
        }
        if (hit) atomicOr(&arm_mask, 1u << k);
    }
    __syncthreads();
    const unsigned mask = arm_mask;
    const M3 I3 = M3{{1, 0, 0, 0, 1, 0, 0, 0, 1}};
#pragma unroll 1
    for (int pp = 0; pp < kRenderPix; pp++) {
        int64_t pix = ((int64_t)blockIdx.y * kRenderPix + pp) * kRenderBlock + threadIdx.x;
        if (pix >= npix) break;
        int r = (int)(pix / a.width), c = (int)(pix - (int64_t)r * a.width);
        float xn = -1.0f + (2.0f * c + 1.0f) / a.width, yn = 1.0f - (2.0f * r + 1.0f) / a.height;
        // eye-space direction (xn / P00, yn / P11, -1): unit length along f, so t = -z_eye
        V3 d = cm.s * (xn / cm.p00) + cm.u * (yn / cm.p11) + cm.f;
        V3 o = cm.eye;
        Hit h{cm.farv, mk(0, 0, 1)};
        int role = VR_BACKGROUND;
        const float tmin = cm.nearv;
        if (a.has_plane && ray_box(o, d, mk(0, 0, (float)PM_PLANE_TOP - 0.01f), I3, mk(3.0f, 3.0f, 0.01f), tmin, h))
            role = VR_PLANE;
        if (a.has_table && ray_box(o, d, a.table_c, I3, a.table_h, tmin, h)) role = VR_TABLE;
        for (int ob = 0; ob < a.n_objects; ob++) {
            const float *q = pr + RP_OBJ + ob * 12;
            V3 c0 = mk(q[0], q[1], q[2]);
            M3 R = m3_at(q + 3);
            bool hit = a.object_shape == PS_SHAPE_CYLINDER
                           ? ray_cylinder(o, d, c0, R, a.object_half.x, a.object_half.z, tmin, h)
                           : ray_box(o, d, c0, R, a.object_half, tmin, h);
            if (hit) role = VR_OBJECT1 + ob;
        }
        if (mask && ray_meets_sphere(o, d, mk(pr[RP_ARM_BOUND], pr[RP_ARM_BOUND + 1], pr[RP_ARM_BOUND + 2]),
                                     pr[RP_ARM_BOUND + 3], h.t)) {
            for (int k = 0; k < RENDER_CAPSULES; k++) {
                if (!(mask & (1u << k))) continue;
                const float *q = pr + RP_CAPS + k * 7;
                if (ray_capsule(o, d, mk(q[0], q[1], q[2]), mk(q[3], q[4], q[5]), q[6], tmin, h)) role = VR_ROBOT;
            }
            for (int k = 0; k < PM_NUM_SPHERES; k++) {
                if (!(mask & (1u << (RENDER_CAPSULES + k)))) continue;
                const float *q = pr + RP_SPH + k * 4;
                if (ray_sphere(o, d, mk(q[0], q[1], q[2]), q[3], tmin, h)) role = VR_ROBOT;
            }
        }
        float dep = 1.0f;
        const float *col = rgba + role * 4;
        float cr = col[0], cg = col[1], cb = col[2];
        if (role != VR_BACKGROUND) {
            float ze = -h.t;
            dep = 0.5f * ((cm.p22 * ze + cm.p23) / h.t) + 0.5f;
            float nl = fabsf(h.n.x * cm.light[0] + h.n.y * cm.light[1] + h.n.z * cm.light[2]);
            float sh = 0.35f + 0.65f * nl;
            cr *= sh;
            cg *= sh;
            cb *= sh;
        }
        // ghost targets: alpha-blended over whatever is behind, no depth write
        for (int g = 0; g < 2; g++) {
            int shape = a.vis.target_shape[g];
            if (shape < 0) continue;
            const float *q = pr + RP_TGT + g * 12;
            V3 c0 = mk(q[0], q[1], q[2]);
            M3 R = m3_at(q + 3);
            V3 hh = mk(a.vis.target_half[g][0], a.vis.target_half[g][1], a.vis.target_half[g][2]);
            Hit gh{h.t, mk(0, 0, 1)};
            bool hit = shape == PS_SHAPE_CYLINDER ? ray_cylinder(o, d, c0, R, hh.x, hh.z, tmin, gh)
                       : shape == PS_VISUAL_SPHERE ? ray_sphere(o, d, c0, hh.x, tmin, gh)
                                                   : ray_box(o, d, c0, R, hh, tmin, gh);
            if (hit) {
                const float *tc = rgba + (VR_TARGET1 + g) * 4;
                float al = tc[3];
                cr = al * tc[0] + (1.0f - al) * cr;
                cg = al * tc[1] + (1.0f - al) * cg;
                cb = al * tc[2] + (1.0f - al) * cb;
            }
        }
        int64_t at = env * npix + pix;
        if (depth) depth[at] = dep;
        if (rgb) {
            rgb[at * 3 + 0] = (uint8_t)fminf(fmaxf(cr * 255.0f + 0.5f, 0.0f), 255.0f);
            rgb[at * 3 + 1] = (uint8_t)fminf(fmaxf(cg * 255.0f + 0.5f, 0.0f), 255.0f);
            rgb[at * 3 + 2] = (uint8_t)fminf(fmaxf(cb * 255.0f + 0.5f, 0.0f), 255.0f);
        }
    }
}

struct Tran {
    double m[16];  // row-major inv(P V)
};

// tran @ (x, y, z, 1) with the accumulation OpenBLAS's dgemm kernel uses for a
// 4-deep product (one fused multiply-add per term, k ascending), then the
// homogeneous divide (pybullet.py:140-143, 225-229)
PS_D void pix_to_world(const Tran &T, double x, double y, double z, double out[3]) {
    double w = fma(T.m[15], 1.0, fma(T.m[14], z, fma(T.m[13], y, T.m[12] * x)));
#pragma unroll
    for (int r = 0; r < 3; r++) {
        double v = fma(T.m[r * 4 + 3], 1.0, fma(T.m[r * 4 + 2], z, fma(T.m[r * 4 + 1], y, T.m[r * 4 + 0] * x)));
        out[r] = v / w;
    }
}

// render()'s post-processing of getCameraImage's depth (pybullet.py:203-262),
// per env and pixel: NDC of np.mgrid (left/top pixel edges, the reference's
// convention), valid = depth < 0.99 and the workspace box on the world point,
// the world point and pixels_2d.
constexpr int kDeprojBlock = 256;

__global__ __launch_bounds__(kDeprojBlock) void k_deproject_image(int64_t n_env, int width, int height, Tran T,
                                                                  const float *depth, double *points,
                                                                  uint8_t *valid, double *pix2d) {
#pragma clang fp contract(off)
    // the block's points / pixels_2d are staged in LDS and leave as
    // lane-contiguous 8-byte stores (a wave writes 512 contiguous bytes per
    // instruction) instead of 24- and 16-byte strided ones
    __shared__ double sp[kDeprojBlock * 3];
    __shared__ double sx[kDeprojBlock * 2];
    const int64_t npix = (int64_t)width * height, total = n_env * npix;
    const int64_t g0 = (int64_t)blockIdx.x * kDeprojBlock, g = g0 + threadIdx.x;
    if (g < total) {
        int64_t pix = g % npix;
        int r = (int)(pix / width), c = (int)(pix - (int64_t)r * width);
        // np.mgrid[-1:1:2/h, -1:1:2/w]: index * step + start; then y *= -1
        double x = opaque(__dmul_rn((double)c, 2.0 / width)) + -1.0;
        double y = -(opaque(__dmul_rn((double)r, 2.0 / height)) + -1.0);
        double z = (double)depth[g];
        double zn = opaque(__dmul_rn(2.0, z)) - 1.0;
        double p[3];
        pix_to_world(T, x, y, zn, p);
        bool ok = z < 0.99 && p[2] > 0.0 && p[2] < 0.67 && p[0] > -0.5 && p[0] < 0.2;
        if (valid) valid[g] = ok;
        sp[threadIdx.x * 3 + 0] = p[0];
        sp[threadIdx.x * 3 + 1] = p[1];
        sp[threadIdx.x * 3 + 2] = p[2];
        // (xy + 1) / 2, x *= w, y *= h, y = h - y
        double px = opaque(x + 1.0) / 2.0, py = opaque(y + 1.0) / 2.0;
        sx[threadIdx.x * 2 + 0] = px * (double)width;
        sx[threadIdx.x * 2 + 1] = (double)height - opaque(py * (double)height);
    }
    __syncthreads();
    const int64_t n_here = total - g0 < kDeprojBlock ? total - g0 : kDeprojBlock;
    if (points)
        for (int k = threadIdx.x; k < n_here * 3; k += kDeprojBlock) points[g0 * 3 + k] = sp[k];
    if (pix2d)
        for (int k = threadIdx.x; k < n_here * 2; k += kDeprojBlock) pix2d[g0 * 2 + k] = sx[k];
}

// PyBullet.deproject(depth, pixels, tran_pix_world) (pybullet.py:109-146) for
// n pixels (col, row) per env
__global__ __launch_bounds__(256) void k_deproject_pixels(int64_t n_env, int n, int width, int height, Tran T,
                                                          const float *depth, const int32_t *pixels, double *points) {
#pragma clang fp contract(off)
    int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n_env * n) return;
    int64_t env = g / n;
    int pc = pixels[g * 2 + 0], prow = pixels[g * 2 + 1];
    if (pc < 0 || pc >= width || prow < 0 || prow >= height) {
        // outside the image (numpy would raise; the host wrapper does): no read, NaN point
        points[g * 3 + 0] = points[g * 3 + 1] = points[g * 3 + 2] = __builtin_nan("");
        return;
    }
    // x = px * 1 / w (integer numerator, true division), x *= 2, x -= 1; the same for
    // (h - py); z = 2 depth[py, px] - 1
    double x = opaque(opaque((double)pc / (double)width) * 2.0) - 1.0;
    double y = opaque(opaque((double)(height - prow) / (double)height) * 2.0) - 1.0;
    double z = opaque(2.0 * (double)depth[env * (int64_t)width * height + (int64_t)prow * width + pc]) - 1.0;
    double p[3];
    pix_to_world(T, x, y, z, p);
    points[g * 3 + 0] = p[0];
    points[g * 3 + 1] = p[1];
    points[g * 3 + 2] = p[2];
}

}  // namespace

// ------------------------------------------------------------------- C ABI
extern "C" {

int ps_abi_version(void) { return PS_ABI_VERSION; }

int ps_default_config(int task, int control, int reward, ps_config *out) {
    if (!out || task < 0 || task >= PS_NUM_TASKS || control < 0 || control > 1 || reward < 0 || reward > 1)
        return PS_ERR_ARG;
    memset(out, 0, sizeof *out);
    out->task = task;
    out->control = control;
    out->reward = reward;
    // Reach/Push/Slide block the gripper (panda_tasks.py:62,78,94)
    out->block_gripper = task == PS_TASK_REACH || task == PS_TASK_PUSH || task == PS_TASK_SLIDE;
    out->has_table = 1;
    out->has_plane = 1;
    out->n_objects = task_nobj(task);
    out->object_shape = task == PS_TASK_SLIDE ? PS_SHAPE_CYLINDER : PS_SHAPE_BOX;
    out->base[0] = (float)PM_BASE_X;
    if (task == PS_TASK_SLIDE) {
        out->object_half[0] = out->object_half[1] = (float)(PM_SLIDE_OBJECT_SIZE / 2);
        out->object_half[2] = (float)(PM_SLIDE_OBJECT_SIZE / 2 / 2);
        out->object_friction = (float)PM_SLIDE_FRICTION;
        out->table_cx = (float)PM_SLIDE_TABLE_CX;
        out->table_hx = (float)PM_SLIDE_TABLE_HX;
    } else {
        out->object_half[0] = out->object_half[1] = out->object_half[2] = (float)(PM_OBJECT_SIZE / 2);
        out->object_friction = (float)PM_DEFAULT_FRICTION;
        out->table_cx = (float)PM_TABLE_CX;
        out->table_hx = (float)PM_TABLE_HX;
    }
    out->table_hy = (float)PM_TABLE_HY;
    out->object_mass = (float)(task == PS_TASK_STACK ? PM_STACK_MASS1 : PM_CUBE_MASS);
    out->object2_mass = (float)PM_STACK_MASS2;
    return PS_OK;
}

int ps_state_layout(int64_t num_envs, ps_layout *out) {
    if (!out || num_envs <= 0 || num_envs > PS_MAX_ENVS) return PS_ERR_ARG;
    int64_t stride = (num_envs + 63) & ~(int64_t)63;
    out->num_envs = num_envs;
    out->stride = stride;
    out->float_offset = 0;
    out->goal_offset = out->float_offset + (int64_t)PS_NUM_FLOAT_ROWS * stride * 4;
    out->rng_offset = out->goal_offset + (int64_t)PS_MAX_GOAL_DIM * stride * 8;
    out->elapsed_offset = out->rng_offset + (int64_t)PS_NUM_RNG_ROWS * stride * 8;
    out->total_bytes = out->elapsed_offset + stride * 4;
    return PS_OK;
}

int ps_create(const ps_config *cfg, int64_t num_envs, int device, ps_ctx **out) {
    if (!cfg || !out || num_envs <= 0 || num_envs > PS_MAX_ENVS) return PS_ERR_ARG;
    if (cfg->task < 0 || cfg->task >= PS_NUM_TASKS || cfg->control < 0 || cfg->control > 1 || cfg->reward < 0 ||
        cfg->reward > 1 || cfg->n_objects < 0 || cfg->n_objects > 2 || cfg->object_shape < 0 || cfg->object_shape > 1)
        return PS_ERR_ARG;
    if (cfg->n_objects > 0) {
        // compiled-in shapes: cubes (isotropic), one upright z cylinder
        if (cfg->object_shape == PS_SHAPE_BOX &&
            (cfg->object_half[0] != cfg->object_half[1] || cfg->object_half[1] != cfg->object_half[2]))
            return PS_ERR_UNSUPPORTED;
        if (cfg->object_shape == PS_SHAPE_CYLINDER &&
            (cfg->n_objects != 1 || cfg->object_half[0] != cfg->object_half[1]))
            return PS_ERR_UNSUPPORTED;
        if (!(cfg->object_mass > 0.0f) || (cfg->n_objects == 2 && !(cfg->object2_mass > 0.0f))) return PS_ERR_ARG;
    }
    ps_ctx *c = new (std::nothrow) ps_ctx;
    if (!c) return PS_ERR_ARG;
    memset(c, 0, sizeof *c);
    c->cfg = *cfg;
    c->num_envs = num_envs;
    c->device = device;
    c->gains_dirty = 1;
    ps_state_layout(num_envs, &c->lay);
    *out = c;
    return PS_OK;
}

void ps_destroy(ps_ctx *ctx) {
    if (ctx && ctx->render_prims) (void)hipFree(ctx->render_prims);
    if (ctx && ctx->gstash) (void)hipFree(ctx->gstash);
    delete ctx;
}

const char *ps_last_error(const ps_ctx *ctx) { return ctx ? ctx->err : "null context"; }

int ps_obs_dim(const ps_ctx *c) { return (c->cfg.block_gripper ? 6 : 7) + task_obs_dim(c->cfg.task); }

int ps_action_dim(const ps_ctx *c) {
    return (c->cfg.control == PS_CONTROL_EE ? 3 : 7) + (c->cfg.block_gripper ? 0 : 1);
}

int ps_goal_dim(const ps_ctx *c) { return task_goal_dim(c->cfg.task); }

int ps_max_episode_steps(const ps_ctx *c) {
    return c->cfg.task == PS_TASK_STACK ? PM_STACK_MAX_EPISODE_STEPS : PM_MAX_EPISODE_STEPS;
}

int ps_init_state(ps_ctx *c, void *state, void *stream) {
    if (!c || !state) return fail(c, PS_ERR_ARG, "null argument");
    KParams P = params_of(c, state);
    hipLaunchKernelGGL(k_init_state, grid_of(P.n, kBlock), dim3(kBlock), 0, (hipStream_t)stream, P);
    c->gains_dirty = 1;
    return check_launch(c);
}

int ps_mark_motor_rows_dirty(ps_ctx *c) {
    if (!c) return PS_ERR_ARG;
    c->gains_dirty = 1;
    return PS_OK;
}

int ps_reset(ps_ctx *c, void *state, const uint8_t *mask, const uint64_t *seeds, float *obs, float *ag, float *dg,
             void *stream) {
    if (!c || !state) return fail(c, PS_ERR_ARG, "null argument");
    if (!scene_matches_task(c->cfg)) return fail(c, PS_ERR_UNSUPPORTED, "scene does not match the task");
    KParams P = params_of(c, state);
    dim3 g = grid_of(P.n, kBlock), b(kBlock);
    hipStream_t st = (hipStream_t)stream;
    // the next step rewrites the gain rows: a reset is where a caller starts
    // with a fresh or swapped-in buffer, whose address a caching allocator may
    // have handed out before (so the pointer test of the step launcher alone
    // would not see it)
    c->gains_dirty = 1;
#define PS_LAUNCH_RESET(T) hipLaunchKernelGGL(k_reset<T>, g, b, 0, st, P, mask, seeds, obs, ag, dg)
    switch (c->cfg.task) {
        case PS_TASK_REACH: PS_LAUNCH_RESET(PS_TASK_REACH); break;
        case PS_TASK_PUSH: PS_LAUNCH_RESET(PS_TASK_PUSH); break;
        case PS_TASK_PICK_AND_PLACE: PS_LAUNCH_RESET(PS_TASK_PICK_AND_PLACE); break;
        case PS_TASK_SLIDE: PS_LAUNCH_RESET(PS_TASK_SLIDE); break;
        case PS_TASK_STACK: PS_LAUNCH_RESET(PS_TASK_STACK); break;
        default: PS_LAUNCH_RESET(PS_TASK_FLIP); break;
    }
#undef PS_LAUNCH_RESET
    return check_launch(c);
}

int ps_step(ps_ctx *c, void *state, const float *actions, float *obs, float *ag, float *dg, float *reward,
            uint8_t *terminated, uint8_t *truncated, int autoreset, float *final_obs, float *final_ag,
            void *stream) {
    if (!c || !state || !actions || !reward || !terminated || !truncated)
        return fail(c, PS_ERR_ARG, "null argument");
    if (!scene_matches_task(c->cfg)) return fail(c, PS_ERR_UNSUPPORTED, "scene does not match the task");
    hipStream_t st = (hipStream_t)stream;
    if (ensure_stash(c, st) != PS_OK) return fail(c, PS_ERR_HIP, "hipMalloc of the Stack stash failed");
    const ps_step_io io{actions, obs, ag, dg, reward, terminated, truncated, final_obs, final_ag, autoreset};
    const int lanes = ps_step_lanes(c);
    const bool ee = c->cfg.control == PS_CONTROL_EE;
    int rc;
#define PS_STEP_TASK_CASE(T)                                                                              \
    case T:                                                                                               \
        rc = ee ? PS_STEP_LAUNCHER_NAME(T, 0)(c, state, io, lanes, st) : PS_STEP_LAUNCHER_NAME(T, 1)(c, state, io, lanes, st); \
        break;
    switch (c->cfg.task) {
        PS_STEP_TASK_CASE(0) PS_STEP_TASK_CASE(1) PS_STEP_TASK_CASE(2)
        PS_STEP_TASK_CASE(3) PS_STEP_TASK_CASE(4) PS_STEP_TASK_CASE(5)
        default: return fail(c, PS_ERR_ARG, "bad task");
    }
#undef PS_STEP_TASK_CASE
    if (rc == PS_OK) {
        c->gains_dirty = 0;
        c->gains_state = state;
    }
    return rc;
}

int ps_set_lanes_per_env(ps_ctx *c, int lanes) {
#ifdef PS_EXPERIMENT_G2
    // the two-lanes-per-env kernels of the experiment build
    if (c && lanes == 2 && c->cfg.n_objects <= 1) {
        c->lanes_per_env = lanes;
        return PS_OK;
    }
#endif
    if (!c || !(lanes == 0 || lanes == 1 || lanes == 8 || lanes == 16)) return PS_ERR_ARG;
    if (lanes > 1 && c->cfg.n_objects > 1) return fail(c, PS_ERR_UNSUPPORTED, "8 or 16 lanes per env: one object at most");
    c->lanes_per_env = lanes;
    return PS_OK;
}

int ps_step_lanes(const ps_ctx *c) {
    if (!c) return PS_ERR_ARG;
    if (c->lanes_per_env) return c->lanes_per_env;
    if (c->cfg.n_objects > 1) return 1;
    if (c->num_envs <= PS_GROUP16_AUTO_MAX_ENVS) return 16;
    return c->num_envs <= PS_GROUP8_AUTO_MAX_ENVS ? 8 : 1;
}

int ps_set_episode_stats(ps_ctx *c, float *stats) {
    if (!c) return PS_ERR_ARG;
    c->epstats = stats;
    return PS_OK;
}

int ps_set_nonfinite_guard(ps_ctx *c, uint8_t *flags, int reset_nonfinite) {
    if (!c) return PS_ERR_ARG;
    c->nonfinite = flags;
    c->reset_nonfinite = reset_nonfinite ? 1 : 0;
    return PS_OK;
}

int ps_sim_step(ps_ctx *c, void *state, int n_substeps, void *stream) {
    if (!c || !state || n_substeps < 0) return fail(c, PS_ERR_ARG, "bad argument");
    hipStream_t st = (hipStream_t)stream;
    if (ensure_stash(c, st) != PS_OK) return fail(c, PS_ERR_HIP, "hipMalloc of the Stack stash failed");
    if (c->cfg.n_objects == 0) return PS_SIM_LAUNCHER_NAME(0, 0)(c, state, n_substeps, st);
    if (c->cfg.n_objects == 2) return PS_SIM_LAUNCHER_NAME(2, 0)(c, state, n_substeps, st);
    if (c->cfg.object_shape == PS_SHAPE_CYLINDER) return PS_SIM_LAUNCHER_NAME(1, 1)(c, state, n_substeps, st);
    return PS_SIM_LAUNCHER_NAME(1, 0)(c, state, n_substeps, st);
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

int ps_rng_rotation(ps_ctx *c, void *state, const uint8_t *mask, double *out, void *stream) {
    if (!c || !state || !out) return fail(c, PS_ERR_ARG, "null argument");
    KParams P = params_of(c, state);
    hipLaunchKernelGGL(k_rng_rotation, grid_of(P.n, kBlock), dim3(kBlock), 0, (hipStream_t)stream, P, mask, out);
    return check_launch(c);
}

int ps_base_state(ps_ctx *c, const void *state, int object, float *pos, float *quat, float *euler, float *lin_vel,
                  float *ang_vel, void *stream) {
    if (!c || !state) return fail(c, PS_ERR_ARG, "null argument");
    if (object < 0 || object >= c->cfg.n_objects) return fail(c, PS_ERR_UNSUPPORTED, "scene has no such object");
    KParams P = params_of(c, (void *)state);
    hipLaunchKernelGGL(k_base_state, grid_of(P.n, kBlock), dim3(kBlock), 0, (hipStream_t)stream, P, object, pos,
                       quat, euler, lin_vel, ang_vel);
    return check_launch(c);
}

int ps_compute_reward(int task, int reward_type, const void *ag, int ag_is_double, const void *dg, int dg_is_double,
                      float *reward, uint8_t *success, int64_t n, void *stream) {
    if (!ag || !dg || n < 0 || task < 0 || task >= PS_NUM_TASKS || reward_type < 0 || reward_type > 1)
        return PS_ERR_ARG;
    if (n == 0) return PS_OK;
    hipLaunchKernelGGL(k_compute_reward, grid_of(n, 256), dim3(256), 0, (hipStream_t)stream, task, reward_type, ag,
                       ag_is_double, dg, dg_is_double, reward, success, n);
    return hipGetLastError() == hipSuccess ? PS_OK : PS_ERR_HIP;
}


int ps_camera(const float target[3], float distance, float yaw, float pitch, float roll, int width, int height,
              float view[16], float proj[16], double tran_pix_world[16]) {
    if (!target || !view || !proj || width <= 0 || height <= 0) return PS_ERR_ARG;
    ps_camera_math::view_from_yaw_pitch_roll(target, distance, yaw, pitch, roll, view);
    ps_camera_math::projection_fov(60.0, (double)width / height, 0.1, 100.0, proj);
    if (tran_pix_world) {
        // np.linalg.inv(P @ V) of the reshape(order='F') matrices, in double
        double P[16], V[16], PV[16];
        for (int r = 0; r < 4; r++)
            for (int c = 0; c < 4; c++) {
                P[r * 4 + c] = proj[c * 4 + r];
                V[r * 4 + c] = view[c * 4 + r];
            }
        for (int r = 0; r < 4; r++)
            for (int c = 0; c < 4; c++) {
                double acc = 0.0;
                for (int k = 0; k < 4; k++) acc += P[r * 4 + k] * V[k * 4 + c];
                PV[r * 4 + c] = acc;
            }
        if (!ps_camera_math::invert4(PV, tran_pix_world)) return PS_ERR_ARG;
    }
    return PS_OK;
}

int ps_render(ps_ctx *c, const void *state, const float view[16], const float proj[16], int width, int height,
              const ps_visual *vis, const float *targets, float *depth, uint8_t *rgb, void *stream) {
    if (!c || !state || !view || !proj || !vis || width <= 0 || height <= 0) return fail(c, PS_ERR_ARG, "null argument");
    if (!c->render_prims) {
        if (hipMalloc((void **)&c->render_prims, sizeof(float) * RENDER_PRIM_FLOATS * c->num_envs) != hipSuccess) {
            c->render_prims = nullptr;
            return fail(c, PS_ERR_HIP, "hipMalloc of the render scratch failed");
        }
    }
    KParams P = params_of(c, (void *)state);
    hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL(k_render_prep, grid_of(P.n, kBlock), dim3(kBlock), 0, st, P, c->cfg.n_objects, targets,
                       c->render_prims);
    RenderArgs a;
    a.cam = cam_of(view, proj);
    a.width = width;
    a.height = height;
    a.n_objects = c->cfg.n_objects;
    a.object_shape = c->cfg.object_shape;
    a.object_half = mk(c->cfg.object_half[0], c->cfg.object_half[1], c->cfg.object_half[2]);
    // create_table: box of half extents (length, width, height) / 2 at (x_offset, 0, -height / 2)
    a.table_c = mk(c->cfg.table_cx, 0.0f, (float)PM_TABLE_TOP - 0.2f);
    a.table_h = mk(c->cfg.table_hx, c->cfg.table_hy, 0.2f);
    a.has_table = c->cfg.has_table;
    a.has_plane = c->cfg.has_plane;
    a.vis = *vis;
    int64_t npix = (int64_t)width * height;
    int64_t tiles = (npix + kRenderBlock * kRenderPix - 1) / (kRenderBlock * kRenderPix);
    if (tiles > 65535) return fail(c, PS_ERR_ARG, "image too large (more than 65 535 pixel tiles)");
    dim3 g((unsigned)c->num_envs, (unsigned)tiles);
    hipLaunchKernelGGL(k_render, g, dim3(kRenderBlock), 0, st, a, c->render_prims, depth, rgb);
    return check_launch(c);
}

int ps_deproject_image(ps_ctx *c, const float *depth, const double tran_pix_world[16], int width, int height,
                       double *points, uint8_t *valid, double *pixels_2d, void *stream) {
    if (!c || !depth || !tran_pix_world || width <= 0 || height <= 0) return fail(c, PS_ERR_ARG, "null argument");
    Tran T;
    memcpy(T.m, tran_pix_world, sizeof T.m);
    int64_t n = c->num_envs * (int64_t)width * height;
    hipLaunchKernelGGL(k_deproject_image, grid_of(n, kDeprojBlock), dim3(kDeprojBlock), 0, (hipStream_t)stream,
                       c->num_envs, width, height, T, depth, points, valid, pixels_2d);
    return check_launch(c);
}

int ps_deproject_pixels(ps_ctx *c, const float *depth, const int32_t *pixels, int n, const double tran_pix_world[16],
                        int width, int height, double *points, void *stream) {
    if (!c || !depth || !pixels || !points || !tran_pix_world || n < 0 || width <= 0 || height <= 0)
        return fail(c, PS_ERR_ARG, "null argument");
    if (n == 0) return PS_OK;
    Tran T;
    memcpy(T.m, tran_pix_world, sizeof T.m);
    int64_t tot = c->num_envs * (int64_t)n;
    hipLaunchKernelGGL(k_deproject_pixels, grid_of(tot, 256), dim3(256), 0, (hipStream_t)stream, c->num_envs, n,
                       width, height, T, depth, pixels, points);
    return check_launch(c);
}

}  // extern "C"
