// ps_common.h — fp32 vector algebra and the compile-time Panda model for the
// gfx950 kernels.  All model numbers come from include/panda_model.h; the URDF
// origin rotations (multiples of pi/2 about x, -pi/4 about z) are made exact so
// the compiler folds the 0/+-1 entries out of every frame product.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "panda_model.h"
#include "pandasim.h"

#define PS_D __device__ __forceinline__
#define PS_HD __host__ __device__ __forceinline__

// Phase timing (diagnostic build only, -DPS_PROFILE_PHASES; scripts/phase_profile.py):
// each wave accumulates s_memtime deltas per phase and lane 0 adds them to
// ps_phase_cycles at the end of the kernel.  Compiled out of the product.
#define PS_NUM_PHASES 8
#define PS_NUM_PROF_SLOTS 24  // phases + PGS counters (lane iterations, wave iterations, substeps, robot-contact slots run,
                              // the wave's open row gates: pair slots, ground slots, robot slots, joint limits;
                              // 16-18: sub-phases of rows+contacts -- 16 joint rows, 17 gripper contact
                              // candidates, 18 object ground/pair contacts -- the rest of it, the gripper
                              // rows, stays in 3; 20-23: gripper bounding tests -- (env, box) pairs
                              // passing them and boxes passing for some env of the wave, box-object
                              // then box-ground)
#define PS_ITP_WORDS 10
#ifdef PS_PROFILE_PHASES
// (32-bit: one kernel's wave-cycles per phase fit, and 64-bit accumulators
// cost the instrumented kernel another PS_NUM_PROF_SLOTS VGPRs at 512)
struct PhaseTimer {
    uint32_t last, acc[PS_NUM_PROF_SLOTS];
    // the lane's last 20 substeps, 16 bits each, newest in the low half of
    // itp[0]: PGS iterations (bits 0-7), gripper slots nr (8-10), box-box
    // slots np (11-13) (one-lane kernels; scripts/iter_dump.py)
    uint32_t itp[PS_ITP_WORDS];
};
#define PS_PROF_PARAM , PhaseTimer &pt
#define PS_PROF_ARG , pt
#define PS_PROF_COUNT_PARAM , int &prof_it
#define PS_PROF_COUNT_ARG , prof_it
#define PS_PHASE(k)                                        \
    do {                                                   \
        uint32_t ps_t_now = (uint32_t)__builtin_amdgcn_s_memtime(); \
        pt.acc[k] += ps_t_now - pt.last;                   \
        pt.last = ps_t_now;                                \
    } while (0)
#else
#define PS_PROF_PARAM
#define PS_PROF_ARG
#define PS_PROF_COUNT_PARAM
#define PS_PROF_COUNT_ARG
#define PS_PHASE(k) do {} while (0)
#endif

// Row dump (diagnostic build only, -DPS_DEBUG_ROW_DUMP; scripts/row_dump.py):
// the group solver's inputs and the impulse change of every row of the first
// PGS iteration pair of substeps 0 and 1, per lane, PS_DUMP_ROWS floats per
// lane and substep (the -O3 group-kernel investigation).
// Compiled out of the product.
#define PS_DUMP_ROWS 256
#define PS_DUMP_LANES 4096  // lanes dumped (the first 4 096 of the grid)
#ifdef PS_DEBUG_ROW_DUMP
#define PS_DUMP_PARAM , float *dump
#define PS_DUMP_ARG , dump
#else
#define PS_DUMP_PARAM
#define PS_DUMP_ARG
#endif

namespace ps {

// ------------------------------------------------------------------ vectors
struct V3 {
    float x, y, z;
};
PS_HD V3 mk(float x, float y, float z) { return V3{x, y, z}; }
PS_HD V3 operator+(V3 a, V3 b) { return V3{a.x + b.x, a.y + b.y, a.z + b.z}; }
PS_HD V3 operator-(V3 a, V3 b) { return V3{a.x - b.x, a.y - b.y, a.z - b.z}; }
PS_HD V3 operator-(V3 a) { return V3{-a.x, -a.y, -a.z}; }
PS_HD V3 operator*(V3 a, float s) { return V3{a.x * s, a.y * s, a.z * s}; }
PS_HD V3 operator*(float s, V3 a) { return V3{a.x * s, a.y * s, a.z * s}; }
PS_HD float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
PS_HD V3 cross(V3 a, V3 b) { return V3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
PS_D float norm(V3 a) { return sqrtf(dot(a, a)); }
// v_sqrt_f32 / v_rcp_f32 alone (1 ulp): sqrtf and '/' expand to correctly
// rounded sequences of ~13 and ~10 VALU instructions; the contact candidate
// streams (Slide's box-cylinder: ~80 of them per pair) use these
PS_D float fast_sqrt(float x) { return __builtin_amdgcn_sqrtf(x); }
PS_D float fast_rcp(float x) { return __builtin_amdgcn_rcpf(x); }
PS_D float fast_norm(V3 a) { return fast_sqrt(dot(a, a)); }
// c + a * s with one fma per component
PS_HD V3 fma3(V3 a, float s, V3 c) { return V3{fmaf(a.x, s, c.x), fmaf(a.y, s, c.y), fmaf(a.z, s, c.z)}; }

// row-major 3x3
struct M3 {
    float m[9];
};
PS_HD V3 col(const M3 &A, int c) { return V3{A.m[c], A.m[3 + c], A.m[6 + c]}; }
PS_HD V3 mul(const M3 &A, V3 v) {
    return V3{A.m[0] * v.x + A.m[1] * v.y + A.m[2] * v.z, A.m[3] * v.x + A.m[4] * v.y + A.m[5] * v.z,
              A.m[6] * v.x + A.m[7] * v.y + A.m[8] * v.z};
}
PS_HD V3 tmul(const M3 &A, V3 v) {
    return V3{A.m[0] * v.x + A.m[3] * v.y + A.m[6] * v.z, A.m[1] * v.x + A.m[4] * v.y + A.m[7] * v.z,
              A.m[2] * v.x + A.m[5] * v.y + A.m[8] * v.z};
}

// symmetric 3x3 stored xx, yy, zz, xy, xz, yz
struct S3 {
    float xx, yy, zz, xy, xz, yz;
};
PS_HD V3 mul(const S3 &I, V3 v) {
    return V3{I.xx * v.x + I.xy * v.y + I.xz * v.z, I.xy * v.x + I.yy * v.y + I.yz * v.z,
              I.xz * v.x + I.yz * v.y + I.zz * v.z};
}
PS_HD S3 operator+(const S3 &a, const S3 &b) {
    return S3{a.xx + b.xx, a.yy + b.yy, a.zz + b.zz, a.xy + b.xy, a.xz + b.xz, a.yz + b.yz};
}
// m * (|r|^2 E - r r^T)  (parallel-axis term)
PS_HD S3 shift(float m, V3 r) {
    return S3{m * (r.y * r.y + r.z * r.z), m * (r.x * r.x + r.z * r.z), m * (r.x * r.x + r.y * r.y),
              -m * r.x * r.y, -m * r.x * r.z, -m * r.y * r.z};
}
// R diag(I) R^T
PS_HD S3 rotate_diag(const M3 &R, float ix, float iy, float iz) {
    const float *m = R.m;
    return S3{m[0] * m[0] * ix + m[1] * m[1] * iy + m[2] * m[2] * iz,
              m[3] * m[3] * ix + m[4] * m[4] * iy + m[5] * m[5] * iz,
              m[6] * m[6] * ix + m[7] * m[7] * iy + m[8] * m[8] * iz,
              m[0] * m[3] * ix + m[1] * m[4] * iy + m[2] * m[5] * iz,
              m[0] * m[6] * ix + m[1] * m[7] * iy + m[2] * m[8] * iz,
              m[3] * m[6] * ix + m[4] * m[7] * iy + m[5] * m[8] * iz};
}

// quaternion (x, y, z, w)
struct Q4 {
    float x, y, z, w;
};
PS_HD Q4 qmul(Q4 a, Q4 b) {
    return Q4{a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y, a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z,
              a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x, a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z};
}
PS_HD M3 quat_to_mat(Q4 q) {
    float d = q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w, s = 2.0f / d;
    float xs = q.x * s, ys = q.y * s, zs = q.z * s;
    float wx = q.w * xs, wy = q.w * ys, wz = q.w * zs, xx = q.x * xs, xy = q.x * ys, xz = q.x * zs, yy = q.y * ys,
          yz = q.y * zs, zz = q.z * zs;
    return M3{{1.0f - (yy + zz), xy - wz, xz + wy, xy + wz, 1.0f - (xx + zz), yz - wx, xz - wy, yz + wx,
               1.0f - (xx + yy)}};
}
// btMatrix3x3::getRotation
PS_D Q4 mat_to_quat(const M3 &M) {
    const float *m = M.m;
    float tr = m[0] + m[4] + m[8];
    Q4 q;
    if (tr > 0.0f) {
        float s = sqrtf(tr + 1.0f);
        q.w = s * 0.5f;
        s = 0.5f / s;
        q.x = (m[7] - m[5]) * s;
        q.y = (m[2] - m[6]) * s;
        q.z = (m[3] - m[1]) * s;
    } else if (m[0] < m[4] ? (m[4] < m[8]) : (m[0] < m[8])) {  // i = 2
        float s = sqrtf(m[8] - m[0] - m[4] + 1.0f);
        q.z = s * 0.5f;
        s = 0.5f / s;
        q.w = (m[3] - m[1]) * s;
        q.x = (m[6] + m[2]) * s;
        q.y = (m[7] + m[5]) * s;
    } else if (m[0] < m[4]) {  // i = 1
        float s = sqrtf(m[4] - m[8] - m[0] + 1.0f);
        q.y = s * 0.5f;
        s = 0.5f / s;
        q.w = (m[2] - m[6]) * s;
        q.z = (m[5] + m[7]) * s;
        q.x = (m[3] + m[1]) * s;
    } else {  // i = 0
        float s = sqrtf(m[0] - m[4] - m[8] + 1.0f);
        q.x = s * 0.5f;
        s = 0.5f / s;
        q.w = (m[7] - m[5]) * s;
        q.y = (m[1] + m[3]) * s;
        q.z = (m[2] + m[6]) * s;
    }
    return q;
}

// symmetric 9x9 packed lower-triangular index
PS_HD constexpr int sidx(int i, int j) { return i >= j ? i * (i + 1) / 2 + j : j * (j + 1) / 2 + i; }

// ---------------------------------------------------------------- the model
struct LinkDef {
    int parent, type, dof;
    double o[3], rpy[3], axis[3];
    double mass, com[3], aabb[3];
};

#define PS_LINKDEF(idx, par, typ, ox, oy, oz, rr, pp, yy, ax, ay, az, dof_, m, cx, cy, cz, bx, by, bz) \
    LinkDef{par, typ, dof_, {ox, oy, oz}, {rr, pp, yy}, {ax, ay, az}, m, {cx, cy, cz}, {bx, by, bz}},

PS_HD constexpr LinkDef link_def(int i) {
    const LinkDef t[PM_NUM_LINKS] = {PM_LINK_TABLE(PS_LINKDEF)};
    return t[i];
}

struct M3d {
    double m[9];
};
// exact URDF origin rotations
PS_HD constexpr M3d origin_rot(int i) {
    LinkDef d = link_def(i);
    if (d.rpy[0] == PM_HALF_PI_URDF) return M3d{{1, 0, 0, 0, 0, -1, 0, 1, 0}};
    if (d.rpy[0] == -PM_HALF_PI_URDF) return M3d{{1, 0, 0, 0, 0, 1, 0, -1, 0}};
    if (d.rpy[2] == -PM_QUARTER_PI_URDF) {
        const double c = 0.70710678118654752440;
        return M3d{{c, c, 0, -c, c, 0, 0, 0, 1}};
    }
    return M3d{{1, 0, 0, 0, 1, 0, 0, 0, 1}};
}
PS_HD constexpr double link_inertia(int i, int axis) {
    LinkDef d = link_def(i);
    double lx = d.aabb[0], ly = d.aabb[1], lz = d.aabb[2];
    return axis == 0 ? d.mass / 12.0 * (ly * ly + lz * lz)
                     : (axis == 1 ? d.mass / 12.0 * (lx * lx + lz * lz) : d.mass / 12.0 * (lx * lx + ly * ly));
}

struct DofDef {
    int link;
    double lo, hi;
};
#define PS_DOFDEF(d, link, lo, hi) DofDef{link, lo, hi},
PS_HD constexpr DofDef dof_def(int d) {
    const DofDef t[PM_NUM_DOFS] = {PM_DOF_TABLE(PS_DOFDEF)};
    return t[d];
}

struct SphereDef {
    int link;
    double c[3], r, mu;
};
#define PS_SPHDEF(link, x, y, z, r, mu) SphereDef{link, {x, y, z}, r, mu},
PS_HD constexpr SphereDef sphere_def(int s) {
    const SphereDef t[PM_NUM_SPHERES] = {PM_SPHERE_TABLE(PS_SPHDEF)};
    return t[s];
}

// gripper collision boxes (PM_BOX_TABLE) and the wrist sphere (PM_WRIST_SPHERE)
struct BoxDef {
    int link;
    double c[3], h[3], mu;
};
#define PS_BOXDEF(link, cx, cy, cz, hx, hy, hz, mu) BoxDef{link, {cx, cy, cz}, {hx, hy, hz}, mu},
PS_HD constexpr BoxDef box_def(int b) {
    const BoxDef t[PM_NUM_BOXES] = {PM_BOX_TABLE(PS_BOXDEF)};
    return t[b];
}
PS_HD constexpr SphereDef wrist_def() {
    const SphereDef t[1] = {PM_WRIST_SPHERE(PS_SPHDEF)};
    return t[0];
}
PS_HD constexpr double joint_force(int d) {
    const double f[PM_NUM_DOFS] = PM_JOINT_FORCES;
    return f[d];
}
PS_HD constexpr double neutral_q(int d) {
    const double f[PM_NUM_DOFS] = PM_NEUTRAL_Q;
    return f[d];
}

// ------------------------------------------------------- lane groups
// Sum over a group of 16 lanes (one DPP row), the same bits in every lane of
// the group: each step adds a value and its partner's, and a + b == b + a
// (row_ror:8 pairs lanes i, i^8; row_half_mirror pairs j, 7-j within each
// half row; quad_perm [1,0,3,2] and [2,3,0,1] pair i, i^1 and i, i^2).
// (bound_ctrl: a lane whose source is out of its row reads 0 -- none is, for
// the controls used here -- so the destination needs no zeroing move first,
// as update_dpp's `old` operand did: one VALU op less per DPP read)
template <int CTRL>
PS_D float dpp_f(float x) {
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), CTRL, 0xF, 0xF, true));
}
// The step kernels' logical block (round 6).  A group kernel's wave covers
// 64 / G envs, so T = G / 2 consecutive waves share each 128-byte line of a
// state row; blocks are observed to go round-robin over the 8 XCDs (b and
// b + 8 share one, MI355X_MICROARCH.md), so those waves sat on different XCDs
// and each XCD's L2 fetched the line again: FETCH 934 B per env-step at 8 lanes
// and 1 424 B at 16 against 210 and 161 on one lane (profiles/r06m_*).  Two
// bijective remaps put a line's waves on one XCD: the whole range (the blocks
// of one XCD take consecutive envs) and tiles (runs of T consecutive waves on
// one XCD, the runs dealt over the XCDs in turn).  Timed on the same sources
// (profiles/r06o_ab.log, r06p_ab.log, three rotations each), the whole-range
// remap costs 0.9 % at 8 lanes and nothing at 16, the tiles nothing at 8 and
// 1.2 % at 16: the product takes tiles at 8 lanes and the whole range at 16.
// Speed only: an env's results do not depend on the wave it runs in (the
// group tests and scripts/compare_libs.py, bit for bit).
// PS_XCD_REMAP (scripts/build_variants.py): 0 none, 1 the product's choice,
// 2 the whole range at 8 and 16 lanes, 3 tiles at 8 and 16 lanes.
#ifndef PS_XCD_REMAP
#define PS_XCD_REMAP 1
#endif
// runs of T consecutive logical blocks on one XCD, the runs dealt over the
// XCDs in turn; the blocks past the last whole run of 8 T keep their order
template <uint32_t T>
PS_D uint32_t xcd_tiles(uint32_t b, uint32_t n) {
    const uint32_t whole = n / (8u * T) * (8u * T);
    if (b >= whole) return b;
    const uint32_t x = b % 8u, j = b / 8u;
    return ((j / T) * 8u + x) * T + j % T;
}
// the blocks of one XCD take consecutive logical blocks
PS_D uint32_t xcd_whole(uint32_t b, uint32_t n) {
    const uint32_t q = n / 8u, r = n % 8u, x = b % 8u;
    return (x < r ? x * (q + 1u) : r * (q + 1u) + (x - r) * q) + b / 8u;
}
template <int G>
PS_D uint32_t step_block() {
    const uint32_t b = blockIdx.x;
    constexpr bool TILES = (PS_XCD_REMAP == 1 && G == 8) || PS_XCD_REMAP == 3;
    if constexpr (G == 1 || PS_XCD_REMAP == 0) {
        return b;
    } else if constexpr (TILES) {
        return xcd_tiles<G / 2>(b, gridDim.x);
    } else {
        return xcd_whole(b, gridDim.x);
    }
}

// The additions are kept out of FMA contraction: with one DoF per lane the
// summand is a product, and contracting `J v + dpp(J v)` into fma(J, v, dpp)
// rounds this lane's term differently from the partner's copy of it, so the
// lanes of a group would end with different bits (and could leave the PGS loop
// on different iterations).  PS_EXPERIMENT_GROUP_SUM_CONTRACT (a diagnostic
// build of scripts/build_variants.py, never the product) leaves contraction on,
// to show what it does to the group kernels.
PS_D float group16_sum(float x) {
#ifndef PS_EXPERIMENT_GROUP_SUM_CONTRACT
#pragma clang fp contract(off)
#endif
    x += dpp_f<0x128>(x);  // row_ror:8
    x += dpp_f<0x141>(x);  // row_half_mirror
    x += dpp_f<0xB1>(x);   // quad_perm [1,0,3,2]
    x += dpp_f<0x4E>(x);   // quad_perm [2,3,0,1]
    return x;
}

// lane K of this lane's 16-lane row, in every lane of the row (DPP
// row_newbcast, gfx90a+)
template <int K>
PS_D float group16_bcast(float x) {
    static_assert(K >= 0 && K < 16, "lane of the row");
    return dpp_f<0x150 + K>(x);
}

// the same over groups of 8 lanes: half_mirror pairs lane i with 7 - i, then
// the quad swaps (every lane of the group ends with the same bits)
PS_D float group8_sum(float x) {
#ifndef PS_EXPERIMENT_GROUP_SUM_CONTRACT
#pragma clang fp contract(off)
#endif
    x += dpp_f<0x141>(x);  // row_half_mirror
    x += dpp_f<0xB1>(x);   // quad_perm [1,0,3,2]
    x += dpp_f<0x4E>(x);   // quad_perm [2,3,0,1]
    return x;
}

// lane K of this lane's 8-lane group, in every lane of the group: row_newbcast
// of lane K and of lane 8 + K of the 16-lane row (two independent DPP reads),
// the group's half selected by lane bit 3
template <int K>
PS_D float group8_bcast(float x) {
    static_assert(K >= 0 && K < 8, "lane of the group");
    const float lo = dpp_f<0x150 + K>(x), hi = dpp_f<0x158 + K>(x);
    return (__lane_id() & 8u) ? hi : lo;
}

// groups of 2 lanes (PS_EXPERIMENT_G2, DESIGN.md §12.13: two lanes per env):
// the pair's other lane by quad_perm [1,0,3,2], the same bits in both lanes
PS_D float group2_sum(float x) {
#pragma clang fp contract(off)
    return x + dpp_f<0xB1>(x);
}
// lane K of this lane's pair: quad_perm [K, K, K + 2, K + 2]
template <int K>
PS_D float group2_bcast(float x) {
    static_assert(K == 0 || K == 1, "lane of the pair");
    return dpp_f<K == 0 ? 0xA0 : 0xF5>(x);
}

// compile-time loop
template <int B, int E, typename F>
PS_D void static_for(F &&f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        static_for<B + 1, E>(f);
    }
}

}  // namespace ps
