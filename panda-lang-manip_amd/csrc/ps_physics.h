// ps_physics.h — per-env (one env per lane) fp32 Panda multibody step for
// gfx950.  Same algorithm as the PyBullet 3.2.5 subset used by
// panda_gym/pybullet.py (restated in DESIGN.md §5), derived for a
// register-resident lane:
//   * forward kinematics with exact URDF origin rotations (12 links)
//   * mass matrix by composite rigid bodies in the base frame, bias forces by
//     a recursive Newton-Euler pass with prefix sums (gravity, gyroscopic,
//     btMultiBody damping)
//   * 9x9 Cholesky -> M^-1; joint-space rows (motors, limits) use columns of
//     M^-1 directly; cube-ground rows act only on the cube's 6 DoF;
//     gripper-contact rows carry explicit 9-wide Jacobians
//   * projected Gauss-Seidel in btMultiBodyConstraintSolver order
//   * semi-implicit Euler, exponential-map quaternion update.
#pragma once

#include "ps_common.h"

namespace ps {

struct Frame {
    M3 R;
    V3 o;
};

struct Kin {
    Frame f[PM_NUM_LINKS];
};

// frame of link I given its parent frame and its joint coordinate
template <int I>
PS_D Frame child_frame(const Frame &P, float q) {
    constexpr LinkDef d = link_def(I);
    Frame F;
    M3 Rj;
    // P.R times the constant joint-origin rotation and offset with the zero
    // terms dropped at compile time (IEEE x * 0 is not folded, and the
    // origins are axis permutations or identities: 18 of the 27 products
    // were zeros, in every one of the ~60 frames an env-step builds)
    static_for<0, 3>([&](auto RR) {
        constexpr int r = decltype(RR)::value;
        static_for<0, 3>([&](auto CC) {
            constexpr int c = decltype(CC)::value;
            float acc = 0.0f;
            bool any = false;
            static_for<0, 3>([&](auto KK) {
                constexpr int k = decltype(KK)::value;
                constexpr double w = origin_rot(I).m[k * 3 + c];
                if constexpr (w != 0.0) {
                    const float t = w == 1.0 ? P.R.m[r * 3 + k] : (w == -1.0 ? -P.R.m[r * 3 + k] : P.R.m[r * 3 + k] * (float)w);
                    acc = any ? acc + t : t;
                    any = true;
                }
            });
            Rj.m[r * 3 + c] = acc;
        });
    });
    V3 off = mk(0.0f, 0.0f, 0.0f);
    bool anyo = false;
    static_for<0, 3>([&](auto KK) {
        constexpr int k = decltype(KK)::value;
        if constexpr (d.o[k] != 0.0) {
            const V3 t = col(P.R, k) * (float)d.o[k];
            off = anyo ? off + t : t;
            anyo = true;
        }
    });
    V3 oj = P.o + off;
    if constexpr (d.type == PM_JOINT_REVOLUTE) {
        // libm sincosf (its range-reduction branch doubles as a scheduling
        // fence; __sinf/__cosf measured 12% slower on Push through spills)
        float s, c;
        sincosf(q, &s, &c);
#pragma unroll
        for (int r = 0; r < 3; r++) {
            float a = Rj.m[r * 3 + 0], b = Rj.m[r * 3 + 1];
            F.R.m[r * 3 + 0] = a * c + b * s;
            F.R.m[r * 3 + 1] = b * c - a * s;
            F.R.m[r * 3 + 2] = Rj.m[r * 3 + 2];
        }
        F.o = oj;
    } else if constexpr (d.type == PM_JOINT_PRISMATIC) {
        F.R = Rj;
        V3 ax = mul(Rj, mk((float)d.axis[0], (float)d.axis[1], (float)d.axis[2]));
        F.o = oj + ax * q;
    } else {
        F.R = Rj;
        F.o = oj;
    }
    return F;
}

// R times link I's constant COM offset, zero terms dropped at compile time
template <int I>
PS_D V3 com_offset(const M3 &R) {
    constexpr LinkDef d = link_def(I);
    V3 off = mk(0.0f, 0.0f, 0.0f);
    bool any = false;
    static_for<0, 3>([&](auto KK) {
        constexpr int k = decltype(KK)::value;
        if constexpr (d.com[k] != 0.0) {
            const V3 t = col(R, k) * (float)d.com[k];
            off = any ? off + t : t;
            any = true;
        }
    });
    return off;
}

// all link frames, base-relative (robot base at the origin, identity rotation)
PS_D void fk(const float q[9], Kin &k) {
    Frame base;
    base.R = M3{{1, 0, 0, 0, 1, 0, 0, 0, 1}};
    base.o = mk(0, 0, 0);
    k.f[0] = child_frame<0>(base, q[0]);
    k.f[1] = child_frame<1>(k.f[0], q[1]);
    k.f[2] = child_frame<2>(k.f[1], q[2]);
    k.f[3] = child_frame<3>(k.f[2], q[3]);
    k.f[4] = child_frame<4>(k.f[3], q[4]);
    k.f[5] = child_frame<5>(k.f[4], q[5]);
    k.f[6] = child_frame<6>(k.f[5], q[6]);
    k.f[7] = child_frame<7>(k.f[6], 0.0f);
    k.f[8] = child_frame<8>(k.f[7], 0.0f);
    k.f[9] = child_frame<9>(k.f[8], q[7]);
    k.f[10] = child_frame<10>(k.f[8], q[8]);
    k.f[11] = child_frame<11>(k.f[8], 0.0f);
}

// world axis of DoF d (revolute: frame z; prismatic: frame * axis)
template <int D>
PS_D V3 dof_axis(const Kin &k) {
    constexpr int L = dof_def(D).link;
    constexpr LinkDef d = link_def(L);
    if constexpr (d.type == PM_JOINT_REVOLUTE) return col(k.f[L].R, 2);
    else return mul(k.f[L].R, mk((float)d.axis[0], (float)d.axis[1], (float)d.axis[2]));
}

template <int I>
PS_D V3 com_pos(const Kin &k) {
    constexpr LinkDef d = link_def(I);
    return k.f[I].o + com_offset<I>(k.f[I].R);
}

// ------------------------------------------------------------------ dynamics
struct Comp {
    float m;
    V3 h;  // COM
    S3 I;  // about COM, base frame
};

template <int I>
PS_D Comp link_comp(const Kin &k) {
    constexpr LinkDef d = link_def(I);
    Comp c;
    c.m = (float)d.mass;
    c.h = com_pos<I>(k);
    c.I = rotate_diag(k.f[I].R, (float)link_inertia(I, 0), (float)link_inertia(I, 1), (float)link_inertia(I, 2));
    return c;
}

PS_D Comp combine(const Comp &a, const Comp &b) {
    Comp c;
    c.m = a.m + b.m;
    float inv = 1.0f / c.m;
    c.h = (a.h * a.m + b.h * b.m) * inv;
    // the two parallel-axis terms about the joint COM are one with the
    // reduced mass m_a m_b / (m_a + m_b) and d = h_a - h_b (masses are
    // compile-time constants, so is the factor)
    c.I = a.I + b.I + shift(a.m * b.m * inv, a.h - b.h);
    return c;
}

// Joint-space mass matrix (packed symmetric, 45 floats) by composite rigid
// bodies: for revolute b with composite C_b, the unit-rate momentum is
// P = m_b a_b x (h_b - o_b), L = I_b a_b; M_ab = a_a . (L + (h_b - o_a) x P).
PS_D void mass_matrix(const Kin &k, float M[45]) {
    V3 ax[9], org[9];
    static_for<0, 9>([&](auto D) {
        constexpr int d = decltype(D)::value;
        ax[d] = dof_axis<d>(k);
        org[d] = k.f[dof_def(d).link].o;
    });
    Comp f9 = link_comp<9>(k), f10 = link_comp<10>(k);
    // fingers (prismatic DoFs 7, 8)
    {
        V3 P9 = ax[7] * f9.m, P10 = ax[8] * f10.m;
        M[sidx(7, 7)] = f9.m;
        M[sidx(8, 8)] = f10.m;
        M[sidx(8, 7)] = 0.0f;
#pragma unroll
        for (int a = 0; a < 7; a++) {
            M[sidx(7, a)] = dot(ax[a], cross(f9.h - org[a], P9));
            M[sidx(8, a)] = dot(ax[a], cross(f10.h - org[a], P10));
        }
    }
    Comp c = combine(combine(link_comp<8>(k), f9), f10);
    static_for<0, 7>([&](auto BB) {
        constexpr int b = 6 - decltype(BB)::value;
        c = combine(link_comp<b>(k), c);
        V3 P = cross(ax[b], c.h - org[b]) * c.m;
        V3 L = mul(c.I, ax[b]);
#pragma unroll
        for (int a = 0; a <= b; a++) M[sidx(b, a)] = dot(ax[a], L + cross(c.h - org[a], P));
    });
}

// Bias forces h = C(q,qd) qd + g(q) + damping (RNEA with qdd = 0).  Forward
// pass over the chain; every link force/moment is folded into prefix sums so
// tau_i = a_i . ((N_tot - N_pre_i) - o_i x (F_tot - F_pre_i)) with moments
// about the base origin.
// Frames are produced on the fly (FK fused into the forward sweep) so no
// 12-frame kinematics array is held live next to the dynamics.
template <int I>
PS_D void link_wrench_f(const Frame &f, V3 w, V3 dw, V3 vo, V3 ao, V3 &F, V3 &N) {
    constexpr LinkDef d = link_def(I);
    constexpr float m = (float)d.mass;
    V3 c = f.o + com_offset<I>(f.R);
    V3 rc = c - f.o;
    V3 vc = vo + cross(w, rc);
    V3 ac = ao + cross(dw, rc) + cross(w, cross(w, rc));
    S3 Iw = rotate_diag(f.R, (float)link_inertia(I, 0), (float)link_inertia(I, 1), (float)link_inertia(I, 2));
    V3 Iww = mul(Iw, w);
    // (1-ulp square roots: the damping terms are ~1e-4 of the forces)
    float cl = (float)PM_LINEAR_DAMPING + (float)PM_LINEAR_DAMPING * fast_norm(vc);
    float ca = (float)PM_ANGULAR_DAMPING + (float)PM_ANGULAR_DAMPING * fast_norm(w);
    F = (ac + vc * cl) * m;
    V3 Nc = mul(Iw, dw) + cross(w, Iww) + Iww * ca;
    N = Nc + cross(c, F);  // about the base origin
}

PS_D void bias_forces(const float q[9], const float qd[9], float h[9]) {
    V3 w = mk(0, 0, 0), dw = mk(0, 0, 0), vo = mk(0, 0, 0), ao = mk(0, 0, -(float)PM_GRAVITY_Z);
    Frame f;
    f.R = M3{{1, 0, 0, 0, 1, 0, 0, 0, 1}};
    f.o = mk(0, 0, 0);
    V3 prev_o = f.o;
    V3 Fpre[7], Npre[7], ax[7], org[7];
    V3 Fs = mk(0, 0, 0), Ns = mk(0, 0, 0);
    static_for<0, 7>([&](auto II) {
        constexpr int I = decltype(II)::value;
        f = child_frame<I>(f, q[I]);
        V3 r = f.o - prev_o;
        vo = vo + cross(w, r);
        ao = ao + cross(dw, r) + cross(w, cross(w, r));
        V3 a = col(f.R, 2);
        ax[I] = a;
        org[I] = f.o;
        dw = dw + cross(w, a) * qd[I];
        w = w + a * qd[I];
        Fpre[I] = Fs;
        Npre[I] = Ns;
        V3 F, N;
        link_wrench_f<I>(f, w, dw, vo, ao, F, N);
        Fs = Fs + F;
        Ns = Ns + N;
        prev_o = f.o;
    });
    // link 7 (massless, fixed) and the hand (8): same origin as link 7
    f = child_frame<7>(f, 0.0f);
    f = child_frame<8>(f, 0.0f);
    {
        V3 r = f.o - prev_o;
        vo = vo + cross(w, r);
        ao = ao + cross(dw, r) + cross(w, cross(w, r));
        V3 F, N;
        link_wrench_f<8>(f, w, dw, vo, ao, F, N);
        Fs = Fs + F;
        Ns = Ns + N;
    }
    // fingers: prismatic children of the hand
    static_for<0, 2>([&](auto JJ) {
        constexpr int J = decltype(JJ)::value;
        constexpr int L = 9 + J;
        Frame ff = child_frame<L>(f, q[7 + J]);
        constexpr LinkDef ld = link_def(L);
        V3 a = mul(ff.R, mk((float)ld.axis[0], (float)ld.axis[1], (float)ld.axis[2]));
        float v = qd[7 + J];
        V3 r = ff.o - f.o;
        V3 vf = vo + cross(w, r) + a * v;
        V3 af = ao + cross(dw, r) + cross(w, cross(w, r)) + cross(w, a) * (2.0f * v);
        V3 F, N;
        link_wrench_f<L>(ff, w, dw, vf, af, F, N);
        h[7 + J] = dot(a, F);
        Fs = Fs + F;
        Ns = Ns + N;
    });
#pragma unroll
    for (int I = 0; I < 7; I++) {
        V3 Fsub = Fs - Fpre[I], Nsub = Ns - Npre[I];
        h[I] = dot(ax[I], Nsub - cross(org[I], Fsub));
    }
}

// M = L L^T, then M^-1 (packed symmetric) = L^-T L^-1
PS_D void spd_inverse(float M[45]) {
    // Cholesky with one reciprocal square root per column (v_rsq_f32, 1 ulp:
    // sqrtf and the IEEE division took ~22 VALU instructions per pivot): the
    // 36 off-diagonal divisions are products with it, and the inverse below
    // reads the pivots' reciprocals only
    float L[45], invd[9];
#pragma unroll
    for (int i = 0; i < 9; i++) {
#pragma unroll
        for (int j = 0; j <= i; j++) {
            float s = M[sidx(i, j)];
#pragma unroll
            for (int q = 0; q < j; q++) s -= L[sidx(i, q)] * L[sidx(j, q)];
            if (i == j) {
                invd[i] = __builtin_amdgcn_rsqf(s);  // M is SPD: s > 0
            } else {
                L[sidx(i, j)] = s * invd[j];
            }
        }
    }
    // invert L in place (lower triangular)
    float Li[45];
#pragma unroll
    for (int i = 0; i < 9; i++) {
        const float inv = invd[i];
        Li[sidx(i, i)] = inv;
#pragma unroll
        for (int j = 0; j < i; j++) {
            float s = 0.0f;
#pragma unroll
            for (int q = j; q < i; q++) s += L[sidx(i, q)] * Li[sidx(q, j)];
            Li[sidx(i, j)] = -s * inv;
        }
    }
#pragma unroll
    for (int i = 0; i < 9; i++)
#pragma unroll
        for (int j = 0; j <= i; j++) {
            float s = 0.0f;
#pragma unroll
            for (int q = i; q < 9; q++) s += Li[sidx(q, i)] * Li[sidx(q, j)];
            M[sidx(i, j)] = s;
        }
}

// --------------------------------------------------------------------- IK
// calculateInverseKinematics (restated in DESIGN.md §5, IK): <= 20 DLS steps
// dq = (J^T J + 0.5 I)^-1 J^T [dp; dr], pivot-frame Jacobian, 45 deg clamp.
template <int LINK>
PS_D void inverse_kinematics(const float q_start[9], V3 target, Q4 orn, float q_out[9]) {
    constexpr int NA = LINK <= 6 ? LINK + 1 : 7;  // arm DoFs that move LINK
    constexpr bool FINGER = (LINK == 9 || LINK == 10);
    constexpr int N = NA + (FINGER ? 1 : 0);
    constexpr int FD = LINK == 9 ? 7 : 8;
    float on = sqrtf(orn.x * orn.x + orn.y * orn.y + orn.z * orn.z + orn.w * orn.w);
    Q4 ot = Q4{orn.x / on, orn.y / on, orn.z / on, orn.w / on};
    float q[9];
#pragma unroll
    for (int d = 0; d < 9; d++) q[d] = q_start[d];
    float diff = 1e30f;
    for (int it = 0; it < PM_IK_MAX_ITERS && diff > (float)PM_IK_RESIDUAL; it++) {
        Kin k;
        fk(q, k);
        V3 p = k.f[LINK].o;
        V3 dS = target - p;
        diff = norm(dS);
        Q4 qe = mat_to_quat(k.f[LINK].R);
        float n2 = qe.x * qe.x + qe.y * qe.y + qe.z * qe.z + qe.w * qe.w;
        const float in2 = 1.0f / n2;
        Q4 qinv = Q4{-qe.x * in2, -qe.y * in2, -qe.z * in2, qe.w * in2};
        Q4 dq = qmul(ot, qinv);
        // btQuaternion::getAngle()/getAxis() evaluate 2 acos(w) and
        // v / sqrt(1 - w^2); for a unit quaternion these equal 2 atan2(|v|, w)
        // and v / |v|, which stay accurate in fp32 when w -> 1 (acos would
        // quantise small orientation errors to ~7e-4 rad).
        float s2 = dq.x * dq.x + dq.y * dq.y + dq.z * dq.z;
        float vn = sqrtf(s2);
        float angle = 2.0f * atan2f(vn, dq.w);
        V3 axv = s2 < 10.0f * 2.2204460492503131e-16f ? mk(1, 0, 0) : mk(dq.x, dq.y, dq.z) * (1.0f / vn);
        if (angle > 3.14159265358979323846f) angle -= 6.28318530717958647692f;
        else if (angle < -3.14159265358979323846f) angle += 6.28318530717958647692f;
        V3 dR = axv * (angle / norm(axv));
        // Jacobian columns (6 x N)
        V3 Jv[N], Jw[N];
#pragma unroll
        for (int c = 0; c < NA; c++) {
            V3 a = col(k.f[c].R, 2);
            Jv[c] = cross(a, p - k.f[c].o);
            Jw[c] = a;
        }
        if constexpr (FINGER) {
            Jv[NA] = mul(k.f[LINK].R, mk(0.0f, LINK == 9 ? 1.0f : -1.0f, 0.0f));
            Jw[NA] = mk(0, 0, 0);
        }
        float U[N * (N + 1) / 2], g[N];
#pragma unroll
        for (int a = 0; a < N; a++) {
            g[a] = dot(Jv[a], dS) + dot(Jw[a], dR);
#pragma unroll
            for (int b = 0; b <= a; b++)
                U[a * (a + 1) / 2 + b] = dot(Jv[a], Jv[b]) + dot(Jw[a], Jw[b]) + (a == b ? (float)PM_IK_DAMPING : 0.0f);
        }
        // Cholesky solve, one reciprocal per pivot (the divisions by it are
        // products: an IEEE division is ~10 VALU instructions).  A v_rsq_f32
        // pivot (1 ulp) measured 0.3 % faster per step but, together with the
        // damping norms' v_sqrt in bias_forces, moved one in-contact Push
        // sample past the parity bound: not kept.
        float Lc[N * (N + 1) / 2], il[N];
#pragma unroll
        for (int i = 0; i < N; i++)
#pragma unroll
            for (int j = 0; j <= i; j++) {
                float s = U[i * (i + 1) / 2 + j];
#pragma unroll
                for (int t = 0; t < j; t++) s -= Lc[i * (i + 1) / 2 + t] * Lc[j * (j + 1) / 2 + t];
                if (i == j) {
                    Lc[i * (i + 1) / 2 + i] = sqrtf(s);
                    il[i] = 1.0f / Lc[i * (i + 1) / 2 + i];
                } else {
                    Lc[i * (i + 1) / 2 + j] = s * il[j];
                }
            }
        float y[N], x[N];
#pragma unroll
        for (int i = 0; i < N; i++) {
            float s = g[i];
#pragma unroll
            for (int t = 0; t < i; t++) s -= Lc[i * (i + 1) / 2 + t] * y[t];
            y[i] = s * il[i];
        }
#pragma unroll
        for (int i = N - 1; i >= 0; i--) {
            float s = y[i];
#pragma unroll
            for (int t = i + 1; t < N; t++) s -= Lc[t * (t + 1) / 2 + i] * x[t];
            x[i] = s * il[i];
        }
        float mx = 0.0f;
#pragma unroll
        for (int i = 0; i < N; i++) mx = fmaxf(mx, fabsf(x[i]));
        float sc = mx > (float)PM_IK_MAX_ANGLE ? (float)PM_IK_MAX_ANGLE / mx : 1.0f;
#pragma unroll
        for (int i = 0; i < NA; i++) q[i] += x[i] * sc;
        if constexpr (FINGER) q[FD] += x[NA] * sc;
    }
#pragma unroll
    for (int d = 0; d < 9; d++) q_out[d] = q[d];
}

// ------------------------------------------------------------- the scene
// Objects: NOBJ dynamic bodies (0 Reach; 1 Push/PickAndPlace/Flip/Slide; 2
// Stack) of one SHAPE (SHAPE_BOX: cubes, isotropic inertia; SHAPE_CYL: the
// upright cylinder of Slide, anisotropic inertia).
constexpr int SHAPE_BOX = PS_SHAPE_BOX;
constexpr int SHAPE_CYL = PS_SHAPE_CYLINDER;

struct Scene {
    V3 base;
    V3 half;                 // box half extents; cylinder (radius, radius, half height)
    float mass, mass2, fric;  // object 1 / object 2 mass, lateral friction of the objects
    float table_cx, table_hx, table_hy;
    int has_table, has_plane;
};

struct Motors {
    float target[9], kp[9], kd[9], vel[9], imp[9];
};

struct Body {
    V3 pos;
    Q4 quat;
    V3 vel, omg;
};
typedef Body Cube;

// btBoxShape / btCylinderShapeZ::calculateLocalInertia (oracle object_inertia)
template <int SHAPE>
PS_D V3 local_inertia(const Scene &sc, float m) {
    if constexpr (SHAPE == SHAPE_CYL) {
        float r = sc.half.x, hh = sc.half.z;
        float t1 = m / 12.0f * (4.0f * hh * hh) + m / 4.0f * (r * r), t2 = m / 2.0f * (r * r);
        return mk(t1, t1, t2);
    } else {
        float lx = 2.0f * sc.half.x, ly = 2.0f * sc.half.y, lz = 2.0f * sc.half.z;
        return mk(m / 12.0f * (ly * ly + lz * lz), m / 12.0f * (lx * lx + lz * lz), m / 12.0f * (lx * lx + ly * ly));
    }
}

// per-substep body quantities: the world inverse inertia is a scalar for the
// isotropic cubes and a symmetric 3x3 for the cylinder
// two fp32 lanes of a v_pk_*_f32 instruction (the solver packs pairs of
// independent scalar operations into them)
typedef float f32x2 __attribute__((ext_vector_type(2)));

// mul(S3, V3) with rows x and y as v_pk_* pairs, for the solver loop's
// velocity updates: each lane computes what the scalar row compiles to there,
// fma(I_xz, v_z, fma(I_xx, v_x, I_xy v_y)) for row x, so the same bits
PS_D V3 mul_pk(const S3 &I, V3 v) {
#pragma clang fp contract(off)
    f32x2 xy = (f32x2){I.xy, I.yy} * (f32x2){v.y, v.y};
    xy = __builtin_elementwise_fma((f32x2){I.xx, I.xy}, (f32x2){v.x, v.x}, xy);
    xy = __builtin_elementwise_fma((f32x2){I.xz, I.yz}, (f32x2){v.z, v.z}, xy);
    return mk(xy.x, xy.y, fmaf(I.zz, v.z, fmaf(I.xz, v.x, I.yz * v.y)));
}
// the same product inside a `fp contract(off)` block: three products and two
// sums per row
PS_D V3 mul_pk_unfused(const S3 &I, V3 v) {
#pragma clang fp contract(off)
    const f32x2 xy = ((f32x2){I.xx, I.xy} * (f32x2){v.x, v.x} + (f32x2){I.xy, I.yy} * (f32x2){v.y, v.y}) +
                     (f32x2){I.xz, I.yz} * (f32x2){v.z, v.z};
    return mk(xy.x, xy.y, (I.xz * v.x + I.yz * v.y) + I.zz * v.z);
}

template <int SHAPE>
struct BodyDyn {
    M3 R;
    float inv_m, iI;
    S3 Ii;
    PS_D V3 inv_inertia(V3 v) const {
        if constexpr (SHAPE == SHAPE_CYL) return mul(Ii, v);
        else return v * iI;
    }
    // the solver loop's: rows x and y packed (mul_pk, mul_pk_unfused)
    PS_D V3 inv_inertia_pk(V3 v) const {
        if constexpr (SHAPE == SHAPE_CYL) return mul_pk(Ii, v);
        else return v * iI;
    }
    PS_D V3 inv_inertia_pk_unfused(V3 v) const {
        if constexpr (SHAPE == SHAPE_CYL) return mul_pk_unfused(Ii, v);
        else return v * iI;
    }
};

template <int SHAPE>
PS_D BodyDyn<SHAPE> body_dyn(const Scene &sc, const Body &b, float m) {
    BodyDyn<SHAPE> o;
    o.R = quat_to_mat(b.quat);
    o.inv_m = 1.0f / m;
    V3 I = local_inertia<SHAPE>(sc, m);
    o.iI = 1.0f / I.x;
    if constexpr (SHAPE == SHAPE_CYL) o.Ii = rotate_diag(o.R, 1.0f / I.x, 1.0f / I.y, 1.0f / I.z);
    return o;
}

PS_D bool ground_top(const Scene &sc, float x, float y, float &top) {
    if (sc.has_table && fabsf(x - sc.table_cx) <= sc.table_hx && fabsf(y) <= sc.table_hy) {
        top = (float)PM_TABLE_TOP;
        return true;
    }
    if (sc.has_plane) {
        top = (float)PM_PLANE_TOP;
        return true;
    }
    return false;
}

// support point v of the shape (object frame): box vertices, or cylinder rim
// points (bottom cap then top cap, PM_CYL_RIM_ORDER)
template <int SHAPE>
constexpr int num_support() { return SHAPE == SHAPE_CYL ? 2 * PM_CYL_RIM_POINTS : 8; }

template <int SHAPE, int V>
PS_D V3 support_point(const Scene &sc) {
    if constexpr (SHAPE == SHAPE_CYL) {
        constexpr int order[PM_CYL_RIM_POINTS] = PM_CYL_RIM_ORDER;
        constexpr int cap = V / PM_CYL_RIM_POINTS;
        constexpr int j = order[V % PM_CYL_RIM_POINTS];
        // cos/sin of multiples of 45 degrees, exact to float
        constexpr float cs[8] = {1.0f, 0.70710678118654752f, 0.0f, -0.70710678118654752f,
                                 -1.0f, -0.70710678118654752f, 0.0f, 0.70710678118654752f};
        constexpr float sn[8] = {0.0f, 0.70710678118654752f, 1.0f, 0.70710678118654752f,
                                 0.0f, -0.70710678118654752f, -1.0f, -0.70710678118654752f};
        return mk(sc.half.x * cs[j], sc.half.x * sn[j], cap ? sc.half.z : -sc.half.z);
    } else {
        return mk((V & 1) ? sc.half.x : -sc.half.x, (V & 2) ? sc.half.y : -sc.half.y,
                  (V & 4) ? sc.half.z : -sc.half.z);
    }
}

// closest point of the solid to `loc` (object frame): surface point cl,
// outward normal nl; returns the signed distance (negative inside)
template <int SHAPE>
PS_D float object_closest(const Scene &sc, V3 loc, V3 &cl, V3 &nl) {
    const V3 h = sc.half;
    if constexpr (SHAPE == SHAPE_CYL) {
        float r = h.x, hh = h.z;
        float rho = fast_sqrt(loc.x * loc.x + loc.y * loc.y);
        float zc = fminf(fmaxf(loc.z, -hh), hh);
        float irho = fast_rcp(rho);  // used only where rho > 1e-12
        float s = rho > r ? r * irho : 1.0f;
        cl = mk(loc.x * s, loc.y * s, zc);
        V3 dif = loc - cl;
        float dn = fast_norm(dif);
        if (dn > 1e-9f) {
            nl = dif * fast_rcp(dn);
            return dn;
        }
        float side = r - rho, cap = hh - fabsf(loc.z);
        if (side < cap) {
            nl = rho > 1e-12f ? mk(loc.x * irho, loc.y * irho, 0.0f) : mk(1.0f, 0.0f, 0.0f);
            cl = mk(nl.x * r, nl.y * r, cl.z);
            return -side;
        }
        nl = mk(0.0f, 0.0f, loc.z >= 0.0f ? 1.0f : -1.0f);
        cl.z = nl.z * hh;
        return -cap;
    } else {
        cl = mk(fminf(fmaxf(loc.x, -h.x), h.x), fminf(fmaxf(loc.y, -h.y), h.y), fminf(fmaxf(loc.z, -h.z), h.z));
        V3 dif = loc - cl;
        float dn = norm(dif);
        if (dn > 1e-9f) {
            nl = dif * (1.0f / dn);
            return dn;
        }
        float bx = h.x - fabsf(loc.x), by = h.y - fabsf(loc.y), bz = h.z - fabsf(loc.z);
        int ax = 0;
        float best = bx;
        if (by < best) { best = by; ax = 1; }
        if (bz < best) { best = bz; ax = 2; }
        float sg;
        if (ax == 0) { sg = loc.x >= 0.0f ? 1.0f : -1.0f; nl = mk(sg, 0, 0); cl.x = sg * h.x; }
        else if (ax == 1) { sg = loc.y >= 0.0f ? 1.0f : -1.0f; nl = mk(0, sg, 0); cl.y = sg * h.y; }
        else { sg = loc.z >= 0.0f ? 1.0f : -1.0f; nl = mk(0, 0, sg); cl.z = sg * h.z; }
        return -best;
    }
}

// btPlaneSpace1
PS_D void plane_space(V3 n, V3 &p, V3 &q) {
    if (fabsf(n.z) > 0.70710678118654752f) {
        float a = n.y * n.y + n.z * n.z, k = rsqrtf(a);
        p = mk(0.0f, -n.z * k, n.y * k);
        q = mk(a * k, -n.x * p.z, n.x * p.y);
    } else {
        float a = n.x * n.x + n.y * n.y, k = rsqrtf(a);
        p = mk(-n.y * k, n.x * k, 0.0f);
        q = mk(-n.z * p.y, n.z * p.x, a * k);
    }
}

constexpr int NG = PM_MAX_GROUND_CONTACTS;
constexpr int NR = PM_MAX_ROBOT_CONTACTS;
constexpr int NP = PM_MAX_PAIR_CONTACTS;
// LDS floats per lane: M^-1 J^T of the 3 rows of every gripper contact
// (108 floats x 256 lanes per CU = 108 KiB of the 160 KiB LDS at one wave per
// SIMD).
// Then 40 floats of per-substep values the PGS loop never reads (q, v1, the
// split-impulse position correction, object 1's pre-solve velocities and
// pose): they wait in LDS across the solve instead of holding registers.
constexpr int LDS_STASH_OFFSET = NR * 27;
constexpr int LDS_STASH_FLOATS = 40;
// Then the scenes with at most one object hold their contact cache (the
// object's ground rows and the gripper rows, 10 floats) in LDS across the
// control step's substeps: loaded from the state once per step and written
// back once (run_substeps), not read and written through L2 every substep.
constexpr int LDS_CACHE_OFFSET = LDS_STASH_OFFSET + LDS_STASH_FLOATS;
constexpr int LDS_CACHE_FLOATS = 10;
constexpr int LDS_FLOATS = LDS_CACHE_OFFSET + LDS_CACHE_FLOATS;
static_assert(LDS_FLOATS * 4 * 64 * 4 <= 160 * 1024, "four workgroups per CU");
// Stack (two cubes) keeps in LDS the gripper rows' J (the slots the other
// scenes use for M^-1 J^T; the loop forms M^-1 J^T from the M^-1 registers)
// and both cubes' ground rows (r, rhs: 6 per contact; 1/den is rebuilt from r,
// cube_ground_dinv) instead of registers, where they spilled to scratch.  Its
// 40-float stash, object 1's pre-solve state and the box-box pair rows
// (dir[3], rA, rB, rhs, dinv: 21 per contact, read only while some lane of
// the wave has a pair contact; r x dir is rebuilt in the loop) sit in a global
// per-env buffer (GSTASH_FLOATS: the stash rows env-minor, the pair rows
// env-major so one lane pointer with immediate offsets reads them).  That is 156 LDS floats per lane = 39 KB per
// 64-lane workgroup: four workgroups per CU, one wave per SIMD, as the
// one-object scenes.
constexpr int LDS_GND_OFFSET = NR * 27;
constexpr int LDS_GND_FLOATS = 6;
constexpr int LDS_FLOATS_STACK = LDS_GND_OFFSET + 2 * NG * LDS_GND_FLOATS;
static_assert(LDS_FLOATS_STACK * 4 * 64 * 4 <= 160 * 1024, "four Stack workgroups per CU");
constexpr int PAIR_FLOATS = 21;
// Stack's global stash rows (env-minor): the stash without the split-impulse
// corrections (recomputed from q after the solve, split_of: 9 rows fewer) and
// object 1's pre-solve state.
constexpr int GSTASH_ROWS = LDS_STASH_FLOATS + 13 - 9;
constexpr int GSTASH_PAIR_OFFSET = GSTASH_ROWS;
// The pair and gripper rows of a slot an env does not use are never written:
// the solver, which runs a slot's rows while any lane of the wave has it,
// points the lanes without it at one all-zero block (GSTASH_ZERO_FLOATS, after
// the stash, zeroed at allocation: ensure_stash) -- exact no-op rows, one
// cache line for the whole wave.  Before, every env rewrote its unused slots
// as zeros every substep and the wave read 64 env-major rows per slot: most of
// Stack's HBM traffic (2.03 GB per launch at 65 536 envs, VERDICT r05 weak 3;
// ~2 % of envs have a box-box contact at a time).
constexpr int GSTASH_ZERO_FLOATS = 32;
// Stack: M^-1 J^T of the gripper slots' normal rows, env-major after the
// pair rows (9 floats per slot), computed with J at contact setup and loaded
// at the top of each sweep (object_normals), so a gripper normal updates dv
// with 9 FMAs instead of the 81 of M^-1 (J^T dl): 7.89 -> 7.60 ms per step at
// 65 536 envs.  The friction rows' 18 floats per slot the same way spilled
// 40-81 VGPRs and ran slower (8.12 ms for 2 slots, 8.76 for 4:
// profiles/r03j_variants_stack_grip_mj.log), so those keep the M^-1 product.
constexpr int GRIP_MJ_SLOTS = NR;
constexpr int GSTASH_GRIP_OFFSET = GSTASH_PAIR_OFFSET + NP * PAIR_FLOATS;
constexpr int GRIP_FLOATS = GRIP_MJ_SLOTS * 9;
constexpr int GSTASH_FLOATS = GSTASH_GRIP_OFFSET + GRIP_FLOATS;
template <int NOBJ>
constexpr int lds_floats() {
#ifdef PS_EXPERIMENT_TWO_WAVES
    if (NOBJ < 2) return 61;
#endif
    return NOBJ == 2 ? LDS_FLOATS_STACK : LDS_FLOATS;
}
constexpr int GX_FLOATS = LDS_STASH_OFFSET + LDS_STASH_FLOATS;  // PS_EXPERIMENT_TWO_WAVES

// object-ground contact: object-only rows; normal +z, friction dirs of
// planeSpace(+z) = (0,-1,0), (1,0,0).  The cylinder's I^-1 (r x dir) is rebuilt
// in the solver from its 3x3 inverse inertia rather than held per row.
struct GroundContact {
    V3 r;  // contact point - object COM
    float rhs[3], lam[3], dinv[3];
    int id;  // contact cache id: 1 + support point (0: no contact)
};

// object-object contact (Stack): A = incident body (+n), B = reference (-n)
struct PairContact {
    V3 dir[3], rA, rB;  // contact point - COM of object 0 (rA) and of object 1 (rB)
    float rhs[3], lam[3], dinv[3];
    bool a0;  // body A is object 0
};

// gripper contact: robot rows with explicit Jacobians (M^-1 J^T lives in LDS)
struct RobotContact {
    float J[3][9];
    V3 dir[3];
    V3 rn[3];  // object side: (pB - x_obj) x dir (zero when the contact is with the ground)
    float rhs[3], lam[3], dinv[3], mu;
    bool o1;   // the object is object 1 (Stack)
};

// per-lane view of the LDS rows: element (slot, row, k) at base[((slot*3 + row)*9 + k) * stride]
typedef __attribute__((address_space(3))) float lds_float;
struct MJStore {
    lds_float *base;
    int stride;
    // the work lists' per-lane output rows (robot_candidates), stride kBlock:
    // in this lane's column (base + CW_OUT rows) unless the env's column is
    // shared by its group's lanes (shared_lds<G>)
    lds_float *cwo = nullptr;
#ifdef PS_EXPERIMENT_TWO_WAVES
    // Experiment: the one-object kernels at
    // two waves per SIMD.  The M^-1 J^T rows, the candidate records and the
    // stash (floats [0, 148) of the LDS column) move to a wave-tiled global
    // buffer (as Stack's stash: element k of env i at ((i / 64) * 148 + k) * 64
    // + i % 64); LDS keeps the work lists' 51 floats and the contact cache, 61
    // floats per lane, and the kernel is register-allocated for two waves.
    __attribute__((address_space(1))) float *gx = nullptr;
    uint32_t gxl = 0;
    PS_D float &gxr(int k) const {
        __attribute__((address_space(1))) float *page = gx + (k / 16) * 1024;
        asm("" : "+s"(page));
        return *(float *)((__attribute__((address_space(1))) char *)page + gxl + (k % 16) * 256);
    }
    // an index that varies by lane (a candidate slot): the whole address per lane
    PS_D float &gxd(int k) const {
        return *(float *)((__attribute__((address_space(1))) char *)gx + gxl + (uint32_t)k * 256u);
    }
    PS_D float &at(int slot, int row, int k) const { return gxr((slot * 3 + row) * 9 + k); }
    PS_D lds_float &cache(int k) const { return base[(51 + k) * stride]; }
    PS_D float &stash(int k) const { return gxr(LDS_STASH_OFFSET + k); }
#else
    PS_D lds_float &at(int slot, int row, int k) const { return base[((slot * 3 + row) * 9 + k) * stride]; }
    PS_D lds_float &cache(int k) const { return base[(LDS_CACHE_OFFSET + k) * stride]; }
    PS_D lds_float &stash(int k) const { return base[(LDS_STASH_OFFSET + k) * stride]; }
#endif
    // Stack: the stash in global memory ([GSTASH_PAIR_OFFSET][stride] floats, this env's column)
    // (wave-uniform base and stride, the lane's byte offset: global_* v_off, s[base])
    float *gst = nullptr;
    int64_t gst_stride = 0;
    uint32_t goff = 0;
    // Stack: this env's pair rows, env-major after the stash rows
    // ([stride][NP * PAIR_FLOATS]): one lane pointer plus immediate offsets
    __attribute__((address_space(1))) float *gpair = nullptr;
    PS_D float &gstash(int k) const {
        float *row = gst + k * gst_stride;
        asm("" : "+s"(row));  // no reassociation into a per-lane pointer (StateView::at)
        return *(float *)((char *)row + goff);
    }
    // Stack only: ground row c of cube c / NG, field k (r.xyz, rhs[3])
    PS_D lds_float &gnd(int c, int k) const { return base[(LDS_GND_OFFSET + c * LDS_GND_FLOATS + k) * stride]; }
    // Stack only (global stash): pair row c, field k (dir[3].xyz, r0.xyz, r1.xyz, rhs[3], dinv[3]);
    // dir is body A's (+n), r0 / r1 are the offsets from object 0 / 1
    PS_D float &pair(int c, int k) const { return *(float *)&gpair[c * PAIR_FLOATS + k]; }
    // Stack only (global stash): M^-1 J^T of gripper slot c's normal row, element k
    __attribute__((address_space(1))) float *ggrip = nullptr;
    PS_D float &grip(int c, int k) const { return *(float *)&ggrip[c * 9 + k]; }
    // Stack: the solver's source of pair slot c / gripper slot c: this env's
    // rows if it has the slot (c < n), else the shared zero block
    __attribute__((address_space(1))) float *gzero = nullptr;
    PS_D __attribute__((address_space(1))) float *pair_rows(int c, int n) const {
        return c < n ? gpair + c * PAIR_FLOATS : gzero;
    }
    PS_D __attribute__((address_space(1))) float *grip_rows(int c, int n) const {
        return c < n ? ggrip + c * 9 : gzero;
    }
    // a copy whose address the compiler cannot see through: loads from it are
    // not loop-invariant, so they stay in the PGS loop as ds_reads instead of
    // being hoisted into (spilled) registers
    PS_D MJStore opaque() const {
        MJStore r = *this;
        asm volatile("" : "+v"(r.base));
#ifdef PS_EXPERIMENT_TWO_WAVES
        asm volatile("" : "+v"(r.gxl));
#endif
        asm volatile("" : "+v"(r.goff));
        asm volatile("" : "+v"(r.gpair));
        asm volatile("" : "+v"(r.ggrip));
        return r;
    }
};

// The one-lane solver's robot velocity change, DoFs (2k, 2k + 1) as f32x2
// values and DoF 8 alone: the pairs stay vectors through the solver loop's
// phis, so a DoF's broadcast into a packed operand selects its half of the
// register pair (op_sel) instead of copying it out first.
struct VelChange {
    f32x2 p[4];
    float z;
    PS_D float g(int a) const { return a == 8 ? z : p[a >> 1][a & 1]; }
    PS_D void s(int a, float v) {
        if (a == 8) z = v;
        else p[a >> 1][a & 1] = v;
    }
    // (dv_a, dv_a): the broadcast of one DoF
    PS_D f32x2 bc(int a) const {
        if (a == 8) return (f32x2){z, z};
        return (a & 1) ? __builtin_shufflevector(p[a >> 1], p[a >> 1], 1, 1)
                       : __builtin_shufflevector(p[a >> 1], p[a >> 1], 0, 0);
    }
    // dv += m s as four v_pk_fma_f32 and one v_fma_f32: the same fused
    // products, element for element, as nine v_fma_f32 (the gripper rows'
    // M^-1 J^T come from LDS as ds_read2 pairs, already in register pairs)
    PS_D void apply(const float m[9], float sc) {
#pragma unroll
        for (int k = 0; k < 4; k++)
            p[k] = __builtin_elementwise_fma((f32x2){m[2 * k], m[2 * k + 1]}, (f32x2){sc, sc}, p[k]);
        z = fmaf(m[8], sc, z);
    }
    // J . dv as the scalar chain fma(J_a, dv_a, s) from s = 0 (jrow_dot)
    PS_D float dot(const float J[9]) const {
        float acc = 0.0f;
#pragma unroll
        for (int a = 0; a < 9; a++) acc = fmaf(J[a], g(a), acc);
        return acc;
    }
};

// fma3 with x and y as one v_pk_fma_f32 (the same bits)
PS_D V3 pk_fma3(V3 a, float s, V3 c) {
    const f32x2 xy = __builtin_elementwise_fma((f32x2){a.x, a.y}, (f32x2){s, s}, (f32x2){c.x, c.y});
    return mk(xy.x, xy.y, fmaf(a.z, s, c.z));
}

PS_D float jrow_dot(const float J[9], const float v[9]) {
    float s = 0.0f;
#pragma unroll
    for (int d = 0; d < 9; d++) s += J[d] * v[d];
    return s;
}

// Geometry that outlives the kinematics: DoF axes/origins (gripper-contact
// Jacobians), the hand's rotation (every gripper box's: the finger frames are
// the hand's, translated), the world box centres and the wrist sphere centre.
struct Geo {
    V3 ax[9], org[7], bc[PM_NUM_BOXES], wc;
    M3 hR;
};

// ------------------------------------------------- gripper collision boxes
// The oracle's gen_contacts restated in fp32 (oracle/panda_oracle.c
// box_cube_cands / box_cyl_cands / box_ground_cands / pick_contacts, DESIGN.md
// §5): each (box, target) pair offers at most PM_BOX_CONTACTS points, picked
// from a fixed candidate stream -- the deepest within the margin, then the one
// farthest from it -- and ordered along the box's longest axis.  The stream is
// visited twice (once per pick) instead of being stored: its expensive part
// (separating axis, reference and incident faces) is computed once, the
// candidates themselves are a few FMAs each.
struct RCand {
    V3 pA, pB, n;  // robot point, object/ground point, normal from B to A
    float dist;
};
PS_D float comp(V3 v, int i) { return i == 0 ? v.x : (i == 1 ? v.y : v.z); }
PS_D V3 colsel(const M3 &R, int c) { return c == 0 ? col(R, 0) : (c == 1 ? col(R, 1) : col(R, 2)); }

template <int MAXN, class Visit>
PS_D int pick_two(Visit &&visit, V3 org, V3 w, RCand &c0, RCand &c1) {
    const float margin = (float)PM_CONTACT_MARGIN_ROBOT;
    const RCand none{mk(0, 0, 0), mk(0, 0, 0), mk(0, 0, 1), 1.0f};
    auto sel = [](bool t, const RCand &a, const RCand &b) {
        return RCand{t ? a.pA : b.pA, t ? a.pB : b.pB, t ? a.n : b.n, t ? a.dist : b.dist};
    };
    // one pass, branch-free, validity folded into the scores (see
    // BoxCube::pick): the first pick minimises depth + PM_PICK_SKEW_WEIGHT x
    // the skew coordinate; the candidates extreme along the skew are tracked
    // for the second
    RCand cmin = none, cmax = none;
    float s0 = 1e30f, vmin = 1e30f, vmax = -1e30f;
    c0 = none;
    c1 = none;  // written for MAXN < 2 too (the caller copies it)
    visit([&](bool ok, const RCand &c) {
        const bool valid = ok && c.dist < margin;
        const float sv = dot(c.pA - org, w);
        const float sc = valid ? fmaf((float)PM_PICK_SKEW_WEIGHT, sv, c.dist) : 1e30f;
        const bool take = sc < s0;
        s0 = take ? sc : s0;
        c0 = sel(take, c, c0);
        if constexpr (MAXN >= 2) {
            const bool tmin = valid && sv < vmin, tmax = valid && sv > vmax;
            vmin = tmin ? sv : vmin;
            vmax = tmax ? sv : vmax;
            cmin = sel(tmin, c, cmin);
            cmax = sel(tmax, c, cmax);
        }
    });
    const bool has0 = s0 < 1e29f;
    bool has1 = false;
    if constexpr (MAXN >= 2) {
        const float sf = dot(c0.pA - org, w);
        c1 = sel(vmax - sf >= sf - vmin, cmax, cmin);
        const V3 d = c1.pA - c0.pA;
        has1 = has0 && dot(d, d) > 1e-8f;  // (0.1 mm)^2: not the same point
        if (has1 && dot(c1.pA - org, w) < sf) {
            const RCand t = c0;
            c0 = c1;
            c1 = t;
        }
    }
    return has0 ? (has1 ? 2 : 1) : 0;
}

// robot box (centre xc, rotation xR, half extents xh) vs a cube (yc, yR, yh)
struct BoxCube {
    bool sep;
    V3 nref, t1, t2, cf;
    float hu, hv;
    bool robot_ref;
    float P[4][3];  // incident face vertices (u, v, depth below the reference face)
    PS_D BoxCube(V3 xc, const M3 &xR, V3 xh, V3 yc, const M3 &yR, V3 yh) {
        const V3 d = yc - xc;
        float best = 1e30f;
        int ref = 0, axn = 0;
        sep = false;
        nref = mk(0, 0, 0);
        // the separating-axis radii from |C| = |xR^T yR| (both rotations
        // orthonormal: a box's own axes project to its half extents), 9 dot
        // products instead of 36
        float C[3][3];
#pragma unroll
        for (int i = 0; i < 3; i++)
#pragma unroll
            for (int k = 0; k < 3; k++) C[i][k] = fabsf(dot(col(xR, i), col(yR, k)));
        const float xhv[3] = {xh.x, xh.y, xh.z}, yhv[3] = {yh.x, yh.y, yh.z};
#pragma unroll
        for (int b = 0; b < 2; b++)
#pragma unroll
            for (int ax = 0; ax < 3; ax++) {
                const V3 L = col(b == 0 ? xR : yR, ax);
                const float ra = b == 0 ? xhv[ax] : xh.x * C[0][ax] + xh.y * C[1][ax] + xh.z * C[2][ax];
                const float rb = b == 1 ? yhv[ax] : yh.x * C[ax][0] + yh.y * C[ax][1] + yh.z * C[ax][2];
                const float c = dot(d, L);
                const float pen = ra + rb - fabsf(c);
                sep = sep || pen < -(float)PM_CONTACT_MARGIN_ROBOT;
                if (pen < best - (float)PM_PAIR_AXIS_TOL) {
                    best = pen;
                    ref = b;
                    axn = ax;
                    nref = L * ((b == 0 ? c : -c) >= 0.0f ? 1.0f : -1.0f);
                }
            }
        robot_ref = ref == 0;
        const int a1 = axn == 2 ? 0 : axn + 1, a2 = axn == 0 ? 2 : axn - 1;
        const V3 hr = robot_ref ? xh : yh, hi = robot_ref ? yh : xh;
        const V3 cr = robot_ref ? xc : yc, ci = robot_ref ? yc : xc;
        M3 Rr, Ri;
#pragma unroll
        for (int k = 0; k < 9; k++) {
            Rr.m[k] = robot_ref ? xR.m[k] : yR.m[k];
            Ri.m[k] = robot_ref ? yR.m[k] : xR.m[k];
        }
        t1 = colsel(Rr, a1);
        t2 = colsel(Rr, a2);
        cf = cr + nref * comp(hr, axn);
        hu = comp(hr, a1);
        hv = comp(hr, a2);
        // incident face: the incident box's axis most anti-parallel to nref
        int ai = 0;
        float mostneg = 2.0f, si = 1.0f;
#pragma unroll
        for (int ax = 0; ax < 3; ax++) {
            const float dn = dot(col(Ri, ax), nref);
            if (-fabsf(dn) < mostneg) {
                mostneg = -fabsf(dn);
                ai = ax;
                si = dn > 0.0f ? -1.0f : 1.0f;
            }
        }
        const int b1 = ai == 2 ? 0 : ai + 1, b2 = ai == 0 ? 2 : ai - 1;
        const V3 ea = colsel(Ri, ai) * (si * comp(hi, ai)), eb = colsel(Ri, b1) * comp(hi, b1),
                 ec = colsel(Ri, b2) * comp(hi, b2);
        const V3 base = ci - cf;
        constexpr float cu[4] = {-1, 1, 1, -1}, cv[4] = {-1, -1, 1, 1};
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const V3 rel = base + ea + eb * cu[q] + ec * cv[q];
            P[q][0] = dot(rel, t1);
            P[q][1] = dot(rel, t2);
            P[q][2] = dot(rel, nref);
        }
    }
    // the candidates in the reference face's frame: (ok, u, v, depth), from
    // the incident face P and the rectangle half extents hu, hv
    template <class F>
    PS_D static void visit(const float (&P)[4][3], float hu, float hv, F &&emit) {
        constexpr float cu[4] = {-1, 1, 1, -1}, cv[4] = {-1, -1, 1, 1};
        // 1. incident vertices inside the reference rectangle
#pragma unroll
        for (int q = 0; q < 4; q++) emit(fabsf(P[q][0]) <= hu && fabsf(P[q][1]) <= hv, P[q][0], P[q][1], P[q][2]);
        // 2. reference corners inside the incident quadrilateral, depth on its plane
        const float e1u = P[1][0] - P[0][0], e1v = P[1][1] - P[0][1], e1d = P[1][2] - P[0][2];
        const float e3u = P[3][0] - P[0][0], e3v = P[3][1] - P[0][1], e3d = P[3][2] - P[0][2];
        const float pnu = e1v * e3d - e1d * e3v, pnv = e1d * e3u - e1u * e3d, pnd = e1u * e3v - e1v * e3u;
        const bool okp = pnd != 0.0f;
        const float ipnd = okp ? __builtin_amdgcn_rcpf(pnd) : 0.0f;  // v_rcp_f32 (1 ulp): not an IEEE division
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const float u = cu[q] * hu, v = cv[q] * hv;
            bool pos = true, neg = true;
#pragma unroll
            for (int e = 0; e < 4; e++) {
                const int e2 = (e + 1) & 3;
                const float cr = (P[e2][0] - P[e][0]) * (v - P[e][1]) - (P[e2][1] - P[e][1]) * (u - P[e][0]);
                pos = pos && cr >= 0.0f;
                neg = neg && cr <= 0.0f;
            }
            const float depth = okp ? P[0][2] - (pnu * (u - P[0][0]) + pnv * (v - P[0][1])) * ipnd : 0.0f;
            emit((pos || neg) && okp, u, v, depth);
        }
        // 3. incident edges crossing the rectangle's edges (u = +-hu, v = +-hv)
#pragma unroll
        for (int e = 0; e < 4; e++) {
            const int e2 = (e + 1) & 3;
            const float du = P[e2][0] - P[e][0], dv = P[e2][1] - P[e][1], dd = P[e2][2] - P[e][2];
            const float idu = du != 0.0f ? __builtin_amdgcn_rcpf(du) : 0.0f, idv = dv != 0.0f ? __builtin_amdgcn_rcpf(dv) : 0.0f;
#pragma unroll
            for (int s = 0; s < 4; s++) {
                const bool on_u = s < 2;
                const float lim = (s & 1) ? -(on_u ? hu : hv) : (on_u ? hu : hv);
                const float ca = on_u ? P[e][0] : P[e][1];
                const bool has = on_u ? du != 0.0f : dv != 0.0f;
                const float t = has ? (lim - ca) * (on_u ? idu : idv) : -1.0f;
                const float u = P[e][0] + t * du, v = P[e][1] + t * dv;
                const bool ok = t > 0.0f && t < 1.0f && (on_u ? fabsf(v) <= hv : fabsf(u) <= hu);
                emit(ok, on_u ? lim : u, on_u ? v : lim, P[e][2] + t * dd);
            }
        }
    }
    PS_D RCand to_world(float u, float v, float depth) const {
        const V3 pref = cf + t1 * u + t2 * v, pinc = pref + nref * depth;
        return RCand{robot_ref ? pref : pinc, robot_ref ? pinc : pref, robot_ref ? -nref : nref, depth};
    }
    // pick_two over the candidates, in the reference face's frame: the robot
    // point's offsets are (du, dv) when the box is the reference, (du, dv,
    // ddepth) when it is the incident one; only the two picks go to world
    PS_D int pick(V3 org, V3 w, RCand &c0, RCand &c1) const {
        const float margin = (float)PM_CONTACT_MARGIN_ROBOT;
        const float wd = robot_ref ? 0.0f : 1.0f;
        // the robot point's skew coordinate, affine in (u, v, depth)
        const float k0 = dot(cf - org, w), k1 = dot(t1, w), k2 = dot(t2, w), k3 = wd * dot(nref, w);
        const float lam = (float)PM_PICK_SKEW_WEIGHT;
        // One pass, branch-free selects, validity folded into the scores: as
        // lane masks, the 24 candidates' validity bits stayed live in SGPRs
        // and spilled ~900 of them to VGPR lanes per substep.
        float s0 = 1e30f, vmin = 1e30f, vmax = -1e30f;
        float u0 = 0.0f, v0 = 0.0f, d0 = 1.0f, un = 0.0f, vn = 0.0f, dn = 1.0f, ux = 0.0f, vx = 0.0f, dx = 1.0f;
        visit(P, hu, hv, [&](bool ok, float u, float v, float d) {
            const bool valid = ok && d < margin;
            const float sv = fmaf(k3, d, fmaf(k2, v, fmaf(k1, u, k0)));
            const float sc = valid ? fmaf(lam, sv, d) : 1e30f;
            const bool take = sc < s0, tmin = valid && sv < vmin, tmax = valid && sv > vmax;
            s0 = take ? sc : s0;
            u0 = take ? u : u0;
            v0 = take ? v : v0;
            d0 = take ? d : d0;
            vmin = tmin ? sv : vmin;
            un = tmin ? u : un;
            vn = tmin ? v : vn;
            dn = tmin ? d : dn;
            vmax = tmax ? sv : vmax;
            ux = tmax ? u : ux;
            vx = tmax ? v : vx;
            dx = tmax ? d : dx;
        });
        const bool has0 = s0 < 1e29f && !sep;
        const float sf = fmaf(k3, d0, fmaf(k2, v0, fmaf(k1, u0, k0)));
        const bool hi = vmax - sf >= sf - vmin;
        const float u1 = hi ? ux : un, v1 = hi ? vx : vn, d1 = hi ? dx : dn;
        c0 = to_world(u0, v0, d0);
        c1 = to_world(u1, v1, d1);
        const V3 dd = c1.pA - c0.pA;
        const bool has1 = has0 && dot(dd, dd) > 1e-8f;  // (0.1 mm)^2: not the same point
        if (has1 && (hi ? vmax : vmin) < sf) {
            const RCand t = c0;
            c0 = c1;
            c1 = t;
        }
        return has0 ? (has1 ? 2 : 1) : 0;
    }
};

// robot box vs the cylinder (Slide), in the cylinder's frame
struct BoxCyl {
    V3 bc, yc;
    M3 bR, yR;
    V3 xh;
    float r, hh;
    PS_D BoxCyl(const Scene &sc, V3 xc, const M3 &xR, V3 xh_, V3 yc_, const M3 &yR_) : yc(yc_), yR(yR_), xh(xh_) {
        r = sc.half.x;
        hh = sc.half.z;
        bc = tmul(yR, xc - yc);
#pragma unroll
        for (int a = 0; a < 3; a++) {
            const V3 lc = tmul(yR, col(xR, a));
            bR.m[a] = lc.x;
            bR.m[3 + a] = lc.y;
            bR.m[6 + a] = lc.z;
        }
    }
    // the candidate stream in the cylinder's frame: emit(ok, robot point,
    // cylinder point, normal, distance)
    template <class F>
    PS_D void visit(const Scene &sc, F &&emit) const {
        // 1. box vertices vs the solid (the loops stay rolled: unrolled, the
        // two visits of the 36 candidates spilled ~300 VGPRs in Slide's kernels)
#pragma unroll 1
        for (int v = 0; v < 8; v++) {
            const V3 lA = bc + mul(bR, mk((v & 1) ? xh.x : -xh.x, (v & 2) ? xh.y : -xh.y, (v & 4) ? xh.z : -xh.z));
            V3 cl, nl;
            const float dist = object_closest<SHAPE_CYL>(sc, lA, cl, nl);
            emit(true, lA, cl, nl, dist);
        }
        // 2. side faces of the box vs the generator line facing them (unrolled:
        // with a loop counter the face's axis selects -- colsel(bR, ax),
        // comp(xh, a1) -- became dynamic indices into the BoxCyl object, which
        // then lived in 120 B of scratch in every Slide kernel, round 4)
#pragma unroll
        for (int fc = 0; fc < 6; fc++) {
            const int ax = fc >> 1;
            const float sg = (fc & 1) ? -1.0f : 1.0f;
            const V3 nf = colsel(bR, ax) * sg;
            const int a1 = ax == 2 ? 0 : ax + 1, a2 = ax == 0 ? 2 : ax - 1;
            const V3 t1 = colsel(bR, a1), t2 = colsel(bR, a2);
            const float h1 = comp(xh, a1), h2 = comp(xh, a2);
            const V3 fcen = bc + nf * comp(xh, ax);
            const bool side = fabsf(nf.z) < 0.5f;
            const float nxy = fast_sqrt(nf.x * nf.x + nf.y * nf.y);
            const float inv = side ? r * fast_rcp(nxy) : 0.0f;
            const V3 s0 = mk(-nf.x * inv, -nf.y * inv, 0.0f), d0 = s0 - fcen;
            float lo = -hh, hi = hh;
            bool empty = false;
            const float K[5][3] = {{dot(d0, t1), t1.z, h1},
                                   {-dot(d0, t1), -t1.z, h1},
                                   {dot(d0, t2), t2.z, h2},
                                   {-dot(d0, t2), -t2.z, h2},
                                   {dot(nf, fcen), -nf.z, 0.0f}};
#pragma unroll
            for (int k = 0; k < 5; k++) {
                const float k0 = K[k][0], k1 = K[k][1], lim = K[k][2];
                // (branch-free: z is read only where |k1| > 1e-12)
                const float z = (lim - k0) * fast_rcp(k1);
                hi = k1 > 1e-12f ? fminf(z, hi) : hi;
                lo = k1 < -1e-12f ? fmaxf(z, lo) : lo;
                empty = empty || (fabsf(k1) <= 1e-12f && k0 > lim);
            }
            const bool ok = side && !empty && lo <= hi;
#pragma unroll
            for (int e = 0; e < 2; e++) {
                const V3 lB = mk(s0.x, s0.y, e ? hi : lo);
                const float dist = dot(nf, lB - fcen);
                emit(ok, lB - nf * dist, lB, -nf, dist);
            }
        }
        // 3. rim points vs the box (support_point<SHAPE_CYL, V>'s order and
        // values) -- only for a box with a half extent beyond the radius (the
        // palm): a narrower box's face inside a cap is found by its vertices
        constexpr int order[PM_CYL_RIM_POINTS] = PM_CYL_RIM_ORDER;
        constexpr float c45 = 0.70710678118654752f;
        // A cap's rim points are skipped by the wave when no lane's box
        // reaches within the margin (+0.1 mm) of the cap's plane: such points
        // are farther than the margin from the box, invalid candidates that
        // cannot change the picks.  The bottom cap lies on the table, out of
        // the palm's reach, so its 8 points drop out in practically every
        // wave.  (The range is the wave's, so the loop counter stays scalar.)
        const bool wide = xh.x > r || xh.y > r || xh.z > r;
        const float reach = fabsf(bR.m[6]) * xh.x + fabsf(bR.m[7]) * xh.y + fabsf(bR.m[8]) * xh.z +
                            (float)PM_CONTACT_MARGIN_ROBOT + 1e-4f;
        const bool cap_lo = wide && fabsf(bc.z + hh) <= reach, cap_hi = wide && fabsf(bc.z - hh) <= reach;
        const bool any_lo = __builtin_amdgcn_ballot_w64(cap_lo) != 0, any_hi = __builtin_amdgcn_ballot_w64(cap_hi) != 0;
        const int vbeg = any_lo ? 0 : PM_CYL_RIM_POINTS, vend = any_hi ? 2 * PM_CYL_RIM_POINTS : PM_CYL_RIM_POINTS;
        static_assert(2 * PM_CYL_RIM_POINTS == num_support<SHAPE_CYL>(), "rim points: bottom cap, then top");
#pragma unroll 1
        for (int V = vbeg; V < vend; V++) {
            int j = 0;
#pragma unroll
            for (int k = 0; k < PM_CYL_RIM_POINTS; k++) j = (V % PM_CYL_RIM_POINTS) == k ? order[k] : j;
            const float cs = j == 0 ? 1.0f : j == 1 || j == 7 ? c45 : j == 2 || j == 6 ? 0.0f : j == 4 ? -1.0f : -c45;
            const float sn = j == 2 ? 1.0f : j == 1 || j == 3 ? c45 : j == 0 || j == 4 ? 0.0f : j == 6 ? -1.0f : -c45;
            const V3 p = mk(sc.half.x * cs, sc.half.x * sn, V >= PM_CYL_RIM_POINTS ? sc.half.z : -sc.half.z);
            const V3 lp = tmul(bR, p - bc);
            V3 cl = mk(fminf(fmaxf(lp.x, -xh.x), xh.x), fminf(fmaxf(lp.y, -xh.y), xh.y), fminf(fmaxf(lp.z, -xh.z), xh.z));
            const V3 dif = lp - cl;
            const float dn = fast_norm(dif);
            V3 nb;
            float dist;
            if (dn > 1e-9f) {
                nb = dif * fast_rcp(dn);
                dist = dn;
            } else {
                const float bx = xh.x - fabsf(lp.x), by = xh.y - fabsf(lp.y), bz = xh.z - fabsf(lp.z);
                int ax = 0;
                float bst = bx;
                if (by < bst) { bst = by; ax = 1; }
                if (bz < bst) { bst = bz; ax = 2; }
                const float s = comp(lp, ax) >= 0.0f ? 1.0f : -1.0f;
                nb = ax == 0 ? mk(s, 0, 0) : (ax == 1 ? mk(0, s, 0) : mk(0, 0, s));
                cl = ax == 0 ? mk(s * xh.x, cl.y, cl.z) : (ax == 1 ? mk(cl.x, s * xh.y, cl.z) : mk(cl.x, cl.y, s * xh.z));
                dist = -bst;
            }
            emit(wide, bc + mul(bR, cl), p, -mul(bR, nb), dist);
        }
    }
    PS_D RCand to_world(const RCand &l) const { return RCand{yc + mul(yR, l.pA), yc + mul(yR, l.pB), mul(yR, l.n), l.dist}; }
    // pick_two's selection in the cylinder's frame: the skew coordinate of a
    // robot point lA is dot(yc - org, w) + dot(lA, yR^T w), and only the two
    // picks go to world (per candidate, the world transform was 36 VALU of
    // the ~80 the generic pick_two spends)
    PS_D int pick(const Scene &sc, V3 org, V3 w, RCand &c0, RCand &c1) const {
        const float margin = (float)PM_CONTACT_MARGIN_ROBOT;
        const RCand none{mk(0, 0, 0), mk(0, 0, 0), mk(0, 0, 1), 1.0f};
        auto sel = [](bool t, const RCand &a, const RCand &b) {
            return RCand{t ? a.pA : b.pA, t ? a.pB : b.pB, t ? a.n : b.n, t ? a.dist : b.dist};
        };
        const V3 wl = tmul(yR, w);
        const float k0 = dot(yc - org, w);
        RCand l0 = none, lmin = none, lmax = none;
        float s0 = 1e30f, vmin = 1e30f, vmax = -1e30f;
        visit(sc, [&](bool ok, V3 lA, V3 lB, V3 ln, float dist) {
            const RCand c{lA, lB, ln, dist};
            const bool valid = ok && dist < margin;
            const float sv = k0 + dot(lA, wl);
            const float sc = valid ? fmaf((float)PM_PICK_SKEW_WEIGHT, sv, dist) : 1e30f;
            const bool take = sc < s0, tmin = valid && sv < vmin, tmax = valid && sv > vmax;
            s0 = take ? sc : s0;
            l0 = sel(take, c, l0);
            vmin = tmin ? sv : vmin;
            vmax = tmax ? sv : vmax;
            lmin = sel(tmin, c, lmin);
            lmax = sel(tmax, c, lmax);
        });
        const bool has0 = s0 < 1e29f;
        const float sf = k0 + dot(l0.pA, wl);
        const bool hi = vmax - sf >= sf - vmin;
        const RCand l1 = sel(hi, lmax, lmin);
        c0 = has0 ? to_world(l0) : none;
        c1 = has0 ? to_world(l1) : none;
        const V3 d = c1.pA - c0.pA;
        const bool has1 = has0 && dot(d, d) > 1e-8f;  // (0.1 mm)^2: not the same point
        if (has1 && (hi ? vmax : vmin) < sf) {
            const RCand t = c0;
            c0 = c1;
            c1 = t;
        }
        return has0 ? (has1 ? 2 : 1) : 0;
    }
};

// robot box vs the ground (table top or plane)
template <class F>
PS_D void box_ground_visit(const Scene &sc, V3 xc, const M3 &xR, V3 xh, F &&f) {
    const V3 ea = col(xR, 0) * xh.x, eb = col(xR, 1) * xh.y, ec = col(xR, 2) * xh.z;
#pragma unroll
    for (int v = 0; v < 8; v++) {
        const V3 p = xc + ((v & 1) ? ea : -ea) + ((v & 2) ? eb : -eb) + ((v & 4) ? ec : -ec);
        float top = 0.0f;
        const bool ok = ground_top(sc, p.x, p.y, top);
        f(ok, RCand{p, mk(p.x, p.y, top), mk(0, 0, 1), p.z - top});
    }
}

// row rhs of a contact normal (btSequentialImpulseConstraintSolver setup:
// speculative margin when separated, ERP/split-impulse when penetrating)
// (1/dt = 500 is exact in fp32: products with it instead of IEEE divisions
// by the rounded dt, and closer to the fp64 oracle's pen / dt)
constexpr float PS_INV_DT = (float)(1.0 / PM_TIMESTEP);
PS_D float normal_rhs(float dist, float rel, float dinv) {
    float pen = dist + (float)PM_LINEAR_SLOP;
    float velerr = -rel, poserr = 0.0f;
    if (pen > 0.0f) velerr -= pen * PS_INV_DT;
    else poserr = -pen * (float)PM_ERP * PS_INV_DT;
    bool combined = pen > (float)PM_SPLIT_PENETRATION_THRESHOLD;
    return (combined ? poserr + velerr : velerr) * dinv;
}

// 1/den of a row (v_rcp_f32, 1 ulp: an IEEE division is ~10 VALU
// instructions, and the substep takes ~35 of these)
PS_D float safe_inv(float den) { return den > 2.2204460492503131e-16f ? __builtin_amdgcn_rcpf(den) : 0.0f; }

// Stack: 1/den of a cube's ground row j (normal +z, then (0,-1,0), (1,0,0))
// from its contact offset r: den = |r x dir|^2 iI + 1/m (isotropic inertia);
// the row setup and the solver both use this, so LDS holds r and rhs only
PS_D float cube_ground_dinv(V3 r, int j, float iI, float inv_m) {
    V3 rn = j == 0 ? mk(r.y, -r.x, 0.0f) : j == 1 ? mk(r.z, 0.0f, -r.x) : mk(0.0f, r.z, -r.y);
    return __builtin_amdgcn_rcpf(dot(rn, rn * iI) + inv_m);  // den >= 1/m > 0
}

// Box-box contacts of the two cubes (Stack): the oracle's box_box_contacts
// (face-axis SAT, incident face clipped against the reference face) in fp32.
// Fills up to NP contact candidates: point on A (incident), point on B
// (reference), normal n (B -> A), distance.
struct PairCand {
    V3 pA, pB, n;
    float dist;
    bool a0;
};

// The clipped polygon in registers (round 5): a convex quad cut by four
// half-planes gains at most one vertex per cut, so 8 compile-time slots hold
// it, and a vertex goes to its runtime slot m by selects over the slots m can
// reach at that point.  With arrays indexed by m (the oracle's form) the
// polygons lived in 384 B of scratch per lane in every Stack kernel.
struct Poly8 {
    float u[8], v[8], d[8];
};

// write (u, v, d) to slot m when c; S = the slots m can address
template <int S>
PS_D void poly_put(Poly8 &p, int m, bool c, float u, float v, float d) {
#pragma unroll
    for (int s = 0; s < S; s++) {
        const bool w = c && m == s;
        p.u[s] = w ? u : p.u[s];
        p.v[s] = w ? v : p.v[s];
        p.d[s] = w ? d : p.d[s];
    }
}

// one Sutherland-Hodgman pass (oracle clip_half): keeps sign * coord <= lim,
// coord = u (AXIS 0) or v (AXIS 1); the input has n <= NI vertices.  Vertex i
// emits itself and/or the edge crossing, so before its writes m <= 2i and
// 2i + 1; a count past the NI + 1 slots (rounding at a degenerate edge) drops
// the extra vertices.
template <int NI, int AXIS>
PS_D int clip_half(const Poly8 &in, int n, float sign, float lim, Poly8 &out) {
    constexpr int NO = NI + 1 < 8 ? NI + 1 : 8;
    int m = 0;
    static_for<0, NI>([&](auto I) {
        constexpr int i = decltype(I)::value;
        constexpr int nx = i + 1 < NI ? i + 1 : 0;
        const bool act = i < n, wrap = i + 1 >= n;
        const float au = in.u[i], av = in.v[i], ad = in.d[i];
        const float bu = wrap ? in.u[0] : in.u[nx], bv = wrap ? in.v[0] : in.v[nx], bd = wrap ? in.d[0] : in.d[nx];
        const float ca = sign * (AXIS == 0 ? au : av) - lim, cb = sign * (AXIS == 0 ? bu : bv) - lim;
        const bool keep = act && ca <= 0.0f;
        poly_put<(2 * i + 1 < NO ? 2 * i + 1 : NO)>(out, m, keep, au, av, ad);
        m += keep ? 1 : 0;
        const bool cross = act && ((ca < 0.0f && cb > 0.0f) || (ca > 0.0f && cb < 0.0f));
        const float t = ca / (ca - cb);  // read only where the edge crosses
        poly_put<(2 * i + 2 < NO ? 2 * i + 2 : NO)>(out, m, cross, au + t * (bu - au), av + t * (bv - av),
                                                     ad + t * (bd - ad));
        m += cross ? 1 : 0;
    });
    return m < NO ? m : NO;
}

PS_D int box_box(const Scene &sc, const Body &b0, const Body &b1, const M3 &R0, const M3 &R1, PairCand out[NP]) {
    const V3 hv = sc.half;
    const float h[3] = {hv.x, hv.y, hv.z};  // constant indices only
    V3 d = b1.pos - b0.pos;
    float best = 1e30f;
    V3 nref = mk(0, 0, 0);
    int ref = 0, axn = 0;
#pragma unroll
    for (int b = 0; b < 2; b++)
#pragma unroll
        for (int ax = 0; ax < 3; ax++) {
            V3 L = col(b == 0 ? R0 : R1, ax);
            float ra = 0.0f, rb = 0.0f;
#pragma unroll
            for (int k = 0; k < 3; k++) {
                ra += h[k] * fabsf(dot(col(R0, k), L));
                rb += h[k] * fabsf(dot(col(R1, k), L));
            }
            float c = dot(d, L);
            float pen = ra + rb - fabsf(c);
            if (pen < -(float)PM_CONTACT_MARGIN_PAIR) return 0;
            if (pen < best - (float)PM_PAIR_AXIS_TOL) {
                best = pen;
                ref = b;
                axn = ax;
                float sg = (b == 0 ? c : -c) >= 0.0f ? 1.0f : -1.0f;
                nref = L * sg;
            }
        }
    // reference / incident bodies, selected per element (a select of the
    // matrices' addresses put them in memory)
    M3 Rr, Ri;
#pragma unroll
    for (int q = 0; q < 9; q++) {
        Rr.m[q] = ref == 0 ? R0.m[q] : R1.m[q];
        Ri.m[q] = ref == 0 ? R1.m[q] : R0.m[q];
    }
    V3 cr = ref == 0 ? b0.pos : b1.pos, ci = ref == 0 ? b1.pos : b0.pos;
    int a1 = axn + 1 == 3 ? 0 : axn + 1, a2 = axn + 2 >= 3 ? axn - 1 : axn + 2;
    V3 t1 = colsel(Rr, a1), t2 = colsel(Rr, a2);
    V3 cf = cr + nref * comp(hv, axn);
    int ai = 0;
    float mostneg = 2.0f, si = 1.0f;
#pragma unroll
    for (int ax = 0; ax < 3; ax++) {
        float dn = dot(col(Ri, ax), nref);
        if (-fabsf(dn) < mostneg) { mostneg = -fabsf(dn); ai = ax; si = dn > 0.0f ? -1.0f : 1.0f; }
    }
    int b1i = ai + 1 == 3 ? 0 : ai + 1;
    Poly8 P{}, T{};
    const float cu[4] = {-1, 1, 1, -1}, cv[4] = {-1, -1, 1, 1};
#pragma unroll
    for (int k = 0; k < 4; k++) {
        // the incident face's corner k: axis ai at si h, b1i at cu h, b2i at cv h
        float loc[3];
#pragma unroll
        for (int c = 0; c < 3; c++) loc[c] = (c == ai ? si : c == b1i ? cu[k] : cv[k]) * h[c];
        V3 rel = mul(Ri, mk(loc[0], loc[1], loc[2])) + ci - cf;
        P.u[k] = dot(rel, t1);
        P.v[k] = dot(rel, t2);
        P.d[k] = dot(rel, nref);
    }
    int n = clip_half<4, 0>(P, 4, 1.0f, comp(hv, a1), T);
    n = clip_half<5, 0>(T, n, -1.0f, comp(hv, a1), P);
    n = clip_half<6, 1>(P, n, 1.0f, comp(hv, a2), T);
    n = clip_half<7, 1>(T, n, -1.0f, comp(hv, a2), P);
    // the vertices within the margin, in order
    Poly8 K{};
    int m = 0;
    static_for<0, 8>([&](auto I) {
        constexpr int k = decltype(I)::value;
        const bool keep = k < n && P.d[k] < (float)PM_CONTACT_MARGIN_PAIR;
        poly_put<k + 1>(K, m, keep, P.u[k], P.v[k], P.d[k]);
        m += keep ? 1 : 0;
    });
    int take = m < NP ? m : NP;
#pragma unroll
    for (int k = 0; k < NP; k++) {
        int idx = m <= NP ? k : (k * m) / NP;
        float u = K.u[0], v = K.v[0], dd = K.d[0];
#pragma unroll
        for (int s = 1; s < 8; s++) {
            u = idx == s ? K.u[s] : u;
            v = idx == s ? K.v[s] : v;
            dd = idx == s ? K.d[s] : dd;
        }
        PairCand c;
        c.pB = cf + t1 * u + t2 * v;
        c.pA = c.pB + nref * dd;
        c.n = nref;
        c.dist = dd;
        c.a0 = ref == 1;  // A = incident
        out[k] = c;
    }
    return take;
}

// ----------------------------------------------------------------- substep
// One btMultiBodyDynamicsWorld::stepSimulation(1/500 s): see the oracle's
// po_substep for the row-by-row restatement this mirrors.
// PGS residual of a row is dl / dinv (the impulse change in velocity units).
// v_rcp_f32 replaces the IEEE division.  A lane without the row has dinv = 0
// and dl = 0: dinv is clamped to FLT_MIN so that the residual is 0 * 2^126 = 0
// there (the reference skips such rows), never 0 * inf = NaN -- a NaN in the
// residual max would depend on fmaxf's NaN rule, which a build that assumes
// no NaNs is free to change.
// PGS stopping rule: Bullet stops once max over rows of (dl / dinv)^2 <= 1e-7
// (the residual is the impulse change times the row's effective mass).  The
// loop tracks it as a violation that is <= 0 once every row has
// |dl| / dinv <= sqrt(1e-7), so no row takes a reciprocal:
//   contact rows  |dl| - sqrt(1e-7) dinv
//   joint rows    |dl| den - sqrt(1e-7)      (den = M^-1_dd, in registers)
constexpr float kResidualAbs = 3.16227766e-4f;


// A row-family gate with a layout hint of how often it is open (the cube's
// ground rows and gripper slots 0-1: open; slots 2-3 and joint limits:
// closed).  A lone wave pays ~20 cycles for a taken branch (the instruction
// stream is refetched: profiles/r03a_issue_probe.jsonl, 8- vs 128-instruction
// loop bodies); laying the open blocks out as fall-through took Push from
// 3.18 to 3.14 ms and Reach from 1.47 to 1.44 ms per step at 65 536 envs.
#define PS_GATE(cond, likely) __builtin_expect(!!(cond), (likely))
PS_D float row_viol(float dl, float dinv) { return fmaf(-kResidualAbs, dinv, fabsf(dl)); }
// The solver's running residual max: llvm.maximum (v_maximum3_f32).  With
// fmaxf (llvm.maxnum) the IEEE-mode lowering re-canonicalised the running max
// (v_max x, x, x) at every row: ~30 VALU instructions per Push iteration.  The
// values are finite (the residual's 1/den is clamped, see kResidualAbs), where
// both give the same bits.  The impulse clamps stay fminf(fmaxf()): as
// v_med3_f32 (the same bits too) they made Push 0.25 % slower
// (profiles/r05v_ab.log).
// A NaN row violation (an env whose state is already non-finite) keeps res at
// NaN, so that lane never meets `res <= 0` and runs the 50-iteration cap; it is
// masked like any other lane, so no other env's rows or bits change, and the
// NaN/Inf guard flags (and optionally resets) the env after the step
// (test_gpu_contacts.py::test_nonfinite_guard_flags_and_resets: every other
// env equal bit for bit to a run without the corrupted one).
PS_D float res_max(float a, float b) { return __builtin_elementwise_maximum(a, b); }
PS_D float clamp_impulse(float x, float lo, float hi) { return fminf(fmaxf(x, lo), hi); }
PS_D float joint_viol(float dl, float den) { return fmaf(fabsf(dl), den, -kResidualAbs); }

// The warm start's contact cache (state rows PS_F_WG0.. of this env, see
// include/pandasim.h): read at contact generation, written after the solve.
// Addresses are re-derived at each access from wave-uniform values (row base,
// stride, the wave's first env) and the lane id (v_mbcnt), so no per-lane
// pointer or index stays live through the solve.  The step kernels run one
// 64-lane wave per workgroup with G lanes per env, so env = (step_block * 64
// + lane) / G.  With G > 1 every lane of a group computes the same values;
// lanes of a group past the batch end (live = false) compute a copy of the
// last env and store nothing.
// Scenes with at most one object (IN_LDS) use rows WG0..WG0ID and WR..WRID
// only, held in LDS slots 0-4 and 5-9 over the substeps (cache_to_lds,
// cache_from_lds); Stack reads and writes the state rows directly.
template <int G, int NOBJ>
struct WarmCache {
    static constexpr bool IN_LDS = NOBJ <= 1;
    float *base;  // &f[PS_F_WG0 * stride]
    int64_t stride;
    bool live;
    MJStore lds;
    PS_D static int slot(int row) { return row < PS_F_WG1 ? row - PS_F_WG0 : 5 + (row - PS_F_WR); }
    PS_D float &at(int row) const {
        // a 32-bit byte offset from a wave-uniform row base (ps_create caps
        // the batch at PS_MAX_ENVS), as StateView
        const uint32_t e = (uint32_t)(((uint64_t)step_block<G>() * 64 + __lane_id()) / G) * 4u;
        return *(float *)((char *)(base + (int64_t)(row - PS_F_WG0) * stride) + e);
    }
    PS_D float load(int row) const {
        if constexpr (IN_LDS) return lds.cache(slot(row));
        else return at(row);
    }
    PS_D void store(int row, float v) const {
        if constexpr (IN_LDS) lds.cache(slot(row)) = v;
        else if (G == 1 || live) at(row) = v;
    }
    // once per control step, around the substep loop
    PS_D void to_lds() const {
        if constexpr (IN_LDS) {
#pragma unroll
            for (int k = 0; k < 5; k++) {
                lds.cache(k) = at(PS_F_WG0 + k);
                lds.cache(5 + k) = at(PS_F_WR + k);
            }
        }
    }
    PS_D void from_lds() const {
        if constexpr (IN_LDS) {
            if (G == 1 || live) {
#pragma unroll
                for (int k = 0; k < 5; k++) {
                    at(PS_F_WG0 + k) = lds.cache(k);
                    at(PS_F_WR + k) = lds.cache(5 + k);
                }
            }
        }
    }
};
// slot k's id (1 + feature, 0 = empty) of a packed id row
PS_D unsigned cache_id(unsigned pack, int k) { return (pack >> (5 * k)) & 31u; }
// normal impulse cached for `id` among the 4 slots (0 when absent)
PS_D float cache_lookup(const float lam[4], unsigned pack, unsigned id) {
    float l = 0.0f;
#pragma unroll
    for (int k = 0; k < 4; k++) l = cache_id(pack, k) == id ? lam[k] : l;
    return l;
}

// Friction-cone projection factor (resolveConeFrictionConstraintRows): lim/|f|
// when |f|^2 = m2 exceeds lim^2, else 1.  Raw v_rsq_f32: rsqrtf's denormal
// rescaling costs three instructions per cone row; m2 is clamped to FLT_MIN
// instead, so a denormal m2 cannot produce inf (and 0 * inf) there.
// lim = mu * lam_n takes the normal impulse as it is: every normal row clamps
// it to [0, upper] (and warm starts are 0.85 x a clamped impulse), so the
// oracle's max(lam_n, 0) is the identity here and only cost a v_max (plus a
// canonicalising one) per cone.
PS_D float cone_scale(float m2, float lim) {
    return m2 > lim * lim ? lim * __builtin_amdgcn_rsqf(fmaxf(m2, 1.17549435e-38f)) : 1.0f;
}

// Projected Gauss-Seidel with G = 16 or 8 lanes per env (the small-batch
// step kernels): every lane of a group ran the same setup, and
// the 15 velocity DoFs (robot 0-8, then the object's omega 9-11 and v 12-14)
// are dealt to the lanes: lane e owns DoFs e + k G for k < 16 / G (G = 16: one
// DoF per lane; G = 8: two) with their slices of every row's J and M^-1 J^T.
// A row is then one product per owned DoF, a group sum (group_sum: the same
// bits in every lane, so every lane computes the same impulse), the clamp,
// and one FMA per owned DoF -- about 11 instructions for a row the one-lane
// solver spends 20-60 on.  Row order, gates, bounds and the stopping rule are
// the one-lane solver's.  Returns the full velocity change in every lane.
template <int G>
PS_D float group_sum(float x) {
    if constexpr (G == 16) return group16_sum(x);
    else if constexpr (G == 8) return group8_sum(x);
    else return group2_sum(x);
}
template <int G, int K>
PS_D float group_bcast(float x) {
    if constexpr (G == 16) return group16_bcast<K>(x);
    else if constexpr (G == 8) return group8_bcast<K>(x);
    else return group2_bcast<K>(x);
}
template <int NOBJ, int SHAPE, bool STD_MOTORS, int G>
PS_D void group_pgs(const Motors &mt, const float Mi[45], const MJStore &lds, unsigned gate_lim, unsigned lim_up,
                    unsigned lim_on, unsigned gate_gnd, unsigned gate_robot, const float dinvj[9],
                    const float lim_rhs[9], float lim_lam[9], const float mot_rhs[9], float mot_lam[9],
                    GroundContact gc[NG], RobotContact rc[NR], const BodyDyn<SHAPE> &od, float gmu, float dv[9],
                    V3 &dw, V3 &dvl PS_PROF_COUNT_PARAM PS_DUMP_PARAM) {
    // (G = 2: the PS_EXPERIMENT_G2 kernels, eight DoF slots per lane)
    static_assert((G == 16 || G == 8 || G == 2) && NOBJ <= 1, "groups of 16, 8 or 2 lanes hold 9 robot + 6 object DoFs");
#ifdef PS_DEBUG_ROW_DUMP
    int dk = 0;
    auto rec = [&](float x) {
        if (dump && dk < PS_DUMP_ROWS) dump[dk] = x;
        dk++;
    };
#pragma unroll
    for (int d = 0; d < 9; d++) { rec(mot_rhs[d]); rec(dinvj[d]); rec(lim_rhs[d]); }
#pragma unroll
    for (int c = 0; c < NG; c++)
#pragma unroll
        for (int j = 0; j < 3; j++) { rec(gc[c].rhs[j]); rec(gc[c].dinv[j]); }
#pragma unroll
    for (int c = 0; c < NR; c++)
#pragma unroll
        for (int j = 0; j < 3; j++) { rec(rc[c].rhs[j]); rec(rc[c].dinv[j]); rec(rc[c].lam[j]); }
    rec(__builtin_bit_cast(float, gate_lim | (gate_gnd << 9) | (gate_robot << 13)));
    bool dump_on = dump != nullptr;
#define PS_REC(x) do { if (dump_on) rec(x); } while (0)
#else
#define PS_REC(x) do {} while (0)
#endif
    constexpr int K = 16 / G;  // DoFs per lane
    const int e = (int)(__lane_id() & (unsigned)(G - 1));
    // lane e's slices: rows e + k G of M^-1 (joint rows), object-only rows, robot rows
    float mrow[K][9], midg[9];
#pragma unroll
    for (int d = 0; d < 9; d++) {
#pragma unroll
        for (int k = 0; k < K; k++) {
            float v = 0.0f;
#pragma unroll
            for (int r = 0; r < 9; r++) v = e + k * G == r ? Mi[sidx(r, d)] : v;
            mrow[k][d] = v;
        }
        midg[d] = Mi[sidx(d, d)];
    }
    auto oslice = [&](int k, V3 a, V3 l) {
        const int dof = e + k * G;
        float v = 0.0f;
        v = dof == 9 ? a.x : v;
        v = dof == 10 ? a.y : v;
        v = dof == 11 ? a.z : v;
        v = dof == 12 ? l.x : v;
        v = dof == 13 ? l.y : v;
        v = dof == 14 ? l.z : v;
        return v;
    };
    float gJ[NG][3][K], gM[NG][3][K];
#pragma unroll
    for (int c = 0; c < NG; c++)
#pragma unroll
        for (int j = 0; j < 3; j++)
#pragma unroll
            for (int k = 0; k < K; k++) {
                gJ[c][j][k] = gM[c][j][k] = 0.0f;
                if constexpr (NOBJ > 0) {
                    V3 dir = j == 0 ? mk(0, 0, 1) : (j == 1 ? mk(0, -1, 0) : mk(1, 0, 0));
                    V3 rn = cross(gc[c].r, dir);
                    gJ[c][j][k] = oslice(k, rn, dir);
                    gM[c][j][k] = oslice(k, od.inv_inertia(rn), dir * od.inv_m);
                }
            }
    float rJ[NR][3][K], rM[NR][3][K];
    {
        const MJStore W = lds.opaque();
#pragma unroll
        for (int c = 0; c < NR; c++)
#pragma unroll
            for (int j = 0; j < 3; j++)
#pragma unroll
                for (int k = 0; k < K; k++) {
                    const int dof = e + k * G;
                    float v = 0.0f;
#pragma unroll
                    for (int r = 0; r < 9; r++) v = dof == r ? rc[c].J[j][r] : v;
                    float m = (float)W.at(c, j, dof < 9 ? dof : 8);
                    m = dof < 9 ? m : 0.0f;
                    if constexpr (NOBJ > 0) {
                        // the object is body B: -rn, -dir
                        V3 rn = rc[c].rn[j], dir = rc[c].dir[j];
                        v += oslice(k, mk(-rn.x, -rn.y, -rn.z), mk(-dir.x, -dir.y, -dir.z));
                        m += oslice(k, od.inv_inertia(mk(-rn.x, -rn.y, -rn.z)), dir * -od.inv_m);
                    }
                    rJ[c][j][k] = v;
                    rM[c][j][k] = m;
                }
    }
    float dvm[K];  // this lane's velocity changes (DoFs e + k G)
#pragma unroll
    for (int k = 0; k < K; k++) dvm[k] = 0.0f;
    // KL: the first slot a row's J can be non-zero in.  The object's DoFs
    // (9-14) sit in slots k >= 9 / G, so an object-only row (ground contacts)
    // skips the slots below at compile time (IEEE 0 * x is not folded)
    constexpr int KOBJ = 9 / G;
    using KAll = std::integral_constant<int, 0>;
    using KObj = std::integral_constant<int, KOBJ>;
    auto prod = [&](auto KL, const float J[K]) {
        constexpr int k0 = decltype(KL)::value;
        float p = J[k0] * dvm[k0];
#pragma unroll
        for (int k = k0 + 1; k < K; k++) p = fmaf(J[k], dvm[k], p);
        return p;
    };
    // G = 8: a lane's two DoFs updated by one v_pk_fma_f32 (the same bits)
    auto apply2 = [&](float m0, float m1, float dl) {
        const f32x2 x = __builtin_elementwise_fma((f32x2){m0, m1}, (f32x2){dl, dl}, (f32x2){dvm[0], dvm[K - 1]});
        dvm[0] = x.x;
        dvm[K - 1] = x.y;
    };
    auto apply = [&](auto KL, const float M[K], float dl) {
        if constexpr (K == 2 && decltype(KL)::value == 0) {
            apply2(M[0], M[1], dl);
        } else {
#pragma unroll
            for (int k = decltype(KL)::value; k < K; k++) dvm[k] = fmaf(M[k], dl, dvm[k]);
        }
    };
    // warm start (see the one-lane solver)
#pragma unroll
    for (int c = 0; c < NG; c++)
        if (NOBJ > 0 && (gate_gnd & (1u << c))) apply(KObj{}, gM[c][0], gc[c].lam[0]);
#pragma unroll
    for (int c = 0; c < NR; c++)
        if (gate_robot & (1u << c)) apply(KAll{}, rM[c][0], rc[c].lam[0]);

    float res = 0.0f;
    // a joint row's J is e_d: its product is the velocity change of DoF d,
    // held by lane d % G in slot d / G: one broadcast instead of a sum
    auto jrow = [&](auto DD, float sgn, float rhs, float &lam, float lo, float hi) {
        constexpr int d = decltype(DD)::value;
        float s = group_bcast<G, d % G>(dvm[d / G]);
        float dl = rhs - dinvj[d] * (sgn * s);
        float nl = clamp_impulse(lam + dl, lo, hi);
        dl = nl - lam;
        lam = nl;
        PS_REC(dl);
        if constexpr (K == 2) {
            apply2(mrow[0][d], mrow[K - 1][d], sgn * dl);
        } else {
#pragma unroll
            for (int k = 0; k < K; k++) dvm[k] = fmaf(mrow[k][d], sgn * dl, dvm[k]);
        }
        res = res_max(res, joint_viol(dl, midg[d]));
    };
    auto limit_row = [&](auto DD) {
        constexpr int d = decltype(DD)::value;
        if (gate_lim & (1u << d)) {
            float sgn = (lim_up >> d) & 1u ? -1.0f : 1.0f;
            float hi = (lim_on >> d) & 1u ? (float)PM_LIMIT_MAX_IMPULSE : 0.0f;
            jrow(DD, sgn, lim_rhs[d], lim_lam[d], 0.0f, hi);
        }
    };
    auto motor_row = [&](auto DD) {
        constexpr int d = decltype(DD)::value;
        float imp = STD_MOTORS ? (float)(joint_force(d) * PM_TIMESTEP) : mt.imp[d];
        jrow(DD, 1.0f, mot_rhs[d], mot_lam[d], -imp, imp);
    };
    // rows d = 8..0 and 0..8 with compile-time d
    auto down = [&](auto row) { static_for<0, 9>([&](auto I) { row(std::integral_constant<int, 8 - decltype(I)::value>{}); }); };
    auto up = [&](auto row) { static_for<0, 9>([&](auto I) { row(I); }); };
    auto normal = [&](auto KL, const float Jm[K], const float Mm[K], float rhs, float dinv, float &lam) {
        float s = group_sum<G>(prod(KL, Jm));
        float dl = rhs - dinv * s;
        float nl = clamp_impulse(lam + dl, 0.0f, (float)PM_CONTACT_UPPER);
        dl = nl - lam;
        lam = nl;
        PS_REC(dl);
        apply(KL, Mm, dl);
        res = res_max(res, row_viol(dl, dinv));
    };
    auto cone = [&](auto KL, const float J[3][K], const float M[3][K], const float rhs[3], const float dinv[3],
                    float lam[3], float mu) {
        // G = 8: the two rows side by side as f32x2 (v_pk_*) around their
        // group sums: the scalar rows' operations, fused where they were
        // fused, so the same bits (x = row 1, y = row 2).  G = 16 keeps the
        // scalar rows: fewer instructions with the pairs, but 0.8 % slower at
        // C2 (profiles/r05aa_ab.log)
        float dla, dlb;
        if constexpr (K == 1) {
            const float sa = group_sum<G>(prod(KL, J[1])), sb = group_sum<G>(prod(KL, J[2]));
            dla = rhs[1] - dinv[1] * sa;
            dlb = rhs[2] - dinv[2] * sb;
            float a = lam[1] + dla, b = lam[2] + dlb;
            const float lim = mu * lam[0];  // lam[0] >= 0: the normal row's clamp
            const float sc = cone_scale(a * a + b * b, lim);
            a *= sc;
            b *= sc;
            dla = a - lam[1];
            dlb = b - lam[2];
            lam[1] = a;
            lam[2] = b;
        } else {
#pragma clang fp contract(off)
            constexpr int k0 = decltype(KL)::value;
            f32x2 p = (f32x2){J[1][k0], J[2][k0]} * (f32x2){dvm[k0], dvm[k0]};
#pragma unroll
            for (int k = k0 + 1; k < K; k++)
                p = __builtin_elementwise_fma((f32x2){J[1][k], J[2][k]}, (f32x2){dvm[k], dvm[k]}, p);
            const f32x2 s2 = {group_sum<G>(p.x), group_sum<G>(p.y)};
            const f32x2 lam12 = {lam[1], lam[2]};
            const f32x2 ab = lam12 + __builtin_elementwise_fma(-(f32x2){dinv[1], dinv[2]}, s2, (f32x2){rhs[1], rhs[2]});
            const float lim = mu * lam[0];  // lam[0] >= 0: the normal row's clamp
            const float sc = cone_scale(fmaf(ab.x, ab.x, ab.y * ab.y), lim);
            const f32x2 dl2 = __builtin_elementwise_fma(ab, (f32x2){sc, sc}, -lam12);
            const f32x2 nl2 = ab * (f32x2){sc, sc};
            lam[1] = nl2.x;
            lam[2] = nl2.y;
            dla = dl2.x;
            dlb = dl2.y;
        }
        PS_REC(dla);
        PS_REC(dlb);
        if constexpr (K == 2 && decltype(KL)::value == 0) {
            apply2(M[1][0], M[1][1], dla);
            apply2(M[2][0], M[2][1], dlb);
        } else {
#pragma unroll
            for (int k = decltype(KL)::value; k < K; k++) dvm[k] = fmaf(M[2][k], dlb, fmaf(M[1][k], dla, dvm[k]));
        }
        res = res_max(res, res_max(row_viol(dla, dinv[1]), row_viol(dlb, dinv[2])));
    };
    // the object's ground normals touch only object DoFs: they commute with
    // the joint rows (robot DoFs only), so they run in the motor rows' block,
    // ungated (a slot a lane lacks is an all-zero no-op), where their
    // dependent chains interleave with the motor rows'
    auto ground_normals = [&]() {
        if constexpr (NOBJ > 0) {
#pragma unroll
            for (int c = 0; c < NG; c++) normal(KObj{}, gJ[c][0], gM[c][0], gc[c].rhs[0], gc[c].dinv[0], gc[c].lam[0]);
        }
    };
    auto contacts = [&]() {
#pragma unroll
        for (int c = 0; c < NR; c++)
            if (gate_robot & (1u << c)) normal(KAll{}, rJ[c][0], rM[c][0], rc[c].rhs[0], rc[c].dinv[0], rc[c].lam[0]);
#pragma unroll
        for (int c = 0; c < NG; c++)
            if (NOBJ > 0 && (gate_gnd & (1u << c))) cone(KObj{}, gJ[c], gM[c], gc[c].rhs, gc[c].dinv, gc[c].lam, gmu);
#pragma unroll
        for (int c = 0; c < NR; c++)
            if (gate_robot & (1u << c)) cone(KAll{}, rJ[c], rM[c], rc[c].rhs, rc[c].dinv, rc[c].lam, rc[c].mu);
    };
    // (the gates stay scalar tests inside the loop, as in the one-lane
    // solver's PS_REGATE)
    auto regate = [&]() { asm volatile("" : "+s"(gate_lim), "+s"(gate_gnd), "+s"(gate_robot)); };
    for (int it = 0; it < PM_SOLVER_ITERATIONS; it += 2) {
#ifdef PS_PROFILE_PHASES
        prof_it++;
#endif
        res = 0.0f;
        regate();
        down(motor_row);
        ground_normals();
        if (gate_lim != 0u) down(limit_row);
        contacts();
        if (res <= 0.0f) break;
#ifdef PS_PROFILE_PHASES
        prof_it++;
#endif
        res = 0.0f;
        regate();
        if (gate_lim != 0u) up(limit_row);
        up(motor_row);
        ground_normals();
        contacts();
#ifdef PS_DEBUG_ROW_DUMP
        rec(res);
        dump_on = false;
#endif
        if (res <= 0.0f) break;
    }
#undef PS_REC
    // every lane of the group gets the whole velocity change
    static_for<0, 9>([&](auto DD) {
        constexpr int d = decltype(DD)::value;
        dv[d] = __shfl(dvm[d / G], d % G, G);
    });
    if constexpr (NOBJ > 0) {
        float o[6];
        static_for<0, 6>([&](auto JJ) {
            constexpr int dof = 9 + decltype(JJ)::value;
            o[dof - 9] = __shfl(dvm[dof / G], dof % G, G);
        });
        dw = mk(o[0], o[1], o[2]);
        dvl = mk(o[3], o[4], o[5]);
    }
}

// Gripper contact candidates (oracle gen_contacts 3-4): per object, then the
// ground, the gripper boxes (PM_BOX_CONTACTS points each) and then the wrist
// sphere; the first NR fill the slots.  Cache ids 1 + (proxy * 3 + target) * 2
// + point.  Each slot's record (RobotCand, 14 floats) goes to LDS at the end of
// the M^-1 J^T area, which the row setup overwrites only after it has read the
// slot (slot s's rows are written to floats [27 s, 27 s + 27), its record sits
// at [52 + 14 s, 66 + 14 s)).  Returns the number of slots used.
struct RobotCand {
    V3 pA, pB, n;
    float dist, mu;
    int link;
    int obj;  // -1: ground
    int id;   // cache id: 1 + (proxy * 3 + target) * 2 + point (target 2: the ground)
    static constexpr int FLOATS = 14, OFFSET = NR * 27 - NR * 14;
    PS_D void store(const MJStore &L, int s) const {
        const float v[FLOATS] = {pA.x, pA.y, pA.z, pB.x, pB.y, pB.z, n.x, n.y, n.z, dist, mu,
                                 (float)link, (float)obj, (float)id};
#pragma unroll
        for (int k = 0; k < FLOATS; k++) {
#ifdef PS_EXPERIMENT_TWO_WAVES
            L.gxd(OFFSET + s * FLOATS + k) = v[k];
#else
            L.base[(OFFSET + s * FLOATS + k) * L.stride] = v[k];
#endif
        }
    }
    PS_D static RobotCand load(const MJStore &L, int s) {
        float v[FLOATS];
#pragma unroll
        for (int k = 0; k < FLOATS; k++) {
#ifdef PS_EXPERIMENT_TWO_WAVES
            v[k] = L.gxd(OFFSET + s * FLOATS + k);
#else
            v[k] = L.base[(OFFSET + s * FLOATS + k) * L.stride];
#endif
        }
        return RobotCand{mk(v[0], v[1], v[2]), mk(v[3], v[4], v[5]), mk(v[6], v[7], v[8]), v[9], v[10],
                         (int)v[11], (int)v[12], (int)v[13]};
    }
};
static_assert(RobotCand::OFFSET + NR * RobotCand::FLOATS <= NR * 27, "candidate records inside the M^-1 J^T area");

// position of the j-th (from 0) set bit of m (j < popcount(m)), branch-free
PS_D int nth_set_bit(uint64_t m, int j) {
    int pos = 0;
#pragma unroll
    for (int w = 32; w >= 1; w >>= 1) {
        const uint64_t low = m & ((1ull << w) - 1ull);
        const int c = __builtin_popcountll(low);
        const bool up = j >= c;
        j = up ? j - c : j;
        pos += up ? w : 0;
        m = up ? (m >> w) : low;
    }
    return pos;
}

// Candidate work lists.  The bounding tests pass for few lanes of a wave (Push,
// 65 536 envs: 2.2 lanes of 64 per box-object test that passes anywhere, 14 per
// box-ground one; profiles/r04f_phase_push.log), and run per lane the pair's
// candidate block cost the whole wave a block per box.  Instead the (env, box)
// pairs that pass are numbered box-major across the wave (ballot + popcount),
// the owners park their geometry in their own LDS column, and active lane k
// evaluates pair k of the round -- one block per round for the wave, not one per
// box -- and leaves its picks in its column, which the owners read back in box
// order (the slot order of the per-lane version: the same values, bit for bit).
// Scratch: floats [0, 51) of each column, below the RobotCand records.
constexpr int CW_IN = 0;    // owner: hR (9), box centres (3 x 3), object position (3), rotation (9)
constexpr int CW_OUT = 30;  // worker: pick 0 (pA, pB, n, dist), pick 1, count
constexpr int CW_OUT_FLOATS = 21;
// the work lists' per-lane output rows are one wave wide: row q of worker lane
// c at cwo0[q * CW_LANES + c] (the step kernels' kBlock, asserted equal in
// ps_env.h: a workgroup of another width would overwrite other waves' rows)
constexpr int CW_LANES = 64;
static_assert(CW_OUT + CW_OUT_FLOATS <= RobotCand::OFFSET, "work-list scratch below the candidate records");

// The group kernels (G > 1) keep one LDS column per env, shared by the
// group's lanes: every lane of a group computes the same values, so the
// M^-1 J^T rows, candidate records, stash and cache are written with the same
// bits by each (round 5; round 3's attempt at this changed the bits, most
// likely through the FMA-contracted group sums of §12.8, since fixed).  The
// work lists' outputs, which differ per lane, keep a per-lane area.  LDS per
// workgroup 40.4 KB -> 7.9 KB (G = 16) / 10.4 KB (G = 8); C3 and C4 0.6 %
// faster.
template <int G>
constexpr bool shared_lds() { return G > 1; }

template <int NOBJ, int SHAPE, int G>
PS_D int robot_candidates(const Scene &sc, const Geo &geo, const Body *bd, const M3 *oR, const MJStore &lds PS_PROF_PARAM) {
    int nr = 0;
    auto offer = [&](const RobotCand &c) {
        c.store(lds, nr);
        nr++;
    };
    constexpr SphereDef ws = wrist_def();
    constexpr int NBX = PM_NUM_BOXES;
    const uint32_t lane = __lane_id();
    const uint64_t act = __ballot(true);  // G == 1: lanes past the batch end have returned
    const int nact = __builtin_popcountll(act);
    const int rank = __builtin_popcountll(act & ((1ull << lane) - 1ull));
    // G > 1: every lane of a group holds the same env; its first lane owns the pairs
    const uint32_t leader = lane & ~(uint32_t)(G - 1);
    const uint64_t below = (1ull << leader) - 1ull;
    constexpr bool SHARED = shared_lds<G>();
    // column 0 of the wave's LDS block; lane c's column (its env's when shared)
    lds_float *const col0 = lds.base - (SHARED ? lane / G : lane);
    auto at = [&](int k, int c) -> lds_float & { return col0[k * lds.stride + (SHARED ? c / G : c)]; };
    // worker lane c's output row q (stride CW_LANES = kBlock)
    lds_float *const cwo0 = lds.cwo - lane;
    auto wout = [&](int q, int c) -> lds_float & { return cwo0[q * CW_LANES + c]; };
    static_for<0, NOBJ + 1>([&](auto TT) {
        constexpr int TGT = decltype(TT)::value == NOBJ ? 2 : decltype(TT)::value;
        constexpr bool GROUND = TGT == 2;
        // a conservative bounding test per box first (no candidate of a pair
        // that fails it is within the margin, so the picks are unchanged)
        bool nearb[NBX];
        uint64_t m[NBX];
        int pre[NBX + 1];
        pre[0] = 0;
        static_for<0, NBX>([&](auto BB) {
            constexpr int B = decltype(BB)::value;
            constexpr BoxDef bx = box_def(B);
            const V3 xh = mk((float)bx.h[0], (float)bx.h[1], (float)bx.h[2]);
            const V3 xc = geo.bc[B];
            if constexpr (GROUND) {
                const V3 ea = col(geo.hR, 0) * xh.x, eb = col(geo.hR, 1) * xh.y, ec = col(geo.hR, 2) * xh.z;
                const float low = xc.z - (fabsf(ea.z) + fabsf(eb.z) + fabsf(ec.z));
                nearb[B] = low < (float)PM_TABLE_TOP + (float)PM_CONTACT_MARGIN_ROBOT;  // the highest ground
            } else {
                // the object's centre against the box: its distance to the box
                // beyond the object's bounding radius (+ margin) means no
                // candidate can be within the margin (a sphere around the
                // object: |half| bounds a box and, with half = (r, r, h), a
                // cylinder)
                const V3 l = tmul(geo.hR, bd[TGT].pos - xc);
                const V3 ex = mk(fmaxf(fabsf(l.x) - xh.x, 0.0f), fmaxf(fabsf(l.y) - xh.y, 0.0f), fmaxf(fabsf(l.z) - xh.z, 0.0f));
                const float robj = sqrtf(dot(sc.half, sc.half)) + (float)PM_CONTACT_MARGIN_ROBOT;
                nearb[B] = dot(ex, ex) < robj * robj;
            }
            m[B] = __ballot(nearb[B] && lane == leader);
            pre[B + 1] = pre[B] + __builtin_popcountll(m[B]);
#ifdef PS_PROFILE_PHASES
            pt.acc[GROUND ? 22 : 20] += __builtin_popcountll(m[B]);
            pt.acc[GROUND ? 23 : 21] += m[B] != 0;
#endif
        });
        const int total = pre[NBX];
        if (total > 0) {
            // the owner's geometry, in its own column
#pragma unroll
            for (int k = 0; k < 9; k++) lds.base[(CW_IN + k) * lds.stride] = geo.hR.m[k];
#pragma unroll
            for (int b = 0; b < NBX; b++) {
                lds.base[(CW_IN + 9 + 3 * b) * lds.stride] = geo.bc[b].x;
                lds.base[(CW_IN + 10 + 3 * b) * lds.stride] = geo.bc[b].y;
                lds.base[(CW_IN + 11 + 3 * b) * lds.stride] = geo.bc[b].z;
            }
            if constexpr (!GROUND) {
                lds.base[(CW_IN + 18) * lds.stride] = bd[TGT].pos.x;
                lds.base[(CW_IN + 19) * lds.stride] = bd[TGT].pos.y;
                lds.base[(CW_IN + 20) * lds.stride] = bd[TGT].pos.z;
#pragma unroll
                for (int k = 0; k < 9; k++) lds.base[(CW_IN + 21 + k) * lds.stride] = oR[TGT].m[k];
            }
            for (int r = 0; r < total; r += nact) {
                __syncthreads();
                const int k = r + rank;
                if (k < total) {
                    int B = 0;
#pragma unroll
                    for (int b = 1; b < NBX; b++) B = k >= pre[b] ? b : B;
                    uint64_t mb = m[0];
                    int pb = 0;
#pragma unroll
                    for (int b = 1; b < NBX; b++) {
                        mb = B == b ? m[b] : mb;
                        pb = B == b ? pre[b] : pb;
                    }
                    const int own = nth_set_bit(mb, k - pb);
                    M3 hR;
#pragma unroll
                    for (int q = 0; q < 9; q++) hR.m[q] = at(CW_IN + q, own);
                    // (selected per component: selects of whole vectors went
                    // through a stack array)
                    const int cb = CW_IN + 9 + 3 * B;
                    const V3 xc = mk(at(cb, own), at(cb + 1, own), at(cb + 2, own));
                    float hx = (float)box_def(0).h[0], hy = (float)box_def(0).h[1], hz = (float)box_def(0).h[2];
#pragma unroll
                    for (int b = 1; b < NBX; b++) {
                        hx = B == b ? (float)box_def(b).h[0] : hx;
                        hy = B == b ? (float)box_def(b).h[1] : hy;
                        hz = B == b ? (float)box_def(b).h[2] : hz;
                    }
                    const V3 xh = mk(hx, hy, hz);
                    // the pick's skew direction (PM_PICK_SKEW, box frame), world
                    const V3 w = mul(hR, mk((float)PM_PICK_SKEW_X, (float)PM_PICK_SKEW_Y, (float)PM_PICK_SKEW_Z));
                    RCand c0, c1;
                    int ns;
                    if constexpr (GROUND) {
                        ns = pick_two<PM_BOX_GROUND_CONTACTS>([&](auto &&f) { box_ground_visit(sc, xc, hR, xh, f); }, xc, w,
                                                              c0, c1);
                    } else {
                        const V3 yc = mk(at(CW_IN + 18, own), at(CW_IN + 19, own), at(CW_IN + 20, own));
                        M3 yR;
#pragma unroll
                        for (int q = 0; q < 9; q++) yR.m[q] = at(CW_IN + 21 + q, own);
                        if constexpr (SHAPE == SHAPE_CYL) {
                            const BoxCyl bcy(sc, xc, hR, xh, yc, yR);
                            ns = bcy.pick(sc, xc, w, c0, c1);
                        } else {
                            const BoxCube bcu(xc, hR, xh, yc, yR, sc.half);
                            ns = bcu.pick(xc, w, c0, c1);
                        }
                    }
                    const float out[21] = {c0.pA.x, c0.pA.y, c0.pA.z, c0.pB.x, c0.pB.y, c0.pB.z, c0.n.x, c0.n.y, c0.n.z,
                                           c0.dist, c1.pA.x, c1.pA.y, c1.pA.z, c1.pB.x, c1.pB.y, c1.pB.z, c1.n.x, c1.n.y,
                                           c1.n.z, c1.dist, (float)ns};
                    const int nout = GROUND && PM_BOX_GROUND_CONTACTS < 2 ? 10 : 20;
#pragma unroll
                    for (int q = 0; q < 20; q++)
                        if (q < nout) lds.cwo[q * CW_LANES] = out[q];
                    lds.cwo[20 * CW_LANES] = out[20];
                }
                __syncthreads();
                // the owners take their pairs of this round, in box order
                static_for<0, NBX>([&](auto BB) {
                    constexpr int B = decltype(BB)::value;
                    constexpr BoxDef bx = box_def(B);
                    const int idx = pre[B] + __builtin_popcountll(m[B] & below) - r;
                    if (nearb[B] && idx >= 0 && idx < nact) {
                        const int wl = nth_set_bit(act, idx);
                        const int ns = (int)wout(20, wl);
                        const float mu = (float)bx.mu * (GROUND ? (float)PM_DEFAULT_FRICTION : sc.fric);
                        const int obj = GROUND ? -1 : TGT;
#pragma unroll
                        for (int c = 0; c < 2; c++) {
                            if (nr < NR && ns > c) {
                                const int o = 10 * c;
                                offer(RobotCand{mk(wout(o, wl), wout(o + 1, wl), wout(o + 2, wl)),
                                                mk(wout(o + 3, wl), wout(o + 4, wl), wout(o + 5, wl)),
                                                mk(wout(o + 6, wl), wout(o + 7, wl), wout(o + 8, wl)), wout(o + 9, wl), mu,
                                                bx.link, obj, 1 + c + (B * 3 + TGT) * 2});
                            }
                        }
                    }
                });
            }
        }
        constexpr int WID = 1 + (PM_NUM_BOXES * 3 + TGT) * 2;
        if constexpr (GROUND) {
            float top;
            if (nr < NR && ground_top(sc, geo.wc.x, geo.wc.y, top)) {
                const float dist = geo.wc.z - (float)ws.r - top;
                if (dist < (float)PM_CONTACT_MARGIN_SPHERE) {
                    const V3 pA = geo.wc - mk(0, 0, (float)ws.r);
                    offer(RobotCand{pA, mk(pA.x, pA.y, top), mk(0, 0, 1), dist, (float)(ws.mu * PM_DEFAULT_FRICTION),
                                    ws.link, -1, WID});
                }
            }
        } else {
            const V3 loc = tmul(oR[TGT], geo.wc - bd[TGT].pos);
            V3 cl, nl;
            const float dist = object_closest<SHAPE>(sc, loc, cl, nl) - (float)ws.r;
            if (nr < NR && dist < (float)PM_CONTACT_MARGIN_SPHERE) {
                const V3 n = mul(oR[TGT], nl);
                offer(RobotCand{geo.wc - n * (float)ws.r, bd[TGT].pos + mul(oR[TGT], cl), n, dist,
                                (float)ws.mu * sc.fric, ws.link, TGT, WID});
            }
        }
    });
    return nr;
}

// STD_MOTORS: the motors are the ones RobotTaskEnv.step sets (POSITION_CONTROL
// on all nine joints with the fixed Panda gains and forces, panda.py:40-56), so
// only the targets are per-env; otherwise every gain comes from `mt`.
// The split-impulse position correction of joint d's limit rows (the joint
// rows' setup in substep, same expressions): a function of q alone, so Stack
// rebuilds it after the solve instead of keeping 9 stash rows per substep.
PS_D float split_of(int d, float qd_) {
    float split = 0.0f;
#pragma unroll
    for (int side = 0; side < 2; side++) {
        const double LO = dof_def(d).lo, HI = dof_def(d).hi;
        const float lo_h = (float)LO, lo_t = (float)(LO - (double)lo_h);
        const float hi_h = (float)HI, hi_t = (float)(HI - (double)hi_h);
        float pen = side ? (hi_h - qd_) + hi_t : (qd_ - lo_h) - lo_t;
        float sgn = side ? -1.0f : 1.0f;
        bool on = pen <= 0.0f;
        bool combined = pen > (float)PM_SPLIT_PENETRATION_THRESHOLD;
        if (on && !combined) split += sgn * (-pen) * (float)PM_SPLIT_LIMIT_ERP;
    }
    return split;
}

template <int NOBJ, int SHAPE, bool STD_MOTORS, int G = 1>
PS_D void substep(const Scene &sc, float q[9], float qd[9], const Motors &mt, Body *bd, const MJStore &lds,
                  const WarmCache<G, NOBJ> &wc PS_PROF_PARAM PS_DUMP_PARAM) {
    static_assert(NOBJ >= 0 && NOBJ <= 2, "objects");
    static_assert(NOBJ < 2 || SHAPE == SHAPE_BOX, "Stack stacks cubes");
    constexpr int NB = NOBJ > 0 ? NOBJ : 1;  // array extents
    constexpr bool ANISO = SHAPE == SHAPE_CYL;
    const float dt = (float)PM_TIMESTEP;
    float Mi[45], hb[9];
    Geo geo;
    // phases are fenced so the scheduler does not interleave them (each one's
    // transient state is large; overlapping them is what spilled to scratch)
    bias_forces(q, qd, hb);
    PS_PHASE(0);
    __builtin_amdgcn_sched_barrier(0);
    {
        Kin k;
        fk(q, k);
        static_for<0, 9>([&](auto D) {
            constexpr int d = decltype(D)::value;
            geo.ax[d] = dof_axis<d>(k);
            if constexpr (d < 7) geo.org[d] = k.f[d].o;
        });
        geo.hR = k.f[8].R;  // links 9 and 10 carry the hand's rotation
        static_for<0, PM_NUM_BOXES>([&](auto BB) {
            constexpr int B = decltype(BB)::value;
            constexpr BoxDef b = box_def(B);
            geo.bc[B] = k.f[b.link].o + mul(k.f[b.link].R, mk((float)b.c[0], (float)b.c[1], (float)b.c[2])) + sc.base;
        });
        {
            constexpr SphereDef w = wrist_def();
            geo.wc = k.f[w.link].o + mul(k.f[w.link].R, mk((float)w.c[0], (float)w.c[1], (float)w.c[2])) + sc.base;
        }
        mass_matrix(k, Mi);
    }
#ifdef PS_PROFILE_PHASES
    // (diagnostic build: M and M^-1 are forced out where their phases end;
    // the product sinks them into the candidate code)
#pragma unroll
    for (int k = 0; k < 45; k++) asm volatile("" ::"v"(Mi[k]));
#endif
    PS_PHASE(1);
    __builtin_amdgcn_sched_barrier(0);
    spd_inverse(Mi);
#ifdef PS_PROFILE_PHASES
#pragma unroll
    for (int k = 0; k < 45; k++) asm volatile("" ::"v"(Mi[k]));
#endif
    PS_PHASE(2);
    __builtin_amdgcn_sched_barrier(0);
    // gripper contact candidates: geometry only, so they are found here, where
    // few registers are live, and wait in LDS (robot_candidates)
    int nr;
    {
        M3 oR[NB];
#pragma unroll
        for (int b = 0; b < NB; b++) oR[b] = NOBJ > 0 ? quat_to_mat(bd[b].quat) : M3{{1, 0, 0, 0, 1, 0, 0, 0, 1}};
        nr = robot_candidates<NOBJ, SHAPE, G>(sc, geo, bd, oR, lds PS_PROF_ARG);
    }
    PS_PHASE(17);
    __builtin_amdgcn_sched_barrier(0);
    // M^-1 for the joint rows stays in registers: re-reading it from LDS in
    // every PGS iteration exposed the LDS latency once per motor row (Push
    // 4.56 -> 3.99 ms, Reach 2.97 -> 1.98 ms per step of 65 536 envs).
    float v1[9];
#pragma unroll
    for (int a = 0; a < 9; a++) {
        float s = 0.0f;
#pragma unroll
        for (int b = 0; b < 9; b++) s -= Mi[sidx(a, b)] * hb[b];
        v1[a] = qd[a] + dt * s;
    }
    // objects: gravity + btMultiBody base damping, plus the gyroscopic torque
    // -w x (I w) for the (anisotropic) cylinder
    V3 cw1[NB], cv1[NB];
    BodyDyn<SHAPE> od[NB];
#pragma unroll
    for (int b = 0; b < NB; b++) {
        cw1[b] = mk(0, 0, 0);
        cv1[b] = mk(0, 0, 0);
    }
#pragma unroll
    for (int b = 0; b < NOBJ; b++) {
        od[b] = body_dyn<SHAPE>(sc, bd[b], b == 0 ? sc.mass : sc.mass2);
        float cl = (float)PM_LINEAR_DAMPING + (float)PM_LINEAR_DAMPING * norm(bd[b].vel);
        float ca = (float)PM_ANGULAR_DAMPING + (float)PM_ANGULAR_DAMPING * norm(bd[b].omg);
        cv1[b] = bd[b].vel + (mk(0, 0, (float)PM_GRAVITY_Z) - bd[b].vel * cl) * dt;
        cw1[b] = bd[b].omg - bd[b].omg * (ca * dt);
        if constexpr (ANISO) {
            V3 I = local_inertia<SHAPE>(sc, b == 0 ? sc.mass : sc.mass2);
            S3 Iw = rotate_diag(od[b].R, I.x, I.y, I.z);
            V3 gyro = od[b].inv_inertia(cross(bd[b].omg, mul(Iw, bd[b].omg)));
            cw1[b] = cw1[b] - gyro * dt;
        }
    }

    // ---- joint-space rows: limits and motors.  A joint can be beyond at most
    // one of its limits, so each joint carries one limit row whose side is a
    // bit of lim_up; rows that are off have bounds [0, 0] and are exact no-ops.
    float dinvj[9];
    float lim_rhs[9], lim_lam[9];
    unsigned lim_on = 0u, lim_up = 0u;
    float split_dq[9];
    float mot_rhs[9], mot_lam[9];
#pragma unroll
    for (int d = 0; d < 9; d++) {
        float den = Mi[sidx(d, d)];
        dinvj[d] = safe_inv(den);
        split_dq[d] = 0.0f;
        lim_rhs[d] = 0.0f;
        lim_lam[d] = 0.0f;
#pragma unroll
        for (int side = 0; side < 2; side++) {
            // the limit as fp32 head + tail (lo = lo_h + lo_t): q - lo_h is
            // exact near the limit, so the row switches where the fp64 limit
            // puts it (a joint pressed onto -3.0718 by its motor sits exactly
            // at fp32(-3.0718) = -3.0717999935, 6.5e-9 inside the double
            // limit: on with the fp32 constant, off in Bullet and the oracle)
            // (folded to constants: the loop is unrolled)
            const double LO = dof_def(d).lo, HI = dof_def(d).hi;
            const float lo_h = (float)LO, lo_t = (float)(LO - (double)lo_h);
            const float hi_h = (float)HI, hi_t = (float)(HI - (double)hi_h);
            float pen = side ? (hi_h - q[d]) + hi_t : (q[d] - lo_h) - lo_t;
            float sgn = side ? -1.0f : 1.0f;
            bool on = pen <= 0.0f;
            float velerr = -sgn * v1[d];
            bool combined = pen > (float)PM_SPLIT_PENETRATION_THRESHOLD;
            float poserr = -pen * (float)PM_ERP * PS_INV_DT;
            if (on) {
                lim_on |= 1u << d;
                lim_up |= side ? 1u << d : 0u;
                lim_rhs[d] = (combined ? poserr + velerr : velerr) * dinvj[d];
                if (!combined) split_dq[d] += sgn * (-pen) * (float)PM_SPLIT_LIMIT_ERP;
            }
        }
        float kp = STD_MOTORS ? (float)PM_MOTOR_KP : mt.kp[d], kd = STD_MOTORS ? (float)PM_MOTOR_KD : mt.kd[d];
        float vel = STD_MOTORS ? 0.0f : mt.vel[d];
        float target = kp * (mt.target[d] - q[d]) * PS_INV_DT + v1[d] + kd * (vel - v1[d]);
        mot_rhs[d] = (target - v1[d]) * dinvj[d];
        mot_lam[d] = 0.0f;
    }

    PS_PHASE(16);
    // ---- contacts (oracle gen_contacts order: ground per object, pairs, gripper)
    GroundContact gc[NB][NG];
    int ng[NB];
#pragma unroll
    for (int b = 0; b < NB; b++) {
        ng[b] = 0;
#pragma unroll
        for (int s = 0; s < NG; s++)
            gc[b][s] = GroundContact{mk(0, 0, 0), {0, 0, 0}, {0, 0, 0}, {0, 0, 0}, 0};
    }
    const float gmu = sc.fric * (float)PM_DEFAULT_FRICTION;
    if constexpr (NOBJ == 2) {
        // unused LDS ground rows must be all-zero no-ops
#pragma unroll
        for (int c = 0; c < 2 * NG; c++)
#pragma unroll
            for (int k = 0; k < LDS_GND_FLOATS; k++) lds.gnd(c, k) = 0.0f;
    }
    const float warm = (float)PM_WARMSTART_FACTOR;
#pragma unroll
    for (int b = 0; b < NOBJ; b++) {
        // the previous substep's ground contacts of this object (ids = 1 +
        // support point, packed 5 bits per slot)
        const int grow = b == 0 ? PS_F_WG0 : PS_F_WG1;
        float plam[NG];
#pragma unroll
        for (int k = 0; k < NG; k++) plam[k] = wc.load(grow + k);
        const unsigned pid = (unsigned)wc.load(grow + NG);
        static_for<0, num_support<SHAPE>()>([&](auto VV) {
            constexpr int V = decltype(VV)::value;
            V3 pw = bd[b].pos + mul(od[b].R, support_point<SHAPE, V>(sc));
            float top;
            if (ng[b] < NG && ground_top(sc, pw.x, pw.y, top)) {
                float dist = pw.z - top;
                if (dist < (float)PM_CONTACT_MARGIN_GROUND) {
                    V3 r = pw - bd[b].pos;
                    // normal (0,0,1), t1 (0,-1,0), t2 (1,0,0)
                    V3 dirs[3] = {mk(0, 0, 1), mk(0, -1, 0), mk(1, 0, 0)};
                    GroundContact g;
                    g.r = r;
#pragma unroll
                    for (int j = 0; j < 3; j++) {
                        V3 rn = cross(r, dirs[j]);
                        V3 w = od[b].inv_inertia(rn);
                        float den = dot(rn, w) + dot(dirs[j], dirs[j]) * od[b].inv_m;
                        g.dinv[j] = NOBJ == 2 ? cube_ground_dinv(r, j, od[b].iI, od[b].inv_m) : safe_inv(den);
                        float rel = dot(rn, cw1[b]) + dot(dirs[j], cv1[b]);
                        g.lam[j] = 0.0f;
                        g.rhs[j] = j == 0 ? normal_rhs(dist, rel, g.dinv[0]) : -rel * g.dinv[j];
                    }
                    g.lam[0] = warm * cache_lookup(plam, pid, V + 1);
                    g.id = V + 1;
                    if (NOBJ == 2) {
                        // Stack: the cubes' read-only ground-row data live in LDS
                        const int at = b * NG + ng[b];
                        lds.gnd(at, 0) = g.r.x; lds.gnd(at, 1) = g.r.y; lds.gnd(at, 2) = g.r.z;
#pragma unroll
                        for (int j = 0; j < 3; j++) lds.gnd(at, 3 + j) = g.rhs[j];
#pragma unroll
                        for (int s = 0; s < NG; s++)
                            if (s == ng[b]) {
                                gc[b][s].lam[0] = g.lam[0];
                                gc[b][s].id = g.id;
                            }
                    } else {
#pragma unroll
                        for (int s = 0; s < NG; s++)
                            if (s == ng[b]) gc[b][s] = g;
                    }
                    ng[b]++;
                }
            }
        });
        // the new ids are packed from the slots after the loop (packing inside
        // it, by a shift of 5 * ng[b], turned the select into compile-time
        // slots into a dynamic index and gc[][] into scratch)
        unsigned nid = 0u;
#pragma unroll
        for (int k = 0; k < NG; k++) nid |= (unsigned)gc[b][k].id << (5 * k);
        wc.store(grow + NG, (float)nid);
    }
    PairContact pc[NP];
    int np = 0;
    if constexpr (NOBJ == 2) {
        PairCand cand[NP];
        np = box_box(sc, bd[0], bd[1], od[0].R, od[1].R, cand);
        // the previous substep's pair contacts: points in object 1's frame,
        // matched by distance (btPersistentManifold::getCacheEntry)
        float pl[NP];
        V3 ppt[NP];
        const int pn = (int)wc.load(PS_F_WPN);
#pragma unroll
        for (int k = 0; k < NP; k++) {
            pl[k] = wc.load(PS_F_WP + k);
            ppt[k] = mk(wc.load(PS_F_WPPT + 3 * k), wc.load(PS_F_WPPT + 3 * k + 1), wc.load(PS_F_WPPT + 3 * k + 2));
        }
        const float pmu = sc.fric * sc.fric;
        (void)pmu;
#pragma unroll
        for (int c = 0; c < NP; c++) {
            PairContact &p = pc[c];
            if (c < np) {
                const PairCand &cd = cand[c];
                int A = cd.a0 ? 0 : 1;
                V3 dirs[3];
                dirs[0] = cd.n;
                plane_space(cd.n, dirs[1], dirs[2]);
                V3 rA = cd.pA - (A == 0 ? bd[0].pos : bd[1].pos), rB = cd.pB - (A == 0 ? bd[1].pos : bd[0].pos);
                p.a0 = cd.a0;
                p.rA = A == 0 ? rA : rB;  // stored by object index: offset from object 0's COM
                p.rB = A == 0 ? rB : rA;  // and from object 1's
#pragma unroll
                for (int j = 0; j < 3; j++) {
                    V3 dj = dirs[j];
                    p.dir[j] = dj;
                    const V3 rnA = cross(rA, dj), rnB = cross(rB, dj);
                    float iIA = A == 0 ? od[0].iI : od[1].iI, iIB = A == 0 ? od[1].iI : od[0].iI;
                    float imA = A == 0 ? od[0].inv_m : od[1].inv_m, imB = A == 0 ? od[1].inv_m : od[0].inv_m;
                    float den = dot(rnA, rnA) * iIA + dot(rnB, rnB) * iIB + dot(dj, dj) * (imA + imB);
                    p.dinv[j] = safe_inv(den);
                    V3 wA = A == 0 ? cw1[0] : cw1[1], vA = A == 0 ? cv1[0] : cv1[1];
                    V3 wB = A == 0 ? cw1[1] : cw1[0], vB = A == 0 ? cv1[1] : cv1[0];
                    float rel = dot(rnA, wA) + dot(dj, vA) - dot(rnB, wB) - dot(dj, vB);
                    p.lam[j] = 0.0f;
                    p.rhs[j] = j == 0 ? normal_rhs(cd.dist, rel, p.dinv[0]) : -rel * p.dinv[j];
                }
                V3 lp = tmul(od[0].R, cd.pB - bd[0].pos);
                float best = (float)(PM_CONTACT_BREAKING_THRESHOLD * PM_CONTACT_BREAKING_THRESHOLD), l0 = 0.0f;
#pragma unroll
                for (int k = 0; k < NP; k++) {
                    V3 d = ppt[k] - lp;
                    float d2 = dot(d, d);
                    bool hit = k < pn && d2 < best;
                    best = hit ? d2 : best;
                    l0 = hit ? pl[k] : l0;
                }
                p.lam[0] = warm * l0;
                wc.store(PS_F_WPPT + 3 * c, lp.x);
                wc.store(PS_F_WPPT + 3 * c + 1, lp.y);
                wc.store(PS_F_WPPT + 3 * c + 2, lp.z);
            } else {
                p.a0 = true;
                p.rA = p.rB = mk(0, 0, 0);
#pragma unroll
                for (int j = 0; j < 3; j++) {
                    p.dir[j] = mk(0, 0, 0);
                    p.rhs[j] = p.lam[j] = p.dinv[j] = 0.0f;
                }
            }
            // the read-only part of the row goes to the global stash
            // (PAIR_FLOATS); the slots this env does not use are not written
            // (the solver reads the zero block for them: MJStore::pair_rows)
            if (c < np) {
#pragma unroll
                for (int j = 0; j < 3; j++) {
                    lds.pair(c, 3 * j + 0) = p.dir[j].x; lds.pair(c, 3 * j + 1) = p.dir[j].y; lds.pair(c, 3 * j + 2) = p.dir[j].z;
                    lds.pair(c, 15 + j) = p.rhs[j];
                    lds.pair(c, 18 + j) = p.dinv[j];
                }
                lds.pair(c, 9) = p.rA.x; lds.pair(c, 10) = p.rA.y; lds.pair(c, 11) = p.rA.z;
                lds.pair(c, 12) = p.rB.x; lds.pair(c, 13) = p.rB.y; lds.pair(c, 14) = p.rB.z;
            }
        }
        wc.store(PS_F_WPN, (float)np);
    }
    RobotContact rc[NR];
    {
        PS_PHASE(18);
        // 2) rows of each used slot: J (registers), M^-1 J^T (LDS), rhs, bounds;
        //    the normal starts from the cached impulse of the same feature
        float prl[NR];
#pragma unroll
        for (int k = 0; k < NR; k++) prl[k] = wc.load(PS_F_WR + k);
        const unsigned prid = (unsigned)wc.load(PS_F_WRID);
        unsigned nrid = 0u;
#pragma unroll
        for (int sl = 0; sl < NR; sl++) {
            RobotContact &c = rc[sl];
            if (sl < nr) {
                const RobotCand cd = RobotCand::load(lds, sl);
                V3 dirs[3];
                dirs[0] = cd.n;
                plane_space(cd.n, dirs[1], dirs[2]);
                c.mu = cd.mu;
                c.o1 = cd.obj == 1;
                bool on_obj = NOBJ > 0 && cd.obj >= 0;
                V3 p = cd.pA - sc.base;
                V3 opos = NOBJ == 2 && cd.obj == 1 ? bd[NB - 1].pos : bd[0].pos;
                V3 rB = cd.pB - opos;
                V3 ow = NOBJ == 2 && cd.obj == 1 ? cw1[NB - 1] : cw1[0];
                V3 ov = NOBJ == 2 && cd.obj == 1 ? cv1[NB - 1] : cv1[0];
                float oim = NOBJ == 2 && cd.obj == 1 ? od[NB - 1].inv_m : od[0].inv_m;
#pragma unroll
                for (int j = 0; j < 3; j++) {
                    V3 dj = dirs[j];
#pragma unroll
                    for (int D = 0; D < 7; D++) c.J[j][D] = dot(geo.ax[D], cross(p - geo.org[D], dj));
                    c.J[j][7] = cd.link == 9 ? dot(geo.ax[7], dj) : 0.0f;
                    c.J[j][8] = cd.link == 10 ? dot(geo.ax[8], dj) : 0.0f;
                    float den = 0.0f;
#pragma unroll
                    for (int a = 0; a < 9; a++) {
                        float s = 0.0f;
#pragma unroll
                        for (int b = 0; b < 9; b++) s += Mi[sidx(a, b)] * c.J[j][b];
                        lds.at(sl, j, a) = NOBJ == 2 ? c.J[j][a] : s;  // Stack: J (M^-1 J^T rebuilt in the loop)
                        if constexpr (NOBJ == 2)
                            if (j == 0) lds.grip(sl, a) = s;
                        den += c.J[j][a] * s;
                    }
                    float rel = jrow_dot(c.J[j], v1);
                    c.rn[j] = on_obj ? cross(rB, dj) : mk(0, 0, 0);
                    c.dir[j] = on_obj ? dj : mk(0, 0, 0);  // object side only
                    if constexpr (NOBJ > 0) {
                        V3 w = ANISO ? od[0].inv_inertia(c.rn[j])
                                     : c.rn[j] * (NOBJ == 2 && cd.obj == 1 ? od[NB - 1].iI : od[0].iI);
                        if (on_obj) {
                            den += dot(c.rn[j], w) + dot(dj, dj) * oim;
                            rel -= dot(c.rn[j], ow) + dot(dj, ov);
                        }
                    }
                    c.dinv[j] = safe_inv(den);
                    c.lam[j] = 0.0f;
                    c.rhs[j] = j == 0 ? normal_rhs(cd.dist, rel, c.dinv[0]) : -rel * c.dinv[j];
                }
                c.lam[0] = warm * cache_lookup(prl, prid, (unsigned)cd.id);
                nrid |= (unsigned)cd.id << (5 * sl);
            } else {
                // unused slot: all-zero rows (finite M^-1 J^T too) are no-ops in PGS
                c.mu = 0.0f;
                c.o1 = false;
#pragma unroll
                for (int j = 0; j < 3; j++) {
#pragma unroll
                    for (int a = 0; a < 9; a++) {
                        c.J[j][a] = 0.0f;
                        lds.at(sl, j, a) = 0.0f;  // (Stack's grip rows: MJStore::grip_rows reads the zero block)
                    }
                    c.dir[j] = c.rn[j] = mk(0, 0, 0);
                    c.rhs[j] = c.lam[j] = c.dinv[j] = 0.0f;
                }
            }
        }
        wc.store(PS_F_WRID, (float)nrid);
    }
    PS_PHASE(3);
    __builtin_amdgcn_sched_barrier(0);
    // per-substep values the solver never reads wait outside the registers:
    // in LDS, or (Stack, whose LDS holds its ground rows) in the global stash
    // (Stack: its global stash has no split-impulse rows, 18..26: split_of
    // rebuilds them from q after the solve, and the rows above shift down)
    auto gk = [](int k) { return NOBJ == 2 && k >= 27 ? k - 9 : k; };
    auto put = [&](int k, float v) {
        if constexpr (NOBJ == 2) lds.gstash(gk(k)) = v;
        else lds.stash(k) = v;
    };
    auto get = [&](const MJStore &S, int k) -> float {
        if constexpr (NOBJ == 2) return S.gstash(gk(k));
        else return S.stash(k);
    };
#pragma unroll
    for (int d = 0; d < 9; d++) {
        put(d, q[d]);
        put(9 + d, v1[d]);
        if constexpr (NOBJ != 2) put(18 + d, split_dq[d]);
    }
    if constexpr (NOBJ > 0) {
        put(27, cw1[0].x); put(28, cw1[0].y); put(29, cw1[0].z);
        put(30, cv1[0].x); put(31, cv1[0].y); put(32, cv1[0].z);
        put(33, bd[0].pos.x); put(34, bd[0].pos.y); put(35, bd[0].pos.z);
        put(36, bd[0].quat.x); put(37, bd[0].quat.y); put(38, bd[0].quat.z); put(39, bd[0].quat.w);
    }
    if constexpr (NOBJ == 2) {
        put(40, cw1[1].x); put(41, cw1[1].y); put(42, cw1[1].z);
        put(43, cv1[1].x); put(44, cv1[1].y); put(45, cv1[1].z);
        put(46, bd[1].pos.x); put(47, bd[1].pos.y); put(48, bd[1].pos.z);
        put(49, bd[1].quat.x); put(50, bd[1].quat.y); put(51, bd[1].quat.z); put(52, bd[1].quat.w);
    }

    // ---- projected Gauss-Seidel
    // Every row kind is gated by a wave-uniform ballot (a scalar branch: the
    // block runs if any lane of the wave needs it); inside, lanes without the
    // row hold all-zero data or [0, 0] bounds, which leave every impulse and
    // velocity untouched, so no per-lane exec masking or phi copies remain.
    float dv[9];
#pragma unroll
    for (int d = 0; d < 9; d++) dv[d] = 0.0f;
    V3 dw[NB], dvl[NB];
#pragma unroll
    for (int b = 0; b < NB; b++) {
        dw[b] = mk(0, 0, 0);
        dvl[b] = mk(0, 0, 0);
    }
    float res;
    MJStore L = lds;

    // Row-family gates, fixed for the whole solve: bit k is set when some lane
    // of the wave has that row.  Taken at the solver's entry (full exec) and
    // made wave-uniform, so each gate in the loop is a scalar test and branch;
    // a ballot inside the loop is re-masked by the lanes still iterating and
    // costs two VALU instructions per row.  Lanes that have converged are
    // masked off inside a block either way, so the results do not change.
    auto wave_bits = [&](auto pred, int n) {
        unsigned m = 0u;
        for (int k = 0; k < n; k++) m |= __builtin_amdgcn_ballot_w64(pred(k)) ? 1u << k : 0u;
        return (unsigned)__builtin_amdgcn_readfirstlane((int)m);
    };
    unsigned gate_lim = wave_bits([&](int d) { return ((lim_on >> d) & 1u) != 0u; }, 9);
    unsigned gate_ground[NB];
#pragma unroll
    for (int b = 0; b < NB; b++) gate_ground[b] = wave_bits([&](int c) { return c < ng[b]; }, NG);
    unsigned gate_pair = wave_bits([&](int c) { return c < np; }, NP);
#ifdef PS_EXPERIMENT_NO_PAIR_ROWS
    gate_pair = 0u;  // timing experiment only (wrong physics): Stack's solve without its box-box rows
#endif
    unsigned gate_robot = wave_bits([&](int c) { return c < nr; }, NR);
#ifdef PS_EXPERIMENT_NO_ROBOT_ROWS
    gate_robot = 0u;  // timing experiment only (wrong physics): the solve without the gripper rows
#endif

#ifdef PS_PROFILE_PHASES
    int prof_it = 0;
#define PS_COUNT_IT() prof_it++
#else
#define PS_COUNT_IT() do {} while (0)
#endif
    // the solver stops when every row's violation (row_viol, joint_viol) is <= 0
    static_assert(PM_SOLVER_ITERATIONS % 2 == 0, "iteration pairs");
    // The gates are wave-uniform SGPR values.  Hoisted out of the PGS loop,
    // whose exit is per lane, their bit tests become lane masks that are
    // rebuilt against exec at every gated row (a v_cndmask + v_cmp pair
    // each); redefining them at the top of each half-iteration (an empty asm
    // with an "s" operand) keeps the tests scalar, inside the loop.
#define PS_REGATE()                                                                        \
    do {                                                                                   \
        asm volatile("" : "+s"(gate_lim), "+s"(gate_pair), "+s"(gate_robot));              \
        for (int b_ = 0; b_ < NB; b_++) asm volatile("" : "+s"(gate_ground[b_]));         \
    } while (0)
    if constexpr (G == 1) {
    VelChange dvv;
#pragma unroll
    for (int k = 0; k < 4; k++) dvv.p[k] = (f32x2){0.0f, 0.0f};
    dvv.z = 0.0f;
    // dv += M^-1 e_d f: rows a >= d of column d (its lower part, which no
    // other column pairs) as v_pk_fma_f32 over the aligned dv pairs (2k,
    // 2k + 1), the rest as v_fma_f32 -- the same fused products
    auto mcol_apply = [&](int d, float f) {
        const int a0 = (d + 1) & ~1;  // first even row >= d
#pragma unroll
        for (int a = 0; a < 9; a++)
            if (a < a0 || a == 8) dvv.s(a, fmaf(Mi[sidx(a, d)], f, dvv.g(a)));
#pragma unroll
        for (int a = a0; a < 8; a += 2)
            dvv.p[a >> 1] = __builtin_elementwise_fma((f32x2){Mi[sidx(a, d)], Mi[sidx(a + 1, d)]}, (f32x2){f, f},
                                                      dvv.p[a >> 1]);
    };
    auto joint_row = [&](int d, float sgn, float rhs, float &lam, float lo, float hi) {
        float dl = rhs - dinvj[d] * (sgn * dvv.g(d));
        float nl = clamp_impulse(lam + dl, lo, hi);
        dl = nl - lam;
        lam = nl;
        mcol_apply(d, sgn * dl);
        res = res_max(res, joint_viol(dl, Mi[sidx(d, d)]));
    };
    auto limit_row = [&](int d) {
        if (PS_GATE(gate_lim & (1u << d), 0)) {
            float sgn = (lim_up >> d) & 1u ? -1.0f : 1.0f;
            float hi = (lim_on >> d) & 1u ? (float)PM_LIMIT_MAX_IMPULSE : 0.0f;
            joint_row(d, sgn, lim_rhs[d], lim_lam[d], 0.0f, hi);
        }
    };
    auto motor_row = [&](int d) {
        float imp = STD_MOTORS ? (float)(joint_force(d) * PM_TIMESTEP) : mt.imp[d];
        joint_row(d, 1.0f, mot_rhs[d], mot_lam[d], -imp, imp);
    };
    // body-side velocity change of object `o1 ? 1 : 0` (Stack selects; the
    // other scenes have one object and the select folds away)
    auto obj_add = [&](bool o1, V3 ddw, V3 ddv) {
        if constexpr (NOBJ == 2) {
            // a 0/1 weight per object: one FMA per component instead of a
            // select and an add
            const float s1 = o1 ? 1.0f : 0.0f, s0 = o1 ? 0.0f : 1.0f;
            dw[0] = fma3(ddw, s0, dw[0]);
            dvl[0] = fma3(ddv, s0, dvl[0]);
            dw[NB - 1] = fma3(ddw, s1, dw[NB - 1]);
            dvl[NB - 1] = fma3(ddv, s1, dvl[NB - 1]);
        } else {
            dw[0] = dw[0] + ddw;
            dvl[0] = dvl[0] + ddv;
        }
    };
    auto obj_dw = [&](bool o1) { return NOBJ == 2 && o1 ? dw[NB - 1] : dw[0]; };
    auto obj_dv = [&](bool o1) { return NOBJ == 2 && o1 ? dvl[NB - 1] : dvl[0]; };
    // Stack pair rows in the objects' own frame: with rn0 = r0 x d, rn1 = r1 x d
    // the row velocity is sg * pair_rel (sg = +1 when body A is object 0), and
    // an impulse dl on A moves object 0 by +sg dl and object 1 by -sg dl
    auto pair_rel = [&](V3 rn0, V3 rn1, V3 d) {
        return dot(rn0, dw[0]) + dot(d, dvl[0]) - dot(rn1, dw[NB - 1]) - dot(d, dvl[NB - 1]);
    };
    auto pair_apply = [&](V3 rn0, V3 rn1, V3 d, float sdl) {
        dw[0] = pk_fma3(rn0, sdl * od[0].iI, dw[0]);
        dvl[0] = pk_fma3(d, sdl * od[0].inv_m, dvl[0]);
        dw[NB - 1] = pk_fma3(rn1, -sdl * od[NB - 1].iI, dw[NB - 1]);
        dvl[NB - 1] = pk_fma3(d, -sdl * od[NB - 1].inv_m, dvl[NB - 1]);
    };
    (void)pair_rel;
    (void)pair_apply;

    // Stack keeps the gripper rows' J, not M^-1 J^T, in LDS: the warm start and
    // the friction rows apply dv += M^-1 g for the generalized impulse g (J^T
    // dl, or both friction rows' J^T dl summed: one product with the M^-1
    // registers per contact and sweep); the normal rows read their M^-1 J^T
    // from the global stash (GRIP_MJ_SLOTS)
    auto mi_apply = [&](const float g[9]) {
        // column by column: each dv[a] still takes b = 0..8 in order (the
        // same bits as a row-by-row product), with the columns' lower parts
        // packed (mcol_apply)
#pragma unroll
        for (int b = 0; b < 9; b++) mcol_apply(b, g[b]);
    };
    (void)mi_apply;

    // ---- warm start: the normals that matched a cached contact start from
    // 0.85 x its impulse, applied to the velocity change before the first
    // iteration (btMultiBodyConstraintSolver::setupMultiBodyContactConstraint);
    // lanes without a cache hit carry lam = 0, a no-op
    {
        MJStore W = lds.opaque();
#pragma unroll
        for (int b = 0; b < NOBJ; b++)
#pragma unroll
            for (int c = 0; c < NG; c++)
                if (PS_GATE(gate_ground[b] & (1u << c), 1)) {
                    const float l0 = gc[b][c].lam[0];
                    V3 gr = gc[b][c].r;
                    if (NOBJ == 2) {
                        const int at = b * NG + c;
                        gr = mk(W.gnd(at, 0), W.gnd(at, 1), W.gnd(at, 2));
                    }
                    dw[b] = dw[b] + od[b].inv_inertia(mk(gr.y * l0, -gr.x * l0, 0.0f));
                    dvl[b].z = fmaf(l0, od[b].inv_m, dvl[b].z);
                }
        if constexpr (NOBJ == 2) {
#pragma unroll
            for (int c = 0; c < NP; c++)
                if (gate_pair & (1u << c)) {
                    const auto *pr = W.pair_rows(c, np);
                    auto pv = [&](int k) { return mk(pr[k], pr[k + 1], pr[k + 2]); };
                    const float sl = pc[c].a0 ? pc[c].lam[0] : -pc[c].lam[0];
                    const V3 d0 = pv(0);
                    pair_apply(cross(pv(9), d0), cross(pv(12), d0), d0, sl);
                }
        }
#pragma unroll
        for (int c = 0; c < NR; c++)
            if (PS_GATE(gate_robot & (1u << c), c < 2)) {
                const RobotContact &r = rc[c];
                const float l0 = r.lam[0];
                float Jl[9];
#pragma unroll
                for (int a = 0; a < 9; a++) Jl[a] = NOBJ == 2 ? (float)W.at(c, 0, a) : r.J[0][a];
                if constexpr (NOBJ == 2) {
                    float g[9];
#pragma unroll
                    for (int a = 0; a < 9; a++) g[a] = Jl[a] * l0;
                    mi_apply(g);
                } else {
                    float w[9];
#pragma unroll
                    for (int a = 0; a < 9; a++) w[a] = W.at(c, 0, a);
#pragma unroll
                    for (int a = 0; a < 9; a++) dvv.s(a, fmaf(w[a], l0, dvv.g(a)));
                }
                if constexpr (NOBJ > 0) {
                    float im = NOBJ == 2 && r.o1 ? od[NB - 1].inv_m : od[0].inv_m;
                    V3 ddw = ANISO ? od[0].inv_inertia(r.rn[0] * -l0)
                                   : r.rn[0] * (-l0 * (NOBJ == 2 && r.o1 ? od[NB - 1].iI : od[0].iI));
                    obj_add(r.o1, ddw, r.dir[0] * (-l0 * im));
                }
            }
    }

    float gmj[GRIP_MJ_SLOTS][9];  // Stack: see object_normals
    auto object_normals = [&]() {
        if constexpr (NOBJ == 2) {
        // Stack: the cubes' ground normals and the pair normals touch only
        // the cubes' DoFs, so they commute with the joint rows and run right
        // after the motor rows, ungated for the ground (a slot a lane lacks
        // has 1/den = 0: an exact no-op).  The pair rows' read-only data come from the global stash
        // (PAIR_FLOATS).  Every slot's loads are issued here, before the
        // ground rows, so their L2 latency runs under those rows and the wave
        // waits once per sweep, not once per contact (unused slots hold
        // all-zero rows).
        float pf[NP][11];
        if constexpr (NOBJ == 2) {
            if (gate_pair) {
#pragma unroll
                for (int c = 0; c < NP; c++) {
                    const auto *pr = L.pair_rows(c, np);
#pragma unroll
                    for (int k = 0; k < 3; k++) {
                        pf[c][k] = pr[k];
                        pf[c][3 + k] = pr[9 + k];
                        pf[c][6 + k] = pr[12 + k];
                    }
                    pf[c][9] = pr[15];
                    pf[c][10] = pr[18];
                }
                __builtin_amdgcn_sched_barrier(0);
            }
            {
                // the gripper normal rows' M^-1 J^T, loaded here so the L2
                // latency runs under the ground rows
#pragma unroll
                for (int c = 0; c < GRIP_MJ_SLOTS; c++)
                    if (gate_robot & (1u << c)) {
                        const auto *gr = L.grip_rows(c, nr);
#pragma unroll
                        for (int k = 0; k < 9; k++) gmj[c][k] = gr[k];
                    }
                __builtin_amdgcn_sched_barrier(0);
            }
        }
#pragma unroll
        for (int b = 0; b < NOBJ; b++) {
            const float inv_m = od[b].inv_m;
#pragma unroll
            for (int c = 0; c < NG; c++) {
                    GroundContact &g = gc[b][c];
                    V3 gr = g.r;
                    float grhs = g.rhs[0], gdinv = g.dinv[0];
                    if (NOBJ == 2) {  // Stack: row data in LDS
                        const int at = b * NG + c;
                        gr = mk(L.gnd(at, 0), L.gnd(at, 1), L.gnd(at, 2));
                        grhs = L.gnd(at, 3);
                        // a slot this env does not have (the gate is the wave's) gets
                        // 1/den = 0, so its rows stay exact no-ops: with the zeroed
                        // offset alone, 1/den would be the cube's mass and the row
                        // would push back on any downward velocity change
                        gdinv = c < ng[b] ? cube_ground_dinv(gr, 0, od[b].iI, inv_m) : 0.0f;
                    }
                    V3 rn = mk(gr.y, -gr.x, 0.0f);  // r x (0,0,1); zero terms dropped below
                    float dl = grhs - gdinv * (rn.x * dw[b].x + rn.y * dw[b].y + dvl[b].z);
                    float nl = clamp_impulse(g.lam[0] + dl, 0.0f, (float)PM_CONTACT_UPPER);
                    dl = nl - g.lam[0];
                    g.lam[0] = nl;
                    if constexpr (ANISO) {
                        // I^-1 (r x n) dl rebuilt here: 9 FMAs instead of 3 registers per row
                        dw[b] = dw[b] + od[b].inv_inertia(mk(rn.x * dl, rn.y * dl, 0.0f));
                    } else {
                        float dI = dl * od[b].iI;
                        dw[b].x = fmaf(rn.x, dI, dw[b].x);
                        dw[b].y = fmaf(rn.y, dI, dw[b].y);
                    }
                    dvl[b].z = fmaf(dl, inv_m, dvl[b].z);
                    res = res_max(res, row_viol(dl, gdinv));
                }
        }
        if constexpr (NOBJ == 2) {
            if (gate_pair) {
#pragma unroll
                for (int c = 0; c < NP; c++)
                    if (gate_pair & (1u << c)) {
                        PairContact &p = pc[c];
                        const float sg = p.a0 ? 1.0f : -1.0f;  // A = object 0: +1
                        const V3 d0 = mk(pf[c][0], pf[c][1], pf[c][2]);
                        const V3 rn0 = cross(mk(pf[c][3], pf[c][4], pf[c][5]), d0);
                        const V3 rn1 = cross(mk(pf[c][6], pf[c][7], pf[c][8]), d0);
                        float jv = sg * pair_rel(rn0, rn1, d0);
                        float dl = pf[c][9] - pf[c][10] * jv;
                        float nl = clamp_impulse(p.lam[0] + dl, 0.0f, (float)PM_CONTACT_UPPER);
                        dl = nl - p.lam[0];
                        p.lam[0] = nl;
                        pair_apply(rn0, rn1, d0, sg * dl);
                        res = res_max(res, row_viol(dl, pf[c][10]));
                    }
            }
        }
        }
    };
    auto contacts = [&]() {
        // normals: the gripper contacts (the objects' ground and pair
        // normals ran with the motor rows: ground_normals, object_normals)
#pragma unroll
        for (int c = 0; c < NR; c++)
            if (PS_GATE(gate_robot & (1u << c), c < 2)) {
                RobotContact &r = rc[c];
                // M^-1 J^T column first: its LDS latency hides under the dot
                float mj[9], Jl[9];
#pragma unroll
                for (int a = 0; a < 9; a++) Jl[a] = NOBJ == 2 ? (float)L.at(c, 0, a) : r.J[0][a];
                if constexpr (NOBJ != 2) {
#pragma unroll
                    for (int a = 0; a < 9; a++) mj[a] = L.at(c, 0, a);
                }
                __builtin_amdgcn_sched_barrier(0);
                float jv = dvv.dot(Jl);
                if (NOBJ > 0) jv -= dot(r.rn[0], obj_dw(r.o1)) + dot(r.dir[0], obj_dv(r.o1));
                float dl = r.rhs[0] - r.dinv[0] * jv;
                float nl = clamp_impulse(r.lam[0] + dl, 0.0f, (float)PM_CONTACT_UPPER);
                dl = nl - r.lam[0];
                r.lam[0] = nl;
                if constexpr (NOBJ == 2) {
                    dvv.apply(gmj[c], dl);
                } else {
                    dvv.apply(mj, dl);
                }
                if constexpr (NOBJ == 1) {
                    // one object: fma straight into its velocity change
                    dw[0] = ANISO ? dw[0] + od[0].inv_inertia_pk(r.rn[0] * -dl) : pk_fma3(r.rn[0], -dl * od[0].iI, dw[0]);
                    dvl[0] = pk_fma3(r.dir[0], -dl * od[0].inv_m, dvl[0]);
                } else if constexpr (NOBJ == 2) {
                    float im = r.o1 ? od[NB - 1].inv_m : od[0].inv_m;
                    float iI = r.o1 ? od[NB - 1].iI : od[0].iI;
                    obj_add(r.o1, r.rn[0] * (-dl * iI), r.dir[0] * (-dl * im));
                }
                res = res_max(res, row_viol(dl, r.dinv[0]));
            }
        // friction cones (Stack: the pair rows' loads first, as above)
        float pq[NP][16];
        if constexpr (NOBJ == 2) {
            if (gate_pair) {
#pragma unroll
                for (int c = 0; c < NP; c++) {
                    const auto *pr = L.pair_rows(c, np);
#pragma unroll
                    for (int k = 0; k < 12; k++) pq[c][k] = pr[3 + k];  // d1, d2, r0, r1
                    pq[c][12] = pr[16];
                    pq[c][13] = pr[17];
                    pq[c][14] = pr[19];
                    pq[c][15] = pr[20];
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        }

#pragma unroll
        for (int b = 0; b < NOBJ; b++) {
            const float inv_m = od[b].inv_m;
#pragma unroll
            for (int c = 0; c < NG; c++)
                if (PS_GATE(gate_ground[b] & (1u << c), 1)) {
                    GroundContact &g = gc[b][c];
                    V3 gr = g.r;
                    float grhs1 = g.rhs[1], grhs2 = g.rhs[2], gdinv1 = g.dinv[1], gdinv2 = g.dinv[2];
                    if (NOBJ == 2) {  // Stack: row data in LDS
                        const int at = b * NG + c;
                        gr = mk(L.gnd(at, 0), L.gnd(at, 1), L.gnd(at, 2));
                        grhs1 = L.gnd(at, 4);
                        grhs2 = L.gnd(at, 5);
                        const bool on = c < ng[b];  // as in the normal sweep
                        gdinv1 = on ? cube_ground_dinv(gr, 1, od[b].iI, inv_m) : 0.0f;
                        gdinv2 = on ? cube_ground_dinv(gr, 2, od[b].iI, inv_m) : 0.0f;
                    }
                    // The two friction rows (directions (0,-1,0) and (1,0,0), so
                    // r x dir = (r.z, 0, -r.x) and (0, r.z, -r.y)) side by side
                    // as f32x2 (v_pk_mul/fma/add_f32): the operations the scalar
                    // rows compiled to, fused where they were fused, so the same
                    // bits; x = row a, y = row b.
                    float dla, dlb;
                    {
#pragma clang fp contract(off)
                        const f32x2 gz = {gr.z, gr.z};
                        const f32x2 t = (f32x2){gr.x, gr.y} * (f32x2){dw[b].z, dw[b].z};
                        const f32x2 u = __builtin_elementwise_fma(gz, (f32x2){dw[b].x, dw[b].y}, -t);
                        const f32x2 w = u + (f32x2){-dvl[b].y, dvl[b].x};
                        const f32x2 lam12 = {g.lam[1], g.lam[2]};
                        const f32x2 s2 = lam12 + __builtin_elementwise_fma(-(f32x2){gdinv1, gdinv2}, w,
                                                                           (f32x2){grhs1, grhs2});
                        const float lim = gmu * g.lam[0];  // >= 0: the normal row's clamp
                        // |f|^2 as each kernel's scalar rows contracted it (the
                        // one-object kernels fused row b's square, Stack's row a's);
                        // |f| > mu N: project onto the cone (lim * rsq(m2) <= 1 there)
                        const float m2 = NOBJ == 2 ? fmaf(s2.x, s2.x, s2.y * s2.y) : fmaf(s2.y, s2.y, s2.x * s2.x);
                        const float sc2 = cone_scale(m2, lim);
                        const f32x2 dl2 = __builtin_elementwise_fma(s2, (f32x2){sc2, sc2}, -lam12);
                        const f32x2 nl2 = s2 * (f32x2){sc2, sc2};
                        g.lam[1] = nl2.x;
                        g.lam[2] = nl2.y;
                        dla = dl2.x;
                        dlb = dl2.y;
                        if constexpr (ANISO) {
                            // I^-1 (r1 dla + r2 dlb)
                            const f32x2 zab = gz * dl2;
                            dw[b] = dw[b] + od[b].inv_inertia_pk_unfused(mk(zab.x, zab.y, fmaf(-gr.x, dla, -gr.y * dlb)));
                        } else {
                            const f32x2 ab = dl2 * (f32x2){od[b].iI, od[b].iI};
                            const f32x2 wxy = __builtin_elementwise_fma(gz, ab, (f32x2){dw[b].x, dw[b].y});
                            dw[b].z = fmaf(-gr.y, ab.y, fmaf(-gr.x, ab.x, dw[b].z));
                            dw[b].x = wxy.x;
                            dw[b].y = wxy.y;
                        }
                        const f32x2 vxy = __builtin_elementwise_fma((f32x2){dlb, -dla}, (f32x2){inv_m, inv_m},
                                                                    (f32x2){dvl[b].x, dvl[b].y});
                        dvl[b].x = vxy.x;
                        dvl[b].y = vxy.y;
                    }
                    res = res_max(res, res_max(row_viol(dla, gdinv1), row_viol(dlb, gdinv2)));
                }
        }
        if constexpr (NOBJ == 2) {
            const float pmu = sc.fric * sc.fric;
            if (gate_pair) {
#pragma unroll
                for (int c = 0; c < NP; c++)
                    if (gate_pair & (1u << c)) {
                        PairContact &p = pc[c];
                        auto pv = [&](int k) { return mk(pq[c][k], pq[c][k + 1], pq[c][k + 2]); };
                        const float sg = p.a0 ? 1.0f : -1.0f;
                        const V3 d1 = pv(0), d2 = pv(3), r0 = pv(6), r1 = pv(9);
                        const V3 rn01 = cross(r0, d1), rn02 = cross(r0, d2), rn11 = cross(r1, d1), rn12 = cross(r1, d2);
                        float ja = sg * pair_rel(rn01, rn11, d1);
                        float jb = sg * pair_rel(rn02, rn12, d2);
                        float dla = pq[c][12] - pq[c][14] * ja, dlb = pq[c][13] - pq[c][15] * jb;
                        float sa = p.lam[1] + dla, sb = p.lam[2] + dlb;
                        float lim = pmu * p.lam[0];
                        float m2 = sa * sa + sb * sb;
                        float s = cone_scale(m2, lim);
                        sa *= s;
                        sb *= s;
                        dla = sa - p.lam[1];
                        dlb = sb - p.lam[2];
                        p.lam[1] = sa;
                        p.lam[2] = sb;
                        pair_apply(rn01, rn11, d1, sg * dla);
                        pair_apply(rn02, rn12, d2, sg * dlb);
                        res = res_max(res, res_max(row_viol(dla, pq[c][14]), row_viol(dlb, pq[c][15])));
                    }
            }
        }
#pragma unroll
        for (int c = 0; c < NR; c++)
            if (PS_GATE(gate_robot & (1u << c), c < 2)) {
                RobotContact &r = rc[c];
                float mj1[9], mj2[9], J1[9], J2[9];
#pragma unroll
                for (int a = 0; a < 9; a++) {
                    J1[a] = NOBJ == 2 ? (float)L.at(c, 1, a) : r.J[1][a];
                    J2[a] = NOBJ == 2 ? (float)L.at(c, 2, a) : r.J[2][a];
                }
                if constexpr (NOBJ != 2) {
#pragma unroll
                    for (int a = 0; a < 9; a++) {
                        mj1[a] = L.at(c, 1, a);
                        mj2[a] = L.at(c, 2, a);
                    }
                }
                __builtin_amdgcn_sched_barrier(0);
                float ja, jb;
                if constexpr (NOBJ != 2) {
                    // the two rows' dot products side by side: (J1_a, J2_a) x
                    // (dv_a, dv_a), each lane the scalar chain's FMAs
#pragma clang fp contract(off)
                    f32x2 j2 = {0.0f, 0.0f};
#pragma unroll
                    for (int a = 0; a < 9; a++) j2 = __builtin_elementwise_fma((f32x2){J1[a], J2[a]}, dvv.bc(a), j2);
                    ja = j2.x;
                    jb = j2.y;
                } else {
                    ja = dvv.dot(J1);
                    jb = dvv.dot(J2);
                }
                if (NOBJ > 0) {
                    V3 ow = obj_dw(r.o1), ov = obj_dv(r.o1);
                    ja -= dot(r.rn[1], ow) + dot(r.dir[1], ov);
                    jb -= dot(r.rn[2], ow) + dot(r.dir[2], ov);
                }
                float dla, dlb;
                if constexpr (NOBJ != 2) {
                    // from the two rows' velocities on, the rows side by side as
                    // f32x2 (v_pk_*) with the scalar rows' operations and
                    // fusions (the same bits); the object's dot products above
                    // stay scalar (pairing rn[1] with rn[2] would fight
                    // pk_fma3's (x, y) pairs of the same registers)
#pragma clang fp contract(off)
                    const f32x2 lam12 = {r.lam[1], r.lam[2]};
                    const f32x2 s2 = lam12 + __builtin_elementwise_fma(-(f32x2){r.dinv[1], r.dinv[2]}, (f32x2){ja, jb},
                                                                       (f32x2){r.rhs[1], r.rhs[2]});
                    const float lim = r.mu * r.lam[0];  // >= 0: the normal row's clamp
                    const float sc2 = cone_scale(fmaf(s2.x, s2.x, s2.y * s2.y), lim);
                    const f32x2 dl2 = __builtin_elementwise_fma(s2, (f32x2){sc2, sc2}, -lam12);
                    const f32x2 nl2 = s2 * (f32x2){sc2, sc2};
                    r.lam[1] = nl2.x;
                    r.lam[2] = nl2.y;
                    dla = dl2.x;
                    dlb = dl2.y;
                } else {
                    dla = r.rhs[1] - r.dinv[1] * ja;
                    dlb = r.rhs[2] - r.dinv[2] * jb;
                    float sa = r.lam[1] + dla, sb = r.lam[2] + dlb;
                    const float lim = r.mu * r.lam[0];  // >= 0: the normal row's clamp
                    const float m2 = sa * sa + sb * sb;
                    const float s = cone_scale(m2, lim);
                    sa *= s;
                    sb *= s;
                    dla = sa - r.lam[1];
                    dlb = sb - r.lam[2];
                    r.lam[1] = sa;
                    r.lam[2] = sb;
                }
                if constexpr (NOBJ == 2) {
                    float g[9];
#pragma unroll
                    for (int a = 0; a < 9; a++) g[a] = fmaf(J2[a], dlb, J1[a] * dla);
                    mi_apply(g);
                } else {
                    dvv.apply(mj1, dla);
                    dvv.apply(mj2, dlb);
                }
                if constexpr (NOBJ == 1) {
                    if constexpr (ANISO) {
                        dw[0] = dw[0] + od[0].inv_inertia_pk(fma3(r.rn[2], -dlb, r.rn[1] * -dla));
                    } else {
                        float aI = -dla * od[0].iI, bI = -dlb * od[0].iI;
                        dw[0] = pk_fma3(r.rn[2], bI, pk_fma3(r.rn[1], aI, dw[0]));
                    }
                    float am = -dla * od[0].inv_m, bm = -dlb * od[0].inv_m;
                    dvl[0] = pk_fma3(r.dir[2], bm, pk_fma3(r.dir[1], am, dvl[0]));
                } else if constexpr (NOBJ == 2) {
                    float im = r.o1 ? od[NB - 1].inv_m : od[0].inv_m;
                    // two objects are cubes (isotropic inverse inertia)
                    float iI = r.o1 ? od[NB - 1].iI : od[0].iI;
                    float aI = -dla * iI, bI = -dlb * iI;
                    V3 ddw = mk(fmaf(r.rn[2].x, bI, r.rn[1].x * aI), fmaf(r.rn[2].y, bI, r.rn[1].y * aI),
                                fmaf(r.rn[2].z, bI, r.rn[1].z * aI));
                    float am = -dla * im, bm = -dlb * im;
                    V3 ddv = mk(fmaf(r.dir[2].x, bm, r.dir[1].x * am), fmaf(r.dir[2].y, bm, r.dir[1].y * am),
                                fmaf(r.dir[2].z, bm, r.dir[1].z * am));
                    obj_add(r.o1, ddw, ddv);
                }
                res = res_max(res, res_max(row_viol(dla, r.dinv[1]), row_viol(dlb, r.dinv[2])));
            }
    };

    // One object (not Stack): its ground normals touch only the object's
    // DoFs and commute with the joint rows, so they run ungated in the motor
    // rows' block (a slot a lane lacks is an all-zero no-op) -- Bullet's
    // order up to commuting rows
    auto ground_normals = [&]() {
        if constexpr (NOBJ == 1) {
#pragma unroll
            for (int c = 0; c < NG; c++) {
                GroundContact &g = gc[0][c];
                const V3 rn = mk(g.r.y, -g.r.x, 0.0f);  // r x (0,0,1)
                float dl = g.rhs[0] - g.dinv[0] * (rn.x * dw[0].x + rn.y * dw[0].y + dvl[0].z);
                const float nl = clamp_impulse(g.lam[0] + dl, 0.0f, (float)PM_CONTACT_UPPER);
                dl = nl - g.lam[0];
                g.lam[0] = nl;
                if constexpr (ANISO) {
                    dw[0] = dw[0] + od[0].inv_inertia_pk(mk(rn.x * dl, rn.y * dl, 0.0f));
                } else {
                    const float dI = dl * od[0].iI;
                    dw[0].x = fmaf(rn.x, dI, dw[0].x);
                    dw[0].y = fmaf(rn.y, dI, dw[0].y);
                }
                dvl[0].z = fmaf(dl, od[0].inv_m, dvl[0].z);
                res = res_max(res, row_viol(dl, g.dinv[0]));
            }
        }
    };

    // btSequentialImpulseConstraintSolver alternates the order of the
    // non-contact rows by iteration parity: even iterations run them in
    // reverse (motors 8..0, then limits 8..0), odd ones forward (limits 0..8,
    // then motors 0..8).  The loop is unrolled by two so both orders are
    // straight-line code; each env still stops at its own residual.
    for (int it = 0; it < PM_SOLVER_ITERATIONS; it += 2) {
        PS_COUNT_IT();
        L = lds.opaque();
        res = 0.0f;
        PS_REGATE();
        // one object: M^-1 enters each iteration pair in VGPRs (an empty asm
        // with a "v" operand), else the allocator parks it in AGPRs and
        // every motor row reads its column back (v_accvgpr_read): the PGS
        // loop's AGPR reads 442 -> 340 per iteration pair, Push 3.03 ->
        // 3.01 ms (profiles/r03h_variants_pin.log; Reach, no object, got
        // slower and keeps the allocator's choice)
        if constexpr (NOBJ == 1) {
#pragma unroll
            for (int k = 0; k < 45; k++) asm volatile("" : "+v"(Mi[k]));
        }
#pragma unroll
        for (int d = 8; d >= 0; d--) motor_row(d);
        ground_normals();
        object_normals();
        if (PS_GATE(gate_lim != 0u, 0)) {
#pragma unroll
            for (int d = 8; d >= 0; d--) limit_row(d);
        }
        contacts();
        if (res <= 0.0f) break;
        PS_COUNT_IT();
        L = lds.opaque();
        res = 0.0f;
        PS_REGATE();
        if (PS_GATE(gate_lim != 0u, 0)) {
#pragma unroll
            for (int d = 0; d < 9; d++) limit_row(d);
        }
#pragma unroll
        for (int d = 0; d < 9; d++) motor_row(d);
        ground_normals();
        object_normals();
        contacts();
        if (res <= 0.0f) break;
    }
#pragma unroll
    for (int a = 0; a < 9; a++) dv[a] = dvv.g(a);
    } else {
        group_pgs<NOBJ, SHAPE, STD_MOTORS, G>(mt, Mi, lds, gate_lim, lim_up, lim_on, gate_ground[0], gate_robot,
                                              dinvj, lim_rhs, lim_lam, mot_rhs, mot_lam, gc[0], rc, od[0], gmu,
                                              dv, dw[0], dvl[0] PS_PROF_COUNT_ARG PS_DUMP_ARG);
    }

    // the contacts' final normal impulses become the cache of the next
    // substep (solveGroupCacheFriendlyFinish writes m_appliedImpulse back)
#pragma unroll
    for (int b = 0; b < NOBJ; b++)
#pragma unroll
        for (int c = 0; c < NG; c++) wc.store((b == 0 ? PS_F_WG0 : PS_F_WG1) + c, gc[b][c].lam[0]);
    if constexpr (NOBJ == 2) {
#pragma unroll
        for (int c = 0; c < NP; c++) wc.store(PS_F_WP + c, pc[c].lam[0]);
    }
#pragma unroll
    for (int c = 0; c < NR; c++) wc.store(PS_F_WR + c, rc[c].lam[0]);

    PS_PHASE(4);
#ifdef PS_PROFILE_PHASES
    {
        int wmax = prof_it, wnr = nr;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            wmax = max(wmax, __shfl_xor(wmax, o));
            wnr = max(wnr, __shfl_xor(wnr, o));
        }
        pt.acc[8] += prof_it;
        pt.acc[9] += wmax;
#pragma unroll
        for (int k = PS_ITP_WORDS - 1; k > 0; k--) pt.itp[k] = (pt.itp[k] << 16) | (pt.itp[k - 1] >> 16);
        pt.itp[0] = (pt.itp[0] << 16) | (uint32_t)min(prof_it, 255) | ((uint32_t)nr << 8) | ((uint32_t)np << 11);
        pt.acc[10] += 1;
        pt.acc[11] += wnr;
        // the wave's open row gates (wave-uniform: every lane adds the same)
        unsigned ngnd = 0;
        for (int b = 0; b < NB; b++) ngnd += __builtin_popcount(gate_ground[b]);
        pt.acc[12] += __builtin_popcount(gate_pair);
        pt.acc[13] += ngnd;
        pt.acc[14] += __builtin_popcount(gate_robot);
        pt.acc[15] += gate_lim != 0u;
    }
#endif
    {
        // reload through an opaque address: no store-to-load forwarding, so
        // the registers really were free during the solve
        MJStore S = lds.opaque();
#pragma unroll
        for (int d = 0; d < 9; d++) {
            q[d] = get(S, d);
            v1[d] = get(S, 9 + d);
            split_dq[d] = NOBJ == 2 ? split_of(d, q[d]) : get(S, 18 + d);
        }
        if constexpr (NOBJ > 0) {
            cw1[0] = mk(get(S, 27), get(S, 28), get(S, 29));
            cv1[0] = mk(get(S, 30), get(S, 31), get(S, 32));
            bd[0].pos = mk(get(S, 33), get(S, 34), get(S, 35));
            bd[0].quat = Q4{get(S, 36), get(S, 37), get(S, 38), get(S, 39)};
        }
        if constexpr (NOBJ == 2) {
            cw1[1] = mk(get(S, 40), get(S, 41), get(S, 42));
            cv1[1] = mk(get(S, 43), get(S, 44), get(S, 45));
            bd[1].pos = mk(get(S, 46), get(S, 47), get(S, 48));
            bd[1].quat = Q4{get(S, 49), get(S, 50), get(S, 51), get(S, 52)};
        }
    }
    // ---- integrate (btMultiBody::stepPositionsMultiDof)
#pragma unroll
    for (int d = 0; d < 9; d++) {
        qd[d] = v1[d] + dv[d];
        q[d] += dt * qd[d] + split_dq[d];
    }
#pragma unroll
    for (int b = 0; b < NOBJ; b++) {
        Body &cb = bd[b];
        cb.omg = cw1[b] + dw[b];
        cb.vel = cv1[b] + dvl[b];
        cb.pos = cb.pos + cb.vel * dt;
        float ang = norm(cb.omg);
        if (ang * dt > 0.5f * 1.5707963267948966f) ang = 0.5f * 1.5707963267948966f / dt;
        float f = ang < 0.001f ? (0.5f * dt - (dt * dt * dt) * 0.020833333333f * ang * ang) : sinf(0.5f * ang * dt) / ang;
        Q4 dq = Q4{cb.omg.x * f, cb.omg.y * f, cb.omg.z * f, cosf(0.5f * ang * dt)};
        Q4 nq = qmul(dq, cb.quat);
        float nn = rsqrtf(nq.x * nq.x + nq.y * nq.y + nq.z * nq.z + nq.w * nq.w);
        cb.quat = Q4{nq.x * nn, nq.y * nn, nq.z * nn, nq.w * nn};
    }
    PS_PHASE(5);
}

}  // namespace ps
