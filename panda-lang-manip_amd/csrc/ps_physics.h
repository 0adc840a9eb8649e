// ps_physics.h — per-env (one env per lane) fp32 Panda multibody step for
// gfx950.  Same algorithm as the PyBullet 3.2.5 subset used by
// panda_gym/pybullet.py (restated in DESIGN.md §Physics), derived for a
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
    constexpr M3d Ro = origin_rot(I);
    Frame F;
    M3 Rj;
#pragma unroll
    for (int r = 0; r < 3; r++)
#pragma unroll
        for (int c = 0; c < 3; c++)
            Rj.m[r * 3 + c] = P.R.m[r * 3 + 0] * (float)Ro.m[0 * 3 + c] + P.R.m[r * 3 + 1] * (float)Ro.m[1 * 3 + c] +
                              P.R.m[r * 3 + 2] * (float)Ro.m[2 * 3 + c];
    V3 oj = P.o + mul(P.R, mk((float)d.o[0], (float)d.o[1], (float)d.o[2]));
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
    return k.f[I].o + mul(k.f[I].R, mk((float)d.com[0], (float)d.com[1], (float)d.com[2]));
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
    c.I = a.I + b.I + shift(a.m, a.h - c.h) + shift(b.m, b.h - c.h);
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
    V3 c = f.o + mul(f.R, mk((float)d.com[0], (float)d.com[1], (float)d.com[2]));
    V3 rc = c - f.o;
    V3 vc = vo + cross(w, rc);
    V3 ac = ao + cross(dw, rc) + cross(w, cross(w, rc));
    S3 Iw = rotate_diag(f.R, (float)link_inertia(I, 0), (float)link_inertia(I, 1), (float)link_inertia(I, 2));
    V3 Iww = mul(Iw, w);
    float cl = (float)PM_LINEAR_DAMPING + (float)PM_LINEAR_DAMPING * norm(vc);
    float ca = (float)PM_ANGULAR_DAMPING + (float)PM_ANGULAR_DAMPING * norm(w);
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
    float L[45];
#pragma unroll
    for (int i = 0; i < 9; i++) {
#pragma unroll
        for (int j = 0; j <= i; j++) {
            float s = M[sidx(i, j)];
#pragma unroll
            for (int q = 0; q < j; q++) s -= L[sidx(i, q)] * L[sidx(j, q)];
            if (i == j) L[sidx(i, i)] = sqrtf(s);
            else L[sidx(i, j)] = s / L[sidx(j, j)];
        }
    }
    // invert L in place (lower triangular)
    float Li[45];
#pragma unroll
    for (int i = 0; i < 9; i++) {
        float inv = 1.0f / L[sidx(i, i)];
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
// calculateInverseKinematics (restated in DESIGN.md §IK): <= 20 DLS steps
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
        Q4 qinv = Q4{-qe.x / n2, -qe.y / n2, -qe.z / n2, qe.w / n2};
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
        // Cholesky solve
        float Lc[N * (N + 1) / 2];
#pragma unroll
        for (int i = 0; i < N; i++)
#pragma unroll
            for (int j = 0; j <= i; j++) {
                float s = U[i * (i + 1) / 2 + j];
#pragma unroll
                for (int t = 0; t < j; t++) s -= Lc[i * (i + 1) / 2 + t] * Lc[j * (j + 1) / 2 + t];
                if (i == j) Lc[i * (i + 1) / 2 + i] = sqrtf(s);
                else Lc[i * (i + 1) / 2 + j] = s / Lc[j * (j + 1) / 2 + j];
            }
        float y[N], x[N];
#pragma unroll
        for (int i = 0; i < N; i++) {
            float s = g[i];
#pragma unroll
            for (int t = 0; t < i; t++) s -= Lc[i * (i + 1) / 2 + t] * y[t];
            y[i] = s / Lc[i * (i + 1) / 2 + i];
        }
#pragma unroll
        for (int i = N - 1; i >= 0; i--) {
            float s = y[i];
#pragma unroll
            for (int t = i + 1; t < N; t++) s -= Lc[t * (t + 1) / 2 + i] * x[t];
            x[i] = s / Lc[i * (i + 1) / 2 + i];
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
struct Scene {
    V3 base;
    float half, mass;
    int has_table, has_plane, has_cube;
};

struct Motors {
    float target[9], kp[9], kd[9], vel[9], imp[9];
};

struct Cube {
    V3 pos;
    Q4 quat;
    V3 vel, omg;
};

PS_D bool ground_top(const Scene &sc, float x, float y, float &top) {
    if (sc.has_table && fabsf(x - (float)PM_TABLE_CX) <= (float)PM_TABLE_HX && fabsf(y) <= (float)PM_TABLE_HY) {
        top = (float)PM_TABLE_TOP;
        return true;
    }
    if (sc.has_plane) {
        top = (float)PM_PLANE_TOP;
        return true;
    }
    return false;
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
// LDS floats per lane: M^-1 J^T of the 3 rows of every gripper contact
// (108 floats x 256 lanes per CU = 108 KiB of the 160 KiB LDS at one wave per
// SIMD); the diagnostic PS_MI_LDS build appends the packed M^-1.
// Then 40 floats of per-substep values the PGS loop never reads (q, v1, the
// split-impulse position correction, the object's pre-solve velocities and
// pose): they wait in LDS across the solve instead of holding registers.
constexpr int LDS_STASH_OFFSET = NR * 27;
constexpr int LDS_STASH_FLOATS = 40;
constexpr int LDS_MI_OFFSET = LDS_STASH_OFFSET + LDS_STASH_FLOATS;
#ifdef PS_MI_LDS
constexpr int LDS_FLOATS = LDS_MI_OFFSET + 45;
#else
constexpr int LDS_FLOATS = LDS_MI_OFFSET;
#endif

// cube-ground contact: cube-only rows; normal +z, friction dirs of planeSpace(+z) = (0,-1,0), (1,0,0)
struct GroundContact {
    V3 r;  // contact point - cube COM
    float rhs[3], lam[3], dinv[3];
};

// gripper contact: robot rows with explicit Jacobians (M^-1 J^T lives in LDS)
struct RobotContact {
    float J[3][9];
    V3 dir[3];
    V3 rn[3];  // cube side: (pB - x_cube) x dir (zero when the contact is with the ground)
    float rhs[3], lam[3], dinv[3], mu;
};

// per-lane view of the LDS rows: element (slot, row, k) at base[((slot*3 + row)*9 + k) * stride]
typedef __attribute__((address_space(3))) float lds_float;
struct MJStore {
    lds_float *base;
    int stride;
    PS_D lds_float &at(int slot, int row, int k) const { return base[((slot * 3 + row) * 9 + k) * stride]; }
    PS_D lds_float &mi(int k) const { return base[(LDS_MI_OFFSET + k) * stride]; }
    PS_D lds_float &stash(int k) const { return base[(LDS_STASH_OFFSET + k) * stride]; }
    // a copy whose address the compiler cannot see through: loads from it are
    // not loop-invariant, so they stay in the PGS loop as ds_reads instead of
    // being hoisted into (spilled) registers
    PS_D MJStore opaque() const {
        MJStore r = *this;
        asm volatile("" : "+v"(r.base));
        return r;
    }
};

PS_D float jrow_dot(const float J[9], const float v[9]) {
    float s = 0.0f;
#pragma unroll
    for (int d = 0; d < 9; d++) s += J[d] * v[d];
    return s;
}

// Geometry that outlives the kinematics: DoF axes/origins (gripper-contact
// Jacobians) and world sphere centres.
struct Geo {
    V3 ax[9], org[7], spw[PM_NUM_SPHERES];
};

// ----------------------------------------------------------------- substep
// One btMultiBodyDynamicsWorld::stepSimulation(1/500 s): see the oracle's
// po_substep for the row-by-row restatement this mirrors.
// PGS residual of a row is dl / dinv (the impulse change in velocity units).
// v_rcp_f32 replaces the IEEE division; a zero dinv gives 0 * inf = NaN, which
// fmaxf() in the residual max ignores, matching the reference's skip.
PS_D float res_scale(float dinv) { return __builtin_amdgcn_rcpf(dinv); }

// STD_MOTORS: the motors are the ones RobotTaskEnv.step sets (POSITION_CONTROL
// on all nine joints with the fixed Panda gains and forces, panda.py:40-56), so
// only the targets are per-env; otherwise every gain comes from `mt`.
template <bool HAS_CUBE, bool STD_MOTORS>
PS_D void substep(const Scene &sc, float q[9], float qd[9], const Motors &mt, Cube &cb, const MJStore &lds PS_PROF_PARAM) {
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
        static_for<0, PM_NUM_SPHERES>([&](auto SS) {
            constexpr int S = decltype(SS)::value;
            constexpr SphereDef s = sphere_def(S);
            geo.spw[S] = k.f[s.link].o + mul(k.f[s.link].R, mk((float)s.c[0], (float)s.c[1], (float)s.c[2])) + sc.base;
        });
        mass_matrix(k, Mi);
    }
    PS_PHASE(1);
    __builtin_amdgcn_sched_barrier(0);
    spd_inverse(Mi);
    PS_PHASE(2);
    __builtin_amdgcn_sched_barrier(0);
    // M^-1 for the joint rows stays in registers: re-reading it from LDS in
    // every PGS iteration exposed the LDS latency once per motor row (Push
    // 4.56 -> 3.99 ms, Reach 2.97 -> 1.98 ms per step of 65 536 envs).
    // PS_MI_LDS keeps the LDS variant for comparison.
#ifdef PS_MI_LDS
    constexpr bool MI_REGS = false;
#else
    constexpr bool MI_REGS = true;
#endif
    if constexpr (!MI_REGS) {
#pragma unroll
        for (int k = 0; k < 45; k++) lds.mi(k) = Mi[k];
    }
    float v1[9];
#pragma unroll
    for (int a = 0; a < 9; a++) {
        float s = 0.0f;
#pragma unroll
        for (int b = 0; b < 9; b++) s -= Mi[sidx(a, b)] * hb[b];
        v1[a] = qd[a] + dt * s;
    }
    // cube: gravity + btMultiBody damping (isotropic inertia: no gyroscopic term)
    V3 cw1 = mk(0, 0, 0), cv1 = mk(0, 0, 0);
    float inv_I = 0.0f, inv_m = 0.0f;
    if constexpr (HAS_CUBE) {
        float l = 2.0f * sc.half;
        inv_I = 1.0f / (sc.mass / 12.0f * (2.0f * l * l));
        inv_m = 1.0f / sc.mass;
        float cl = (float)PM_LINEAR_DAMPING + (float)PM_LINEAR_DAMPING * norm(cb.vel);
        float ca = (float)PM_ANGULAR_DAMPING + (float)PM_ANGULAR_DAMPING * norm(cb.omg);
        cv1 = cb.vel + (mk(0, 0, (float)PM_GRAVITY_Z) - cb.vel * cl) * dt;
        cw1 = cb.omg - cb.omg * (ca * dt);
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
        dinvj[d] = den > 2.2204460492503131e-16f ? 1.0f / den : 0.0f;
        split_dq[d] = 0.0f;
        lim_rhs[d] = 0.0f;
        lim_lam[d] = 0.0f;
#pragma unroll
        for (int side = 0; side < 2; side++) {
            float lo = (float)dof_def(d).lo, hi = (float)dof_def(d).hi;
            float pen = side ? hi - q[d] : q[d] - lo;
            float sgn = side ? -1.0f : 1.0f;
            bool on = pen <= 0.0f;
            float velerr = -sgn * v1[d];
            bool combined = pen > (float)PM_SPLIT_PENETRATION_THRESHOLD;
            float poserr = -pen * (float)PM_ERP / dt;
            if (on) {
                lim_on |= 1u << d;
                lim_up |= side ? 1u << d : 0u;
                lim_rhs[d] = (combined ? poserr + velerr : velerr) * dinvj[d];
                if (!combined) split_dq[d] += sgn * (-pen) * (float)PM_SPLIT_LIMIT_ERP;
            }
        }
        float kp = STD_MOTORS ? (float)PM_MOTOR_KP : mt.kp[d], kd = STD_MOTORS ? (float)PM_MOTOR_KD : mt.kd[d];
        float vel = STD_MOTORS ? 0.0f : mt.vel[d];
        float target = kp * (mt.target[d] - q[d]) / dt + v1[d] + kd * (vel - v1[d]);
        mot_rhs[d] = (target - v1[d]) * dinvj[d];
        mot_lam[d] = 0.0f;
    }

    // ---- contacts
    GroundContact gc[NG];
#pragma unroll
    for (int s = 0; s < NG; s++) gc[s] = GroundContact{mk(0, 0, 0), {0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
    int ng = 0;
    RobotContact rc[NR];
    int nr = 0;
    M3 Rc;
    if constexpr (HAS_CUBE) {
        Rc = quat_to_mat(cb.quat);
        const float h = sc.half;
#pragma unroll
        for (int v = 0; v < 8; v++) {
            V3 loc = mk((v & 1) ? h : -h, (v & 2) ? h : -h, (v & 4) ? h : -h);
            V3 pw = cb.pos + mul(Rc, loc);
            float top;
            if (ng < NG && ground_top(sc, pw.x, pw.y, top)) {
                float dist = pw.z - top;
                if (dist < (float)PM_CONTACT_MARGIN_GROUND) {
                    V3 r = pw - cb.pos;
                    // normal (0,0,1), t1 (0,-1,0), t2 (1,0,0)
                    V3 dirs[3] = {mk(0, 0, 1), mk(0, -1, 0), mk(1, 0, 0)};
                    GroundContact g;
                    g.r = r;
#pragma unroll
                    for (int j = 0; j < 3; j++) {
                        V3 rn = cross(r, dirs[j]);
                        float den = dot(rn, rn) * inv_I + dot(dirs[j], dirs[j]) * inv_m;
                        g.dinv[j] = den > 2.2204460492503131e-16f ? 1.0f / den : 0.0f;
                        float rel = dot(rn, cw1) + dot(dirs[j], cv1);
                        g.lam[j] = 0.0f;
                        if (j == 0) {
                            float pen = dist + (float)PM_LINEAR_SLOP;
                            float velerr = -rel, poserr = 0.0f;
                            if (pen > 0.0f) velerr -= pen / dt;
                            else poserr = -pen * (float)PM_ERP / dt;
                            bool combined = pen > (float)PM_SPLIT_PENETRATION_THRESHOLD;
                            g.rhs[0] = (combined ? poserr + velerr : velerr) * g.dinv[0];
                        } else {
                            g.rhs[j] = -rel * g.dinv[j];
                        }
                    }
#pragma unroll
                    for (int s = 0; s < NG; s++)
                        if (s == ng) gc[s] = g;
                    ng++;
                }
            }
        }
    }
    {
        // 1) candidate gripper contacts in spec order (spheres vs cube, then
        //    spheres vs ground) -> small records; the first NR active ones
        //    are assigned slots 0..NR-1 (select into compile-time slots)
        struct Cand {
            V3 pA, pB, n;
            float dist, mu;
            int link;
            bool on_cube;
        };
        Cand slot[NR];
#pragma unroll
        for (int s = 0; s < NR; s++) slot[s] = Cand{mk(0, 0, 0), mk(0, 0, 0), mk(0, 0, 1), 1.0f, 0.0f, 8, false};
        auto offer = [&](const Cand &c) {
#pragma unroll
            for (int s = 0; s < NR; s++)
                if (s == nr) slot[s] = c;
            nr++;
        };
#ifndef PS_DBG_NO_RC
        if constexpr (HAS_CUBE) {
            const float h = sc.half;
            static_for<0, PM_NUM_SPHERES>([&](auto SS) {
                constexpr int S = decltype(SS)::value;
                constexpr SphereDef s = sphere_def(S);
                V3 loc = tmul(Rc, geo.spw[S] - cb.pos);
                V3 cl = mk(fminf(fmaxf(loc.x, -h), h), fminf(fmaxf(loc.y, -h), h), fminf(fmaxf(loc.z, -h), h));
                V3 dif = loc - cl;
                float dn = norm(dif);
                V3 nl;
                float dist;
                if (dn > 1e-9f) {
                    nl = dif * (1.0f / dn);
                    dist = dn - (float)s.r;
                } else {
                    float bx = h - fabsf(loc.x), by = h - fabsf(loc.y), bz = h - fabsf(loc.z);
                    int ax = 0;
                    float best = bx;
                    if (by < best) { best = by; ax = 1; }
                    if (bz < best) { best = bz; ax = 2; }
                    float sg;
                    if (ax == 0) { sg = loc.x >= 0.0f ? 1.0f : -1.0f; nl = mk(sg, 0, 0); cl.x = sg * h; }
                    else if (ax == 1) { sg = loc.y >= 0.0f ? 1.0f : -1.0f; nl = mk(0, sg, 0); cl.y = sg * h; }
                    else { sg = loc.z >= 0.0f ? 1.0f : -1.0f; nl = mk(0, 0, sg); cl.z = sg * h; }
                    dist = -best - (float)s.r;
                }
                if (nr < NR && dist < (float)PM_CONTACT_MARGIN_SPHERE) {
                    V3 n = mul(Rc, nl);
                    offer(Cand{geo.spw[S] - n * (float)s.r, cb.pos + mul(Rc, cl), n, dist,
                               (float)(s.mu * PM_DEFAULT_FRICTION), s.link, true});
                }
            });
        }
        static_for<0, PM_NUM_SPHERES>([&](auto SS) {
            constexpr int S = decltype(SS)::value;
            constexpr SphereDef s = sphere_def(S);
            float top;
            if (nr < NR && ground_top(sc, geo.spw[S].x, geo.spw[S].y, top)) {
                float dist = geo.spw[S].z - (float)s.r - top;
                if (dist < (float)PM_CONTACT_MARGIN_SPHERE) {
                    V3 pA = geo.spw[S] - mk(0, 0, (float)s.r);
                    offer(Cand{pA, pA, mk(0, 0, 1), dist, (float)(s.mu * PM_DEFAULT_FRICTION), s.link, false});
                }
            }
        });
#endif
        // 2) rows of each used slot: J (registers), M^-1 J^T (LDS), rhs, bounds
#pragma unroll
        for (int sl = 0; sl < NR; sl++) {
            if (sl < nr) {
                const Cand &cd = slot[sl];
                RobotContact &c = rc[sl];
                V3 dirs[3];
                dirs[0] = cd.n;
                plane_space(cd.n, dirs[1], dirs[2]);
                c.mu = cd.mu;
                V3 p = cd.pA - sc.base;
                V3 rB = cd.pB - cb.pos;
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
                        lds.at(sl, j, a) = s;
                        den += c.J[j][a] * s;
                    }
                    float rel = jrow_dot(c.J[j], v1);
                    c.rn[j] = cd.on_cube ? cross(rB, dj) : mk(0, 0, 0);
                    c.dir[j] = cd.on_cube ? dj : mk(0, 0, 0);  // cube side only
                    if (cd.on_cube) {
                        den += dot(c.rn[j], c.rn[j]) * inv_I + dot(dj, dj) * inv_m;
                        rel -= dot(c.rn[j], cw1) + dot(dj, cv1);
                    }
                    c.dinv[j] = den > 2.2204460492503131e-16f ? 1.0f / den : 0.0f;
                    c.lam[j] = 0.0f;
                    if (j == 0) {
                        float pen = cd.dist + (float)PM_LINEAR_SLOP;
                        float velerr = -rel, poserr = 0.0f;
                        if (pen > 0.0f) velerr -= pen / dt;
                        else poserr = -pen * (float)PM_ERP / dt;
                        bool combined = pen > (float)PM_SPLIT_PENETRATION_THRESHOLD;
                        c.rhs[0] = (combined ? poserr + velerr : velerr) * c.dinv[0];
                    } else {
                        c.rhs[j] = -rel * c.dinv[j];
                    }
                }
            } else {
                // unused slot: all-zero rows (finite M^-1 J^T too) are no-ops in PGS
                RobotContact &c = rc[sl];
                c.mu = 0.0f;
#pragma unroll
                for (int j = 0; j < 3; j++) {
#pragma unroll
                    for (int a = 0; a < 9; a++) {
                        c.J[j][a] = 0.0f;
                        lds.at(sl, j, a) = 0.0f;
                    }
                    c.dir[j] = mk(0, 0, 0);
                    c.rn[j] = mk(0, 0, 0);
                    c.rhs[j] = c.lam[j] = c.dinv[j] = 0.0f;
                }
            }
        }
    }
    PS_PHASE(3);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int d = 0; d < 9; d++) {
        lds.stash(d) = q[d];
        lds.stash(9 + d) = v1[d];
        lds.stash(18 + d) = split_dq[d];
    }
    if constexpr (HAS_CUBE) {
        lds.stash(27) = cw1.x; lds.stash(28) = cw1.y; lds.stash(29) = cw1.z;
        lds.stash(30) = cv1.x; lds.stash(31) = cv1.y; lds.stash(32) = cv1.z;
        lds.stash(33) = cb.pos.x; lds.stash(34) = cb.pos.y; lds.stash(35) = cb.pos.z;
        lds.stash(36) = cb.quat.x; lds.stash(37) = cb.quat.y; lds.stash(38) = cb.quat.z; lds.stash(39) = cb.quat.w;
    }

    // ---- projected Gauss-Seidel
    // Every row kind is gated by a wave-uniform ballot (a scalar branch: the
    // block runs if any lane of the wave needs it); inside, lanes without the
    // row hold all-zero data or [0, 0] bounds, which leave every impulse and
    // velocity untouched, so no per-lane exec masking or phi copies remain.
    float dv[9];
#pragma unroll
    for (int d = 0; d < 9; d++) dv[d] = 0.0f;
    V3 dw = mk(0, 0, 0), dvl = mk(0, 0, 0);
    float res;
    MJStore L = lds;

    auto joint_row = [&](int d, float sgn, float rhs, float &lam, float lo, float hi) {
        float dl = rhs - dinvj[d] * (sgn * dv[d]);
        float nl = fminf(fmaxf(lam + dl, lo), hi);
        dl = nl - lam;
        lam = nl;
        float f = sgn * dl;
        if constexpr (MI_REGS) {
#pragma unroll
            for (int a = 0; a < 9; a++) dv[a] += Mi[sidx(a, d)] * f;
        } else {
#pragma unroll
            for (int a = 0; a < 9; a++) dv[a] += L.mi(sidx(a, d)) * f;
        }
        float x = dl * (MI_REGS ? Mi[sidx(d, d)] : (float)L.mi(sidx(d, d)));  // residual dl / dinv
        res = fmaxf(res, x * x);
    };
    auto limit_row = [&](int d) {
        if (__builtin_amdgcn_ballot_w64((lim_on >> d) & 1u)) {
            float sgn = (lim_up >> d) & 1u ? -1.0f : 1.0f;
            float hi = (lim_on >> d) & 1u ? (float)PM_LIMIT_MAX_IMPULSE : 0.0f;
            joint_row(d, sgn, lim_rhs[d], lim_lam[d], 0.0f, hi);
        }
    };
    auto motor_row = [&](int d) {
        float imp = STD_MOTORS ? (float)(joint_force(d) * PM_TIMESTEP) : mt.imp[d];
        joint_row(d, 1.0f, mot_rhs[d], mot_lam[d], -imp, imp);
    };

    auto contacts = [&]() {
        // normals: ground contacts then gripper contacts
        if constexpr (HAS_CUBE) {
#pragma unroll
            for (int c = 0; c < NG; c++)
                if (__builtin_amdgcn_ballot_w64(c < ng)) {
                    GroundContact &g = gc[c];
                    V3 rn = mk(g.r.y, -g.r.x, 0.0f);  // r x (0,0,1)
                    float dl = g.rhs[0] - g.dinv[0] * (dot(rn, dw) + dvl.z);
                    float nl = fminf(fmaxf(g.lam[0] + dl, 0.0f), (float)PM_CONTACT_UPPER);
                    dl = nl - g.lam[0];
                    g.lam[0] = nl;
                    dw = dw + rn * (dl * inv_I);
                    dvl.z += dl * inv_m;
                    float x = dl * res_scale(g.dinv[0]);
                    res = fmaxf(res, x * x);
                }
        }
#pragma unroll
        for (int c = 0; c < NR; c++)
            if (__builtin_amdgcn_ballot_w64(c < nr)) {
                RobotContact &r = rc[c];
                float jv = jrow_dot(r.J[0], dv);
                if (HAS_CUBE) jv -= dot(r.rn[0], dw) + dot(r.dir[0], dvl);
                float dl = r.rhs[0] - r.dinv[0] * jv;
                float nl = fminf(fmaxf(r.lam[0] + dl, 0.0f), (float)PM_CONTACT_UPPER);
                dl = nl - r.lam[0];
                r.lam[0] = nl;
#pragma unroll
                for (int a = 0; a < 9; a++) dv[a] += L.at(c, 0, a) * dl;
                if (HAS_CUBE) {
                    dw = dw - r.rn[0] * (dl * inv_I);
                    dvl = dvl - r.dir[0] * (dl * inv_m);
                }
                float x = dl * res_scale(r.dinv[0]);
                res = fmaxf(res, x * x);
            }
        // friction cones
        if constexpr (HAS_CUBE) {
#pragma unroll
            for (int c = 0; c < NG; c++)
                if (__builtin_amdgcn_ballot_w64(c < ng)) {
                    GroundContact &g = gc[c];
                    V3 r1 = mk(g.r.z, 0.0f, -g.r.x);  // r x (0,-1,0)
                    V3 r2 = mk(0.0f, g.r.z, -g.r.y);  // r x (1,0,0)
                    float dla = g.rhs[1] - g.dinv[1] * (dot(r1, dw) - dvl.y);
                    float dlb = g.rhs[2] - g.dinv[2] * (dot(r2, dw) + dvl.x);
                    float sa = g.lam[1] + dla, sb = g.lam[2] + dlb;
                    float lim = (float)(PM_DEFAULT_FRICTION * PM_DEFAULT_FRICTION) * fmaxf(g.lam[0], 0.0f);
                    float m2 = sa * sa + sb * sb;
                    // |f| > mu N: project onto the cone (lim * rsq(m2) <= 1 there)
                    float s = m2 > lim * lim ? lim * rsqrtf(m2) : 1.0f;
                    sa *= s;
                    sb *= s;
                    dla = sa - g.lam[1];
                    dlb = sb - g.lam[2];
                    g.lam[1] = sa;
                    g.lam[2] = sb;
                    dw = dw + (r1 * dla + r2 * dlb) * inv_I;
                    dvl = dvl + mk(dlb, -dla, 0.0f) * inv_m;
                    float ra = dla * res_scale(g.dinv[1]), rb = dlb * res_scale(g.dinv[2]);
                    float x = fabsf(ra) > fabsf(rb) ? ra : rb;
                    res = fmaxf(res, x * x);
                }
        }
#pragma unroll
        for (int c = 0; c < NR; c++)
            if (__builtin_amdgcn_ballot_w64(c < nr)) {
                RobotContact &r = rc[c];
                float ja = jrow_dot(r.J[1], dv), jb = jrow_dot(r.J[2], dv);
                if (HAS_CUBE) {
                    ja -= dot(r.rn[1], dw) + dot(r.dir[1], dvl);
                    jb -= dot(r.rn[2], dw) + dot(r.dir[2], dvl);
                }
                float dla = r.rhs[1] - r.dinv[1] * ja, dlb = r.rhs[2] - r.dinv[2] * jb;
                float sa = r.lam[1] + dla, sb = r.lam[2] + dlb;
                float lim = r.mu * fmaxf(r.lam[0], 0.0f);
                float m2 = sa * sa + sb * sb;
                float s = m2 > lim * lim ? lim * rsqrtf(m2) : 1.0f;
                sa *= s;
                sb *= s;
                dla = sa - r.lam[1];
                dlb = sb - r.lam[2];
                r.lam[1] = sa;
                r.lam[2] = sb;
#pragma unroll
                for (int a = 0; a < 9; a++) dv[a] += L.at(c, 1, a) * dla + L.at(c, 2, a) * dlb;
                if (HAS_CUBE) {
                    dw = dw - (r.rn[1] * dla + r.rn[2] * dlb) * inv_I;
                    dvl = dvl - (r.dir[1] * dla + r.dir[2] * dlb) * inv_m;
                }
                float ra = dla * res_scale(r.dinv[1]), rb = dlb * res_scale(r.dinv[2]);
                float x = fabsf(ra) > fabsf(rb) ? ra : rb;
                res = fmaxf(res, x * x);
            }
    };

    // btSequentialImpulseConstraintSolver alternates the order of the
    // non-contact rows by iteration parity: even iterations run them in
    // reverse (motors 8..0, then limits 8..0), odd ones forward (limits 0..8,
    // then motors 0..8).  The loop is unrolled by two so both orders are
    // straight-line code; each env still stops at its own residual.
    static_assert(PM_SOLVER_ITERATIONS % 2 == 0, "iteration pairs");
    for (int it = 0; it < PM_SOLVER_ITERATIONS; it += 2) {
        L = lds.opaque();
        res = 0.0f;
#pragma unroll
        for (int d = 8; d >= 0; d--) motor_row(d);
        if (__builtin_amdgcn_ballot_w64(lim_on != 0u)) {
#pragma unroll
            for (int d = 8; d >= 0; d--) limit_row(d);
        }
        contacts();
        if (res <= (float)PM_SOLVER_RESIDUAL_THRESHOLD) break;
        L = lds.opaque();
        res = 0.0f;
        if (__builtin_amdgcn_ballot_w64(lim_on != 0u)) {
#pragma unroll
            for (int d = 0; d < 9; d++) limit_row(d);
        }
#pragma unroll
        for (int d = 0; d < 9; d++) motor_row(d);
        contacts();
        if (res <= (float)PM_SOLVER_RESIDUAL_THRESHOLD) break;
    }

    PS_PHASE(4);
    {
        // reload through an opaque address: no store-to-load forwarding, so
        // the registers really were free during the solve
        MJStore S = lds.opaque();
#pragma unroll
        for (int d = 0; d < 9; d++) {
            q[d] = S.stash(d);
            v1[d] = S.stash(9 + d);
            split_dq[d] = S.stash(18 + d);
        }
        if constexpr (HAS_CUBE) {
            cw1 = mk(S.stash(27), S.stash(28), S.stash(29));
            cv1 = mk(S.stash(30), S.stash(31), S.stash(32));
            cb.pos = mk(S.stash(33), S.stash(34), S.stash(35));
            cb.quat = Q4{S.stash(36), S.stash(37), S.stash(38), S.stash(39)};
        }
    }
    // ---- integrate (btMultiBody::stepPositionsMultiDof)
#pragma unroll
    for (int d = 0; d < 9; d++) {
        qd[d] = v1[d] + dv[d];
        q[d] += dt * qd[d] + split_dq[d];
    }
    if constexpr (HAS_CUBE) {
        cb.omg = cw1 + dw;
        cb.vel = cv1 + dvl;
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
