// ps_render.h — batched camera images of the Panda scenes (pybullet.py:69-264):
// the camera matrices of computeViewMatrixFromYawPitchRoll /
// computeProjectionMatrixFOV, a ray-cast getCameraImage (one lane per pixel,
// every env of the batch) and render()'s deprojection of the depth buffer
// into a filtered world point cloud.
//
// getCameraImage rasterises the URDF meshes; the Panda meshes are not in this
// image, so the arm is drawn as capsules between its joint frames plus the
// gripper's contact spheres.  Table, plane, objects and
// ghost targets are exact.  Depth follows the OpenGL convention the
// reference's deprojection assumes: window depth in [0, 1] of the projection
// matrix, 1 where nothing is hit.
#pragma once

#include "ps_physics.h"

namespace ps {

// visual roles (ps_visual.rgba rows)
enum { VR_PLANE = 0, VR_TABLE, VR_OBJECT1, VR_OBJECT2, VR_TARGET1, VR_TARGET2, VR_ROBOT, VR_BACKGROUND };

constexpr int RENDER_CAPSULES = 8;
// per-env primitive table written by k_render_prep, read into LDS by k_render
//   capsules: a.xyz b.xyz r            (8 x 7)
//   spheres:  c.xyz r                  (6 x 4)
//   objects:  pos.xyz R(row-major 9)   (2 x 12)
//   targets:  pos.xyz R(row-major 9)   (2 x 12)
constexpr int RP_CAPS = 0;
constexpr int RP_SPH = RP_CAPS + RENDER_CAPSULES * 7;
constexpr int RP_OBJ = RP_SPH + PM_NUM_SPHERES * 4;
constexpr int RP_TGT = RP_OBJ + 2 * 12;
constexpr int RP_ARM_BOUND = RP_TGT + 2 * 12;  // centre.xyz, radius of a sphere around every arm primitive
constexpr int RENDER_PRIM_FLOATS = RP_ARM_BOUND + 4;

struct Hit {
    float t;
    V3 n;
};

// v_rcp_f32 (1 ulp): the ray tests only need image-quality reciprocals, and the
// IEEE division would cost ten instructions each
PS_D float frcp(float x) { return __builtin_amdgcn_rcpf(x); }

// slab test of the ray (o, d) against the box of half extents h centred at c
// with rotation R (columns = box axes); t in [tmin, t.t) updates the hit
PS_D bool ray_box(V3 o, V3 d, V3 c, const M3 &R, V3 h, float tmin, Hit &hit) {
    V3 lo = tmul(R, o - c), ld = tmul(R, d);
    float t0 = -3.0e38f, t1 = 3.0e38f;
    int ax = 0;
    float sg = 1.0f;
    const float oo[3] = {lo.x, lo.y, lo.z}, dd[3] = {ld.x, ld.y, ld.z}, hh[3] = {h.x, h.y, h.z};
#pragma unroll
    for (int k = 0; k < 3; k++) {
        float inv = frcp(dd[k]);  // +-inf for an axis-parallel ray: the slab test still holds
        float ta = (-hh[k] - oo[k]) * inv, tb = (hh[k] - oo[k]) * inv;
        float tn = fminf(ta, tb), tf = fmaxf(ta, tb);
        if (tn > t0) {
            t0 = tn;
            ax = k;
            sg = dd[k] > 0.0f ? -1.0f : 1.0f;
        }
        t1 = fminf(t1, tf);
    }
    if (!(t0 <= t1) || t0 < tmin || t0 >= hit.t) return false;
    hit.t = t0;
    // selects, not col(R, ax): a runtime column index would send R to scratch
    V3 n = ax == 0 ? mk(R.m[0], R.m[3], R.m[6]) : ax == 1 ? mk(R.m[1], R.m[4], R.m[7]) : mk(R.m[2], R.m[5], R.m[8]);
    hit.n = n * sg;
    return true;
}

// upright (local z) capped cylinder of radius r and half height hh
PS_D bool ray_cylinder(V3 o, V3 d, V3 c, const M3 &R, float r, float hh, float tmin, Hit &hit) {
    V3 lo = tmul(R, o - c), ld = tmul(R, d);
    bool got = false;
    float a = ld.x * ld.x + ld.y * ld.y;
    if (a > 1e-20f) {
        float b = lo.x * ld.x + lo.y * ld.y, cc = lo.x * lo.x + lo.y * lo.y - r * r;
        float disc = b * b - a * cc;
        if (disc >= 0.0f) {
            float t = (-b - sqrtf(disc)) * frcp(a);
            float z = lo.z + t * ld.z;
            if (t >= tmin && t < hit.t && fabsf(z) <= hh) {
                hit.t = t;
                float ir = frcp(r);
                hit.n = mul(R, mk((lo.x + t * ld.x) * ir, (lo.y + t * ld.y) * ir, 0.0f));
                got = true;
            }
        }
    }
    if (fabsf(ld.z) > 1e-20f) {
#pragma unroll
        for (int s = 0; s < 2; s++) {
            float zc = s ? hh : -hh;
            float t = (zc - lo.z) * frcp(ld.z);
            float x = lo.x + t * ld.x, y = lo.y + t * ld.y;
            if (t >= tmin && t < hit.t && x * x + y * y <= r * r) {
                hit.t = t;
                hit.n = col(R, 2) * (s ? 1.0f : -1.0f);
                got = true;
            }
        }
    }
    return got;
}

// does the ray meet the sphere (c, r) at some t < tmax?  (culling only)
PS_D bool ray_meets_sphere(V3 o, V3 d, V3 c, float r, float tmax) {
    V3 oc = o - c;
    float a = dot(d, d), b = dot(oc, d), cc = dot(oc, oc) - r * r;
    if (cc <= 0.0f) return true;  // the eye is inside
    float disc = b * b - a * cc;
    return disc >= 0.0f && b < 0.0f && (-b - sqrtf(disc)) < tmax * a;
}

PS_D bool ray_sphere(V3 o, V3 d, V3 c, float r, float tmin, Hit &hit) {
    V3 oc = o - c;
    float a = dot(d, d), b = dot(oc, d), cc = dot(oc, oc) - r * r;
    float disc = b * b - a * cc;
    if (disc < 0.0f) return false;
    float t = (-b - sqrtf(disc)) * frcp(a);
    if (t < tmin || t >= hit.t) return false;
    hit.t = t;
    V3 p = oc + d * t;
    hit.n = p * frcp(r);
    return true;
}

// capsule = segment [pa, pb] swept by radius r
PS_D bool ray_capsule(V3 o, V3 d, V3 pa, V3 pb, float r, float tmin, Hit &hit) {
    V3 ba = pb - pa, oa = o - pa;
    float baba = dot(ba, ba), bard = dot(ba, d), baoa = dot(ba, oa), rdoa = dot(d, oa), oaoa = dot(oa, oa);
    float dd = dot(d, d);
    float a = baba * dd - bard * bard, b = baba * rdoa - baoa * bard, c = baba * oaoa - baoa * baoa - r * r * baba;
    float h = b * b - a * c;
    if (h < 0.0f) return false;
    float t = (-b - sqrtf(h)) * frcp(a);
    float y = baoa + t * bard;
    if (!(y > 0.0f && y < baba)) {
        // caps
        V3 oc = y <= 0.0f ? oa : o - pb;
        b = dot(d, oc);
        c = dot(oc, oc) - r * r;
        h = b * b - dd * c;
        if (h < 0.0f) return false;
        t = (-b - sqrtf(h)) * frcp(dd);
    }
    if (!(t >= tmin && t < hit.t)) return false;
    V3 p = o + d * t - pa;
    float s = fminf(fmaxf(dot(p, ba) * frcp(baba), 0.0f), 1.0f);
    V3 n = p - ba * s;
    hit.t = t;
    hit.n = n * frcp(r);
    return true;
}

}  // namespace ps

// ---------------------------------------------------------------- camera
// Host arithmetic (no GPU): b3ComputeViewMatrixFromYawPitchRoll with
// upAxisIndex 2 and b3ComputeProjectionMatrixFOV, column-major float[16] as
// pybullet returns them (pybullet.py:90-101, 173-183).
namespace ps_camera_math {

inline void view_from_yaw_pitch_roll(const float target[3], double distance, double yaw, double pitch, double roll,
                                     float view[16]) {
    const double d2r = 3.14159265358979323846 / 180.0;
    double y = yaw * d2r, p = pitch * d2r, r = roll * d2r;
    // eyeRot.setEulerZYX(yaw, roll, pitch): R = Rz(yaw) Ry(roll) Rx(pitch)
    double cy = cos(y), sy = sin(y), cr = cos(r), sr = sin(r), cp = cos(p), sp = sin(p);
    double Rz[9] = {cy, -sy, 0, sy, cy, 0, 0, 0, 1};
    double Ry[9] = {cr, 0, sr, 0, 1, 0, -sr, 0, cr};
    double Rx[9] = {1, 0, 0, 0, cp, -sp, 0, sp, cp};
    double T[9], R[9];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            T[i * 3 + j] = 0;
            for (int k = 0; k < 3; k++) T[i * 3 + j] += Ry[i * 3 + k] * Rx[k * 3 + j];
        }
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            R[i * 3 + j] = 0;
            for (int k = 0; k < 3; k++) R[i * 3 + j] += Rz[i * 3 + k] * T[k * 3 + j];
        }
    // forward axis 1: eye at -distance along y, up +z, both rotated
    double eye0[3] = {0.0, -distance, 0.0}, up0[3] = {0.0, 0.0, 1.0};
    double eye[3], up[3];
    for (int i = 0; i < 3; i++) {
        eye[i] = R[i * 3 + 0] * eye0[0] + R[i * 3 + 1] * eye0[1] + R[i * 3 + 2] * eye0[2] + target[i];
        up[i] = R[i * 3 + 0] * up0[0] + R[i * 3 + 1] * up0[1] + R[i * 3 + 2] * up0[2];
    }
    // b3ComputeViewMatrixFromPositions: gluLookAt
    double f[3] = {target[0] - eye[0], target[1] - eye[1], target[2] - eye[2]};
    double fn = sqrt(f[0] * f[0] + f[1] * f[1] + f[2] * f[2]);
    for (double &v : f) v /= fn;
    double un = sqrt(up[0] * up[0] + up[1] * up[1] + up[2] * up[2]);
    for (double &v : up) v /= un;
    double s[3] = {f[1] * up[2] - f[2] * up[1], f[2] * up[0] - f[0] * up[2], f[0] * up[1] - f[1] * up[0]};
    double sn = sqrt(s[0] * s[0] + s[1] * s[1] + s[2] * s[2]);
    for (double &v : s) v /= sn;
    double u[3] = {s[1] * f[2] - s[2] * f[1], s[2] * f[0] - s[0] * f[2], s[0] * f[1] - s[1] * f[0]};
    for (int i = 0; i < 3; i++) {
        view[i * 4 + 0] = (float)s[i];
        view[i * 4 + 1] = (float)u[i];
        view[i * 4 + 2] = (float)-f[i];
        view[i * 4 + 3] = 0.0f;
    }
    view[12] = (float)-(s[0] * eye[0] + s[1] * eye[1] + s[2] * eye[2]);
    view[13] = (float)-(u[0] * eye[0] + u[1] * eye[1] + u[2] * eye[2]);
    view[14] = (float)(f[0] * eye[0] + f[1] * eye[1] + f[2] * eye[2]);
    view[15] = 1.0f;
}

inline void projection_fov(double fov, double aspect, double nearv, double farv, float proj[16]) {
    double ys = 1.0 / tan(3.14159265358979323846 / 180.0 * fov / 2.0), xs = ys / aspect;
    for (int i = 0; i < 16; i++) proj[i] = 0.0f;
    proj[0] = (float)xs;
    proj[5] = (float)ys;
    proj[10] = (float)((farv + nearv) / (nearv - farv));
    proj[11] = -1.0f;
    proj[14] = (float)(2.0 * farv * nearv / (nearv - farv));
}

// inverse of a row-major 4x4 (Gauss-Jordan, partial pivoting); false if singular
inline bool invert4(const double A[16], double out[16]) {
    double m[4][8];
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 8; j++) m[i][j] = j < 4 ? A[i * 4 + j] : (j - 4 == i ? 1.0 : 0.0);
    for (int c = 0; c < 4; c++) {
        int p = c;
        for (int r = c + 1; r < 4; r++)
            if (fabs(m[r][c]) > fabs(m[p][c])) p = r;
        if (m[p][c] == 0.0) return false;
        if (p != c)
            for (int j = 0; j < 8; j++) {
                double t = m[c][j];
                m[c][j] = m[p][j];
                m[p][j] = t;
            }
        double iv = 1.0 / m[c][c];
        for (int j = 0; j < 8; j++) m[c][j] *= iv;
        for (int r = 0; r < 4; r++)
            if (r != c) {
                double f = m[r][c];
                for (int j = 0; j < 8; j++) m[r][j] -= f * m[c][j];
            }
    }
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) out[i * 4 + j] = m[i][j + 4];
    return true;
}

}  // namespace ps_camera_math
