"""TEST INFRASTRUCTURE ONLY (tests/, never the product path): numpy restatement
of the camera-image path of panda_gym/pybullet.py (§8(f) rank 4), the checker
for libpandasim's ps_camera / ps_render / ps_deproject_*.

* camera():   computeViewMatrixFromYawPitchRoll(upAxisIndex=2) and
              computeProjectionMatrixFOV (pybullet.py:69-107).  PyBullet is not
              installed, so this is restated from Bullet3's published
              b3ComputeViewMatrixFromYawPitchRoll (eye rotation as the
              quaternion of b3Quaternion::setEulerZYX(yaw, roll, pitch)) --
              parity of the matrices is UNPINNED; tran_pix_world and everything
              downstream are pinned by the reference-generated goldens
              (tests/golden/make_render_golden.py).
* deproject_image(): render()'s post-processing (pybullet.py:193-262), the same
              numpy operations in the same order.
* deproject():  PyBullet.deproject (pybullet.py:109-146).
* raycast_depth(): an independent, vectorised ray caster of the scene the
              kernels draw (plane, table, objects, the arm's capsule proxies and
              gripper spheres), for small images: the GPU depth buffer is
              checked against it.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

import oracle as O

# capsule proxies of the arm: (link frame index a or -1 = base origin, b, radius);
# the hand bar is handled separately (same constants as csrc/pandasim.hip k_render_prep)
ARM_CAPSULES = [(-1, 0, 0.07), (1, 2, 0.065), (2, 3, 0.06), (3, 4, 0.06), (5, 6, 0.055), (6, 7, 0.05)]
WRIST = (0.0, 0.0, 0.04)  # flange (link 8 origin) -> palm, in the hand frame, radius 0.045
HAND_BAR = ((0.0, -0.09, 0.03), (0.0, 0.09, 0.03), 0.03)
PLANE_TOP, TABLE_TOP = -0.4, 0.0


def _quat_zyx(yaw, pitch, roll):
    """b3Quaternion::setEulerZYX(yawZ, pitchY, rollX) -> (x, y, z, w)."""
    hy, hp, hr = yaw * 0.5, pitch * 0.5, roll * 0.5
    cy, sy, cp, sp, cr, sr = np.cos(hy), np.sin(hy), np.cos(hp), np.sin(hp), np.cos(hr), np.sin(hr)
    return np.array([sr * cp * cy - cr * sp * sy, cr * sp * cy + sr * cp * sy, cr * cp * sy - sr * sp * cy,
                     cr * cp * cy + sr * sp * sy])


def _quat_mat(q):
    x, y, z, w = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def camera(target=(0.0, 0.0, 0.0), distance=1.4, yaw=45.0, pitch=-30.0, roll=0.0, width=480, height=480):
    """-> (view tuple(16), proj tuple(16), tran_pix_world (4, 4)) as get_cam2world_transforms returns them."""
    d2r = np.pi / 180.0
    target = np.asarray(target, np.float64)
    R = _quat_mat(_quat_zyx(yaw * d2r, roll * d2r, pitch * d2r))  # upAxisIndex 2: setEulerZYX(yaw, roll, pitch)
    eye = R @ np.array([0.0, -distance, 0.0]) + target
    up = R @ np.array([0.0, 0.0, 1.0])
    f = target - eye
    f /= np.linalg.norm(f)
    up = up / np.linalg.norm(up)
    s = np.cross(f, up)
    s /= np.linalg.norm(s)
    u = np.cross(s, f)
    V = np.eye(4)
    V[0, :3], V[1, :3], V[2, :3] = s, u, -f
    V[0, 3], V[1, 3], V[2, 3] = -s @ eye, -u @ eye, f @ eye
    ys = 1.0 / np.tan(d2r * 60.0 / 2.0)
    near, far = 0.1, 100.0
    P = np.zeros((4, 4))
    P[0, 0], P[1, 1] = ys / (width / height), ys
    P[2, 2], P[2, 3], P[3, 2] = (far + near) / (near - far), 2 * far * near / (near - far), -1.0
    view = tuple(float(v) for v in V.astype(np.float32).reshape(-1, order="F"))
    proj = tuple(float(v) for v in P.astype(np.float32).reshape(-1, order="F"))
    Pm = np.asarray(proj).reshape([4, 4], order="F")
    Vm = np.asarray(view).reshape([4, 4], order="F")
    return view, proj, np.linalg.inv(np.matmul(Pm, Vm))


def deproject_image(depth, tran_pix_world, rgb=None):
    """render()'s arithmetic after getCameraImage (pybullet.py:193-262) on one
    depth buffer (h, w) -> points (N, 3), colors (N, 3) or None, pixels_2d (N, 2),
    and the flat pixel indices kept."""
    height, width = depth.shape
    y, x = np.mgrid[-1:1:2 / height, -1:1:2 / width]
    y *= -1.
    x, y, z = x.reshape(-1), y.reshape(-1), np.asarray(depth, np.float64).reshape(-1)
    h = np.ones_like(z)
    pixels = np.stack([x, y, z, h], axis=1)
    flat = np.arange(height * width)
    idxs = z < 0.99
    pixels = pixels[idxs]
    flat = flat[idxs]
    colors = None if rgb is None else rgb[:, :, :3].reshape(height * width, 3)[idxs]
    pixels[:, 2] = 2 * pixels[:, 2] - 1
    points = np.matmul(tran_pix_world, pixels.T).T
    points /= points[:, 3:4]
    points = points[:, :3]
    pixels_2d = pixels[:, :2]
    pixels_2d += np.array([1., 1.])
    pixels_2d /= 2
    pixels_2d[:, 0] *= width
    pixels_2d[:, 1] *= height
    pixels_2d[:, 1] = height - pixels_2d[:, 1]
    keep = (points[:, 2] > 0.0) & (points[:, 0] < 0.2) & (points[:, 2] < 0.67) & (points[:, 0] > -0.5)
    return points[keep], None if colors is None else colors[keep], pixels_2d[keep], flat[keep]


def deproject(depth, pixels, tran_pix_world, width=480, height=480):
    """PyBullet.deproject (pybullet.py:109-146)."""
    pixels = np.asarray(pixels)
    x = pixels[:, 0] * 1 / width
    x = x * 2 - 1
    y = (height - pixels[:, 1]) * 1 / height
    y = y * 2 - 1
    z = 2 * np.asarray(depth, np.float64)[pixels[:, 1], pixels[:, 0]] - 1
    p = np.stack([x, y, z, np.ones_like(z)], axis=1)
    pts = np.matmul(tran_pix_world, p.T).T
    pts /= pts[:, 3:4]
    return pts[:, :3]


# ------------------------------------------------------------ ray caster
def scene_primitives(cfg, env):
    """Capsules [(a, b, r)], spheres [(c, r)] of the arm (fp64 oracle FK)."""
    R = (C.c_double * 9 * 12)()
    o = (C.c_double * 3 * 12)()
    O.lib().po_link_frames.argtypes = [C.POINTER(O.Config), C.POINTER(O.Env), C.c_void_p, C.c_void_p]
    O.lib().po_link_frames(C.byref(cfg), C.byref(env), R, o)
    Rn = np.array([[R[i][k] for k in range(9)] for i in range(12)]).reshape(12, 3, 3)
    on = np.array([[o[i][k] for k in range(3)] for i in range(12)])
    base = np.array([cfg.base[k] for k in range(3)], np.float64)
    caps = []
    for a, b, r in ARM_CAPSULES:
        caps.append((base if a < 0 else on[a], on[b], r))
    caps.append((on[7], on[8] + Rn[8] @ np.array(WRIST), 0.045))
    ha, hb, hr = HAND_BAR
    caps.append((on[8] + Rn[8] @ np.array(ha), on[8] + Rn[8] @ np.array(hb), hr))
    ns = O.lib().po_num_spheres()
    c = (C.c_double * 3 * ns)()
    rr = (C.c_double * ns)()
    O.lib().po_gripper_spheres.argtypes = [C.POINTER(O.Config), C.POINTER(O.Env), C.c_void_p, C.c_void_p]
    O.lib().po_gripper_spheres(C.byref(cfg), C.byref(env), c, rr)
    sph = [(np.array([c[s][k] for k in range(3)]), rr[s]) for s in range(ns)]
    return caps, sph


def _rays(view, proj, width, height):
    V = np.asarray(view, np.float64).reshape(4, 4, order="F")
    P = np.asarray(proj, np.float64).reshape(4, 4, order="F")
    Rv, t = V[:3, :3], V[:3, 3]
    eye = -Rv.T @ t
    s, u, f = Rv[0], Rv[1], -Rv[2]
    j, i = np.meshgrid(np.arange(width), np.arange(height))
    xn = -1 + (2 * j + 1) / width
    yn = 1 - (2 * i + 1) / height
    d = (xn[..., None] / P[0, 0]) * s + (yn[..., None] / P[1, 1]) * u + f
    near = P[2, 3] / (P[2, 2] - 1)
    far = P[2, 3] / (P[2, 2] + 1)
    return eye, d.reshape(-1, 3), P, near, far


def _box(eye, d, c, R, h):
    lo = (eye - c) @ R
    ld = d @ R
    with np.errstate(divide="ignore", invalid="ignore"):
        ta = (-np.asarray(h) - lo) / ld
        tb = (np.asarray(h) - lo) / ld
    t0 = np.nanmax(np.minimum(ta, tb), axis=1)
    t1 = np.nanmin(np.maximum(ta, tb), axis=1)
    return np.where(t0 <= t1, t0, np.inf)


def _sphere(eye, d, c, r):
    oc = eye - c
    a = np.sum(d * d, 1)
    b = d @ oc
    cc = oc @ oc - r * r
    disc = b * b - a * cc
    with np.errstate(invalid="ignore"):
        t = (-b - np.sqrt(disc)) / a
    return np.where(disc >= 0, t, np.inf)


def _capsule(eye, d, pa, pb, r):
    t = np.full(d.shape[0], np.inf)
    # sphere caps, then the cylinder body (axis segment, clipped to the segment)
    t = np.minimum(t, _sphere(eye, d, pa, r))
    t = np.minimum(t, _sphere(eye, d, pb, r))
    ba = pb - pa
    L2 = ba @ ba
    oa = eye - pa
    dp = d - np.outer(d @ ba / L2, ba)
    op = oa - (oa @ ba / L2) * ba
    a = np.sum(dp * dp, 1)
    b = dp @ op
    cc = op @ op - r * r
    disc = b * b - a * cc
    with np.errstate(invalid="ignore", divide="ignore"):
        tc = (-b - np.sqrt(disc)) / a
    y = (oa @ ba) + tc * (d @ ba)
    ok = (disc >= 0) & (y > 0) & (y < L2)
    return np.minimum(t, np.where(ok, tc, np.inf))


def _cylinder(eye, d, c, R, r, hh):
    lo = (eye - c) @ R
    ld = d @ R
    a = ld[:, 0] ** 2 + ld[:, 1] ** 2
    b = lo[0] * ld[:, 0] + lo[1] * ld[:, 1]
    cc = lo[0] ** 2 + lo[1] ** 2 - r * r
    disc = b * b - a * cc
    with np.errstate(invalid="ignore", divide="ignore"):
        ts = (-b - np.sqrt(disc)) / a
        z = lo[2] + ts * ld[:, 2]
        t = np.where((disc >= 0) & (np.abs(z) <= hh), ts, np.inf)
        for zc in (-hh, hh):
            tcap = (zc - lo[2]) / ld[:, 2]
            x, y = lo[0] + tcap * ld[:, 0], lo[1] + tcap * ld[:, 1]
            t = np.minimum(t, np.where(x * x + y * y <= r * r, tcap, np.inf))
    return t


def raycast_depth(cfg, env, view, proj, width, height):
    """OpenGL window depth (h, w) of the scene the GPU draws (targets do not write depth)."""
    eye, d, P, near, far = _rays(view, proj, width, height)
    ts = []
    if cfg.has_plane:
        ts.append(_box(eye, d, np.array([0, 0, PLANE_TOP - 0.01]), np.eye(3), (3.0, 3.0, 0.01)))
    if cfg.has_table:
        ts.append(_box(eye, d, np.array([cfg.table_cx, 0.0, TABLE_TOP - 0.2]), np.eye(3),
                       (cfg.table_hx, cfg.table_hy, 0.2)))
    half = np.array([cfg.object_half[k] for k in range(3)], np.float64)
    for ob in range(cfg.n_objects):
        body = env.obj[ob]
        c = np.array(body.pos[:])
        R = _quat_mat(np.array(body.quat[:]))
        if cfg.object_shape == 1:
            ts.append(_cylinder(eye, d, c, R, half[0], half[2]))
        else:
            ts.append(_box(eye, d, c, R, half))
    caps, sph = scene_primitives(cfg, env)
    for a, b, r in caps:
        ts.append(_capsule(eye, d, a, b, r))
    for c, r in sph:
        ts.append(_sphere(eye, d, c, r))
    t = np.full(d.shape[0], np.inf)
    for tt in ts:
        tt = np.where(tt >= near, tt, np.inf)
        t = np.minimum(t, tt)
    t = np.where(t < far, t, np.inf)
    with np.errstate(invalid="ignore", divide="ignore"):
        dep = 0.5 * ((P[2, 2] * (-t) + P[2, 3]) / t) + 0.5
    return np.where(np.isfinite(t), dep, 1.0).reshape(height, width)
