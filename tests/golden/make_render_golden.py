"""Generate the camera-image golden vectors from the reference's own
panda_gym.pybullet.PyBullet.render / deproject / get_cam2world_transforms
(pybullet.py:69-264).

Run in the survey/build container (it needs /root/reference; the GPU box does
not have it):  python tests/golden/make_render_golden.py

What is imported from the reference: panda_gym.pybullet (the PyBullet wrapper
class).  Its absent third-party imports are placeholder modules (see
make_golden.py); cv2.cvtColor(img, COLOR_BGR2RGB) is given its documented
meaning for a 3-channel image (reverse the channel order).  The physics client
handed to the wrapper is a stand-in whose computeViewMatrixFromYawPitchRoll /
computeProjectionMatrixFOV return the oracle's restated matrices
(oracle/render_oracle.py -- PyBullet itself is absent, so those two are not
pinned) and whose getCameraImage returns a given depth buffer (the oracle ray
caster's depth of a PandaPush-v3 scene, float32 like pybullet's, with a few
edge values planted) and random RGBA pixels.  Everything the reference
computes from them -- tran_pix_world, the filtered point cloud, colours,
pixels_2d, the waypoint projections, deproject() -- is the golden.

Output: tests/golden/render.npz (data only).
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
OUT = os.path.join(HERE, "render.npz")

CAMERAS = [  # (width, height, target, distance, yaw, pitch, roll): pybullet.py defaults and task_classes/* calls
    (64, 48, (0.0, 0.0, 0.0), 1.4, 45.0, -30.0, 0.0),
    (80, 80, (-0.1, 0.1, 0.0), 0.9, 90.0, -70.0, 0.0),
    (96, 72, (0.0, 0.0, 0.1), 0.6, 0.0, -30.0, 0.0),
    (120, 90, (0.0, 0.0, 0.0), 1.2, 45.0, -30.0, 0.0),
]


def main():
    sys.path.insert(0, HERE)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import make_golden as MG
    import oracle as O
    import render_oracle as RO

    MG._placeholder_modules()
    p = sys.modules["pybullet"]
    p.DIRECT, p.GUI, p.ER_BULLET_HARDWARE_OPENGL = 2, 1, 131072
    sys.modules["cv2"].COLOR_BGR2RGB = 4
    sys.modules["cv2"].cvtColor = lambda img, code: np.ascontiguousarray(img[..., ::-1])
    sys.path.insert(0, REF)
    import panda_gym.pybullet as pbm

    class FakeClient:
        def __init__(self, view, proj, depth, px):
            self.view, self.proj, self.depth, self.px = view, proj, depth, px

        def computeViewMatrixFromYawPitchRoll(self, **kw):
            return self.view

        def computeProjectionMatrixFOV(self, **kw):
            return self.proj

        def getCameraImage(self, width, height, viewMatrix, projectionMatrix, renderer):
            assert tuple(viewMatrix) == tuple(self.view) and tuple(projectionMatrix) == tuple(self.proj)
            return width, height, self.px, self.depth, None

    cfg = O.config("push")
    env = O.new_env(cfg)
    O.reset(cfg, env, seed=12345)
    rng = np.random.default_rng(2024)
    out = {}
    for k, (w, h, tgt, dist, yaw, pitch, roll) in enumerate(CAMERAS):
        view, proj, _ = RO.camera(tgt, dist, yaw, pitch, roll, w, h)
        depth = RO.raycast_depth(cfg, env, view, proj, w, h).astype(np.float32)
        flat = depth.reshape(-1)
        # plant edge values: the 0.99 threshold and its float32 neighbours, far plane, near plane
        for v in (0.99, np.nextafter(np.float32(0.99), 0), np.nextafter(np.float32(0.99), 2), 1.0, 0.0):
            flat[rng.integers(flat.size)] = np.float32(v)
        px = tuple(int(v) for v in rng.integers(0, 256, size=h * w * 4))
        sim = object.__new__(pbm.PyBullet)
        sim.connection_mode = p.GUI
        sim.physics_client = FakeClient(view, proj, tuple(float(v) for v in flat), px)
        waypoints = rng.uniform(-0.3, 0.3, size=(5, 3)) + np.array([0.0, 0.0, 0.3])
        rgb, dep, points, colors, pixels_2d, wp = sim.render(width=w, height=h, target_position=np.array(tgt),
                                                             distance=dist, yaw=yaw, pitch=pitch, roll=roll,
                                                             waypoints=waypoints)
        _, _, tran = sim.get_cam2world_transforms(width=w, height=h, target_position=np.array(tgt), distance=dist,
                                                  yaw=yaw, pitch=pitch, roll=roll)
        pix = np.stack([rng.integers(0, w, 40), rng.integers(0, h, 40)], axis=1)
        dp = sim.deproject(dep, pix.copy(), tran, width=w, height=h)
        pre = f"c{k}_"
        out.update({pre + "camera": np.array([w, h, *tgt, dist, yaw, pitch, roll], np.float64),
                    pre + "view": np.array(view, np.float32), pre + "proj": np.array(proj, np.float32),
                    pre + "depth_in": flat.reshape(h, w), pre + "px_in": np.array(px, np.uint8).reshape(h, w, 4),
                    pre + "waypoints": waypoints, pre + "tran": tran, pre + "rgb": rgb, pre + "depth": dep,
                    pre + "points": points, pre + "colors": colors, pre + "pixels_2d": pixels_2d,
                    pre + "waypoints_proj": np.array(wp, np.int64), pre + "pixels": pix, pre + "deproject": dp})
        print(f"camera {k}: {w}x{h}, {points.shape[0]} points kept of {w * h}")
    out["n_cameras"] = np.array(len(CAMERAS))
    np.savez_compressed(OUT, **out)
    print("wrote", OUT, os.path.getsize(OUT), "bytes")


if __name__ == "__main__":
    main()
