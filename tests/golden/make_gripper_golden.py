"""Extract the Panda hand and finger collision hulls the reference ships, as a
fixture for the collision proxies of include/panda_model.h.

Run in the survey/build container (it needs /root/reference; the GPU box does
not have it):  python tests/golden/make_gripper_golden.py

Source (reference data, read as bytes -- nothing is imported or executed):
  panda_gym/envs/contact_graspnet/gripper_models/panda_gripper/hand.stl    (200 triangles)
  panda_gym/envs/contact_graspnet/gripper_models/panda_gripper/finger.stl  (32 triangles)
  panda_gym/envs/contact_graspnet/gripper_models/panda_gripper/panda_gripper.obj
      (the hand plus both fingers placed fully open: 138 vertices, 264 faces)

Frames.  contact-graspnet's gripper frame closes along x; the URDF hand frame
(franka panda.urdf, which PyBullet loads: panda.py:37) closes along y, its
finger joints sit at z = 0.0584 with axes +y (panda_leftfinger, link 9) and
-y (panda_rightfinger, link 10, its mesh turned by pi about z).  The map is a
rotation by -90 degrees about z:  (x, y, z)_urdf = (y, -x, z)_graspnet.  The
unrotated finger.stl is then the left finger (its body extends to +y, away
from the centre line, its pad face at y = 0); panda_gripper.obj's finger at
graspnet -x is that finger translated by the full opening (0.04 m) and the
joint height, which the CPU test checks.

Output: tests/golden/panda_gripper_hulls.npz (data only): unique hull
vertices of the hand (hand frame) and of the left finger (link-9 frame) in
the URDF frames, and the obj's three components mapped the same way.
"""
from __future__ import annotations

import os
import struct

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = "/root/reference/panda_gym/envs/contact_graspnet/gripper_models/panda_gripper"
OUT = os.path.join(HERE, "panda_gripper_hulls.npz")


def stl_vertices(path: str) -> np.ndarray:
    """Unique vertices of a binary STL (80-byte header, uint32 count, 50-byte triangles)."""
    b = open(path, "rb").read()
    n = struct.unpack("<I", b[80:84])[0]
    assert len(b) == 84 + 50 * n, path
    tri = np.frombuffer(b[84:84 + 50 * n], dtype=np.dtype([("n", "<f4", 3), ("v", "<f4", (3, 3)), ("a", "<u2")]))
    return np.unique(tri["v"].reshape(-1, 3).astype(np.float64), axis=0)


def obj_components(path: str) -> list:
    """Vertex sets of the connected components of an OBJ mesh."""
    V, F = [], []
    for line in open(path):
        s = line.split()
        if s and s[0] == "v":
            V.append([float(t) for t in s[1:4]])
        elif s and s[0] == "f":
            F.append([int(t.split("/")[0]) - 1 for t in s[1:]])
    V = np.array(V)
    parent = list(range(len(V)))

    def find(a):
        while parent[a] != a:
            parent[a] = parent[parent[a]]
            a = parent[a]
        return a

    for f in F:
        for k in f[1:]:
            ra, rb = find(f[0]), find(k)
            if ra != rb:
                parent[ra] = rb
    comps = {}
    for i in range(len(V)):
        comps.setdefault(find(i), []).append(i)
    return sorted((V[idx] for idx in comps.values()), key=lambda c: (len(c), c[:, 0].mean()))


def to_urdf(p: np.ndarray) -> np.ndarray:
    """graspnet gripper frame -> URDF hand frame: rotation by -90 deg about z."""
    return np.stack([p[:, 1], -p[:, 0], p[:, 2]], axis=1)


def main():
    hand = to_urdf(stl_vertices(os.path.join(SRC, "hand.stl")))
    finger = to_urdf(stl_vertices(os.path.join(SRC, "finger.stl")))
    comps = [to_urdf(c) for c in obj_components(os.path.join(SRC, "panda_gripper.obj"))]
    assert [len(c) for c in comps] == [18, 18, 102], [len(c) for c in comps]
    np.savez(OUT, hand=hand, finger_left=finger, obj_finger_a=comps[0], obj_finger_b=comps[1], obj_hand=comps[2])
    print(OUT, {"hand": hand.shape, "finger": finger.shape})
    print("hand extents", hand.max(0) - hand.min(0), "finger extents", finger.max(0) - finger.min(0))


if __name__ == "__main__":
    main()
