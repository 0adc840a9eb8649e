"""Batched counterpart of panda_gym.pybullet.PyBullet (pybullet.py:16-799).

``PandaSim`` owns one structure-of-arrays state buffer (a torch uint8 tensor on
the GPU) for B identical scenes and exposes the subset of the PyBullet wrapper
that the Robot/Task plugins of the hot path call, each method acting on all B
scenes at once.  Compute goes through libpandasim.so (HIP, gfx950); simple
field reads/writes are tensor views of the state buffer.
"""
from __future__ import annotations

import contextlib
import ctypes as C
import itertools
import math
from typing import Dict, Optional, Sequence

import numpy as np
import torch

from . import _lib as L

TASKS = {"reach": 0, "push": 1, "pick_and_place": 2, "slide": 3, "stack": 4, "flip": 5}
CONTROLS = {"ee": 0, "joints": 1}
REWARDS = {"sparse": 0, "dense": 1}
JOINT_TO_DOF = {0: 0, 1: 1, 2: 2, 3: 3, 4: 4, 5: 5, 6: 6, 9: 7, 10: 8}
DT_SUBSTEP = 1.0 / 500


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else C.c_void_p(t.data_ptr())


class PandaSim:
    """B Panda scenes on one GPU (one process per GPU)."""

    def __init__(self, task: str = "reach", control_type: str = "ee", reward_type: str = "sparse", num_envs: int = 1,
                 device="cuda", n_substeps: int = 20, config: Optional[L.Config] = None):
        if not torch.cuda.is_available():
            raise L.PandasimError("PandaSim needs a ROCm GPU (there is no CPU fallback)")
        self.device = torch.device(device)
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.num_envs = int(num_envs)
        self.n_substeps = int(n_substeps)
        if config is not None:
            self.cfg = config
        elif task is None:
            # empty world, built up by loadURDF/create_* as PyBullet() + Robot/Task constructors do
            self.cfg = L.default_config(0, 0, 0)
            self.cfg.has_table = self.cfg.has_plane = self.cfg.n_objects = 0
            self.cfg.base[0] = 0.0
        else:
            self.cfg = L.default_config(TASKS[task], CONTROLS[control_type], REWARDS[reward_type])
        self._lib = L.lib()
        self._ctx = None
        self._create_ctx()
        # body name -> kind ("robot", "object", "ghost"); objects -> their index
        self._bodies: Dict[str, str] = {"panda": "robot"}
        self.finger_spinning_friction = 0.0  # panda.py:49-50 sets 0.001 (set_spinning_friction)
        self._objects: Dict[str, int] = {}
        names = {0: [], 1: ["object"], 2: ["object1", "object2"]}[self.cfg.n_objects]
        for k, name in enumerate(names):
            self._bodies[name] = "object"
            self._objects[name] = k
        self._ghost_pos: Dict[str, torch.Tensor] = {}
        self._ghost_orn: Dict[str, torch.Tensor] = {}
        # visual-only properties of created bodies (rgba, ghost shape): rendering
        self._rgba: Dict[str, np.ndarray] = {}
        self._ghost_shape: Dict[str, tuple] = {}
        self.layout = L.layout(self.num_envs)
        self.state = torch.zeros(self.layout.total_bytes, dtype=torch.uint8, device=self.device)
        self._bind_views()
        self._saved: Dict[int, torch.Tensor] = {}
        self._ids = itertools.count()
        self._call("ps_init_state", self._ctx, _ptr(self.state), self._stream())

    # ---------------------------------------------------------------- plumbing
    def _create_ctx(self):
        """(Re)create the context for the current scene config.  The state
        buffer's layout depends only on num_envs, so the state survives."""
        if self._ctx:
            self._lib.ps_destroy(self._ctx)
            self._ctx = None
        ctx = C.c_void_p()
        L.check(self._lib.ps_create(C.byref(self.cfg), self.num_envs, self.device.index, C.byref(ctx)),
                what="ps_create")
        self._ctx = ctx

    def _bind_views(self):
        lay, s = self.layout, self.state
        n = lay.stride
        self.f = s[lay.float_offset:lay.float_offset + L.NUM_FLOAT_ROWS * n * 4].view(torch.float32).view(
            L.NUM_FLOAT_ROWS, n)
        self.goal = s[lay.goal_offset:lay.goal_offset + L.MAX_GOAL_DIM * n * 8].view(torch.float64).view(
            L.MAX_GOAL_DIM, n)
        self.rng = s[lay.rng_offset:lay.rng_offset + L.NUM_RNG_ROWS * n * 8].view(torch.int64).view(L.NUM_RNG_ROWS, n)
        self.elapsed = s[lay.elapsed_offset:lay.elapsed_offset + n * 4].view(torch.int32)

    def _stream(self):
        return C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def _call(self, name: str, *args):
        with torch.cuda.device(self.device):
            rc = getattr(self._lib, name)(*args)
        L.check(rc, self._ctx, name)

    def rows(self, row: int, count: int) -> torch.Tensor:
        """[B, count] view-copy of float rows (env-major)."""
        return self.f[row:row + count, :self.num_envs].t()

    def set_rows(self, row: int, values: torch.Tensor) -> None:
        values = torch.as_tensor(values, dtype=torch.float32, device=self.device)
        if values.dim() == 1:
            values = values.unsqueeze(0).expand(self.num_envs, -1)
        self.f[row:row + values.shape[1], :self.num_envs] = values.t()

    @property
    def obs_dim(self) -> int:
        return self._lib.ps_obs_dim(self._ctx)

    @property
    def action_dim(self) -> int:
        return self._lib.ps_action_dim(self._ctx)

    @property
    def goal_dim(self) -> int:
        return self._lib.ps_goal_dim(self._ctx)

    @property
    def max_episode_steps(self) -> int:
        return self._lib.ps_max_episode_steps(self._ctx)

    def goals(self) -> torch.Tensor:
        """[B, goal_dim] float64 view-copy of the fused path's goals."""
        return self.goal[:self.goal_dim, :self.num_envs].t()

    @property
    def dt(self) -> float:
        """pybullet.py:47-50: timestep * n_substeps (0.04 s)."""
        return DT_SUBSTEP * self.n_substeps

    def close(self) -> None:
        if getattr(self, "_ctx", None):
            self._lib.ps_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------- scene construction
    # pybullet.py:507-799.  The scene is compiled into the kernels
    # (include/panda_model.h): these calls accept exactly the bodies of the
    # Reach/Push/PickAndPlace scenes and raise NotImplementedError otherwise.
    @contextlib.contextmanager
    def no_rendering(self):
        """pybullet.py:502-507: GUI rendering toggle; images come from render()."""
        yield

    def place_visualizer(self, target_position=None, distance=None, yaw=None, pitch=None) -> None:
        """pybullet.py:499-508: camera placement; no-op without rendering."""

    def loadURDF(self, body_name: str, fileName: str, basePosition=None, useFixedBase: bool = False,
                 **kwargs) -> None:
        """pybullet.py:522-529: only the fixed-base Franka Panda is modelled."""
        if not str(fileName).endswith("franka_panda/panda.urdf") or not useFixedBase:
            raise NotImplementedError(f"loadURDF({fileName!r}, useFixedBase={useFixedBase}): only the fixed-base "
                                      "franka_panda/panda.urdf is compiled in")
        base = [0.0, 0.0, 0.0] if basePosition is None else [float(x) for x in basePosition]
        for k in range(3):
            self.cfg.base[k] = base[k]
        self._bodies = {n: k for n, k in self._bodies.items() if k != "robot"}
        self._bodies[body_name] = "robot"
        self._create_ctx()

    def create_plane(self, z_offset: float) -> None:
        """pybullet.py:726-739."""
        if abs(z_offset - PLANE_Z) > 1e-12:
            raise NotImplementedError(f"create_plane(z_offset={z_offset}): only z_offset={PLANE_Z} is compiled in")
        self.cfg.has_plane = 1
        self._create_ctx()

    def create_table(self, length: float, width: float, height: float, x_offset: float = 0.0,
                     lateral_friction=None, spinning_friction=None) -> None:
        """pybullet.py:741-771: a static box with its top at z = 0 (default friction)."""
        if lateral_friction is not None or spinning_friction is not None:
            raise NotImplementedError("create_table: only the default table friction is compiled in")
        self.cfg.has_table = 1
        self.cfg.table_cx, self.cfg.table_hx, self.cfg.table_hy = float(x_offset), length / 2, width / 2
        self._create_ctx()

    def _add_object(self, body_name: str, shape: int, half, mass: float, lateral_friction, position) -> None:
        n = self.cfg.n_objects
        fric = 0.5 if lateral_friction is None else float(lateral_friction)
        if n >= 2 or mass <= 0:
            raise NotImplementedError("at most two dynamic objects (Stack) are compiled in")
        f32 = lambda v: [float(np.float32(x)) for x in v]  # the config holds float32
        if n == 1 and (shape != self.cfg.object_shape or f32(half) != list(self.cfg.object_half)
                       or f32([fric]) != [self.cfg.object_friction] or shape != L.SHAPE_BOX):
            raise NotImplementedError("a second object must be a cube like the first (Stack)")
        if shape == L.SHAPE_BOX and max(half) != min(half):
            raise NotImplementedError("boxes must be cubes (isotropic inertia)")
        self.cfg.object_shape = shape
        for k in range(3):
            self.cfg.object_half[k] = float(half[k])
        self.cfg.object_friction = fric
        if n == 0:
            self.cfg.object_mass = float(mass)
        else:
            self.cfg.object2_mass = float(mass)
        self.cfg.n_objects = n + 1
        # the fused-kernel task matching the scene (the plugin path ignores it)
        self.cfg.task = {1: TASKS["slide"] if shape == L.SHAPE_CYLINDER else TASKS["push"], 2: TASKS["stack"]}[n + 1]
        self._bodies[body_name] = "object"
        self._objects[body_name] = n
        self._create_ctx()
        self.set_base_pose(body_name, position, [0.0, 0.0, 0.0, 1.0])

    def create_box(self, body_name: str, half_extents, mass: float, position, rgba_color=None, specular_color=None,
                   ghost: bool = False, lateral_friction=None, spinning_friction=None, texture=None) -> None:
        """pybullet.py:516-582: a dynamic cube (Push/PickAndPlace/Flip; two for Stack) or a ghost marker."""
        self._note_visual(body_name, rgba_color, L.SHAPE_BOX, [float(x) for x in half_extents], ghost)
        if ghost:
            self._add_ghost(body_name, position)
            return
        if spinning_friction:
            raise NotImplementedError("create_box: torsional friction rows (non-zero object spinning friction) "
                                      "are not modelled")
        self._add_object(body_name, L.SHAPE_BOX, [float(x) for x in half_extents], mass, lateral_friction, position)

    def create_cylinder(self, body_name: str, radius: float, height: float, mass: float, position, rgba_color=None,
                        specular_color=None, ghost: bool = False, lateral_friction=None,
                        spinning_friction=None) -> None:
        """pybullet.py:584-623: the upright cylinder of Slide (axis z), or a ghost marker."""
        self._note_visual(body_name, rgba_color, L.SHAPE_CYLINDER, [radius, radius, height / 2], ghost)
        if ghost:
            self._add_ghost(body_name, position)
            return
        if spinning_friction:
            raise NotImplementedError("create_cylinder: torsional friction rows (non-zero object spinning "
                                      "friction) are not modelled")
        self._add_object(body_name, L.SHAPE_CYLINDER, [radius, radius, height / 2], mass, lateral_friction, position)

    def create_sphere(self, body_name: str, radius: float, mass: float, position, rgba_color=None,
                      specular_color=None, ghost: bool = False) -> None:
        """pybullet.py:665-693: ghost target markers only."""
        self._note_visual(body_name, rgba_color, L.VISUAL_SPHERE, [radius, radius, radius], ghost)
        if not ghost:
            raise NotImplementedError("create_sphere: only ghost spheres (targets) are supported")
        self._add_ghost(body_name, position)

    def set_lateral_friction(self, body: str, link: int, lateral_friction: float) -> None:
        """pybullet.py:773-785: the compiled-in gripper proxies carry panda.py:47-48's values."""
        if not (self._bodies.get(body) == "robot" and int(link) in (9, 10) and lateral_friction == 1.0):
            raise NotImplementedError("set_lateral_friction: only the Panda fingers' 1.0 is compiled in")

    def set_spinning_friction(self, body: str, link: int, spinning_friction: float) -> None:
        """pybullet.py:787-799.  A contact's torsional friction coefficient is the
        product of its two bodies' spinning frictions
        (btManifoldResult::calculateCombinedSpinningFriction); every body but
        the fingers keeps Bullet's default 0, so the fingers' value (panda.py:49-50)
        yields no torsional friction row in any contact of these scenes.  A
        non-zero value on another body would create such rows, which the kernels
        do not build: it raises."""
        kind = self._bodies.get(body)
        if kind == "robot" and int(link) in (9, 10):
            self.finger_spinning_friction = float(spinning_friction)
            return
        if kind in ("object", "robot") and float(spinning_friction) == 0.0:
            return
        raise NotImplementedError("set_spinning_friction: torsional friction rows (a non-zero spinning friction "
                                  "on a body other than the fingers) are not modelled")

    def _note_visual(self, body_name, rgba_color, shape, half, ghost) -> None:
        rgba = np.zeros(4) if rgba_color is None else np.asarray(rgba_color, np.float64)  # pybullet.py:536
        self._rgba[body_name] = rgba
        if ghost:
            self._ghost_shape[body_name] = (shape, [float(h) for h in half])

    def _add_ghost(self, body_name: str, position) -> None:
        self._bodies[body_name] = "ghost"
        self._ghost_pos[body_name] = torch.zeros(self.num_envs, 3, dtype=torch.float64, device=self.device)
        self._ghost_orn[body_name] = torch.zeros(self.num_envs, 4, dtype=torch.float64, device=self.device)
        self._ghost_orn[body_name][:, 3] = 1.0
        self.set_base_pose(body_name, position, [0.0, 0.0, 0.0, 1.0])

    def _kind(self, body: str) -> str:
        if body not in self._bodies:
            raise KeyError(f"unknown body {body!r}")
        return self._bodies[body]

    # ----------------------------------------------------- camera images
    # pybullet.py:69-264 (§8(f) rank 4).  Batched: one image per env.
    def get_cam2world_transforms(self, width: int = 480, height: int = 480, target_position=np.zeros(3),
                                 distance: float = 1.4, yaw: float = 45, pitch: float = -30, roll: float = 0):
        """pybullet.py:69-107: (view_matrix, proj_matrix) as pybullet's 16-float
        tuples and tran_pix_world = inv(P @ V) (4, 4) float64."""
        target_position = np.zeros(3) if target_position is None else target_position
        t = (C.c_float * 3)(*[float(x) for x in target_position])
        view, proj, tran = (C.c_float * 16)(), (C.c_float * 16)(), (C.c_double * 16)()
        L.check(self._lib.ps_camera(t, float(distance), float(yaw), float(pitch), float(roll), int(width),
                                    int(height), view, proj, tran), what="ps_camera")
        return tuple(view[:]), tuple(proj[:]), np.array(tran[:], np.float64).reshape(4, 4)

    def _visual(self) -> L.Visual:
        """Colours by role and ghost-target shapes: from the create_* calls of
        the plugin path, else the registered task's _create_scene (tasks/*.py)."""
        v = L.Visual()
        cols = {"plane": (0.15, 0.15, 0.15, 1.0), "table": (0.95, 0.95, 0.95, 1.0), "robot": (0.9, 0.9, 0.92, 1.0),
                "background": (0.78, 0.85, 0.92, 1.0), "object1": (0.1, 0.9, 0.1, 1.0),
                "object2": (0.1, 0.9, 0.1, 1.0), "target1": (0.1, 0.9, 0.1, 0.3), "target2": (0.1, 0.9, 0.1, 0.3)}
        task = self.cfg.task
        half = [float(self.cfg.object_half[k]) for k in range(3)]
        shapes = [(L.SHAPE_BOX, half), (-1, [0.0] * 3)]
        if task == TASKS["reach"]:
            shapes[0] = (L.VISUAL_SPHERE, [0.02] * 3)  # reach.py:31-38
        elif task == TASKS["slide"]:
            shapes[0] = (L.SHAPE_CYLINDER, half)  # slide.py:43-51
        elif task == TASKS["stack"]:  # stack.py:33-61: blue object1/target1, green object2/target2
            cols.update(object1=(0.1, 0.1, 0.9, 1.0), target1=(0.1, 0.1, 0.9, 0.3))
            shapes[1] = (L.SHAPE_BOX, half)
        elif task == TASKS["flip"]:  # flip.py:33-47 (textured cube drawn in its mean colour)
            cols.update(object1=(0.55, 0.55, 0.55, 1.0), target1=(1.0, 1.0, 1.0, 0.5))
        objs = sorted(self._objects.items(), key=lambda kv: kv[1])
        for name, k in objs:
            if name in self._rgba:
                cols[f"object{k + 1}"] = tuple(self._rgba[name])
        ghosts = list(self._ghost_shape.items())
        if ghosts:
            shapes = [(-1, [0.0] * 3), (-1, [0.0] * 3)]
            for g, (name, (shape, h)) in enumerate(ghosts[:2]):
                shapes[g] = (shape, h)
                cols[f"target{g + 1}"] = tuple(self._rgba[name])
        for r, role in enumerate(L.ROLES):
            for k in range(4):
                v.rgba[r][k] = float(cols[role][k])
        for g in range(2):
            v.target_shape[g] = int(shapes[g][0])
            for k in range(3):
                v.target_half[g][k] = float(shapes[g][1][k])
        return v

    def _target_poses(self) -> torch.Tensor:
        """[B, 2, 7] f32 ghost-target poses: the plugin path's set_base_pose
        calls, else the fused path's goals as each task's reset places them
        (reach.py:49, push.py:72, stack.py:97-98, flip.py:66)."""
        B = self.num_envs
        out = torch.zeros(B, 2, 7, dtype=torch.float32, device=self.device)
        out[:, :, 6] = 1.0
        out[:, :, 2] = -100.0
        names = list(self._ghost_shape)[:2]
        if names:
            for g, n in enumerate(names):
                out[:, g, :3] = self._ghost_pos[n].float()
                out[:, g, 3:] = self._ghost_orn[n].float()
            return out
        goals = self.goals().float()
        if self.cfg.task == TASKS["flip"]:
            out[:, 0, :3] = torch.tensor([0.0, 0.0, 3 * 0.04 / 2], device=self.device)
            out[:, 0, 3:] = goals[:, :4]
        else:
            out[:, 0, :3] = goals[:, :3]
            if self.cfg.task == TASKS["stack"]:
                out[:, 1, :3] = goals[:, 3:6]
        return out

    @staticmethod
    def _check_image_size(width: int, height: int) -> None:
        # render() builds its NDC grid with np.mgrid[-1:1:2/n], whose length is
        # ceil(2 / (2/n)): for some n that is n + 1 and the reference's
        # np.stack of the grid with the depth buffer raises
        for n in (width, height):
            if int(math.ceil(2.0 / (2.0 / n))) != n:
                raise ValueError(f"render: np.mgrid[-1:1:2/{n}] has {int(math.ceil(2.0 / (2.0 / n)))} entries, not "
                                 f"{n}; the reference's deprojection cannot stack it with a {n}-pixel axis")

    def get_camera_image(self, width: int, height: int, view_matrix, proj_matrix, rgb: bool = True):
        """getCameraImage (pybullet.py:186-192) of every env: depth [B, h, w]
        f32 (OpenGL window depth) and rgb [B, h, w, 3] u8 (RGB order)."""
        B = self.num_envs
        depth = torch.empty(B, height, width, dtype=torch.float32, device=self.device)
        img = torch.empty(B, height, width, 3, dtype=torch.uint8, device=self.device) if rgb else None
        view = (C.c_float * 16)(*[float(x) for x in view_matrix])
        proj = (C.c_float * 16)(*[float(x) for x in proj_matrix])
        vis = self._visual()
        targets = self._target_poses().contiguous()
        self._call("ps_render", self._ctx, _ptr(self.state), view, proj, int(width), int(height), C.byref(vis),
                   _ptr(targets), _ptr(depth), _ptr(img), self._stream())
        return depth, img

    def render(self, width: int = 480, height: int = 480, target_position=np.zeros(3), distance: float = 1.4,
               yaw: float = 45, pitch: float = -30, roll: float = 0, waypoints=None, env: Optional[int] = None):
        """PyBullet.render (pybullet.py:149-264) for every env.

        env=None: a dict of batched tensors -- rgb [B, h, w, 3] u8 (channels
        swapped as the reference's cv2.cvtColor(BGR2RGB) of pybullet's RGBA
        leaves them), depth [B, h, w] f32, points [B, h*w, 3] f64, valid
        [B, h*w] bool (the reference keeps points[valid[b]] in pixel order),
        colors [B, h*w, 3] u8, pixels_2d [B, h*w, 2] f64, waypoints_proj.
        env=i: the reference's tuple (rgb, depth, points, colors, pixels_2d,
        waypoints_proj) of env i as numpy arrays."""
        self._check_image_size(width, height)
        view, proj, tran = self.get_cam2world_transforms(width, height, target_position, distance, yaw, pitch, roll)
        depth, img = self.get_camera_image(width, height, view, proj)
        B, n = self.num_envs, width * height
        points = torch.empty(B, n, 3, dtype=torch.float64, device=self.device)
        valid = torch.empty(B, n, dtype=torch.uint8, device=self.device)
        pix2d = torch.empty(B, n, 2, dtype=torch.float64, device=self.device)
        T = (C.c_double * 16)(*tran.reshape(-1).tolist())
        self._call("ps_deproject_image", self._ctx, _ptr(depth), T, int(width), int(height), _ptr(points),
                   _ptr(valid), _ptr(pix2d), self._stream())
        waypoints_proj = []
        if waypoints is not None:
            PV = np.matmul(np.asarray(proj).reshape([4, 4], order="F"), np.asarray(view).reshape([4, 4], order="F"))
            for point in waypoints:
                x, y, z, w = np.matmul(PV, np.array([point[0], point[1], point[2], 1]))
                x, y = (x / w + 1) / 2 * width, (y / w + 1) / 2 * height
                waypoints_proj.append([int(x), int(height - y)])
        out = {"rgb": img.flip(-1), "depth": depth, "points": points, "valid": valid.bool(),
               "colors": img.reshape(B, n, 3), "pixels_2d": pix2d, "waypoints_proj": waypoints_proj}
        if env is None:
            return out
        keep = out["valid"][env].cpu().numpy()
        return (out["rgb"][env].cpu().numpy(), out["depth"][env].double().cpu().numpy(),
                out["points"][env].cpu().numpy()[keep], out["colors"][env].cpu().numpy()[keep],
                out["pixels_2d"][env].cpu().numpy()[keep], waypoints_proj)

    def deproject(self, depth, pixels, tran_pix_world, width: int = 480, height: int = 480) -> torch.Tensor:
        """PyBullet.deproject (pybullet.py:109-146) per env: depth [B, h, w]
        (or one [h, w] image for every env), pixels [n, 2] or [B, n, 2]
        (column, row) -> world points [B, n, 3] float64."""
        B = self.num_envs
        depth = torch.as_tensor(depth, device=self.device).to(torch.float32)
        if depth.dim() == 2:
            depth = depth.unsqueeze(0).expand(B, -1, -1)
        depth = depth.contiguous()
        pixels = torch.as_tensor(np.asarray(pixels) if not torch.is_tensor(pixels) else pixels,
                                 device=self.device).to(torch.int32)
        if pixels.dim() == 2:
            pixels = pixels.unsqueeze(0).expand(B, -1, -1)
        pixels = pixels.contiguous()
        if depth.shape != (B, height, width) or pixels.shape[0] != B or pixels.shape[2] != 2:
            raise ValueError(f"deproject: depth {tuple(depth.shape)} / pixels {tuple(pixels.shape)} do not match "
                             f"{B} envs of {height}x{width}")
        if pixels.numel() and (int(pixels[..., 0].min()) < 0 or int(pixels[..., 0].max()) >= width
                               or int(pixels[..., 1].min()) < 0 or int(pixels[..., 1].max()) >= height):
            raise IndexError("deproject: pixel outside the image")  # numpy's depth[rows, cols] raises too
        n = pixels.shape[1]
        points = torch.empty(B, n, 3, dtype=torch.float64, device=self.device)
        T = (C.c_double * 16)(*np.asarray(tran_pix_world, np.float64).reshape(-1).tolist())
        self._call("ps_deproject_pixels", self._ctx, _ptr(depth), _ptr(pixels), int(n), T, int(width), int(height),
                   _ptr(points), self._stream())
        return points

    # ------------------------------------------------------- per-env RNGs
    def seed(self, seeds, mask=None) -> None:
        """seeding.np_random(seed) per env (core.py:244): seeds [B] uint64 (int64 bits)."""
        seeds = torch.as_tensor(seeds, device=self.device).to(torch.int64).reshape(self.num_envs).contiguous()
        m = None if mask is None else torch.as_tensor(mask, device=self.device).to(torch.uint8).contiguous()
        self._call("ps_rng_seed", self._ctx, _ptr(self.state), _ptr(m), _ptr(seeds), self._stream())

    def random_rotation(self, mask=None) -> torch.Tensor:
        """Rotation.random().as_quat() of every env's Flip goal stream -> [B, 4] float64."""
        out = torch.empty(self.num_envs, 4, dtype=torch.float64, device=self.device)
        m = None if mask is None else torch.as_tensor(mask, device=self.device).to(torch.uint8).contiguous()
        self._call("ps_rng_rotation", self._ctx, _ptr(self.state), _ptr(m), _ptr(out), self._stream())
        return out

    def uniform(self, low, high, mask=None) -> torch.Tensor:
        """Generator.uniform(low, high) of every env's own PCG64 stream -> [B, n] float64."""
        lo = [float(x) for x in (low if hasattr(low, "__len__") else [low])]
        hi = [float(x) for x in (high if hasattr(high, "__len__") else [high])]
        n = len(lo)
        if n != len(hi) or not 1 <= n <= L.PS_MAX_UNIFORM:
            raise ValueError("uniform: low/high must have the same length, 1..8")
        out = torch.empty(self.num_envs, n, dtype=torch.float64, device=self.device)
        m = None if mask is None else torch.as_tensor(mask, device=self.device).to(torch.uint8).contiguous()
        self._call("ps_rng_uniform", self._ctx, _ptr(self.state), _ptr(m), n, (C.c_double * n)(*lo),
                   (C.c_double * n)(*hi), _ptr(out), self._stream())
        return out

    # ------------------------------------------------------------ stepping
    def step(self) -> None:
        """pybullet.py:52-55: n_substeps stepSimulation() calls."""
        self._call("ps_sim_step", self._ctx, _ptr(self.state), self.n_substeps, self._stream())

    def save_state(self) -> int:
        """pybullet.py:61-68: in-memory snapshot; returns a state id."""
        sid = next(self._ids)
        self._saved[sid] = self.state.clone()
        return sid

    def restore_state(self, state_id: int) -> None:
        """pybullet.py:266-272.  Unknown/removed ids raise (pybullet.error in the reference)."""
        if state_id not in self._saved:
            raise L.PandasimError(f"restoreState: unknown state id {state_id}")
        self.state.copy_(self._saved[state_id])
        self._call("ps_mark_motor_rows_dirty", self._ctx)  # the snapshot's motor rows

    def remove_state(self, state_id: int) -> None:
        """pybullet.py:274-280."""
        if self._saved.pop(state_id, None) is None:
            raise L.PandasimError(f"removeState: unknown state id {state_id}")

    # -------------------------------------------------------------- getters
    def link_state(self, link: int):
        B = self.num_envs
        pos = torch.empty(B, 3, device=self.device)
        quat = torch.empty(B, 4, device=self.device)
        lv = torch.empty(B, 3, device=self.device)
        av = torch.empty(B, 3, device=self.device)
        self._call("ps_link_state", self._ctx, _ptr(self.state), int(link), _ptr(pos), _ptr(quat), _ptr(lv), _ptr(av),
                   self._stream())
        return pos, quat, lv, av

    def get_link_position(self, body: str, link: int) -> torch.Tensor:
        return self.link_state(link)[0]

    def get_link_orientation(self, body: str, link: int) -> torch.Tensor:
        return self.link_state(link)[1]

    def get_link_velocity(self, body: str, link: int) -> torch.Tensor:
        return self.link_state(link)[2]

    def get_link_angular_velocity(self, body: str, link: int) -> torch.Tensor:
        return self.link_state(link)[3]

    def get_joint_angle(self, body: str, joint: int) -> torch.Tensor:
        return self.f[L.F_Q + JOINT_TO_DOF[joint], :self.num_envs].clone()

    def get_joint_velocity(self, body: str, joint: int) -> torch.Tensor:
        return self.f[L.F_QD + JOINT_TO_DOF[joint], :self.num_envs].clone()

    def _object_rows(self, body: str) -> int:
        return L.OBJECT_ROWS[self._objects[body]]

    def _base_state(self, body: str):
        B = self.num_envs
        pos, euler, vel, avel = (torch.empty(B, 3, device=self.device) for _ in range(4))
        quat = torch.empty(B, 4, device=self.device)
        self._call("ps_base_state", self._ctx, _ptr(self.state), self._objects[body], _ptr(pos), _ptr(quat),
                   _ptr(euler), _ptr(vel), _ptr(avel), self._stream())
        return pos, quat, euler, vel, avel

    def get_base_position(self, body: str) -> torch.Tensor:
        """getBasePositionAndOrientation[0] (pybullet.py:284-294)."""
        kind = self._kind(body)
        if kind == "ghost":
            return self._ghost_pos[body].clone()
        if kind == "robot":
            return torch.tensor([float(x) for x in self.cfg.base], device=self.device).expand(self.num_envs, 3)
        return self.rows(self._object_rows(body), 3).clone()

    def get_base_orientation(self, body: str) -> torch.Tensor:
        """getBasePositionAndOrientation[1] (pybullet.py:296-306), (x, y, z, w)."""
        kind = self._kind(body)
        if kind == "ghost":
            return self._ghost_orn[body].clone()
        if kind == "robot":
            return torch.tensor([0.0, 0.0, 0.0, 1.0], device=self.device).expand(self.num_envs, 4)
        return self.rows(self._object_rows(body) + 3, 4).clone()

    def get_base_rotation(self, body: str, type: str = "euler") -> torch.Tensor:
        """pybullet.py:308-325: getEulerFromQuaternion of the base orientation."""
        if type == "quaternion":
            return self.get_base_orientation(body)
        if type != "euler":
            raise ValueError("""type must be "euler" or "quaternion".""")
        if self._kind(body) == "object":
            return self._base_state(body)[2]
        return euler_from_quaternion(self.get_base_orientation(body))

    def get_base_velocity(self, body: str) -> torch.Tensor:
        """getBaseVelocity[0] (pybullet.py:327-337)."""
        if self._kind(body) != "object":
            return torch.zeros(self.num_envs, 3, device=self.device)
        return self.rows(self._object_rows(body) + 7, 3).clone()

    def get_base_angular_velocity(self, body: str) -> torch.Tensor:
        """getBaseVelocity[1] (pybullet.py:339-349)."""
        if self._kind(body) != "object":
            return torch.zeros(self.num_envs, 3, device=self.device)
        return self.rows(self._object_rows(body) + 10, 3).clone()

    # -------------------------------------------------------------- setters
    def set_joint_angles(self, body: str, joints: Sequence[int], angles) -> None:
        """resetJointState (pybullet.py:441-460): position set, velocity zeroed;
        the robot's cached contacts break (the links are teleported)."""
        angles = torch.as_tensor(angles, dtype=torch.float32, device=self.device)
        for k, j in enumerate(joints):
            d = JOINT_TO_DOF[int(j)]
            self.f[L.F_Q + d, :self.num_envs] = angles[..., k]
            self.f[L.F_QD + d, :self.num_envs] = 0.0
        self.f[L.F_WR:L.F_WRID + 1, :self.num_envs] = 0.0

    def set_joint_angle(self, body: str, joint: int, angle) -> None:
        self.set_joint_angles(body, [joint], torch.as_tensor(angle, dtype=torch.float32).reshape(-1, 1)
                              if torch.as_tensor(angle).dim() else [angle])

    def set_base_pose(self, body: str, position, orientation) -> None:
        """resetBasePositionAndOrientation (pybullet.py:427-439).  PyBullet's
        init-pose command zeroes the base linear and angular velocity with the
        pose; the object's cached contacts break (it is teleported).  A 3-vector
        orientation is Euler angles (getQuaternionFromEuler)."""
        orientation = torch.as_tensor(orientation, dtype=torch.float64, device=self.device)
        if orientation.shape[-1] == 3:
            orientation = quaternion_from_euler(orientation)
        kind = self._kind(body)
        if kind == "robot":
            raise NotImplementedError("the Panda base is fixed (loadURDF useFixedBase=True)")
        if kind == "ghost":
            pos = torch.as_tensor(position, dtype=torch.float64, device=self.device)
            self._ghost_pos[body][:] = pos.expand(self.num_envs, 3)
            self._ghost_orn[body][:] = orientation.expand(self.num_envs, 4)
            return
        row = self._object_rows(body)
        self.set_rows(row, torch.as_tensor(position, device=self.device).to(torch.float32))
        self.set_rows(row + 3, orientation.to(torch.float32))
        self.f[row + 7:row + 13, :self.num_envs] = 0.0
        g = L.F_WG0 if self._objects[body] == 0 else L.F_WG1
        self.f[g:g + 5, :self.num_envs] = 0.0
        self.f[L.F_WR:L.NUM_FLOAT_ROWS, :self.num_envs] = 0.0  # gripper and object-object contacts

    def control_joints(self, body: str, joints: Sequence[int], target_angles, forces) -> None:
        """setJointMotorControlArray(POSITION_CONTROL) (pybullet.py:462-477)."""
        t = torch.as_tensor(target_angles, dtype=torch.float32, device=self.device)
        for k, j in enumerate(joints):
            d = JOINT_TO_DOF[int(j)]
            self.f[L.F_MTARGET + d, :self.num_envs] = t[..., k]
            self.f[L.F_MKP + d, :self.num_envs] = 0.1
            self.f[L.F_MKD + d, :self.num_envs] = 1.0
            self.f[L.F_MVEL + d, :self.num_envs] = 0.0
            self.f[L.F_MIMP + d, :self.num_envs] = float(forces[k]) * DT_SUBSTEP
        self._call("ps_mark_motor_rows_dirty", self._ctx)  # a fused step rewrites the gains

    def inverse_kinematics(self, body: str, link: int, position, orientation) -> torch.Tensor:
        """calculateInverseKinematics from the current joints (pybullet.py:479-497) -> [B, 9]."""
        B = self.num_envs
        pos = torch.as_tensor(position, dtype=torch.float32, device=self.device).expand(B, 3).contiguous()
        orn = torch.as_tensor(orientation, dtype=torch.float32, device=self.device).expand(B, 4).contiguous()
        out = torch.empty(B, 9, device=self.device)
        self._call("ps_inverse_kinematics", self._ctx, _ptr(self.state), int(link), _ptr(pos), _ptr(orn), _ptr(out),
                   self._stream())
        return out


# ---------------------------------------------------------------- helpers
PLANE_Z = -0.4                      # tasks/*.py: create_plane(z_offset=-0.4)


def euler_from_quaternion(q: torch.Tensor) -> torch.Tensor:
    """getEulerFromQuaternion (Bullet btQuaternion::getEulerZYX convention, as
    ps_task.h::euler_from_quat) for (..., 4) (x, y, z, w) tensors."""
    x, y, z, w = q.unbind(-1)
    sarg = -2.0 * (x * z - w * y)
    roll = torch.atan2(2.0 * (y * z + w * x), w * w - x * x - y * y + z * z)
    pitch = torch.asin(sarg.clamp(-1.0, 1.0))
    yaw = torch.atan2(2.0 * (x * y + w * z), w * w + x * x - y * y - z * z)
    lo, hi = sarg <= -0.99999, sarg >= 0.99999
    roll = torch.where(lo | hi, torch.zeros_like(roll), roll)
    pitch = torch.where(lo, torch.full_like(pitch, -0.5 * math.pi), torch.where(hi, torch.full_like(pitch, 0.5 * math.pi),
                                                                              pitch))
    yaw = torch.where(lo, 2.0 * torch.atan2(x, -y), torch.where(hi, 2.0 * torch.atan2(-x, y), yaw))
    return torch.stack([roll, pitch, yaw], -1)


def quaternion_from_euler(e: torch.Tensor) -> torch.Tensor:
    """getQuaternionFromEuler (roll about x, pitch about y, yaw about z) -> (x, y, z, w)."""
    r, p, y = (e * 0.5).unbind(-1)
    cr, sr, cp, sp, cy, sy = torch.cos(r), torch.sin(r), torch.cos(p), torch.sin(p), torch.cos(y), torch.sin(y)
    return torch.stack([sr * cp * cy - cr * sp * sy, cr * sp * cy + sr * cp * sy, cr * cp * sy - sr * sp * cy,
                        cr * cp * cy + sr * sp * sy], -1)
