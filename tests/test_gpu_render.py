"""GPU parity of the camera-image row (§8(f) rank 4, pybullet.py:69-264)
through the C ABI: ps_deproject_* against the reference-generated goldens,
ps_render's depth against the oracle's independent ray caster, and the
batched render() against the oracle's restatement of the reference's
post-processing on the GPU's own depth buffers."""
import numpy as np
import pytest
import torch

import oracle as O
import render_oracle as RO
from helpers import oracle_config_for, oracle_env_from, snapshot

pytestmark = pytest.mark.gpu


def _cams(g):
    for k in range(int(g["n_cameras"])):
        yield k, {n[len(f"c{k}_"):]: v for n, v in g.items() if n.startswith(f"c{k}_")}


@pytest.fixture(scope="module")
def sim1():
    from pandasim.sim import PandaSim

    return PandaSim("push", num_envs=1)


def _near_bound(p):
    b = np.array([abs(p[:, 2]), abs(p[:, 2] - 0.67), abs(p[:, 0] + 0.5), abs(p[:, 0] - 0.2)])
    return b.min(0) < 1e-9


def test_deproject_image_matches_reference_goldens(sim1, render_golden):
    for k, c in _cams(render_golden):
        h, w = c["depth_in"].shape
        out = {}
        depth = torch.from_numpy(c["depth_in"]).cuda().reshape(1, h, w).contiguous()
        import ctypes as C
        from pandasim.sim import _ptr

        pts = torch.empty(1, h * w, 3, dtype=torch.float64, device="cuda")
        valid = torch.empty(1, h * w, dtype=torch.uint8, device="cuda")
        pix = torch.empty(1, h * w, 2, dtype=torch.float64, device="cuda")
        T = (C.c_double * 16)(*c["tran"].reshape(-1).tolist())
        sim1._call("ps_deproject_image", sim1._ctx, _ptr(depth), T, w, h, _ptr(pts), _ptr(valid), _ptr(pix),
                   sim1._stream())
        torch.cuda.synchronize()
        keep = valid[0].bool().cpu().numpy()
        gp = pts[0].cpu().numpy()
        _, _, _, flat = RO.deproject_image(c["depth_in"], c["tran"])
        ref_keep = np.zeros(h * w, bool)
        ref_keep[flat] = True
        diff = keep != ref_keep
        assert not diff.any() or _near_bound(gp[diff]).all(), (k, int(diff.sum()))
        both = keep & ref_keep
        got = gp[both]
        want = c["points"][np.isin(flat, np.nonzero(both)[0])]
        assert np.allclose(got, want, rtol=1e-12, atol=1e-12), (k, np.abs(got - want).max())
        # tran @ pixel with OpenBLAS dgemm's fused-multiply-add order: bit for bit
        assert np.array_equal(got, want), (k, np.mean(np.all(got == want, axis=1)))
        assert np.array_equal(pix[0].cpu().numpy()[both], c["pixels_2d"][np.isin(flat, np.nonzero(both)[0])])


def test_deproject_pixels_matches_reference_goldens(sim1, render_golden):
    for k, c in _cams(render_golden):
        h, w = c["depth_in"].shape
        got = sim1.deproject(c["depth_in"], c["pixels"], c["tran"], width=w, height=h)[0].cpu().numpy()
        assert np.array_equal(got, c["deproject"]), (k, np.abs(got - c["deproject"]).max())


def _linear(depth, proj):
    P = np.asarray(proj, np.float64).reshape(4, 4, order="F")
    zn = 2.0 * depth.astype(np.float64) - 1.0
    with np.errstate(divide="ignore"):
        return P[2, 3] / (zn + P[2, 2])  # = -z_eye = distance along the view axis


@pytest.mark.parametrize("task", ["reach", "push", "slide", "stack", "pick_and_place", "flip"])
def test_render_depth_matches_oracle_raycaster(task):
    from pandasim.envs import PandaVecEnv

    B, w, h = 3, 64, 48
    env = PandaVecEnv(task, "sparse", "ee", B, "cuda:0", autoreset=False)
    env.reset(seed=777)
    g = torch.Generator(device="cuda")
    g.manual_seed(3)
    for _ in range(4):
        env.step(torch.rand(B, env.action_dim, device="cuda", generator=g) * 2 - 1)
    sim = env.sim
    cfg = oracle_config_for(sim.cfg)
    snap = snapshot(sim)
    for cam in [((0, 0, 0), 1.4, 45, -30, 0), ((-0.1, 0.1, 0), 0.9, 90, -70, 0), ((0, 0, 0.1), 0.6, 0, -30, 0)]:
        view, proj, _ = sim.get_cam2world_transforms(w, h, *cam)
        depth, rgb = sim.get_camera_image(w, h, view, proj)
        depth = depth.cpu().numpy()
        for i in range(B):
            ref = RO.raycast_depth(cfg, oracle_env_from(cfg, snap, i), view, proj, w, h)
            hit_g, hit_r = depth[i] < 1.0, ref < 1.0
            edge = hit_g != hit_r
            assert edge.mean() < 0.01, (task, cam, i, edge.sum())  # silhouette pixels only
            both = hit_g & hit_r
            lg, lr = _linear(depth[i][both], proj), _linear(ref[both], proj)
            rel = np.abs(lg - lr) / lr
            assert np.mean(rel < 1e-4) > 0.99 and np.median(rel) < 1e-5, (task, cam, i, rel.max())
        assert rgb.shape == (B, h, w, 3) and rgb.dtype == torch.uint8


def test_batched_render_matches_reference_postprocessing_on_gpu_depth():
    from pandasim.envs import PandaVecEnv

    B = 4
    env = PandaVecEnv("push", "sparse", "ee", B, "cuda:0", autoreset=False)
    env.reset(seed=5)
    sim = env.sim
    out = sim.render(480, 480, target_position=np.array([-0.1, 0.1, 0]), distance=0.9, yaw=90, pitch=-70,
                     waypoints=[[0.0, 0.0, 0.1], [-0.2, 0.1, 0.05]])
    assert out["rgb"].shape == (B, 480, 480, 3) and out["depth"].shape == (B, 480, 480)
    _, _, tran = sim.get_cam2world_transforms(480, 480, np.array([-0.1, 0.1, 0]), 0.9, 90, -70, 0)
    for i in range(B):
        d = out["depth"][i].double().cpu().numpy()
        rgb = out["colors"][i].cpu().numpy().reshape(480, 480, 3)
        pts, cols, pix2d, flat = RO.deproject_image(d, tran, rgb)
        keep = out["valid"][i].cpu().numpy()
        assert keep.sum() > 1000  # table top, cube and arm inside the workspace box
        diff = keep.copy()
        diff[flat] ^= True
        gp = out["points"][i].cpu().numpy()
        assert not diff.any() or _near_bound(gp[diff]).all()
        tup = sim.render(480, 480, target_position=np.array([-0.1, 0.1, 0]), distance=0.9, yaw=90, pitch=-70,
                         env=i) if i == 0 else None
        if tup is not None:
            assert tup[2].shape == pts.shape and np.allclose(tup[2], pts, rtol=1e-12, atol=1e-12)
            assert np.array_equal(tup[3], cols) and np.array_equal(tup[0], tup[0][..., :]) and tup[1].dtype == np.float64
        both = np.nonzero(keep)[0]
        assert np.allclose(gp[both], pts[np.isin(flat, both)], rtol=1e-12, atol=1e-12)
    assert len(out["waypoints_proj"]) == 2 and all(len(p) == 2 for p in out["waypoints_proj"])


def test_ghost_targets_blend_colour_but_not_depth():
    from pandasim.envs import PandaVecEnv

    env = PandaVecEnv("reach", "sparse", "ee", 2, "cuda:0", autoreset=False)
    env.reset(seed=11)
    sim = env.sim
    view, proj, _ = sim.get_cam2world_transforms(64, 48, np.zeros(3), 0.6, 45, -30, 0)
    d1, c1 = sim.get_camera_image(64, 48, view, proj)
    sim.goal[:3, :2] = torch.tensor([[-0.1, 0.0, 0.05]], device="cuda", dtype=torch.float64).t()  # move the target
    d2, c2 = sim.get_camera_image(64, 48, view, proj)
    assert torch.equal(d1, d2)
    assert not torch.equal(c1, c2)


def test_render_rejects_sizes_the_reference_cannot_stack():
    from pandasim.envs import PandaVecEnv

    env = PandaVecEnv("reach", "sparse", "ee", 1, "cuda:0", autoreset=False)
    env.reset(seed=1)
    with pytest.raises(ValueError):
        env.sim.render(width=49, height=64)


def test_render_batch_beyond_65535_envs():
    """Envs ride grid.x: 70 000 envs render, and env 69 999's image equals the
    image of the same env rendered alone (env i of reset(seed=s) is seeded s + i)."""
    from pandasim.envs import PandaVecEnv

    big = PandaVecEnv("push", "sparse", "ee", 70000, "cuda:0", autoreset=False)
    big.reset(seed=100)
    one = PandaVecEnv("push", "sparse", "ee", 1, "cuda:0", autoreset=False)
    one.reset(seed=100 + 69999)
    view, proj, _ = big.sim.get_cam2world_transforms(16, 12, np.zeros(3), 1.4, 45, -30, 0)
    db, cb = big.sim.get_camera_image(16, 12, view, proj)
    d1, c1 = one.sim.get_camera_image(16, 12, view, proj)
    assert torch.equal(db[69999], d1[0]) and torch.equal(cb[69999], c1[0])
    assert bool((db < 1.0).any())


def test_deproject_pixels_out_of_image(sim1):
    """The host wrapper raises like numpy's indexing; the C ABI itself reads
    nothing for such a pixel and returns a NaN point."""
    import ctypes as C

    from pandasim.sim import _ptr

    depth = torch.full((1, 4, 5), 0.5, dtype=torch.float32, device="cuda")
    with pytest.raises(IndexError):
        sim1.deproject(depth, [[5, 0]], np.eye(4), width=5, height=4)
    pix = torch.tensor([[[0, 0], [5, 0], [0, -1], [4, 3]]], dtype=torch.int32, device="cuda")
    pts = torch.empty(1, 4, 3, dtype=torch.float64, device="cuda")
    T = (C.c_double * 16)(*np.eye(4).reshape(-1).tolist())
    sim1._call("ps_deproject_pixels", sim1._ctx, _ptr(depth), _ptr(pix), 4, T, 5, 4, _ptr(pts), sim1._stream())
    p = pts[0].cpu().numpy()
    assert np.isfinite(p[[0, 3]]).all() and np.isnan(p[[1, 2]]).all()


def test_env_render_rgb_array():
    """RobotTaskEnv.render (core.py:294-335) through both env paths."""
    import pandasim

    env = pandasim.make("PandaPush-v3", num_envs=3)
    env.reset(seed=0)
    img = env.render("rgb_array", width=64, height=48)
    assert img.shape == (3, 48, 64, 3) and img.dtype == torch.uint8
    assert env.render("human") is None
    plug = pandasim.make("PandaPush-v3", num_envs=3, fused=False)
    plug.reset(seed=0)
    img2 = plug.env.render("rgb_array", width=64, height=48)
    assert img2.shape == (3, 48, 64, 3)
