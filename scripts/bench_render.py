#!/usr/bin/env python
"""Camera-image row (§8(f) rank 4) throughput on one GPU: batched
getCameraImage (k_render_prep + k_render) and render()'s deprojection
(k_deproject_image) at the reference's default 480x480, B envs of a task.
Prints one JSON line; --png writes a montage of the first envs' images.

usage: python scripts/bench_render.py [--env-id PandaPush-v3] [--batch 64] [--reps 10] [--png out.png]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "panda-lang-manip_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--env-id", default="PandaPush-v3")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--size", type=int, default=480)
    ap.add_argument("--png", default=None)
    a = ap.parse_args()
    import ctypes as C

    import torch

    import pandasim
    from pandasim.sim import _ptr

    env = pandasim.make(a.env_id, num_envs=a.batch)
    env.reset(seed=12345)
    g = torch.Generator(device="cuda")
    g.manual_seed(0)
    for _ in range(5):
        env.step(torch.rand(a.batch, env.action_dim, device="cuda", generator=g) * 2 - 1, copy=False)
    sim, W, H, B = env.sim, a.size, a.size, a.batch
    view, proj, tran = sim.get_cam2world_transforms(W, H, np.array([-0.1, 0.1, 0.0]), 0.9, 90, -70, 0)
    n = W * H
    pts = torch.empty(B, n, 3, dtype=torch.float64, device="cuda")
    valid = torch.empty(B, n, dtype=torch.uint8, device="cuda")
    pix = torch.empty(B, n, 2, dtype=torch.float64, device="cuda")
    T = (C.c_double * 16)(*tran.reshape(-1).tolist())

    def deproject(depth):
        sim._call("ps_deproject_image", sim._ctx, _ptr(depth), T, W, H, _ptr(pts), _ptr(valid), _ptr(pix),
                  sim._stream())

    depth, rgb = sim.get_camera_image(W, H, view, proj)
    deproject(depth)
    torch.cuda.synchronize()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    e[0].record()
    for _ in range(a.reps):
        depth, rgb = sim.get_camera_image(W, H, view, proj)
    e[1].record()
    for _ in range(a.reps):
        deproject(depth)
    e[2].record()
    torch.cuda.synchronize()
    t_img = e[0].elapsed_time(e[1]) / a.reps
    t_dep = e[1].elapsed_time(e[2]) / a.reps
    dep_bytes = n * B * (4 + 24 + 1 + 16)  # read depth f32; write point f64x3, valid u8, pixels_2d f64x2
    img_bytes = n * B * (4 + 3)  # write depth f32 + rgb u8x3
    out = {"metric": "camera images/s (batched getCameraImage + render() deprojection)", "env_id": a.env_id,
           "batch": B, "width": W, "height": H,
           "images_per_s": round(B / ((t_img + t_dep) * 1e-3), 1),
           "get_camera_image_ms": round(t_img, 4), "deproject_ms": round(t_dep, 4),
           "render_mpix_per_s": round(n * B / (t_img * 1e-3) / 1e6, 1),
           "render_write_gbs": round(img_bytes / (t_img * 1e-3) / 1e9, 1),
           "deproject_roofline": {"bound": "hbm", "achieved": round(dep_bytes / (t_dep * 1e-3) / 1e9, 1),
                                  "peak": 8000.0, "unit": "GB/s",
                                  "frac": round(dep_bytes / (t_dep * 1e-3) / 1e9 / 8000.0, 4),
                                  "bytes_per_pixel": 45},
           "valid_points_per_image": round(float(valid.float().sum()) / B, 1)}
    print(json.dumps(out), flush=True)
    if a.png:
        from PIL import Image

        k = min(B, 4)
        im = rgb[:k].cpu().numpy()
        d = depth[:k].cpu().numpy()
        P = np.asarray(proj, np.float64).reshape(4, 4, order="F")
        lin = P[2, 3] / (2.0 * d - 1.0 + P[2, 2])
        lin = np.where(d < 1.0, lin, np.nan)
        lo, hi = np.nanmin(lin), np.nanmax(lin)
        dv = np.nan_to_num((hi - lin) / (hi - lo + 1e-9), nan=0.0)
        dimg = (np.stack([dv] * 3, -1) * 255).astype(np.uint8)
        top = np.concatenate(list(im), axis=1)
        bot = np.concatenate(list(dimg), axis=1)
        Image.fromarray(np.concatenate([top, bot], axis=0)).save(a.png)


if __name__ == "__main__":
    main()
