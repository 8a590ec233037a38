"""Generate the golden vectors that pin the CPU restatement (oracle/) to the reference.

Run in the build container only (it imports the reference's importable pure-Python maths from
/root/reference; the reference never travels to the GPU box):

    python tests/golden/make_golden.py

The reference ships no tests or fixtures for the rasterizer, and its CUDA cannot be
compiled here; what IS importable on CPU is the maths on either side of the
rasterizer call, so the fixtures pin exactly that:
  * camera_golden.npz  world_view_transform / full_proj_transform / camera_center of seeded
                       cameras built with utils/graphics_utils.py:38-84 the way
                       scene/cameras.py:76-81 builds them;
  * sh_golden.npz      eval_sh (utils/sh_utils.py:57-112) for degrees 0..3 on seeded coefficients
                       and directions, plus render()'s two colour pre-passes
                       (gaussian_renderer/__init__.py:269-274 and :280-287);
  * pipeline_flags.json the hot-path flag defaults of arguments/__init__.py:66-72, 96.
"""
from __future__ import annotations

import json
import math
import os
import sys

import numpy as np
import torch

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def main():
    sys.path.insert(0, REF)
    from utils.graphics_utils import getProjectionMatrix, getWorld2View2, focal2fov  # noqa: E402
    from utils.sh_utils import eval_sh  # noqa: E402
    import arguments  # noqa: E402

    rng = np.random.default_rng(1234)
    # ---- cameras -----------------------------------------------------------------------------
    Rs, Ts, fx, fy, Ws, Hs, wvts, fulls, centers = [], [], [], [], [], [], [], [], []
    for i in range(6):
        q = rng.normal(size=4)
        q /= np.linalg.norm(q)
        w, x, y, z = q
        R = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                      [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                      [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])
        T = rng.normal(size=3) * 2
        W, H = [(64, 48), (97, 61), (400, 400), (800, 800), (1008, 756), (1920, 1080)][i]
        f = 0.8 * W
        FoVx, FoVy = focal2fov(f, W), focal2fov(f, H)
        # scene/cameras.py:76-81
        wvt = torch.tensor(getWorld2View2(R, T, np.array([0.0, 0.0, 0.0]), 1.0)).transpose(0, 1)
        proj = getProjectionMatrix(znear=0.01, zfar=100.0, fovX=FoVx, fovY=FoVy).transpose(0, 1)
        full = wvt.unsqueeze(0).bmm(proj.unsqueeze(0)).squeeze(0)
        center = wvt.inverse()[3, :3]
        Rs.append(R); Ts.append(T); fx.append(FoVx); fy.append(FoVy); Ws.append(W); Hs.append(H)
        wvts.append(wvt.numpy()); fulls.append(full.numpy()); centers.append(center.numpy())
    np.savez(os.path.join(OUT, "camera_golden.npz"), R=np.stack(Rs), T=np.stack(Ts),
             FoVx=np.array(fx), FoVy=np.array(fy), W=np.array(Ws), H=np.array(Hs),
             world_view_transform=np.stack(wvts), full_proj_transform=np.stack(fulls),
             camera_center=np.stack(centers))

    # ---- SH ------------------------------------------------------------------------------------
    g = torch.Generator().manual_seed(7)
    P = 512
    xyz = torch.rand((P, 3), generator=g) * 2 - 1
    campos = torch.tensor([0.3, -0.2, -4.0])
    feats = torch.randn((P, 16, 3), generator=g) * 0.5          # get_features layout [P,16,3]
    lang = torch.randn((P, 3), generator=g)
    dir_pp = xyz - campos.repeat(P, 1)
    dirs = dir_pp / dir_pp.norm(dim=1, keepdim=True)
    shs_view = feats.transpose(1, 2).view(-1, 3, 16)
    out = {"xyz": xyz.numpy(), "campos": campos.numpy(), "features": feats.numpy(),
           "language_feature": lang.numpy()}
    for deg in range(4):
        sh2rgb = eval_sh(deg, shs_view, dirs)
        out[f"eval_sh_deg{deg}"] = sh2rgb.numpy()
        out[f"colors_precomp_deg{deg}"] = torch.clamp_min(sh2rgb + 0.5, 0.0).numpy()
    s2l = eval_sh(0, lang.view(-1, 3, 1), dirs)
    out["language_feature_precomp"] = (s2l / (s2l.norm(dim=-1, keepdim=True) + 1e-9)).numpy()
    np.savez(os.path.join(OUT, "sh_golden.npz"), **out)

    # ---- pipeline flags ------------------------------------------------------------------------
    import argparse
    parser = argparse.ArgumentParser()
    pp = arguments.PipelineParams(parser)
    flags = {k: getattr(pp, k) for k in ("convert_SHs_python", "compute_cov3D_python", "debug",
                                         "use_confidence")}
    mp = arguments.ModelParams(parser)
    flags["sh_degree"] = mp.sh_degree
    op = arguments.OptimizationParams(parser)
    flags["include_feature"] = op.include_feature
    with open(os.path.join(OUT, "pipeline_flags.json"), "w") as fh:
        json.dump(flags, fh, indent=1, sort_keys=True)
    print("wrote", sorted(os.listdir(OUT)))


if __name__ == "__main__":
    main()
