"""Shared test inputs: one seeded scene -> the same arrays for the oracle and the HIP path."""
from __future__ import annotations

import math

import numpy as np
import torch

from gsr_amd.synthetic import make_cameras, make_gaussians


def scene(P=256, W=64, H=48, cam=1, seed=0, sh_degree=3, active_degree=3, mode="sh",
          cov_mode="scale_rot", feature="sh", bg=(0.1, 0.2, 0.3), scale_mult=1.0,
          confidence=None, n_cams=4):
    """Return (kwargs for oracle.OracleRaster, extra info).  mode: 'sh' (in-kernel SH) or
    'colors' (colors_precomp); cov_mode: 'scale_rot' or 'cov3D'; feature: 'sh' | 'precomp' |
    None."""
    g = make_gaussians(P, sh_degree=sh_degree, seed=seed, scale_mult=scale_mult)
    c = make_cameras(max(n_cams, cam + 1), W, H, seed=seed)[cam]
    kw = dict(
        means3D=g.xyz.numpy(),
        opacities=g.get_opacity().numpy(),
        viewmatrix=c.world_view_transform.numpy(),
        projmatrix=c.full_proj_transform.numpy(),
        campos=c.camera_center.numpy(),
        tanfovx=math.tan(c.FoVx * 0.5),
        tanfovy=math.tan(c.FoVy * 0.5),
        image_height=H, image_width=W,
        bg=np.asarray(bg, np.float32),
        sh_degree=active_degree,
        include_feature=feature is not None,
    )
    gen = torch.Generator().manual_seed(seed + 17)
    if mode == "sh":
        kw["shs"] = g.get_features().numpy()
    else:
        kw["colors_precomp"] = torch.rand((P, 3), generator=gen).numpy()
    if cov_mode == "scale_rot":
        kw["scales"] = g.get_scaling().numpy()
        kw["rotations"] = g.get_rotation().numpy()
    else:
        # build_scaling_rotation + strip_symmetric (utils/general_utils.py:74-120), float64 -> f32
        s = g.get_scaling().double()
        q = g.get_rotation().double()
        r, x, y, z = q.unbind(-1)
        R = torch.stack([1 - 2 * (y * y + z * z), 2 * (x * y - r * z), 2 * (x * z + r * y),
                         2 * (x * y + r * z), 1 - 2 * (x * x + z * z), 2 * (y * z - r * x),
                         2 * (x * z - r * y), 2 * (y * z + r * x), 1 - 2 * (x * x + y * y)],
                        -1).view(-1, 3, 3)
        L = R @ torch.diag_embed(s)
        S = L @ L.transpose(1, 2)
        kw["cov3D_precomp"] = torch.stack([S[:, 0, 0], S[:, 0, 1], S[:, 0, 2], S[:, 1, 1],
                                           S[:, 1, 2], S[:, 2, 2]], -1).float().numpy()
    if feature == "sh":
        kw["shs_language"] = g.language_feature.numpy()
    elif feature == "precomp":
        kw["language_feature_precomp"] = torch.randn((P, 3), generator=gen).numpy()
    if confidence is not None:
        kw["confidence"] = np.asarray(confidence, np.float32).reshape(P)
    return kw


def to_torch_call(kw, device="cuda", requires_grad=True):
    """Build (GaussianRasterizationSettings, inputs dict of leaf tensors) for the HIP path."""
    from diff_gaussian_rasterization import GaussianRasterizationSettings

    def t(x):
        return None if x is None else torch.tensor(np.asarray(x), device=device)

    P = kw["means3D"].shape[0]
    settings = GaussianRasterizationSettings(
        image_height=kw["image_height"], image_width=kw["image_width"],
        tanfovx=kw["tanfovx"], tanfovy=kw["tanfovy"], bg=t(kw["bg"]), scale_modifier=1.0,
        viewmatrix=t(kw["viewmatrix"]), projmatrix=t(kw["projmatrix"]),
        sh_degree=kw["sh_degree"], campos=t(kw["campos"]), prefiltered=False, debug=False,
        include_feature=kw["include_feature"],
        confidence=t(kw["confidence"]).view(P, 1) if kw.get("confidence") is not None else None)
    inp = {}
    for name, key in (("means3D", "means3D"), ("opacities", "opacities"), ("shs", "shs"),
                      ("colors_precomp", "colors_precomp"), ("scales", "scales"),
                      ("rotations", "rotations"), ("cov3D_precomp", "cov3D_precomp"),
                      ("shs_language", "shs_language"),
                      ("language_feature_precomp", "language_feature_precomp")):
        v = kw.get(key)
        if v is not None:
            tv = t(v).float()
            if name == "opacities":
                tv = tv.view(P, 1)
            inp[name] = tv.clone().requires_grad_(requires_grad)
    inp["means2D"] = torch.zeros((P, 3), device=device, requires_grad=requires_grad)
    return settings, inp
