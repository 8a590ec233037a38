"""Seeded synthetic scenes: Gaussians in the GaussianModel parameterisation
(scene/gaussian_model.py:146-183, 189-214) and LLFF-style forward-facing cameras.

There is no dataset or checkpoint in this environment, so every test, the smoke check and the
benchmark draw their inputs from here; the CPU baseline sees the same tensors.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np
import torch

from .camera import focal2fov, look_at_R, make_camera

SH_C0 = 0.28209479177387814


def RGB2SH(rgb):
    return (rgb - 0.5) / SH_C0  # utils/sh_utils.py:114-115


@dataclass
class GaussianParams:
    """Raw (pre-activation) parameters, as GaussianModel stores them."""
    xyz: torch.Tensor              # [P,3]
    features_dc: torch.Tensor      # [P,1,3]
    features_rest: torch.Tensor    # [P,(D+1)^2-1,3]
    scaling: torch.Tensor          # [P,3] log-scale
    rotation: torch.Tensor         # [P,4] unnormalised quaternion (w,x,y,z)
    opacity: torch.Tensor          # [P,1] logit
    language_feature: torch.Tensor  # [P,3]
    confidence: torch.Tensor       # [P,1]
    max_sh_degree: int = 3

    @property
    def P(self):
        return int(self.xyz.shape[0])

    def to(self, device):
        kw = {k: getattr(self, k).to(device) for k in ("xyz", "features_dc", "features_rest",
                                                      "scaling", "rotation", "opacity",
                                                      "language_feature", "confidence")}
        return GaussianParams(max_sh_degree=self.max_sh_degree, **kw)

    # activations of scene/gaussian_model.py:26-41,146-183
    def get_xyz(self):
        return self.xyz

    def get_scaling(self):
        return torch.exp(self.scaling)

    def get_rotation(self):
        return torch.nn.functional.normalize(self.rotation)

    def get_opacity(self):
        return torch.sigmoid(self.opacity)

    def get_features(self):
        return torch.cat((self.features_dc, self.features_rest), dim=1)

    def parameters(self):
        return [self.xyz, self.features_dc, self.features_rest, self.scaling, self.rotation,
                self.opacity, self.language_feature]


def make_gaussians(P: int, sh_degree: int = 3, seed: int = 0, extent: float = 1.0,
                   scale_mult: float = 1.0) -> GaussianParams:
    g = torch.Generator().manual_seed(seed)
    xyz = (torch.rand((P, 3), generator=g) * 2 - 1) * extent
    spacing = (8.0 / max(P, 1)) ** (1.0 / 3.0) * extent
    scale = (torch.rand((P, 3), generator=g) + 0.5) * 0.5 * spacing * scale_mult
    rot = torch.randn((P, 4), generator=g)
    opac = torch.rand((P, 1), generator=g) * 0.8 + 0.1
    rgb = torch.rand((P, 1, 3), generator=g)
    nrest = (sh_degree + 1) ** 2 - 1
    rest = torch.randn((P, nrest, 3), generator=g) * 0.05
    lang = torch.randn((P, 3), generator=g)
    return GaussianParams(xyz=xyz.float(), features_dc=RGB2SH(rgb).float(),
                          features_rest=rest.float(), scaling=torch.log(scale).float(),
                          rotation=rot.float(), opacity=torch.log(opac / (1 - opac)).float(),
                          language_feature=lang.float(), confidence=torch.ones((P, 1)),
                          max_sh_degree=sh_degree)


def make_cameras(n: int, width: int, height: int, seed: int = 0, device="cpu", distance=4.0,
                 jitter=0.5):
    """Camera 0 sits at (0,0,-distance) looking +z (R = I, T = (0,0,distance)); cameras 1..n-1
    are jittered in x,y on the same plane and look at the origin.  focal = 0.8 * width."""
    focal = 0.8 * width
    fovx, fovy = focal2fov(focal, width), focal2fov(focal, height)
    cams = []
    for i in range(n):
        if i == 0:
            c = np.array([0.0, 0.0, -distance])
        else:
            rng = np.random.default_rng(seed * 100003 + i)
            jx, jy = rng.uniform(-jitter, jitter, size=2)
            c = np.array([jx, jy, -distance])
        R = look_at_R(c)
        T = -R.T @ c
        cams.append(make_camera(R, T, fovx, fovy, width, height, uid=i, device=device))
    return cams


def upstream_grads(H: int, W: int, seed: int = 1, device="cpu"):
    g = torch.Generator().manual_seed(seed)
    dimg = torch.randn((3, H, W), generator=g)
    ddepth = torch.randn((1, H, W), generator=g)
    dfeat = torch.randn((3, H, W), generator=g)
    return dimg.to(device), ddepth.to(device), dfeat.to(device)


def training_targets(n: int, H: int, W: int, seed: int = 2, device="cpu"):
    """Synthetic per-camera training targets for the train-step benchmark: a ground-truth image
    [3,H,W] in [0,1] and a monocular depth map [1,H,W] in [1,3] (the shape train.py reads from
    viewpoint_cam.original_image / depth_mono, train.py:97,117)."""
    g = torch.Generator().manual_seed(seed)
    gts = [torch.rand((3, H, W), generator=g).to(device) for _ in range(n)]
    monos = [(1.0 + 2.0 * torch.rand((1, H, W), generator=g)).to(device) for _ in range(n)]
    return gts, monos
