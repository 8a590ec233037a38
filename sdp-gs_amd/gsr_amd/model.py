"""Parameter store with GaussianModel's getters (scene/gaussian_model.py:146-183).

The rasterizer's inputs are the activated parameters: get_xyz, get_scaling = exp(_scaling),
get_rotation = normalize(_rotation), get_opacity = sigmoid(_opacity),
get_features = cat(f_dc, f_rest), get_language_feature, get_covariance.  render() (the caller of
the hot path) reads exactly these, plus active_sh_degree / max_sh_degree / confidence.
"""
from __future__ import annotations

import torch

from .synthetic import GaussianParams


def build_rotation(r):
    """utils/general_utils.py:88-107 (device-agnostic)."""
    norm = torch.sqrt(r[:, 0] * r[:, 0] + r[:, 1] * r[:, 1] + r[:, 2] * r[:, 2] + r[:, 3] * r[:, 3])
    q = r / norm[:, None]
    R = torch.zeros((q.size(0), 3, 3), device=r.device, dtype=r.dtype)
    w, x, y, z = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    R[:, 0, 0] = 1 - 2 * (y * y + z * z)
    R[:, 0, 1] = 2 * (x * y - w * z)
    R[:, 0, 2] = 2 * (x * z + w * y)
    R[:, 1, 0] = 2 * (x * y + w * z)
    R[:, 1, 1] = 1 - 2 * (x * x + z * z)
    R[:, 1, 2] = 2 * (y * z - w * x)
    R[:, 2, 0] = 2 * (x * z - w * y)
    R[:, 2, 1] = 2 * (y * z + w * x)
    R[:, 2, 2] = 1 - 2 * (x * x + y * y)
    return R


def build_covariance_from_scaling_rotation(scaling, scaling_modifier, rotation):
    """scene/gaussian_model.py:27-31 + utils/general_utils.py:73-120."""
    s = scaling_modifier * scaling
    L = build_rotation(rotation) @ torch.diag_embed(s)
    cov = L @ L.transpose(1, 2)
    return torch.stack([cov[:, 0, 0], cov[:, 0, 1], cov[:, 0, 2], cov[:, 1, 1], cov[:, 1, 2],
                        cov[:, 2, 2]], dim=1)


class SplatModel:
    """Leaf tensors in GaussianModel's raw parameterisation with its activation getters."""

    # scene/gaussian_model.py:33-41 (setup_functions)
    scaling_activation = staticmethod(torch.exp)
    opacity_activation = staticmethod(torch.sigmoid)
    rotation_activation = staticmethod(torch.nn.functional.normalize)
    scaling_inverse_activation = staticmethod(torch.log)

    def __init__(self, params: GaussianParams, device="cuda", active_sh_degree=None):
        p = params.to(device)
        self.max_sh_degree = p.max_sh_degree
        self.active_sh_degree = p.max_sh_degree if active_sh_degree is None else active_sh_degree
        self._xyz = p.xyz.clone().requires_grad_(True)
        self._features_dc = p.features_dc.clone().requires_grad_(True)
        self._features_rest = p.features_rest.clone().requires_grad_(True)
        self._scaling = p.scaling.clone().requires_grad_(True)
        self._rotation = p.rotation.clone().requires_grad_(True)
        self._opacity = p.opacity.clone().requires_grad_(True)
        self._language_feature = p.language_feature.clone().requires_grad_(True)
        self.confidence = p.confidence.clone()

    def parameters(self):
        return [p for p in (self._xyz, self._features_dc, self._features_rest, self._scaling,
                            self._rotation, self._opacity, self._language_feature) if p is not None]

    @property
    def get_xyz(self):
        return self._xyz

    @property
    def get_scaling(self):
        return self.scaling_activation(self._scaling)

    @property
    def get_rotation(self):
        return self.rotation_activation(self._rotation)

    @property
    def get_opacity(self):
        return self.opacity_activation(self._opacity)

    @property
    def get_features(self):
        return torch.cat((self._features_dc, self._features_rest), dim=1)

    @property
    def get_language_feature(self):
        return self._language_feature

    def get_covariance(self, scaling_modifier=1):
        # the reference passes the raw _rotation here (scene/gaussian_model.py:185-186)
        return build_covariance_from_scaling_rotation(self.get_scaling, scaling_modifier,
                                                      self._rotation)

    @classmethod
    def from_point_cloud(cls, points, colors, max_sh_degree=3, device="cuda"):
        """create_from_pcd (scene/gaussian_model.py:189-214): SH DC from the colours (RGB2SH),
        isotropic log-scales from the mean squared 3-NN distance (distCUDA2 = gsr_dist_knn3,
        clamped at 1e-7), identity rotations, opacity logit(0.1), confidence 1; the language
        feature starts at zero as training_setup creates it (:223-226)."""
        from .knn import distCUDA2
        pts =torch.tensor(points).float().to(device)
        C0 = 0.28209479177387814  # utils/sh_utils.py RGB2SH
        fused_color = (torch.tensor(colors).float().to(device) - 0.5) / C0
        P = pts.shape[0]
        features = torch.zeros((P, 3, (max_sh_degree + 1) ** 2), device=device)
        features[:, :3, 0] = fused_color
        dist2 = torch.clamp_min(distCUDA2(pts)[0], 0.0000001)
        scales = torch.log(torch.sqrt(dist2))[..., None].repeat(1, 3)
        rots = torch.zeros((P, 4), device=device)
        rots[:, 0] = 1
        x = 0.1 * torch.ones((P, 1), dtype=torch.float, device=device)
        opacities = torch.log(x / (1 - x))  # inverse_sigmoid (utils/general_utils.py)
        gp = GaussianParams(xyz=pts, features_dc=features[:, :, 0:1].transpose(1, 2).contiguous(),
                            features_rest=features[:, :, 1:].transpose(1, 2).contiguous(),
                            scaling=scales, rotation=rots, opacity=opacities,
                            language_feature=torch.zeros((P, 3), device=device),
                            confidence=torch.ones_like(opacities), max_sh_degree=max_sh_degree)
        m = cls(gp, device=device, active_sh_degree=0)
        m.max_radii2D = torch.zeros((P,), device=device)
        return m

    def training_setup(self, training_args, spatial_lr_scale=1.0, prune_from_iter=500):
        """scene/gaussian_model.py:217-271: densification statistics, parameters as nn.Parameter,
        the named param groups (language group first when include_feature) and
        Adam(lr=0.0, eps=1e-15) -- here the one-launch FusedAdam.  `args.prune_from_iter`
        (arguments/__init__.py:92) is what prune_points consults."""
        from types import SimpleNamespace

        from .optim import FusedAdam
        ta = training_args
        P = self._xyz.shape[0]
        dev = self._xyz.device
        self.percent_dense = ta.percent_dense
        self.spatial_lr_scale = spatial_lr_scale
        self.args = SimpleNamespace(prune_from_iter=prune_from_iter)
        self.xyz_gradient_accum = torch.zeros((P, 1), device=dev)
        self.denom = torch.zeros((P, 1), device=dev)
        self.max_radii2D = torch.zeros((P,), device=dev)
        for name in ("_xyz", "_features_dc", "_features_rest", "_scaling", "_rotation",
                     "_opacity", "_language_feature"):
            setattr(self, name, torch.nn.Parameter(getattr(self, name).detach()
                                                   .requires_grad_(True)))
        groups = [
            {"params": [self._xyz], "lr": ta.position_lr_init * spatial_lr_scale, "name": "xyz"},
            {"params": [self._features_dc], "lr": ta.feature_lr, "name": "f_dc"},
            {"params": [self._features_rest], "lr": ta.feature_lr / 20.0, "name": "f_rest"},
            {"params": [self._opacity], "lr": ta.opacity_lr, "name": "opacity"},
            {"params": [self._scaling], "lr": ta.scaling_lr, "name": "scaling"},
            {"params": [self._rotation], "lr": ta.rotation_lr, "name": "rotation"},
        ]
        if getattr(ta, "include_feature", True):
            groups = [{"params": [self._language_feature], "lr": ta.language_feature_lr,
                       "name": "language_feature"}] + groups[1:3] + groups[:1] + groups[3:]
        else:
            self._language_feature = None
        self.optimizer = FusedAdam(groups, lr=0.0, eps=1e-15)
        return self.optimizer


# the reference's densification methods (scene/gaussian_model.py:400-612) on libgsr
from . import densify as _densify  # noqa: E402

_densify.install(SplatModel)

# the reference's PLY methods (scene/gaussian_model.py:286-398)
from . import ply as _ply  # noqa: E402

_ply.install(SplatModel)
