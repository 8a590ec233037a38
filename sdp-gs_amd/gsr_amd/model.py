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
        return [self._xyz, self._features_dc, self._features_rest, self._scaling, self._rotation,
                self._opacity, self._language_feature]

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
