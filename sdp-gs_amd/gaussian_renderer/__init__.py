"""Drop-in counterpart of gaussian_renderer/__init__.py::render() (:209-338), the caller of the hot
path.  Same signature, same flag-driven input assembly (compute_cov3D_python, convert_SHs_python,
use_confidence, opt.include_feature, override_color / override_language) and the same returned
dict; the only deliberate difference is that screenspace_points follows the model's device
instead of a hard-coded "cuda" (:217), so the function is device-agnostic.
"""
from __future__ import annotations

import math
import os
import sys

import torch

_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if _PKG_ROOT not in sys.path:
    sys.path.insert(0, _PKG_ROOT)

from diff_gaussian_rasterization import (GaussianRasterizationSettings, GaussianRasterizer,  # noqa: E402
                                         rasterize_gaussians_fused, rasterize_views_fused)
from gsr_amd.sh import eval_sh  # noqa: E402

_RAW = ("_features_dc", "_features_rest", "_opacity", "_scaling", "_rotation")


def _fused_eligible(pc, pipe, opt, override_color, override_language) -> bool:
    """True when the fused entry point computes what render() would: a model with GaussianModel's
    standard activations (scene/gaussian_model.py:33-41), scales/rotations (not a Python cov3D),
    no overrides.  Both colour paths qualify: with convert_SHs_python=False render() hands the
    rasterizer get_features (SH evaluated in-kernel, forward.cu:20-71); with the reference's
    default convert_SHs_python=True it evaluates the same function in Python
    (gaussian_renderer/__init__.py:269-287: eval_sh + 0.5, clamp_min 0; language features
    eval_sh(0)/(norm + 1e-9)), which the fused preprocess evaluates in-kernel with the matching
    gradient (clamp_min passes the gradient where the value is >= 0, the kernel's `clamped` bit
    blocks it where it is < 0).  GSR_FUSED=0 forces the unfused path."""
    if os.environ.get("GSR_FUSED", "1") == "0":
        return False
    if pipe.compute_cov3D_python or override_color is not None:
        return False
    # opt.include_feature = False with the Python colour path: the reference renders the colours
    # again as the feature channels (language_feature_precomp = colors_precomp, :296-298), so
    # "feature" is the bg-0 colour blend and its gradient reaches the SH leaves through the
    # colours -- the unfused branch below does exactly that.  With the
    # in-kernel SH path (convert_SHs_python = False) colors_precomp is None and both branches
    # render zero feature channels.
    if not opt.include_feature and pipe.convert_SHs_python:
        return False
    if opt.include_feature and (override_language is not None
                                or getattr(pc, "_language_feature", None) is None):
        return False
    if not all(isinstance(getattr(pc, n, None), torch.Tensor) for n in _RAW):
        return False
    return (getattr(pc, "scaling_activation", None) is torch.exp
            and getattr(pc, "opacity_activation", None) is torch.sigmoid
            and getattr(pc, "rotation_activation", None) is torch.nn.functional.normalize)


class _RenderPkg(dict):
    """render()'s result dict with entries computed on first access (train.py never reads
    "opacity", so the fused path does not launch its sigmoid per view).  Behaves as the plain
    dict the reference returns: keys, iteration, `in`, get() and copies see every entry.  A lazy
    entry is evaluated from the model as it is at first access."""

    def __init__(self, items, lazy):
        super().__init__(items)
        self._lazy = dict(lazy)

    def _fill(self):
        for k in list(self._lazy):
            self[k]
        return self

    def __missing__(self, key):
        if key in self._lazy:
            value = self._lazy.pop(key)()
            self[key] = value
            return value
        raise KeyError(key)

    def __contains__(self, key):
        return super().__contains__(key) or key in self._lazy

    def get(self, key, default=None):
        return self[key] if key in self else default

    def __iter__(self):
        return dict.__iter__(self._fill())

    def __len__(self):
        return super().__len__() + len(self._lazy)

    def keys(self):
        return dict.keys(self._fill())

    def values(self):
        return dict.values(self._fill())

    def items(self):
        return dict.items(self._fill())

    def copy(self):
        return dict(dict.items(self._fill()))


_ZEROS = {}  # (device, views) -> zero buffer of the last shape asked for (means2D leaves)


def _zero_leaf(xyz, views=None):
    """A new leaf tensor (requires_grad, own .grad) whose values are zeros, like
    torch.zeros_like(xyz, requires_grad=True) -- shape [views, *xyz.shape] when views is given
    (render_views) -- backed by a zero buffer shared by all calls of the same shape: the buffer is
    never written (the rasterizer only returns means2D's gradient)."""
    shape = tuple(xyz.shape) if views is None else (int(views),) + tuple(xyz.shape)
    key = (xyz.device, views is not None)
    z = _ZEROS.get(key)
    if z is None or tuple(z.shape) != shape or z.dtype != xyz.dtype:
        z = torch.zeros(shape, dtype=xyz.dtype, device=xyz.device)
        _ZEROS[key] = z
    return z.detach().requires_grad_(True)


def render(viewpoint_camera, pc, pipe, bg_color: torch.Tensor, opt, scaling_modifier=1.0,
           override_color=None, override_language=None):
    xyz = pc.get_xyz
    fused = _fused_eligible(pc, pipe, opt, override_color, override_language)
    if fused:
        # the kernel never reads means2D's values, only returns its gradient: a fresh zero leaf
        # stands in for the reference's zeros_like(...) + 0 non-leaf (fill + add); its .grad is
        # the same per-view screen-space gradient.  The leaf is a new tensor over one cached
        # zero buffer per device and shape, so a view costs no fill kernel.
        screenspace_points = _zero_leaf(xyz)
    else:
        screenspace_points = torch.zeros_like(xyz, dtype=xyz.dtype, requires_grad=True,
                                              device=xyz.device) + 0
        try:
            screenspace_points.retain_grad()
        except Exception:
            pass

    tanfovx = math.tan(viewpoint_camera.FoVx * 0.5)
    tanfovy = math.tan(viewpoint_camera.FoVy * 0.5)
    if pipe.use_confidence:
        confidence = pc.confidence
    elif fused:
        confidence = None  # the kernels treat a missing confidence as ones (no fill per view)
    else:
        confidence = torch.ones_like(pc.confidence)
    raster_settings = GaussianRasterizationSettings(
        image_height=int(viewpoint_camera.image_height),
        image_width=int(viewpoint_camera.image_width),
        tanfovx=tanfovx,
        tanfovy=tanfovy,
        bg=bg_color,
        scale_modifier=scaling_modifier,
        viewmatrix=viewpoint_camera.world_view_transform,
        projmatrix=viewpoint_camera.full_proj_transform,
        sh_degree=pc.active_sh_degree,
        campos=viewpoint_camera.camera_center,
        prefiltered=False,
        include_feature=True,
        confidence=confidence,
        debug=pipe.debug)
    rasterizer = GaussianRasterizer(raster_settings=raster_settings)

    if fused:
        # Default configuration: the activations / cat of GaussianModel's getters run inside the
        # preprocess kernel and the backward writes the raw leaves' grads (identical outputs).
        lang = pc._language_feature if opt.include_feature else None
        rendered_image, rendered_depth, rendered_alpha, language_feature_image, radii = \
            rasterize_gaussians_fused(xyz, screenspace_points, pc._features_dc,
                                      pc._features_rest, pc._opacity, pc._scaling, pc._rotation,
                                      lang, raster_settings)
        return _RenderPkg({"render": rendered_image,
                           "depth": rendered_depth,
                           "alpha": rendered_alpha,
                           "feature": language_feature_image,
                           "viewspace_points": screenspace_points,
                           "radii": radii,
                           "color": None},
                          {"opacity": lambda: pc.get_opacity,
                           "visibility_filter": lambda: radii > 0})

    means3D = xyz
    means2D = screenspace_points
    opacity = pc.get_opacity

    scales = rotations = cov3D_precomp = None
    if pipe.compute_cov3D_python:
        cov3D_precomp = pc.get_covariance(scaling_modifier)
    else:
        scales = pc.get_scaling
        rotations = pc.get_rotation

    shs = shs_language = colors_precomp = language_feature_precomp = None
    if override_color is None:
        if pipe.convert_SHs_python:
            shs_view = pc.get_features.transpose(1, 2).view(-1, 3, (pc.max_sh_degree + 1) ** 2)
            dir_pp = (xyz - viewpoint_camera.camera_center.repeat(pc.get_features.shape[0], 1))
            dir_pp_normalized = dir_pp / dir_pp.norm(dim=1, keepdim=True)
            sh2rgb = eval_sh(pc.active_sh_degree, shs_view, dir_pp_normalized)
            colors_precomp = torch.clamp_min(sh2rgb + 0.5, 0.0)
        else:
            shs = pc.get_features
    else:
        colors_precomp = override_color

    if opt.include_feature:
        if override_language is None:
            if pipe.convert_SHs_python:
                lf = pc.get_language_feature
                shs_view = lf.view(-1, 3, 1)
                dir_pp = (xyz - viewpoint_camera.camera_center.repeat(lf.shape[0], 1))
                dir_pp_normalized = dir_pp / dir_pp.norm(dim=1, keepdim=True)
                sh2language = eval_sh(0, shs_view, dir_pp_normalized)
                language_feature_precomp = sh2language / (sh2language.norm(dim=-1, keepdim=True) + 1e-9)
            else:
                shs_language = pc.get_language_feature
        else:
            language_feature_precomp = override_language
    else:
        language_feature_precomp = colors_precomp

    rendered_image, rendered_depth, rendered_alpha, language_feature_image, radii = rasterizer(
        means3D=means3D,
        means2D=means2D,
        shs=shs,
        shs_language=shs_language,
        colors_precomp=colors_precomp,
        language_feature_precomp=language_feature_precomp,
        opacities=opacity,
        scales=scales,
        rotations=rotations,
        cov3D_precomp=cov3D_precomp)

    return {"render": rendered_image,
            "depth": rendered_depth,
            "alpha": rendered_alpha,
            "opacity": opacity,
            "feature": language_feature_image,
            "viewspace_points": screenspace_points,
            "visibility_filter": radii > 0,
            "radii": radii,
            "color": colors_precomp}


class ViewGrad:
    """Per-view handle on the screen-space gradient of a multi-view call: `.grad` is view v's
    [P,3] slice of the shared [V,P,3] leaf -- what the reference reads from
    viewspace_point_tensor.grad (train.py:220, add_densification_stats)."""
    __slots__ = ("leaf", "index")

    def __init__(self, leaf, index):
        self.leaf, self.index = leaf, index

    @property
    def grad(self):
        g = self.leaf.grad
        return None if g is None else g[self.index]


def _settings(cam, pc, pipe, bg_color, scaling_modifier, confidence):
    return GaussianRasterizationSettings(
        image_height=int(cam.image_height), image_width=int(cam.image_width),
        tanfovx=math.tan(cam.FoVx * 0.5), tanfovy=math.tan(cam.FoVy * 0.5), bg=bg_color,
        scale_modifier=scaling_modifier, viewmatrix=cam.world_view_transform,
        projmatrix=cam.full_proj_transform, sh_degree=pc.active_sh_degree,
        campos=cam.camera_center, prefiltered=False, include_feature=True,
        confidence=confidence, debug=pipe.debug)


def render_views(viewpoint_cameras, pc, pipe, bg_color: torch.Tensor, opt, scaling_modifier=1.0,
                 streams=None):
    """render() for several cameras of one step: a list of render()'s dicts, one per camera,
    with identical values.  Where render() would take the fused path and the cameras share an
    image size, every view's forward is issued by ONE host call (and, through autograd, every
    backward by one call): diff_gaussian_rasterization.rasterize_views_fused, views spread over
    `streams`.  The dicts' images are views into [V,...] tensors; "viewspace_points" is a
    ViewGrad whose .grad is that view's screen-space gradient.  Otherwise (unfused
    configurations, mixed image sizes) this is render() per camera."""
    cams = list(viewpoint_cameras)
    if not cams:
        return []
    same = len({(int(c.image_height), int(c.image_width)) for c in cams}) == 1
    if not (same and _fused_eligible(pc, pipe, opt, None, None)):
        return [render(c, pc, pipe, bg_color, opt, scaling_modifier) for c in cams]
    xyz = pc.get_xyz
    V = len(cams)
    means2D = _zero_leaf(xyz, V)
    confidence = pc.confidence if pipe.use_confidence else None
    settings = [_settings(c, pc, pipe, bg_color, scaling_modifier, confidence) for c in cams]
    lang = pc._language_feature if opt.include_feature else None
    color, depth, alpha, feature, radii = rasterize_views_fused(
        xyz, means2D, pc._features_dc, pc._features_rest, pc._opacity, pc._scaling, pc._rotation,
        lang, settings, streams)
    # the stacked [V,...] outputs: a caller seeding the backward of every view at once uses
    # these (autograd on the per-view slices would materialise a [V,...] zero gradient per view)
    stacked = {"render": color, "depth": depth, "alpha": alpha, "feature": feature,
               "viewspace_points": means2D, "radii": radii}
    # per-view images by unbind: a loss over some or all of them back-propagates through ONE
    # stack of the per-view gradients (indexing would add a [V,...] zero tensor per view)
    per = [t.unbind(0) for t in (color, depth, alpha, feature)]
    out = []
    for v in range(V):
        r = radii[v]
        out.append(_RenderPkg({"render": per[0][v], "depth": per[1][v], "alpha": per[2][v],
                               "feature": per[3][v], "viewspace_points": ViewGrad(means2D, v),
                               "radii": r, "color": None, "views": stacked, "view_index": v},
                              {"opacity": lambda: pc.get_opacity,
                               "visibility_filter": (lambda r=r: r > 0)}))
    return out
