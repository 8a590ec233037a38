"""MI355X drop-in for the `diff_gaussian_rasterization` package.

Mirrors the Python surface of submodules/diff-gaussian-rasterization/diff_gaussian_rasterization/
__init__.py (GaussianRasterizationSettings :157-169, GaussianRasterizer :171-220,
_RasterizeGaussians :44-155) in its *extended* form -- the one gaussian_renderer/__init__.py:228-243
and :315-326 actually calls (include_feature / confidence settings, shs_language /
language_feature_precomp inputs, five outputs image/depth/alpha/feature/radii).
The native side is libgsr.so (include/gsr.h), hand-written HIP for gfx950; there is no CPU path.
"""
from __future__ import annotations

import os
import time
import sys
from typing import NamedTuple, Optional

import torch
import torch.nn as nn

_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if _PKG_ROOT not in sys.path:
    sys.path.insert(0, _PKG_ROOT)

from gsr_amd import _lib  # noqa: E402

__all__ = ["GaussianRasterizationSettings", "GaussianRasterizer", "rasterize_gaussians",
           "rasterize_gaussians_extended", "rasterize_gaussians_fused", "mark_visible"]

# counts of the most recent forward: num_rendered is the reference's value (the boundary's first
# return value, kept in ctx.num_rendered), num_instances the tile instances actually binned after
# the exact tile cull (include/gsr.h gsr_last_forward_instances; bench.py's algorithmic bytes)
LAST_STATS = {"num_rendered": 0, "num_instances": 0, "P": 0}


def cpu_deep_copy_tuple(input_tuple):
    # diff_gaussian_rasterization/__init__.py:17-19
    return tuple(item.cpu().clone() if isinstance(item, torch.Tensor) else item for item in input_tuple)


def _opt(t: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
    """None or an empty tensor (the reference's torch.Tensor([]) placeholder) -> None."""
    if t is None or (isinstance(t, torch.Tensor) and t.numel() == 0):
        return None
    return t


def _dev_f32(t: Optional[torch.Tensor], name: str, device) -> Optional[torch.Tensor]:
    if t is None:
        return None
    if not t.is_cuda:
        raise RuntimeError(f"{name} must be a tensor on the HIP device (got {t.device}); "
                           "libgsr has no CPU path")
    if t.device != device:
        raise RuntimeError(f"{name} is on {t.device}, expected {device}")
    if t.dtype != torch.float32:
        t = t.float()
    return t.contiguous()


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else t.data_ptr()


def rasterize_gaussians(means3D, means2D, sh, colors_precomp, opacities, scales, rotations,
                        cov3Ds_precomp, raster_settings):
    """Vendored 2-output entry point (diff_gaussian_rasterization/__init__.py:21-42): (color, radii)."""
    color, _depth, _alpha, _feature, radii = _RasterizeGaussians.apply(
        means3D, means2D, sh, None, colors_precomp, None, opacities, scales, rotations,
        cov3Ds_precomp, raster_settings)
    return color, radii


def rasterize_gaussians_extended(means3D, means2D, sh, sh_language, colors_precomp,
                                 language_feature_precomp, opacities, scales, rotations,
                                 cov3Ds_precomp, raster_settings):
    """Extended entry point: (color, depth, alpha, feature, radii)."""
    return _RasterizeGaussians.apply(means3D, means2D, sh, sh_language, colors_precomp,
                                     language_feature_precomp, opacities, scales, rotations,
                                     cov3Ds_precomp, raster_settings)


class _RasterizeGaussians(torch.autograd.Function):
    @staticmethod
    def forward(ctx, means3D, means2D, sh, sh_language, colors_precomp, language_feature_precomp,
                opacities, scales, rotations, cov3Ds_precomp, raster_settings):
        rs = raster_settings
        if means3D.ndim != 2 or means3D.shape[1] != 3:
            raise RuntimeError("means3D must have dimensions (num_points, 3)")
        dev = means3D.device
        P = int(means3D.shape[0])
        H, W = int(rs.image_height), int(rs.image_width)
        include_feature = bool(getattr(rs, "include_feature", False))

        m3 = _dev_f32(means3D, "means3D", dev)
        shs = _dev_f32(_opt(sh), "shs", dev)
        shl = _dev_f32(_opt(sh_language), "shs_language", dev) if include_feature else None
        col = _dev_f32(_opt(colors_precomp), "colors_precomp", dev)
        lfp = _dev_f32(_opt(language_feature_precomp), "language_feature_precomp", dev) if include_feature else None
        if lfp is not None:
            shl = None  # precomputed features take precedence over in-kernel evaluation
        op = _dev_f32(opacities, "opacities", dev)
        sc = _dev_f32(_opt(scales), "scales", dev)
        rot = _dev_f32(_opt(rotations), "rotations", dev)
        cov = _dev_f32(_opt(cov3Ds_precomp), "cov3D_precomp", dev)
        conf = _opt(getattr(rs, "confidence", None))
        conf = _dev_f32(conf, "confidence", dev)
        bg = _dev_f32(rs.bg, "bg", dev)
        view = _dev_f32(rs.viewmatrix, "viewmatrix", dev)
        proj = _dev_f32(rs.projmatrix, "projmatrix", dev)
        campos = _dev_f32(rs.campos, "campos", dev)
        M = int(shs.shape[1]) if shs is not None and shs.ndim >= 2 else 0
        if shs is not None and shs.ndim == 2:  # [P, 3*M] flat layout
            M = shs.shape[1] // 3

        fopts = dict(dtype=torch.float32, device=dev)
        color = torch.empty((3, H, W), **fopts)
        depth = torch.empty((1, H, W), **fopts)
        alpha = torch.empty((1, H, W), **fopts)
        feature = torch.empty((3, H, W), **fopts)
        radii = torch.empty((P,), dtype=torch.int32, device=dev)
        holder = _lib.BufferHolder(dev)
        L = _lib.load()
        nr = _lib.ctypes.c_int(0)
        stream = _lib.raw_stream(dev)
        args = (P, M, _ptr(bg), _ptr(m3), _ptr(col), _ptr(op), _ptr(sc), _ptr(rot),
                float(rs.scale_modifier), _ptr(cov), _ptr(view), _ptr(proj), float(rs.tanfovx),
                float(rs.tanfovy), H, W, _ptr(shs), int(rs.sh_degree), _ptr(campos),
                int(bool(rs.prefiltered)), _ptr(shl), _ptr(lfp), _ptr(conf), int(include_feature),
                _ptr(color), _ptr(depth), _ptr(alpha), _ptr(feature), _ptr(radii),
                _lib.ctypes.byref(nr), _lib.alloc_callback(), holder.key, stream,
                _debug_flags(rs.debug))
        try:
            with _lib.on_device(dev):
                rc = L.gsr_rasterize_gaussians(*args)
            _lib.check(rc)
        except Exception:
            if rs.debug:
                cpu_args = cpu_deep_copy_tuple((rs.bg, means3D, colors_precomp, opacities, scales,
                                                rotations, rs.scale_modifier, cov3Ds_precomp,
                                                rs.viewmatrix, rs.projmatrix, rs.tanfovx,
                                                rs.tanfovy, H, W, sh, rs.sh_degree, rs.campos,
                                                rs.prefiltered, rs.debug))
                torch.save(cpu_args, "snapshot_fw.dump")
                print("\nAn error occured in forward. Please forward snapshot_fw.dump for debugging.")
            raise
        finally:
            holder.release()
        num_rendered = int(nr.value)
        LAST_STATS["num_rendered"] = num_rendered
        LAST_STATS["num_instances"] = int(L.gsr_last_forward_instances())
        LAST_STATS["P"] = P

        ctx.raster_settings = rs
        ctx.gsr_flags = _debug_flags(rs.debug)
        ctx.num_rendered = num_rendered
        ctx.meta = dict(P=P, M=M, H=H, W=W, include_feature=include_feature,
                        has_shs=shs is not None, has_shl=shl is not None,
                        has_col=col is not None, has_lfp=lfp is not None,
                        has_sc=sc is not None, has_cov=cov is not None,
                        op_shape=tuple(opacities.shape))
        empty = torch.empty(0, device=dev)
        geom, binning, image = (b if b is not None else torch.empty(0, dtype=torch.uint8, device=dev)
                                for b in holder.bufs)
        ctx.save_for_backward(m3, radii, shs if shs is not None else empty,
                              shl if shl is not None else empty, col if col is not None else empty,
                              lfp if lfp is not None else empty, sc if sc is not None else empty,
                              rot if rot is not None else empty, cov if cov is not None else empty,
                              conf if conf is not None else empty, bg, view, proj, campos,
                              geom, binning, image)
        ctx.mark_non_differentiable(radii)
        # outputs the loss does not use arrive as None (the kernels take NULL as zero) instead of
        # autograd materialising zero images and an int zero radii tensor per view
        ctx.set_materialize_grads(False)
        return color, depth, alpha, feature, radii

    @staticmethod
    def backward(ctx, grad_color, grad_depth, grad_alpha, grad_feature, _grad_radii):
        rs = ctx.raster_settings
        mt = ctx.meta
        (m3, radii, shs, shl, col, lfp, sc, rot, cov, conf, bg, view, proj, campos, geom, binning,
         image) = ctx.saved_tensors
        o = lambda t, flag: t if flag else None  # noqa: E731
        shs, shl, col, lfp = o(shs, mt["has_shs"]), o(shl, mt["has_shl"]), o(col, mt["has_col"]), o(lfp, mt["has_lfp"])
        sc, rot, cov = o(sc, mt["has_sc"]), o(rot, mt["has_sc"]), o(cov, mt["has_cov"])
        conf = conf if conf.numel() > 0 else None
        P, M, H, W = mt["P"], mt["M"], mt["H"], mt["W"]
        dev = m3.device

        def g(t):
            return None if t is None else t.contiguous().float()

        dcol = g(grad_color)
        if dcol is None:
            dcol = torch.zeros((3, H, W), dtype=torch.float32, device=dev)
        ddep, dalp = g(grad_depth), g(grad_alpha)
        dfeat = g(grad_feature) if mt["include_feature"] else None

        fopts = dict(dtype=torch.float32, device=dev)
        d_means2D = torch.empty((P, 3), **fopts)
        d_colors = torch.empty((P, 3), **fopts) if col is not None else None
        d_opac = torch.empty((P, 1), **fopts)
        d_means3D = torch.empty((P, 3), **fopts)
        d_cov = torch.empty((P, 6), **fopts) if cov is not None else None
        d_sh = torch.empty((P, M, 3), **fopts) if shs is not None else None
        d_sc = torch.empty((P, 3), **fopts) if sc is not None else None
        d_rot = torch.empty((P, 4), **fopts) if sc is not None else None
        d_shl = torch.empty((P, 3), **fopts) if shl is not None else None
        d_lfp = torch.empty((P, 3), **fopts) if lfp is not None else None

        L = _lib.load()
        stream = _lib.raw_stream(dev)
        args = (P, M, ctx.num_rendered, _ptr(bg), _ptr(m3), _ptr(radii), _ptr(col), _ptr(sc),
                _ptr(rot), float(rs.scale_modifier), _ptr(cov), _ptr(view), _ptr(proj),
                float(rs.tanfovx), float(rs.tanfovy), H, W, _ptr(dcol), _ptr(ddep), _ptr(dalp),
                _ptr(dfeat), _ptr(shs), int(rs.sh_degree), _ptr(campos), _ptr(shl), _ptr(lfp),
                _ptr(conf), int(mt["include_feature"]), _ptr(geom) if geom.numel() else None,
                _ptr(binning) if binning.numel() else None, _ptr(image) if image.numel() else None,
                _ptr(d_means2D), _ptr(d_colors), _ptr(d_opac), _ptr(d_means3D), _ptr(d_cov),
                _ptr(d_sh), _ptr(d_sc), _ptr(d_rot), _ptr(d_shl), _ptr(d_lfp), stream,
                ctx.gsr_flags)
        try:
            with _lib.on_device(dev):
                rc = L.gsr_rasterize_gaussians_backward(*args)
            _lib.check(rc)
        except Exception:
            if rs.debug:
                torch.save(cpu_deep_copy_tuple((rs.bg, m3, radii, col, sc, rot, rs.scale_modifier,
                                                cov, rs.viewmatrix, rs.projmatrix, rs.tanfovx,
                                                rs.tanfovy, grad_color, shs, rs.sh_degree,
                                                rs.campos, geom, ctx.num_rendered, binning, image,
                                                rs.debug)), "snapshot_bw.dump")
                print("\nAn error occured in backward. Writing snapshot_bw.dump for debugging.\n")
            raise
        # order of forward inputs: means3D, means2D, sh, sh_language, colors_precomp,
        # language_feature_precomp, opacities, scales, rotations, cov3Ds_precomp, raster_settings
        d_opac = d_opac.view(mt["op_shape"])
        return (d_means3D, d_means2D, d_sh, d_shl, d_colors, d_lfp, d_opac, d_sc, d_rot, d_cov, None)


def rasterize_gaussians_fused(means3D, means2D, features_dc, features_rest, opacity_raw,
                              scaling_raw, rotation_raw, language_feature, raster_settings):
    """Fused-activation entry point (include/gsr.h gsr_rasterize_gaussians_fused).

    Takes GaussianModel's raw leaves (_xyz, _features_dc, _features_rest, _opacity, _scaling,
    _rotation, _language_feature; scene/gaussian_model.py:147-180) and applies get_features' cat,
    sigmoid, exp and normalize inside the preprocess kernel; the backward returns the raw leaves'
    gradients directly.  Same outputs as rasterize_gaussians_extended with
    shs = get_features, opacities = get_opacity, scales = get_scaling, rotations = get_rotation,
    shs_language = get_language_feature.
    """
    return _RasterizeGaussiansFused.apply(means3D, means2D, features_dc, features_rest, opacity_raw,
                                          scaling_raw, rotation_raw, language_feature,
                                          raster_settings)


class _RasterizeGaussiansFused(torch.autograd.Function):
    @staticmethod
    def forward(ctx, means3D, means2D, features_dc, features_rest, opacity_raw, scaling_raw,
                rotation_raw, language_feature, raster_settings):
        rs = raster_settings
        if means3D.ndim != 2 or means3D.shape[1] != 3:
            raise RuntimeError("means3D must have dimensions (num_points, 3)")
        dev = means3D.device
        P = int(means3D.shape[0])
        H, W = int(rs.image_height), int(rs.image_width)
        include_feature = bool(getattr(rs, "include_feature", False))
        m3 = _dev_f32(means3D, "means3D", dev)
        dc = _dev_f32(features_dc, "features_dc", dev)
        rest = _dev_f32(_opt(features_rest), "features_rest", dev)
        op = _dev_f32(opacity_raw, "opacity", dev)
        sc = _dev_f32(scaling_raw, "scaling", dev)
        rot = _dev_f32(rotation_raw, "rotation", dev)
        lf = _dev_f32(_opt(language_feature), "language_feature", dev) if include_feature else None
        conf = _dev_f32(_opt(getattr(rs, "confidence", None)), "confidence", dev)
        bg = _dev_f32(rs.bg, "bg", dev)
        view = _dev_f32(rs.viewmatrix, "viewmatrix", dev)
        proj = _dev_f32(rs.projmatrix, "projmatrix", dev)
        campos = _dev_f32(rs.campos, "campos", dev)
        if dc.numel() != 3 * P or (rest is not None and rest.numel() % (3 * max(P, 1))):
            raise RuntimeError("features_dc must be [P,1,3] and features_rest [P,K,3]")
        M = 1 + (rest.numel() // (3 * P) if rest is not None and P else 0)

        fopts = dict(dtype=torch.float32, device=dev)
        color = torch.empty((3, H, W), **fopts)
        depth = torch.empty((1, H, W), **fopts)
        alpha = torch.empty((1, H, W), **fopts)
        feature = torch.empty((3, H, W), **fopts)
        radii = torch.empty((P,), dtype=torch.int32, device=dev)
        holder = _lib.BufferHolder(dev)
        L = _lib.load()
        nr = _lib.ctypes.c_int(0)
        stream = _lib.raw_stream(dev)
        pre = _precolor_lookup(dev, campos, m3, dc, rest, int(rs.sh_degree), M)
        try:
            with _lib.on_device(dev):
                head = (P, M, _ptr(bg), _ptr(m3), _ptr(dc), _ptr(rest), _ptr(op), _ptr(sc),
                        _ptr(rot), float(rs.scale_modifier), _ptr(view), _ptr(proj),
                        float(rs.tanfovx), float(rs.tanfovy), H, W, int(rs.sh_degree),
                        _ptr(campos), int(bool(rs.prefiltered)), _ptr(lf), _ptr(conf),
                        int(include_feature))
                tail = (_ptr(color), _ptr(depth), _ptr(alpha), _ptr(feature), _ptr(radii),
                        _lib.ctypes.byref(nr), _lib.alloc_callback(), holder.key, stream,
                        _debug_flags(rs.debug))
                if pre is not None:  # colour + clamp bits from the multi-view pre-pass
                    rc = L.gsr_rasterize_gaussians_fused_precolor(
                        *head, _ptr(pre[0]), _ptr(pre[1]), *tail)
                else:
                    rc = L.gsr_rasterize_gaussians_fused(*head, *tail)
            _lib.check(rc)
        finally:
            holder.release()
        num_rendered = int(nr.value)
        LAST_STATS["num_rendered"] = num_rendered
        LAST_STATS["num_instances"] = int(L.gsr_last_forward_instances())
        LAST_STATS["P"] = P

        ctx.raster_settings = rs
        ctx.gsr_flags = _debug_flags(rs.debug)
        ctx.num_rendered = num_rendered
        ctx.pre_jac = None if pre is None else pre[2]
        ctx.jac_event = None if pre is None else _jac_ready(dev)
        # grad-into-leaves mode: only when every differentiable input is itself the float32
        # contiguous leaf (then the kernel's pointer IS the parameter's storage)
        leaves = (means3D, features_dc, features_rest, opacity_raw, scaling_raw, rotation_raw,
                  language_feature)
        used = (m3, dc, rest, op, sc, rot, lf)
        ctx.leaves = None
        if grad_into_leaves() and all(
                t is None or (t.is_leaf and t.requires_grad and u is not None
                              and u.data_ptr() == t.data_ptr())
                for t, u in zip(leaves, used)):
            ctx.leaves = leaves
        ctx.meta = dict(P=P, M=M, H=H, W=W, include_feature=include_feature,
                        has_rest=rest is not None, has_lf=lf is not None,
                        shapes=(tuple(features_dc.shape),
                                None if rest is None else tuple(features_rest.shape),
                                tuple(opacity_raw.shape), tuple(scaling_raw.shape),
                                tuple(rotation_raw.shape)))
        empty = torch.empty(0, device=dev)
        geom, binning, image = (b if b is not None else torch.empty(0, dtype=torch.uint8, device=dev)
                                for b in holder.bufs)
        ctx.save_for_backward(m3, radii, dc, rest if rest is not None else empty, op, sc, rot,
                              lf if lf is not None else empty,
                              conf if conf is not None else empty, bg, view, proj, campos,
                              geom, binning, image)
        ctx.mark_non_differentiable(radii)
        # outputs the loss does not use arrive as None (the kernels take NULL as zero) instead of
        # autograd materialising zero images and an int zero radii tensor per view
        ctx.set_materialize_grads(False)
        return color, depth, alpha, feature, radii

    @staticmethod
    def backward(ctx, grad_color, grad_depth, grad_alpha, grad_feature, _grad_radii):
        rs = ctx.raster_settings
        mt = ctx.meta
        (m3, radii, dc, rest, op, sc, rot, lf, conf, bg, view, proj, campos, geom, binning,
         image) = ctx.saved_tensors
        rest = rest if mt["has_rest"] else None
        lf = lf if mt["has_lf"] else None
        conf = conf if conf.numel() > 0 else None
        P, M, H, W = mt["P"], mt["M"], mt["H"], mt["W"]
        dev = m3.device

        def g(t):
            return None if t is None else t.contiguous().float()

        dcol = g(grad_color)
        if dcol is None:
            dcol = torch.zeros((3, H, W), dtype=torch.float32, device=dev)
        ddep, dalp = g(grad_depth), g(grad_alpha)
        dfeat = g(grad_feature) if mt["include_feature"] else None
        s_dc, s_rest, s_op, s_sc, s_rot = mt["shapes"]
        fopts = dict(dtype=torch.float32, device=dev)
        into_leaves = ctx.leaves is not None
        accumulate = into_leaves
        # deferred SH gradients (gsr_amd.pipeline.ViewPipeline): this view stores dL/dRGB [P,3]
        # and the step's flush writes features_dc / features_rest .grad once for all its views
        defer = _SH_DEFER.get(dev.index) if into_leaves else None
        direct = ctx.leaves
        if defer is not None:
            direct = tuple(None if k in (1, 2) else t for k, t in enumerate(ctx.leaves))
        if into_leaves and all(t is None or t.grad is None for t in direct):
            # first view after zero_grad(set_to_none=True): the kernel's store mode writes every
            # element of fresh .grad tensors (zeros for culled Gaussians) -- no memset, no read
            accumulate = False
            for t in direct:
                if t is not None:
                    t.grad = torch.empty_like(t, memory_format=torch.contiguous_format)
        d_rgb = None
        if into_leaves:
            # add straight into the parameters' .grad (created as zeros when absent, as
            # AccumulateGrad would); culled Gaussians are not touched at all
            grads = []
            for t in direct:
                if t is not None and t.grad is None:
                    t.grad = torch.zeros_like(t, memory_format=torch.contiguous_format)
                grads.append(None if t is None else t.grad)
            if any(gr is not None and not gr.is_contiguous() for gr in grads):
                raise RuntimeError("grad-into-leaves needs contiguous .grad tensors")
            d_means3D, d_dc, d_rest, d_op, d_sc, d_rot, d_lf = grads
            d_means2D = torch.empty((P, 3), **fopts)  # always stored by the kernel
            if defer is not None:
                d_rgb = torch.empty((3, P), **fopts)  # planar dL/dRGB (include/gsr.h)
                defer.add(ctx.leaves, d_rgb, campos, m3, int(rs.sh_degree), M)
        else:
            d_means2D = torch.empty((P, 3), **fopts)
            d_means3D = torch.empty((P, 3), **fopts)
            d_dc = torch.empty(s_dc, **fopts)
            d_rest = torch.empty(s_rest, **fopts) if rest is not None else None
            d_op = torch.empty(s_op, **fopts)
            d_sc = torch.empty(s_sc, **fopts)
            d_rot = torch.empty(s_rot, **fopts)
            d_lf = torch.empty((P, 3), **fopts) if lf is not None else None
        L = _lib.load()
        cur = torch.cuda.current_stream(dev)
        stream = cur.cuda_stream
        if into_leaves:
            _order_leaf_grads(dev, cur)
        if d_rgb is not None and ctx.pre_jac is not None and ctx.jac_event is not None:
            cur.wait_event(ctx.jac_event)  # the Jacobian came from the pre-pass's side stream
        with _lib.on_device(dev):
            rc = L.gsr_rasterize_gaussians_fused_backward_deferred(
                P, M, ctx.num_rendered, _ptr(bg), _ptr(m3), _ptr(radii), _ptr(dc), _ptr(rest),
                _ptr(op), _ptr(sc), _ptr(rot), float(rs.scale_modifier), _ptr(view), _ptr(proj),
                float(rs.tanfovx), float(rs.tanfovy), H, W, _ptr(dcol), _ptr(ddep), _ptr(dalp),
                _ptr(dfeat), int(rs.sh_degree), _ptr(campos), _ptr(lf), _ptr(conf),
                int(mt["include_feature"]), _ptr(geom) if geom.numel() else None,
                _ptr(binning) if binning.numel() else None, _ptr(image) if image.numel() else None,
                _ptr(d_means2D), _ptr(d_means3D), _ptr(d_dc), _ptr(d_rest), _ptr(d_op),
                _ptr(d_sc), _ptr(d_rot), _ptr(d_lf), _ptr(d_rgb),
                _ptr(ctx.pre_jac) if d_rgb is not None else None, int(accumulate), stream,
                ctx.gsr_flags)
        _lib.check(rc)
        if into_leaves:
            # one event per device, re-recorded: a later wait_event has already captured the
            # previous record (hipStreamWaitEvent waits for the record current at the call)
            prev = _LEAF_GRAD_EVENT.get(dev.index)
            ev = prev[0] if prev is not None else torch.cuda.Event()
            ev.record(cur)
            _LEAF_GRAD_EVENT[dev.index] = (ev, cur.stream_id)
        # forward inputs: means3D, means2D, features_dc, features_rest, opacity_raw, scaling_raw,
        # rotation_raw, language_feature, raster_settings
        if into_leaves:
            return None, d_means2D, None, None, None, None, None, None, None
        return d_means3D, d_means2D, d_dc, d_rest, d_op, d_sc, d_rot, d_lf, None


def rasterize_views_fused(means3D, means2D, features_dc, features_rest, opacity_raw, scaling_raw,
                          rotation_raw, language_feature, raster_settings_list, streams=None):
    """Several views of the same Gaussians in one host call (include/gsr.h
    gsr_rasterize_views_fused / _backward): per view exactly rasterize_gaussians_fused's outputs,
    stacked along a leading view axis -- color [V,3,H,W], depth [V,1,H,W], alpha [V,1,H,W],
    feature [V,3,H,W], radii [V,P] -- with means2D a [V,P,3] tensor whose gradient is every
    view's screen-space gradient.  One forward and one backward call issue all views' kernels, so
    per view the host costs a few launches instead of a Python render() + autograd node, and the
    first phases of the next views (preprocess, depth sort, read-back) are queued before a view's
    binning waits for its read-back.  streams: HIP streams the views are spread over (view v on
    streams[v % len]); default the current stream.  Every view must share the image size and the
    non-camera settings (background, scale modifier, SH degree, feature/confidence flags)."""
    return _RasterizeViewsFused.apply(means3D, means2D, features_dc, features_rest, opacity_raw,
                                      scaling_raw, rotation_raw, language_feature,
                                      tuple(raster_settings_list), tuple(streams or ()))


# test hook: extra debug bits of the multi-view backward (include/gsr_testing.h GSR_DEBUG_TEST_*)
_TEST_BWD_BITS = [0]


def _view_streams(streams):
    """The streams a multi-view forward bins its views on: the side streams (streams[1:]).  The
    backward's merged blend runs on the last of them, idle by then."""
    return tuple(streams[1:])


class _RasterizeViewsFused(torch.autograd.Function):
    @staticmethod
    def forward(ctx, means3D, means2D, features_dc, features_rest, opacity_raw, scaling_raw,
                rotation_raw, language_feature, settings, streams):
        V = len(settings)
        if V == 0:
            raise RuntimeError("rasterize_views_fused needs at least one view")
        rs0 = settings[0]
        if means3D.ndim != 2 or means3D.shape[1] != 3:
            raise RuntimeError("means3D must have dimensions (num_points, 3)")
        dev = means3D.device
        P = int(means3D.shape[0])
        H, W = int(rs0.image_height), int(rs0.image_width)
        include_feature = bool(getattr(rs0, "include_feature", False))
        for rs in settings[1:]:
            if ((int(rs.image_height), int(rs.image_width)) != (H, W)
                    or bool(getattr(rs, "include_feature", False)) != include_feature
                    or rs.bg is not rs0.bg or float(rs.scale_modifier) != float(rs0.scale_modifier)
                    or int(rs.sh_degree) != int(rs0.sh_degree)
                    or bool(rs.prefiltered) != bool(rs0.prefiltered)
                    or getattr(rs, "confidence", None) is not getattr(rs0, "confidence", None)
                    or bool(rs.debug) != bool(rs0.debug)):
                raise RuntimeError("rasterize_views_fused: views must share the image size and "
                                   "the non-camera settings")
        m3 = _dev_f32(means3D, "means3D", dev)
        dc = _dev_f32(features_dc, "features_dc", dev)
        rest = _dev_f32(_opt(features_rest), "features_rest", dev)
        op = _dev_f32(opacity_raw, "opacity", dev)
        sc = _dev_f32(scaling_raw, "scaling", dev)
        rot = _dev_f32(rotation_raw, "rotation", dev)
        lf = _dev_f32(_opt(language_feature), "language_feature", dev) if include_feature else None
        conf = _dev_f32(_opt(getattr(rs0, "confidence", None)), "confidence", dev)
        bg = _dev_f32(rs0.bg, "bg", dev)
        if dc.numel() != 3 * P or (rest is not None and rest.numel() % (3 * max(P, 1))):
            raise RuntimeError("features_dc must be [P,1,3] and features_rest [P,K,3]")
        M = 1 + (rest.numel() // (3 * P) if rest is not None and P else 0)
        degree = int(rs0.sh_degree)

        fopts = dict(dtype=torch.float32, device=dev)
        color = torch.empty((V, 3, H, W), **fopts)
        depth = torch.empty((V, 1, H, W), **fopts)
        alpha = torch.empty((V, 1, H, W), **fopts)
        feature = torch.empty((V, 3, H, W), **fopts)
        radii = torch.empty((V, P), dtype=torch.int32, device=dev)
        views = (_lib.GsrView * V)()
        holders = [_lib.BufferHolder(dev) for _ in range(V)]
        # the views' preprocess / sorts / binning on the side streams, their merged blends on the
        # call's stream (include/gsr.h); with one stream everything runs there
        vstreams = _view_streams(streams)
        cams, pres = [], []
        n_img, n_rad = 4 * H * W, 4 * P
        for v, rs in enumerate(settings):
            view = _dev_f32(rs.viewmatrix, "viewmatrix", dev)
            proj = _dev_f32(rs.projmatrix, "projmatrix", dev)
            campos = _dev_f32(rs.campos, "campos", dev)
            cams.append((view, proj, campos, float(rs.tanfovx), float(rs.tanfovy)))
            pre = _precolor_lookup(dev, campos, m3, dc, rest, degree, M)
            pres.append(pre)
            w = views[v]
            w.viewmatrix, w.projmatrix, w.campos = _ptr(view), _ptr(proj), _ptr(campos)
            w.tan_fovx, w.tan_fovy = float(rs.tanfovx), float(rs.tanfovy)
            if pre is not None:
                w.pre_color, w.pre_clamp = _ptr(pre[0]), _ptr(pre[1])
            w.out_color = color.data_ptr() + v * 3 * n_img
            w.out_depth = depth.data_ptr() + v * n_img
            w.out_alpha = alpha.data_ptr() + v * n_img
            w.out_feature = feature.data_ptr() + v * 3 * n_img
            w.radii = radii.data_ptr() + v * n_rad
            w.alloc_ctx = holders[v].key
            if vstreams:
                w.stream = vstreams[v % len(vstreams)].cuda_stream
        L = _lib.load()
        cur = torch.cuda.current_stream(dev)
        flags = _debug_flags(rs0.debug)
        t_host = time.perf_counter()
        try:
            with _lib.on_device(dev):
                rc = L.gsr_rasterize_views_fused(
                    V, views, H, W, P, M, _ptr(bg), _ptr(m3), _ptr(dc), _ptr(rest), _ptr(op),
                    _ptr(sc), _ptr(rot), float(rs0.scale_modifier), degree,
                    int(bool(rs0.prefiltered)), _ptr(lf), _ptr(conf), int(include_feature),
                    _lib.alloc_callback(), max(1, len(vstreams)), cur.cuda_stream, flags)
            _lib.check(rc)
        finally:
            for h in holders:
                h.release()
        LAST_STATS["views_fwd_host_s"] = time.perf_counter() - t_host  # host time of the call
        LAST_STATS["num_rendered"] = int(views[V - 1].num_rendered)
        LAST_STATS["num_instances"] = int(views[V - 1].num_instances)
        LAST_STATS["P"] = P
        ctx.view_counts = [(int(views[v].num_rendered), int(views[v].num_instances))
                           for v in range(V)]
        LAST_STATS["view_counts"] = list(ctx.view_counts)  # (num_rendered, num_instances) per view
        ctx.views = views
        ctx.streams = streams
        ctx.gsr_flags = flags
        ctx.cams = cams
        ctx.pre_jacs = [None if p is None else p[2] for p in pres]
        ctx.jac_event = _jac_ready(dev) if any(p is not None for p in pres) else None
        leaves = (means3D, features_dc, features_rest, opacity_raw, scaling_raw, rotation_raw,
                  language_feature)
        used = (m3, dc, rest, op, sc, rot, lf)
        ctx.leaves = None
        if grad_into_leaves() and all(
                t is None or (t.is_leaf and t.requires_grad and u is not None
                              and u.data_ptr() == t.data_ptr())
                for t, u in zip(leaves, used)):
            ctx.leaves = leaves
        ctx.meta = dict(V=V, P=P, M=M, H=H, W=W, degree=degree, include_feature=include_feature,
                        scale_modifier=float(rs0.scale_modifier),
                        shapes=(tuple(features_dc.shape),
                                None if rest is None else tuple(features_rest.shape),
                                tuple(opacity_raw.shape), tuple(scaling_raw.shape),
                                tuple(rotation_raw.shape)))
        ctx.params = (m3, dc, rest, op, sc, rot, lf, conf, bg)
        ctx.buffers = [h.bufs for h in holders]  # the views' scratch, alive until the backward
        ctx.radii = radii
        ctx.mark_non_differentiable(radii)
        ctx.set_materialize_grads(False)
        return color, depth, alpha, feature, radii

    @staticmethod
    def backward(ctx, grad_color, grad_depth, grad_alpha, grad_feature, _grad_radii):
        mt = ctx.meta
        V, P, M, H, W = mt["V"], mt["P"], mt["M"], mt["H"], mt["W"]
        m3, dc, rest, op, sc, rot, lf, conf, bg = ctx.params
        dev = m3.device
        fopts = dict(dtype=torch.float32, device=dev)

        def per_view(t, v, shape):
            if t is None:
                return None
            x = t[v]
            if x.dtype != torch.float32:
                x = x.float()
            return x if x.is_contiguous() else x.contiguous()

        keep = []  # per-view upstream-gradient tensors that must outlive the call
        zero_col = None
        views = ctx.views
        # the backward blends of all views run merged into one launch on views[0].stream
        # (include/gsr.h), beside the per-Gaussian backwards on the call's stream: the last side
        # stream
        views[0].stream = ctx.streams[-1].cuda_stream if len(ctx.streams) > 1 else None
        into_leaves = ctx.leaves is not None
        defer = _SH_DEFER.get(dev.index) if into_leaves else None
        # the SH gradients formed in this call's per-Gaussian launch (ShGradDeferral.fuse_views)
        fuse_sh = (defer is not None and defer.fuse_views and not defer.views and V <= 8
                   and all(j is not None for j in ctx.pre_jacs))
        if fuse_sh:
            defer.fused = True
            defer = None
        d_means2D = torch.empty((V, P, 3), **fopts)
        d_rgb = torch.empty((V, 3, P), **fopts) if defer is not None else None
        for v in range(V):
            w = views[v]
            gc = per_view(grad_color, v, (3, H, W))
            if gc is None:
                if zero_col is None:
                    zero_col = torch.zeros((3, H, W), **fopts)
                gc = zero_col
            gd = per_view(grad_depth, v, (1, H, W))
            ga = per_view(grad_alpha, v, (1, H, W))
            gf = per_view(grad_feature, v, (3, H, W)) if mt["include_feature"] else None
            keep += [gc, gd, ga, gf]
            w.dL_dout_color, w.dL_dout_depth = _ptr(gc), _ptr(gd)
            w.dL_dout_alpha, w.dL_dout_feature = _ptr(ga), _ptr(gf)
            w.dL_dmeans2D = d_means2D.data_ptr() + v * 12 * P
            if d_rgb is not None:
                w.dL_dcolor_sh = d_rgb.data_ptr() + v * 12 * P
                w.pre_jac = _ptr(ctx.pre_jacs[v])
            else:
                w.dL_dcolor_sh = None
                w.pre_jac = _ptr(ctx.pre_jacs[v]) if fuse_sh else None
        s_dc, s_rest, s_op, s_sc, s_rot = mt["shapes"]
        accumulate = into_leaves
        if into_leaves:
            direct = ctx.leaves
            if defer is not None:
                direct = tuple(None if k in (1, 2) else t for k, t in enumerate(ctx.leaves))
            if all(t is None or t.grad is None for t in direct):
                accumulate = False  # first views after zero_grad(set_to_none=True): store mode
                for t in direct:
                    if t is not None:
                        t.grad = torch.empty_like(t, memory_format=torch.contiguous_format)
            grads = []
            for t in direct:
                if t is not None and t.grad is None:
                    t.grad = torch.zeros_like(t, memory_format=torch.contiguous_format)
                grads.append(None if t is None else t.grad)
            if any(gr is not None and not gr.is_contiguous() for gr in grads):
                raise RuntimeError("grad-into-leaves needs contiguous .grad tensors")
            d_means3D, d_dc, d_rest, d_op, d_sc, d_rot, d_lf = grads
            if defer is not None:
                for v, (view, proj, campos, tx, ty) in enumerate(ctx.cams):
                    defer.add(ctx.leaves, d_rgb[v], campos, m3, mt["degree"], M)
        else:
            d_means3D = torch.empty((P, 3), **fopts)
            d_dc = torch.empty(s_dc, **fopts)
            d_rest = torch.empty(s_rest, **fopts) if rest is not None else None
            d_op = torch.empty(s_op, **fopts)
            d_sc = torch.empty(s_sc, **fopts)
            d_rot = torch.empty(s_rot, **fopts)
            d_lf = torch.empty((P, 3), **fopts) if lf is not None else None
        L = _lib.load()
        cur = torch.cuda.current_stream(dev)
        if into_leaves:
            _order_leaf_grads(dev, cur)
        if (d_rgb is not None or fuse_sh) and ctx.jac_event is not None:
            cur.wait_event(ctx.jac_event)  # the Jacobians came from the pre-pass's side stream
        t_host = time.perf_counter()
        args = (V, views, H, W, P, M, _ptr(bg), _ptr(m3), _ptr(dc), _ptr(rest), _ptr(op),
                _ptr(sc), _ptr(rot), mt["scale_modifier"], mt["degree"], _ptr(lf), _ptr(conf),
                int(mt["include_feature"]), _ptr(d_means3D), _ptr(d_dc), _ptr(d_rest),
                _ptr(d_op), _ptr(d_sc), _ptr(d_rot), _ptr(d_lf), int(accumulate),
                cur.cuda_stream, ctx.gsr_flags | _TEST_BWD_BITS[0])
        slices = _ROW_SLICES.get(dev.index) if into_leaves else None
        if slices is not None and not slices.active:
            slices = None  # an earlier chunk of a chunked step (ViewPipeline.run_views)
        errors = []
        with _lib.on_device(dev):
            if slices is None:
                rc = L.gsr_rasterize_views_fused_backward(*args)
            else:
                def on_rows(_ctx, a, b):  # the leaves' rows [a, b) are final once this runs
                    try:
                        slices.on_rows(a, b)
                    except Exception as exc:  # noqa: BLE001 -- re-raised after the C call
                        errors.append(exc)
                cb = _lib.ROWS_FN(on_rows)
                rc = L.gsr_rasterize_views_fused_backward_sliced(*args, slices.rows(P), cb, None)
        _lib.check(rc)
        if errors:
            raise errors[0]
        LAST_STATS["views_bwd_host_s"] = time.perf_counter() - t_host
        if into_leaves:
            prev = _LEAF_GRAD_EVENT.get(dev.index)
            ev = prev[0] if prev is not None else torch.cuda.Event()
            ev.record(cur)
            _LEAF_GRAD_EVENT[dev.index] = (ev, cur.stream_id)
        del keep  # read on the views' streams, which the call joined back into this stream
        # inputs: means3D, means2D, features_dc, features_rest, opacity_raw, scaling_raw,
        # rotation_raw, language_feature, settings, streams
        if into_leaves:
            return None, d_means2D, None, None, None, None, None, None, None, None
        return d_means3D, d_means2D, d_dc, d_rest, d_op, d_sc, d_rot, d_lf, None, None


_GRAD_INTO_LEAVES = None
_DETERMINISTIC = None


def deterministic(enable: Optional[bool] = None) -> bool:
    """Query / set the deterministic backward (default: env GSR_DETERMINISTIC=1).  The reference's
    backward adds gradients with unordered float atomics (backward.cu:523-554), so two runs differ
    in the last bits; with this on, the blend backward stores per-instance gradient rows and sums
    each Gaussian's rows in a fixed order (include/gsr.h GSR_DEBUG_DETERMINISTIC): bitwise
    reproducible gradients, at some cost in speed and binning-buffer memory.  A forward's mode is
    kept for its backward."""
    global _DETERMINISTIC
    if enable is not None:
        _DETERMINISTIC = bool(enable)
    if _DETERMINISTIC is None:
        _DETERMINISTIC = os.environ.get("GSR_DETERMINISTIC", "0") == "1"
    return _DETERMINISTIC


def _debug_flags(debug) -> int:
    """The C-ABI `debug` word: bit 0 the reference's debug flag, bit 1 deterministic backward."""
    return int(bool(debug)) | (2 if deterministic() else 0)
# device index -> ShGradDeferral collecting the views of the current multi-view step
_SH_DEFER = {}
# device index -> ShPrecolor of the current multi-view step
_PRECOLOR = {}


def _precolor_lookup(dev, campos, m3, dc, rest, degree, M):
    pc = _PRECOLOR.get(dev.index)
    if pc is None:
        return None
    return pc.lookup(campos, m3, dc, rest, degree, M)


def _jac_ready(dev):
    """The active pre-pass's Jacobian-done event (None: written on the pre-pass's own stream
    ahead of everything, nothing to wait for); a backward reading pre_jac waits for it."""
    pc = _PRECOLOR.get(dev.index)
    return None if pc is None else pc.jac_event


class ShPrecolor:
    """Multi-view colour pre-pass of one step on one device (include/gsr.h gsr_sh_precolor).
    One pass over the SH rows computes, for every camera of the step, the fused forward's colour
    and clamp bits and the backward's colour Jacobian; while installed (``with``), fused
    forwards whose camera centre (same tensor), leaves and SH degree match use them instead of
    reading the 192-byte SH rows again, and -- under ShGradDeferral -- so do their backwards.
    Outputs are identical (the same device functions, gsr_sh.h)."""

    def __init__(self, means3D, features_dc, features_rest, degree, campos_list, buffers=None,
                 rows: bool = False):
        """buffers: optional list of (colour [3,P], clamp [P] u8, Jacobian [9,P]) per camera to
        reuse (written on the current stream, so every earlier reader must be ordered before it).
        Colour and Jacobian are planar (include/gsr.h gsr_sh_precolor).

        rows: nothing is computed here; compute_rows(a, b) fills rows [a, b) (the next step's
        pre-pass issued slice by slice behind the optimizer, gsr_amd.trainer), and `complete`
        says when every row has been filled."""
        self.device = means3D.device
        self.keys = (means3D.data_ptr(), features_dc.data_ptr(),
                     features_rest.data_ptr() if features_rest is not None else 0, int(degree))
        P = int(means3D.shape[0])
        self.P = P
        self.M = 1 + (features_rest.numel() // (3 * P) if features_rest is not None and P else 0)
        fopts = dict(dtype=torch.float32, device=self.device)
        self.views = {}
        cams = [_dev_f32(c, "campos", self.device) for c in campos_list]
        if buffers is not None and len(buffers) == len(cams) and all(
                b[0].shape == (3, P) and b[2].shape == (9, P) for b in buffers):
            bufs = list(buffers)
        else:
            bufs = [(torch.empty((3, P), **fopts),
                     torch.empty((P,), dtype=torch.uint8, device=self.device),
                     torch.empty((9, P), **fopts)) for _ in cams]
        self.buffers = bufs
        self.jac_event = None
        n = len(cams)
        self._m3c = means3D.contiguous()
        self._args = None
        self._done_rows = 0
        if n and P:
            arr = lambda xs: (_lib.ctypes.c_void_p * n)(*[x.data_ptr() for x in xs])  # noqa: E731
            self._args = ((self.M, int(degree), _ptr(self._m3c), _ptr(features_dc),
                           _ptr(features_rest), n, arr(cams)),
                          (arr([b[0] for b in bufs]), arr([b[1] for b in bufs]),
                           arr([b[2] for b in bufs])))
            if not rows:
                self.compute_rows(0, P)
        for c, b in zip(cams, bufs):
            self.views[c.data_ptr()] = b
        self._campos = cams  # keep the keyed tensors alive

    @property
    def complete(self) -> bool:
        return self._args is None or self._done_rows >= self.P

    def compute_rows(self, a: int, b: int):
        """The pre-pass of rows [a, b) of every camera, on the current stream."""
        if self._args is None or b <= a:
            return
        head, outs = self._args
        with _lib.on_device(self.device):
            rc = _lib.load().gsr_sh_precolor_rows(self.P, int(a), int(min(b, self.P)), *head,
                                                  *outs, _lib.raw_stream(self.device))
        _lib.check(rc)
        self._done_rows += max(0, min(b, self.P) - a)

    def lookup(self, campos, m3, dc, rest, degree, M):
        keys = (m3.data_ptr(), dc.data_ptr(), rest.data_ptr() if rest is not None else 0,
                int(degree))
        if keys != self.keys or M != self.M:
            return None
        return self.views.get(campos.data_ptr())

    def __enter__(self):
        if self.device.index in _PRECOLOR:
            raise RuntimeError("a colour pre-pass is already active on this device")
        _PRECOLOR[self.device.index] = self
        return self

    def __exit__(self, *exc):
        _PRECOLOR.pop(self.device.index, None)
        return False


_ROW_SLICES = {}  # device index -> BackwardRowSlices


class BackwardRowSlices:
    """While installed (``with BackwardRowSlices(dev, on_rows, slices):``), a grad-into-leaves
    backward of the multi-view call (rasterize_views_fused) runs its per-Gaussian part in
    `slices` row ranges (include/gsr.h gsr_rasterize_views_fused_backward_sliced) and calls
    on_rows(a, b) as soon as rows [a, b) of every leaf gradient it writes are final on the
    current stream -- gsr_amd.pipeline starts those rows' all-reduce there, so the reduction of
    one slice overlaps the next slice's compute.  `ran` tells whether a
    backward used it."""

    def __init__(self, device, on_rows, slices: int = 4):
        self.device = torch.device(device)
        self.on_rows = on_rows
        self.slices = max(1, int(slices))
        self.ran = False
        self.active = True  # False: backwards pass it by (an earlier chunk of a chunked step)

    def rows(self, P):
        # the slices' all-reduce treats the rows as final: a second sliced backward in the same
        # scope would add gradients the other ranks never receive
        if self.ran:
            raise RuntimeError("BackwardRowSlices: a second grad-into-leaves multi-view backward in "
                               "one slicing scope; its rows were already all-reduced (issue one "
                               "multi-view backward per step, or deactivate the scope for the "
                               "earlier ones)")
        self.ran = True
        if self.slices <= 1 or P <= 256:
            return 0
        per = -(-P // self.slices)
        return -(-per // 256) * 256

    def __enter__(self):
        if self.device.index in _ROW_SLICES:
            raise RuntimeError("backward row slices are already installed on this device")
        _ROW_SLICES[self.device.index] = self
        return self

    def __exit__(self, *exc):
        _ROW_SLICES.pop(self.device.index, None)
        return False


class ShGradDeferral:
    """Deferred SH gradients of one multi-view step on one device (include/gsr.h
    gsr_rasterize_gaussians_fused_backward_deferred / gsr_sh_grad_flush).  While installed
    (``with ShGradDeferral(dev):``), grad-into-leaves backwards store each view's clamp-masked
    dL/dRGB [P,3] instead of read-modify-writing the 192-byte SH gradient rows, and flush()
    writes features_dc / features_rest .grad once: sum over the views of basis(dir_v) x dRGB_v,
    the reference's own per-view SH backward (backward.cu:20-139) summed in view order.  The
    .grad of the SH leaves is only complete after flush() (the context's exit flushes)."""

    def __init__(self, device, on_rows=None, chunk_rows: int = 0, fuse_views: bool = False):
        """on_rows(a, b): called after the flush of Gaussian rows [a, b) has been issued on the
        current stream (gsr_amd.parallel.GradAllReducer starts that slice's all-reduce there);
        chunk_rows > 0 splits the flush into row ranges of that size (multiple of 256).

        fuse_views: a multi-view backward of at most 8 views with the colour pre-pass forms the
        SH gradients in its own per-Gaussian launch instead of deferring them (include/gsr.h
        gsr_view.pre_jac: the flush fused, same values) -- for callers whose multi-view call holds
        the whole step (gsr_amd.pipeline.ViewPipeline.run_views).  `fused` then says so: those
        SH gradients are final when that backward's rows are."""
        self.device = torch.device(device)
        self.views = []
        self.leaves = None
        self.on_rows = on_rows
        self.chunk_rows = int(chunk_rows)
        self.fuse_views = bool(fuse_views)
        self.fused = False  # a multi-view backward wrote the SH gradients itself
        self.views_flushed = False  # a flush wrote SH gradients (the on_rows hooks ran)

    def __enter__(self):
        if self.device.index in _SH_DEFER:
            raise RuntimeError("an SH-gradient deferral is already active on this device")
        _SH_DEFER[self.device.index] = self
        return self

    def __exit__(self, *exc):
        _SH_DEFER.pop(self.device.index, None)
        if exc[0] is None:
            self.flush()
        self.views = []
        return False

    def add(self, leaves, d_rgb, campos, means3D, degree, M):
        if self.leaves is not None and any(a is not b for a, b in zip(self.leaves, leaves)):
            raise RuntimeError("deferred SH gradients: views of one step must share the leaves")
        if self.views and (self.views[0][3], self.views[0][4]) != (degree, M):
            raise RuntimeError("deferred SH gradients: views of one step must share the SH degree")
        self.leaves = leaves
        self.views.append((d_rgb, campos, torch.cuda.current_stream(self.device), degree, M,
                           means3D))

    def flush(self):
        """Write the SH leaves' .grad for the collected views on the current stream (which must
        be ordered after every view's backward, e.g. joined by ViewPipeline.run)."""
        if not self.views:
            return
        self.views_flushed = True
        _, dc, rest = self.leaves[0], self.leaves[1], self.leaves[2]
        d_rgb0, _, _, degree, M, m3 = self.views[0]
        P = int(m3.shape[0])
        cur = torch.cuda.current_stream(self.device)
        # one flag for both planes: add when either already holds a gradient (a missing one is
        # then created as zeros), store when neither does
        accumulate = any(t is not None and t.grad is not None for t in (dc, rest))
        for t in (dc, rest):
            if t is not None and t.grad is None:
                t.grad = (torch.zeros_like if accumulate else torch.empty_like)(
                    t, memory_format=torch.contiguous_format)
        n = len(self.views)
        camp = (_lib.ctypes.c_void_p * n)(*[v[1].data_ptr() for v in self.views])
        step = P if self.chunk_rows <= 0 else max(256, (self.chunk_rows // 256) * 256)
        rest_w = 3 * (M - 1)
        L = _lib.load()
        for a in range(0, P, step):  # row slices: the kernel is per Gaussian, pointers offset
            b = min(P, a + step)
            # planar [3][P] dL/dRGB: rows [a, b) start at element a of each plane
            rgbs = (_lib.ctypes.c_void_p * n)(*[v[0].data_ptr() + 4 * a for v in self.views])
            with _lib.on_device(self.device):
                rc = L.gsr_sh_grad_flush(b - a, M, degree, _ptr(m3) + 12 * a, n, camp, rgbs, P,
                                         _ptr(dc.grad) + 12 * a,
                                         (_ptr(rest.grad) + 4 * rest_w * a)
                                         if rest is not None else None,
                                         int(accumulate), cur.cuda_stream)
            _lib.check(rc)
            if self.on_rows is not None:
                self.on_rows(a, b)
        for v in self.views:  # buffers made on the views' streams, read here on this one
            v[0].record_stream(cur)
            v[1].record_stream(cur)
        self.views = []
# device index -> (event after the last grad-into-leaves backward, id of the stream it ran on)
_LEAF_GRAD_EVENT = {}


def _order_leaf_grads(dev, stream):
    """grad-into-leaves backwards read-modify-write the leaves' .grad without atomics, so two
    of them issued on different streams (gsr_amd.pipeline.ViewPipeline) must not overlap: the
    stream of this backward waits for the previous one when that ran on another stream."""
    prev = _LEAF_GRAD_EVENT.get(dev.index)
    if prev is not None and prev[1] != stream.stream_id:
        stream.wait_event(prev[0])


def grad_into_leaves(enable: Optional[bool] = None) -> bool:
    """Query / set the fused path's grad-into-leaves mode (default: env GSR_GRAD_INTO_LEAVES=1).

    When on, and the fused entry point receives the model's leaf tensors themselves, the backward
    kernel adds the raw-parameter gradients of the visible Gaussians straight into each leaf's
    .grad (include/gsr.h accumulate = 1) and returns None for them, instead of materialising
    fresh [P,...] gradients that autograd then adds view by view.  loss.backward() +
    optimizer.step() see identical .grad values; torch.autograd.grad() on those leaves and
    per-leaf grad hooks do not (they are bypassed), hence opt-in."""
    global _GRAD_INTO_LEAVES
    if enable is not None:
        _GRAD_INTO_LEAVES = bool(enable)
    if _GRAD_INTO_LEAVES is None:
        _GRAD_INTO_LEAVES = os.environ.get("GSR_GRAD_INTO_LEAVES", "0") == "1"
    return _GRAD_INTO_LEAVES


class GaussianRasterizationSettings(NamedTuple):
    # vendored fields (diff_gaussian_rasterization/__init__.py:157-169)
    image_height: int
    image_width: int
    tanfovx: float
    tanfovy: float
    bg: torch.Tensor
    scale_modifier: float
    viewmatrix: torch.Tensor
    projmatrix: torch.Tensor
    sh_degree: int
    campos: torch.Tensor
    prefiltered: bool
    debug: bool = False
    # extended fields used by gaussian_renderer/__init__.py:241-242
    include_feature: bool = False
    confidence: Optional[torch.Tensor] = None


class GaussianRasterizer(nn.Module):
    def __init__(self, raster_settings):
        super().__init__()
        self.raster_settings = raster_settings

    def markVisible(self, positions):
        # diff_gaussian_rasterization/__init__.py:176-185
        with torch.no_grad():
            rs = self.raster_settings
            return mark_visible(positions, rs.viewmatrix, rs.projmatrix)

    def forward(self, means3D, means2D, opacities, shs=None, colors_precomp=None, scales=None,
                rotations=None, cov3D_precomp=None, shs_language=None,
                language_feature_precomp=None):
        rs = self.raster_settings
        # argument checks of diff_gaussian_rasterization/__init__.py:191-195
        if (shs is None and colors_precomp is None) or (shs is not None and colors_precomp is not None):
            raise Exception('Please provide excatly one of either SHs or precomputed colors!')
        if ((scales is None or rotations is None) and cov3D_precomp is None) or \
                ((scales is not None or rotations is not None) and cov3D_precomp is not None):
            raise Exception('Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!')
        return rasterize_gaussians_extended(means3D, means2D, shs, shs_language, colors_precomp,
                                            language_feature_precomp, opacities, scales, rotations,
                                            cov3D_precomp, rs)


def check_forwards(wait: bool = True):
    """Raise if a forward since the last check failed (a one-sweep sort gave up its bounded
    look-back, or an out-of-range id had to be clamped).  Such a call's outputs and gradients are
    NaN on the device and its backward raises once the failure is published; this check is the
    blocking form (wait=True) for the end of a training step (include/gsr.h gsr_check_forwards)."""
    _lib.check_forwards(wait)


def mark_visible(positions, viewmatrix, projmatrix):
    """_C.mark_visible (rasterize_points.cu:198-217): bool[P], view-space z > 0.2."""
    dev = positions.device
    m3 = _dev_f32(positions, "positions", dev)
    view = _dev_f32(viewmatrix, "viewmatrix", dev)
    proj = _dev_f32(projmatrix, "projmatrix", dev)
    P = int(m3.shape[0])
    present = torch.zeros((P,), dtype=torch.bool, device=dev)
    if P:
        with _lib.on_device(dev):
            _lib.check(_lib.load().gsr_mark_visible(P, _ptr(m3), _ptr(view), _ptr(proj),
                                                   _ptr(present),
                                                   _lib.raw_stream(dev)))
    return present
