"""`_C`-compatible shim over libgsr.so: the three functions the reference's pybind11 module
exports (submodules/diff-gaussian-rasterization/ext.cpp:15-19) with their exact argument lists and
return tuples (rasterize_points.cu:35-55/114, 117-140/195, 198-217).

A maintainer who keeps the reference's own vendored wrapper (diff_gaussian_rasterization/
__init__.py) only has to change its `from . import _C` line to import this module.  Empty tensors
(torch.Tensor([])) mean "absent", exactly as in the reference.
"""
from __future__ import annotations

import ctypes

import torch

from gsr_amd import _lib


def _opt(t):
    return None if t is None or t.numel() == 0 else t


def _f32(t, dev):
    if t is None:
        return None
    if not t.is_cuda:
        raise RuntimeError("libgsr has no CPU path: tensors must live on the HIP device")
    return t.to(device=dev, dtype=torch.float32).contiguous()


def _p(t):
    return None if t is None else t.data_ptr()


def _forward_flags(debug):
    from . import _debug_flags
    return _debug_flags(debug)


def rasterize_gaussians(background, means3D, colors, opacity, scales, rotations, scale_modifier,
                        cov3D_precomp, viewmatrix, projmatrix, tan_fovx, tan_fovy, image_height,
                        image_width, sh, degree, campos, prefiltered, debug):
    if means3D.ndimension() != 2 or means3D.size(1) != 3:
        raise RuntimeError("means3D must have dimensions (num_points, 3)")
    dev = means3D.device
    P, H, W = int(means3D.size(0)), int(image_height), int(image_width)
    m3 = _f32(means3D, dev)
    shs = _f32(_opt(sh), dev)
    M = int(shs.size(1)) if shs is not None else 0
    out_color = torch.zeros((3, H, W), dtype=torch.float32, device=dev)
    radii = torch.zeros((P,), dtype=torch.int32, device=dev)
    holder = _lib.BufferHolder(dev)
    nr = ctypes.c_int(0)
    keep = [_f32(x, dev) for x in (background, _opt(colors), opacity, _opt(scales),
                                   _opt(rotations), _opt(cov3D_precomp), viewmatrix, projmatrix,
                                   campos)]
    bg, col, op, sc, rot, cov, view, proj, cp = keep
    flags = _forward_flags(debug)
    try:
        with torch.cuda.device(dev):
            rc = _lib.load().gsr_rasterize_gaussians(
                P, M, _p(bg), _p(m3), _p(col), _p(op), _p(sc), _p(rot), float(scale_modifier),
                _p(cov), _p(view), _p(proj), float(tan_fovx), float(tan_fovy), H, W, _p(shs),
                int(degree), _p(cp), int(bool(prefiltered)), None, None, None, 0, _p(out_color),
                None, None, None, _p(radii), ctypes.byref(nr), _lib.alloc_callback(), holder.key,
                torch.cuda.current_stream(dev).cuda_stream, flags)
        _lib.check(rc)
    finally:
        holder.release()
    empty = torch.empty((0,), dtype=torch.uint8, device=dev)
    geom, binning, img = (b if b is not None else empty for b in holder.bufs)
    return int(nr.value), out_color, radii, geom, binning, img


def rasterize_gaussians_backward(background, means3D, radii, colors, scales, rotations,
                                 scale_modifier, cov3D_precomp, viewmatrix, projmatrix, tan_fovx,
                                 tan_fovy, dL_dout_color, sh, degree, campos, geomBuffer, R,
                                 binningBuffer, imageBuffer, debug):
    dev = means3D.device
    P = int(means3D.size(0))
    H, W = int(dL_dout_color.size(1)), int(dL_dout_color.size(2))
    shs = _f32(_opt(sh), dev)
    M = int(shs.size(1)) if shs is not None else 0
    o = dict(dtype=torch.float32, device=dev)
    # rasterize_points.cu:151-159 (every buffer returned; libgsr writes all of them)
    d_means3D = torch.empty((P, 3), **o)
    d_means2D = torch.empty((P, 3), **o)
    d_colors = torch.empty((P, 3), **o)
    d_opacity = torch.empty((P, 1), **o)
    d_cov3D = torch.empty((P, 6), **o)
    d_sh = torch.zeros((P, M, 3), **o)
    d_scales = torch.zeros((P, 3), **o)
    d_rot = torch.zeros((P, 4), **o)
    m3 = _f32(means3D, dev)
    bg, col, sc, rot, cov, view, proj, cp, dpix = (
        _f32(x, dev) for x in (background, _opt(colors), _opt(scales), _opt(rotations),
                               _opt(cov3D_precomp), viewmatrix, projmatrix, campos, dL_dout_color))
    rad = radii.to(dev, torch.int32).contiguous() if radii is not None and radii.numel() else None
    g = geomBuffer if geomBuffer.numel() else None
    b = binningBuffer if binningBuffer.numel() else None
    i = imageBuffer if imageBuffer.numel() else None
    # The forward's layout: the buffer's size tells it when only the default layout fits (no
    # device read); a buffer large enough for the deterministic layout too is tagged by its
    # forward (include/gsr.h GSR_DEBUG_LAYOUT_FROM_BUFFER: one 4-byte read).  A buffer too small
    # for R instances (R larger than its forward's num_rendered) raises instead of letting the
    # kernels read past it.
    flags = int(bool(debug))
    if int(R) > 0:
        L = _lib.load()
        need, need_det = int(L.gsr_binning_buffer_bytes(int(R))), int(L.gsr_binning_buffer_bytes_det(int(R)))
        have = 0 if b is None else b.numel() * b.element_size()
        if have < need:
            raise RuntimeError(f"binningBuffer holds {have} bytes, {need} needed for R = {int(R)} "
                               "instances: not the buffer of a forward with this num_rendered")
        if have >= need_det:
            flags |= 4
    with torch.cuda.device(dev):
        rc = _lib.load().gsr_rasterize_gaussians_backward(
            P, M, int(R), _p(bg), _p(m3), _p(rad), _p(col), _p(sc), _p(rot), float(scale_modifier),
            _p(cov), _p(view), _p(proj), float(tan_fovx), float(tan_fovy), H, W, _p(dpix), None,
            None, None, _p(shs), int(degree), _p(cp), None, None, None, 0, _p(g), _p(b), _p(i),
            _p(d_means2D), _p(d_colors), _p(d_opacity), _p(d_means3D), _p(d_cov3D),
            _p(d_sh) if shs is not None else None, _p(d_scales) if sc is not None else None,
            _p(d_rot) if sc is not None else None, None, None,
            torch.cuda.current_stream(dev).cuda_stream, flags)
    _lib.check(rc)
    return d_means2D, d_colors, d_opacity, d_means3D, d_cov3D, d_sh, d_scales, d_rot


def mark_visible(means3D, viewmatrix, projmatrix):
    from . import mark_visible as _mv
    return _mv(means3D, viewmatrix, projmatrix)
