"""Training losses on libgsr (include/gsr_loss.h).

Mirrors the loss calls of train.py around the rasterizer:
  photometric_loss(image, gt, lambda_dssim) -> (loss, Ll1)
        = ((1 - lambda) * l1_loss(image, gt) + lambda * (1 - ssim(image, gt)), l1_loss(image, gt))
        (train.py:99-100; utils/loss_utils.py:106-162) as ONE forward and ONE backward kernel
  ssim(img1, img2, mask=None, window_size=11, size_average=True)     (loss_utils.py:129-162)
  pearson_corrcoef(preds, target)                (torchmetrics.functional, train.py:22,126-149)
  depth_pearson_loss(depth_mono, depth, offset=200.0)
        = min(1 - pearson(depth_mono, depth), 1 - pearson(1 / (-depth_mono + offset), depth))
        (train.py:126-129) without the host sync of Python's min() on tensors
  train_view_loss(image, depth, gt, depth_mono, lambda_dssim, depth_weight)
        = photometric_loss + depth_weight * depth_pearson_loss as one autograd node with pooled
        scratch (the per-view loss of train.py:99-131; what gsr_amd.trainer uses)
Gradients flow to the rendered image / depth (the first argument of ssim, either argument of
pearson_corrcoef, `depth` of depth_pearson_loss).  No CPU path.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib


def _stream(t):
    return _lib.raw_stream(t.device)


def _check(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what} failed with status {rc}")


def _cuda(*ts):
    for t in ts:
        if not t.is_cuda:
            raise RuntimeError("gsr losses run on HIP tensors only (no CPU path)")


def _ptr(t):
    return None if t is None else t.data_ptr()


class _Photometric(torch.autograd.Function):
    """out[3] = (loss, l1 mean, ssim mean) of image vs gt, [C,H,W]."""

    @staticmethod
    def forward(ctx, image, gt, lambda_dssim):
        _cuda(image, gt)
        if image.shape != gt.shape or image.dim() != 3:
            raise ValueError("photometric loss expects image and gt of the same [C,H,W] shape")
        if gt.requires_grad:
            raise ValueError("gradients flow to the rendered image only (gt must not require grad)")
        x = image.detach().contiguous().float()
        y = gt.detach().contiguous().float()
        C, H, W = x.shape
        L = _lib.load()
        scratch = torch.empty(int(L.gsr_photometric_scratch_bytes(C, H, W)), dtype=torch.uint8,
                              device=x.device)
        out = torch.empty(3, dtype=torch.float32, device=x.device)
        need = int(image.requires_grad)
        with _lib.on_device(x.device):
            _check(L.gsr_photometric_loss(C, H, W, x.data_ptr(), y.data_ptr(),
                                          float(lambda_dssim), need, out.data_ptr(),
                                          scratch.data_ptr(), _stream(x)), "gsr_photometric_loss")
        ctx.save_for_backward(x, y)
        ctx.scratch = scratch
        ctx.lam = float(lambda_dssim)
        return out

    @staticmethod
    def backward(ctx, g):
        x, y = ctx.saved_tensors
        C, H, W = x.shape
        g = g.contiguous()
        dx = torch.empty_like(x)
        with _lib.on_device(x.device):
            _check(_lib.load().gsr_photometric_loss_backward(
                C, H, W, x.data_ptr(), y.data_ptr(), ctx.lam, g.data_ptr(), g.data_ptr() + 4,
                g.data_ptr() + 8, dx.data_ptr(), ctx.scratch.data_ptr(), _stream(x)),
                "gsr_photometric_loss_backward")
        return dx, None, None


def photometric_loss(image, gt, lambda_dssim=0.2):
    """(loss, Ll1) of train.py:99-100 in one pass (lambda_dssim: arguments/__init__.py:87)."""
    out = _Photometric.apply(image, gt, lambda_dssim)
    return out[0], out[1]


def ssim(img1, img2, mask=None, window_size=11, size_average=True):
    """utils/loss_utils.py:129-162 (11x11 window only; gradient to img1)."""
    if window_size != 11:
        raise ValueError("gsr ssim implements the reference's window_size=11")
    if mask is not None:
        img1 = img1 * mask + (1 - mask)
        img2 = img2 * mask + (1 - mask)
    if img1.dim() == 3:
        if not size_average:
            raise ValueError("size_average=False needs batched [B,C,H,W] input (as the reference)")
        return _Photometric.apply(img1, img2, 0.0)[2]
    maps = [_Photometric.apply(a, b, 0.0)[2] for a, b in zip(img1, img2)]
    per_image = torch.stack(maps)
    return per_image.mean() if size_average else per_image


class _Pearson(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, y, variants, offset):
        _cuda(x, y)
        if x.shape != y.shape or x.dim() not in (1, 2):
            raise ValueError("pearson expects preds and target of the same [N] or [N, K] shape")
        xs = x.detach().reshape(x.shape[0], -1).contiguous().float()
        ys = y.detach().reshape(y.shape[0], -1).contiguous().float()
        N, K = xs.shape
        L = _lib.load()
        scratch = torch.empty(int(L.gsr_pearson_scratch_bytes(K, variants)), dtype=torch.uint8,
                              device=xs.device)
        r = torch.empty(variants * K, dtype=torch.float32, device=xs.device)
        loss = torch.empty(K, dtype=torch.float32, device=xs.device)
        with _lib.on_device(xs.device):
            _check(L.gsr_pearson_loss(N, K, xs.data_ptr(), ys.data_ptr(), variants, float(offset),
                                      r.data_ptr(), loss.data_ptr(), scratch.data_ptr(),
                                      _stream(xs)), "gsr_pearson_loss")
        ctx.save_for_backward(xs, ys)
        ctx.scratch, ctx.variants, ctx.offset, ctx.shape = scratch, variants, offset, x.shape
        return loss, r

    @staticmethod
    def backward(ctx, g_loss, g_r):
        xs, ys = ctx.saved_tensors
        N, K = xs.shape
        need_x, need_y = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        # r-output grads are folded in as -g (loss = 1 - r) for the single-variant form
        g = -g_r[:K] if ctx.variants == 1 else torch.zeros(K, device=xs.device)
        if g_loss is not None:
            g = g + g_loss
        g = g.contiguous().float()
        dx = torch.empty_like(xs) if need_x else None
        dy = torch.empty_like(ys) if need_y else None
        if need_x and ctx.variants != 1:
            raise ValueError("depth_pearson_loss: gradients flow to the rendered depth only")
        with _lib.on_device(xs.device):
            _check(_lib.load().gsr_pearson_loss_backward(
                N, K, xs.data_ptr(), ys.data_ptr(), ctx.variants, float(ctx.offset), g.data_ptr(),
                _ptr(dy), _ptr(dx), ctx.scratch.data_ptr(), _stream(xs)),
                "gsr_pearson_loss_backward")
        return (None if dx is None else dx.reshape(ctx.shape),
                None if dy is None else dy.reshape(ctx.shape), None, None)


def pearson_corrcoef(preds, target):
    """torchmetrics.functional.pearson_corrcoef: r per column, squeezed ([N] -> scalar)."""
    _, r = _Pearson.apply(preds, target, 1, 0.0)
    return r.squeeze()


def depth_pearson_loss(depth_mono, depth, offset=200.0):
    """train.py:126-129: min(1 - r(mono, depth), 1 - r(1 / (-mono + offset), depth)); gradient to
    depth (either [H,W]-like tensor, flattened to a column as the reference's reshape(-1, 1))."""
    loss, _ = _Pearson.apply(depth_mono.reshape(-1, 1), depth.reshape(-1, 1), 2, offset)
    return loss.squeeze()


# ---- one autograd node for train.py's per-view loss ----------------------------------------------
# Scratch buffers keyed by (kind, shape, device, stream): a buffer is taken by a forward and given
# back once its backward has been issued (or at once without autograd), so the next forward on the
# same stream -- ordered after that backward -- reuses it; another stream gets its own.
_POOL = {}


def _take(key, nbytes, device):
    free = _POOL.setdefault(key, [])
    return free.pop() if free else torch.empty(nbytes, dtype=torch.uint8, device=device)


def _give(key, buf):
    _POOL.setdefault(key, []).append(buf)


class _TrainViewLoss(torch.autograd.Function):
    """loss = (1 - lambda) L1 + lambda (1 - SSIM) of (image, gt) + depth_weight * the Pearson depth
    term of (depth_mono, depth) (train.py:99-100,117-131), as ONE autograd node over
    gsr_view_loss: the forward is two launches (SSIM tiles + Pearson partial sums in one grid,
    then one reduction writing every output and the total), the backward one; no intermediate
    autograd nodes, torch ops or allocations on the steady state."""

    @staticmethod
    def forward(ctx, image, depth, gt, depth_mono, lambda_dssim, depth_weight, offset):
        _cuda(image, depth, gt, depth_mono)
        if image.shape != gt.shape or image.dim() != 3:
            raise ValueError("photometric loss expects image and gt of the same [C,H,W] shape")
        if depth.numel() != depth_mono.numel():
            raise ValueError("depth and depth_mono must have the same number of pixels")
        x = image.detach().contiguous().float()
        y = gt.detach().contiguous().float()
        d = depth.detach().reshape(-1).contiguous().float()
        m = depth_mono.detach().reshape(-1).contiguous().float()
        C, H, W = x.shape
        N = d.numel()
        L = _lib.load()
        dev = x.device
        s = _stream(x)
        kv = ("view", C, H, W, dev.index, s)
        sv = _take(kv, int(L.gsr_view_loss_scratch_bytes(C, H, W)), dev)
        out = torch.empty(5, dtype=torch.float32, device=dev)  # loss, l1, ssim, depth term, total
        total = torch.empty((), dtype=torch.float32, device=dev)
        need = int(image.requires_grad or depth.requires_grad)
        with _lib.on_device(dev):
            _check(L.gsr_view_loss(C, H, W, x.data_ptr(), y.data_ptr(), float(lambda_dssim), N,
                                   d.data_ptr(), m.data_ptr(), float(offset), float(depth_weight),
                                   need, out.data_ptr(), total.data_ptr(), sv.data_ptr(), s),
                   "gsr_view_loss")
        if need:
            ctx.save_for_backward(x, y, d, m)
            ctx.bufs = (kv, sv)
            ctx.args = (float(lambda_dssim), float(depth_weight), float(offset))
            ctx.dshape = depth.shape
        else:
            _give(kv, sv)
        ctx.mark_non_differentiable(out)
        ctx.set_materialize_grads(False)  # `out` never gets a gradient: no zero-filled tensor
        return total, out

    @staticmethod
    def backward(ctx, g_total, g_out):
        x, y, d, m = ctx.saved_tensors
        kv, sv = ctx.bufs
        lam, w, offset = ctx.args
        C, H, W = x.shape
        if g_total is None:
            _give(kv, sv)
            return None, None, None, None, None, None, None
        L = _lib.load()
        g = g_total.reshape(1).contiguous().float()
        dx = torch.empty_like(x)
        dd = torch.empty_like(d)
        s = _stream(x)
        with _lib.on_device(x.device):
            _check(L.gsr_view_loss_backward(C, H, W, x.data_ptr(), y.data_ptr(), lam, d.numel(),
                                            d.data_ptr(), m.data_ptr(), offset, w, g.data_ptr(),
                                            dx.data_ptr(), dd.data_ptr(), sv.data_ptr(), s),
                   "gsr_view_loss_backward")
        _give(kv, sv)
        return (dx if ctx.needs_input_grad[0] else None,
                dd.view(ctx.dshape) if ctx.needs_input_grad[1] else None,
                None, None, None, None, None)


class _TrainViewsLoss(torch.autograd.Function):
    """train_view_loss for the V views of a multi-view step as ONE autograd node over
    gsr_view_loss_views: images [V,C,H,W] and depths [V,...] are the multi-view call's stacked
    outputs, so the gradient reaches them as [V,...] tensors directly (no per-view slices to
    stack); per view the values are gsr_view_loss's, bit for bit."""

    @staticmethod
    def forward(ctx, images, depths, gts, monos, lambda_dssim, depth_weight, offset):
        _cuda(images, depths, *gts, *monos)
        V = int(images.shape[0])
        if images.dim() != 4 or len(gts) != V or len(monos) != V or depths.shape[0] != V:
            raise ValueError("train_views_loss expects images [V,C,H,W], depths [V,...] and V "
                             "ground truths / monocular depths")
        x = images.detach().contiguous().float()
        d = depths.detach().reshape(V, -1).contiguous().float()
        C, H, W = (int(n) for n in x.shape[1:])
        N = int(d.shape[1])
        ys = [g.detach().contiguous().float() for g in gts]
        ms = [m.detach().reshape(-1).contiguous().float() for m in monos]
        for y, m in zip(ys, ms):
            if tuple(y.shape) != (C, H, W) or m.numel() != N:
                raise ValueError("every gt must be [C,H,W] and every depth_mono N pixels")
        L = _lib.load()
        dev = x.device
        s = _stream(x)
        kv = ("views", V, C, H, W, dev.index, s)
        sv = _take(kv, V * int(L.gsr_view_loss_scratch_bytes(C, H, W)), dev)
        out = torch.empty((V, 5), dtype=torch.float32, device=dev)
        total = torch.empty(V, dtype=torch.float32, device=dev)
        need = int(images.requires_grad or depths.requires_grad)
        gp = (ctypes.c_void_p * V)(*[y.data_ptr() for y in ys])
        mp = (ctypes.c_void_p * V)(*[m.data_ptr() for m in ms])
        with _lib.on_device(dev):
            _check(L.gsr_view_loss_views(V, C, H, W, x.data_ptr(), gp, float(lambda_dssim), N,
                                         d.data_ptr(), mp, float(offset), float(depth_weight),
                                         need, out.data_ptr(), total.data_ptr(), sv.data_ptr(), s),
                   "gsr_view_loss_views")
        if need:
            ctx.save_for_backward(x, d, *ys, *ms)
            ctx.V = V
            ctx.bufs = (kv, sv)
            ctx.args = (float(lambda_dssim), float(depth_weight), float(offset))
            ctx.dshape = depths.shape
        else:
            _give(kv, sv)
        ctx.mark_non_differentiable(out)
        ctx.set_materialize_grads(False)
        return total, out

    @staticmethod
    def backward(ctx, g_total, g_out):
        saved = ctx.saved_tensors
        V = ctx.V
        x, d, ys, ms = saved[0], saved[1], saved[2:2 + V], saved[2 + V:]
        kv, sv = ctx.bufs
        lam, w, offset = ctx.args
        C, H, W = (int(n) for n in x.shape[1:])
        if g_total is None:
            _give(kv, sv)
            return None, None, None, None, None, None, None
        L = _lib.load()
        g = g_total.reshape(V).contiguous().float()
        dx = torch.empty_like(x)
        dd = torch.empty_like(d)
        gp = (ctypes.c_void_p * V)(*[y.data_ptr() for y in ys])
        mp = (ctypes.c_void_p * V)(*[m.data_ptr() for m in ms])
        with _lib.on_device(x.device):
            _check(L.gsr_view_loss_views_backward(V, C, H, W, x.data_ptr(), gp, lam,
                                                  int(d.shape[1]), d.data_ptr(), mp, offset, w,
                                                  g.data_ptr(), dx.data_ptr(), dd.data_ptr(),
                                                  sv.data_ptr(), _stream(x)),
                   "gsr_view_loss_views_backward")
        _give(kv, sv)
        return (dx if ctx.needs_input_grad[0] else None,
                dd.view(ctx.dshape) if ctx.needs_input_grad[1] else None,
                None, None, None, None, None)


def train_views_loss(images, depths, gt_images, depth_monos, lambda_dssim=0.2, depth_weight=0.05,
                     offset=200.0):
    """train_view_loss of V views at once (at most 8): images [V,C,H,W], depths [V,...] (e.g.
    gaussian_renderer.render_views' stacked outputs), sequences of V ground truths and monocular
    depths.  Returns (the V totals [V], the outputs [V,5]: photometric, L1, SSIM, depth term,
    total); every view's values equal train_view_loss's."""
    return _TrainViewsLoss.apply(images, depths, tuple(gt_images), tuple(depth_monos),
                                 lambda_dssim, depth_weight, offset)


def train_view_loss(image, depth, gt_image, depth_mono, lambda_dssim=0.2, depth_weight=0.05,
                    offset=200.0):
    """train.py:99-131 for one view with the depth branch: (total loss, Ll1).  Gradients flow to
    the rendered image and depth."""
    total, out = _TrainViewLoss.apply(image, depth, gt_image, depth_mono, lambda_dssim,
                                      depth_weight, offset)
    return total, out[1]
