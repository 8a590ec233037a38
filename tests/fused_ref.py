"""The benchmarked render path and its CPU-oracle counterpart (shared by tests/test_fused_parity.py
and __graft_entry__.smoke()).

bench.py times render() (sdp-gs_amd/gaussian_renderer, the counterpart of
gaussian_renderer/__init__.py:209-338) with the reference's default pipeline flags
(arguments/__init__.py:66-72).  That takes the fused entry point -- GaussianModel's cat / sigmoid /
exp / normalize (scene/gaussian_model.py:33-41,146-183) evaluated inside the kernels -- with the
multi-view colour pre-pass (ShPrecolor), deferred SH gradients (ShGradDeferral), gradients added
straight into the leaves' .grad, and the views spread over HIP streams (gsr_amd.pipeline.
ViewPipeline).  `run_bench_path` runs exactly that; `run_oracle_path` restates it on the CPU:

* oracle inputs: the activated parameters the kernels evaluate (gsr_test_activations runs the
  kernels' own sigmoid / exp / normalize; they are pinned bit for bit to torch's getters by
  test_fused_activations_equal_torch), SH = cat(features_dc, features_rest), language feature =
  _language_feature (the oracle's in-kernel SH / language paths, forward.cu:20-71);
* raw-leaf gradients: the oracle's gradients of the activated inputs chained through the
  activations in float64 and summed over the views in float64 (sigmoid: y (1 - y); exp: y;
  F.normalize: (g - q^ (q^ . g)) / |q|; cat: split).
"""
from __future__ import annotations

import json
import math
import os

import numpy as np
import torch

from oracle.oracle import OracleRaster

LEAVES = ("_xyz", "_features_dc", "_features_rest", "_opacity", "_scaling", "_rotation",
          "_language_feature")
IMAGES = ("render", "depth", "alpha", "feature")


class Pipe:  # arguments/__init__.py:66-72 (the reference's defaults)
    convert_SHs_python = True
    compute_cov3D_python = False
    debug = False
    use_confidence = False


class Opt:
    include_feature = True


def kernel_activations(m):
    """(opacity [P], scaling [P,3], rotation [P,4]) exactly as the fused kernels evaluate them."""
    from gsr_amd import _lib
    L = _lib.load()
    P = int(m._xyz.shape[0])
    op = torch.empty(P, device=m._xyz.device)
    sc = torch.empty((P, 3), device=m._xyz.device)
    rot = torch.empty((P, 4), device=m._xyz.device)
    _lib.check(L.gsr_test_activations(m._opacity.data_ptr(), m._scaling.data_ptr(),
                                      m._rotation.data_ptr(), P, op.data_ptr(), sc.data_ptr(),
                                      rot.data_ptr(), torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    return op, sc, rot


def run_bench_path(m, cams, grads, streams=3, defer_sh=True, precolor=True, lag=1, multi=False,
                   capture=None):
    """bench.py's step on `cams`: render + backward of the fixed upstream grads (image, depth,
    feature), grad-into-leaves, views over `streams` HIP streams.  multi: every view in one
    multi-view call (gaussian_renderer.render_views, ViewPipeline.run_views -- bench.py's default
    issue); else per view render() with view i's backward issued after view i + lag's forward
    (bench.py --per-view --lag, default 1; 0 = together).  Returns (per-view numpy dicts of the
    images, radii and screen-space gradient, leaf grads float64).  capture (multi only): called
    with the render_views packages after the forward, before the backward."""
    import diff_gaussian_rasterization as dgr
    from gaussian_renderer import render, render_views
    from gsr_amd.pipeline import ViewPipeline
    bg = torch.zeros(3, device=m._xyz.device)
    prev = dgr.grad_into_leaves()
    dgr.grad_into_leaves(True)
    try:
        for n in LEAVES:
            getattr(m, n).grad = None
        vp = ViewPipeline(m._xyz.device, depth=streams, defer_sh=defer_sh, precolor=precolor)

        def fwd(cam):
            return render(cam, m, Pipe(), bg, Opt())

        def bwd(pkg):
            torch.autograd.backward([pkg["render"], pkg["depth"], pkg["feature"]], list(grads))
            out = {k: pkg[k].detach().clone() for k in IMAGES + ("radii",)}
            out["means2D"] = pkg["viewspace_points"].grad.detach().clone()
            return out

        def all_views(cs, strs):
            pkgs = render_views(cs, m, Pipe(), bg, Opt(), streams=strs)
            if capture is not None:
                capture(pkgs)
            st = pkgs[0]["views"]
            V = len(pkgs)
            torch.autograd.backward([st["render"], st["depth"], st["feature"]],
                                    [g.expand(V, *g.shape) for g in grads])
            outs = []
            for pkg in pkgs:
                out = {k: pkg[k].detach().clone() for k in IMAGES + ("radii",)}
                out["means2D"] = pkg["viewspace_points"].grad.detach().clone()
                outs.append(out)
            return outs

        if multi:
            outs = vp.run_views(cams, all_views, model=m)
        elif lag > 0:
            outs = vp.run(cams, fwd, model=m, bwd=bwd, lag=lag)
        else:
            outs = vp.run(cams, lambda cam: bwd(fwd(cam)), model=m)
        torch.cuda.synchronize()
    finally:
        dgr.grad_into_leaves(prev)
    views = [{k: v.cpu().numpy() for k, v in o.items()} for o in outs]
    leaf_grads = {n: (getattr(m, n).grad.detach().cpu().numpy().astype(np.float64)
                      if getattr(m, n).grad is not None else
                      np.zeros(tuple(getattr(m, n).shape)))  # P == 0: no gradient written
                  for n in LEAVES}
    return views, leaf_grads


def run_oracle_path(m, cams, grads, act, progress=None):
    """The CPU oracle on the same views: per-view images / radii / screen-space gradients and the
    raw-leaf gradients (float64, summed over the views)."""
    op, sc, rot = (t.detach().cpu().numpy() for t in act)
    xyz = m._xyz.detach().cpu().numpy()
    shs = torch.cat((m._features_dc, m._features_rest), 1).detach().cpu().numpy()
    lang = m._language_feature.detach().cpu().numpy()
    dimg, ddep, dfeat = (g.detach().cpu().numpy() for g in grads)
    q = m._rotation.detach().cpu().numpy().astype(np.float64)
    nq = np.maximum(np.linalg.norm(q, axis=1, keepdims=True), 1e-12)
    qh = q / nq
    y = op.astype(np.float64).reshape(-1, 1)
    views, acc = [], None
    for i, cam in enumerate(cams):
        orc = OracleRaster(
            means3D=xyz, opacities=op, viewmatrix=cam.world_view_transform.cpu().numpy(),
            projmatrix=cam.full_proj_transform.cpu().numpy(),
            campos=cam.camera_center.cpu().numpy(), tanfovx=math.tan(cam.FoVx * 0.5),
            tanfovy=math.tan(cam.FoVy * 0.5), image_height=cam.image_height,
            image_width=cam.image_width, bg=np.zeros(3, np.float32), sh_degree=m.active_sh_degree,
            shs=shs, scales=sc, rotations=rot, shs_language=lang, include_feature=True)
        og = orc.backward(dimg, ddep, None, dfeat)
        views.append(dict(render=orc.color, depth=orc.depth, alpha=orc.alpha,
                          feature=orc.feature, radii=orc.radii, means2D=og["means2D"],
                          margin=orc.margin(), ranges=orc.ranges(), point_list=orc.point_list(),
                          n_contrib=orc.n_contrib(), final_T=orc.final_T(),
                          xy=orc.means2D(), conic_opacity=orc.conic_opacity(),
                          decisions=orc.accept_bits(), clamped=orc.clamped()))
        g = {k: og[k].astype(np.float64)
             for k in ("means3D", "sh", "opacity", "scales", "rotations", "sh_language")}
        gq = g["rotations"]
        raw = {
            "_xyz": g["means3D"],
            "_features_dc": g["sh"][:, :1, :],
            "_features_rest": g["sh"][:, 1:, :],
            "_opacity": g["opacity"].reshape(-1, 1) * (y * (1.0 - y)),
            "_scaling": g["scales"] * sc.astype(np.float64),
            "_rotation": (gq - qh * np.sum(qh * gq, axis=1, keepdims=True)) / nq,
            "_language_feature": g["sh_language"],
        }
        acc = raw if acc is None else {k: acc[k] + raw[k] for k in raw}
        del orc
        if progress:
            progress(f"oracle view {i + 1}/{len(cams)} done")
    return views, acc


# A pixel may decide alpha >= 1/255 or T < 1e-4 differently on GPU and oracle only when one of its
# decisions lies within a few float ulps of the threshold (oracle margin, OracleRaster.margin);
# 1e-4 relative covers the worst accumulated error of T over a pixel's list by ~10x.
FLIP_MARGIN = 1e-4
FLIP_TOL = 1e-5


def flipped_pixels(a, b, tol=FLIP_TOL):
    """(pixels off by more than tol in any image, the subset the oracle marks as near a
    threshold) -- boolean [H, W] maps."""
    off = np.zeros(b["margin"].shape, bool)
    for k in IMAGES:
        d = np.abs(a[k] - b[k])
        off |= (d.reshape(-1, *b["margin"].shape).max(0) > tol)
    return off, off & (b["margin"] < FLIP_MARGIN)


def decision_flips(a, b):
    """Pixels whose blend decisions differ between two oracle evaluations (float32 vs float64):
    their n_contrib differs, or their final T by more than rounding (a flipped 1/255 splat moves
    T by ~0.4 %, a flipped T < 1e-4 stop changes n_contrib)."""
    Ta, Tb = a["final_T"].astype(np.float64), b["final_T"].astype(np.float64)
    flips = (a["n_contrib"] != b["n_contrib"]) | (np.abs(Ta - Tb) > 1e-4 * np.maximum(Tb, 1e-4))
    # tiles whose instance lists differ (a radius rounded to another integer, a near-plane
    # cull decided the other way): every pixel of the tile
    ra, rb = a["ranges"].reshape(-1, 2), b["ranges"].reshape(-1, 2)
    H, W = flips.shape
    gx = (W + 15) // 16
    for t in range(ra.shape[0]):
        sa, ea = ra[t]
        sb, eb = rb[t]
        if ea - sa != eb - sb or not np.array_equal(a["point_list"][sa:ea], b["point_list"][sb:eb]):
            ty, tx = divmod(t, gx)
            flips[ty * 16:(ty + 1) * 16, tx * 16:(tx + 1) * 16] = True
    return flips


def flip_gaussians(b, flips, P, ncs=None):
    """Gaussians whose gradients see the flipped pixels: with ncs (the n_contrib maps of the
    evaluations compared) the pixel's contributors in either of them -- list positions
    [0, max n_contrib) of its tile -- else every Gaussian of the pixel's tile list."""
    hit = np.zeros(P, bool)
    if not flips.any():
        return hit
    H, W = flips.shape
    gx = (W + 15) // 16
    ys, xs = np.nonzero(flips)
    if ncs is None:
        for t in np.unique((ys // 16) * gx + xs // 16):
            s, e = b["ranges"][t]
            hit[b["point_list"][s:e]] = True
        return hit
    lim = np.max([np.asarray(n).reshape(H, W)[ys, xs] for n in ncs], axis=0)
    tiles = (ys // 16) * gx + xs // 16
    for t in np.unique(tiles):
        s, e = b["ranges"][t]
        L = int(lim[tiles == t].max())
        hit[b["point_list"][s:min(e, s + L)]] = True
    return hit


def pixel_contributors(b, flips, P, thr=0.99 / 255.0, extra=2):
    """Gaussians that can contribute to the flipped pixels in either of two evaluations whose
    decisions differ by rounding: per pixel, the tile-list entries with float32 alpha within 1 %
    of the 1/255 threshold or above it (power <= 0) before the float32 run's n_contrib, plus the
    first `extra` such entries after it (a T < 1e-4 stop decided one entry later).  The blend
    test follows forward.cu:337-357 (the oracle's alpha, its pixel centre convention)."""
    hit = np.zeros(P, bool)
    if not flips.any():
        return hit
    H, W = flips.shape
    gx = (W + 15) // 16
    nc = np.asarray(b["n_contrib"]).reshape(H, W)
    xy, co = b["xy"].astype(np.float64), b["conic_opacity"].astype(np.float64)
    for y, x in zip(*np.nonzero(flips)):
        s, e = b["ranges"][(y // 16) * gx + x // 16]
        ids = b["point_list"][s:e].astype(np.int64)
        dx, dy = xy[ids, 0] - x, xy[ids, 1] - y
        a, bb, c, o = co[ids].T
        power = -0.5 * (a * dx * dx + c * dy * dy) - bb * dx * dy
        alpha = np.minimum(0.99, o * np.exp(np.minimum(power, 0.0)))
        cand = (power <= 1e-6) & (alpha >= thr)
        pos = np.arange(ids.size)
        n = int(nc[y, x])
        late = np.nonzero(cand & (pos >= n))[0][:extra]
        hit[ids[cand & (pos < n)]] = True
        hit[ids[late]] = True
    return hit


def grad_stats(got, ref, exclude=None):
    """max|d| / max|ref| and the entry-wise picture behind it (entry-wise statistics skip the
    rows in `exclude`, Gaussians behind a threshold-flipped pixel)."""
    got = got.reshape(ref.shape).astype(np.float64)
    d = np.abs(got - ref)
    scale = float(np.abs(ref).max())
    big = np.abs(ref) >= 1e-2 * scale
    if exclude is not None and exclude.any():
        big = big & ~exclude.reshape((-1,) + (1,) * (ref.ndim - 1))
    rel_big = d[big] / np.abs(ref[big]) if big.any() else np.zeros(1)
    return {"scale": scale, "max_abs": float(d.max()) if d.size else 0.0,
            "rel_max": float(d.max()) / scale if scale > 0 else float(d.max()),
            "rel_big_p999": float(np.quantile(rel_big, 0.999)) if rel_big.size else 0.0,
            "rel_big_max": float(rel_big.max()) if rel_big.size else 0.0,
            "n": int(ref.size), "n_big": int(big.sum())}


def compare(tag, vg, vo, gg, go, stats_path=None, leaves=LEAVES):
    """Per-view images, radii, screen-space gradients and the summed raw-leaf gradients; returns
    the statistics (also appended to stats_path as one JSON line)."""
    st = {"case": tag, "views": [], "grads": {}}
    P = vo[0]["radii"].shape[0] if vo else 0
    hit_all = np.zeros(P, bool)
    for a, b in zip(vg, vo):
        v = {"radii_equal": bool(np.array_equal(a["radii"], b["radii"]))}
        off, flips = flipped_pixels(a, b)
        keep = ~flips
        for k in IMAGES:
            d = np.abs(a[k] - b[k]).reshape(-1, *keep.shape)
            v[k] = float(d.max()) if d.size else 0.0
            v[k + "_unflipped"] = float(d[:, keep].max()) if keep.any() else 0.0
        v["pixels_off"] = int(off.sum())
        v["pixels_flipped"] = int(flips.sum())
        v["pixels_near_threshold"] = int((b["margin"] < FLIP_MARGIN).sum())
        if off.any():
            i = int(np.argmax(np.where(off, np.abs(a["render"] - b["render"]).max(0), -1)))
            v["worst_off_margin"] = float(b["margin"].reshape(-1)[i])
        hit = flip_gaussians(b, flips, P)
        hit_all |= hit
        v["gaussians_behind_flips"] = int(hit.sum())
        v["means2D"] = grad_stats(a["means2D"][:, :2], b["means2D"][:, :2], hit)
        st["views"].append(v)
    for n in leaves:
        st["grads"][n] = grad_stats(gg[n], go[n], hit_all)
    if stats_path:
        os.makedirs(os.path.dirname(stats_path), exist_ok=True)
        with open(stats_path, "a") as fh:
            fh.write(json.dumps(st) + "\n")
    return st


def splat_records(pkgs):
    """Per view of a render_views call: the splat records its preprocess wrote ([P, 16] float32,
    gsr_testing.h gsr_test_splat_records), read from the views' geometry buffers, which the
    autograd node of the stacked outputs keeps for the backward."""
    from gsr_amd import _lib
    L = _lib.load()
    node = pkgs[0]["views"]["render"].grad_fn
    P = int(pkgs[0]["radii"].shape[0])
    torch.cuda.synchronize()
    out = []
    for view in node.views:  # the gsr_view structs: each view's carve of the call's scratch
        rec = np.zeros((P, 16), np.float32)
        _lib.check(L.gsr_test_splat_records(view.geom_buffer, P, rec.ctypes.data,
                                            torch.cuda.current_stream().cuda_stream))
        out.append(rec)
    return out
