"""PyTorch-CPU restatement of render()'s rasterizer: the CPU baseline BASELINE.json names.

TEST INFRASTRUCTURE / CPU BASELINE ONLY (bench.py's cpu_baseline leg and tests/): never imported by
the product package.  BASELINE.json: "the reference CPU baseline is PyTorch-CPU render() on the host
cores, timed in the same run" -- the reference has no CPU rasterizer, so this is the rasterizer
written as PyTorch tensor code, float32, forward and autograd backward, on torch's CPU threads:

* preprocess (forward.cu:155-256): projection, 3D -> 2D covariance (forward.cu:74-152), conic,
  radius, SH colour (forward.cu:20-71 via the reference's eval_sh order), tile rectangles;
* binning (rasterizer_impl.cu:70-138): every tile of each Gaussian's 3-sigma rectangle,
  repeat_interleave + a stable sort by (tile, float32 depth bits) -- the reference's key;
* blend (forward.cu:261-374): per tile, the [pixels x instances] alpha matrix, transmittance by
  cumprod, the reference's alpha >= 1/255, power <= 0, 0.99 clamp and T < 1e-4 termination,
  the eight channels (rgb, depth, alpha, feature) as one weighted matrix product;
* backward: autograd.  The blend's graph is built and back-propagated one tile at a time into
  detached per-Gaussian leaves (means2D, conic, opacity, colour, depth, feature) -- a whole-image
  graph would hold ~10 [pixels x instances] tensors per tile (tens of GB at the headline size) --
  then one autograd pass through the preprocess.

Numerics follow torch's float32 kernels (exp, matmul): it is a timing baseline, checked against
the C oracle to image tolerance in tests/test_torch_cpu.py, not a parity reference.
"""
from __future__ import annotations

import math

import torch

SH_C0 = 0.28209479177387814
SH_C1 = 0.4886025119029199
SH_C2 = (1.0925484305920792, -1.0925484305920792, 0.31539156525252005, -1.0925484305920792,
         0.5462742152960396)
SH_C3 = (-0.5900435899266435, 2.890611442640554, -0.4570457994644658, 0.3731763325901154,
         -0.4570457994644658, 1.445305721320277, -0.5900435899266435)
BLOCK = 16


def eval_sh(deg, sh, d):
    """utils/sh_utils.py eval_sh order: sh [P, M, 3], d [P, 3] unit -> [P, 3]."""
    x, y, z = d[:, 0:1], d[:, 1:2], d[:, 2:3]
    r = SH_C0 * sh[:, 0]
    if deg > 0:
        r = r - SH_C1 * y * sh[:, 1] + SH_C1 * z * sh[:, 2] - SH_C1 * x * sh[:, 3]
    if deg > 1:
        xx, yy, zz, xy, yz, xz = x * x, y * y, z * z, x * y, y * z, x * z
        r = (r + SH_C2[0] * xy * sh[:, 4] + SH_C2[1] * yz * sh[:, 5]
             + SH_C2[2] * (2 * zz - xx - yy) * sh[:, 6] + SH_C2[3] * xz * sh[:, 7]
             + SH_C2[4] * (xx - yy) * sh[:, 8])
    if deg > 2:
        r = (r + SH_C3[0] * y * (3 * xx - yy) * sh[:, 9] + SH_C3[1] * xy * z * sh[:, 10]
             + SH_C3[2] * y * (4 * zz - xx - yy) * sh[:, 11]
             + SH_C3[3] * z * (2 * zz - 3 * xx - 3 * yy) * sh[:, 12]
             + SH_C3[4] * x * (4 * zz - xx - yy) * sh[:, 13] + SH_C3[5] * z * (xx - yy) * sh[:, 14]
             + SH_C3[6] * x * (xx - 3 * yy) * sh[:, 15])
    return r


def preprocess(means3D, opacities, shs, scales, rotations, shs_language, deg, viewmatrix,
               projmatrix, campos, tanfovx, tanfovy, H, W):
    """Per-Gaussian screen-space quantities (differentiable) and the integer binning data."""
    P = means3D.shape[0]
    view = viewmatrix.view(4, 4)
    proj = projmatrix.view(4, 4)
    hom = torch.cat([means3D, torch.ones((P, 1), dtype=means3D.dtype)], 1)
    pv = hom @ view
    ph = hom @ proj
    pw = 1.0 / (ph[:, 3:4] + 1e-7)
    pp = ph[:, :2] * pw
    pix = torch.stack([((pp[:, 0] + 1.0) * W - 1.0) * 0.5, ((pp[:, 1] + 1.0) * H - 1.0) * 0.5], 1)
    q = rotations
    r, x, y, z = q.unbind(-1)
    R = torch.stack([1 - 2 * (y * y + z * z), 2 * (x * y - r * z), 2 * (x * z + r * y),
                     2 * (x * y + r * z), 1 - 2 * (x * x + z * z), 2 * (y * z - r * x),
                     2 * (x * z - r * y), 2 * (y * z + r * x), 1 - 2 * (x * x + y * y)],
                    -1).view(P, 3, 3)
    L = R @ torch.diag_embed(scales)
    Sig = L @ L.transpose(1, 2)
    t = pv[:, :3]
    limx, limy = 1.3 * tanfovx, 1.3 * tanfovy
    fx, fy = W / (2 * tanfovx), H / (2 * tanfovy)
    tz = t[:, 2]
    tx = torch.clamp(t[:, 0] / tz, -limx, limx) * tz
    ty = torch.clamp(t[:, 1] / tz, -limy, limy) * tz
    zero = torch.zeros_like(tz)
    J = torch.stack([fx / tz, zero, -fx * tx / (tz * tz), zero, fy / tz, -fy * ty / (tz * tz)],
                    -1).view(P, 2, 3)
    T = J @ view[:3, :3].t()
    cov2 = T @ Sig @ T.transpose(1, 2)
    a = cov2[:, 0, 0] + 0.3
    b = cov2[:, 0, 1]
    c = cov2[:, 1, 1] + 0.3
    det = a * c - b * b
    conic = torch.stack([c / det, -b / det, a / det], 1)
    d = means3D - campos
    rgb = torch.clamp_min(eval_sh(deg, shs, d / d.norm(dim=1, keepdim=True)) + 0.5, 0.0)
    u = SH_C0 * shs_language
    feat = u / (u.norm(dim=-1, keepdim=True) + 1e-9)
    depth = pv[:, 2]
    with torch.no_grad():  # radius and tile rectangle (forward.cu:198-206, auxiliary.h:46-56)
        mid = 0.5 * (a + c)
        lam = mid + torch.sqrt(torch.clamp_min(mid * mid - det, 0.1))
        radius = torch.ceil(3.0 * torch.sqrt(lam))
        gx, gy = (W + BLOCK - 1) // BLOCK, (H + BLOCK - 1) // BLOCK
        x0 = torch.clamp(((pix[:, 0] - radius) / BLOCK).to(torch.int64), 0, gx)
        y0 = torch.clamp(((pix[:, 1] - radius) / BLOCK).to(torch.int64), 0, gy)
        x1 = torch.clamp(((pix[:, 0] + radius + BLOCK - 1) / BLOCK).to(torch.int64), 0, gx)
        y1 = torch.clamp(((pix[:, 1] + radius + BLOCK - 1) / BLOCK).to(torch.int64), 0, gy)
        visible = (tz > 0.2) & (det != 0) & ((x1 - x0) * (y1 - y0) > 0)
    return dict(pix=pix, conic=conic, opacity=opacities.view(P), rgb=rgb, depth=depth, feat=feat,
                rect=(x0, y0, x1, y1), visible=visible, radius=radius.to(torch.int32), gx=gx, gy=gy)


def bin_instances(pre):
    """duplicateWithKeys + SortPairs: instance Gaussian ids sorted by (tile, depth), and each
    tile's [start, end) range."""
    x0, y0, x1, y1 = pre["rect"]
    vis = pre["visible"]
    ids = torch.nonzero(vis).view(-1)
    w, h = (x1 - x0)[ids], (y1 - y0)[ids]
    n = w * h
    gid = torch.repeat_interleave(ids, n)
    start = torch.cumsum(n, 0) - n
    k = torch.arange(gid.shape[0]) - torch.repeat_interleave(start, n)
    ww = torch.repeat_interleave(w, n)
    tx = x0[gid] + k % ww
    ty = y0[gid] + k // ww
    tile = ty * pre["gx"] + tx
    dbits = pre["depth"].detach().contiguous().view(torch.int32)[gid].to(torch.int64) & 0xFFFFFFFF
    order = torch.sort((tile << 32) | dbits, stable=True).indices
    gid, tile = gid[order], tile[order]
    ntiles = pre["gx"] * pre["gy"]
    counts = torch.bincount(tile, minlength=ntiles)
    ends = torch.cumsum(counts, 0)
    return gid, ends - counts, ends


def blend_tile(ids, x0, y0, W, H, pix, conic, op, vals):
    """One tile's eight channels (and final T) from its instance list, front to back."""
    ys = torch.arange(y0, min(y0 + BLOCK, H), dtype=torch.float32)
    xs = torch.arange(x0, min(x0 + BLOCK, W), dtype=torch.float32)
    py, px = torch.meshgrid(ys, xs, indexing="ij")
    py, px = py.reshape(-1, 1), px.reshape(-1, 1)
    dx = pix[ids, 0][None] - px
    dy = pix[ids, 1][None] - py
    cn = conic[ids]
    power = -0.5 * (cn[:, 0][None] * dx * dx + cn[:, 2][None] * dy * dy) - cn[:, 1][None] * dx * dy
    alpha = torch.clamp_max(op[ids][None] * torch.exp(power), 0.99)
    take = (power <= 0) & (alpha >= 1.0 / 255.0)
    a = torch.where(take, alpha, torch.zeros_like(alpha))
    Tin = torch.cumprod(torch.cat([torch.ones_like(a[:, :1]), 1 - a[:, :-1]], 1), 1)
    # forward.cu:346-351: a splat that would take T below 1e-4 ends the pixel (not blended)
    live = (Tin * (1 - a) >= 1e-4).to(a.dtype)
    live = torch.cumprod(torch.where(take, live, torch.ones_like(live)), 1)
    wgt = a * Tin * live
    C = wgt @ vals[ids]
    Tf = torch.prod(1 - a * live, 1)
    return C, Tf, ys.numel(), xs.numel()


def render(means3D, opacities, shs, scales, rotations, shs_language, deg, cam, bg,
           upstream=None):
    """render()'s outputs (color, depth, alpha, feature, radii) on the CPU; with upstream =
    (dL/dcolor, dL/ddepth, dL/dfeature) also the backward (gradients in the leaves' .grad)."""
    H, W = cam["H"], cam["W"]
    pre = preprocess(means3D, opacities, shs, scales, rotations, shs_language, deg, cam["view"],
                     cam["proj"], cam["campos"], cam["tanfovx"], cam["tanfovy"], H, W)
    gid, starts, ends = bin_instances(pre)
    keys = ("pix", "conic", "opacity", "rgb", "depth", "feat")
    leaves = {k: pre[k].detach().requires_grad_(upstream is not None) for k in keys}
    P = means3D.shape[0]
    vals = torch.cat([leaves["rgb"], leaves["depth"][:, None], torch.ones((P, 1)),
                      leaves["feat"]], 1)
    out = torch.zeros((8, H, W))
    Tfin = torch.ones((H, W))
    gx = pre["gx"]
    for t in range(gx * pre["gy"]):
        s, e = int(starts[t]), int(ends[t])
        if e <= s:
            continue
        ty, tx = divmod(t, gx)
        with torch.set_grad_enabled(upstream is not None):
            C, Tf, h, w = blend_tile(gid[s:e], tx * BLOCK, ty * BLOCK, W, H, leaves["pix"],
                                     leaves["conic"], leaves["opacity"], vals)
            if upstream is not None:
                dC = torch.cat([upstream[0][:, ty * BLOCK:ty * BLOCK + h, tx * BLOCK:tx * BLOCK + w],
                                upstream[1][:, ty * BLOCK:ty * BLOCK + h, tx * BLOCK:tx * BLOCK + w],
                                torch.zeros((1, h, w)),
                                upstream[2][:, ty * BLOCK:ty * BLOCK + h, tx * BLOCK:tx * BLOCK + w]
                                ], 0).reshape(8, -1).t()
                dT = (upstream[0][:, ty * BLOCK:ty * BLOCK + h, tx * BLOCK:tx * BLOCK + w]
                      * bg[:, None, None]).sum(0).reshape(-1)
                torch.autograd.backward([C, Tf], [dC, dT])
        out[:, ty * BLOCK:ty * BLOCK + h, tx * BLOCK:tx * BLOCK + w] = C.detach().t().reshape(8, h, w)
        Tfin[ty * BLOCK:ty * BLOCK + h, tx * BLOCK:tx * BLOCK + w] = Tf.detach().reshape(h, w)
    if upstream is not None:
        torch.autograd.backward([pre[k] for k in keys if leaves[k].grad is not None],
                                [leaves[k].grad for k in keys if leaves[k].grad is not None])
    color = out[:3] + Tfin[None] * bg[:, None, None]
    radii = torch.where(pre["visible"], pre["radius"], torch.zeros_like(pre["radius"]))
    return color, out[3:4], out[4:5], out[5:8], radii


def camera_dict(cam):
    return dict(H=int(cam.image_height), W=int(cam.image_width),
                view=cam.world_view_transform.detach().cpu().float().reshape(-1),
                proj=cam.full_proj_transform.detach().cpu().float().reshape(-1),
                campos=cam.camera_center.detach().cpu().float(),
                tanfovx=math.tan(cam.FoVx * 0.5), tanfovy=math.tan(cam.FoVy * 0.5))
