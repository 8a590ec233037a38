"""Differentiable float64 PyTorch restatement of the rasterizer forward, used ONLY to cross-check
the hand-derived backward of the oracle (and through it the HIP backward) with autograd.

The discrete decisions (which splats land in which tile, in which order, and where each pixel's
blending stopped) are taken from the oracle's forward state; everything continuous is recomputed
in float64 with autograd.  Valid where no threshold is crossed and alpha < 0.99 (the reference's
0.99 clamp is straight-through in its backward, backward.cu:499 vs :538), which the test scenes
guarantee (opacity <= 0.9).  means2D is an additive NDC offset so its gradient equals the
reference's NDC-scaled dL/dmean2D (backward.cu:460-461, 545-546).
"""
from __future__ import annotations

import numpy as np
import torch

SH_C0 = 0.28209479177387814
SH_C1 = 0.4886025119029199
SH_C2 = [1.0925484305920792, -1.0925484305920792, 0.31539156525252005, -1.0925484305920792,
         0.5462742152960396]
SH_C3 = [-0.5900435899266435, 2.890611442640554, -0.4570457994644658, 0.3731763325901154,
         -0.4570457994644658, 1.445305721320277, -0.5900435899266435]


def sh_eval(deg, sh, d):
    """sh: [P,M,3], d: [P,3] unit -> [P,3]"""
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


def render_f64(kw, orc, leaves):
    """leaves: dict of float64 leaf tensors (means3D, means2D, opacities, shs | colors_precomp,
    scales + rotations | cov3D_precomp, shs_language | language_feature_precomp).
    Returns color [3,H,W], depth [1,H,W], alpha [1,H,W], feature [3,H,W]."""
    H, W = kw["image_height"], kw["image_width"]
    view = torch.tensor(kw["viewmatrix"], dtype=torch.float64).view(4, 4)
    proj = torch.tensor(kw["projmatrix"], dtype=torch.float64).view(4, 4)
    campos = torch.tensor(kw["campos"], dtype=torch.float64)
    bg = torch.tensor(kw["bg"], dtype=torch.float64)
    tanx, tany = kw["tanfovx"], kw["tanfovy"]
    fx, fy = W / (2 * tanx), H / (2 * tany)
    m = leaves["means3D"]
    P = m.shape[0]
    hom = torch.cat([m, torch.ones((P, 1), dtype=m.dtype)], 1)
    pv = hom @ view
    ph = hom @ proj
    pw = 1.0 / (ph[:, 3:4] + 1e-7)
    pp = ph[:, :2] * pw + leaves["means2D"][:, :2]
    pix_x = ((pp[:, 0] + 1.0) * W - 1.0) * 0.5
    pix_y = ((pp[:, 1] + 1.0) * H - 1.0) * 0.5
    if "cov3D_precomp" in leaves:
        c = leaves["cov3D_precomp"]
        Sig = torch.stack([c[:, 0], c[:, 1], c[:, 2], c[:, 1], c[:, 3], c[:, 4], c[:, 2], c[:, 4],
                           c[:, 5]], -1).view(P, 3, 3)
    else:
        s = leaves["scales"]
        q = leaves["rotations"]  # NOT normalised (forward.cu:127)
        r, x, y, z = q.unbind(-1)
        R = torch.stack([1 - 2 * (y * y + z * z), 2 * (x * y - r * z), 2 * (x * z + r * y),
                         2 * (x * y + r * z), 1 - 2 * (x * x + z * z), 2 * (y * z - r * x),
                         2 * (x * z - r * y), 2 * (y * z + r * x), 1 - 2 * (x * x + y * y)],
                        -1).view(P, 3, 3)
        L = R @ torch.diag_embed(s)
        Sig = L @ L.transpose(1, 2)
    t = pv[:, :3]
    limx, limy = 1.3 * tanx, 1.3 * tany
    tx = torch.clamp(t[:, 0] / t[:, 2], -limx, limx) * t[:, 2]
    ty = torch.clamp(t[:, 1] / t[:, 2], -limy, limy) * t[:, 2]
    tz = t[:, 2]
    zero = torch.zeros_like(tz)
    J = torch.stack([fx / tz, zero, -fx * tx / (tz * tz), zero, fy / tz, -fy * ty / (tz * tz)],
                    -1).view(P, 2, 3)
    Wr = view[:3, :3].t()  # W2C rotation
    T = J @ Wr
    cov2 = T @ Sig @ T.transpose(1, 2)
    a = cov2[:, 0, 0] + 0.3
    b = cov2[:, 0, 1]
    cc = cov2[:, 1, 1] + 0.3
    det = a * cc - b * b
    con_a, con_b, con_c = cc / det, -b / det, a / det
    op = leaves["opacities"].view(P)
    if kw.get("confidence") is not None:
        op = op * torch.tensor(kw["confidence"], dtype=torch.float64).view(P)
    if "shs" in leaves:
        d = m - campos
        d = d / d.norm(dim=1, keepdim=True)
        rgb = torch.clamp_min(sh_eval(kw["sh_degree"], leaves["shs"], d) + 0.5, 0.0)
    else:
        rgb = leaves["colors_precomp"]
    if kw["include_feature"] and "language_feature_precomp" in leaves:
        feat = leaves["language_feature_precomp"]
    elif kw["include_feature"] and "shs_language" in leaves:
        u = SH_C0 * leaves["shs_language"]
        feat = u / (u.norm(dim=-1, keepdim=True) + 1e-9)
    else:
        feat = torch.zeros((P, 3), dtype=torch.float64)
    depth = pv[:, 2]
    vals = torch.cat([rgb, depth[:, None], torch.ones((P, 1), dtype=torch.float64), feat], 1)

    plist = orc.point_list().astype(np.int64)
    ranges = orc.ranges()
    ncon = orc.n_contrib()
    gx = orc.gx
    out = torch.zeros((8, H, W), dtype=torch.float64)
    outT = torch.ones((H, W), dtype=torch.float64)
    out_list = []
    Tfin = []
    for tile in range(ranges.shape[0]):
        ty0, tx0 = (tile // gx) * 16, (tile % gx) * 16
        ys = torch.arange(ty0, min(ty0 + 16, H))
        xs = torch.arange(tx0, min(tx0 + 16, W))
        if len(ys) == 0 or len(xs) == 0:
            continue
        yy, xx = torch.meshgrid(ys, xs, indexing="ij")
        pyf, pxf = yy.reshape(-1).double(), xx.reshape(-1).double()
        s, e = int(ranges[tile, 0]), int(ranges[tile, 1])
        npx = pyf.shape[0]
        if e <= s:
            C = torch.zeros((npx, 8), dtype=torch.float64)
            Tf = torch.ones((npx,), dtype=torch.float64)
        else:
            ids = torch.tensor(plist[s:e])
            dx = pix_x[ids][None, :] - pxf[:, None]
            dy = pix_y[ids][None, :] - pyf[:, None]
            power = -0.5 * (con_a[ids][None] * dx * dx + con_c[ids][None] * dy * dy) - con_b[ids][None] * dx * dy
            alpha = op[ids][None] * torch.exp(power)
            nc = torch.tensor(ncon[yy.reshape(-1), xx.reshape(-1)].astype(np.int64))
            k = torch.arange(e - s)[None, :]
            mask = (power <= 0) & (alpha >= 1.0 / 255.0) & (k < nc[:, None])
            am = torch.where(mask, alpha, torch.zeros_like(alpha))
            one_m = 1 - am
            Tex = torch.cumprod(torch.cat([torch.ones((npx, 1), dtype=torch.float64), one_m[:, :-1]], 1), 1)
            wgt = am * Tex
            C = wgt @ vals[ids]
            Tf = Tex[:, -1] * one_m[:, -1]
        out_list.append((yy.reshape(-1), xx.reshape(-1), C, Tf))
    # scatter (non in-place ops to keep autograd simple)
    flat = torch.zeros((H * W, 8), dtype=torch.float64)
    Tflat = torch.ones((H * W,), dtype=torch.float64)
    idx_all, C_all, T_all = [], [], []
    for yy, xx, C, Tf in out_list:
        idx_all.append(yy * W + xx)
        C_all.append(C)
        T_all.append(Tf)
    idx = torch.cat(idx_all)
    flat = flat.index_put((idx,), torch.cat(C_all))
    Tflat = Tflat.index_put((idx,), torch.cat(T_all))
    flat = flat.t().reshape(8, H, W)
    Tflat = Tflat.view(H, W)
    color = flat[:3] + Tflat[None] * bg[:, None, None]
    dep = flat[3:4]
    alp = flat[4:5]
    fea = flat[5:8] if kw["include_feature"] else torch.zeros((3, H, W), dtype=torch.float64)
    return color, dep, alp, fea, Tflat


def leaves_from_kw(kw):
    L = {}
    for k in ("means3D", "shs", "colors_precomp", "scales", "rotations", "cov3D_precomp",
              "shs_language", "language_feature_precomp"):
        if kw.get(k) is not None:
            L[k] = torch.tensor(np.asarray(kw[k]), dtype=torch.float64).requires_grad_(True)
    P = L["means3D"].shape[0]
    L["opacities"] = torch.tensor(np.asarray(kw["opacities"]), dtype=torch.float64).view(P, 1).requires_grad_(True)
    L["means2D"] = torch.zeros((P, 3), dtype=torch.float64, requires_grad=True)
    return L
