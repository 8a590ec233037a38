"""Float64 evaluation of the benchmarked path and the rounding scale of every gradient entry
(used by tests/test_f64_parity.py and tests/test_f64_oracle.py).

TEST INFRASTRUCTURE: the CPU oracle's float64 build (oracle/Makefile libgsr_oracle_f64.so: the same
restatement -- same expressions, same order, same float32 inputs and float constants -- in
double) gives gradients whose own rounding is ~1e-16; the float32 checker and the GPU both differ
from it by their float32 rounding.  How large may a float32 rounding error of one entry be?  An
entry is a sum over pixels and views of per-pixel terms, chained through the per-Gaussian
backward (linear in the blend's per-Gaussian sums); a float32 evaluation of a sum of terms t_j can
be off by about u * sum |t_j| (u = 2^-24) times a small factor for the summation depth.  So per
entry i:

    B_i = sum over views, over the blend's 13 per-Gaussian sums k:  |J_ik| * A_k

where A_k = sum over pixels of |term| of sum k, each term weighted by the length of the float32
chain it went through -- T is the forward's product over the pixel's contributors, recovered by
one division per splat replayed, so its rounding grows with that chain (oracle_blend_rows(mass=1);
dL/dalpha replaced by the absolute values of its channel terms) -- and J = d(raw-leaf entry) / d(sum k) of the per-Gaussian
backward in float64 (oracle_backward_rows on unit rows; exact, it is linear).  An error of
|gpu - f64| <= C * u * B_i is float32 rounding of the entry's own terms; a systematic error (a
missing or mis-weighted term) is of the order of the term itself, ~1/(C u) times larger.
"""
from __future__ import annotations

import math

import numpy as np

from fused_ref import LEAVES
from oracle.oracle import OracleRaster

U32 = 2.0 ** -24  # float32 unit roundoff

# slot of the oracle's accumulator block -> (region offset in units of P, stride, index)
_ACC = {"col": (0, 3), "dep": (3, 1), "feat": (4, 3), "m2d": (7, 3), "con": (10, 4), "op": (14, 1)}
SLOTS = ([("col", c) for c in range(3)] + [("dep", 0)] + [("feat", c) for c in range(3)] +
         [("m2d", 0), ("m2d", 1)] + [("con", 0), ("con", 1), ("con", 3)] + [("op", 0)])


def _slot_view(rows, P, slot):
    off, stride = _ACC[slot[0]]
    return rows[off * P:(off + stride) * P].reshape(P, stride)[:, slot[1]]


def _raw_chain(g, op, sc, qh, nq):
    """The oracle's gradients of the activated inputs -> the raw leaves (float64), as
    fused_ref.run_oracle_path: sigmoid, exp, F.normalize, cat split."""
    y = op.astype(np.float64).reshape(-1, 1)
    gq = g["rotations"].astype(np.float64)
    return {
        "_xyz": g["means3D"].astype(np.float64),
        "_features_dc": g["sh"][:, :1, :].astype(np.float64),
        "_features_rest": g["sh"][:, 1:, :].astype(np.float64),
        "_opacity": g["opacity"].reshape(-1, 1).astype(np.float64) * (y * (1.0 - y)),
        "_scaling": g["scales"].astype(np.float64) * sc.astype(np.float64),
        "_rotation": (gq - qh * np.sum(qh * gq, axis=1, keepdims=True)) / nq,
        "_language_feature": g["sh_language"].astype(np.float64),
    }


def oracle_inputs(m, act):
    import torch
    op, sc, rot = (t.detach().cpu().numpy() for t in act)
    return dict(
        xyz=m._xyz.detach().cpu().numpy(),
        shs=torch.cat((m._features_dc, m._features_rest), 1).detach().cpu().numpy(),
        lang=m._language_feature.detach().cpu().numpy(), op=op, sc=sc, rot=rot,
        q=m._rotation.detach().cpu().numpy().astype(np.float64), deg=m.active_sh_degree)


def _raster(inp, cam, variant, lists=None, decisions=None, clamp=None, geometry=None):
    return OracleRaster(lists=lists, decisions=decisions, clamp=clamp, geometry=geometry,
        variant=variant, means3D=inp["xyz"], opacities=inp["op"],
        viewmatrix=cam.world_view_transform.cpu().numpy(),
        projmatrix=cam.full_proj_transform.cpu().numpy(), campos=cam.camera_center.cpu().numpy(),
        tanfovx=math.tan(cam.FoVx * 0.5), tanfovy=math.tan(cam.FoVy * 0.5),
        image_height=cam.image_height, image_width=cam.image_width, bg=np.zeros(3, np.float32),
        sh_degree=inp["deg"], shs=inp["shs"], scales=inp["sc"], rotations=inp["rot"],
        shs_language=inp["lang"], include_feature=True)


def run_f64_path(inp, cams, grads, progress=None, bound=True, lists=None, decisions=None,
                 clamps=None, geometry=None):
    """The float64 oracle on the views of the benchmarked path: per-view images / radii / margin /
    lists, the raw-leaf gradients summed over the views, and (bound) the per-entry rounding scale
    B (float64 arrays shaped like the leaves).  lists: per view (point_list, ranges) to blend
    instead of the float64 binning -- the float32 run's, so that a radius that rounds to another
    integer in float64 does not add or drop a Gaussian from whole tiles.  decisions: per view the
    float32 run's blend decisions (OracleRaster.accept_bits: n_contrib and, per pixel, which list
    positions it blended) in place of float64's own alpha >= 1/255, power <= 0 and T < 1e-4
    tests -- float64 then sums exactly the terms float32 summed, so every
    remaining difference is rounding.  clamps: per view the float32 run's SH colour clamp bits
    (OracleRaster.clamped) in place of float64's own result < 0 tests: the per-Gaussian decision
    that masks a channel's dL/dRGB (backward.cu:390-391), locked the same way.  geometry: per
    view the float32 run's projected splats (screen means, conic + opacity): the float32 pixel
    coordinate carries up to half an ulp (6e-5 px at x ~ 1500), which the Gaussian's falloff turns
    into ~1e-4 relative changes of G at a splat's edge -- a float32 preprocess effect the blend's
    rounding scale does not model; with it locked the float64 blend sums exactly the float32
    terms and the bound covers the blend and backward arithmetic."""
    dimg, ddep, dfeat = (g.detach().cpu().numpy() for g in grads)
    q = inp["q"]
    nq = np.maximum(np.linalg.norm(q, axis=1, keepdims=True), 1e-12)
    qh = q / nq
    views, acc, B = [], None, None
    for i, cam in enumerate(cams):
        o = _raster(inp, cam, "f64", None if lists is None else lists[i],
                    None if decisions is None else decisions[i],
                    None if clamps is None else clamps[i],
                    None if geometry is None else geometry[i])
        P = o.P
        rows = o.blend_rows(dimg, ddep, None, dfeat)
        raw = _raw_chain(o.backward_rows(rows), inp["op"], inp["sc"], qh, nq)
        acc = raw if acc is None else {k: acc[k] + raw[k] for k in raw}
        views.append(dict(render=o.color, depth=o.depth, alpha=o.alpha, feature=o.feature,
                          radii=o.radii, margin=o.margin(), ranges=o.ranges(),
                          point_list=o.point_list(), n_contrib=o.n_contrib(),
                          final_T=o.final_T()))
        if bound:
            mass = o.blend_rows(dimg, ddep, None, dfeat, mass=True)
            for slot in SLOTS:
                unit = np.zeros_like(rows)
                _slot_view(unit, P, slot)[:] = 1.0
                A = _slot_view(mass, P, slot)
                J = _raw_chain(o.backward_rows(unit), inp["op"], inp["sc"], qh, nq)
                term = {k: np.abs(J[k]) * A.reshape((P,) + (1,) * (J[k].ndim - 1)) for k in J}
                B = term if B is None else {k: B[k] + term[k] for k in term}
                if progress and P >= 1_000_000:
                    progress(f"f64 view {i + 1}: rounding scale of slot {slot} done")
        del o
        if progress:
            progress(f"f64 oracle view {i + 1}/{len(cams)} done")
    return views, acc, B


def rounding_stats(got, f32, f64, B, exclude=None, C=None, rel=1e-5):
    """Per-entry errors against float64 for entries >= 1 % of the tensor's maximum (rows in
    `exclude` -- Gaussians behind a threshold flip -- left out): relative errors of `got` and of
    the float32 oracle, their ratios to the rounding scale u * B, and how many `got` entries
    meet |got - f64| <= 2 |f32 - f64| (VERDICT r3's per-entry form) or <= 1e-5 |f64|.  With C:
    the failures of |d| <= max(rel |f64|, C u B) (rel = 0: the rounding bound alone)."""
    ref = f64.astype(np.float64)
    g = got.reshape(ref.shape).astype(np.float64)
    o = f32.reshape(ref.shape).astype(np.float64)
    b = B.reshape(ref.shape)
    scale = float(np.abs(ref).max())
    big = np.abs(ref) >= 1e-2 * scale
    if exclude is not None and exclude.any():
        big &= ~exclude.reshape((-1,) + (1,) * (ref.ndim - 1))
    dg, do = np.abs(g - ref)[big], np.abs(o - ref)[big]
    r, bb = np.abs(ref[big]), b[big]
    ub = U32 * np.maximum(bb, 1e-300)
    out = {"n_big": int(big.sum()), "scale": scale}
    if not big.any():
        return out
    for name, d in (("gpu", dg), ("f32", do)):
        out[name + "_rel_max"] = float((d / r).max())
        out[name + "_rel_p999"] = float(np.quantile(d / r, 0.999))
        out[name + "_ratio_max"] = float((d / ub).max())
        out[name + "_ratio_p999"] = float(np.quantile(d / ub, 0.999))
        out[name + "_abs_max_over_scale"] = float(np.abs((g if name == "gpu" else o) - ref).max()
                                                  / scale)
    out["gpu_within_2x_f32"] = float(np.mean(dg <= 2.0 * do))
    out["gpu_within_1e-5"] = float(np.mean(dg <= 1e-5 * r))
    out["f32_within_1e-5"] = float(np.mean(do <= 1e-5 * r))
    if C is not None:
        ok = (dg <= np.maximum(rel * r, C * ub))
        out["gpu_fail"] = int((~ok).sum())
        out["f32_fail"] = int((~(do <= np.maximum(rel * r, C * ub))).sum())
    return out


def controls_1e5(inp, cams, grads, geometry, lock):
    """The float64 gradients of two negative controls under the decision lock (VERDICT r5 item
    1): "colour" -- the colour terms off by 1e-5 (the image's upstream gradient scaled); "conic"
    -- the conic the float64 blend evaluates off by 1e-5 (the locked float32 splats' conic
    scaled).  A bound that passes both is not tight enough to catch a 1e-5 systematic error."""
    gd = (grads[0] * (1.0 + 1e-5), grads[1], grads[2])
    _, colour, _ = run_f64_path(inp, cams, gd, bound=False, geometry=geometry, **lock)
    geo = []
    for xy, co in geometry:
        co = co.copy()
        co[:, :3] *= np.float32(1.0 + 1e-5)
        geo.append((xy, co))
    _, conic, _ = run_f64_path(inp, cams, grads, bound=False, geometry=geo, **lock)
    return {"colour": colour, "conic": conic}
