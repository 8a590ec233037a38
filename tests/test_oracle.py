"""Pins the CPU restatement (oracle/) before it is trusted as the parity oracle.

* golden vectors generated from the reference's own importable Python (tests/golden/make_golden.py):
  camera matrices and the SH colour evaluation;
* analytic known answers and the edge cases of SURVEY.md 8(c)(2);
* a float64 autograd cross-check of the hand-derived backward (tests/torch_ref.py).
"""
import json
import math
import os

import numpy as np
import pytest
import torch

from oracle.oracle import OracleRaster, mark_visible
from gsr_amd import camera as gcam
from scenes import scene
from torch_ref import leaves_from_kw, render_f64

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _cam_identity(W, H, z_cam=-4.0, f=None):
    f = 0.8 * W if f is None else f
    fovx, fovy = gcam.focal2fov(f, W), gcam.focal2fov(f, H)
    c = gcam.make_camera(np.eye(3), np.array([0.0, 0.0, -z_cam]), fovx, fovy, W, H)
    return c, fovx, fovy


def _base_kw(c, W, H, fovx, fovy, bg=(0.0, 0.0, 0.0)):
    return dict(viewmatrix=c.world_view_transform.numpy(), projmatrix=c.full_proj_transform.numpy(),
                campos=c.camera_center.numpy(), tanfovx=math.tan(fovx / 2), tanfovy=math.tan(fovy / 2),
                image_height=H, image_width=W, bg=np.asarray(bg, np.float32))


# ---------------------------------------------------------------------------------------------
# golden vectors from the reference Python
# ---------------------------------------------------------------------------------------------
def test_camera_matrices_match_reference_golden():
    d = np.load(os.path.join(GOLD, "camera_golden.npz"))
    for i in range(d["R"].shape[0]):
        c = gcam.make_camera(d["R"][i], d["T"][i], float(d["FoVx"][i]), float(d["FoVy"][i]),
                             int(d["W"][i]), int(d["H"][i]))
        np.testing.assert_array_equal(c.world_view_transform.numpy(), d["world_view_transform"][i])
        np.testing.assert_array_equal(c.full_proj_transform.numpy(), d["full_proj_transform"][i])
        np.testing.assert_array_equal(c.camera_center.numpy(), d["camera_center"][i])


@pytest.mark.parametrize("deg", [0, 1, 2, 3])
def test_oracle_sh_colour_matches_reference_eval_sh(deg):
    """In-kernel SH (forward.cu:20-71) == render()'s Python path clamp_min(eval_sh + 0.5, 0)
    (gaussian_renderer/__init__.py:269-274) on the reference's own eval_sh outputs."""
    d = np.load(os.path.join(GOLD, "sh_golden.npz"))
    xyz, campos = d["xyz"], d["campos"]
    P = xyz.shape[0]
    W, H = 64, 48
    # camera centred at the golden campos looking +z: every Gaussian is in front (z_view in [3, 5])
    f = 0.8 * W
    fovx, fovy = gcam.focal2fov(f, W), gcam.focal2fov(f, H)
    c = gcam.make_camera(np.eye(3), -campos.astype(np.float64), fovx, fovy, W, H)
    kw = _base_kw(c, W, H, fovx, fovy)
    kw["campos"] = campos  # the exact golden campos (float32)
    s = np.full((P, 3), 0.01, np.float32)
    q = np.tile(np.array([1, 0, 0, 0], np.float32), (P, 1))
    # large FoV so every splat lands on screen and is kept (rgb is only stored for kept splats)
    kw["tanfovx"] = kw["tanfovy"] = 2.0
    o = OracleRaster(means3D=xyz, opacities=np.full((P,), 0.5, np.float32), shs=d["features"],
                     sh_degree=deg, scales=s, rotations=q, include_feature=False, **kw)
    vis = o.radii > 0
    assert vis.sum() > 0.9 * P
    np.testing.assert_allclose(o.rgb()[vis], d[f"colors_precomp_deg{deg}"][vis], rtol=0, atol=3e-6)


def test_oracle_language_feature_paths_agree_with_reference_golden():
    """shs_language in-kernel path == language_feature_precomp built by render()'s Python path
    (gaussian_renderer/__init__.py:280-287), compared on rendered feature images."""
    d = np.load(os.path.join(GOLD, "sh_golden.npz"))
    xyz, P = d["xyz"], d["xyz"].shape[0]
    W, H = 64, 48
    c, fovx, fovy = _cam_identity(W, H)
    kw = _base_kw(c, W, H, fovx, fovy)
    common = dict(means3D=xyz, opacities=np.full((P,), 0.3, np.float32),
                  colors_precomp=np.full((P, 3), 0.5, np.float32),
                  scales=np.full((P, 3), 0.05, np.float32),
                  rotations=np.tile(np.array([1, 0, 0, 0], np.float32), (P, 1)),
                  include_feature=True, **kw)
    a = OracleRaster(shs_language=d["language_feature"], **common)
    b = OracleRaster(language_feature_precomp=d["language_feature_precomp"], **common)
    assert np.abs(a.feature).max() > 0.1
    np.testing.assert_allclose(a.feature, b.feature, rtol=0, atol=2e-6)


def test_pipeline_flag_defaults_golden():
    with open(os.path.join(GOLD, "pipeline_flags.json")) as fh:
        flags = json.load(fh)
    # the defaults the drop-in render() counterpart must honour
    assert flags == {"compute_cov3D_python": False, "convert_SHs_python": True, "debug": False,
                     "include_feature": True, "sh_degree": 3, "use_confidence": False}


# ---------------------------------------------------------------------------------------------
# analytic known answers and edge cases
# ---------------------------------------------------------------------------------------------
def test_single_gaussian_known_answer():
    W, H = 65, 49  # odd sizes: the projected centre (W-1)/2, (H-1)/2 is an exact pixel centre
    c, fovx, fovy = _cam_identity(W, H)
    kw = _base_kw(c, W, H, fovx, fovy, bg=(0.25, 0.5, 0.75))
    o_val, col = np.float32(0.6), np.array([[0.2, 0.4, 0.8]], np.float32)
    sigma = 0.02
    o = OracleRaster(means3D=np.zeros((1, 3), np.float32), opacities=np.array([o_val]),
                     colors_precomp=col, cov3D_precomp=np.array([[sigma ** 2, 0, 0, sigma ** 2, 0, sigma ** 2]], np.float32),
                     include_feature=False, **kw)
    cy, cx = (H - 1) // 2, (W - 1) // 2
    T = np.float32(1) * (np.float32(1) - o_val)
    for ch in range(3):
        expect = col[0, ch] * o_val * np.float32(1) + T * kw["bg"][ch]
        assert o.color[ch, cy, cx] == expect
    assert o.n_contrib()[cy, cx] == 1
    assert o.final_T()[cy, cx] == T
    assert o.depth[0, cy, cx] == np.float32(4.0) * o_val
    assert o.alpha[0, cy, cx] == o_val
    # radius: ceil(3 sqrt(lambda_max)); isotropic a = c, b = 0 so mid^2 - det = 0 and the
    # reference's max(0.1, .) floor (forward.cu:230) gives lambda = a + sqrt(0.1)
    f = W / (2 * math.tan(fovx / 2))
    lam = (f * sigma / 4.0) ** 2 + 0.3 + math.sqrt(0.1)
    assert o.radii[0] == math.ceil(3 * math.sqrt(lam))
    assert o.num_rendered == o.tiles_touched()[0] >= 1


def test_culling_edge_cases():
    W, H = 64, 48
    c, fovx, fovy = _cam_identity(W, H)
    kw = _base_kw(c, W, H, fovx, fovy)
    # 0: behind the near plane (view z = 4 - 3.9 = 0.1 <= 0.2); 1: far off-screen;
    # 2: visible; 3: clipped at the left border
    xyz = np.array([[0, 0, -3.9], [500, 0, 0], [0, 0, 0], [-1.9, 0, 0]], np.float32)
    P = xyz.shape[0]
    o = OracleRaster(means3D=xyz, opacities=np.full((P,), 0.5, np.float32),
                     colors_precomp=np.ones((P, 3), np.float32),
                     scales=np.full((P, 3), 0.05, np.float32),
                     rotations=np.tile(np.array([1, 0, 0, 0], np.float32), (P, 1)),
                     include_feature=False, **kw)
    r = o.radii
    assert r[0] == 0 and r[1] == 0 and r[2] > 0 and r[3] > 0
    tt = o.tiles_touched()
    assert tt[0] == 0 and tt[1] == 0 and tt[2] > 0
    np.testing.assert_array_equal(mark_visible(xyz, kw["viewmatrix"], kw["projmatrix"]),
                                  [False, True, True, True])


def test_det_zero_is_culled():
    W, H = 64, 48
    f = 4.0  # focal == view depth -> J = diag(1, 1) for a point on the optical axis
    fov = gcam.focal2fov(f, W)
    fovy = gcam.focal2fov(f, H)
    c = gcam.make_camera(np.eye(3), np.array([0.0, 0.0, 4.0]), fov, fovy, W, H)
    kw = _base_kw(c, W, H, fov, fovy)
    cov = np.array([[1.0, 1.3, 0.0, 1.0, 0.0, 1.0]], np.float32)  # 2D cov + 0.3 I is singular
    o = OracleRaster(means3D=np.zeros((1, 3), np.float32), opacities=np.array([0.5], np.float32),
                     colors_precomp=np.ones((1, 3), np.float32), cov3D_precomp=cov,
                     include_feature=False, **kw)
    assert o.radii[0] == 0 and o.num_rendered == 0


def test_equal_depth_ties_keep_gaussian_order():
    W, H = 32, 32
    c, fovx, fovy = _cam_identity(W, H)
    kw = _base_kw(c, W, H, fovx, fovy)
    xyz = np.zeros((3, 3), np.float32)  # identical depth (and position)
    P = 3
    cols = np.array([[1, 0, 0], [0, 1, 0], [0, 0, 1]], np.float32)
    o = OracleRaster(means3D=xyz, opacities=np.array([0.5, 0.5, 0.5], np.float32),
                     colors_precomp=cols, scales=np.full((P, 3), 0.2, np.float32),
                     rotations=np.tile(np.array([1, 0, 0, 0], np.float32), (P, 1)),
                     include_feature=False, **kw)
    pl = o.point_list()
    rg = o.ranges()
    for t in range(rg.shape[0]):
        seg = pl[rg[t, 0]:rg[t, 1]]
        if len(seg):
            assert list(seg) == sorted(seg)
    # front-to-back in index order: red gets the largest weight
    cy, cx = 15, 15
    assert o.color[0, cy, cx] > o.color[1, cy, cx] > o.color[2, cy, cx]


def test_early_termination_alpha_clamp_and_skip():
    W, H = 32, 32
    c, fovx, fovy = _cam_identity(W, H)
    kw = _base_kw(c, W, H, fovx, fovy)
    n = 8
    xyz = np.zeros((n + 1, 3), np.float32)
    xyz[:, 2] = np.linspace(-1, 1, n + 1).astype(np.float32)
    op = np.full((n + 1,), 1.0, np.float32)  # alpha clamps to 0.99
    op[0] = 0.003  # front-most: alpha < 1/255, skipped everywhere
    o = OracleRaster(means3D=xyz, opacities=op, colors_precomp=np.ones((n + 1, 3), np.float32),
                     scales=np.full((n + 1, 3), 0.5, np.float32),
                     rotations=np.tile(np.array([1, 0, 0, 0], np.float32), (n + 1, 1)),
                     include_feature=False, **kw)
    cy, cx = 15, 15
    # T: 1 -> 0.01 -> 1e-4 (0.0001 * ... next test_T < 1e-4 stops): exactly two splats blended
    T = np.float32(1)
    T = T * (np.float32(1) - np.float32(0.99))
    assert o.final_T()[cy, cx] < 0.0101
    assert o.n_contrib()[cy, cx] <= 4
    assert o.final_T()[cy, cx] >= 1e-4


def test_active_degree_below_max_uses_stride_M():
    d = np.load(os.path.join(GOLD, "sh_golden.npz"))
    xyz, campos = d["xyz"][:64], d["campos"]
    P = xyz.shape[0]
    W, H = 64, 48
    f = 0.8 * W
    fovx, fovy = gcam.focal2fov(f, W), gcam.focal2fov(f, H)
    c = gcam.make_camera(np.eye(3), -campos.astype(np.float64), fovx, fovy, W, H)
    kw = _base_kw(c, W, H, fovx, fovy)
    kw["campos"] = campos
    kw["tanfovx"] = kw["tanfovy"] = 2.0
    o = OracleRaster(means3D=xyz, opacities=np.full((P,), 0.5, np.float32),
                     shs=d["features"][:64], sh_degree=1, scales=np.full((P, 3), 0.01, np.float32),
                     rotations=np.tile(np.array([1, 0, 0, 0], np.float32), (P, 1)),
                     include_feature=False, **kw)
    vis = o.radii > 0
    np.testing.assert_allclose(o.rgb()[vis], d["colors_precomp_deg1"][:64][vis], atol=3e-6, rtol=0)


def test_empty_scene():
    W, H = 32, 16
    c, fovx, fovy = _cam_identity(W, H)
    kw = _base_kw(c, W, H, fovx, fovy, bg=(1, 1, 1))
    o = OracleRaster(means3D=np.zeros((0, 3), np.float32), opacities=np.zeros((0,), np.float32),
                     colors_precomp=np.zeros((0, 3), np.float32), scales=np.zeros((0, 3), np.float32),
                     rotations=np.zeros((0, 4), np.float32), include_feature=False, **kw)
    assert o.num_rendered == 0
    # no splats: every pixel shows the background (the reference's P == 0 early-out instead
    # returns its zero-initialised image, rasterize_points.cu:68,81; the C-ABI mirrors that)
    np.testing.assert_array_equal(o.color, np.ones((3, H, W), np.float32))


def test_confidence_is_identity_at_one():
    kw = scene(P=128, W=48, H=32, mode="colors", feature="precomp")
    a = OracleRaster(**kw)
    b = OracleRaster(confidence=np.ones((128,), np.float32), **kw)
    np.testing.assert_array_equal(a.color, b.color)
    np.testing.assert_array_equal(a.feature, b.feature)


def test_depth_and_alpha_superposition_identities():
    """depth == vanilla render of colors_precomp = z * 1_3 with bg 0; alpha == render of 1_3."""
    kw = scene(P=200, W=48, H=40, mode="colors", feature=None, bg=(0, 0, 0))
    base = OracleRaster(**kw)
    z = base.depths()
    kz = dict(kw)
    kz["colors_precomp"] = np.repeat(z[:, None], 3, 1).astype(np.float32)
    dz = OracleRaster(**kz)
    np.testing.assert_array_equal(base.depth[0], dz.color[0])
    k1 = dict(kw)
    k1["colors_precomp"] = np.ones_like(kw["colors_precomp"])
    a1 = OracleRaster(**k1)
    np.testing.assert_array_equal(base.alpha[0], a1.color[0])


# ---------------------------------------------------------------------------------------------
# autograd cross-check of the backward
# ---------------------------------------------------------------------------------------------
CASES = [
    dict(mode="sh", cov_mode="scale_rot", feature="sh"),
    dict(mode="colors", cov_mode="scale_rot", feature="precomp"),
    dict(mode="sh", cov_mode="cov3D", feature=None),
    dict(mode="colors", cov_mode="cov3D", feature="sh", bg=(0.0, 0.0, 0.0)),
]


@pytest.mark.parametrize("case", range(len(CASES)))
def test_oracle_backward_matches_float64_autograd(case):
    kw = scene(P=96, W=40, H=34, seed=3 + case, **CASES[case])
    orc = OracleRaster(**kw)
    H, W = kw["image_height"], kw["image_width"]
    g = torch.Generator().manual_seed(11)
    dimg = torch.randn((3, H, W), generator=g)
    ddep = torch.randn((1, H, W), generator=g) * 0.3
    dalp = torch.randn((1, H, W), generator=g)
    dfea = torch.randn((3, H, W), generator=g)
    grads = orc.backward(dimg.numpy(), ddep.numpy(), dalp.numpy(), dfea.numpy())

    leaves = leaves_from_kw(kw)
    color, dep, alp, fea, _ = render_f64(kw, orc, leaves)
    # forward agreement (float32 oracle vs float64 model)
    np.testing.assert_allclose(orc.color, color.detach().numpy(), atol=2e-5, rtol=0)
    np.testing.assert_allclose(orc.depth, dep.detach().numpy(), atol=1e-4, rtol=0)
    loss = (color * dimg.double()).sum() + (dep * ddep.double()).sum() + (alp * dalp.double()).sum()
    if kw["include_feature"]:
        loss = loss + (fea * dfea.double()).sum()
    loss.backward()
    pairs = [("means3D", "means3D"), ("means2D", "means2D"), ("opacity", "opacities"),
             ("colors", "colors_precomp"), ("sh", "shs"), ("scales", "scales"),
             ("rotations", "rotations"), ("cov3D", "cov3D_precomp"),
             ("sh_language", "shs_language"), ("language_feature", "language_feature_precomp")]
    checked = 0
    for gname, lname in pairs:
        if lname not in leaves or grads.get(gname) is None:
            continue
        ref = leaves[lname].grad.numpy().reshape(grads[gname].shape)
        got = grads[gname]
        scale = max(np.abs(ref).max(), 1e-6)
        err = np.abs(got - ref).max() / scale
        assert err < 1e-5, f"{gname}: max err {err:.3e} (scale {scale:.3e})"
        checked += 1
    assert checked >= 5


@pytest.mark.parametrize("mode", ["sh", "colors"])
def test_oracle_threads_match_sequential(mode):
    """oracle_set_threads only splits loops into fixed chunks: the forward is bit-identical to the
    sequential restatement, the backward differs only by the association of its per-chunk sums."""
    from oracle.oracle import set_threads
    kw = scene(P=3000, W=97, H=61, seed=11, mode=mode, feature="sh")
    rng = np.random.default_rng(0)
    g = [rng.standard_normal(s).astype(np.float32) for s in ((3, 61, 97), (1, 61, 97), (1, 61, 97),
                                                             (3, 61, 97))]
    res = []
    try:
        for n in (1, 5):
            assert set_threads(n) == n
            o = OracleRaster(**kw)
            res.append((o.color.copy(), o.depth.copy(), o.feature.copy(), o.radii.copy(),
                        o.point_list(), o.backward(*g)))
    finally:
        set_threads(1)
    (c1, d1, f1, r1, p1, g1), (c5, d5, f5, r5, p5, g5) = res
    for a, b in ((c1, c5), (d1, d5), (f1, f5), (r1, r5), (p1, p5)):
        np.testing.assert_array_equal(a, b)
    for k, v in g1.items():
        if v is None:
            continue
        scale = max(float(np.abs(v).max()), 1e-12)
        assert float(np.abs(v - g5[k]).max()) / scale <= 1e-6, k


def test_splat_exp_accuracy():
    """The blend's deterministic exp (oracle/gsr_oracle.c splat_exp, shared with the kernels):
    within 1.01 ulp of exp on [-87, 0] (CUDA's expf, which the reference calls, is specified to
    2 ulp) and 0 below -104."""
    from oracle.oracle import splat_exp
    xs = np.concatenate([np.linspace(-87.0, 0.0, 1 << 22, dtype=np.float64).astype(np.float32),
                         np.float32(-5.54) + np.arange(-2000, 2000, dtype=np.float32) * 1e-6])
    f = splat_exp(xs)
    e = np.exp(xs.astype(np.float64))
    ulp = np.spacing(e.astype(np.float32)).astype(np.float64)
    assert float(np.max(np.abs(f - e) / ulp)) <= 1.02
    assert np.mean(f == e.astype(np.float32)) > 0.9  # ~90.6 % correctly rounded
    assert np.all(splat_exp(np.array([-104.5, -1e30, -np.inf], np.float32)) == 0.0)
