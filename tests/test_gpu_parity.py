"""HIP path (libgsr.so through the drop-in diff_gaussian_rasterization API) vs the CPU oracle.

Tolerances: the library and the oracle evaluate the same float32 expressions in the same order
(-ffp-contract=off on both sides) and the same exp for the blend weights (splat_exp), so every
alpha / transmittance decision agrees; images are compared at atol 1e-5 (north_star: <= 1e-5).  Backward gradients are summed
with float atomics in a different order than the oracle's sequential loop, so they are compared
as max|gpu - oracle| / max|oracle| <= 1e-5 per tensor.  Integer outputs (radii, num_rendered,
sort results) must match exactly.
"""
import math

import numpy as np
import pytest
import torch

from oracle.oracle import OracleRaster, mark_visible as oracle_mark_visible
from scenes import scene, to_torch_call

pytestmark = pytest.mark.gpu

FWD_ATOL = 1e-5
GRAD_REL = 1e-5


def run_gpu(kw, grads=None, bwd=True):
    from diff_gaussian_rasterization import GaussianRasterizer
    settings, inp = to_torch_call(kw)
    rast = GaussianRasterizer(settings)
    outs = rast(means3D=inp["means3D"], means2D=inp["means2D"], opacities=inp["opacities"],
                shs=inp.get("shs"), colors_precomp=inp.get("colors_precomp"),
                scales=inp.get("scales"), rotations=inp.get("rotations"),
                cov3D_precomp=inp.get("cov3D_precomp"), shs_language=inp.get("shs_language"),
                language_feature_precomp=inp.get("language_feature_precomp"))
    color, depth, alpha, feature, radii = outs
    res = dict(color=color.detach().cpu().numpy(), depth=depth.detach().cpu().numpy(),
               alpha=alpha.detach().cpu().numpy(), feature=feature.detach().cpu().numpy(),
               radii=radii.cpu().numpy())
    if bwd and grads is not None:
        dimg, ddep, dalp, dfea = [None if g is None else torch.tensor(g, device="cuda") for g in grads]
        loss = (color * dimg).sum()
        if ddep is not None:
            loss = loss + (depth * ddep).sum()
        if dalp is not None:
            loss = loss + (alpha * dalp).sum()
        if dfea is not None and kw["include_feature"]:
            loss = loss + (feature * dfea).sum()
        loss.backward()
        res["grads"] = {k: (None if v.grad is None else v.grad.detach().cpu().numpy())
                        for k, v in inp.items()}
    torch.cuda.synchronize()
    return res


GRAD_MAP = [("means3D", "means3D"), ("means2D", "means2D"), ("opacity", "opacities"),
            ("colors", "colors_precomp"), ("sh", "shs"), ("scales", "scales"),
            ("rotations", "rotations"), ("cov3D", "cov3D_precomp"), ("sh_language", "shs_language"),
            ("language_feature", "language_feature_precomp")]


def compare(kw, with_bwd=True, seed=5, extra_grads=True):
    H, W = kw["image_height"], kw["image_width"]
    rng = np.random.default_rng(seed)
    dimg = rng.standard_normal((3, H, W)).astype(np.float32)
    ddep = rng.standard_normal((1, H, W)).astype(np.float32) * 0.3 if extra_grads else None
    dalp = rng.standard_normal((1, H, W)).astype(np.float32) if extra_grads else None
    dfea = rng.standard_normal((3, H, W)).astype(np.float32) if extra_grads else None
    orc = OracleRaster(**kw)
    gpu = run_gpu(kw, (dimg, ddep, dalp, dfea), bwd=with_bwd)
    np.testing.assert_array_equal(gpu["radii"], orc.radii)
    for name in ("color", "depth", "alpha", "feature"):
        np.testing.assert_allclose(gpu[name], getattr(orc, name), atol=FWD_ATOL, rtol=0,
                                   err_msg=name)
    if not with_bwd:
        return orc, gpu
    og = orc.backward(dimg, ddep, dalp, dfea if kw["include_feature"] else None)
    checked = 0
    for oname, iname in GRAD_MAP:
        if og.get(oname) is None or iname not in gpu["grads"]:
            continue
        got = gpu["grads"][iname].reshape(og[oname].shape)
        ref = og[oname]
        scale = max(float(np.abs(ref).max()), 1e-6)
        err = float(np.abs(got - ref).max()) / scale
        assert err <= GRAD_REL, f"{iname}: rel err {err:.2e} (scale {scale:.2e})"
        checked += 1
    assert checked >= 5
    return orc, gpu


CONFIGS = [
    dict(P=64, W=64, H=48, mode="sh", cov_mode="scale_rot", feature="sh"),
    dict(P=1024, W=97, H=61, mode="sh", cov_mode="scale_rot", feature="sh"),
    dict(P=1024, W=97, H=61, mode="colors", cov_mode="scale_rot", feature="precomp"),
    dict(P=1024, W=64, H=48, mode="sh", cov_mode="cov3D", feature=None),
    dict(P=4096, W=128, H=96, mode="colors", cov_mode="cov3D", feature="sh", bg=(0, 0, 0)),
    dict(P=4096, W=200, H=120, mode="sh", cov_mode="scale_rot", feature="sh", active_degree=1),
    dict(P=1, W=64, H=48, mode="sh", cov_mode="scale_rot", feature="sh", cam=0),
    dict(P=2000, W=64, H=48, mode="sh", cov_mode="scale_rot", feature="sh", scale_mult=6.0),
]


@pytest.mark.parametrize("i", range(len(CONFIGS)))
def test_forward_backward_parity(i):
    compare(scene(seed=i, **CONFIGS[i]))


def test_parity_without_extra_upstream_grads():
    compare(scene(P=2048, W=96, H=80, seed=9, feature="sh"), extra_grads=False)


def test_confidence_parity():
    P = 1024
    conf = np.random.default_rng(0).uniform(0.2, 1.0, P)
    compare(scene(P=P, W=80, H=64, seed=4, confidence=conf))


@pytest.mark.parametrize("det", [False, True])
def test_C_shim_matches_oracle_vanilla_api(det):
    """The `_C`-compatible shim with the reference's exact pybind signatures
    (rasterize_points.cu:35-55, 117-140): forward tuple and the 8 backward grads.  det: the
    deterministic backward, switched off again between forward and backward (the shim keeps the
    forward's mode for its backward)."""
    import diff_gaussian_rasterization as dgr
    from diff_gaussian_rasterization import _C
    kw = scene(P=3000, W=97, H=61, seed=8, mode="sh", cov_mode="scale_rot", feature=None)
    d = lambda x: torch.tensor(np.asarray(x), device="cuda")  # noqa: E731
    E = torch.Tensor([]).cuda()
    P = kw["means3D"].shape[0]
    prev = dgr.deterministic()
    dgr.deterministic(det)
    try:
        num_rendered, color, radii, geom, binning, img = _C.rasterize_gaussians(
            d(kw["bg"]), d(kw["means3D"]), E, d(kw["opacities"]).view(P, 1), d(kw["scales"]),
            d(kw["rotations"]), 1.0, E, d(kw["viewmatrix"]), d(kw["projmatrix"]), kw["tanfovx"],
            kw["tanfovy"], kw["image_height"], kw["image_width"], d(kw["shs"]), kw["sh_degree"],
            d(kw["campos"]), False, False)
    finally:
        dgr.deterministic(prev)
    orc = OracleRaster(**kw)
    assert num_rendered > 0
    np.testing.assert_array_equal(radii.cpu().numpy(), orc.radii)
    np.testing.assert_allclose(color.cpu().numpy(), orc.color, atol=FWD_ATOL, rtol=0)
    dpix = np.random.default_rng(3).standard_normal(orc.color.shape).astype(np.float32)
    grads = _C.rasterize_gaussians_backward(
        d(kw["bg"]), d(kw["means3D"]), radii, E, d(kw["scales"]), d(kw["rotations"]), 1.0, E,
        d(kw["viewmatrix"]), d(kw["projmatrix"]), kw["tanfovx"], kw["tanfovy"], d(dpix),
        d(kw["shs"]), kw["sh_degree"], d(kw["campos"]), geom, num_rendered, binning, img, False)
    og = orc.backward(dpix, None, None, None)
    names = ["means2D", "colors", "opacity", "means3D", "cov3D", "sh", "scales", "rotations"]
    for n, g in zip(names, grads):
        ref = og[n]
        got = g.cpu().numpy().reshape(ref.shape)
        err = float(np.abs(got - ref).max()) / max(float(np.abs(ref).max()), 1e-6)
        assert err <= GRAD_REL, (n, err)


def test_empty_scene_returns_zero_images():
    kw = scene(P=1, W=32, H=16)
    for k in ("means3D", "shs", "scales", "rotations", "shs_language"):
        kw[k] = kw[k][:0]
    kw["opacities"] = kw["opacities"][:0]
    gpu = run_gpu(kw, bwd=False)
    assert np.all(gpu["color"] == 0) and gpu["radii"].shape == (0,)


def test_mark_visible_parity():
    from diff_gaussian_rasterization import mark_visible
    kw = scene(P=5000, W=64, H=48, cam=2)
    xyz = kw["means3D"].copy()
    xyz[::7, 2] = -3.95  # behind the near plane of the jittered camera
    got = mark_visible(torch.tensor(xyz, device="cuda"), torch.tensor(kw["viewmatrix"], device="cuda"),
                       torch.tensor(kw["projmatrix"], device="cuda")).cpu().numpy()
    np.testing.assert_array_equal(got, oracle_mark_visible(xyz, kw["viewmatrix"], kw["projmatrix"]))


def test_forward_is_deterministic():
    kw = scene(P=20000, W=160, H=120, seed=2)
    a = run_gpu(kw, bwd=False)
    b = run_gpu(kw, bwd=False)
    for name in ("color", "depth", "alpha", "feature", "radii"):
        np.testing.assert_array_equal(a[name], b[name])


@pytest.mark.parametrize("n,bits,kind", [(1, 8, "int"), (4095, 13, "int"), (4097, 32, "int"),
                                         (1_000_003, 32, "int"), (3_000_000, 13, "int"),
                                         (8191, 4, "int"), (1_000_000, 32, "depth"),
                                         (1_000_000, 32, "depth_narrow"),
                                         (2_500_000, 12, "tiles"),
                                         # even digit splits: 17 bits = 6 + 6 + 5, 20 = 7 + 7 + 6
                                         (300_001, 17, "int"), (65_537, 20, "int")])
def test_radix_sort_sorted_and_stable(n, bits, kind):
    """One-sweep radix sort (gsr_sort.hip) == numpy's stable argsort, bit for bit: full 32-bit
    keys, float-bit depth keys (shared top bytes), skewed tile ids, partial last partitions."""
    from gsr_amd import _lib
    L = _lib.load()
    rng = np.random.default_rng(n)
    if kind == "depth":
        keys = rng.lognormal(1.0, 0.5, size=n).astype(np.float32).view(np.uint32) + 0
    elif kind == "depth_narrow":  # constant top byte: that pass is a copy
        keys = rng.uniform(3.0, 5.0, size=n).astype(np.float32).view(np.uint32) + 0
    elif kind == "tiles":
        keys = np.minimum(rng.exponential(300.0, size=n), (1 << bits) - 1).astype(np.uint32)
    else:
        keys = rng.integers(0, 1 << bits, size=n, dtype=np.uint64).astype(np.uint32)
    keys[: n // 3] = keys[0]  # many ties
    vals = np.arange(n, dtype=np.uint32)
    k = torch.tensor(keys.view(np.int32), device="cuda")
    v = torch.tensor(vals.view(np.int32), device="cuda")
    scratch = torch.empty(int(L.gsr_test_sort_scratch_bytes(n)), dtype=torch.uint8, device="cuda")
    _lib.check(L.gsr_test_radix_sort_pairs(k.data_ptr(), v.data_ptr(), n, bits, scratch.data_ptr(),
                                           torch.cuda.current_stream().cuda_stream))
    order = np.argsort(keys, kind="stable")
    np.testing.assert_array_equal(k.cpu().numpy().view(np.uint32), keys[order])
    np.testing.assert_array_equal(v.cpu().numpy().view(np.uint32), vals[order])


@pytest.mark.gpu
def test_radix_sort_concurrent_streams():
    """Several one-sweep sorts in flight at once on separate streams (as the view streams and two
    processes on one GPU produce): the look-back must never wait on a partition that cannot be
    dispatched (ticketed partitions, gsr_sort.hip), so every sort completes without the look-back
    timeout and matches numpy's stable argsort.  (Correctness under overlap only: the blockIdx
    variant, GSR_SORT_TICKET=0, also passes this in one process; its failure was seen with two
    processes sharing the GPU, scripts/dist_rehearsal.sh.)"""
    import threading
    from gsr_amd import _lib
    L = _lib.load()
    n, nthreads, reps = 3_000_000, 4, 6
    rng = np.random.default_rng(7)
    keys = [rng.lognormal(1.0, 0.5, size=n).astype(np.float32).view(np.uint32) + 0
            for _ in range(nthreads)]
    orders = [np.argsort(k, kind="stable") for k in keys]
    dev = [(torch.tensor(k.view(np.int32), device="cuda"),
            torch.empty(n, dtype=torch.int32, device="cuda"),
            torch.empty(int(L.gsr_test_sort_scratch_bytes(n)), dtype=torch.uint8, device="cuda"),
            torch.cuda.Stream()) for k in keys]
    torch.cuda.synchronize()
    errors = []

    def worker(i):
        k0, v, scratch, s = dev[i]
        try:
            for _ in range(reps):
                k = k0.clone()
                v.copy_(torch.arange(n, dtype=torch.int32, device="cuda"))
                torch.cuda.synchronize()
                rc = L.gsr_test_radix_sort_pairs(k.data_ptr(), v.data_ptr(), n, 32,
                                                 scratch.data_ptr(), s.cuda_stream)
                if rc != 0:
                    errors.append((i, rc, L.gsr_last_error()))
                    return
                s.synchronize()
                got = v.cpu().numpy().view(np.uint32)
                if not np.array_equal(got, orders[i].astype(np.uint32)):
                    errors.append((i, "order mismatch"))
                    return
        except Exception as e:  # surfaced below
            errors.append((i, repr(e)))

    threads = [threading.Thread(target=worker, args=(i,)) for i in range(nthreads)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=100)
    assert not any(t.is_alive() for t in threads), "a sort thread did not finish"
    assert not errors, errors


@pytest.mark.parametrize("n,frac_culled", [(1_000_000, 0.0), (1_000_000, 0.2), (70_001, 0.5),
                                           (4097, 1.0)])
def test_radix_sort_sentinel_copy_pass(n, frac_culled):
    """Depth-sort mode: culled keys (0xffffffff) may land anywhere; every other key must be in
    stable sorted order.  Depths in [3, 5) share their top byte, so that pass is a plain copy."""
    from gsr_amd import _lib
    L = _lib.load()
    rng = np.random.default_rng(n)
    keys = rng.uniform(3.0, 5.0, size=n).astype(np.float32).view(np.uint32) + 0
    keys[: n // 4] = keys[0]  # ties
    culled = rng.random(n) < frac_culled
    keys[culled] = 0xFFFFFFFF
    vals = np.arange(n, dtype=np.uint32)
    k = torch.tensor(keys.view(np.int32), device="cuda")
    v = torch.tensor(vals.view(np.int32), device="cuda")
    scratch = torch.empty(int(L.gsr_test_sort_scratch_bytes(n)), dtype=torch.uint8, device="cuda")
    _lib.check(L.gsr_test_radix_sort_pairs_sentinel(k.data_ptr(), v.data_ptr(), n, 32,
                                                    scratch.data_ptr(),
                                                    torch.cuda.current_stream().cuda_stream))
    gk = k.cpu().numpy().view(np.uint32)
    gv = v.cpu().numpy().view(np.uint32)
    np.testing.assert_array_equal(np.sort(gv), vals)          # a permutation
    np.testing.assert_array_equal(gk, keys[gv])                # pairs travel together
    keep = ~culled[gv]
    order = np.argsort(keys, kind="stable")
    order = order[~culled[order]]
    np.testing.assert_array_equal(gv[keep], order)


@pytest.mark.parametrize("n,kind,frac_culled", [
    (1_000_000, "narrow", 0.2),   # constant top byte: 3 of 4 passes run
    (1_000_000, "wide", 0.0),     # every pass runs
    (70_001, "const", 0.3),       # one distinct real key: only the last pass runs (a copy)
    (4097, "narrow", 1.0),        # every key a sentinel
    (2_000_003, "mid", 0.1)])     # constant second byte too: passes 0 and 3 skipped?
def test_radix_sort_planned(n, kind, frac_culled):
    """The depth sort's planned form (gsr_sort.hip radix_planned_kernel): passes whose digit is
    constant over the non-sentinel keys do not run, the rest alternate so that the result lands
    in the fixed output pair -- the same keys and values as the unplanned sort, bit for bit, and
    the non-sentinel keys in stable sorted order."""
    from gsr_amd import _lib
    L = _lib.load()
    rng = np.random.default_rng(n + len(kind))
    if kind == "narrow":
        keys = rng.uniform(3.0, 5.0, size=n).astype(np.float32).view(np.uint32) + 0
    elif kind == "wide":
        keys = rng.lognormal(1.0, 2.0, size=n).astype(np.float32).view(np.uint32) + 0
    elif kind == "const":
        keys = np.full(n, 0x40400000, np.uint32)
    else:  # two middle bytes constant, low and high bytes varying
        keys = (rng.integers(0, 256, size=n, dtype=np.uint32) |
                (rng.integers(0, 64, size=n, dtype=np.uint32) << 24) | 0x00ABCD00).astype(np.uint32)
    keys[: n // 5] = keys[0]
    culled = rng.random(n) < frac_culled
    keys[culled] = 0xFFFFFFFF
    vals = np.arange(n, dtype=np.uint32)
    scratch = torch.empty(int(L.gsr_test_sort_scratch_bytes(n)), dtype=torch.uint8, device="cuda")
    out = []
    for planned in (False, True):
        k = torch.tensor(keys.view(np.int32), device="cuda")
        v = torch.tensor(vals.view(np.int32), device="cuda")
        st = torch.cuda.current_stream().cuda_stream
        if planned:
            rc = L.gsr_test_radix_sort_pairs_planned(k.data_ptr(), v.data_ptr(), n, 32, 1,
                                                     scratch.data_ptr(), st)
        else:
            rc = L.gsr_test_radix_sort_pairs_sentinel(k.data_ptr(), v.data_ptr(), n, 32,
                                                      scratch.data_ptr(), st)
        _lib.check(rc)
        out.append((k.cpu().numpy().view(np.uint32), v.cpu().numpy().view(np.uint32)))
    np.testing.assert_array_equal(out[0][0], out[1][0])
    np.testing.assert_array_equal(out[0][1], out[1][1])
    gv = out[1][1]
    keep = ~culled[gv]
    order = np.argsort(keys, kind="stable")
    np.testing.assert_array_equal(gv[keep], order[~culled[order]])
    # without sentinels the planned sort is a full stable sort too
    if frac_culled == 0.0:
        k = torch.tensor(keys.view(np.int32), device="cuda")
        v = torch.tensor(vals.view(np.int32), device="cuda")
        _lib.check(L.gsr_test_radix_sort_pairs_planned(k.data_ptr(), v.data_ptr(), n, 32, 0,
                                                       scratch.data_ptr(),
                                                       torch.cuda.current_stream().cuda_stream))
        np.testing.assert_array_equal(v.cpu().numpy().view(np.uint32), order)


@pytest.mark.parametrize("n", [1, 2047, 2049, 5_000_001])
def test_scan(n):
    from gsr_amd import _lib
    L = _lib.load()
    x = np.random.default_rng(n).integers(0, 50, size=n).astype(np.uint32)
    xi = torch.tensor(x.view(np.int32), device="cuda")
    out = torch.empty_like(xi)
    scratch = torch.empty(int(L.gsr_test_scan_scratch_bytes(n)), dtype=torch.uint8, device="cuda")
    for inclusive in (1, 0):
        _lib.check(L.gsr_test_scan(xi.data_ptr(), out.data_ptr(), n, inclusive, scratch.data_ptr(),
                                   torch.cuda.current_stream().cuda_stream))
        c = np.cumsum(x, dtype=np.uint64).astype(np.uint32)
        ref = c if inclusive else np.concatenate([[0], c[:-1]]).astype(np.uint32)
        np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), ref)


@pytest.mark.parametrize("n,views", [(1, 1), (2049, 3), (1_000_000, 3), (5_000_001, 2)])
def test_scan_lookback(n, views):
    """The batched forward's single-pass look-back scan (gsr_sort.hip scan_lookback_views_kernel,
    several views per launch, ticketed partitions) == numpy's inclusive cumsum of every view."""
    from gsr_amd import _lib
    L = _lib.load()
    x = np.random.default_rng(n + views).integers(0, 50, size=views * n).astype(np.uint32)
    xi = torch.tensor(x.view(np.int32), device="cuda")
    out = torch.empty_like(xi)
    words = int(L.gsr_test_scan_lookback_words(n))
    scratch = torch.empty(views * words * 8 + 16, dtype=torch.uint8, device="cuda")
    _lib.check(L.gsr_test_scan_lookback(xi.data_ptr(), out.data_ptr(), n, views,
                                        scratch.data_ptr(), torch.cuda.current_stream().cuda_stream))
    ref = np.cumsum(x.reshape(views, n), axis=1, dtype=np.uint64).astype(np.uint32)
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32).reshape(views, n), ref)


def test_splat_exp_is_the_oracles_exp():
    """The blends' exp(power) (gsr_device.h splat_exp) is bit-identical to the oracle's
    (oracle/gsr_oracle.c splat_exp) -- so GPU and oracle take the same alpha >= 1/255 and
    T < 1e-4 decisions -- on every 5th float of [-6, 0) (the alpha-relevant range), every float of
    [-5.6, -5.5] (around ln(1/255)) and a 2^24-point sweep of [-87, 0]; it is within 1.01 ulp of
    exp there (OCML's expf is also checked against the same bound) and 0 below -104."""
    from gsr_amd import _lib
    from oracle.oracle import splat_exp
    L = _lib.load()
    lo = np.float32(-6.0)
    a = np.arange(np.float32(-2.0 ** -20).view(np.uint32), lo.view(np.uint32) + 1, 5, dtype=np.uint32)
    c = np.arange(np.float32(-5.5).view(np.uint32), np.float32(-5.6).view(np.uint32) + 1,
                  dtype=np.uint32)
    sweep = np.linspace(-87.0, 0.0, 1 << 24, dtype=np.float64).astype(np.float32)
    xs = np.concatenate([a.view(np.float32), c.view(np.float32), sweep,
                         np.array([0.0, -0.0, -87.3, -103.9, -104.0, -104.5, -1e30, -np.inf],
                                  np.float32)]).astype(np.float32)
    x = torch.tensor(xs, device="cuda")
    ref, fast = torch.empty_like(x), torch.empty_like(x)
    _lib.check(L.gsr_test_expf_pair(x.data_ptr(), ref.data_ptr(), fast.data_ptr(), x.numel(),
                                    torch.cuda.current_stream().cuda_stream))
    f = fast.cpu().numpy()
    o = splat_exp(xs)
    bad = np.nonzero(f.view(np.uint32) != o.view(np.uint32))[0]
    assert bad.size == 0, (xs[bad[:5]], f[bad[:5]], o[bad[:5]])
    m = xs >= -87.0
    e = np.exp(xs[m].astype(np.float64))
    ulp = np.spacing(e.astype(np.float32)).astype(np.float64)
    assert float(np.max(np.abs(f[m] - e) / ulp)) <= 1.02
    assert float(np.max(np.abs(ref.cpu().numpy()[m] - e) / ulp)) <= 1.02
    assert np.all(f[xs < -104.0] == 0.0)


@pytest.mark.parametrize("P,W,H", [(100_000, 800, 800)])
def test_config2_full_size_parity(P, W, H):
    """BASELINE config 2 at full size (100k Gaussians, 800x800, SH degree 3), fwd + bwd."""
    compare(scene(P=P, W=W, H=H, seed=0, cam=0, mode="sh", feature="sh"))


def test_config3_full_size_forward_parity():
    """BASELINE config 3 scale (1M Gaussians, 1008x756): forward parity vs the oracle."""
    kw = scene(P=1_000_000, W=1008, H=756, seed=0, cam=1, mode="sh", feature="sh")
    compare(kw, with_bwd=False)


def test_backward_twice_through_one_forward():
    """retain_graph: a second backward through the same forward gives the same gradients (the
    accumulators zeroed by the forward's preprocess are used once; the second backward clears
    them itself)."""
    from diff_gaussian_rasterization import GaussianRasterizer
    kw = scene(P=3000, W=97, H=61, seed=4)
    settings, inp = to_torch_call(kw)
    color, depth, _, _, _ = GaussianRasterizer(settings)(
        means3D=inp["means3D"], means2D=inp["means2D"], opacities=inp["opacities"],
        shs=inp.get("shs"), colors_precomp=inp.get("colors_precomp"), scales=inp.get("scales"),
        rotations=inp.get("rotations"), cov3D_precomp=inp.get("cov3D_precomp"))
    g = torch.randn(color.shape, device="cuda", generator=torch.Generator("cuda").manual_seed(0))
    loss = (color * g).sum() + depth.sum()
    first = torch.autograd.grad(loss, [inp["means3D"], inp["opacities"]], retain_graph=True)
    second = torch.autograd.grad(loss, [inp["means3D"], inp["opacities"]])
    for a, b in zip(first, second):
        # float atomics: two backwards differ in the last bits (as the reference's); a stale or
        # doubled accumulator would differ by whole gradients
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6 * float(b.abs().max()))
