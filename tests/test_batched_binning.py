"""The multi-view call's batched forward (gsr_api.cpp views_forward_batched): the views' preprocesses in one multi-view launch, then one launch per
binning stage for a group of views (instance-count sums with the pinned read-back, depth-sort
passes, scan, duplication, tile-sort passes, ranges, schedules, blend).  The forward has no float
atomics, so every view's images, radii and instance counts must be bitwise those of the
single-view call (render() per camera, reference path rasterizer_impl.cu:200-340) -- including a
view that sees no Gaussian (R = 0 inside a batch), a view count the groups do not divide evenly,
and one view alone."""
import numpy as np
import pytest
import torch

from fused_ref import IMAGES, Opt, Pipe
from gsr_amd.camera import look_at_R, make_camera
from gsr_amd.model import SplatModel
from gsr_amd.synthetic import make_cameras, make_gaussians

pytestmark = pytest.mark.gpu


def _away_camera(W, H, like):
    """A camera at (0, 0, -4) looking away from the scene: every Gaussian behind its near plane."""
    c = np.array([0.0, 0.0, -4.0])
    R = look_at_R(c, target=np.array([0.0, 0.0, -8.0]))
    return make_camera(R, -R.T @ c, like.FoVx, like.FoVy, W, H, uid=99, device="cuda")


def _batched_vs_single(m, cams):
    import diff_gaussian_rasterization as dgr
    from gaussian_renderer import render, render_views
    bg = torch.zeros(3, device="cuda")
    streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(2)]
    pkgs = render_views(cams, m, Pipe(), bg, Opt(), streams=streams)
    counts = list(dgr.LAST_STATS["view_counts"])
    multi = [{k: p[k].detach().clone() for k in IMAGES + ("radii",)} for p in pkgs]
    del pkgs
    torch.cuda.synchronize()
    assert len(counts) == len(cams)
    for v, cam in enumerate(cams):
        one = render(cam, m, Pipe(), bg, Opt())
        torch.cuda.synchronize()
        assert counts[v] == (dgr.LAST_STATS["num_rendered"], dgr.LAST_STATS["num_instances"]), v
        for k in IMAGES + ("radii",):
            assert torch.equal(multi[v][k], one[k].detach()), (v, k)
    return counts


def test_batched_forward_wide_ids_equals_single_view():
    """Ids too wide to share a 32-bit word with a tile id or a tile count (2048x2048: 16384 tiles,
    300k Gaussians > 2^18 and 2^17): the batched forward falls back to the pair tile sort and the
    gathered depth-sort payload (gsr_api.cpp phase 1 / 2a), still bitwise the single-view call."""
    W = H = 2048
    tiles = (W // 16) * (H // 16)
    P = 300_000
    assert P > 1 << (32 - (tiles - 1).bit_length()) and P > 1 << (32 - tiles.bit_length())
    m = SplatModel(make_gaussians(P, sh_degree=3, seed=7), device="cuda")
    cams = [c.to("cuda") for c in make_cameras(2, W, H, seed=7)]
    counts = _batched_vs_single(m, cams)
    assert all(c[1] > 0 for c in counts)


def test_batched_forward_one_tile_image():
    """A 16x12 image is ONE tile: no tile bits, so no keys-only packing (tile << 32 does not fit)
    and no tile sort at all -- the batched forward keeps the duplication's depth order, bitwise the
    single-view call (round 6: it used to pick a 32-bit pack shift and the launch refused it)."""
    W, H = 16, 12
    m = SplatModel(make_gaussians(3_000, sh_degree=3, seed=11), device="cuda")
    cams = [c.to("cuda") for c in make_cameras(3, W, H, seed=11, distance=4.0)]
    counts = _batched_vs_single(m, cams)
    assert any(c[1] > 0 for c in counts)


def test_batched_forward_17_tile_bits():
    """More than 2^16 tiles (4128x4096: 258 x 256 = 66048 tiles, 17 tile bits, 3 tile-sort passes):
    the duplication does not count the tile sort's digit totals (its LDS histogram holds two
    passes), the tile sort runs its own totals launch -- still bitwise the single-view call."""
    W, H = 4128, 4096
    assert ((W // 16) * (H // 16) - 1).bit_length() == 17
    m = SplatModel(make_gaussians(20_000, sh_degree=3, seed=17), device="cuda")
    cams = [c.to("cuda") for c in make_cameras(2, W, H, seed=17)]
    counts = _batched_vs_single(m, cams)
    assert all(c[1] > 0 for c in counts)


@pytest.mark.parametrize("nviews,distance", [(1, 4.0), (7, 4.0), (10, 4.0), (5, 1.6)])
def test_batched_forward_equals_single_view(nviews, distance):
    """(distance 4: every binned depth in [2, 8), one top byte -- the batched depth sort leaves its
    last pass out; distance 1.6: depths on both sides of 2 -- all four passes.)"""
    import diff_gaussian_rasterization as dgr
    from gaussian_renderer import render, render_views
    W, H = 240, 180
    m = SplatModel(make_gaussians(30_000, sh_degree=3, seed=5), device="cuda")
    cams = [c.to("cuda") for c in make_cameras(nviews, W, H, seed=5, distance=distance)]
    if nviews > 3:
        cams[3] = _away_camera(W, H, cams[0])
    bg = torch.zeros(3, device="cuda")
    streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(2)]
    pkgs = render_views(cams, m, Pipe(), bg, Opt(), streams=streams)
    counts = list(dgr.LAST_STATS["view_counts"])
    multi = [{k: p[k].detach().clone() for k in IMAGES + ("radii",)} for p in pkgs]
    del pkgs
    torch.cuda.synchronize()
    assert len(counts) == nviews
    for v, cam in enumerate(cams):
        one = render(cam, m, Pipe(), bg, Opt())
        torch.cuda.synchronize()
        assert counts[v] == (dgr.LAST_STATS["num_rendered"], dgr.LAST_STATS["num_instances"]), v
        for k in IMAGES + ("radii",):
            assert torch.equal(multi[v][k], one[k].detach()), (v, k)
    if nviews > 3:
        assert counts[3] == (0, 0)
        assert float(multi[3]["alpha"].abs().max()) == 0.0
        assert counts[0][1] > 0


def test_merged_preprocess_bwd_equals_per_view_launches():
    """The multi-view backward's merged per-Gaussian launch (gsr_backward.hip
    preprocess_bwd_views_kernel: model inputs evaluated once, rows loaded one view ahead,
    per-view gradients summed in registers in view order) against one launch per view on the
    SAME gradient rows (the blend skipped on the repeats, include/gsr_testing.h test bits):
    every leaf gradient and every view's screen-space gradient bitwise equal."""
    import diff_gaussian_rasterization as dgr
    from fused_ref import LEAVES
    from gaussian_renderer import render_views
    from gsr_amd.pipeline import ViewPipeline
    from gsr_amd.synthetic import upstream_grads
    NO_BLEND, PER_VIEW = 256, 512
    W, H = 240, 180
    m = SplatModel(make_gaussians(30_000, sh_degree=3, seed=13), device="cuda")
    cams = [c.to("cuda") for c in make_cameras(3, W, H, seed=13)]
    grads = upstream_grads(H, W, seed=3, device="cuda")
    bg = torch.zeros(3, device="cuda")
    direct = [n for n in LEAVES if n not in ("_features_dc", "_features_rest")]  # SH: deferred
    prev = dgr.grad_into_leaves()
    dgr.grad_into_leaves(True)

    def fn(cs, strs):
        pkgs = render_views(cs, m, Pipe(), bg, Opt(), streams=strs)
        st = pkgs[0]["views"]
        V = len(pkgs)
        seeds = [g.expand(V, *g.shape) for g in grads]
        outs = []
        for bits in (0, NO_BLEND, NO_BLEND | PER_VIEW):
            for n in LEAVES:
                getattr(m, n).grad = None
            st["viewspace_points"].grad = None
            dgr._TEST_BWD_BITS[0] = bits
            torch.autograd.backward([st["render"], st["depth"], st["feature"]], seeds,
                                    retain_graph=True)
            o = {n: getattr(m, n).grad.detach().clone() for n in direct}
            o["means2D"] = st["viewspace_points"].grad.detach().clone()
            outs.append(o)
        return outs

    try:
        vp = ViewPipeline(torch.device("cuda"), depth=3, defer_sh=True, precolor=True)
        merged, merged_again, per_view = vp.run_views(cams, fn, model=m)
        torch.cuda.synchronize()
    finally:
        dgr._TEST_BWD_BITS[0] = 0
        dgr.grad_into_leaves(prev)
    for k in merged:
        assert torch.equal(merged[k], merged_again[k]), k  # the rows survive a backward
        assert torch.equal(merged_again[k], per_view[k]), k
    assert float(merged["_xyz"].abs().max()) > 0.0
