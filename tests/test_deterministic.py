"""Deterministic backward (diff_gaussian_rasterization.deterministic, include/gsr.h
GSR_DEBUG_DETERMINISTIC; SURVEY.md section 5 "optional deterministic mode: per-tile partials +
segmented reduce").  The reference's blend backward adds with unordered float atomics
(backward.cu:523-554), so two runs of the same backward differ in the last bits; in this mode the
gradients of repeated runs are bitwise equal, the forward outputs are those of the default mode,
and the gradients stay within the default mode's oracle tolerance (same scale-relative 1e-5 the
parity tests use; the default mode is pinned to the oracle in test_fused_parity / test_gpu_parity).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


class _Pipe:
    convert_SHs_python = True
    compute_cov3D_python = False
    debug = False
    use_confidence = False


class _Opt:
    include_feature = True


def _scene(n=30_000, W=320, H=240, views=3):
    from gsr_amd.model import SplatModel
    from gsr_amd.synthetic import make_cameras, make_gaussians, upstream_grads
    dev = torch.device("cuda", 0)
    model = SplatModel(make_gaussians(n, sh_degree=3, seed=11), device=dev)
    cams = [c.to(dev) for c in make_cameras(views, W, H, seed=12)]
    return model, cams, upstream_grads(H, W, seed=13, device=dev)


def _run(model, cams, grads, det, fused=True, streams=1):
    """One multi-view step (render + backward of fixed upstream gradients per view); returns the
    forward images of the first view and every parameter's gradient."""
    import diff_gaussian_rasterization as dgr
    from gaussian_renderer import render
    from gsr_amd.pipeline import ViewPipeline
    prev_det = dgr.deterministic()
    dgr.deterministic(det)
    dimg, ddep, dfeat = grads
    bg = torch.zeros(3, device=dimg.device)
    outs = []

    def one_view(cam):
        pkg = render(cam, model, _Pipe(), bg, _Opt())
        if not outs:
            outs.extend(t.detach().clone() for t in (pkg["render"], pkg["depth"], pkg["feature"]))
        torch.autograd.backward([pkg["render"], pkg["depth"], pkg["feature"]], [dimg, ddep, dfeat])

    try:
        for p in model.parameters():
            p.grad = None
        if fused:
            ViewPipeline(dimg.device, depth=streams).run(cams, one_view, model=model)
        else:
            for cam in cams:
                one_view(cam)
        torch.cuda.synchronize()
    finally:
        dgr.deterministic(prev_det)
    return outs, [p.grad.detach().clone() for p in model.parameters()]


@pytest.mark.parametrize("fused,streams", [(True, 1), (True, 2), (False, 1)])
def test_deterministic_backward_is_bitwise_reproducible(fused, streams, monkeypatch):
    import diff_gaussian_rasterization as dgr
    if not fused:
        monkeypatch.setenv("GSR_FUSED", "0")
    model, cams, grads = _scene()
    prev = dgr.grad_into_leaves()
    dgr.grad_into_leaves(fused)
    try:
        out_a, g_a = _run(model, cams, grads, True, fused, streams)
        out_b, g_b = _run(model, cams, grads, True, fused, streams)
        out_d, g_d = _run(model, cams, grads, False, fused, streams)
    finally:
        dgr.grad_into_leaves(prev)
    for x, y, z in zip(out_a, out_b, out_d):
        assert torch.equal(x, y) and torch.equal(x, z)  # the forward does not depend on the mode
    for p, a, b, d in zip(model.parameters(), g_a, g_b, g_d):
        assert torch.equal(a, b), tuple(p.shape)
        scale = float(d.abs().max())
        assert float((a - d).abs().max()) <= 1e-5 * scale + 1e-30, tuple(p.shape)
    assert any(float(d.abs().max()) > 0 for d in g_d)


def test_deterministic_backward_full_size_rows():
    """Bench-sized view (1008x756, 200k Gaussians): every instance row of the binning buffer is
    written (replayed rows and the zero rows behind each tile's last contributor), so repeated
    runs agree bitwise and match the default mode at its tolerance."""
    import diff_gaussian_rasterization as dgr
    model, cams, grads = _scene(n=200_000, W=1008, H=756, views=1)
    prev = dgr.grad_into_leaves()
    dgr.grad_into_leaves(True)
    try:
        _, g_a = _run(model, cams, grads, True)
        _, g_b = _run(model, cams, grads, True)
        _, g_d = _run(model, cams, grads, False)
    finally:
        dgr.grad_into_leaves(prev)
    _, g_e = _run(model, cams, grads, False)
    differ = sum(int((d != e).sum()) for d, e in zip(g_d, g_e))
    print(f"default mode: {differ} gradient elements differ between two runs")
    for a, b, d in zip(g_a, g_b, g_d):
        assert torch.equal(a, b)
        assert float((a - d).abs().max()) <= 1e-5 * float(d.abs().max()) + 1e-30


def test_C_backward_takes_the_layout_from_the_binning_buffer():
    """the reference-signature `_C` backward (only `debug` travels with the buffers)
    uses the layout its forward wrote into the binning buffer's tag word, whatever the global
    deterministic() mode is at backward time: a deterministic forward's backward stays bitwise
    reproducible after the mode was switched off, a default forward's backward runs its atomic
    layout after the mode was switched on, and a buffer without the tag is refused."""
    import numpy as np
    import diff_gaussian_rasterization as dgr
    from diff_gaussian_rasterization import _C
    from gsr_amd import _lib
    from scenes import scene
    kw = scene(P=40_000, W=320, H=240, seed=3, mode="sh", feature=None)
    d = lambda x: torch.tensor(np.asarray(x), device="cuda")  # noqa: E731
    E = torch.Tensor([]).cuda()
    P = kw["means3D"].shape[0]

    def fwd():
        return _C.rasterize_gaussians(
            d(kw["bg"]), d(kw["means3D"]), E, d(kw["opacities"]).view(P, 1), d(kw["scales"]),
            d(kw["rotations"]), 1.0, E, d(kw["viewmatrix"]), d(kw["projmatrix"]), kw["tanfovx"],
            kw["tanfovy"], kw["image_height"], kw["image_width"], d(kw["shs"]), kw["sh_degree"],
            d(kw["campos"]), False, False)

    def bwd(f, dpix, binning=None):
        nr, color, radii, geom, b, img = f
        g = _C.rasterize_gaussians_backward(
            d(kw["bg"]), d(kw["means3D"]), radii, E, d(kw["scales"]), d(kw["rotations"]), 1.0, E,
            d(kw["viewmatrix"]), d(kw["projmatrix"]), kw["tanfovx"], kw["tanfovy"], dpix,
            d(kw["shs"]), kw["sh_degree"], d(kw["campos"]), geom, nr, b if binning is None else binning,
            img, False)
        torch.cuda.synchronize()
        return g

    prev = dgr.deterministic()
    try:
        dgr.deterministic(True)
        f_det = fwd()
        dgr.deterministic(False)
        f_std = fwd()
        dpix = torch.randn_like(f_det[1])
        a, b = bwd(f_det, dpix), bwd(f_det, dpix)  # mode off now: the buffer says deterministic
        for x, y in zip(a, b):
            assert torch.equal(x, y)
        dgr.deterministic(True)
        c = bwd(f_std, dpix)  # mode on now: the buffer says atomics
        for x, y in zip(a, c):
            assert float((x - y).abs().max()) <= 1e-5 * float(y.abs().max()) + 1e-30
        # a buffer large enough for either layout is identified by its tag: junk is refused
        junk = torch.zeros_like(f_det[4])
        with pytest.raises(_lib.GsrError, match="binningBuffer"):
            bwd(f_std, dpix, binning=junk)
        # a buffer too small for R instances is refused on the host (no device read)
        with pytest.raises(RuntimeError, match="binningBuffer"):
            bwd(f_std, dpix, binning=f_std[4][: f_std[4].numel() // 2])
    finally:
        dgr.deterministic(prev)
