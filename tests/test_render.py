"""render() drop-in (gaussian_renderer/__init__.py:209-338) on the HIP path: the pipeline flags
select equivalent computations, gradients reach every GaussianModel parameter."""
import numpy as np
import pytest
import torch

from gsr_amd.model import SplatModel
from gsr_amd.synthetic import make_cameras, make_gaussians

pytestmark = pytest.mark.gpu


class Pipe:
    def __init__(self, sh_py=True, cov_py=False, conf=False):
        self.convert_SHs_python = sh_py
        self.compute_cov3D_python = cov_py
        self.debug = False
        self.use_confidence = conf


class Opt:
    include_feature = True


def _setup(P=20000, W=200, H=150):
    from gaussian_renderer import render
    m = SplatModel(make_gaussians(P, seed=5), device="cuda")
    cam = make_cameras(3, W, H, seed=1)[2].to("cuda")
    return render, m, cam


def test_render_dict_and_grads():
    render, m, cam = _setup()
    pkg = render(cam, m, Pipe(sh_py=False), torch.zeros(3, device="cuda"), Opt())
    assert set(pkg) == {"render", "depth", "alpha", "opacity", "feature", "viewspace_points",
                        "visibility_filter", "radii", "color"}
    assert pkg["render"].shape == (3, 150, 200) and pkg["depth"].shape == (1, 150, 200)
    loss = pkg["render"].mean() + pkg["depth"].mean() + pkg["feature"].abs().mean()
    loss.backward()
    for p in m.parameters():
        assert p.grad is not None and torch.isfinite(p.grad).all() and p.grad.abs().sum() > 0
    vs = pkg["viewspace_points"].grad
    assert vs is not None and vs[:, :2].abs().sum() > 0 and torch.all(vs[:, 2] == 0)


def test_viewspace_points_are_fresh_zero_leaves_per_view():
    """The fused path's means2D leaves share one cached zero buffer (no fill per view): each view
    still gets its own zero-valued leaf whose .grad holds only that view's screen-space gradient,
    exactly what a fresh zeros_like(..., requires_grad=True) would give."""
    render, m, cam = _setup()
    cams = [cam] + [c.to("cuda") for c in make_cameras(2, 200, 150, seed=9)]
    bg = torch.zeros(3, device="cuda")
    pkgs = [render(c, m, Pipe(sh_py=False), bg, Opt()) for c in cams]
    leaves = [p["viewspace_points"] for p in pkgs]
    assert len({id(t) for t in leaves}) == len(leaves)
    for t in leaves:
        assert t.is_leaf and t.requires_grad and t.grad is None and not torch.any(t)
    sum(p["render"].sum() for p in pkgs).backward()
    for c, p in zip(cams, pkgs):  # each .grad equals the view rendered alone
        m2 = SplatModel(make_gaussians(20000, seed=5), device="cuda")
        q = render(c, m2, Pipe(sh_py=False), bg, Opt())
        q["render"].sum().backward()
        torch.testing.assert_close(p["viewspace_points"].grad, q["viewspace_points"].grad,
                                   atol=1e-5 * float(q["viewspace_points"].grad.abs().max()),
                                   rtol=0)
    assert not torch.any(leaves[0])  # the shared buffer is never written


def test_python_and_kernel_sh_paths_agree(monkeypatch):
    # both sides with torch's activations (the fused path's in-kernel sigmoid differs by ulps)
    monkeypatch.setenv("GSR_FUSED", "0")
    render, m, cam = _setup()
    bg = torch.tensor([0.1, 0.2, 0.3], device="cuda")
    a = render(cam, m, Pipe(sh_py=True), bg, Opt())
    b = render(cam, m, Pipe(sh_py=False), bg, Opt())
    assert torch.equal(a["radii"], b["radii"])
    torch.testing.assert_close(a["render"], b["render"], atol=2e-6, rtol=0)
    torch.testing.assert_close(a["feature"], b["feature"], atol=2e-6, rtol=0)
    torch.testing.assert_close(a["depth"], b["depth"], atol=0, rtol=0)


def test_python_covariance_path_agrees():
    render, m, cam = _setup()
    bg = torch.zeros(3, device="cuda")
    a = render(cam, m, Pipe(sh_py=False, cov_py=False), bg, Opt())
    b = render(cam, m, Pipe(sh_py=False, cov_py=True), bg, Opt())
    same = (a["radii"] == b["radii"]).float().mean().item()
    assert same > 0.999
    assert (a["render"] - b["render"]).abs().mean().item() < 1e-5


def _leaf_grads(m):
    return [p.grad.clone() for p in m.parameters()]


def _zero(m):
    for p in m.parameters():
        p.grad = None


@pytest.mark.parametrize("conf,sh_py", [(False, False), (True, False), (False, True)])
def test_fused_activation_path_matches_unfused(monkeypatch, conf, sh_py):
    """render() -> gsr_rasterize_gaussians_fused (sigmoid / exp / normalize / cat and, for the
    reference's default convert_SHs_python=True, the Python eval_sh colour + language pre-pass,
    all in-kernel) vs GSR_FUSED=0 (the torch getters / eval_sh + gsr_rasterize_gaussians): same
    images, same raw gradients up to the ulp-level difference of torch's vs the kernel's
    arithmetic."""
    import gaussian_renderer as gr
    render, m, cam = _setup()
    if conf:
        gen = torch.Generator(device="cuda").manual_seed(11)
        m.confidence = torch.rand(m.confidence.shape, device="cuda", generator=gen)
    bg = torch.tensor([0.1, 0.2, 0.3], device="cuda")
    pipe = Pipe(sh_py=sh_py, conf=conf)
    assert gr._fused_eligible(m, pipe, Opt(), None, None)
    outs = []
    for fused in ("1", "0"):
        monkeypatch.setenv("GSR_FUSED", fused)
        _zero(m)
        pkg = render(cam, m, pipe, bg, Opt())
        g = torch.Generator(device="cuda").manual_seed(3)
        loss = ((pkg["render"] * torch.rand(pkg["render"].shape, device="cuda", generator=g)).sum()
                + (pkg["depth"] * 0.01).sum() + pkg["alpha"].sum() + pkg["feature"].sum())
        loss.backward()
        outs.append((pkg, _leaf_grads(m), pkg["viewspace_points"].grad.clone()))
    (a, ga, va), (b, gb, vb) = outs
    same = (a["radii"] == b["radii"]).float().mean().item()
    assert same > 0.9999
    for k in ("render", "depth", "alpha", "feature"):
        # an ulp of opacity can move a pair across the alpha >= 1/255 or T >= 1e-4 threshold:
        # allow a handful of such pixels, bounded by one 1/255-weight blend term
        d = (a[k] - b[k]).abs()
        tol = 1e-4 + 1e-4 * b[k].abs()
        assert (d > tol).float().mean().item() < 1e-4, k
        assert d.max().item() < 2e-2 * max(1.0, b[k].abs().max().item()), k
    names = ["xyz", "f_dc", "f_rest", "scaling", "rotation", "opacity", "language"]
    for n, x, y in zip(names, ga, gb):
        scale = y.abs().max().item() + 1e-12
        err = (x - y).abs().max().item() / scale
        assert err < 2e-3, (n, err)
    torch.testing.assert_close(va, vb, atol=1e-3 * vb.abs().max().item(), rtol=1e-3)


def test_grad_into_leaves_equals_autograd_accumulation():
    """Fused backward with accumulate = 1 (grads added into the leaves' .grad) over three views
    equals autograd's own accumulation of the per-view gradients (to float-atomic ordering: the
    blend backward's global atomics, like the reference's, are not order-deterministic)."""
    import diff_gaussian_rasterization as dgr
    render, m, _ = _setup()
    cams = [c.to("cuda") for c in make_cameras(3, 200, 150, seed=1)]
    bg = torch.zeros(3, device="cuda")
    res = []
    try:
        for mode in (False, True):
            dgr.grad_into_leaves(mode)
            _zero(m)
            vs = []
            for c in cams:
                pkg = render(c, m, Pipe(sh_py=False), bg, Opt())
                (pkg["render"].sum() + pkg["feature"].sum() + pkg["depth"].mean()).backward()
                vs.append(pkg["viewspace_points"].grad.clone())
            res.append((_leaf_grads(m), vs))
    finally:
        dgr.grad_into_leaves(False)
    (ga, va), (gb, vb) = res
    for x, y in zip(ga + va, gb + vb):
        torch.testing.assert_close(x, y, rtol=1e-4, atol=1e-5 * y.abs().max().item())


@pytest.mark.parametrize("into_leaves", [True, False])
def test_view_pipeline_two_streams_equals_sequential(into_leaves):
    """gsr_amd.pipeline.ViewPipeline: six views issued round-robin on two HIP streams (view k+1's
    forward overlapping view k's backward; grad-into-leaves read-modify-writes ordered by the
    library's per-device event), SH gradients deferred to one flush per step
    (diff_gaussian_rasterization.ShGradDeferral) and the multi-view colour pre-pass (ShPrecolor),
    in every combination, give the same accumulated gradients and per-view screen-space gradients
    as the strictly sequential loop (to float-atomic ordering)."""
    import diff_gaussian_rasterization as dgr
    from gsr_amd.pipeline import ViewPipeline
    render, m, _ = _setup()
    cams = [c.to("cuda") for c in make_cameras(6, 200, 150, seed=2)]
    bg = torch.zeros(3, device="cuda")
    res = []
    try:
        dgr.grad_into_leaves(into_leaves)
        for depth, defer, pre in ((1, False, False), (2, True, True), (1, True, False),
                                  (2, False, True), (3, True, True)):
            _zero(m)
            pipe = ViewPipeline(torch.device("cuda"), depth=depth, defer_sh=defer, precolor=pre)

            def one(c):
                pkg = render(c, m, Pipe(sh_py=True), bg, Opt())
                (pkg["render"].sum() + pkg["feature"].sum() + pkg["depth"].mean()).backward()
                return pkg["viewspace_points"].grad.clone()

            vs = pipe.run(cams, one, model=m)
            torch.cuda.synchronize()
            res.append((_leaf_grads(m), vs))
    finally:
        dgr.grad_into_leaves(False)
    ga, va = res[0]
    for gb, vb in res[1:]:
        for x, y in zip(ga + va, gb + vb):
            torch.testing.assert_close(x, y, rtol=1e-4, atol=1e-5 * y.abs().max().item())


def test_sh_grad_deferral_accumulates_into_existing_grads():
    """A deferred step adds into SH .grad tensors that already hold values (the all-reduce
    bucket views of GradAllReducer.attach_grads): flush(accumulate = 1) == sequential sum."""
    import diff_gaussian_rasterization as dgr
    from gsr_amd.pipeline import ViewPipeline
    render, m, _ = _setup()
    cams = [c.to("cuda") for c in make_cameras(3, 200, 150, seed=4)]
    bg = torch.zeros(3, device="cuda")
    res = []
    try:
        dgr.grad_into_leaves(True)
        for defer in (False, True):
            for p in m.parameters():
                p.grad = torch.full_like(p, 0.25)

            def one(c):
                pkg = render(c, m, Pipe(sh_py=False), bg, Opt())
                (pkg["render"] * 2.0).sum().backward()

            ViewPipeline(torch.device("cuda"), depth=2, defer_sh=defer).run(cams, one)
            torch.cuda.synchronize()
            res.append(_leaf_grads(m))
    finally:
        dgr.grad_into_leaves(False)
    for x, y in zip(*res):
        torch.testing.assert_close(x, y, rtol=1e-4, atol=1e-5 * y.abs().max().item())


def test_precolor_forward_is_bit_identical():
    """The multi-view colour pre-pass (gsr_sh_precolor, sh_to_rgb of gsr_sh.h) feeds the fused
    forward exactly the colours and clamp bits its own preprocess computes: every output is
    bitwise equal, and so is the backward through the precomputed Jacobian up to atomic order."""
    import diff_gaussian_rasterization as dgr
    render, m, _ = _setup()
    cams = [c.to("cuda") for c in make_cameras(2, 200, 150, seed=6)]
    bg = torch.tensor([0.1, 0.2, 0.3], device="cuda")
    with torch.no_grad():
        ref = [render(c, m, Pipe(sh_py=True), bg, Opt()) for c in cams]
        with dgr.ShPrecolor(m._xyz, m._features_dc, m._features_rest, m.active_sh_degree,
                            [c.camera_center for c in cams]):
            got = [render(c, m, Pipe(sh_py=True), bg, Opt()) for c in cams]
    for a, b in zip(ref, got):
        for k in ("render", "depth", "alpha", "feature", "radii"):
            assert torch.equal(a[k], b[k]), k


def test_fused_render_of_empty_model():
    """render() on a GaussianModel with no Gaussians (the reference rasterizer returns zero images
    for P = 0, rasterize_points.cu:81): the fused path accepts the empty leaves (null data
    pointers) in the forward and the backward, in both grad modes."""
    import diff_gaussian_rasterization as dgr
    render, m, cam = _setup(P=10)
    for n in ("_xyz", "_features_dc", "_features_rest", "_opacity", "_scaling", "_rotation",
              "_language_feature"):
        setattr(m, n, getattr(m, n)[:0].detach().clone().requires_grad_(True))
    bg = torch.tensor([0.1, 0.2, 0.3], device="cuda")
    try:
        for into in (False, True):
            dgr.grad_into_leaves(into)
            pkg = render(cam, m, Pipe(sh_py=True), bg, Opt())
            assert torch.all(pkg["render"] == 0) and pkg["radii"].shape == (0,)
            (pkg["render"].sum() + pkg["depth"].sum()).backward()
            torch.cuda.synchronize()
    finally:
        dgr.grad_into_leaves(False)
