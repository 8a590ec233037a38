"""Same-call failure of a forward whose sort gave up.

The one-sweep sorts bound their decoupled look-back spin (gsr_sort.hip); the reference would
__trap() on an invalid state inside the call (auxiliary.h:156-160).  Here the call that produced
the bad sort is the one that fails: its outputs are NaN, its backward raises once the status is
published, and gsr_check_forwards / gsr_forward_status report it.  The give-up path is forced with
the gsr_test_force_sort_timeout hook (every look-back takes it), then the hook is cleared and a
normal call is checked clean.
"""
import pytest
import torch

from scenes import scene, to_torch_call

pytestmark = pytest.mark.gpu


def _call(requires_grad=True):
    from diff_gaussian_rasterization import GaussianRasterizer
    # enough Gaussians and instances for several sort partitions (look-backs happen only past
    # the first partition)
    kw = scene(P=60_000, W=320, H=240, seed=3, mode="sh", feature="sh")
    settings, inp = to_torch_call(kw, device="cuda")
    out = GaussianRasterizer(settings)(
        means3D=inp["means3D"], means2D=inp["means2D"], opacities=inp["opacities"],
        shs=inp["shs"], scales=inp["scales"], rotations=inp["rotations"],
        shs_language=inp["shs_language"])
    return out, inp


def test_forced_sort_timeout_fails_the_same_call():
    from gsr_amd import _lib
    import diff_gaussian_rasterization as dgr
    L = _lib.load()
    dgr.check_forwards(wait=True)  # nothing pending from earlier tests
    _lib.check(L.gsr_test_force_sort_timeout(1))
    try:
        (color, depth, alpha, feature, radii), inp = _call()
        torch.cuda.synchronize()
    finally:
        _lib.check(L.gsr_test_force_sort_timeout(0))
    # device-side poison of this call's outputs
    assert torch.isnan(color).all() and torch.isnan(depth).all()
    # its backward fails (the status is published: we synchronized above) ...
    with pytest.raises(Exception, match="look-back timed out"):
        (color.nan_to_num().sum() + depth.nan_to_num().sum()).backward()
    # ... and the blocking check reports nothing further once that call was reported
    dgr.check_forwards(wait=True)

    # again without a backward: the step-end check raises for the failed forward
    _lib.check(L.gsr_test_force_sort_timeout(1))
    try:
        with torch.no_grad():
            _call(requires_grad=False)
    finally:
        _lib.check(L.gsr_test_force_sort_timeout(0))
    with pytest.raises(_lib.GsrError, match="look-back timed out"):
        dgr.check_forwards(wait=True)

    # the hook cleared: a normal call is finite, its backward runs, and the checks are clean
    (color, depth, alpha, feature, radii), inp = _call()
    (color.sum() + depth.sum()).backward()
    torch.cuda.synchronize()
    assert torch.isfinite(color).all() and torch.isfinite(inp["means3D"].grad).all()
    dgr.check_forwards(wait=True)


def test_sh_deferral_flush_with_one_plane_grad_present():
    """ShGradDeferral.flush with features_dc.grad present and features_rest.grad None adds into
    zeros: equals the flush with both grads absent, plus the existing dc grad."""
    import diff_gaussian_rasterization as dgr
    from gaussian_renderer import render
    from gsr_amd.model import SplatModel
    from gsr_amd.synthetic import make_cameras, make_gaussians, upstream_grads
    from gsr_amd.pipeline import ViewPipeline
    from fused_ref import Opt, Pipe

    m = SplatModel(make_gaussians(20_000, sh_degree=3, seed=4), device="cuda")
    cams = [c.to("cuda") for c in make_cameras(2, 160, 120, seed=4)]
    grads = upstream_grads(120, 160, seed=1, device="cuda")
    bg = torch.zeros(3, device="cuda")

    def run(pre_dc):
        for n in ("_xyz", "_features_dc", "_features_rest", "_opacity", "_scaling", "_rotation",
                  "_language_feature"):
            getattr(m, n).grad = None
        if pre_dc is not None:
            m._features_dc.grad = pre_dc.clone()
        prev = dgr.grad_into_leaves()
        dgr.grad_into_leaves(True)
        try:
            def one(cam):
                pkg = render(cam, m, Pipe(), bg, Opt())
                torch.autograd.backward([pkg["render"], pkg["depth"], pkg["feature"]], list(grads))
            ViewPipeline(torch.device("cuda"), depth=1, defer_sh=True).run(cams, one, model=m)
            torch.cuda.synchronize()
        finally:
            dgr.grad_into_leaves(prev)
        return m._features_dc.grad.clone(), m._features_rest.grad.clone()

    dc0, rest0 = run(None)
    offset = torch.randn_like(m._features_dc)
    dc1, rest1 = run(offset)
    torch.testing.assert_close(dc1, dc0 + offset, rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(rest1, rest0, rtol=1e-5, atol=1e-6)  # add-into-zeros vs store order
