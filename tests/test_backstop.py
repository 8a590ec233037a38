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

    # both failures are in the device's sticky fault word (FusedAdam skips while it is set)
    assert _lib.forward_faults() & 1
    _lib.reset_forward_faults()
    assert _lib.forward_faults() == 0

    # the hook cleared: a normal call is finite, its backward runs, and the checks are clean
    (color, depth, alpha, feature, radii), inp = _call()
    (color.sum() + depth.sum()).backward()
    torch.cuda.synchronize()
    assert torch.isfinite(color).all() and torch.isfinite(inp["means3D"].grad).all()
    dgr.check_forwards(wait=True)
    assert _lib.forward_faults() == 0


def _forced_failure(fn):
    """Run fn() with every look-back forced to give up; returns its result."""
    from gsr_amd import _lib
    L = _lib.load()
    _lib.check(L.gsr_test_force_sort_timeout(1))
    try:
        return fn()
    finally:
        _lib.check(L.gsr_test_force_sort_timeout(0))


@pytest.mark.parametrize("det", [False, True])
def test_backward_of_a_failed_forward_poisons_every_gradient(det):
    """a backward that runs although its forward failed (here: the failure was already
    reported by check_forwards, so the host-side check on entry passes) writes NaN to EVERY
    gradient it returns -- store mode through the reference's `_C` signature (all 8 outputs), and
    accumulate mode (grad-into-leaves into pre-filled .grad) through render()'s fused path."""
    import numpy as np
    from gsr_amd import _lib
    import diff_gaussian_rasterization as dgr
    from diff_gaussian_rasterization import _C
    dgr.check_forwards(wait=True)
    prev_det = dgr.deterministic()
    dgr.deterministic(det)  # det: the per-instance-rows layout, whose indices the failed sort left
    try:
        _poison_case()
    finally:
        dgr.deterministic(prev_det)


def _poison_case():
    import numpy as np
    from gsr_amd import _lib
    import diff_gaussian_rasterization as dgr
    from diff_gaussian_rasterization import _C
    kw = scene(P=60_000, W=320, H=240, seed=3, mode="sh", feature=None)
    d = lambda x: torch.tensor(np.asarray(x), device="cuda")  # noqa: E731
    E = torch.Tensor([]).cuda()
    P = kw["means3D"].shape[0]
    nr, color, radii, geom, binning, img = _forced_failure(lambda: _C.rasterize_gaussians(
        d(kw["bg"]), d(kw["means3D"]), E, d(kw["opacities"]).view(P, 1), d(kw["scales"]),
        d(kw["rotations"]), 1.0, E, d(kw["viewmatrix"]), d(kw["projmatrix"]), kw["tanfovx"],
        kw["tanfovy"], kw["image_height"], kw["image_width"], d(kw["shs"]), kw["sh_degree"],
        d(kw["campos"]), False, False))
    torch.cuda.synchronize()
    with pytest.raises(_lib.GsrError):
        dgr.check_forwards(wait=True)
    dpix = torch.randn_like(color)
    grads = _C.rasterize_gaussians_backward(
        d(kw["bg"]), d(kw["means3D"]), radii, E, d(kw["scales"]), d(kw["rotations"]), 1.0, E,
        d(kw["viewmatrix"]), d(kw["projmatrix"]), kw["tanfovx"], kw["tanfovy"], dpix,
        d(kw["shs"]), kw["sh_degree"], d(kw["campos"]), geom, nr, binning, img, False)
    torch.cuda.synchronize()
    names = ["means2D", "colors", "opacity", "means3D", "cov3D", "sh", "scales", "rotations"]
    for n, g in zip(names, grads):
        assert torch.isnan(g).all(), n

    # accumulate mode: the fused backward adds into the leaves' existing .grad
    from gaussian_renderer import render
    from gsr_amd.model import SplatModel
    from gsr_amd.synthetic import make_cameras, make_gaussians
    from fused_ref import LEAVES, Opt, Pipe
    m = SplatModel(make_gaussians(60_000, sh_degree=3, seed=3), device="cuda")
    cam = make_cameras(1, 320, 240, seed=3)[0].to("cuda")
    for n in LEAVES:
        getattr(m, n).grad = torch.ones_like(getattr(m, n))
    prev = dgr.grad_into_leaves()
    dgr.grad_into_leaves(True)
    try:
        pkg = _forced_failure(lambda: render(cam, m, Pipe(), torch.zeros(3, device="cuda"), Opt()))
        torch.cuda.synchronize()
        with pytest.raises(_lib.GsrError):
            dgr.check_forwards(wait=True)
        torch.autograd.backward([pkg["render"], pkg["depth"]],
                                [torch.ones_like(pkg["render"]), torch.ones_like(pkg["depth"])])
        torch.cuda.synchronize()
    finally:
        dgr.grad_into_leaves(prev)
    for n in LEAVES:
        assert torch.isnan(getattr(m, n).grad).all(), n
    _lib.reset_forward_faults()


def test_train_step_with_a_failed_forward_leaves_parameters_unchanged():
    """NaN gradients of a failed forward never reach FusedAdam's parameters or
    moments -- the trainer checks the published status before the step, and FusedAdam skips on
    the device while the fault word is set (a failure not yet published by then)."""
    from gsr_amd import _lib, trainer
    from gsr_amd.model import SplatModel
    from gsr_amd.synthetic import make_cameras, make_gaussians, training_targets
    import diff_gaussian_rasterization as dgr
    dgr.check_forwards(wait=True)
    m = SplatModel(make_gaussians(60_000, sh_degree=3, seed=5), device="cuda")
    args = trainer.OptArgs()
    trainer.make_trainable(m, args)
    cam = make_cameras(1, 320, 240, seed=5)[0].to("cuda")
    gts, monos = training_targets(1, 240, 320, seed=2, device="cuda")
    bg = torch.zeros(3, device="cuda")
    before = [p.detach().clone() for p in m.parameters()]
    raised = False
    try:
        _forced_failure(lambda: trainer.train_iteration(m, cam, gts[0], monos[0], bg, args, 1,
                                                        2.78))
        torch.cuda.synchronize()
    except Exception:
        raised = True
    try:
        dgr.check_forwards(wait=True)
    except _lib.GsrError:
        raised = True
    assert raised
    assert _lib.forward_faults() != 0
    for p, b in zip(m.parameters(), before):
        assert torch.equal(p.detach(), b)
    # the failure is handled: reset the fault word; the next iteration steps normally (a step
    # FusedAdam skipped on the device above, if any, had its step counts taken back)
    _lib.reset_forward_faults()
    m.optimizer.zero_grad(set_to_none=True)
    trainer.train_iteration(m, cam, gts[0], monos[0], bg, args, 2, 2.78)
    torch.cuda.synchronize()
    assert any(not torch.equal(p.detach(), b) for p, b in zip(m.parameters(), before))
    assert all(torch.isfinite(p).all() for p in m.parameters())
    assert all(float(st["step"]) == 1.0 for st in m.optimizer.state.values())


def test_fused_adam_skip_is_one_decision_and_reported():
    """the skip is decided once per step (a guard snapshot every tensor's workgroups
    read), reported to the host through a pinned word, and the next step() takes back the step
    counts of the skipped step and raises -- unless reset_forward_faults() ran since."""
    from gsr_amd import _lib
    from gsr_amd.optim import FusedAdam
    import diff_gaussian_rasterization as dgr
    dgr.check_forwards(wait=True)
    _lib.reset_forward_faults()
    ps = [torch.randn(n, device="cuda").requires_grad_(True) for n in (5000, 333, 70000)]
    opt = FusedAdam([{"params": [p], "lr": 1e-2} for p in ps], eps=1e-15)
    for p in ps:
        p.grad = torch.randn_like(p)
    opt.step()  # a normal step
    torch.cuda.synchronize()
    before = [p.detach().clone() for p in ps]
    moments = [opt.state[p]["exp_avg"].clone() for p in ps]
    # a failed forward: the fault word is set
    with torch.no_grad():
        _forced_failure(_call)
    torch.cuda.synchronize()
    with pytest.raises(_lib.GsrError):
        dgr.check_forwards(wait=True)
    for p in ps:
        p.grad = torch.full_like(p, float("nan"))
    opt.step()  # skipped on the device (no host synchronisation, no error yet)
    torch.cuda.synchronize()
    for p, b, m0 in zip(ps, before, moments):
        assert torch.equal(p.detach(), b) and torch.equal(opt.state[p]["exp_avg"], m0)
    with pytest.raises(RuntimeError, match="skipped"):
        opt.step()  # reports the skipped step; nothing launched
    assert all(float(opt.state[p]["step"]) == 1.0 for p in ps) and opt.skipped_steps == 1
    for p, b in zip(ps, before):
        assert torch.equal(p.detach(), b)
    # handled: reset, finite gradients, the step applies with the right bias correction (step 2)
    _lib.reset_forward_faults()
    for p in ps:
        p.grad = torch.randn_like(p)
    opt.step()
    opt.step()  # resolves the previous (applied) step: no error
    torch.cuda.synchronize()
    assert all(float(opt.state[p]["step"]) == 3.0 for p in ps)
    assert all(not torch.equal(p.detach(), b) for p, b in zip(ps, before))
    # a caller-provided skip slot (the reducer's all-reduced guard) decides alone
    slot = torch.ones(1, device="cuda")
    now = [p.detach().clone() for p in ps]
    opt.step(skip=slot)
    torch.cuda.synchronize()
    assert all(torch.equal(p.detach(), b) for p, b in zip(ps, now))
    with pytest.raises(RuntimeError, match="skipped"):
        opt.step()
    assert all(float(opt.state[p]["step"]) == 3.0 for p in ps)


def test_reducer_guard_skips_the_step_on_the_device():
    """The multi-GPU form at world size 1 (collectives forced on, gloo over the device tensors):
    the step's forward-fault snapshot goes through the gradient all-reduce and FusedAdam skips on
    the reduced slot (tests/test_parallel.py checks the cross-rank sum on CPU)."""
    import os
    import tempfile
    import torch.distributed as dist
    from gsr_amd import _lib, trainer
    from gsr_amd.model import SplatModel
    from gsr_amd.parallel import GradAllReducer
    from gsr_amd.pipeline import ViewPipeline
    from gsr_amd.synthetic import make_cameras, make_gaussians, training_targets
    import diff_gaussian_rasterization as dgr
    dgr.check_forwards(wait=True)
    _lib.reset_forward_faults()
    fd, path = tempfile.mkstemp(prefix="gsr_pg_")
    os.close(fd)
    os.unlink(path)
    dist.init_process_group("gloo", init_method="file://" + path, rank=0, world_size=1)
    try:
        m = SplatModel(make_gaussians(40_000, sh_degree=3, seed=6), device="cuda")
        args = trainer.OptArgs()
        trainer.make_trainable(m, args)
        cams = [c.to("cuda") for c in make_cameras(2, 320, 240, seed=6)]
        gts, monos = training_targets(2, 240, 320, seed=2, device="cuda")
        bg = torch.zeros(3, device="cuda")
        reducer = GradAllReducer(m)
        reducer._active = lambda: True
        pipe = ViewPipeline(torch.device("cuda"), depth=2)
        step = lambda it: trainer.train_step_views(m, cams, gts, monos, bg, args, it, 2.78,  # noqa: E731
                                                   pipe, reducer=reducer)
        step(1)
        torch.cuda.synchronize()
        assert float(reducer.skip_flag()) == 0.0
        before = [p.detach().clone() for p in m.parameters()]
        raised = False
        try:
            _forced_failure(lambda: step(2))
            torch.cuda.synchronize()
        except Exception:
            raised = True
        try:
            dgr.check_forwards(wait=True)
        except _lib.GsrError:
            raised = True
        assert raised
        for p, b in zip(m.parameters(), before):
            assert torch.equal(p.detach(), b)
        _lib.reset_forward_faults()
        step(3)
        torch.cuda.synchronize()
        assert float(reducer.skip_flag()) == 0.0
        assert any(not torch.equal(p.detach(), b) for p, b in zip(m.parameters(), before))
    finally:
        dist.destroy_process_group()
        _lib.reset_forward_faults()


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
