"""The training iteration around the rasterizer (train.py:63-236), on libgsr.

`train_iteration` is the reference's per-iteration body for one camera with the depth branch:

    render(cam) -> loss = (1 - lambda_dssim) * L1 + lambda_dssim * (1 - SSIM)      (train.py:93-100)
                        + depth_weight * min(1 - pearson(d_mono, d), 1 - pearson(1/(200 - d_mono), d))
                                                                                     (train.py:117-131)
    loss.backward()                                                                  (train.py:194)
    max_radii2D / add_densification_stats; densify_and_prune every
    densification_interval iterations inside [densify_from_iter, densify_until_iter) (:218-225)
    optimizer.step(); optimizer.zero_grad(set_to_none=True)                          (:229-231)

The language-feature loss (loss_feature_metric) and the pseudo-view branch (:101-193) need the
scene's CLIP features / MiDaS depth, which a synthetic benchmark does not have; the feature image is
still rendered (include_feature) and the pseudo-view interval is past end_sample_pseudo at the
reference's defaults for most of training.  `train_step_views` is the batched multi-view form of the
same iteration (ViewPipeline over HIP streams, gradients summed over the views, one optimizer step;
with a GradAllReducer the per-view gradients of all ranks are summed first).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Sequence

import torch


@dataclass
class OptArgs:
    """OptimizationParams fields the iteration reads (arguments/__init__.py:73-120)."""
    percent_dense: float = 0.01
    position_lr_init: float = 0.016
    feature_lr: float = 0.0025
    opacity_lr: float = 0.05
    scaling_lr: float = 0.003
    rotation_lr: float = 0.001
    language_feature_lr: float = 0.013
    lambda_dssim: float = 0.2
    densification_interval: int = 100
    densify_from_iter: int = 500
    densify_until_iter: int = 6000
    densify_grad_threshold: float = 0.0013
    prune_threshold: float = 0.01
    depth_weight: float = 0.05
    include_feature: bool = True


class _Pipe:  # PipelineParams defaults (arguments/__init__.py:66-72)
    convert_SHs_python = True
    compute_cov3D_python = False
    debug = False
    use_confidence = False


def make_trainable(model, args: OptArgs, spatial_lr_scale: float = 1.0):
    """GaussianModel.training_setup (scene/gaussian_model.py:217-271) with FusedAdam."""
    model.training_setup(args, spatial_lr_scale=spatial_lr_scale)
    return model


def _view_loss(pkg, gt_image, depth_mono, args: OptArgs):
    from .losses import photometric_loss, train_view_loss
    if depth_mono is not None:  # one autograd node for both terms (losses.train_view_loss)
        loss, _ = train_view_loss(pkg["render"], pkg["depth"], gt_image, depth_mono,
                                  args.lambda_dssim, args.depth_weight)
        return loss
    loss, _ = photometric_loss(pkg["render"], gt_image, args.lambda_dssim)
    return loss


def _densify_due(iteration: int, args: OptArgs) -> bool:
    return (iteration < args.densify_until_iter and iteration > args.densify_from_iter
            and iteration % args.densification_interval == 0)


def densify_step(model, args: OptArgs, iteration: int, extent: float, generator=None):
    """train.py:223-225 (size_threshold None)."""
    model.densify_and_prune(args.densify_grad_threshold, args.prune_threshold, extent, None,
                            iteration, args.include_feature, generator=generator)


def _guard_step():
    """Before the optimizer step: raise if a forward of this step already reported a failure
    (non-blocking, include/gsr.h gsr_check_forwards).  A failure not yet published by then is
    caught on the device: FusedAdam leaves the parameters and moments untouched while the
    step's fault snapshot is set (include/gsr_optim.h), and its next step() raises."""
    import diff_gaussian_rasterization as dgr
    dgr.check_forwards(wait=False)


def _optimizer_step(model, reducer=None):
    """optimizer.step(); with a multi-GPU reducer FusedAdam takes the ranks' summed fault
    snapshot as its skip decision (any rank failed -> every rank skips)."""
    from .optim import FusedAdam
    opt = model.optimizer
    skip = reducer.skip_flag() if reducer is not None else None
    if isinstance(opt, FusedAdam):
        opt.step(skip=skip)
    else:
        opt.step()


def train_iteration(model, cam, gt_image, depth_mono, bg, args: OptArgs, iteration: int,
                    extent: float, pipe=None):
    """One reference iteration on one camera.  Returns the loss tensor (not synchronised)."""
    from gaussian_renderer import render
    pipe = pipe or _Pipe()
    pkg = render(cam, model, pipe, bg, args)
    loss = _view_loss(pkg, gt_image, depth_mono, args)
    loss.backward()
    with torch.no_grad():
        if iteration < args.densify_until_iter:
            model.update_densification_stats(pkg["viewspace_points"], pkg["radii"],
                                             pkg["visibility_filter"])
            if _densify_due(iteration, args):
                densify_step(model, args, iteration, extent)
        _guard_step()
        _optimizer_step(model)
        model.optimizer.zero_grad(set_to_none=True)
    return loss.detach()


def train_step_views(model, cams: Sequence, gt_images: Sequence[torch.Tensor],
                     depth_monos: Sequence[Optional[torch.Tensor]], bg, args: OptArgs,
                     iteration: int, extent: float, pipeline, reducer=None, pipe=None,
                     generator=None, multi: bool = True,
                     next_cams: Optional[Sequence] = None) -> List[torch.Tensor]:
    """The batched iteration: every camera's render + loss + backward + statistics (gradients
    summed over the views), the gradient all-reduce across ranks (reducer, overlapped with the
    step's tail), densification when due (statistics summed / maxed across ranks first,
    identical generator on every rank), one optimizer step.  multi: all views in one multi-view
    call (gaussian_renderer.render_views: one host call for the forwards, one for the backwards;
    the per-view losses are back-propagated together); else view by view on the pipeline's
    streams (render() per view, lagged).

    Multi-GPU (reducer, multi): the optimizer runs in row slices behind the sliced all-reduce,
    each slice followed by the next step's prologue for those rows -- the gradient zeroing and,
    given next_cams (the next step's cameras), its colour pre-pass."""
    from gaussian_renderer import render, render_views
    from .parallel import allreduce_densification_stats
    pipe = pipe or _Pipe()
    if reducer is not None:
        reducer.attach_grads()
    else:
        model.optimizer.zero_grad(set_to_none=True)
    gts = {id(c): (g, d) for c, g, d in zip(cams, gt_images, depth_monos)}

    if multi:
        def all_views(cs, strs):
            from .losses import train_views_loss
            pkgs = render_views(cs, model, pipe, bg, args, streams=strs)
            st = pkgs[0].get("views") if pkgs else None
            monos_ = [gts[id(c)][1] for c in cs]
            if st is not None and len(cs) <= 8 and all(m is not None for m in monos_):
                # every view's loss in one node over the stacked outputs (one launch per stage)
                totals, _ = train_views_loss(st["render"], st["depth"],
                                             [gts[id(c)][0] for c in cs], monos_,
                                             args.lambda_dssim, args.depth_weight)
                totals.backward(torch.ones_like(totals))
                losses = list(totals.detach().unbind(0))
            else:
                losses = [_view_loss(pkg, *gts[id(c)], args) for c, pkg in zip(cs, pkgs)]
                torch.autograd.backward(losses)
            with torch.no_grad():
                if iteration < args.densify_until_iter:
                    if st is not None and hasattr(model, "update_densification_stats_views"):
                        # every view's statistics in one launch (visibility = radii > 0)
                        model.update_densification_stats_views(st["viewspace_points"].grad,
                                                               st["radii"])
                    else:
                        for pkg in pkgs:
                            model.update_densification_stats(pkg["viewspace_points"],
                                                             pkg["radii"],
                                                             pkg["visibility_filter"])
            return [loss.detach() for loss in losses]
        # Multi-GPU: the optimizer step in row slices, each as soon as its rows' all-reduce is
        # done (overlapping the next slice's collective), followed by the next step's gradient
        # zeroing of those rows -- unless this iteration densifies (the step then follows the
        # densification, as in train.py:223-231)
        from .optim import FusedAdam
        opt = model.optimizer
        h = None
        if (reducer is not None and isinstance(opt, FusedAdam) and reducer._active()
                and not reducer.average and not _densify_due(iteration, args)):
            reducer.begin()  # the step's layout (also re-read by run_views)
            h = opt.begin_rows(skip=reducer.guard)
            fill = None

            def after_slice(a, b):
                nonlocal fill
                opt.step_rows(h, a, b)
                reducer.zero_rows(a, b)
                if next_cams is not None:
                    if fill is None:  # this step's forwards and backwards are issued by now
                        fill = pipeline.prepare_next(model, list(next_cams))
                    fill(a, b)
        try:
            losses = pipeline.run_views(cams, all_views, model=model, reducer=reducer,
                                        after_slice=None if h is None else after_slice)
        except BaseException:
            if h is not None:  # no Adam update ran: the step counts go back
                opt.abort_rows(h)
            raise
        with torch.no_grad():
            if h is not None:
                if not pipeline.rows_done:  # no sliced reduction ran: the whole step now
                    opt.step_rows(h, 0, None)
                opt.end_rows(h)
                _guard_step()
                return losses
            if _densify_due(iteration, args):
                allreduce_densification_stats(model.xyz_gradient_accum, model.denom,
                                               model.max_radii2D)
                densify_step(model, args, iteration, extent, generator=generator)
            _guard_step()
            _optimizer_step(model, reducer)
        return losses

    def forward(cam):
        pkg = render(cam, model, pipe, bg, args)
        gt, dm = gts[id(cam)]
        return pkg, _view_loss(pkg, gt, dm, args)

    def backward(fw):
        pkg, loss = fw
        loss.backward()
        with torch.no_grad():
            if iteration < args.densify_until_iter:
                model.update_densification_stats(pkg["viewspace_points"], pkg["radii"],
                                                 pkg["visibility_filter"])
        return loss.detach()

    # view i's backward is issued after view i + 1's forward (ViewPipeline.run(bwd=, lag=1))
    losses = pipeline.run(cams, forward, model=model, reducer=reducer, bwd=backward, lag=1)
    with torch.no_grad():
        if _densify_due(iteration, args):
            allreduce_densification_stats(model.xyz_gradient_accum, model.denom,
                                           model.max_radii2D)
            densify_step(model, args, iteration, extent, generator=generator)
        # after a densification the new parameters have no .grad: Adam skips them, as in the
        # reference (train.py:223-231)
        _guard_step()
        _optimizer_step(model, reducer)
    return losses
