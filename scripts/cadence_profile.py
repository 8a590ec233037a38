"""Where the time of train.py's cadence goes: one view per iteration, one
stream, FusedAdam after every view (gsr_amd.trainer.train_iteration), on bench.py's headline
model (1M Gaussians, 1008x756, 12-camera pool).  Reports per iteration: wall time, the host time
the forwards spent waiting for their instance-count read-back (gsr_test_host_wait_ms), the host
time of each phase (render, loss, backward, optimizer), and -- with --stages -- the GPU time of
every rasterizer stage (hipEvents, one extra instrumented pass).

  python scripts/cadence_profile.py [--iters 48] [--stages]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "sdp-gs_amd")]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=48)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--stages", action="store_true")
    args = ap.parse_args()
    import diff_gaussian_rasterization as dgr
    from gaussian_renderer import render
    from gsr_amd import _lib, trainer
    from gsr_amd.model import SplatModel
    from gsr_amd.synthetic import make_cameras, make_gaussians, training_targets
    dev = torch.device("cuda", 0)
    dgr.grad_into_leaves(True)
    model = SplatModel(make_gaussians(1_000_000, sh_degree=3, seed=0), device=dev)
    targs = trainer.OptArgs()
    trainer.make_trainable(model, targs)
    cams = [c.to(dev) for c in make_cameras(12, 1008, 756, seed=0)]
    gts, monos = training_targets(len(cams), 756, 1008, seed=2, device=dev)
    bg = torch.zeros(3, device=dev)
    L = _lib.load()
    phases = {"render": 0.0, "loss": 0.0, "backward": 0.0, "stats+adam": 0.0}

    def one(i, timed):
        c = cams[i % len(cams)]
        pipe = trainer._Pipe()
        t0 = time.perf_counter()
        pkg = render(c, model, pipe, bg, targs)
        t1 = time.perf_counter()
        loss = trainer._view_loss(pkg, gts[i % len(cams)], monos[i % len(cams)], targs)
        t2 = time.perf_counter()
        loss.backward()
        t3 = time.perf_counter()
        with torch.no_grad():
            model.update_densification_stats(pkg["viewspace_points"], pkg["radii"],
                                             pkg["visibility_filter"])
            trainer._guard_step()
            trainer._optimizer_step(model)
            model.optimizer.zero_grad(set_to_none=True)
        t4 = time.perf_counter()
        if timed:
            phases["render"] += t1 - t0
            phases["loss"] += t2 - t1
            phases["backward"] += t3 - t2
            phases["stats+adam"] += t4 - t3

    for i in range(args.warmup):
        one(i, False)
    torch.cuda.synchronize()
    L.gsr_test_host_wait_ms(1)
    t0 = time.perf_counter()
    for i in range(args.iters):
        one(i, True)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    wait = L.gsr_test_host_wait_ms(1)
    out = {"views_per_s": round(args.iters / el, 2), "ms_per_view": round(1000 * el / args.iters, 4),
           "host_wait_ms_per_view": round(wait / args.iters, 4),
           "host_ms_per_view_by_phase": {k: round(1000 * v / args.iters, 4) for k, v in phases.items()}}
    if args.stages:
        timer = _lib.StageTimer()
        timer.reset()
        timer.enable(True)
        for i in range(12):
            one(i, False)
        torch.cuda.synchronize()
        timer.enable(False)
        out["gpu_stage_ms_per_view"] = {k: round(ms / 12, 4) for k, (ms, c) in timer.collect().items() if c}
    out["api"] = api_table(model, cams, bg, targs)
    print(json.dumps(out), flush=True)


def api_table(model, cams, bg, targs, iters=6):
    """The reference-API leg (bench.py reference_api: render() with GSR_FUSED=0, autograd
    gradients, one view at a time) phase by phase, each phase synchronised: render() total, its
    torch pre-pass alone (getters + Python SH + language normalisation, timed by replaying
    gaussian_renderer/__init__.py:247-287's torch ops), the backward, and the rasterizer's own
    GPU stages (hipEvents)."""
    import diff_gaussian_rasterization as dgr
    from gaussian_renderer import render
    from gsr_amd import _lib, trainer
    from gsr_amd.sh import eval_sh
    prev = os.environ.get("GSR_FUSED")
    os.environ["GSR_FUSED"] = "0"
    prev_leaves = dgr.grad_into_leaves()
    dgr.grad_into_leaves(False)
    H, W = cams[0].image_height, cams[0].image_width
    up = [torch.randn(s, device=bg.device) for s in ((3, H, W), (1, H, W), (3, H, W))]
    t = {"render_ms": 0.0, "backward_ms": 0.0, "torch_prepass_ms": 0.0}

    def sync_time(fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = fn()
        torch.cuda.synchronize()
        return r, 1000.0 * (time.perf_counter() - t0)

    def prepass(cam):
        with torch.no_grad():
            xyz = model.get_xyz
            _ = (model.get_opacity, model.get_scaling, model.get_rotation)
            shs_view = model.get_features.transpose(1, 2).view(-1, 3, (model.max_sh_degree + 1) ** 2)
            d = xyz - cam.camera_center.repeat(model.get_features.shape[0], 1)
            d = d / d.norm(dim=1, keepdim=True)
            col = torch.clamp_min(eval_sh(model.active_sh_degree, shs_view, d) + 0.5, 0.0)
            lf = model.get_language_feature
            return col, lf / lf.norm(dim=1, keepdim=True).clamp_min(1e-12)

    timer = _lib.StageTimer()
    try:
        for i in range(iters + 2):
            cam = cams[i % len(cams)]
            for p in model.parameters():
                p.grad = None
            timer.reset()
            timer.enable(i >= 2)
            pkg, tr = sync_time(lambda: render(cam, model, trainer._Pipe(), bg, targs))
            _, tb = sync_time(lambda: torch.autograd.backward(
                [pkg["render"], pkg["depth"], pkg["feature"]], up))
            timer.enable(False)
            _, tp = sync_time(lambda: prepass(cam))
            if i >= 2:
                t["render_ms"] += tr / iters
                t["backward_ms"] += tb / iters
                t["torch_prepass_ms"] += tp / iters
                st = timer.collect()
                for k, (ms, c) in st.items():
                    if c:
                        t["gpu_" + k + "_ms"] = t.get("gpu_" + k + "_ms", 0.0) + ms / iters
    finally:
        if prev is None:
            os.environ.pop("GSR_FUSED", None)
        else:
            os.environ["GSR_FUSED"] = prev
        dgr.grad_into_leaves(prev_leaves)
    return {k: round(v, 4) for k, v in t.items()}


if __name__ == "__main__":
    main()
