#!/usr/bin/env python3
"""Benchmark: rasterized views/sec (fwd+bwd) of the MI355X Gaussian rasterizer.

Workload (BASELINE.json configs[2] at N=1, configs[3] at N=8): 1,000,000 synthetic Gaussians
(SH degree 3 evaluated in-kernel, language features on), LLFF-style cameras at 1008x756, and
`--views-per-gpu` (default 6) camera views per GPU per step.  One step = for each of this rank's
views: render() (rasterizer forward with colour/depth/alpha/feature outputs; GaussianModel's
activations fused into the kernels) and the backward of fixed synthetic upstream gradients,
accumulating the raw parameters' gradients into their .grad; then, with
N > 1, one bucketed SUM all-reduce of all gradients over RCCL.  Weak scaling: views per GPU fixed.

    python bench.py --gpus N --steps K --warmup W

Prints ONE JSON line on rank 0 (see DESIGN.md section 7 for the roofline byte model).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "sdp-gs_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0     # MI355X_MICROARCH.md chip table (spec)
FP32_PEAK_TFLOPS = 157.3  # vector FP32 (spec)

WORKLOADS = {
    # name: (P, W, H, sh_degree)
    "llff_1m_1008x756": (1_000_000, 1008, 756, 3),
    "cfg2_100k_800x800": (100_000, 800, 800, 3),
    "cfg5_5m_1920x1080": (5_000_000, 1920, 1080, 3),
}


class Pipe:
    # the reference's PipelineParams defaults (arguments/__init__.py:68-71); render() evaluates
    # the Python SH colour / language pre-pass inside the fused HIP preprocess
    convert_SHs_python = True
    compute_cov3D_python = False
    debug = False
    use_confidence = False


class Opt:
    include_feature = True


def algorithmic_bytes(stage, P, Pv, R, T, HW, D=3, C=8, tile_passes=2, acc=True, defer_sh=False,
                      precolor=False, views=6):
    """Bytes each stage must move per launch.
    P Gaussians, Pv visible, R instances, T tiles, HW pixels, C blended channels (rgb, depth,
    alpha, feature x3), acc: the backward adds into existing gradients (read + write),
    defer_sh: the SH gradients are replaced by a stored 12-B dL/dRGB (flushed once per step),
    precolor: the SH rows are replaced by the pre-pass's colour + clamp (13 B, forward) and
    colour Jacobian (36 B, backward)."""
    sh = 12 * (D + 1) ** 2
    sh_fwd = 13 if precolor else sh
    sh_bwd = 36 if (precolor and defer_sh) else sh
    grads = 12 + 12 + 4 + 12 + 16 + 12 + (0 if defer_sh else sh)  # means2D/3D, op, scale, rot, lang, SH
    return {
        # means (all); scale, rot, opacity, SH, language (visible); radii/tiles/key/value (all);
        # 64-B splat record + clamp bits (visible), the 64-B gradient accumulator row it zeroes (all)
        "preprocess": P * 12 + Pv * (12 + 16 + 4 + sh_fwd + 12) + P * 16 + Pv * (64 + 1) + P * 64,
        # one-sweep: digit totals read the keys once, each 8-bit pass reads and writes key+value
        "depth_sort": P * 4 + 4 * P * 16,
        "scan": P * 12,
        # offsets (all), order + 48-B record gather (non-empty), R (tile, id) pairs
        "duplicate": P * 8 + Pv * (4 + 48) + R * 8,
        "tile_sort": R * 4 + tile_passes * R * 16,
        "ranges": R * 4 + T * 8,
        # point_list + 64-B record per instance, ranges/tile_last, C outputs + final_T + n_contrib
        "render_fwd": R * (4 + 64) + T * 12 + HW * (4 * C + 8),
        "acc_zero": P * 64,
        # same gathers, C upstream grads + final_T + n_contrib, one 64-B accumulator row per Gaussian
        "render_bwd": R * (4 + 64) + T * 12 + HW * (4 * C + 8) + Pv * 64,
        # accumulator row + per-Gaussian inputs (visible), radii (all), gradients (RMW when acc)
        "preprocess_bwd": Pv * (64 + 12 + 12 + 16 + 4 + sh_bwd + 12 + 1) + P * 4
                          + ((2 * Pv) if acc else P) * grads + (P * 12 if defer_sh else 0),
        # once per step for V views (reported per launch): SH rows + means in, 49 B per view out
        "sh_precolor": P * (12 + sh) + P * 49 * views,
        # means + V stored dL/dRGB in, SH gradients out (store mode)
        "sh_flush": P * (12 + 12 * views) + P * sh,
    }[stage]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="llff_1m_1008x756", choices=sorted(WORKLOADS))
    ap.add_argument("--views-per-gpu", type=int, default=6)
    ap.add_argument("--cpu-baseline-views", type=int, default=2)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-stage-timing", action="store_true")
    ap.add_argument("--autograd-grads", action="store_true",
                    help="return per-view raw grads to autograd instead of adding them into .grad")
    ap.add_argument("--streams", type=int, default=3,
                    help="views of a step issued round-robin on this many HIP streams "
                         "(gsr_amd.pipeline.ViewPipeline; 1 = strictly sequential)")
    ap.add_argument("--no-defer-sh", action="store_true",
                    help="write the SH gradients in every view's backward instead of one flush "
                         "per step (diff_gaussian_rasterization.ShGradDeferral)")
    ap.add_argument("--no-precolor", action="store_true",
                    help="each view evaluates its SH colour itself instead of the step's pre-pass")
    ap.add_argument("--pmc-file", default=os.path.join(ROOT, "profiles", "pmc_r01.json"))
    args = ap.parse_args()

    from gsr_amd import _lib
    from gsr_amd.model import SplatModel
    from gsr_amd.parallel import GradAllReducer, init_from_env, shard_views
    from gsr_amd.pipeline import ViewPipeline
    from gsr_amd.synthetic import make_cameras, make_gaussians, upstream_grads
    import diff_gaussian_rasterization as dgr
    from gaussian_renderer import render

    dgr.grad_into_leaves(not args.autograd_grads)
    rank, world, local = init_from_env("nccl")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    P, W, H, deg = WORKLOADS[args.workload]

    params = make_gaussians(P, sh_degree=deg, seed=0)
    model = SplatModel(params, device=dev)
    n_views = args.views_per_gpu * world
    cams_all = make_cameras(n_views, W, H, seed=0)
    my_cams = [cams_all[i].to(dev) for i in shard_views(n_views, rank, world)]
    dimg, ddep, dfeat = upstream_grads(H, W, seed=1, device=dev)
    bg = torch.zeros(3, device=dev)
    reducer = GradAllReducer(model.parameters()) if world > 1 else None
    pipe, opt = Pipe(), Opt()
    stats = {"R": [], "Pv": []}
    defer_sh = not args.no_defer_sh and not args.autograd_grads
    views = ViewPipeline(dev, depth=max(1, args.streams), defer_sh=defer_sh,
                         precolor=not args.no_precolor)

    def one_view(cam, record):
        pkg = render(cam, model, pipe, bg, opt)
        torch.autograd.backward([pkg["render"], pkg["depth"], pkg["feature"]],
                                [dimg, ddep, dfeat])
        if record:
            stats["R"].append(dgr.LAST_STATS["num_rendered"])
            stats["Pv"].append(int(pkg["visibility_filter"].sum()))

    def step(record=False):
        if reducer is not None:
            reducer.attach_grads()  # grads accumulate straight into the all-reduce buckets
        else:
            for p in model.parameters():
                p.grad = None
        views.run(my_cams, lambda cam: one_view(cam, record), model=model)
        if reducer is not None:
            reducer.allreduce()

    for _ in range(args.warmup):
        step()
    step(record=True)  # one recorded step for the per-view statistics (not timed)
    timer = _lib.StageTimer()
    # Per-stage table from one fully instrumented, untimed step (events around every stage cost
    # ~7% of a view).  The headline value comes from a clean timed region (no events: with the
    # views on several streams even the dominant kernel's two events per view perturb the
    # overlap); the dominant kernel's launch duration then comes from a second timed region of the
    # same K steps with only that stage bracketed by events.
    all_stages = {}
    dom_stage = None
    if not args.no_stage_timing:
        timer.reset()
        timer.enable(True)
        step()
        timer.enable(False)
        all_stages = timer.collect()
        busy = {n: ms for n, (ms, c) in all_stages.items() if c}
        dom_stage = max(busy, key=busy.get) if busy else None
        timer.reset()

    def timed_region():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([el], device=dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el

    elapsed = timed_region()
    stages = dict(all_stages)
    dom_elapsed = None
    if dom_stage is not None:
        timer.enable(True, stages=[dom_stage])
        dom_elapsed = timed_region()
        timer.enable(False)
        stages[dom_stage] = timer.collect()[dom_stage]  # measured over the second timed region

    total_views = args.steps * n_views
    value = total_views / elapsed
    ms_per_step = 1000.0 * elapsed / args.steps

    R = float(np.mean(stats["R"]))
    Pv = float(np.mean(stats["Pv"]))
    T = ((W + 15) // 16) * ((H + 15) // 16)
    HW = W * H
    kernels = {}
    for name, (ms, calls) in stages.items():
        if calls == 0:
            continue
        avg_ms = ms / calls
        b = algorithmic_bytes(name, P, Pv, R, T, HW, D=deg, acc=not args.autograd_grads,
                              defer_sh=defer_sh, precolor=not args.no_precolor,
                              views=len(my_cams))
        k = {"avg_ms": round(avg_ms, 4), "calls": int(calls), "bytes": int(b),
             "gbs": round(b / (avg_ms * 1e-3) / 1e9, 1)}
        if name in ("render_fwd", "render_bwd"):
            # (pixel, instance) candidate pairs per second: 256 pixels x R instances per view
            k["pair_candidates_per_s_G"] = round(256.0 * R / (avg_ms * 1e-3) / 1e9, 1)
        kernels[name] = k
    roofline = None
    if kernels and dom_stage in kernels:
        dom = dom_stage
        kd = kernels[dom]
        kd["timed_region"] = True
        achieved = kd["gbs"]
        traffic = None
        try:
            with open(args.pmc_file) as fh:
                pmc = json.load(fh)
            if pmc.get("workload") == args.workload and dom in pmc.get("kernels", {}):
                traffic = pmc["kernels"][dom].get("hbm_bytes_per_launch")
        except (OSError, ValueError):
            pass
        roofline = {"kernel": dom, "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                    "algorithmic_bytes": kd["bytes"], "avg_ms": kd["avg_ms"],
                    "timed_region_views_per_s": round(args.steps * n_views / dom_elapsed, 3)}
        try:
            with open(args.pmc_file) as fh:
                pmc = json.load(fh)
            pk = pmc.get("kernels", {}).get(dom, {})
            v = pk.get("valu_active_per_wave_cycle")
            if v is not None and pmc.get("workload") == args.workload:
                # SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES: the blend kernels are VALU/latency-bound
                roofline["valu_active_per_wave_cycle_pmc"] = v
            n_valu = pk.get("counters", {}).get("SQ_INSTS_VALU")
            if n_valu and pmc.get("workload") == args.workload:
                # VALU issue roofline: CDNA4's SIMDs are 32 lanes wide, so a SIMD issues one wave64
                # VALU instruction per 2 cycles (MI355X_MICROARCH.md, Wave scheduling); 256 CUs x 4
                # SIMDs at the 2.4 GHz peak engine clock
                peak = 256 * 4 * 2.4e9 / 2.0
                roofline["valu_issue_frac_pmc"] = round(n_valu / (kd["avg_ms"] * 1e-3) / peak, 4)
        except (OSError, ValueError):
            pass

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.cpu_baseline_views > 0:
        cpu = cpu_baseline(model, cams_all[: args.cpu_baseline_views], dimg, ddep, dfeat, deg)

    if rank == 0:
        line = {
            "metric": "rasterized views/sec (fwd+bwd)",
            "value": round(value, 3),
            "unit": "views/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": "synthetic (seeded Gaussians + LLFF-style cameras, SURVEY.md 8(d))",
            "config": {"workload": args.workload, "gaussians": P, "width": W, "height": H,
                       "sh_degree": deg, "views_per_gpu": args.views_per_gpu,
                       "views_per_step": n_views, "outputs": "rgb+depth+alpha+feature",
                       "parallelism": f"camera-sharded dp{world}",
                       "raster_path": ("fused" if os.environ.get("GSR_FUSED", "1") != "0"
                                       else "unfused"),
                       "grad_mode": "autograd" if args.autograd_grads else "into_leaves",
                       "view_streams": views.depth,
                       "sh_grads": "deferred (one flush per step)" if defer_sh else "per view",
                       "sh_colour": "per view" if args.no_precolor else "multi-view pre-pass",
                       "num_rendered_mean": int(R), "visible_mean": int(Pv), "tiles": T},
            "roofline": roofline,
            "cpu_baseline": cpu,
            "kernels": kernels,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def cpu_baseline(model, cams, dimg, ddep, dfeat, deg):
    """The CPU restatement (oracle/, single-threaded C) on a bounded sample of the same workload:
    `len(cams)` full views (forward + backward).  Rank 0 at N = 1 only."""
    try:
        from oracle.oracle import OracleRaster, build
        build()
    except Exception as exc:  # pragma: no cover - reported, not fatal
        return {"value": None, "error": repr(exc)[:200]}
    with torch.no_grad():
        xyz = model.get_xyz.detach().cpu().numpy()
        kw_common = dict(
            means3D=xyz, opacities=model.get_opacity.detach().cpu().numpy(),
            shs=model.get_features.detach().cpu().numpy(), sh_degree=deg,
            scales=model.get_scaling.detach().cpu().numpy(),
            rotations=model.get_rotation.detach().cpu().numpy(),
            shs_language=model.get_language_feature.detach().cpu().numpy(), include_feature=True,
            bg=np.zeros(3, np.float32))
        dimg_n, ddep_n, dfeat_n = (t.detach().cpu().numpy() for t in (dimg, ddep, dfeat))
    t0 = time.perf_counter()
    for cam in cams:
        orc = OracleRaster(viewmatrix=cam.world_view_transform.cpu().numpy(),
                           projmatrix=cam.full_proj_transform.cpu().numpy(),
                           campos=cam.camera_center.cpu().numpy(),
                           tanfovx=math.tan(cam.FoVx * 0.5), tanfovy=math.tan(cam.FoVy * 0.5),
                           image_height=cam.image_height, image_width=cam.image_width, **kw_common)
        orc.backward(dimg_n, ddep_n, None, dfeat_n)
        del orc
    dt = time.perf_counter() - t0
    return {"value": round(len(cams) / dt, 4), "unit": "views/s", "cores": 1, "kind": "port",
            "sample": f"{len(cams)} full views (fwd+bwd) of the same workload on the oracle "
                      f"(single-threaded C restatement), {dt:.1f} s",
            "cpu": platform.processor() or platform.machine()}


if __name__ == "__main__":
    main()
