#!/usr/bin/env python3
"""Per-step wall times of the headline step (bench.py's workload: 1M Gaussians, 6 views at
1008x756, 3 view streams, grad-into-leaves, deferred SH, colour pre-pass), each step bracketed by
torch.cuda.synchronize(): the distribution shows whether a slow bench run is slow throughout or
has a few stalled steps (host scheduling).  usage: step_times.py [steps] [lag] [streams]"""
import os
import statistics
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "sdp-gs_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import diff_gaussian_rasterization as dgr  # noqa: E402
from bench import Opt, Pipe  # noqa: E402
from gaussian_renderer import render  # noqa: E402
from gsr_amd.model import SplatModel  # noqa: E402
from gsr_amd.pipeline import ViewPipeline  # noqa: E402
from gsr_amd.synthetic import make_cameras, make_gaussians, upstream_grads  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 40
lag = int(sys.argv[2]) if len(sys.argv) > 2 else 0
depth = int(sys.argv[3]) if len(sys.argv) > 3 else 3
dgr.grad_into_leaves(True)
dev = torch.device("cuda", 0)
model = SplatModel(make_gaussians(1_000_000, sh_degree=3, seed=0), device=dev)
cams = [c.to(dev) for c in make_cameras(6, 1008, 756, seed=0)]
dimg, ddep, dfeat = upstream_grads(756, 1008, seed=1, device=dev)
bg = torch.zeros(3, device=dev)
views = ViewPipeline(dev, depth=depth)


def fwd(cam):
    return render(cam, model, Pipe(), bg, Opt())


def bwd(pkg):
    torch.autograd.backward([pkg["render"], pkg["depth"], pkg["feature"]], [dimg, ddep, dfeat])


def step():
    for p in model.parameters():
        p.grad = None
    if lag:
        views.run(cams, fwd, model=model, bwd=bwd, lag=lag)
    else:
        views.run(cams, lambda c: bwd(fwd(c)), model=model)


for _ in range(3):
    step()
torch.cuda.synchronize()
ts = []
for _ in range(steps):
    t0 = time.perf_counter()
    step()
    torch.cuda.synchronize()
    ts.append(1000.0 * (time.perf_counter() - t0))
ts_sorted = sorted(ts)
print(f"lag {lag} streams {depth}: median {statistics.median(ts):.3f} ms  min {ts_sorted[0]:.3f}  "
      f"p90 {ts_sorted[int(0.9 * len(ts)) - 1]:.3f}  max {ts_sorted[-1]:.3f}  "
      f"views/s at median {6000.0 / statistics.median(ts):.0f}")
print("steps:", " ".join(f"{t:.2f}" for t in ts))
