"""Host-side timeline of the bench step (multi-view call): Python perf_counter marks around the
pre-pass, the forward call, the backward call and the flush, plus the library's own marks
(GSR_HOST_TRACE=1: per group w/r = read-back wait begin/end, A = binning allocation, b = per-view
bin setup, a = duplicate issued, t = tile sort issued, f = blend issued, B = per-view blended),
printed for the last steps -- no synchronisation inside the steps.  Compare with a kernel trace
(scripts/trace_timeline.py) to see where the GPU waits for the host."""
import os
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "sdp-gs_amd"))
sys.path.insert(0, ROOT)
os.environ.setdefault("GSR_HOST_TRACE", "1")
import torch  # noqa: E402

import diff_gaussian_rasterization as dgr  # noqa: E402
from bench import Opt, Pipe  # noqa: E402
from gaussian_renderer import render_views  # noqa: E402
from gsr_amd.model import SplatModel  # noqa: E402
from gsr_amd.pipeline import ViewPipeline  # noqa: E402
from gsr_amd.synthetic import make_cameras, make_gaussians, upstream_grads  # noqa: E402

dgr.grad_into_leaves(True)
dev = torch.device("cuda", 0)
model = SplatModel(make_gaussians(1_000_000, sh_degree=3, seed=0), device=dev)
cams = [c.to(dev) for c in make_cameras(12, 1008, 756, seed=0)]
dimg, ddep, dfeat = upstream_grads(756, 1008, seed=1, device=dev)
bg = torch.zeros(3, device=dev)
views = ViewPipeline(dev, depth=4)
marks = []


def mark(what):
    marks.append((what, time.perf_counter()))


def fn(cs, strs):
    mark("fwd_call")
    pkgs = render_views(cs, model, Pipe(), bg, Opt(), streams=strs)
    mark("fwd_ret")
    st = pkgs[0]["views"]
    V = len(pkgs)
    torch.autograd.backward([st["render"], st["depth"], st["feature"]],
                            [dimg.expand(V, *dimg.shape), ddep.expand(V, *ddep.shape),
                             dfeat.expand(V, *dfeat.shape)])
    mark("bwd_ret")


for k in range(8):
    for p in model.parameters():
        p.grad = None
    marks.clear()
    mark("step")
    views.run_views(cams[(6 * k) % 12:(6 * k) % 12 + 6], fn, model=model)
    mark("end")
    if k >= 5:
        t0 = marks[0][1]
        print("step", k, " ".join(f"{w}={1e6 * (t - t0):.0f}" for w, t in marks), flush=True)
torch.cuda.synchronize()
