"""Host cost of bench.py's step with negligible GPU work (P = 1000 Gaussians, 1008x756, 6 views,
3 streams, lag 1, colour pre-pass, deferred SH, grad-into-leaves): wall time per view, then a
cProfile of the same loop (top functions by own time)."""
import cProfile
import io
import os
import pstats
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

dgr.grad_into_leaves(True)
dev = torch.device("cuda", 0)
m = SplatModel(make_gaussians(1000, sh_degree=3, seed=0), device=dev)
cams = [c.to(dev) for c in make_cameras(6, 1008, 756, seed=0)]
dimg, ddep, dfeat = upstream_grads(756, 1008, seed=1, device=dev)
bg = torch.zeros(3, device=dev)
vp = ViewPipeline(dev, depth=3)


def fwd(cam):
    return render(cam, m, Pipe(), bg, Opt())


def bwd(pkg):
    torch.autograd.backward([pkg["render"], pkg["depth"], pkg["feature"]], [dimg, ddep, dfeat])


def steps(n):
    for _ in range(n):
        for p in m.parameters():
            p.grad = None
        vp.run(cams, fwd, model=m, bwd=bwd, lag=1)


steps(20)
torch.cuda.synchronize()
t0 = time.perf_counter()
steps(100)
torch.cuda.synchronize()
print(f"host+tiny GPU per view: {(time.perf_counter() - t0) / 600 * 1e3:.3f} ms")
pr = cProfile.Profile()
pr.enable()
steps(100)
torch.cuda.synchronize()
pr.disable()
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(28)
print(s.getvalue()[:7000])
