"""Host cost of bench.py's multi-view step with negligible GPU work (P = 1000 Gaussians, 1008x756,
6 views, the colour pre-pass, SH gradients in the multi-view backward, grad-into-leaves): wall
time per step, the host time of its phases (pre-pass issue, forward call, backward call), then a
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
from gaussian_renderer import render_views  # noqa: E402
from gsr_amd.model import SplatModel  # noqa: E402
from gsr_amd.pipeline import ViewPipeline  # noqa: E402
from gsr_amd.synthetic import make_cameras, make_gaussians, upstream_grads  # noqa: E402

P = int(os.environ.get("HOST_P", "1000"))
dgr.grad_into_leaves(True)
dev = torch.device("cuda", 0)
m = SplatModel(make_gaussians(P, sh_degree=3, seed=0), device=dev)
cams = [c.to(dev) for c in make_cameras(6, 1008, 756, seed=0)]
dimg, ddep, dfeat = upstream_grads(756, 1008, seed=1, device=dev)
bg = torch.zeros(3, device=dev)
vp = ViewPipeline(dev, depth=4, defer_sh=True, precolor=True)
phase = {"fwd": 0.0, "bwd": 0.0, "pre": 0.0, "n": 0}


def all_views(cs, strs):
    t0 = time.perf_counter()
    pkgs = render_views(cs, m, Pipe(), bg, Opt(), streams=strs)
    t1 = time.perf_counter()
    st = pkgs[0]["views"]
    V = len(pkgs)
    torch.autograd.backward([st["render"], st["depth"], st["feature"]],
                            [dimg.expand(V, *dimg.shape), ddep.expand(V, *ddep.shape),
                             dfeat.expand(V, *dfeat.shape)])
    t2 = time.perf_counter()
    phase["fwd"] += t1 - t0
    phase["bwd"] += t2 - t1
    phase["n"] += 1


def steps(n):
    for _ in range(n):
        for p in m.parameters():
            p.grad = None
        t0 = time.perf_counter()
        vp.run_views(cams, all_views, model=m)
        phase["pre"] += time.perf_counter() - t0


from gsr_amd import _lib  # noqa: E402
steps(20)
torch.cuda.synchronize()
for k in phase:
    phase[k] = 0
_lib.load().gsr_test_host_wait_ms(1)
t0 = time.perf_counter()
steps(100)
torch.cuda.synchronize()
el = time.perf_counter() - t0
wait = _lib.load().gsr_test_host_wait_ms(1)
n = phase["n"]
print(f"P={P}: wall per step {el / 100 * 1e3:.3f} ms; host per step: forward call "
      f"{phase['fwd'] / n * 1e3:.3f} ms (of it waiting for the read-backs {wait / n:.3f} ms), "
      f"backward call {phase['bwd'] / n * 1e3:.3f} ms, run_views total {phase['pre'] / n * 1e3:.3f} ms")
pr = cProfile.Profile()
pr.enable()
steps(50)
torch.cuda.synchronize()
pr.disable()
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(30)
print(s.getvalue()[:8000])
