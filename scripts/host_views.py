"""Host-side cost of the multi-view step (bench.py's headline workload): per step the wall time,
the host time inside the forward / backward C calls, the host time waiting for read-backs, and the
Python time around them.  usage: python scripts/host_views.py [steps] [streams] [P]
(a small P, e.g. 1000, leaves only the host costs: the GPU work per step is then negligible)"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "sdp-gs_amd"))
import torch  # noqa: E402

import diff_gaussian_rasterization as dgr  # noqa: E402
from gaussian_renderer import render_views  # noqa: E402
from gsr_amd import _lib  # noqa: E402
from gsr_amd.model import SplatModel  # noqa: E402
from gsr_amd.pipeline import ViewPipeline  # noqa: E402
from gsr_amd.synthetic import make_cameras, make_gaussians, upstream_grads  # noqa: E402
from tests.fused_ref import Opt, Pipe  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
nstreams = int(sys.argv[2]) if len(sys.argv) > 2 else 4
P = int(sys.argv[3]) if len(sys.argv) > 3 else 1_000_000
dev = torch.device("cuda", 0)
dgr.grad_into_leaves(True)
m = SplatModel(make_gaussians(P, sh_degree=3, seed=0), device=dev)
cams = [c.to(dev) for c in make_cameras(12, 1008, 756, seed=0)]
dimg, ddep, dfeat = upstream_grads(756, 1008, seed=1, device=dev)
bg = torch.zeros(3, device=dev)
vp = ViewPipeline(dev, depth=nstreams)
L = _lib.load()
rows = []


def fn(cs, strs):
    t0 = time.perf_counter()
    pkgs = render_views(cs, m, Pipe(), bg, Opt(), streams=strs)
    t1 = time.perf_counter()
    st = pkgs[0]["views"]
    V = len(pkgs)
    torch.autograd.backward([st["render"], st["depth"], st["feature"]],
                            [dimg.expand(V, *dimg.shape), ddep.expand(V, *ddep.shape),
                             dfeat.expand(V, *dfeat.shape)])
    t2 = time.perf_counter()
    return t0, t1, t2


for k in range(steps + 3):
    for p in m.parameters():
        p.grad = None
    L.gsr_test_host_wait_ms(1)
    torch.cuda.synchronize()
    ta = time.perf_counter()
    t0, t1, t2 = vp.run_views([cams[(6 * k + i) % 12] for i in range(6)], fn, model=m)
    tb = time.perf_counter()
    torch.cuda.synchronize()
    tc = time.perf_counter()
    if k >= 3:
        rows.append((tc - ta, tb - ta, t1 - t0, dgr.LAST_STATS["views_fwd_host_s"],
                     t2 - t1, dgr.LAST_STATS["views_bwd_host_s"], L.gsr_test_host_wait_ms(0)))
import numpy as np  # noqa: E402
r = np.median(np.array(rows), axis=0) * np.array([1e3, 1e3, 1e3, 1e3, 1e3, 1e3, 1.0])
print(f"median ms per step: wall {r[0]:.3f}  host issue {r[1]:.3f}  render_views {r[2]:.3f} "
      f"(C call {r[3]:.3f}, of which read-back waits {r[6]:.3f})  backward {r[4]:.3f} "
      f"(C call {r[5]:.3f})")
