"""Host cost of bench.py's train_step leg with negligible GPU work (P = 1000 Gaussians, 1008x756,
6 views, 3 streams, lag 1): wall time per view of gsr_amd.trainer.train_step_views, then a
cProfile of the same loop (top functions by own time).  usage: host_overhead_train.py [P]"""
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
from gsr_amd import _lib, trainer  # noqa: E402
from gsr_amd.model import SplatModel  # noqa: E402
from gsr_amd.pipeline import ViewPipeline  # noqa: E402
from gsr_amd.synthetic import make_cameras, make_gaussians, training_targets  # noqa: E402

P = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
if os.environ.get("MT") == "0":  # backward on the calling thread (no autograd device thread)
    torch.autograd.set_multithreading_enabled(False)
dgr.grad_into_leaves(True)
dev = torch.device("cuda", 0)
model = SplatModel(make_gaussians(P, sh_degree=3, seed=0), device=dev)
cams = [c.to(dev) for c in make_cameras(6, 1008, 756, seed=0)]
targs = trainer.OptArgs()
trainer.make_trainable(model, targs)
gts, monos = training_targets(6, 756, 1008, seed=2, device=dev)
bg = torch.zeros(3, device=dev)
vp = ViewPipeline(dev, depth=3)


def steps(n):
    for _ in range(n):
        trainer.train_step_views(model, cams, gts, monos, bg, targs, 1, 2.78, vp)


L = _lib.load()
headline = len(sys.argv) > 2 and sys.argv[2] == "headline"
if headline:  # bench.py's headline step instead: fixed upstream gradients, no loss / stats / Adam
    from bench import Opt, Pipe  # noqa: E402
    from gaussian_renderer import render  # noqa: E402
    from gsr_amd.synthetic import upstream_grads  # noqa: E402
    dimg, ddep, dfeat = upstream_grads(756, 1008, seed=1, device=dev)

    def steps(n):  # noqa: F811
        for _ in range(n):
            for p in model.parameters():
                p.grad = None
            vp.run(cams, lambda c: render(c, model, Pipe(), bg, Opt()), model=model,
                   bwd=lambda pkg: torch.autograd.backward(
                       [pkg["render"], pkg["depth"], pkg["feature"]], [dimg, ddep, dfeat]), lag=1)
ctimes = {}
if os.environ.get("CTIME"):  # wall time of every libgsr entry point called by the loop
    for name in [n for n in dir(L) if n.startswith("gsr_") and not n.startswith("gsr_test")]:
        fn = getattr(L, name)

        def timed(*a, _fn=fn, _n=name):
            t = time.perf_counter()
            r = _fn(*a)
            ctimes[_n] = ctimes.get(_n, 0.0) + time.perf_counter() - t
            return r
        setattr(L, name, timed)
steps(10)
torch.cuda.synchronize()
ctimes.clear()
L.gsr_test_host_wait_ms(1)
t0 = time.perf_counter()
steps(50)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / 300 * 1e3
print(f"P={P} {'headline' if headline else 'train'} step per view {dt:.3f} ms, of which "
      f"read-back wait {L.gsr_test_host_wait_ms(1) / 300:.3f} ms", flush=True)
for k, v in sorted(ctimes.items(), key=lambda kv: -kv[1]):
    print(f"  {k}: {v / 300 * 1e3:.4f} ms per view")
pr = cProfile.Profile()
pr.enable()
steps(50)
torch.cuda.synchronize()
pr.disable()
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(30)
print(s.getvalue()[:8000])
