"""Train-step GPU busy fraction: K batched train steps (gsr_amd.trainer.train_step_views, the
bench's train_step leg) after K identical warm-up steps, so the last half of a rocprofv3 kernel
trace is the timed half (scripts/trace_busy.py <dir> <n>).  Also prints the host time per step."""
import os, sys, time
ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "sdp-gs_amd")); sys.path.insert(0, ROOT)
import torch
import diff_gaussian_rasterization as dgr
from gsr_amd import trainer
from gsr_amd.model import SplatModel
from gsr_amd.pipeline import ViewPipeline
from gsr_amd.synthetic import make_cameras, make_gaussians, training_targets

K = int(os.environ.get("STEPS", "5"))
dev = torch.device("cuda", 0)
model = SplatModel(make_gaussians(1_000_000, sh_degree=3, seed=0), device=dev)
cams = [c.to(dev) for c in make_cameras(6, 1008, 756, seed=0)]
targs = trainer.OptArgs()
trainer.make_trainable(model, targs)
gts, monos = training_targets(len(cams), 756, 1008, seed=2, device=dev)
bg = torch.zeros(3, device=dev)
dgr.grad_into_leaves(True)
views = ViewPipeline(dev, depth=int(os.environ.get("STREAMS", "3")), defer_sh=True, precolor=True)
for phase in ("warmup", "timed"):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(K):
        trainer.train_step_views(model, cams, gts, monos, bg, targs, 1 + i, 2.78, views)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"{phase}: host issue {1e3 * (t1 - t0) / K:.3f} ms/step, wall {1e3 * (t2 - t0) / K:.3f} ms/step",
          flush=True)
