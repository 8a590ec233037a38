"""Host issue time of the pieces of one training view (no synchronisation inside the loop): what
the Python / autograd / ctypes layers cost per view on top of the kernels."""
import os, sys, time
ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "sdp-gs_amd")); sys.path.insert(0, ROOT)
import torch
import diff_gaussian_rasterization as dgr
from gaussian_renderer import render
from gsr_amd import trainer
from gsr_amd.model import SplatModel
from gsr_amd.synthetic import make_cameras, make_gaussians, training_targets

P = int(os.environ.get("P", "0"))  # 0 Gaussians: pure host cost
dev = torch.device("cuda", 0)
model = SplatModel(make_gaussians(max(P, 1000), sh_degree=3, seed=0), device=dev)
cam = make_cameras(1, 1008, 756, seed=0)[0].to(dev)
targs = trainer.OptArgs()
trainer.make_trainable(model, targs)
gts, monos = training_targets(1, 756, 1008, seed=2, device=dev)
bg = torch.zeros(3, device=dev)
dgr.grad_into_leaves(True)
acc = {}
def tick(k, t):
    acc[k] = acc.get(k, 0.0) + t
for it in range(2):
    acc.clear()
    n = 100
    for _ in range(n):
        a = time.perf_counter()
        pkg = render(cam, model, trainer._Pipe(), bg, targs)
        b = time.perf_counter()
        loss = trainer._view_loss(pkg, gts[0], monos[0], targs)
        c = time.perf_counter()
        loss.backward()
        d = time.perf_counter()
        with torch.no_grad():
            model.update_densification_stats(pkg["viewspace_points"], pkg["radii"], pkg["visibility_filter"])
        e = time.perf_counter()
        model.optimizer.step()
        model.optimizer.zero_grad(set_to_none=True)
        f = time.perf_counter()
        tick("render", b - a); tick("loss fwd", c - b); tick("backward", d - c); tick("stats", e - d)
        tick("adam+zero", f - e)
    torch.cuda.synchronize()
    print({k: round(1e3 * v / n, 3) for k, v in acc.items()}, "ms per view", flush=True)
