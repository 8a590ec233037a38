"""cProfile of the per-view host path (render + backward) at P = 1000 after warm-up."""
import cProfile, os, pstats, sys, io
ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "sdp-gs_amd")); sys.path.insert(0, ROOT)
import torch
from gsr_amd.model import SplatModel
from gsr_amd.synthetic import make_cameras, make_gaussians, upstream_grads
import diff_gaussian_rasterization as dgr
from gaussian_renderer import render
from bench import Pipe, Opt

dgr.grad_into_leaves(True)
m = SplatModel(make_gaussians(1000, sh_degree=3, seed=0), device="cuda")
cam = make_cameras(1, 1008, 756, seed=0)[0].to("cuda")
dimg, ddep, dfeat = upstream_grads(756, 1008, seed=1, device="cuda")
bg = torch.zeros(3, device="cuda")
def views(n):
    for _ in range(n):
        pkg = render(cam, m, Pipe(), bg, Opt())
        torch.autograd.backward([pkg["render"], pkg["depth"], pkg["feature"]], [dimg, ddep, dfeat])
views(50); torch.cuda.synchronize()
pr = cProfile.Profile(); pr.enable(); views(500); torch.cuda.synchronize(); pr.disable()
s = io.StringIO(); pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(30); print(s.getvalue()[:6000])
