"""Host-side cost of one view's render() + backward() without GPU work (P = 0 Gaussians): the
Python/ctypes/autograd overhead that every view pays on top of its kernels."""
import os, sys, time
ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "sdp-gs_amd")); sys.path.insert(0, ROOT)
import torch
from gsr_amd.model import SplatModel
from gsr_amd.synthetic import make_cameras, make_gaussians, upstream_grads
import diff_gaussian_rasterization as dgr
from gaussian_renderer import render
from bench import Pipe, Opt

dgr.grad_into_leaves(True)
for P in (0, 1000):
    m = SplatModel(make_gaussians(max(P, 1), sh_degree=3, seed=0), device="cuda")
    if P == 0:
        for n in ("_xyz", "_features_dc", "_features_rest", "_opacity", "_scaling", "_rotation", "_language_feature"):
            t = getattr(m, n)
            setattr(m, n, t[:0].detach().clone().requires_grad_(True))
    cam = make_cameras(1, 1008, 756, seed=0)[0].to("cuda")
    dimg, ddep, dfeat = upstream_grads(756, 1008, seed=1, device="cuda")
    bg = torch.zeros(3, device="cuda")
    for it in range(3):
        t0 = time.perf_counter(); n = 200
        tf = tb = 0.0
        for _ in range(n):
            a = time.perf_counter()
            pkg = render(cam, m, Pipe(), bg, Opt())
            b = time.perf_counter()
            torch.autograd.backward([pkg["render"], pkg["depth"], pkg["feature"]], [dimg, ddep, dfeat])
            c = time.perf_counter()
            tf += b - a; tb += c - b
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        print(f"P={P} per view: total {1e3*el/n:.3f} ms, render {1e3*tf/n:.3f} ms, backward {1e3*tb/n:.3f} ms")
