"""Per-view work counters of the blend kernels (build with EXTRA=-DGSR_BLEND_STATS=1 into
sdp-gs_amd/build_stats and run with GSR_LIB_PATH pointing there): list entries per wave, entries
evaluated, entries with at least one contributing lane, contributing (pixel, splat) pairs."""
import ctypes, os, sys
ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "sdp-gs_amd")); sys.path.insert(0, ROOT)
import torch
from gsr_amd import _lib
from gsr_amd.model import SplatModel
from gsr_amd.synthetic import make_cameras, make_gaussians, upstream_grads
import diff_gaussian_rasterization as dgr
from gaussian_renderer import render
from bench import Pipe, Opt

L = _lib.load()
L.gsr_test_blend_stats.restype = ctypes.c_int
L.gsr_test_blend_stats.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
dgr.grad_into_leaves(True)
m = SplatModel(make_gaussians(1_000_000, sh_degree=3, seed=0), device="cuda")
cams = [c.to("cuda") for c in make_cameras(6, 1008, 756, seed=0)]
dimg, ddep, dfeat = upstream_grads(756, 1008, seed=1, device="cuda")
bg = torch.zeros(3, device="cuda")
buf = (ctypes.c_ulonglong * 16)()
for c in cams[:2]:
    pkg = render(c, m, Pipe(), bg, Opt())
    torch.autograd.backward([pkg["render"], pkg["depth"], pkg["feature"]], [dimg, ddep, dfeat])
torch.cuda.synchronize()
L.gsr_test_blend_stats(buf, 1)
pkg = render(cams[2], m, Pipe(), bg, Opt())
torch.autograd.backward([pkg["render"], pkg["depth"], pkg["feature"]], [dimg, ddep, dfeat])
torch.cuda.synchronize()
assert L.gsr_test_blend_stats(buf, 1) == 0
v = list(buf)
waves = v[8]  # BLEND_STAT(8) counts each wave once
R = dgr.LAST_STATS["num_rendered"]
print(f"R={R} waves={waves}")
print(f"fwd: list/wave={v[0]/waves:.1f} evaluated/wave={v[1]/waves:.1f} contrib-entries/wave={v[2]/waves:.1f} "
      f"lanes/contrib-entry={v[3]/max(v[2],1):.1f}")
print(f"bwd imbalance: busiest-wave entries x4 / all entries = {v[10]/max(v[9],1):.3f}")
print(f"bwd: list/wave={v[4]/waves:.1f} evaluated/wave={4*v[5]/waves:.1f} contrib-entries/wave={v[6]/waves:.1f} "
      f"lanes/contrib-entry={v[7]/max(v[6],1):.1f}")
n6 = max(v[6], 1)
print(f"bwd contributing lanes per entry: <=2 {v[11]/n6:.3f}  <=4 {v[12]/n6:.3f}  <=8 {v[13]/n6:.3f}  "
      f"<=16 {v[14]/n6:.3f}")
if os.environ.get("GSR_BLOCK_LISTS", "1") != "0":
    # block-list forward: [0] sum of the wave's longest group list, [1] sum of its four group
    # lists, [2] entries evaluated per group (the "fwd:" line above reads these slots)
    print(f"blk fwd: max-list/wave={v[0]/waves:.1f} group-lists/wave={v[1]/waves:.1f} evaluated/wave-step-slot={v[2]/waves:.1f}")
