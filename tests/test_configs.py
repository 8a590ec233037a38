"""BASELINE configs 1 and 2 on the HIP path against the oracle.

Config 1: 10k synthetic Gaussians, one 400x400 camera, forward only, render() with the reference's
default flags (arguments/__init__.py:66-72: convert_SHs_python=True, so SH degree 0 colours come
from render()'s Python pre-pass in the reference, gaussian_renderer/__init__.py:269-287) -- run
under torch.no_grad() as render.py does (render.py:84), through both the fused entry point render()
takes by default and the reference operator API (GSR_FUSED=0: torch getters + eval_sh + the
vendored-API rasterizer call).
Config 2's colors_precomp variant: 100k Gaussians, 800x800, fwd + bwd with
precomputed colours (and precomputed language features), full size.
"""
import math
import os

import numpy as np
import pytest
import torch

from oracle.oracle import OracleRaster
from scenes import scene
from test_gpu_parity import FWD_ATOL, compare

pytestmark = pytest.mark.gpu


class _Pipe:  # arguments/__init__.py:66-72
    convert_SHs_python = True
    compute_cov3D_python = False
    debug = False
    use_confidence = False


class _Opt:
    include_feature = True


@pytest.mark.parametrize("fused", ["1", "0"])
def test_config1_forward_through_render(fused, monkeypatch):
    from fused_ref import kernel_activations
    from gaussian_renderer import render
    from gsr_amd.model import SplatModel
    from gsr_amd.synthetic import make_cameras, make_gaussians
    monkeypatch.setenv("GSR_FUSED", fused)
    m = SplatModel(make_gaussians(10_000, sh_degree=3, seed=0), device="cuda", active_sh_degree=0)
    cam = make_cameras(1, 400, 400, seed=0)[0].to("cuda")
    bg = torch.zeros(3, device="cuda")
    with torch.no_grad():
        pkg = render(cam, m, _Pipe(), bg, _Opt())
        torch.cuda.synchronize()
        if fused == "1":
            op, sc, rot = (t.cpu().numpy() for t in kernel_activations(m))
        else:  # the getters render() used
            op, sc, rot = (t.cpu().numpy() for t in (m.get_opacity, m.get_scaling, m.get_rotation))
        shs = torch.cat((m._features_dc, m._features_rest), 1).cpu().numpy()
    orc = OracleRaster(
        means3D=m._xyz.detach().cpu().numpy(), opacities=op,
        viewmatrix=cam.world_view_transform.cpu().numpy(),
        projmatrix=cam.full_proj_transform.cpu().numpy(), campos=cam.camera_center.cpu().numpy(),
        tanfovx=math.tan(cam.FoVx * 0.5), tanfovy=math.tan(cam.FoVy * 0.5), image_height=400,
        image_width=400, bg=np.zeros(3, np.float32), sh_degree=0, shs=shs, scales=sc,
        rotations=rot, shs_language=m._language_feature.detach().cpu().numpy(),
        include_feature=True)
    np.testing.assert_array_equal(pkg["radii"].cpu().numpy(), orc.radii)
    for key, ref in (("render", orc.color), ("depth", orc.depth), ("alpha", orc.alpha),
                     ("feature", orc.feature)):
        np.testing.assert_allclose(pkg[key].cpu().numpy(), ref, atol=FWD_ATOL, rtol=0,
                                   err_msg=f"{key} (GSR_FUSED={fused})")
    assert (pkg["visibility_filter"].cpu().numpy() == (orc.radii > 0)).all()
    assert float(np.abs(orc.color).max()) > 0


def test_config2_full_size_colors_precomp_parity():
    """BASELINE config 2 at full size with precomputed colours and language features."""
    compare(scene(P=100_000, W=800, H=800, seed=0, cam=0, mode="colors", feature="precomp"))
