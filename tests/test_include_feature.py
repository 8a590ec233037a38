"""render() / render_views() with opt.include_feature = False.

The reference then passes the colours again as the language-feature input
(gaussian_renderer/__init__.py:296-298: language_feature_precomp = colors_precomp, settings
include_feature=True), so its "feature" output is the colour blend with a zero background and the
feature's gradient reaches the SH leaves through colors_precomp.  With convert_SHs_python = False
colors_precomp is None and the feature channels render as zeros.  Both GSR_FUSED settings must
return the same tensors, and the colour-feature case must match the CPU oracle fed
language_feature_precomp = colors.
"""
import math

import numpy as np
import pytest
import torch

from gsr_amd.model import SplatModel
from gsr_amd.synthetic import make_cameras, make_gaussians, upstream_grads
from oracle.oracle import OracleRaster

pytestmark = pytest.mark.gpu

W, H, P = 200, 150, 20000


class Pipe:
    def __init__(self, sh_py):
        self.convert_SHs_python = sh_py
        self.compute_cov3D_python = False
        self.debug = False
        self.use_confidence = False


class OptNoFeature:
    include_feature = False


def _run(render_fn, cams, sh_py, fused, monkeypatch, multi=False):
    """One forward + backward of fixed upstream gradients (image, depth, feature) per camera;
    returns per-view outputs, the colours' gradient (Python colour path) and the leaf grads."""
    from gaussian_renderer import render_views
    monkeypatch.setenv("GSR_FUSED", fused)
    m = SplatModel(make_gaussians(P, seed=5), device="cuda")
    bg = torch.tensor([0.1, 0.2, 0.3], device="cuda")
    dimg, ddep, dfeat = upstream_grads(H, W, seed=3, device="cuda")
    pkgs = (render_views(cams, m, Pipe(sh_py), bg, OptNoFeature()) if multi else
            [render_fn(c, m, Pipe(sh_py), bg, OptNoFeature()) for c in cams])
    for pkg in pkgs:
        if pkg["color"] is not None:
            pkg["color"].retain_grad()
    loss = sum((p["render"] * dimg).sum() + (p["depth"] * ddep).sum() + (p["feature"] * dfeat).sum()
               for p in pkgs)
    loss.backward()
    torch.cuda.synchronize()
    outs = [{k: pkg[k].detach().clone() for k in ("render", "depth", "alpha", "feature", "radii")}
            for pkg in pkgs]
    cgrads = [None if p["color"] is None else p["color"].grad.clone() for p in pkgs]
    leaves = {n: getattr(m, n).grad.clone() for n in ("_xyz", "_features_dc", "_features_rest",
                                                      "_opacity", "_scaling", "_rotation")}
    return m, outs, cgrads, leaves, (dimg, ddep, dfeat)


@pytest.mark.parametrize("multi", [False, True])
@pytest.mark.parametrize("sh_py", [True, False])
def test_fused_setting_does_not_change_outputs(monkeypatch, sh_py, multi):
    from gaussian_renderer import render
    cams = [c.to("cuda") for c in make_cameras(3, W, H, seed=4)]
    _, a, _, ga, _ = _run(render, cams, sh_py, "1", monkeypatch, multi)
    _, b, _, gb, _ = _run(render, cams, sh_py, "0", monkeypatch, multi)
    for x, y in zip(a, b):
        assert torch.equal(x["radii"], y["radii"])
        for k in ("render", "depth", "alpha", "feature"):
            # the fused activations equal torch's bit for bit; blend sums may differ by ulps
            torch.testing.assert_close(x[k], y[k], atol=2e-6, rtol=0)
        if not sh_py:
            assert not torch.any(x["feature"]), "no colours_precomp: zero feature channels"
    for n in ga:
        scale = float(gb[n].abs().max()) + 1e-12
        assert float((ga[n] - gb[n]).abs().max()) <= 2e-3 * scale, n


def test_colour_feature_matches_oracle(monkeypatch):
    """sh_py = True: feature == the oracle's blend of language_feature_precomp = colors (bg 0),
    and the colours' gradient == the oracle's colour + feature gradients (the same tensor)."""
    from gaussian_renderer import render
    cams = [c.to("cuda") for c in make_cameras(2, W, H, seed=4)]
    m, outs, cgrads, _, (dimg, ddep, dfeat) = _run(render, cams, True, "1", monkeypatch)
    with torch.no_grad():
        op = torch.sigmoid(m._opacity).cpu().numpy()
        sc = torch.exp(m._scaling).cpu().numpy()
        rot = torch.nn.functional.normalize(m._rotation).cpu().numpy()
    for cam, out, cg in zip(cams, outs, cgrads):
        pkg = render(cam, m, Pipe(True), torch.tensor([0.1, 0.2, 0.3], device="cuda"),
                     OptNoFeature())
        colors = pkg["color"].detach().cpu().numpy()
        orc = OracleRaster(
            means3D=m._xyz.detach().cpu().numpy(), opacities=op,
            viewmatrix=cam.world_view_transform.cpu().numpy(),
            projmatrix=cam.full_proj_transform.cpu().numpy(),
            campos=cam.camera_center.cpu().numpy(), tanfovx=math.tan(cam.FoVx * 0.5),
            tanfovy=math.tan(cam.FoVy * 0.5), image_height=H, image_width=W,
            bg=np.array([0.1, 0.2, 0.3], np.float32), colors_precomp=colors, scales=sc,
            rotations=rot, language_feature_precomp=colors, include_feature=True)
        assert np.array_equal(out["radii"].cpu().numpy(), orc.radii)
        for k, ref in (("render", orc.color), ("depth", orc.depth), ("feature", orc.feature)):
            assert float(np.abs(out[k].cpu().numpy() - ref).max()) <= 1e-5, k
        # the feature is the colour blend with a zero background
        assert float(np.abs(orc.feature - (orc.color - orc.final_T()[None] *
                                           np.array([0.1, 0.2, 0.3], np.float32)[:, None, None])
                            ).max()) <= 1e-5
        og = orc.backward(dimg.cpu().numpy(), ddep.cpu().numpy(), None, dfeat.cpu().numpy())
        ref = og["colors"].astype(np.float64) + og["language_feature"]
        got = cg.cpu().numpy().astype(np.float64)
        assert float(np.abs(got - ref).max()) <= 1e-5 * float(np.abs(ref).max())
