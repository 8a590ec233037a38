"""render() drop-in (gaussian_renderer/__init__.py:209-338) on the HIP path: the pipeline flags
select equivalent computations, gradients reach every GaussianModel parameter."""
import numpy as np
import pytest
import torch

from gsr_amd.model import SplatModel
from gsr_amd.synthetic import make_cameras, make_gaussians

pytestmark = pytest.mark.gpu


class Pipe:
    def __init__(self, sh_py=True, cov_py=False, conf=False):
        self.convert_SHs_python = sh_py
        self.compute_cov3D_python = cov_py
        self.debug = False
        self.use_confidence = conf


class Opt:
    include_feature = True


def _setup(P=20000, W=200, H=150):
    from gaussian_renderer import render
    m = SplatModel(make_gaussians(P, seed=5), device="cuda")
    cam = make_cameras(3, W, H, seed=1)[2].to("cuda")
    return render, m, cam


def test_render_dict_and_grads():
    render, m, cam = _setup()
    pkg = render(cam, m, Pipe(sh_py=False), torch.zeros(3, device="cuda"), Opt())
    assert set(pkg) == {"render", "depth", "alpha", "opacity", "feature", "viewspace_points",
                        "visibility_filter", "radii", "color"}
    assert pkg["render"].shape == (3, 150, 200) and pkg["depth"].shape == (1, 150, 200)
    loss = pkg["render"].mean() + pkg["depth"].mean() + pkg["feature"].abs().mean()
    loss.backward()
    for p in m.parameters():
        assert p.grad is not None and torch.isfinite(p.grad).all() and p.grad.abs().sum() > 0
    vs = pkg["viewspace_points"].grad
    assert vs is not None and vs[:, :2].abs().sum() > 0 and torch.all(vs[:, 2] == 0)


def test_python_and_kernel_sh_paths_agree():
    render, m, cam = _setup()
    bg = torch.tensor([0.1, 0.2, 0.3], device="cuda")
    a = render(cam, m, Pipe(sh_py=True), bg, Opt())
    b = render(cam, m, Pipe(sh_py=False), bg, Opt())
    assert torch.equal(a["radii"], b["radii"])
    torch.testing.assert_close(a["render"], b["render"], atol=2e-6, rtol=0)
    torch.testing.assert_close(a["feature"], b["feature"], atol=2e-6, rtol=0)
    torch.testing.assert_close(a["depth"], b["depth"], atol=0, rtol=0)


def test_python_covariance_path_agrees():
    render, m, cam = _setup()
    bg = torch.zeros(3, device="cuda")
    a = render(cam, m, Pipe(sh_py=False, cov_py=False), bg, Opt())
    b = render(cam, m, Pipe(sh_py=False, cov_py=True), bg, Opt())
    same = (a["radii"] == b["radii"]).float().mean().item()
    assert same > 0.999
    assert (a["render"] - b["render"]).abs().mean().item() < 1e-5
