"""Host-side pieces of the path (CPU): SH evaluation, activations, settings API."""
import os

import numpy as np
import pytest
import torch

from gsr_amd.sh import eval_sh
from gsr_amd.synthetic import make_gaussians
from gsr_amd.model import SplatModel, build_covariance_from_scaling_rotation

GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.mark.parametrize("deg", [0, 1, 2, 3])
def test_eval_sh_matches_reference_golden(deg):
    d = np.load(os.path.join(GOLD, "sh_golden.npz"))
    xyz, campos = torch.tensor(d["xyz"]), torch.tensor(d["campos"])
    feats = torch.tensor(d["features"])
    dir_pp = xyz - campos.repeat(xyz.shape[0], 1)
    dirs = dir_pp / dir_pp.norm(dim=1, keepdim=True)
    out = eval_sh(deg, feats.transpose(1, 2).view(-1, 3, 16), dirs)
    np.testing.assert_allclose(out.numpy(), d[f"eval_sh_deg{deg}"], atol=1e-6, rtol=0)


def test_language_feature_prepass_matches_reference_golden():
    d = np.load(os.path.join(GOLD, "sh_golden.npz"))
    xyz, campos = torch.tensor(d["xyz"]), torch.tensor(d["campos"])
    lang = torch.tensor(d["language_feature"])
    dir_pp = xyz - campos.repeat(xyz.shape[0], 1)
    dirs = dir_pp / dir_pp.norm(dim=1, keepdim=True)
    s2l = eval_sh(0, lang.view(-1, 3, 1), dirs)
    f = s2l / (s2l.norm(dim=-1, keepdim=True) + 1e-9)
    np.testing.assert_allclose(f.numpy(), d["language_feature_precomp"], atol=1e-6, rtol=0)


def test_model_getters_and_covariance():
    g = make_gaussians(500, seed=3)
    m = SplatModel(g, device="cpu")
    assert torch.allclose(m.get_scaling, torch.exp(g.scaling))
    assert torch.allclose(m.get_rotation.norm(dim=1), torch.ones(500), atol=1e-6)
    assert m.get_features.shape == (500, 16, 3)
    cov = build_covariance_from_scaling_rotation(m.get_scaling, 1.0, m._rotation)
    # symmetric PSD reconstruction
    S = torch.stack([cov[:, 0], cov[:, 1], cov[:, 2], cov[:, 1], cov[:, 3], cov[:, 4], cov[:, 2],
                     cov[:, 4], cov[:, 5]], 1).view(-1, 3, 3)
    ev = torch.linalg.eigvalsh(S.double())
    assert torch.all(ev > -1e-9)
    s2 = torch.sort(m.get_scaling.double() ** 2, dim=1).values
    torch.testing.assert_close(ev, s2, rtol=1e-4, atol=1e-9)


def test_settings_namedtuple_is_backward_compatible():
    from diff_gaussian_rasterization import GaussianRasterizationSettings
    fields = GaussianRasterizationSettings._fields
    assert fields[:12] == ("image_height", "image_width", "tanfovx", "tanfovy", "bg",
                           "scale_modifier", "viewmatrix", "projmatrix", "sh_degree", "campos",
                           "prefiltered", "debug")
    assert "include_feature" in fields and "confidence" in fields
    s = GaussianRasterizationSettings(10, 10, 1.0, 1.0, None, 1.0, None, None, 0, None, False, False)
    assert s.include_feature is False and s.confidence is None


def test_cpu_tensors_are_rejected_not_rasterized_on_cpu():
    """The product path has no CPU fallback: CPU tensors must raise."""
    from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
    s = GaussianRasterizationSettings(8, 8, 1.0, 1.0, torch.zeros(3), 1.0, torch.eye(4),
                                      torch.eye(4), 0, torch.zeros(3), False, False)
    with pytest.raises(RuntimeError):
        GaussianRasterizer(s)(means3D=torch.zeros((1, 3)), means2D=torch.zeros((1, 3)),
                              opacities=torch.ones((1, 1)), colors_precomp=torch.ones((1, 3)),
                              scales=torch.ones((1, 3)), rotations=torch.tensor([[1., 0, 0, 0]]))


def test_render_pkg_lazy_entries_behave_like_dict_items():
    """render()'s fused-path result dict: "opacity" is computed on first access only, and the
    dict still reports every key of the reference's dict."""
    from gaussian_renderer import _RenderPkg
    calls = []
    pkg = _RenderPkg({"render": 1, "radii": 2}, {"opacity": lambda: calls.append(1) or 3})
    assert "opacity" in pkg and len(pkg) == 3 and calls == []
    assert pkg.get("render") == 1 and pkg.get("missing", 7) == 7
    assert pkg["opacity"] == 3 and pkg["opacity"] == 3 and calls == [1]
    pkg2 = _RenderPkg({"a": 0}, {"b": lambda: 5})
    assert set(pkg2) == {"a", "b"} and dict(pkg2.items()) == {"a": 0, "b": 5}
    import pytest
    with pytest.raises(KeyError):
        pkg2["nope"]


def test_view_pipeline_reducer_with_deferral_needs_the_model():
    """with deferred SH gradients the early all-reduce must leave the SH leaves out;
    without the model they are unknown, so run() refuses (before any GPU work)."""
    from gsr_amd.pipeline import ViewPipeline

    class _Reducer:
        def begin(self):
            raise AssertionError("must not be reached")

    vp = ViewPipeline(torch.device("cuda", 0), depth=1, defer_sh=True)
    with pytest.raises(ValueError, match="model"):
        vp.run([], lambda cam: cam, model=None, reducer=_Reducer())


def test_C_shim_asks_for_the_layout_from_the_buffer():
    """the `_C` shim's backward checks the binning buffer's size against R (a
    buffer too small raises) and passes GSR_DEBUG_LAYOUT_FROM_BUFFER only when the size cannot
    tell the layouts apart, so the library then reads the forward's layout from the tag word --
    no global mode (the GPU side: tests/test_deterministic.py)."""
    import inspect
    from diff_gaussian_rasterization import _C
    src = inspect.getsource(_C.rasterize_gaussians_backward)
    assert "flags |= 4" in src and "gsr_binning_buffer_bytes_det" in src
    assert "if have < need:" in src


def test_row_slices_one_backward_per_scope():
    """a second sliced multi-view backward in one BackwardRowSlices scope would add
    gradients whose rows were already all-reduced -- it raises instead of corrupting them."""
    import diff_gaussian_rasterization as dgr
    seen = []
    sl = dgr.BackwardRowSlices("cpu", lambda a, b: seen.append((a, b)), slices=4)
    assert sl.rows(4096) == 1024
    with pytest.raises(RuntimeError, match="second"):
        sl.rows(4096)
