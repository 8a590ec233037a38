"""The batched training step (gsr_amd.trainer.train_step_views, bench.py's train_step leg) in its
two issue modes: every view in one multi-view call (multi=True, the default) and view by view on
the pipeline's streams (multi=False).  With the deterministic backward both are the same
arithmetic in the same order, so after a step the parameters, the Adam moments and the
densification statistics are bitwise equal.  Reference: train.py:63-236 (render -> loss ->
backward -> add_densification_stats -> optimizer.step)."""
import pytest
import torch

from gsr_amd import trainer
from gsr_amd.model import SplatModel
from gsr_amd.pipeline import ViewPipeline
from gsr_amd.synthetic import make_cameras, make_gaussians, training_targets

pytestmark = pytest.mark.gpu


def _state(m):
    out = {n: getattr(m, n).detach().clone() for n in
           ("_xyz", "_features_dc", "_features_rest", "_opacity", "_scaling", "_rotation",
            "_language_feature")}
    for n in ("xyz_gradient_accum", "denom", "max_radii2D"):
        out[n] = getattr(m, n).detach().clone()
    for g in m.optimizer.param_groups:
        st = m.optimizer.state.get(g["params"][0], {})
        for k in ("exp_avg", "exp_avg_sq"):
            if k in st:
                out[g["name"] + "." + k] = st[k].detach().clone()
    return out


@pytest.mark.parametrize("streams", [1, 4])
def test_multi_view_train_step_equals_per_view(streams):
    import diff_gaussian_rasterization as dgr
    W, H = 240, 180
    cams = [c.to("cuda") for c in make_cameras(4, W, H, seed=21)]
    gts, monos = training_targets(4, H, W, seed=2, device="cuda")
    bg = torch.zeros(3, device="cuda")
    args = trainer.OptArgs()
    prev = (dgr.deterministic(), dgr.grad_into_leaves())
    dgr.deterministic(True)
    dgr.grad_into_leaves(True)
    states = []
    try:
        for multi in (True, False):
            m = SplatModel(make_gaussians(30_000, sh_degree=3, seed=21), device="cuda")
            trainer.make_trainable(m, args)
            vp = ViewPipeline(torch.device("cuda"), depth=streams)
            for it in (1, 2):
                trainer.train_step_views(m, cams, gts, monos, bg, args, it, 2.78, vp,
                                         multi=multi)
            torch.cuda.synchronize()
            states.append(_state(m))
    finally:
        dgr.deterministic(prev[0])
        dgr.grad_into_leaves(prev[1])
    a, b = states
    assert a.keys() == b.keys()
    for k in a:
        assert torch.equal(a[k], b[k]), k
