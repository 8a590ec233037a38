"""Fused Adam: same state layout and results as torch.optim.Adam over
GaussianModel's parameter groups (scene/gaussian_model.py:217-271), including the reference's
densification edits of the optimizer state (:400-470)."""
import pytest
import torch

from gsr_amd.optim import FusedAdam


def _groups(P, device, seed=0):
    g = torch.Generator().manual_seed(seed)
    shapes = {"xyz": (P, 3), "f_dc": (P, 1, 3), "f_rest": (P, 15, 3), "opacity": (P, 1),
              "scaling": (P, 3), "rotation": (P, 4), "language_feature": (P, 3)}
    lrs = {"xyz": 1.6e-4, "f_dc": 2.5e-3, "f_rest": 2.5e-3 / 20, "opacity": 5e-2,
           "scaling": 5e-3, "rotation": 1e-3, "language_feature": 2.5e-3}
    params = {k: torch.nn.Parameter(torch.randn(s, generator=g).to(device)) for k, s in shapes.items()}
    return params, [{"params": [params[k]], "lr": lrs[k], "name": k} for k in shapes]


def test_is_a_torch_adam_with_the_same_state_layout():
    params, groups = _groups(10, "cpu")
    opt = FusedAdam(groups, lr=0.0, eps=1e-15)
    assert isinstance(opt, torch.optim.Adam)
    assert [g["name"] for g in opt.param_groups] == [g["name"] for g in groups]
    assert opt.param_groups[0]["eps"] == 1e-15


def test_no_cpu_path():
    params, groups = _groups(10, "cpu")
    opt = FusedAdam(groups, lr=0.0, eps=1e-15)
    for p in params.values():
        p.grad = torch.ones_like(p)
    with pytest.raises(RuntimeError, match="HIP"):
        opt.step()


def _prune_optimizer(opt, mask):
    # scene/gaussian_model.py:415-431
    out = {}
    for group in opt.param_groups:
        stored = opt.state.get(group["params"][0], None)
        if stored is not None:
            stored["exp_avg"] = stored["exp_avg"][mask]
            stored["exp_avg_sq"] = stored["exp_avg_sq"][mask]
            del opt.state[group["params"][0]]
            group["params"][0] = torch.nn.Parameter(group["params"][0][mask].requires_grad_(True))
            opt.state[group["params"][0]] = stored
        else:
            group["params"][0] = torch.nn.Parameter(group["params"][0][mask].requires_grad_(True))
        out[group["name"]] = group["params"][0]
    return out


def _cat_tensors_to_optimizer(opt, ext):
    # scene/gaussian_model.py:454-476
    out = {}
    for group in opt.param_groups:
        e = ext[group["name"]]
        stored = opt.state.get(group["params"][0], None)
        if stored is not None:
            stored["exp_avg"] = torch.cat((stored["exp_avg"], torch.zeros_like(e)), dim=0)
            stored["exp_avg_sq"] = torch.cat((stored["exp_avg_sq"], torch.zeros_like(e)), dim=0)
            del opt.state[group["params"][0]]
            group["params"][0] = torch.nn.Parameter(torch.cat((group["params"][0], e), dim=0).requires_grad_(True))
            opt.state[group["params"][0]] = stored
        else:
            group["params"][0] = torch.nn.Parameter(torch.cat((group["params"][0], e), dim=0).requires_grad_(True))
        out[group["name"]] = group["params"][0]
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("P,wd", [(1000, 0.0), (4099, 0.0), (3000, 1e-2)])
def test_matches_torch_adam_with_densification(P, wd):
    """Five steps, then a prune + densify edit of the state exactly as the reference does it,
    then five more steps: FusedAdam == torch.optim.Adam (PyTorch's own HIP implementation) to
    float rounding.  P = 4099 exercises the scalar tails, wd the L2 term."""
    _, ga = _groups(P, "cuda", seed=1)
    _, gb = _groups(P, "cuda", seed=1)
    a = torch.optim.Adam(ga, lr=0.0, eps=1e-15, weight_decay=wd)
    b = FusedAdam(gb, lr=0.0, eps=1e-15, weight_decay=wd)
    gen = torch.Generator(device="cuda").manual_seed(7)

    def run(steps):
        for _ in range(steps):
            for x, y in zip(a.param_groups, b.param_groups):
                g = torch.randn(x["params"][0].shape, generator=gen, device="cuda")
                x["params"][0].grad = g.clone()
                y["params"][0].grad = g.clone()
            a.step()
            b.step()
        for x, y in zip(a.param_groups, b.param_groups):
            px, py = x["params"][0], y["params"][0]
            torch.testing.assert_close(py, px, rtol=2e-6, atol=2e-7, msg=x["name"])
            sx, sy = a.state[px], b.state[py]
            torch.testing.assert_close(sy["exp_avg"], sx["exp_avg"], rtol=2e-6, atol=1e-7)
            torch.testing.assert_close(sy["exp_avg_sq"], sx["exp_avg_sq"], rtol=2e-6, atol=1e-9)
            assert float(sy["step"]) == float(sx["step"])

    run(5)
    keep = torch.rand(P, generator=torch.Generator().manual_seed(3)) > 0.3
    keep = keep.cuda()
    _prune_optimizer(a, keep)
    _prune_optimizer(b, keep)
    ext = {x["name"]: torch.randn((257,) + tuple(x["params"][0].shape[1:]), device="cuda")
           for x in a.param_groups}
    _cat_tensors_to_optimizer(a, ext)
    _cat_tensors_to_optimizer(b, ext)
    run(5)


@pytest.mark.gpu
def test_unaligned_views_and_many_tensors():
    """More tensors than one launch takes (chunking) and a parameter whose storage starts off a
    16-byte boundary (vectorised path disabled for it)."""
    base = torch.randn(20 * 1001 + 1, device="cuda")
    ps = [torch.nn.Parameter(torch.randn(1001, device="cuda")) for _ in range(19)]
    ps.append(torch.nn.Parameter(base[1:1002]))  # offset by one float
    qs = [torch.nn.Parameter(p.detach().clone()) for p in ps]
    a = torch.optim.Adam(qs, lr=1e-2)
    b = FusedAdam(ps, lr=1e-2)
    for _ in range(3):
        for p, q in zip(ps, qs):
            g = torch.randn_like(p)
            p.grad, q.grad = g.clone(), g.clone()
        a.step()
        b.step()
    for p, q in zip(ps, qs):
        torch.testing.assert_close(p, q, rtol=2e-6, atol=2e-7)
