"""Test oracle for the densification row: a plain-PyTorch restatement of
GaussianModel's adaptive density control, scene/gaussian_model.py:400-612, and of the statistics
update of train.py:218-220.  Boolean-mask indexing and torch.cat on every tensor, exactly the
reference's sequence of stages, so that gsr_amd.densify can be compared with it array by array
(parameters, Adam moments and step, statistics, confidence, row order).

Test infrastructure only: imported by tests/test_densify.py and scripts/densify_bench.py.
"""
from __future__ import annotations

import copy

import torch
from torch import nn

import sys, os  # noqa: E401
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "sdp-gs_amd"))
from gsr_amd.model import build_rotation  # noqa: E402  (restates utils/general_utils.py:88-107)

NAMES = {"xyz": "_xyz", "f_dc": "_features_dc", "f_rest": "_features_rest",
         "opacity": "_opacity", "language_feature": "_language_feature",
         "scaling": "_scaling", "rotation": "_rotation"}


class RefDensify:
    """Holds the same attributes as GaussianModel; methods restate the reference behaviour."""

    def __init__(self, src):
        """Deep copy of a SplatModel after training_setup (same tensors, same optimizer state),
        re-wrapped around torch.optim.Adam with the same param groups."""
        self.percent_dense = src.percent_dense
        self.args = copy.copy(src.args)
        for k in ("xyz_gradient_accum", "denom", "max_radii2D", "confidence"):
            setattr(self, k, getattr(src, k).clone())
        groups = []
        for g in src.optimizer.param_groups:
            p = nn.Parameter(g["params"][0].detach().clone().requires_grad_(True))
            setattr(self, NAMES[g["name"]], p)
            groups.append({"params": [p], "lr": g["lr"], "name": g["name"]})
        if not any(g["name"] == "language_feature" for g in groups):
            self._language_feature = None
        self.optimizer = torch.optim.Adam(groups, lr=0.0, eps=1e-15)
        for g_src, g in zip(src.optimizer.param_groups, self.optimizer.param_groups):
            st = src.optimizer.state.get(g_src["params"][0])
            if st:
                self.optimizer.state[g["params"][0]] = {k: v.clone() for k, v in st.items()}

    # getters (scene/gaussian_model.py:146-173)
    @property
    def get_xyz(self):
        return self._xyz

    @property
    def get_scaling(self):
        return torch.exp(self._scaling)

    @property
    def get_opacity(self):
        return torch.sigmoid(self._opacity)

    # ---- per-step statistics: train.py:219 + add_densification_stats (:606-609) -------------
    def update_stats(self, viewspace_grad, radii, visibility_filter):
        f = visibility_filter
        self.max_radii2D[f] = torch.max(self.max_radii2D[f], radii[f])
        self.add_stats(viewspace_grad, f)

    def add_stats(self, viewspace_grad, f):
        self.xyz_gradient_accum[f] += torch.norm(viewspace_grad[f, :2], dim=-1, keepdim=True)
        self.denom[f] += 1

    # ---- optimizer surgery (:417-476) ---------------------------------------------------------
    def _swap(self, group, new_param_data, moment_fn):
        old = group["params"][0]
        st = self.optimizer.state.get(old, None)
        newp = nn.Parameter(new_param_data.requires_grad_(True))
        if st is not None:
            st["exp_avg"] = moment_fn(st["exp_avg"])
            st["exp_avg_sq"] = moment_fn(st["exp_avg_sq"])
            del self.optimizer.state[old]
            self.optimizer.state[newp] = st
        group["params"][0] = newp
        setattr(self, NAMES[group["name"]], newp)

    def prune_points(self, mask, iteration):
        if iteration <= self.args.prune_from_iter:
            return
        keep = ~mask
        for group in self.optimizer.param_groups:
            self._swap(group, group["params"][0][keep], lambda t: t[keep])
        for k in ("xyz_gradient_accum", "denom", "max_radii2D", "confidence"):
            setattr(self, k, getattr(self, k)[keep])

    def postfix(self, new):
        n_new = None
        for group in self.optimizer.param_groups:
            ext = new[group["name"]]
            n_new = ext.shape[0]
            self._swap(group, torch.cat((group["params"][0], ext), dim=0),
                       lambda t, e=ext: torch.cat((t, torch.zeros_like(e)), dim=0))
        P = self._xyz.shape[0]
        dev = self._xyz.device
        self.xyz_gradient_accum = torch.zeros((P, 1), device=dev)
        self.denom = torch.zeros((P, 1), device=dev)
        self.max_radii2D = torch.zeros((P,), device=dev)
        self.confidence = torch.cat([self.confidence, torch.ones((n_new, 1), device=dev)], 0)

    def _rows(self, sel, reps=1):
        out = {}
        for group in self.optimizer.param_groups:
            t = group["params"][0][sel]
            out[group["name"]] = t.repeat((reps,) + (1,) * (t.dim() - 1))
        return out

    # ---- densification (:534-604) ----------------------------------------------------------------
    def clone(self, grads, thr, extent):
        sel = torch.where(torch.norm(grads, dim=-1) >= thr, True, False)
        sel = torch.logical_and(sel, self.get_scaling.max(dim=1).values
                                <= self.percent_dense * extent)
        self.postfix(self._rows(sel))

    def split(self, grads, thr, extent, iteration, N=2):
        n = self._xyz.shape[0]
        padded = torch.zeros((n,), device=self._xyz.device)
        padded[:grads.shape[0]] = grads.squeeze()
        sel = torch.where(padded >= thr, True, False)
        sel = torch.logical_and(sel, self.get_scaling.max(dim=1).values
                                > self.percent_dense * extent)
        stds = self.get_scaling[sel].repeat(N, 1)
        samples = torch.normal(mean=torch.zeros((stds.size(0), 3), device=stds.device), std=stds)
        rots = build_rotation(self._rotation[sel]).repeat(N, 1, 1)
        new = self._rows(sel, N)
        new["xyz"] = torch.bmm(rots, samples.unsqueeze(-1)).squeeze(-1) + \
            self.get_xyz[sel].repeat(N, 1)
        new["scaling"] = torch.log(self.get_scaling[sel].repeat(N, 1) / (0.8 * N))
        self.postfix(new)
        drop = torch.cat((sel, torch.zeros(N * int(sel.sum()), device=sel.device, dtype=bool)))
        self.prune_points(drop, iteration)

    def proximity(self, extent, N=3):
        """:513-532, with distCUDA2 from the CPU oracle (oracle/gsr_oracle_knn.c)."""
        from oracle.oracle import dist_knn3
        d, nn = dist_knn3(self._xyz.detach().cpu().numpy())
        dev = self._xyz.device
        dist, nearest = torch.from_numpy(d).to(dev), torch.from_numpy(nn).to(dev)
        sel = torch.logical_and(dist > (5. * extent), self.get_scaling.max(dim=1).values > extent)
        idx = nearest[sel].reshape(-1).long()
        new = {"xyz": (self._xyz[sel].repeat(1, N, 1).reshape(-1, 3) + self._xyz[idx]) / 2,
               "scaling": self._scaling[idx], "opacity": self._opacity[idx],
               "f_dc": torch.zeros_like(self._features_dc[idx]),
               "f_rest": torch.zeros_like(self._features_rest[idx])}
        rot = torch.zeros_like(self._rotation[idx])
        rot[:, 0] = 1
        new["rotation"] = rot
        if self._language_feature is not None:
            new["language_feature"] = self._language_feature[idx]
        self.postfix(new)

    def densify_and_prune(self, max_grad, min_opacity, extent, max_screen_size, iteration):
        grads = self.xyz_gradient_accum / self.denom
        grads[grads.isnan()] = 0.0
        self.clone(grads, max_grad, extent)
        self.split(grads, max_grad, extent, iteration)
        if iteration < 2000:
            self.proximity(extent)
        prune = (self.get_opacity < min_opacity).squeeze()
        if max_screen_size:
            big_vs = self.max_radii2D > max_screen_size
            big_ws = self.get_scaling.max(dim=1).values > 0.1 * extent
            prune = torch.logical_or(torch.logical_or(prune, big_vs), big_ws)
        self.prune_points(prune, iteration)

    # ---- comparison ------------------------------------------------------------------------------
    def arrays(self):
        """name -> tensor of every per-Gaussian array, in a canonical order."""
        out = {}
        for group in self.optimizer.param_groups:
            p = group["params"][0]
            out[group["name"]] = p.detach()
            st = self.optimizer.state.get(p)
            if st:
                out[group["name"] + ".exp_avg"] = st["exp_avg"]
                out[group["name"] + ".exp_avg_sq"] = st["exp_avg_sq"]
                out[group["name"] + ".step"] = st["step"]
        for k in ("xyz_gradient_accum", "denom", "max_radii2D", "confidence"):
            out[k] = getattr(self, k)
        return out


def model_arrays(m):
    """RefDensify.arrays() for a SplatModel driven by gsr_amd.densify (checks that the optimizer
    state is keyed by the current parameters and the attributes are those parameters)."""
    out = {}
    for group in m.optimizer.param_groups:
        p = group["params"][0]
        assert getattr(m, NAMES[group["name"]]) is p
        out[group["name"]] = p.detach()
        st = m.optimizer.state.get(p)
        if st:
            out[group["name"] + ".exp_avg"] = st["exp_avg"]
            out[group["name"] + ".exp_avg_sq"] = st["exp_avg_sq"]
            out[group["name"] + ".step"] = st["step"]
    assert len(m.optimizer.state) == sum(1 for g in m.optimizer.param_groups
                                         if m.optimizer.state.get(g["params"][0]))
    for k in ("xyz_gradient_accum", "denom", "max_radii2D", "confidence"):
        out[k] = getattr(m, k)
    return out
