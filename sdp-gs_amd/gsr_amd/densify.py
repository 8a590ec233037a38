"""Adaptive density control on libgsr (include/gsr_densify.h).

Drop-in replacements for GaussianModel's densification methods (scene/gaussian_model.py:400-612)
and for the statistics update train.py runs after every backward (train.py:218-220).  They take
the model as `self` -- any object with the reference GaussianModel's attributes (`_xyz`,
`_features_dc`, `_features_rest`, `_opacity`, `_scaling`, `_rotation`, `_language_feature`,
`confidence`, `xyz_gradient_accum`, `denom`, `max_radii2D`, `percent_dense`,
`args.prune_from_iter` and an Adam `optimizer` whose param groups are named as in
training_setup, :217-271) -- so `install(GaussianModel)` swaps them in.  Results equal the
reference's (parameters, Adam moments and step, statistics, confidence; ordering of the rows
included); tests/test_densify.py checks that against a restatement of the reference methods.

What changes is the data movement:
  * update_densification_stats / add_densification_stats: one elementwise launch per step instead
    of boolean-mask indexing (each a nonzero() with a device->host sync);
  * densify_and_prune: the per-Gaussian tests run as one classify launch, and the final arrays --
    kept originals, clones, split children, with their Adam moments (zero for new rows),
    confidence (one for new rows) and reset statistics -- are written by ONE gsr_compact_rows
    launch from the old arrays plus a small appendix of new rows, instead of a torch.cat and a
    boolean-index pass per tensor per stage (clone, split, split prune, final prune).
  The appendix rows (clone copies; split children from torch.normal) are computed with the same
  torch calls as the reference, so the split's random samples are the reference's.
There is no CPU path: every function raises on tensors that are not on a HIP device.
"""
from __future__ import annotations

import ctypes

import torch
from torch import nn

from . import _lib

CLONE, SPLIT, LOW_OPACITY, BIG_WS = 1, 2, 4, 8  # GSR_DENSIFY_* (include/gsr_densify.h)
MAX_ARRAYS = 32                                 # GSR_COMPACT_MAX_ARRAYS
_ONE_F32 = 0x3F800000

# training_setup's param-group names (scene/gaussian_model.py:229-258) -> GaussianModel attribute
GROUP_ATTR = {"xyz": "_xyz", "f_dc": "_features_dc", "f_rest": "_features_rest",
              "opacity": "_opacity", "language_feature": "_language_feature",
              "scaling": "_scaling", "rotation": "_rotation"}


def _check(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what} failed with status {rc}")


def _cuda(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError("gsr densification runs on HIP tensors only (no CPU path)")


def _stream(dev):
    return _lib.raw_stream(dev)


def _ptr(t):
    return None if t is None else t.data_ptr()


def _rows(t):
    return int(t.shape[0])


# ---- thin wrappers of the C-ABI --------------------------------------------------------------------
def select_rows(flags: torch.Tensor, mask: int, want: int):
    """Ascending indices i with (flags[i] & mask) == want (gsr_select_rows) -> (index int32 [n],
    count int32 device scalar); index[:count] is the selection."""
    _cuda(flags)
    assert flags.dtype == torch.uint8 and flags.dim() == 1 and flags.is_contiguous()
    n = flags.numel()
    L = _lib.load()
    index = torch.empty(n, dtype=torch.int32, device=flags.device)
    count = torch.empty(1, dtype=torch.int32, device=flags.device)
    scratch = torch.empty(max(int(L.gsr_select_scratch_bytes(n)), 1), dtype=torch.uint8,
                          device=flags.device)
    with _lib.on_device(flags.device):
        _check(L.gsr_select_rows(n, _ptr(flags), mask, want, _ptr(index), _ptr(count),
                                 _ptr(scratch), _stream(flags.device)), "gsr_select_rows")
    return index, count


def compact_rows(arrays, n_old: int, index, n_out: int):
    """One gsr_compact_rows launch.  arrays: list of (src, extra, fill_word, dst) with src / extra
    row-major tensors or None, dst an [n_out, ...] tensor (dtype of 4-byte words)."""
    if not arrays or n_out == 0:
        return
    L = _lib.load()
    dev = arrays[0][3].device
    for c in range(0, len(arrays), MAX_ARRAYS):
        chunk = arrays[c:c + MAX_ARRAYS]
        n = len(chunk)
        src = (ctypes.c_void_p * n)(*[_ptr(a[0]) for a in chunk])
        extra = (ctypes.c_void_p * n)(*[_ptr(a[1]) for a in chunk])
        dst = (ctypes.c_void_p * n)(*[_ptr(a[3]) for a in chunk])
        rb = (ctypes.c_int64 * n)(*[a[3].element_size() * (a[3].numel() // n_out) for a in chunk])
        fill = (ctypes.c_uint32 * n)(*[a[2] for a in chunk])
        for s, e, _, d in chunk:
            _cuda(s, e, d)
            for t in (s, e, d):
                assert t is None or (t.is_contiguous() and t.device == dev)
        with _lib.on_device(dev):
            _check(L.gsr_compact_rows(n, src, extra, dst, rb, fill, n_old, _ptr(index), n_out,
                                      _stream(dev)), "gsr_compact_rows")


def classify(self, grad_accum, denom, grad_threshold, scale_limit, min_opacity=float("-inf"),
             big_limit=None):
    """gsr_densify_classify over self's raw _scaling / _opacity, then the clone and split index
    lists -> (flags u8 [P], clone rows, split rows) (ascending int64; one host read for both
    counts).  denom None: grad_accum already holds the ratio."""
    P = _rows(self._xyz)
    _cuda(grad_accum, denom, self._scaling, self._opacity)
    dev = self._xyz.device
    for t in (grad_accum, denom):
        assert t is None or (t.is_contiguous() and t.numel() == P and t.dtype == torch.float32)
    flags = torch.empty(P, dtype=torch.uint8, device=dev)
    sc, op = self._scaling.detach(), self._opacity.detach()
    assert sc.is_contiguous() and op.is_contiguous() and sc.numel() == 3 * P and op.numel() == P
    with _lib.on_device(dev):
        _check(_lib.load().gsr_densify_classify(
            P, _ptr(grad_accum), _ptr(denom), _ptr(sc), _ptr(op), float(grad_threshold),
            float(scale_limit), float(min_opacity), int(big_limit is not None),
            float(big_limit if big_limit is not None else 0.0), _ptr(flags), None,
            _stream(dev)), "gsr_densify_classify")
    ci, cc = select_rows(flags, CLONE, CLONE)
    si, scount = select_rows(flags, SPLIT, SPLIT)
    nc, ns = (int(x) for x in torch.cat((cc, scount)).tolist())
    return flags, ci[:nc].long(), si[:ns].long()


# ---- statistics (every step) ---------------------------------------------------------------------
_STATS_EVENT = {}  # device index -> (event after the last statistics update, its stream id)


def _stats(self, grad, radii, filt, with_radii, with_grad):
    P = _rows(self.xyz_gradient_accum)
    _cuda(grad, radii, filt)
    if with_grad:
        assert grad.dim() == 2 and grad.stride(1) == 1 and grad.shape[0] == P
    if radii is not None:
        assert radii.dtype == torch.int32 and radii.is_contiguous() and radii.numel() == P
    if filt is not None:
        assert filt.dtype == torch.bool and filt.is_contiguous() and filt.numel() == P
    for t in (self.xyz_gradient_accum, self.denom, self.max_radii2D):
        assert t.is_contiguous() and t.numel() == P
    dev = self.xyz_gradient_accum.device
    stream = torch.cuda.current_stream(dev)
    prev = _STATS_EVENT.get(dev.index)
    if prev is not None and prev[1] != stream.stream_id:
        # the statistics are read-modify-written without atomics: views on other streams
        # (gsr_amd.pipeline.ViewPipeline) add theirs in issue order, as train.py does per view
        stream.wait_event(prev[0])
    with _lib.on_device(dev):
        _check(_lib.load().gsr_densify_stats(
            P, _ptr(grad) if with_grad else None, grad.stride(0) if with_grad else 0,
            _ptr(radii), _ptr(filt), _ptr(self.max_radii2D) if with_radii else None,
            _ptr(self.xyz_gradient_accum) if with_grad else None,
            _ptr(self.denom) if with_grad else None, _stream(dev)), "gsr_densify_stats")
    ev = torch.cuda.Event()
    ev.record(stream)
    _STATS_EVENT[dev.index] = (ev, stream.stream_id)


def update_densification_stats_views(self, viewspace_grads, radii):
    """update_densification_stats of the V views of a multi-view step (render_views' stacked
    outputs: viewspace_grads [V,P,>=2] = the stacked means2D's .grad, radii [V,P]) in one launch,
    visibility radii > 0; equals V calls in view order."""
    P = _rows(self.xyz_gradient_accum)
    _cuda(viewspace_grads, radii)
    V = int(radii.shape[0])
    assert radii.dtype == torch.int32 and radii.is_contiguous() and radii.numel() == V * P
    g = viewspace_grads
    assert g.dim() == 3 and g.shape[0] == V and g.shape[1] == P and g.stride(2) == 1
    for t in (self.xyz_gradient_accum, self.denom, self.max_radii2D):
        assert t.is_contiguous() and t.numel() == P
    dev = self.xyz_gradient_accum.device
    stream = torch.cuda.current_stream(dev)
    prev = _STATS_EVENT.get(dev.index)
    if prev is not None and prev[1] != stream.stream_id:
        stream.wait_event(prev[0])
    with _lib.on_device(dev):
        _check(_lib.load().gsr_densify_stats_views(
            V, P, _ptr(g), g.stride(1), g.stride(0), _ptr(radii), _ptr(self.max_radii2D),
            _ptr(self.xyz_gradient_accum), _ptr(self.denom), _stream(dev)),
            "gsr_densify_stats_views")
    ev = torch.cuda.Event()
    ev.record(stream)
    _STATS_EVENT[dev.index] = (ev, stream.stream_id)


def add_densification_stats(self, viewspace_point_tensor, update_filter):
    """scene/gaussian_model.py:606-609 (xyz_gradient_accum[f] += |grad[f,:2]|; denom[f] += 1)."""
    _stats(self, viewspace_point_tensor.grad, None, update_filter, False, True)


def update_densification_stats(self, viewspace_point_tensor, radii, visibility_filter=None):
    """train.py:219-220 in one launch: max_radii2D[f] = max(max_radii2D[f], radii[f]) followed by
    add_densification_stats(viewspace_point_tensor, f), f = visibility_filter (default radii > 0,
    which is what render() returns as visibility_filter)."""
    _stats(self, viewspace_point_tensor.grad, radii, visibility_filter, True, True)


# ---- array rebuild (prune / append / both) -------------------------------------------------------
def _groups(self):
    for group in self.optimizer.param_groups:
        if group["name"] in GROUP_ATTR:
            yield group


def _rebuild(self, index, n_out, extras=None, fresh_stats=False):
    """Rewrite every per-Gaussian array: output row j <- row index[j] (None: j) of [old rows |
    extras rows].  Parameters take extras[name]; Adam moments are 0 and confidence 1 on extra
    rows; statistics are gathered (prune_points) or reset to zero (fresh_stats:
    densification_postfix).  Mirrors the optimizer-state surgery of _prune_optimizer /
    cat_tensors_to_optimizer (:417-476): new nn.Parameters, state (step included) carried over."""
    n_old = _rows(self._xyz)
    dev = self._xyz.device
    arrays, plan = [], []
    for group in _groups(self):
        p = group["params"][0]
        ext = None if extras is None else extras[group["name"]]
        if ext is not None:
            ext = ext.detach().contiguous()
        newp = torch.empty((n_out,) + tuple(p.shape[1:]), dtype=p.dtype, device=dev)
        arrays.append((p.detach(), ext, 0, newp))
        st = self.optimizer.state.get(p, None)
        moms = {}
        if st is not None:
            for k in ("exp_avg", "exp_avg_sq"):
                moms[k] = torch.empty_like(newp)
                arrays.append((st[k], None, 0, moms[k]))
        plan.append((group, p, newp, st, moms))
    conf = torch.empty((n_out,) + tuple(self.confidence.shape[1:]), dtype=self.confidence.dtype,
                       device=dev)
    arrays.append((self.confidence, None, _ONE_F32, conf))
    stats = {}
    for k in ("xyz_gradient_accum", "denom", "max_radii2D"):
        old = getattr(self, k)
        stats[k] = torch.empty((n_out,) + tuple(old.shape[1:]), dtype=old.dtype, device=dev)
        arrays.append((None if fresh_stats else old, None, 0, stats[k]))
    compact_rows(arrays, n_old, index, n_out)
    for group, p, newp, st, moms in plan:
        newp = nn.Parameter(newp.requires_grad_(True))
        if st is not None:
            st.update(moms)
            del self.optimizer.state[p]
            self.optimizer.state[newp] = st
        group["params"][0] = newp
        setattr(self, GROUP_ATTR[group["name"]], newp)
    self.confidence = conf
    for k, v in stats.items():
        setattr(self, k, v)


def _prune_active(self, iteration):
    return iteration > self.args.prune_from_iter


def prune_points(self, mask, iter, include_feature):
    """scene/gaussian_model.py:434-452: drop the rows where mask is set (only once
    iter > args.prune_from_iter)."""
    if not _prune_active(self, iter):
        return
    _cuda(mask)
    flags = mask.to(torch.uint8).contiguous()
    index, count = select_rows(flags, 1, 0)
    _rebuild(self, index, int(count.item()))


def densification_postfix(self, new_xyz, new_features_dc, new_features_rest, new_language_feature,
                          new_opacities, new_scaling, new_rotation, include_feature):
    """scene/gaussian_model.py:478-511: append rows (zero moments, confidence 1), reset stats."""
    extras = _extras_dict(new_xyz, new_features_dc, new_features_rest, new_language_feature,
                          new_opacities, new_scaling, new_rotation)
    _rebuild(self, None, _rows(self._xyz) + _rows(new_xyz), extras, fresh_stats=True)


def _extras_dict(xyz, f_dc, f_rest, lang, opacity, scaling, rotation):
    d = {"xyz": xyz, "f_dc": f_dc, "f_rest": f_rest, "opacity": opacity, "scaling": scaling,
         "rotation": rotation}
    if lang is not None:
        d["language_feature"] = lang
    return d


# ---- new rows, computed with the reference's torch calls --------------------------------------------
def _clone_rows(self, idx):
    """densify_and_clone's new rows (:571-589): copies of the selected rows."""
    lang = self._language_feature
    return _extras_dict(self._xyz[idx], self._features_dc[idx], self._features_rest[idx],
                        None if lang is None or not _has_group(self, "language_feature")
                        else lang[idx],
                        self._opacity[idx], self._scaling[idx], self._rotation[idx])


def _split_rows(self, idx, N, generator=None):
    """densify_and_split's children (:544-555): N samples from N(0, scale) rotated into place,
    scales shrunk by 0.8 N, everything else repeated (torch.normal draws the reference's
    samples from the same generator; data-parallel replicas pass one identically seeded
    `generator` so that every rank draws the same samples)."""
    from .model import build_rotation
    sel_scaling = self.scaling_activation(self._scaling[idx])   # get_scaling[selected]
    stds = sel_scaling.repeat(N, 1)
    means = torch.zeros((stds.size(0), 3), device=stds.device)
    samples = torch.normal(mean=means, std=stds, generator=generator)
    rots = build_rotation(self._rotation[idx]).repeat(N, 1, 1)
    new_xyz = torch.bmm(rots, samples.unsqueeze(-1)).squeeze(-1) + self._xyz[idx].repeat(N, 1)
    new_scaling = self.scaling_inverse_activation(sel_scaling.repeat(N, 1) / (0.8 * N))
    lang = self._language_feature
    return _extras_dict(new_xyz, self._features_dc[idx].repeat(N, 1, 1),
                        self._features_rest[idx].repeat(N, 1, 1),
                        None if lang is None or not _has_group(self, "language_feature")
                        else lang[idx].repeat(N, 1),
                        self._opacity[idx].repeat(N, 1), new_scaling,
                        self._rotation[idx].repeat(N, 1))


def _has_group(self, name):
    return any(g["name"] == name for g in self.optimizer.param_groups)


def _cat_extras(a, b):
    return {k: torch.cat((a[k], b[k]), dim=0) for k in a}


# ---- the reference's densification entry points ------------------------------------------------
def densify_and_clone(self, grads, grad_threshold, scene_extent, include_feature):
    """scene/gaussian_model.py:566-589."""
    with torch.no_grad():
        g = grads.reshape(-1).contiguous()
        _, idx, _ = classify(self, g, None, grad_threshold, self.percent_dense * scene_extent)
        ext = _clone_rows(self, idx)
        _rebuild(self, None, _rows(self._xyz) + idx.numel(), ext, fresh_stats=True)


def densify_and_split(self, grads, grad_threshold, scene_extent, iter, include_feature=False,
                      N=2, generator=None):
    """scene/gaussian_model.py:534-564 (grads may cover only the first rows: zero padded)."""
    with torch.no_grad():
        P = _rows(self._xyz)
        g = torch.zeros(P, device=self._xyz.device)
        g[:grads.shape[0]] = grads.squeeze()
        flags, _, idx = classify(self, g, None, grad_threshold, self.percent_dense * scene_extent)
        ns = idx.numel()
        ext = _split_rows(self, idx, N, generator)
        if _prune_active(self, iter):
            # append the children and drop the split parents in the same pass
            keep = torch.cat((flags & SPLIT, torch.zeros(N * ns, dtype=torch.uint8,
                                                         device=flags.device)))
            index, count = select_rows(keep, SPLIT, 0)
            _rebuild(self, index, int(count.item()), ext, fresh_stats=True)
        else:
            _rebuild(self, None, P + N * ns, ext, fresh_stats=True)


def densify_and_prune(self, max_grad, min_opacity, extent, max_screen_size, iteration,
                      include_feature=False, generator=None):
    """scene/gaussian_model.py:583-604: clone, split, (proximity before iteration 2000), prune.

    Without proximity the whole update is ONE rebuild: the final keep set is known from the
    classify flags (a clone / split child inherits its parent's opacity; split children get the
    world-space size test on their own shrunk scales), so the rows
    [originals | clones | split children] are filtered and written in a single pass.

    Data parallel (one replica per rank): all-reduce the statistics first
    (gsr_amd.parallel.allreduce_densification_stats) and pass a generator seeded identically on
    every rank; every other step is deterministic, so the replicas stay bit-identical."""
    with torch.no_grad():
        P = _rows(self._xyz)
        big_limit = 0.1 * extent if max_screen_size else None
        flags, cidx, sidx = classify(self, self.xyz_gradient_accum.reshape(-1),
                                     self.denom.reshape(-1), max_grad,
                                     self.percent_dense * extent, min_opacity, big_limit)
        nc, ns = cidx.numel(), sidx.numel()
        ext = _cat_extras(_clone_rows(self, cidx), _split_rows(self, sidx, 2, generator))
        active = _prune_active(self, iteration)
        if iteration < 2000:
            # proximity needs the clone/split result materialised (its KNN runs on it)
            if active:
                keep = torch.cat((flags & SPLIT, torch.zeros(nc + 2 * ns, dtype=torch.uint8,
                                                             device=flags.device)))
                index, count = select_rows(keep, SPLIT, 0)
                _rebuild(self, index, int(count.item()), ext, fresh_stats=True)
            else:
                _rebuild(self, None, P + nc + 2 * ns, ext, fresh_stats=True)
            proximity(self, extent, include_feature)
            prune_mask = (self.get_opacity < min_opacity).squeeze()
            if max_screen_size:
                big_points_vs = self.max_radii2D > max_screen_size
                big_points_ws = self.get_scaling.max(dim=1).values > 0.1 * extent
                prune_mask = torch.logical_or(torch.logical_or(prune_mask, big_points_vs),
                                              big_points_ws)
            prune_points(self, prune_mask, iteration, include_feature)
            return
        if not active:
            _rebuild(self, None, P + nc + 2 * ns, ext, fresh_stats=True)
            return
        drop = LOW_OPACITY | BIG_WS
        new_clone = flags[cidx] & drop
        new_split = flags[sidx] & LOW_OPACITY
        new_split = new_split.repeat(2)
        if max_screen_size:
            big = self.scaling_activation(ext["scaling"][nc:]).max(dim=1).values > 0.1 * extent
            new_split = new_split | (big.to(torch.uint8) * BIG_WS)
            # max_radii2D was just reset to zero by the postfix: 0 > max_screen_size
            if bool(torch.tensor(0.0) > torch.tensor(max_screen_size, dtype=torch.float32)):
                flags = flags | LOW_OPACITY
                new_clone = new_clone | LOW_OPACITY
                new_split = new_split | LOW_OPACITY
        allf = torch.cat((flags, new_clone, new_split))
        index, count = select_rows(allf, SPLIT | drop, 0)
        _rebuild(self, index, int(count.item()), ext, fresh_stats=True)


def proximity(self, scene_extent, include_feature, N=3):
    """scene/gaussian_model.py:513-532: Gaussians far from their neighbours (mean squared 3-NN
    distance > 5 extent) and large (max scale > extent) get N new Gaussians at midpoints towards
    their neighbours (the reference's pairing: sources tiled, neighbour lists interleaved), with
    the neighbour's scale / opacity / language feature, identity rotation and zero colour.
    The 3-NN search is gsr_dist_knn3 (gsr_amd.knn.distCUDA2); the append is one rebuild."""
    from .knn import distCUDA2
    with torch.no_grad():
        dist, nearest = distCUDA2(self._xyz)
        sel = torch.logical_and(dist > (5.0 * scene_extent),
                                self.get_scaling.max(dim=1).values > scene_extent)
        index, count = select_rows(sel.to(torch.uint8), 1, 1)
        idx = index[:int(count.item())].long()
        new_indices = nearest[idx].reshape(-1).long()
        source_xyz = self._xyz[idx].repeat(1, N, 1).reshape(-1, 3)
        new_xyz = (source_xyz + self._xyz[new_indices]) / 2
        new_rotation = torch.zeros_like(self._rotation[new_indices])
        new_rotation[:, 0] = 1
        lang = self._language_feature
        ext = _extras_dict(new_xyz, torch.zeros_like(self._features_dc[new_indices]),
                           torch.zeros_like(self._features_rest[new_indices]),
                           None if lang is None or not _has_group(self, "language_feature")
                           else lang[new_indices],
                           self._opacity[new_indices], self._scaling[new_indices], new_rotation)
        _rebuild(self, None, _rows(self._xyz) + new_xyz.shape[0], ext, fresh_stats=True)


METHODS = ("add_densification_stats", "update_densification_stats",
           "update_densification_stats_views", "prune_points",
           "densification_postfix", "densify_and_clone", "densify_and_split", "densify_and_prune",
           "proximity")


def install(cls):
    """Swap the HIP implementations into a GaussianModel-like class (methods of the same names)."""
    g = globals()
    for name in METHODS:
        setattr(cls, name, g[name])
    return cls
