"""Fused Adam for the Gaussian parameters (include/gsr_optim.h).

`FusedAdam` is a drop-in for the optimizer GaussianModel.training_setup creates
(`torch.optim.Adam(param_groups, lr=0.0, eps=1e-15)`, scene/gaussian_model.py:217-271): it IS a
torch.optim.Adam (same constructor, param groups, state dict with exp_avg / exp_avg_sq / step), so
the reference's learning-rate schedule (`update_learning_rate`, :277) and its densification code,
which edits `optimizer.state` and `group["params"]` directly (:400-470), work unchanged.  Only
`step()` differs: every tensor of every group is updated by ONE HIP launch (one streaming pass,
28 B per element) instead of PyTorch's per-group foreach passes.  There is no CPU path.

Failed forwards (include/gsr_optim.h): the step is skipped ON THE DEVICE when the step's guard
slot is set -- the device's forward fault word snapshot, or, with a multi-GPU reducer, that
snapshot summed over the ranks (``step(skip=reducer.skip_flag())``), so every rank skips together
when any rank's forward failed.  The launch also reports the decision into a pinned host word; the
next step() reads it (no synchronisation in the normal case) and, for a skipped step, takes back
the step counts it had advanced (state["step"]: a skipped step leaves parameters, moments AND
counts as they were) and raises, unless reset_forward_faults() ran since the skipped step -- a
caller that swallows one error does not silently stall.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib

MAX_TENSORS = 16  # GSR_ADAM_MAX_TENSORS


class FusedAdam(torch.optim.Adam):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0,
                 amsgrad=False, *, maximize=False):
        if amsgrad or maximize:
            raise ValueError("FusedAdam implements Adam without amsgrad / maximize")
        super().__init__(params, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay,
                         amsgrad=False, foreach=False)
        self._mailbox = {}     # device -> pinned int32 [1]: 1 = the step's launches skipped it
        self._guard = {}       # device -> float32 [1] device slot: the step's one fault snapshot
        self._pending = None   # (events, mailboxes, stepped states, fault-reset count)
        self.skipped_steps = 0

    def _resolve_pending(self):
        """The previous step's device decision: undo its step counts if it was skipped."""
        pend, self._pending = self._pending, None
        if pend is None:
            return
        events, boxes, states, resets = pend
        for ev in events:
            if not ev.query():
                ev.synchronize()  # rare: the previous step's launch has not finished yet
        if not any(int(b[0]) for b in boxes):
            return
        for st in states:
            st["step"] -= 1
        self.skipped_steps += 1
        if _lib.fault_resets() == resets:
            raise RuntimeError(
                "FusedAdam: the previous step was skipped on the device because a rasterizer "
                "forward of that step failed (on this or another rank); parameters, moments and "
                "step counts are unchanged.  Handle the failure and call "
                "gsr_amd._lib.reset_forward_faults() before stepping again.")

    @torch.no_grad()
    def step(self, closure=None, *, skip=None):
        """One Adam step of every parameter with a gradient.  skip: a one-float device tensor
        whose non-zero value skips the step (GradAllReducer.skip_flag(): the ranks' summed fault
        snapshots); None = this device's own fault word."""
        self._resolve_pending()
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        h = self.begin_rows(skip=skip)
        self.step_rows(h, 0, None)
        self.end_rows(h)
        return loss

    # -- the step in row slices (multi-GPU: Adam on the rows whose all-reduce is done while the
    # next slice's collective runs, gsr_amd.trainer.train_step_views) ---------------------------
    @torch.no_grad()
    def begin_rows(self, *, skip=None):
        """Start a step applied in row ranges: the step counts advance once here and the
        (betas, eps) batches are fixed; step_rows(h, a, b) then updates rows [a, b) of every
        parameter (dim 0), end_rows(h) finishes.  The row ranges must cover every row exactly
        once; the result is bitwise the one of step() (the update is elementwise)."""
        self._resolve_pending()
        batches = {}
        for group in self.param_groups:
            beta1, beta2 = group["betas"]
            for p in group["params"]:
                if p.grad is None:
                    continue
                g = p.grad
                if g.is_sparse:
                    raise RuntimeError("FusedAdam does not support sparse gradients")
                if not p.is_cuda:
                    raise RuntimeError("FusedAdam updates HIP tensors only (no CPU path)")
                if p.dtype != torch.float32 or g.dtype != torch.float32:
                    raise RuntimeError("FusedAdam expects float32 parameters and gradients")
                state = self.state[p]
                if len(state) == 0:  # torch.optim.Adam._init_group layout
                    state["step"] = torch.tensor(0.0, dtype=torch.float32)
                    state["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    state["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                state["step"] += 1
                m, v = state["exp_avg"], state["exp_avg_sq"]
                for t, name in ((p, "param"), (g, "grad"), (m, "exp_avg"), (v, "exp_avg_sq")):
                    if not t.is_contiguous() or t.numel() != p.numel() or t.device != p.device:
                        raise RuntimeError(f"FusedAdam: {name} must be contiguous, on the "
                                           "parameter's device, with the parameter's size")
                key = (p.device, float(beta1), float(beta2), float(group["eps"]))
                batches.setdefault(key, []).append(
                    (p, g, m, v, float(group["lr"]), float(group["weight_decay"]),
                     float(state["step"])))
        skips = {}
        for (dev, _, _, _) in batches:
            if dev in skips:
                continue
            box = self._mailbox.get(dev)
            if box is None:
                box = torch.zeros(1, dtype=torch.int32, pin_memory=True)
                self._mailbox[dev] = box
            box[0] = 0
            if skip is not None and (skip.device != dev or skip.dtype != torch.float32):
                raise ValueError("FusedAdam.step: skip must be a float32 tensor on the parameters' device")
            if skip is None:
                # ONE snapshot of the device's fault word for every launch of the step (chunks of
                # MAX_TENSORS, (betas, eps) batches, row slices): a fault published between two
                # launches cannot leave some rows updated and others not
                slot = self._guard.get(dev)
                if slot is None:
                    slot = torch.zeros(1, dtype=torch.float32, device=dev)
                    self._guard[dev] = slot
                with _lib.on_device(dev):
                    _lib.step_guard(slot)
                skips[dev] = (slot.data_ptr(), box)
            else:
                skips[dev] = (skip.data_ptr(), box)
        states = [self.state[it[0]] for its in batches.values() for it in its]
        return {"batches": batches, "skips": skips, "states": states, "issued": False}

    def abort_rows(self, h):
        """Give back the step counts begin_rows advanced when the step is abandoned before any
        step_rows launch was issued (a forward or backward between them raised): the next step's
        bias corrections then see the counts of the updates actually applied.  Once a
        slice was issued the rows it updated used the advanced counts, so they are kept."""
        if h is None or h["issued"]:
            return
        for st in h["states"]:
            st["step"] -= 1
        h["issued"] = True  # idempotent

    @torch.no_grad()
    def step_rows(self, h, a: int, b):
        """Rows [a, b) of every parameter of the step begun by begin_rows (b None: to the end).
        Issued on the current stream of each parameter's device."""
        L = _lib.load()
        h["issued"] = True
        for (dev, beta1, beta2, eps), items in h["batches"].items():
            stream = _lib.raw_stream(dev)
            skip_ptr, box = h["skips"][dev]
            sel = []
            for it in items:
                rows = it[0].shape[0] if it[0].dim() else 1
                row = it[0].numel() // max(1, rows)
                lo, hi = a, rows if b is None else min(b, rows)
                if hi > lo:
                    sel.append((it, lo * row * 4, (hi - lo) * row))
            for c in range(0, len(sel), MAX_TENSORS):
                chunk = sel[c:c + MAX_TENSORS]
                n = len(chunk)
                ptrs = [(ctypes.c_void_p * n)(*[s[0][k].data_ptr() + s[1] for s in chunk])
                        for k in range(4)]
                numel = (ctypes.c_int64 * n)(*[s[2] for s in chunk])
                lr = (ctypes.c_double * n)(*[s[0][4] for s in chunk])
                wd = (ctypes.c_double * n)(*[s[0][5] for s in chunk])
                steps = (ctypes.c_double * n)(*[s[0][6] for s in chunk])
                with _lib.on_device(dev):
                    rc = L.gsr_adam_step_guarded(n, ptrs[0], ptrs[1], ptrs[2], ptrs[3], numel, lr,
                                                 wd, steps, beta1, beta2, eps, skip_ptr,
                                                 box.data_ptr(), stream)
                if rc != 0:
                    raise RuntimeError(f"gsr_adam_step failed with status {rc}")

    def end_rows(self, h):
        """Finish a step begun by begin_rows: its skip decision is read back by the next step."""
        events, boxes = [], []
        for dev, (_, box) in h["skips"].items():
            with _lib.on_device(dev):
                ev = torch.cuda.Event()
                ev.record(torch.cuda.current_stream(dev))
            events.append(ev)
            boxes.append(box)
        if events:
            self._pending = (events, boxes, h["states"], _lib.fault_resets())
