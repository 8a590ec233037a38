"""Camera-sharded data parallelism.

Every rank holds a full replica of the Gaussians, renders and back-propagates its own shard of the
cameras, then the per-Gaussian gradients are SUM-reduced across ranks with torch.distributed
(backend "nccl" = RCCL over xGMI on MI355X; "gloo" in the CPU tests).  The reference itself is
single-process (utils/general_utils.py:143); this is the one exchange step the sharded path has.

Design for xGMI (7 point-to-point links, ring collectives are per-link bound): the gradients of
all parameter tensors are packed into a few large flat buckets (default 64 MiB) and each bucket is
all-reduced asynchronously while the next one is packed, instead of one collective per tensor.
"""
from __future__ import annotations

import os
from typing import Iterable, List

import torch
import torch.distributed as dist


def shard_views(n_views: int, rank: int, world: int) -> List[int]:
    """Contiguous, balanced camera shard of this rank (ranks differ by at most one view)."""
    base, extra = divmod(n_views, world)
    start = rank * base + min(rank, extra)
    return list(range(start, start + base + (1 if rank < extra else 0)))


class GradAllReducer:
    """Bucketed SUM all-reduce of .grad over the model's parameters.

    ``params`` is the model (anything with ``.parameters()``), a callable returning the current
    parameter list, or a fixed sequence.  With a model or a callable the parameter list is re-read
    at every attach_grads() / allreduce() / begin(): densification (gsr_amd.densify) replaces every
    parameter with a new tensor of another row count, and the flat buffer, its offsets and buckets
    are rebuilt whenever the list (identity or size) changes -- a fixed sequence cannot see that.

    Two ways to use it per step:
      * ``allreduce()`` after the step's backward: one bucketed all-reduce of everything;
      * overlapped (ViewPipeline.run(..., reducer=...)): ``begin()``, then ``reduce_async(params)``
        as soon as those gradients are final (the non-SH leaves, right after the last view's
        backward) and ``reduce_rows_async(param, a, b)`` for row slices finished later (the SH
        gradients, flushed in bucket-sized row ranges), then ``wait()``.  RCCL runs the
        collectives on its own stream, ordered after the work already issued on the current
        stream, so they overlap the flush of the next slice.

    Failed forwards: one extra float after the gradients, ``guard``, carries the
    device's forward-fault snapshot (include/gsr_optim.h gsr_step_guard, written on the current
    stream once every forward of the step is done) through the same SUM all-reduce, merged into
    the collective of the last parameter.  After ``wait()``, ``skip_flag()`` is that slot: non-zero
    on EVERY rank when any rank's forward failed, and ``FusedAdam.step(skip=...)`` then skips the
    step everywhere -- a failed rank's NaN gradients are in every rank's summed gradients.
    """

    _ALIGN = 64  # floats (256 B) between parameter slots of the flat buffer

    def __init__(self, params, bucket_bytes: int = 64 << 20, group=None, average: bool = False):
        self._source = params
        self.group = group
        self.average = average
        self.bucket_bytes = int(bucket_bytes)
        self._sig = None
        self._works = []
        self._sync_layout()

    # -- layout -----------------------------------------------------------------------------------
    def current_params(self) -> List[torch.Tensor]:
        src = self._source
        if hasattr(src, "parameters"):
            ps = src.parameters()
        elif callable(src):
            ps = src()
        else:
            ps = src
        return [p for p in ps if p is not None]

    def _sync_layout(self):
        params = self.current_params()
        sig = tuple((id(p), p.numel(), str(p.device)) for p in params)
        if sig == self._sig:
            return False
        if self._works:
            raise RuntimeError("GradAllReducer: parameters changed while collectives are in flight")
        self._sig = sig
        self.params = params
        dev = params[0].device
        # Every parameter's slot starts on a _ALIGN-float boundary: the kernels writing gradients
        # into it take float4 rows (rotations, SH planes) and refuse unaligned pointers, and the
        # row counts change under densification.  The gaps stay zero on every rank, so reducing
        # them with their neighbours is harmless.
        self.offsets = []
        off = 0
        for p in params:
            self.offsets.append(off)
            off += -(-p.numel() // self._ALIGN) * self._ALIGN
        self.numel = off
        self.flat = torch.zeros(self.numel + 1, dtype=torch.float32, device=dev)
        self.guard = self.flat[self.numel:]  # the step's fault snapshot (see the class docstring)
        per = max(1, self.bucket_bytes // 4)
        self.buckets = [(s, min(s + per, self.numel)) for s in range(0, self.numel, per)]
        self._index = {id(p): i for i, p in enumerate(params)}
        return True

    def _active(self):
        return dist.is_available() and dist.is_initialized() and \
            dist.get_world_size(self.group) > 1

    def attach_grads(self):
        """Zero the flat buffer and make every parameter's .grad a view into it (gradient as
        bucket view): the backward then accumulates straight into the all-reduce buffer and the
        reduction needs no pack / unpack copies.  Call instead of zero_grad().  After a step whose
        row slices were zeroed behind the optimizer (zero_rows over every row, the next step's
        prologue done slice by slice) only the guard slot is cleared."""
        changed = self._sync_layout()
        if changed or not getattr(self, "_prezeroed", False):
            self.flat.zero_()
        else:
            self.guard.zero_()
        self._prezeroed = False
        self._zeroed_rows = 0
        for p, off in zip(self.params, self.offsets):
            p.grad = self.flat[off:off + p.numel()].view_as(p)

    def zero_rows(self, a: int, b: int):
        """Zero rows [a, b) of every parameter's slot in the flat buffer (on the current stream,
        after the optimizer read them): the next step's gradient zeroing, one slice at a time.
        Once the slices cover every row, the next attach_grads() skips its full-buffer fill."""
        views = []
        for i, p in enumerate(self.params):
            _, lo, hi = self._range(p, a, b)
            if hi > lo:
                views.append(self.flat[lo:hi])
        if views:
            torch._foreach_zero_(views)
        rows = self.params[0].shape[0] if self.params else 0
        self._zeroed_rows = getattr(self, "_zeroed_rows", 0) + max(0, min(b, rows) - a)
        same_rows = all(p.shape[0] == rows for p in self.params)
        self._prezeroed = same_rows and self._zeroed_rows >= rows

    def _attached(self, p, off):
        g = p.grad
        return (g is not None and g.is_contiguous() and g.numel() == p.numel()
                and g.data_ptr() == self.flat[off:off + 1].data_ptr())

    def _range(self, p, a=None, b=None):
        """Flat [lo, hi) of rows [a, b) of parameter p (all rows when a is None)."""
        i = self._index.get(id(p))
        if i is None:
            raise KeyError("GradAllReducer: not one of the current parameters")
        off, n = self.offsets[i], p.numel()
        if a is None:
            return i, off, off + n
        row = n // max(1, p.shape[0])
        return i, off + a * row, off + min(b, p.shape[0]) * row

    def _pack(self, i, lo, hi):
        p, off = self.params[i], self.offsets[i]
        if self._attached(p, off):
            return
        dst = self.flat[lo:hi]
        if p.grad is None:
            dst.zero_()
        else:
            dst.copy_(p.grad.reshape(-1)[lo - off:hi - off])

    def _issue(self, lo, hi):
        per = max(1, self.bucket_bytes // 4)
        for a in range(lo, hi, per):
            self._works.append(dist.all_reduce(self.flat[a:min(a + per, hi)],
                                               op=dist.ReduceOp.SUM, group=self.group,
                                               async_op=True))

    # -- overlapped use -----------------------------------------------------------------------------
    def begin(self):
        """Start of a step's reduction: re-read the parameters (after a densification)."""
        self._sync_layout()
        self._works = []
        self._slice_works = []  # (a, b, works) of reduce_row_slices_async, in issue order
        self._guard_works = []
        self._done = set()
        self._guarded = False

    def _write_guard(self):
        """The device's fault snapshot into the guard slot, on the current stream."""
        if self.flat.is_cuda:
            from . import _lib
            _lib.step_guard(self.guard)

    def skip_flag(self):
        """The all-reduced fault slot of this step (a one-float device tensor for
        FusedAdam.step(skip=...)), or None when no guard went through a collective."""
        return self.guard if getattr(self, "_guarded", False) else None

    def reduce_async(self, params: Iterable[torch.Tensor], guard: bool = False):
        """Start the all-reduce of these parameters' whole gradients (no-op at world size 1).
        guard: also reduce the step's fault snapshot (call once the step's forwards are done)."""
        if not self._active():
            return
        spans = []
        n0 = len(self._works)
        if guard:
            self._write_guard()
            spans.append((self.numel, self.numel + 1))
            self._guarded = True
        for p in params:
            i, lo, hi = self._range(p)
            self._pack(i, lo, hi)
            spans.append((lo, hi))
            self._done.add(i)
        spans.sort()
        merged = []
        for lo, hi in spans:  # adjacent tensors of the flat buffer go out as one collective
            if merged and lo - merged[-1][1] < self._ALIGN:  # only alignment padding between
                merged[-1] = (merged[-1][0], hi)
            else:
                merged.append((lo, hi))
        for lo, hi in merged:
            self._issue(lo, hi)
        if guard:
            self._guard_works = self._works[n0:]

    def reduce_rows_async(self, p: torch.Tensor, a: int, b: int):
        """Start the all-reduce of rows [a, b) of p's gradient."""
        if not self._active():
            return
        i, lo, hi = self._range(p, a, b)
        self._pack(i, lo, hi)
        self._issue(lo, hi)
        self._done.add(i)

    def reduce_row_slices_async(self, params: Iterable[torch.Tensor], a: int, b: int):
        """Start the all-reduce of rows [a, b) of several parameters' gradients -- one span per
        parameter, issued as ONE coalesced collective on RCCL (a row slice of the per-Gaussian
        backward, diff_gaussian_rasterization.BackwardRowSlices), so a slice costs one
        collective's latency, not one per parameter."""
        if not self._active():
            return
        spans = []
        for p in params:
            i, lo, hi = self._range(p, a, b)
            if hi <= lo:
                continue
            self._pack(i, lo, hi)
            spans.append((lo, hi))
            self._done.add(i)
        if not spans:
            return
        n0 = len(self._works)
        if len(spans) > 1 and self._coalesce():
            from torch.distributed.distributed_c10d import _coalescing_manager
            group = self.group or dist.group.WORLD
            with _coalescing_manager(group=group, device=self.flat.device, async_ops=True) as cm:
                for lo, hi in spans:
                    dist.all_reduce(self.flat[lo:hi], op=dist.ReduceOp.SUM, group=self.group)
            self._works.append(cm)
        else:
            for lo, hi in spans:
                self._issue(lo, hi)
        self._slice_works.append((a, b, self._works[n0:]))

    def each_reduced_slice(self, fn):
        """For each row slice reduced by reduce_row_slices_async, in issue order: make the
        current stream wait for that slice's collectives, then call fn(a, b) -- work issued there
        (the optimizer on those rows) overlaps the next slices' collectives.  No-op at world
        size 1 (fn is not called: the caller runs its unsliced path).  Returns whether it ran."""
        if not self._active() or not self._slice_works:
            return False
        if self.average:
            raise RuntimeError("each_reduced_slice: averaging reducers are not sliced")
        if not getattr(self, "_guarded", False):
            raise RuntimeError("each_reduced_slice: reduce the step's guard before its slices")
        # fn reads the reduced rows through p.grad: every gradient must be a view of the flat
        # buffer (a detached .grad would give fn the local, unreduced values)
        for p, off in zip(self.params, self.offsets):
            if not self._attached(p, off):
                raise RuntimeError("each_reduced_slice: a parameter's .grad is not a view of the "
                                   "flat all-reduce buffer (call attach_grads() before the backward)")
        for w in self._guard_works:  # the skip decision first (every slice's optimizer reads it)
            w.wait()
        for a, b, works in self._slice_works:
            for w in works:
                w.wait()
            fn(a, b)
        return True

    def _coalesce(self) -> bool:
        """RCCL groups coalesced all-reduces into one launch; gloo issues them one by one."""
        try:
            from torch.distributed.distributed_c10d import _coalescing_manager  # noqa: F401
        except ImportError:  # pragma: no cover - older torch
            return False
        return dist.get_backend(self.group) == "nccl" and self.flat.is_cuda

    def wait(self):
        """Finish the step's reduction: wait for the collectives (their results are ordered
        before later work on the current stream), average if asked, unpack non-view grads."""
        if not self._active():
            return
        for w in self._works:
            w.wait()
        self._works = []
        if self.average:
            self.flat.div_(dist.get_world_size(self.group))
        for i, (p, off) in enumerate(zip(self.params, self.offsets)):
            if i not in self._done or self._attached(p, off):
                continue
            v = self.flat[off:off + p.numel()].view_as(p)
            if p.grad is None:
                p.grad = v.clone()
            else:
                p.grad.copy_(v)

    # -- one-shot ------------------------------------------------------------------------------------
    def allreduce(self):
        if not self._active():
            return
        self.begin()
        self.reduce_async(self.params, guard=True)
        self.wait()


def allreduce_densification_stats(xyz_gradient_accum: torch.Tensor, denom: torch.Tensor,
                                  max_radii2D: torch.Tensor, group=None):
    """Densification statistics across ranks: SUM for the accumulated per-view
    viewspace-gradient norms and view counts, MAX for the screen radii."""
    if not dist.is_available() or not dist.is_initialized() or dist.get_world_size(group) == 1:
        return
    dist.all_reduce(xyz_gradient_accum, op=dist.ReduceOp.SUM, group=group)
    dist.all_reduce(denom, op=dist.ReduceOp.SUM, group=group)
    dist.all_reduce(max_radii2D, op=dist.ReduceOp.MAX, group=group)


def init_from_env(backend: str = "nccl"):
    """One process per GPU (torch.distributed.run env: RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*).
    Returns (rank, world, device index).  GSR_DIST_BACKEND overrides the backend (e.g. "gloo" to
    rehearse several ranks on one GPU: the device index is LOCAL_RANK modulo the visible GPUs)."""
    backend = os.environ.get("GSR_DIST_BACKEND", backend)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()  # does not initialise the device
    dev_index = local % ndev if ndev > 0 else local
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            torch.cuda.set_device(dev_index)
            dist.init_process_group(backend, device_id=torch.device("cuda", dev_index))
        else:
            dist.init_process_group(backend)
    return rank, world, dev_index
