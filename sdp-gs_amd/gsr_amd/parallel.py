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
from typing import Iterable, List, Sequence

import torch
import torch.distributed as dist


def shard_views(n_views: int, rank: int, world: int) -> List[int]:
    """Contiguous, balanced camera shard of this rank (ranks differ by at most one view)."""
    base, extra = divmod(n_views, world)
    start = rank * base + min(rank, extra)
    return list(range(start, start + base + (1 if rank < extra else 0)))


class GradAllReducer:
    """Bucketed SUM all-reduce of .grad over a fixed list of parameters."""

    def __init__(self, params: Sequence[torch.Tensor], bucket_bytes: int = 64 << 20,
                 group=None, average: bool = False):
        self.params = list(params)
        self.group = group
        self.average = average
        dev = self.params[0].device
        self.numel = sum(p.numel() for p in self.params)
        self.flat = torch.zeros(self.numel, dtype=torch.float32, device=dev)
        # bucket boundaries on whole tensors where possible, split big tensors by elements
        per = max(1, bucket_bytes // 4)
        self.buckets = [(s, min(s + per, self.numel)) for s in range(0, self.numel, per)]
        self.offsets = []
        off = 0
        for p in self.params:
            self.offsets.append(off)
            off += p.numel()

    def attach_grads(self):
        """Zero the flat buffer and make every parameter's .grad a view into it (gradient as
        bucket view): the backward then accumulates straight into the all-reduce buffer and
        allreduce() needs no pack / unpack copies.  Call instead of zero_grad()."""
        self.flat.zero_()
        for p, off in zip(self.params, self.offsets):
            p.grad = self.flat[off:off + p.numel()].view_as(p)

    def _attached(self, p, off):
        g = p.grad
        return (g is not None and g.data_ptr() == self.flat[off:off + 1].data_ptr()
                and g.is_contiguous())

    def _pack(self):
        for p, off in zip(self.params, self.offsets):
            n = p.numel()
            if self._attached(p, off):
                continue
            if p.grad is None:
                self.flat[off:off + n].zero_()
            else:
                self.flat[off:off + n].copy_(p.grad.reshape(-1))

    def _unpack(self):
        for p, off in zip(self.params, self.offsets):
            n = p.numel()
            if self._attached(p, off):
                continue
            v = self.flat[off:off + n].view_as(p)
            if p.grad is None:
                p.grad = v.clone()
            else:
                p.grad.copy_(v)

    def allreduce(self):
        if not dist.is_available() or not dist.is_initialized() or dist.get_world_size(self.group) == 1:
            return
        self._pack()
        works = [dist.all_reduce(self.flat[a:b], op=dist.ReduceOp.SUM, group=self.group,
                                 async_op=True) for a, b in self.buckets]
        for w in works:
            w.wait()
        if self.average:
            self.flat.div_(dist.get_world_size(self.group))
        self._unpack()


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
