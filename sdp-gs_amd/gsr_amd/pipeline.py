"""Multi-view step on several HIP streams (several views per GPU per
optimizer step, gradients summed over the views).

Within one step the views only read the Gaussians and add into the same .grad tensors, so view
k+1's forward (preprocess, depth sort, scan, the instance-count read-back, binning and tile sort --
mostly latency-bound launches that leave most CUs idle) can run while view k's backward blend (a
full-chip, VALU-bound launch) is still executing.  ViewPipeline issues view i on stream i mod depth;
the only cross-view dependency, the read-modify-write of the leaves' .grad by the fused backward's
grad-into-leaves mode, is ordered by diff_gaussian_rasterization itself (one event per device,
see ``_order_leaf_grads``), so any multi-stream caller gets correct accumulation, not only this
helper.  The reference renders one view per step on the legacy default stream
(train.py:64-236); with depth = 1 this helper is exactly that sequential loop.

With defer_sh (default), the grad-into-leaves backwards of the step store each view's
clamp-masked colour gradient dL/dRGB [P,3] instead of read-modify-writing the 192-byte SH
gradient rows, and run() writes features_dc / features_rest .grad once at the end
(diff_gaussian_rasterization.ShGradDeferral): the SH gradient of a view is basis(dir) x dL/dRGB,
so the per-view SH traffic drops from 384 to 12 bytes per Gaussian.

With precolor (default) and the model passed to run(), one pre-pass over the SH rows computes
every view's colour, clamp bits and colour Jacobian up front (diff_gaussian_rasterization.
ShPrecolor, gsr_sh_precolor); the views' forward and backward preprocesses then read 12 + 1 and
36 bytes per Gaussian instead of the 192-byte SH rows each.
"""
from __future__ import annotations

import contextlib
from typing import Callable, Iterable, List, Optional, TypeVar

import torch

from . import _lib

T = TypeVar("T")
R = TypeVar("R")


class ViewPipeline:
    """Round-robin per-view work over ``depth`` streams: the caller's current stream plus
    ``depth - 1`` side streams, joined back into the current stream at the end of run()."""

    def __init__(self, device: Optional[torch.device] = None, depth: int = 2,
                 defer_sh: bool = True, precolor: bool = True, bwd_slices: int = 4):
        if depth < 1:
            raise ValueError("depth must be >= 1")
        self.device = torch.device(device) if device is not None else torch.device(
            "cuda", torch.cuda.current_device())
        self.depth = depth
        self.defer_sh = defer_sh
        self.precolor = precolor
        # with a reducer: the multi-view backward's per-Gaussian part in this many row slices,
        # each slice's non-SH gradient rows all-reduced as soon as it is written (run_views)
        self.bwd_slices = bwd_slices
        self._pre_bufs = None  # the pre-pass's per-view buffers, reused step after step
        self.side = [torch.cuda.Stream(device=self.device) for _ in range(depth - 1)]
        self._slices = None  # the step's BackwardRowSlices while run_views issues
        self._prepared = None  # (campos ptrs, ShPrecolor) of the next step, filled slice by slice
        self.rows_done = False

    def run(self, items: Iterable[T], fn: Callable[[T], R], model=None,
            campos_of: Callable[[T], torch.Tensor] = lambda cam: cam.camera_center,
            reducer=None, bwd: Optional[Callable[[R], R]] = None, lag: int = 1) -> List[R]:
        """Call fn(item) for every item, item i issued on stream i mod depth.  fn should do a
        view's render + backward and return host values (or tensors it no longer needs on the
        device): tensors created on a side stream and used after run() on the main stream need
        Tensor.record_stream to be safe under the caching allocator.  With defer_sh the SH
        leaves' .grad is complete when run() returns, not after each view.  model (a
        GaussianModel: _xyz, _features_dc, _features_rest, active_sh_degree) enables the colour
        pre-pass for the cameras campos_of(item).

        reducer (gsr_amd.parallel.GradAllReducer over model's parameters, multi-GPU): the
        step's gradient all-reduce is overlapped with the end of the step -- the non-SH
        gradients (final once the last view's backward is done) are reduced while the deferred
        SH gradients are flushed in bucket-sized row slices, each slice reduced as soon as it is
        flushed.  The reduction is complete (on the current stream) when run() returns.

        bwd: split views -- fn(item) does a view's forward and returns what bwd needs, bwd(that)
        its backward (same stream); view i's backward is issued after view i + lag's forward
        (software-pipelined issue: the next view's latency-bound binning is queued before this
        view's full-chip backward blend).  Returns bwd's results."""
        self._check(reducer, model)
        items = list(items)
        main = torch.cuda.current_stream(self.device)
        streams = [main] + self.side

        def issue(out):
            for i, it in enumerate(items):
                s = streams[i % self.depth]
                with _lib.on_stream(s):
                    out.append(fn(it))
                j = i - lag
                if bwd is not None and j >= 0:
                    with _lib.on_stream(streams[j % self.depth]):
                        out[j] = bwd(out[j])
            if bwd is not None:
                for j in range(max(0, len(items) - lag), len(items)):
                    with _lib.on_stream(streams[j % self.depth]):
                        out[j] = bwd(out[j])
            for s in self.side:
                main.wait_stream(s)
            return out

        return self._step(items, issue, model, campos_of, reducer)

    def run_views(self, items: Iterable[T], fn: Callable[[List[T], List[torch.cuda.Stream]], R],
                  model=None, campos_of: Callable[[T], torch.Tensor] = lambda cam: cam.camera_center,
                  reducer=None, chunks: int = 1, after_slice: Optional[Callable] = None):
        """The step's views in ONE multi-view call: fn(items, streams) renders all of them at once
        (gaussian_renderer.render_views(items, ..., streams=streams): one host call issues every
        view's forward, autograd one call for every backward) and runs their backward; the views
        are spread over this pipeline's streams inside the library, which joins them back into the
        current stream.  Pre-pass, deferred SH gradients and the overlapped all-reduce as run().
        Returns fn's result.

        chunks > 1: the views in that many consecutive chunks, one multi-view call each, chunk c
        issued with streams (2c, 2c + 1) mod depth of [current] + side as its call and binning
        streams -- so chunk c + 1's forward (latency-bound binning) runs beside chunk c's backward
        blend instead of queueing behind it on one stream, and its buffers come from its own
        stream's allocator pool (never memory that an earlier chunk's backward still reads).  The
        grad-into-leaves backwards are ordered by diff_gaussian_rasterization; the row-sliced
        all-reduce (reducer) runs on the last chunk's per-Gaussian backward only.  Returns the
        list of fn's results.

        after_slice(a, b) (with a reducer): called on the current stream for each row slice of
        the per-Gaussian backward once every gradient of rows [a, b) -- SH included -- is reduced,
        in row order, while the later slices' collectives are still running (the optimizer on
        those rows: gsr_amd.trainer.train_step_views).  self.rows_done says whether it ran for
        every row; when it did not (world size 1, no row slices, SH gradients deferred to a
        flush) the caller runs its unsliced path."""
        self._check(reducer, model)
        items = list(items)
        main = torch.cuda.current_stream(self.device)
        streams = [main] + self.side
        n = max(1, min(int(chunks), len(items)))

        def issue(out):
            if n == 1:
                out.append(fn(items, streams))
                return out
            bounds = [round(i * len(items) / n) for i in range(n + 1)]
            for c, (a, b) in enumerate(zip(bounds[:-1], bounds[1:])):
                cs = [streams[(2 * c) % self.depth], streams[(2 * c + 1) % self.depth]]
                if cs[1] is cs[0]:
                    cs = cs[:1]
                if self._slices is not None:  # the leaves' rows are final after the last chunk only
                    self._slices.active = c == n - 1
                with _lib.on_stream(cs[0]):
                    out.append(fn(items[a:b], cs))
            for s in self.side:
                main.wait_stream(s)
            return out

        # one call: the library orders its streams after the current one itself
        out = self._step(items, issue, model, campos_of, reducer, sliced=True,
                         after_slice=after_slice, join_side=n > 1)
        return out[0] if n == 1 else out

    def prepare_next(self, model, items, campos_of=lambda cam: cam.camera_center):
        """The next step's colour pre-pass (SH colour, clamp bits, colour Jacobian of `items`'
        cameras), to be filled row slice by row slice: returns fill(a, b), which issues rows
        [a, b) on the current stream -- after the optimizer updated those rows.  The next run() /
        run_views() over the same cameras uses it when every row was filled and the model's
        tensors are the same (no densification in between); otherwise it computes its own.
        Issue every fill after this step's forwards and backwards (the buffers are this step's)."""
        import diff_gaussian_rasterization as dgr
        if not (self.precolor and items):
            return lambda a, b: None
        campos = [campos_of(it) for it in items]
        pre = dgr.ShPrecolor(model._xyz, model._features_dc, model._features_rest,
                             model.active_sh_degree, campos, buffers=self._pre_bufs, rows=True)
        self._prepared = ([c.data_ptr() for c in campos], pre)
        return pre.compute_rows

    def _check(self, reducer, model):
        if reducer is not None and self.defer_sh and model is None:
            # the early all-reduce must leave out the SH leaves, whose deferred gradients are only
            # written by the flush at the end of the step; without the model they are unknown
            raise ValueError("ViewPipeline.run: a reducer with defer_sh needs model= (the SH "
                             "leaves are reduced after the deferred flush)")

    def _step(self, items, issue, model, campos_of, reducer, sliced=False, after_slice=None,
              join_side=True):
        import diff_gaussian_rasterization as dgr
        main = torch.cuda.current_stream(self.device)
        self.rows_done = False
        pre = contextlib.nullcontext()
        prepared, self._prepared = self._prepared, None
        if self.precolor and model is not None and items:
            campos = [campos_of(it) for it in items]
            if (prepared is not None and prepared[1].complete
                    and prepared[0] == [c.data_ptr() for c in campos]
                    and prepared[1].lookup(campos[0], model._xyz, model._features_dc,
                                           model._features_rest, model.active_sh_degree,
                                           prepared[1].M) is not None):
                # filled slice by slice behind the previous step's optimizer (prepare_next)
                pre = prepared[1]
            else:
                # one kernel ahead of the forward: colours and Jacobians of every view
                pre = dgr.ShPrecolor(model._xyz, model._features_dc, model._features_rest,
                                     model.active_sh_degree, campos, buffers=self._pre_bufs)
            # reuse next step: its pre-pass is issued on this stream after this step's join
            self._pre_bufs = pre.buffers
        if join_side and self.side:
            # inputs prepared on the main stream (zeroed grads, pre-pass): one event for all sides
            # (each event record after a kernel costs the GPU a few us before the next launch)
            ev = torch.cuda.Event()
            ev.record(main)
            for s in self.side:
                s.wait_event(ev)
        out = []
        sh_leaves = ()
        on_rows, chunk = None, 0
        if reducer is not None:
            reducer.begin()
            if self.defer_sh and model is not None:
                dc, rest = model._features_dc, model._features_rest
                sh_leaves = tuple(t for t in (dc, rest) if t is not None)
                row_bytes = sum(t[0].numel() * 4 for t in sh_leaves)
                chunk = max(256, reducer.bucket_bytes // max(1, row_bytes))

                def on_rows(a, b):
                    for t in sh_leaves:
                        reducer.reduce_rows_async(t, a, b)
        # run_views: a multi-view call holding the step's views forms the SH gradients in its
        # per-Gaussian launch (ShGradDeferral.fuse_views); run(): one flush at the end
        defer = (dgr.ShGradDeferral(self.device, on_rows=on_rows, chunk_rows=chunk,
                                    fuse_views=sliced)
                 if self.defer_sh else contextlib.nullcontext())

        def fused():  # the SH rows were written with the others (final with the backward's rows)
            return getattr(defer, "fused", False)

        slices = contextlib.nullcontext()
        guarded = [False]
        if reducer is not None and sliced and self.bwd_slices > 1:
            ids = {id(t) for t in sh_leaves}
            rest = [p for p in reducer.current_params() if id(p) not in ids]

            def on_slice(a, b):
                if not guarded[0]:
                    # the step's fault snapshot ahead of the first slice: every forward of the
                    # step is ordered before the backward, and the optimizer slices need the
                    # reduced skip decision before their rows' collectives are done
                    reducer.reduce_async([], guard=True)
                    guarded[0] = True
                reducer.reduce_row_slices_async(rest + (list(sh_leaves) if fused() else []), a, b)
            slices = dgr.BackwardRowSlices(self.device, on_slice, self.bwd_slices)
            self._slices = slices
        with pre, defer:  # defer's exit: the SH gradients of all views, after the join
            try:
                with slices:
                    issue(out)
            finally:
                self._slices = None
            if reducer is not None:  # every view's backward is done: the non-SH grads are final
                ids = set() if fused() else {id(t) for t in sh_leaves}
                # (with the step's fault snapshot: every forward of the step is done)
                if getattr(slices, "ran", False):  # already reduced slice by slice
                    if not guarded[0]:
                        reducer.reduce_async([], guard=True)
                else:
                    reducer.reduce_async([p for p in reducer.current_params()
                                          if id(p) not in ids], guard=True)
        if reducer is not None:
            if sh_leaves and not defer.views_flushed and not fused():
                reducer.reduce_async(sh_leaves)  # no view produced deferred SH gradients
            if (after_slice is not None and getattr(slices, "ran", False)
                    and (fused() or not sh_leaves)):
                self.rows_done = reducer.each_reduced_slice(after_slice)
            reducer.wait()
        return out
