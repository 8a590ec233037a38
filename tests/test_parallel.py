"""Camera-sharded data parallelism on CPU with the gloo backend (world size 2).

The GPU path uses the same code with backend "nccl" (RCCL); here the per-view render is replaced by
a differentiable CPU stand-in so the sharding + bucketed all-reduce logic is exercised without a
device: the summed gradients of the sharded run must equal the single-process gradients over all
views."""
import os
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from gsr_amd.parallel import GradAllReducer, allreduce_densification_stats, shard_views


def _init_method():
    """File rendezvous: no TCP port to race for between picking it and binding it."""
    fd, path = tempfile.mkstemp(prefix="gsr_pg_")
    os.close(fd)
    os.unlink(path)
    return "file://" + path


def _params(seed=0):
    g = torch.Generator().manual_seed(seed)
    return [torch.randn((1000, 3), generator=g).requires_grad_(True),
            torch.randn((1000, 15, 3), generator=g).requires_grad_(True),
            torch.randn((1000, 1), generator=g).requires_grad_(True)]


def _view_loss(params, v):
    # stand-in for render(view v) + loss: a view-dependent smooth function of every parameter
    w = torch.sin(torch.arange(1, 4, dtype=torch.float32) * (v + 1))
    return ((params[0] * w).sum(1).pow(2).mean() + (params[1].sum(1) * w).pow(2).mean()
            + torch.sigmoid(params[2] * (v + 1)).mean())


def _worker(rank, world, init, n_views, bucket_bytes, attach, q):
    dist.init_process_group("gloo", init_method=init, rank=rank, world_size=world)
    params = _params()
    reducer = GradAllReducer(params, bucket_bytes=bucket_bytes)
    if attach:  # .grad are views into the all-reduce buffer (bench.py's training step)
        reducer.attach_grads()
    for v in shard_views(n_views, rank, world):
        _view_loss(params, v).backward()
    if attach:
        assert all(p.grad.data_ptr() == reducer.flat[o:o + 1].data_ptr()
                   for p, o in zip(params, reducer.offsets))
    reducer.allreduce()
    accum = torch.full((10,), float(rank + 1))
    denom = torch.ones(10)
    radii = torch.arange(10, dtype=torch.float32) * (rank + 1)
    allreduce_densification_stats(accum, denom, radii)
    if rank == 0:
        # numpy copies travel by value (torch tensors go through fd sharing, which races with
        # this process's exit)
        q.put(([p.grad.numpy().copy() for p in params], accum.numpy(), denom.numpy(), radii.numpy()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("n_views,bucket_bytes,attach", [(6, 64 << 20, False), (7, 4096, False),
                                                        (7, 4096, True)])
def test_sharded_allreduce_equals_single_process(n_views, bucket_bytes, attach):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    init = _init_method()
    procs = [ctx.Process(target=_worker, args=(r, 2, init, n_views, bucket_bytes, attach, q)) for r in range(2)]
    for p in procs:
        p.start()
    grads, accum, denom, radii = q.get(timeout=120)
    grads = [torch.from_numpy(g) for g in grads]
    accum, denom, radii = torch.from_numpy(accum), torch.from_numpy(denom), torch.from_numpy(radii)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = _params()
    for v in range(n_views):
        _view_loss(ref, v).backward()
    for g, r in zip(grads, ref):
        torch.testing.assert_close(g, r.grad, rtol=1e-5, atol=1e-6)
    assert torch.all(accum == 3.0) and torch.all(denom == 2.0)
    torch.testing.assert_close(radii, torch.arange(10, dtype=torch.float32) * 2)


class _Model:
    """Stand-in for a GaussianModel: densify() replaces every parameter with a new, longer one
    (gsr_amd.densify._rebuild does the same with nn.Parameters)."""

    def __init__(self):
        self.params = _params()

    def parameters(self):
        return list(self.params)

    def densify(self, extra=300):
        g = torch.Generator().manual_seed(99)
        self.params = [torch.cat([p.detach(), torch.randn((extra,) + tuple(p.shape[1:]),
                                                          generator=g)]).requires_grad_(True)
                       for p in self.params]


def _overlapped_worker(rank, world, init, n_views, q, sliced=False):
    """Two steps with a densification between them; the reducer is built once on the model.
    Step order as ViewPipeline.run(reducer=...): non-SH gradients reduced first, then the 'SH'
    parameter (params[1]) in row slices as they are 'flushed'."""
    dist.init_process_group("gloo", init_method=init, rank=rank, world_size=world)
    model = _Model()
    reducer = GradAllReducer(model, bucket_bytes=4096)
    out = []
    for step in range(2):
        if step == 1:
            model.densify()
        reducer.attach_grads()  # re-reads the (new) parameters
        ps = model.parameters()
        assert reducer.numel == sum(-(-p.numel() // 64) * 64 for p in ps)
        for v in shard_views(n_views, rank, world):
            _view_loss(ps, v + step).backward()
        reducer.begin()
        if sliced:  # the per-Gaussian backward's row slices (BackwardRowSlices), then the guard
            n = ps[0].shape[0]
            for a in range(0, n, 384):
                reducer.reduce_row_slices_async([ps[0], ps[2]], a, min(n, a + 384))
            reducer.reduce_async([], guard=True)
        else:
            reducer.reduce_async([ps[0], ps[2]])
        rows = ps[1].shape[0]
        for a in range(0, rows, 256):
            reducer.reduce_rows_async(ps[1], a, min(rows, a + 256))
        reducer.wait()
        out.append([p.grad.numpy().copy() for p in ps])
    if rank == 0:
        q.put(out)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("sliced", [False, True])
def test_overlapped_allreduce_follows_densification(sliced):
    """after densification replaces the parameters, the reducer rebuilds its flat
    buffer and the new .grad are the ones reduced; the sliced (overlapped) ordering gives the
    single-process gradients.  sliced: the non-SH gradients go out in row
    slices of all their parameters at once (reduce_row_slices_async, as the per-Gaussian
    backward's slices finish), the SH rows as flushed: still the single-process sums."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    init = _init_method()
    procs = [ctx.Process(target=_overlapped_worker, args=(r, 2, init, 5, q, sliced))
             for r in range(2)]
    for p in procs:
        p.start()
    out = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = _Model()
    for step in range(2):
        if step == 1:
            ref.densify()
        ps = ref.parameters()
        for p in ps:
            p.grad = None
        for v in range(5):
            _view_loss(ps, v + step).backward()
        for g, p in zip(out[step], ps):
            torch.testing.assert_close(torch.from_numpy(g), p.grad, rtol=1e-5, atol=1e-6)


def test_shard_views_partition():
    for n in range(0, 20):
        for world in (1, 2, 3, 8):
            shards = [shard_views(n, r, world) for r in range(world)]
            flat = [v for s in shards for v in s]
            assert flat == list(range(n))
            sizes = [len(s) for s in shards]
            assert max(sizes) - min(sizes) <= 1


def _guard_worker(rank, world, init, fail_rank, q):
    """the step's fault snapshot rides the gradient all-reduce (one float after the
    gradients, summed), so every rank learns that some rank's forward failed.  On CPU the device
    guard kernel does not run; the failing rank writes its slot the way gsr_step_guard would."""
    dist.init_process_group("gloo", init_method=init, rank=rank, world_size=world)
    params = _params()
    reducer = GradAllReducer(params, bucket_bytes=4096)
    if rank == fail_rank:
        reducer._write_guard = lambda: reducer.guard.fill_(1.0)
    out = []
    for step in range(2):
        reducer.attach_grads()
        assert float(reducer.guard) == 0.0  # zeroed with the gradients every step
        for v in shard_views(4, rank, world):
            _view_loss(params, v).backward()
        if step == 1:
            reducer._write_guard = lambda: None  # the failure was handled: a clean step
        reducer.begin()
        reducer.reduce_async([params[0], params[2]], guard=True)  # ViewPipeline's early batch
        rows = params[1].shape[0]
        for a in range(0, rows, 256):
            reducer.reduce_rows_async(params[1], a, min(rows, a + 256))
        reducer.wait()
        flag = reducer.skip_flag()
        out.append((None if flag is None else float(flag), [p.grad.numpy().copy() for p in params]))
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


def test_fault_guard_rides_the_allreduce():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    init = _init_method()
    procs = [ctx.Process(target=_guard_worker, args=(r, 2, init, 1, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = _params()
    for v in range(4):
        _view_loss(ref, v).backward()
    for rank in (0, 1):
        (flag0, g0), (flag1, g1) = res[rank]
        assert flag0 == 1.0, (rank, flag0)  # rank 1 failed: every rank skips step 0
        assert flag1 == 0.0, (rank, flag1)
        for gs in (g0, g1):  # the gradient sums are unaffected by the extra slot
            for g, r in zip(gs, ref):
                torch.testing.assert_close(torch.from_numpy(g), r.grad, rtol=1e-5, atol=1e-6)


def test_flat_buffer_slots_stay_aligned_under_row_changes():
    """Every parameter's gradient slot starts on a 256-byte boundary, also for row counts that are
    not multiples of 4 (densification): the multi-view backward writes float4 rows (rotations,
    SH planes) into these slots and refuses unaligned pointers."""
    rows = [1000]
    params = {}

    def current():
        n = rows[0]
        if params.get("n") != n:
            params["n"] = n
            params["t"] = [torch.zeros(n, 3), torch.zeros(n, 45), torch.zeros(n, 1),
                           torch.zeros(n, 3), torch.zeros(n, 4)]
        return params["t"]

    reducer = GradAllReducer(current)
    for n in (1000, 1018987, 7):
        rows[0] = n
        reducer.attach_grads()
        assert all(o % 64 == 0 for o in reducer.offsets)
        assert all(p.grad.data_ptr() % 256 == reducer.flat.data_ptr() % 256 for p in current())
        assert reducer.guard.data_ptr() >= current()[-1].grad.data_ptr() + 4 * n * 4
        reducer.zero_rows(0, n)
        assert reducer._prezeroed
