"""The multi-GPU step's gradient plumbing on the HIP path, in one process (world size 1, gloo
and RCCL over the device tensors): gradient-as-bucket-view (the fused backward accumulates straight into the
all-reduce buffer), the deferred SH flush written into the bucket in row slices, and the
overlapped all-reduce of ViewPipeline.run(reducer=) give the gradients of the same step without a
reducer (the collectives are issued at world size 1 too, so their stream ordering
against the flush is checked).  tests/test_parallel.py covers the cross-rank sums (world size 2,
CPU); this covers the rasterizer-side writes into the bucket, which have no CPU path.
One process only: no GPU work is started in a child process."""
import os

import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu


class _Pipe:
    convert_SHs_python = True
    compute_cov3D_python = False
    debug = False
    use_confidence = False


class _Opt:
    include_feature = True


def _scene(dev):
    from gsr_amd.model import SplatModel
    from gsr_amd.synthetic import make_cameras, make_gaussians, upstream_grads
    model = SplatModel(make_gaussians(20_001, sh_degree=3, seed=3), device=dev)
    cams = [c.to(dev) for c in make_cameras(4, 320, 240, seed=5)]
    grads = upstream_grads(240, 320, seed=7, device=dev)
    return model, cams, grads


def _step(model, cams, grads, views, reducer, multi=False, chunks=1):
    from gaussian_renderer import render, render_views
    dimg, ddep, dfeat = grads
    bg = torch.zeros(3, device=dimg.device)

    def one_view(cam):
        pkg = render(cam, model, _Pipe(), bg, _Opt())
        torch.autograd.backward([pkg["render"], pkg["depth"], pkg["feature"]], [dimg, ddep, dfeat])

    def all_views(cs, strs):  # the multi-view call: its backward runs in row slices
        pkgs = render_views(cs, model, _Pipe(), bg, _Opt(), streams=strs)
        st = pkgs[0]["views"]
        V = len(pkgs)
        torch.autograd.backward([st["render"], st["depth"], st["feature"]],
                                [g.expand(V, *g.shape) for g in (dimg, ddep, dfeat)])

    if reducer is not None:
        reducer.attach_grads()
    else:
        for p in model.parameters():
            p.grad = None
    if multi:
        views.run_views(cams, all_views, model=model, reducer=reducer, chunks=chunks)
    else:
        views.run(cams, one_view, model=model, reducer=reducer)
    torch.cuda.synchronize()
    return [p.grad.detach().clone() for p in model.parameters()]


@pytest.fixture(params=["gloo", "nccl"])
def world1(request, tmp_path):
    """A world-size-1 process group.  gloo: every collective round-trips through host memory, so
    a collective issued before its slice was flushed returns stale zeros.  nccl (= RCCL on ROCm):
    the bench's multi-GPU backend -- its initialisation, its internal stream and the ordering of
    each collective after the flush on the current stream run on the GPU."""
    init = "file://" + os.path.join(str(tmp_path), "pg")
    if request.param == "nccl":
        dist.init_process_group("nccl", init_method=init, rank=0, world_size=1,
                                device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group("gloo", init_method=init, rank=0, world_size=1)
    try:
        yield request.param
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("bucket_bytes,multi,chunks", [(64 << 20, False, 1), (256 << 10, False, 1),
                                                       (64 << 20, True, 1), (256 << 10, True, 1),
                                                       (256 << 10, True, 2)])
def test_bucket_view_grads_equal_plain_step(world1, bucket_bytes, multi, chunks):
    """chunks = 2: the step's views in two multi-view calls on their own streams (run_views
    chunks=; the row-sliced all-reduce on the last chunk only), against the one-call step."""
    import diff_gaussian_rasterization as dgr
    from gsr_amd.parallel import GradAllReducer
    from gsr_amd.pipeline import ViewPipeline
    dev = torch.device("cuda", 0)
    prev = dgr.grad_into_leaves()
    dgr.grad_into_leaves(True)
    try:
        model, cams, grads = _scene(dev)
        views = ViewPipeline(dev, depth=2 * chunks, defer_sh=True, precolor=True)
        ref = _step(model, cams, grads, views, None, multi)
        reducer = GradAllReducer(model, bucket_bytes=bucket_bytes)
        # issue the collectives at world size 1 as well: gloo copies each slice to the host and
        # back, so a collective that ran before its slice was flushed would write stale zeros
        reducer._active = lambda: True
        for _ in range(2):  # the second step reuses the attached buffer (zeroed by attach_grads)
            got = _step(model, cams, grads, views, reducer, multi, chunks)
            for p, g, r in zip(model.parameters(), got, ref):
                assert g.shape == r.shape
                # the backward's float atomics make two runs of a view differ in the last bits
                # (as the reference's); a collective racing its slice would zero whole rows
                err = float((g - r).abs().max())
                assert err <= 1e-5 * float(r.abs().max()) + 1e-30, (tuple(p.shape), err)
            # the .grad tensors are views into the flat all-reduce buffer
            base = reducer.flat.data_ptr()
            end = base + reducer.flat.numel() * 4
            assert all(base <= p.grad.data_ptr() < end for p in model.parameters())
        assert any(float(r.abs().max()) > 0 for r in ref)
        assert float(reducer.skip_flag()) == 0.0  # the fault snapshot went through too
        if world1 == "nccl":
            assert dist.get_backend() == "nccl"
    finally:
        dgr.grad_into_leaves(prev)


def test_sliced_adam_equals_serial_step(world1):
    """the multi-GPU training step with the optimizer in row slices (FusedAdam
    on rows [a, b) as soon as that slice's all-reduce is done, overlapping the next slice's
    collective, then the next step's prologue for those rows: its gradient zeroing and its colour
    pre-pass, used by the next step) gives bitwise the
    parameters, moments and step counts of the serial step (all-reduce, wait, one Adam step) --
    over three iterations, the middle one a densification (which takes the serial order: densify,
    then Adam).  Deterministic backward, so the two runs' gradients are bitwise equal."""
    import diff_gaussian_rasterization as dgr
    from gsr_amd import trainer
    from gsr_amd.model import SplatModel
    from gsr_amd.parallel import GradAllReducer
    from gsr_amd.pipeline import ViewPipeline
    from gsr_amd.synthetic import make_cameras, make_gaussians, training_targets
    dev = torch.device("cuda", 0)
    cams = [c.to(dev) for c in make_cameras(4, 320, 240, seed=5)]
    gts, monos = training_targets(len(cams), 240, 320, seed=2, device=dev)
    bg = torch.zeros(3, device=dev)
    prev_leaves, prev_det = dgr.grad_into_leaves(), dgr.deterministic()
    dgr.grad_into_leaves(True)
    dgr.deterministic(True)
    runs = []
    try:
        for slices in (1, 4):  # 1: no row slices -> the serial step
            model = SplatModel(make_gaussians(20_001, sh_degree=3, seed=3), device=dev)
            args = trainer.OptArgs()
            trainer.make_trainable(model, args)
            reducer = GradAllReducer(model, bucket_bytes=256 << 10)
            reducer._active = lambda: True  # issue the collectives at world size 1 too
            views = ViewPipeline(dev, depth=2, defer_sh=True, precolor=True, bwd_slices=slices)
            gen = torch.Generator(device=dev).manual_seed(0)
            sliced = []
            for it in (599, 600, 601):  # 600: densification due (interval 100)
                trainer.train_step_views(model, cams, gts, monos, bg, args, it, 2.78, views,
                                         reducer=reducer, generator=gen, multi=True,
                                         next_cams=cams)
                # the next step's colour pre-pass, filled slice by slice behind the optimizer
                prep = views._prepared
                sliced.append((views.rows_done, prep is not None and prep[1].complete))
            torch.cuda.synchronize()
            state = [(p.detach().clone(), model.optimizer.state[p]["exp_avg"].clone(),
                      model.optimizer.state[p]["exp_avg_sq"].clone(),
                      float(model.optimizer.state[p]["step"]))
                     for p in model.parameters()]
            runs.append((state, sliced, model._xyz.shape[0]))
    finally:
        dgr.grad_into_leaves(prev_leaves)
        dgr.deterministic(prev_det)
    (ser, ser_sliced, n0), (got, got_sliced, n1) = runs
    assert ser_sliced == [(False, False)] * 3
    # the densification iteration runs serially (no sliced optimizer, no prepared pre-pass)
    assert got_sliced == [(True, True), (False, False), (True, True)]
    assert n0 == n1
    for (p, m, v, st), (q, m2, v2, st2) in zip(ser, got):
        assert torch.equal(p, q) and torch.equal(m, m2) and torch.equal(v, v2) and st == st2


@pytest.mark.timeout(900)
def test_config4_48_cameras_as_8_shards_world1(tmp_path):
    """BASELINE config 4's workload -- 1M Gaussians, a 48-camera pool at
    1008x756, 6 views per GPU over 8 GPUs with an RCCL gradient all-reduce -- at world size 1:
    the pool as 8 sequential 6-view shards through ViewPipeline.run_views (one multi-view call
    each, the row-sliced backward), RCCL initialised and the collectives forced on.  Deterministic
    backward: every shard's gradients are bitwise the plain single-process shard's (no reducer);
    their sum (what 8 ranks' all-reduce adds up) equals the 48 views rendered in ONE process call
    within 1e-6 of each leaf's largest entry (the summation order of shards vs 8-view backward
    launches differs); sampled views' images and radii match the CPU oracle (radii exact, images
    within 1e-5 away from oracle-marked threshold pixels).  Hardware scaling stays the driver's
    8-GPU SCALE run."""
    import numpy as np

    import diff_gaussian_rasterization as dgr
    from fused_ref import IMAGES, compare, kernel_activations, run_oracle_path
    from gaussian_renderer import render_views
    from gsr_amd.model import SplatModel
    from gsr_amd.parallel import GradAllReducer
    from gsr_amd.pipeline import ViewPipeline
    from gsr_amd.synthetic import make_cameras, make_gaussians, upstream_grads
    from oracle.oracle import set_threads
    dev = torch.device("cuda", 0)
    init = "file://" + os.path.join(str(tmp_path), "pg")
    dist.init_process_group("nccl", init_method=init, rank=0, world_size=1, device_id=dev)
    prev_leaves, prev_det = dgr.grad_into_leaves(), dgr.deterministic()
    dgr.grad_into_leaves(True)
    dgr.deterministic(True)
    try:
        model = SplatModel(make_gaussians(1_000_000, sh_degree=3, seed=0), device=dev)
        cams = [c.to(dev) for c in make_cameras(48, 1008, 756, seed=0)]
        dimg, ddep, dfeat = upstream_grads(756, 1008, seed=1, device=dev)
        bg = torch.zeros(3, device=dev)
        shards = [cams[6 * r:6 * r + 6] for r in range(8)]
        sample = {0: None, 47: None}  # view index -> its images and radii
        views = ViewPipeline(dev, depth=2, defer_sh=True, precolor=True)

        def step(cs, reducer, keep=None):
            def all_views(items, strs):
                pkgs = render_views(items, model, _Pipe(), bg, _Opt(), streams=strs)
                st = pkgs[0]["views"]
                V = len(pkgs)
                torch.autograd.backward([st["render"], st["depth"], st["feature"]],
                                        [g.expand(V, *g.shape) for g in (dimg, ddep, dfeat)])
                if keep is not None:
                    for i, pkg in enumerate(pkgs):
                        k = keep + i
                        if k in sample:
                            sample[k] = {n: pkg[n].detach().cpu().numpy()
                                         for n in IMAGES + ("radii",)}
            if reducer is not None:
                reducer.attach_grads()
            else:
                for p in model.parameters():
                    p.grad = None
            views.run_views(cs, all_views, model=model, reducer=reducer)
            if reducer is not None:
                reducer.wait()
            torch.cuda.synchronize()
            return [p.grad.detach().clone() for p in model.parameters()]

        plain = [step(s, None) for s in shards]
        reducer = GradAllReducer(model)
        reducer._active = lambda: True  # issue the RCCL collectives at world size 1 too
        for r, s in enumerate(shards):
            got = step(s, reducer, keep=6 * r)
            for g, w in zip(got, plain[r]):
                assert torch.equal(g, w), r
        assert dist.get_backend() == "nccl"
        total = [torch.stack([plain[r][k] for r in range(8)]).sum(0) for k in range(len(plain[0]))]
        del plain
        one = step(cams, None)  # the 48 views in one process call
        for t, o in zip(total, one):
            scale = float(o.abs().max())
            assert scale > 0
            assert float((t - o).abs().max()) <= 1e-6 * scale
        # sampled views against the CPU oracle
        n = int(os.environ.get("OMP_NUM_THREADS") or 0) or (os.cpu_count() or 1)
        set_threads(min(n, 32))
        act = kernel_activations(model)
        idx = sorted(sample)
        vo, _ = run_oracle_path(model, [cams[i] for i in idx], (dimg, ddep, dfeat), act)
        vg = [dict(sample[i], means2D=np.zeros((1_000_000, 3), np.float32)) for i in idx]
        st = compare("cfg4_world1", vg, vo, {}, {}, leaves=())
        for i, v in zip(idx, st["views"]):
            assert v["radii_equal"], i
            assert v["pixels_off"] == v["pixels_flipped"], (i, v)
            for k in IMAGES:
                assert v[k + "_unflipped"] <= 1e-5, (i, k, v)
    finally:
        dgr.grad_into_leaves(prev_leaves)
        dgr.deterministic(prev_det)
        dist.destroy_process_group()
