"""Densification on libgsr (gsr_amd.densify, include/gsr_densify.h) against the restatement of the
reference's adaptive density control (tests/densify_ref.py <- scene/gaussian_model.py:400-612,
train.py:218-220).  Integer / byte work and row moves are bit-exact; the only float arithmetic in
the kernels (the statistics' sqrt(gx^2 + gy^2), exp / sigmoid of the classify tests) is checked
exactly too, including inputs placed ON the thresholds."""
import numpy as np
import pytest
import torch

from densify_ref import RefDensify, model_arrays

from gsr_amd import densify
from gsr_amd.model import SplatModel
from gsr_amd.synthetic import make_gaussians


class TA:
    """OptimizationParams fields training_setup reads (arguments/__init__.py:75-98)."""
    percent_dense = 0.01
    position_lr_init = 0.016
    feature_lr = 0.0025
    opacity_lr = 0.05
    scaling_lr = 0.003
    rotation_lr = 0.001
    language_feature_lr = 0.013

    def __init__(self, include_feature=True):
        self.include_feature = include_feature


THR = 0.0013       # densify_grad_threshold (arguments/__init__.py:94)
EXTENT = 2.78      # percent_dense * extent ~ the median max scale of make_gaussians
MIN_OP = 0.18      # ~10 % of make_gaussians' opacities below


def _model(P, seed=0, include_feature=True, state=True, big_rows=0):
    m = SplatModel(make_gaussians(P, seed=seed), device="cuda")
    m.training_setup(TA(include_feature))
    gen = torch.Generator(device="cuda").manual_seed(seed + 1)
    with torch.no_grad():
        if big_rows:
            m._scaling[:big_rows] = np.log(0.5)
    m.denom = torch.randint(0, 4, (P, 1), generator=gen, device="cuda").float()
    m.xyz_gradient_accum = torch.rand((P, 1), generator=gen, device="cuda") * 2 * THR * m.denom
    m.max_radii2D = torch.randint(0, 60, (P,), generator=gen, device="cuda").float()
    m.confidence = torch.rand((P, 1), generator=gen, device="cuda")
    if state:
        for g in m.optimizer.param_groups:
            p = g["params"][0]
            m.optimizer.state[p] = {
                "step": torch.tensor(7.0),
                "exp_avg": torch.randn(p.shape, generator=gen, device="cuda"),
                "exp_avg_sq": torch.rand(p.shape, generator=gen, device="cuda")}
    return m


def _assert_same(m, ref):
    a, b = model_arrays(m), ref.arrays()
    assert list(a) == list(b)
    for k in a:
        assert a[k].shape == b[k].shape, k
        assert torch.equal(a[k], b[k]), k


# ---- host-side checks (no GPU) -------------------------------------------------------------------
def test_no_cpu_path():
    t = torch.zeros(8, dtype=torch.uint8)
    with pytest.raises(RuntimeError, match="HIP"):
        densify.select_rows(t, 1, 0)


def test_install_exposes_reference_method_names():
    for name in ("add_densification_stats", "prune_points", "densification_postfix",
                 "densify_and_clone", "densify_and_split", "densify_and_prune", "proximity"):
        assert getattr(SplatModel, name) is getattr(densify, name)


# ---- GPU parity ------------------------------------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("n", [0, 1, 15, 4095, 4096, 4097, 1_000_003])
def test_select_rows_matches_nonzero(n):
    gen = torch.Generator(device="cuda").manual_seed(n)
    flags = torch.randint(0, 16, (n + 1,), generator=gen, device="cuda", dtype=torch.uint8)
    for f in (flags[:n], flags[1:]):  # 16-B aligned and misaligned starts
        for mask, want in ((1, 1), (6, 0), (0, 0), (15, 9)):
            idx, cnt = densify.select_rows(f, mask, want)
            exp = torch.nonzero((f & mask) == want).flatten()
            assert int(cnt.item()) == exp.numel()
            assert torch.equal(idx[:exp.numel()].long(), exp)


@pytest.mark.gpu
def test_compact_rows_gather_fill_extra():
    gen = torch.Generator(device="cuda").manual_seed(3)
    n_old, n_ext = 10_000, 777
    widths = [1, 3, 4, 45, 2]
    src = [torch.randn((n_old, w), generator=gen, device="cuda") for w in widths]
    ext = [torch.randn((n_ext, w), generator=gen, device="cuda") for w in widths]
    keep = torch.rand(n_old + n_ext, generator=gen, device="cuda") > 0.3
    index = torch.nonzero(keep).flatten().to(torch.int32)
    n_out = index.numel()
    dst = [torch.empty((n_out, w), device="cuda") for w in widths]
    arrays = [(src[0], ext[0], 0, dst[0]),            # both parts
              (src[1], None, 0x3F800000, dst[1]),      # extra rows -> 1.0
              (None, ext[2], 0, dst[2]),               # old rows -> 0
              (src[3], ext[3], 0, dst[3]),             # wide rows (features_rest)
              (None, None, 0, dst[4])]                 # all zero
    densify.compact_rows(arrays, n_old, index, n_out)
    li = index.long()
    for w, s, e, (a_src, a_ext, fill, d) in zip(widths, src, ext, arrays):
        full_s = s if a_src is not None else torch.full_like(s, float(np.frombuffer(
            np.uint32(fill).tobytes(), np.float32)[0]))
        full_e = e if a_ext is not None else torch.full_like(e, float(np.frombuffer(
            np.uint32(fill).tobytes(), np.float32)[0]))
        assert torch.equal(d, torch.cat((full_s, full_e))[li]), w
    # identity index, more arrays than one launch takes
    many = [(src[1], ext[1], 0, torch.empty((n_old + n_ext, 3), device="cuda"))
            for _ in range(densify.MAX_ARRAYS + 3)]
    densify.compact_rows(many, n_old, None, n_old + n_ext)
    for a in many:
        assert torch.equal(a[3], torch.cat((src[1], ext[1])))


@pytest.mark.gpu
def test_stats_match_reference():
    P = 200_003
    m = _model(P)
    ref = RefDensify(m)
    gen = torch.Generator(device="cuda").manual_seed(9)
    for step in range(5):
        radii = torch.randint(-2, 30, (P,), generator=gen, device="cuda", dtype=torch.int32)
        radii.clamp_(min=0)
        vs = torch.zeros((P, 3), device="cuda", requires_grad=True)
        vs.grad = torch.randn((P, 3), generator=gen, device="cuda") * 1e-3
        vs.grad[:, 2] = 0
        vis = radii > 0
        if step % 2:
            m.update_densification_stats(vs, radii, vis)
        else:
            m.update_densification_stats(vs, radii)  # filter derived from radii > 0
        ref.update_stats(vs.grad, radii, vis)
        f2 = torch.rand(P, generator=gen, device="cuda") > 0.5
        m.add_densification_stats(vs, f2)
        ref.add_stats(vs.grad, f2)
    assert torch.equal(m.max_radii2D, ref.max_radii2D)
    assert torch.equal(m.denom, ref.denom)
    # sqrt(x*x + y*y) vs torch.norm's reduction: allow an ulp per step
    torch.testing.assert_close(m.xyz_gradient_accum, ref.xyz_gradient_accum, rtol=1e-6, atol=0)
    exact = (m.xyz_gradient_accum == ref.xyz_gradient_accum).float().mean().item()
    print(f"stats accum bit-exact fraction {exact:.6f}")


@pytest.mark.gpu
def test_classify_exact_on_thresholds():
    """Thresholds taken from the data itself: rows sitting exactly on a threshold expose any ulp of
    difference between the kernel's expf / sigmoid / division and torch's."""
    P = 300_000
    m = _model(P, seed=4, big_rows=100)
    g = (m.xyz_gradient_accum / m.denom).reshape(-1)
    g[g.isnan()] = 0.0
    smax = torch.exp(m._scaling.detach()).max(dim=1).values
    op = torch.sigmoid(m._opacity.detach()).reshape(-1)
    rows = [5, 77, 1234, 99_999]
    for k in rows:
        thr, lim, mo, big = g[k].item(), smax[k].item(), op[k].item(), smax[k + 1].item()
        flags, cidx, sidx = densify.classify(m, m.xyz_gradient_accum.reshape(-1),
                                             m.denom.reshape(-1), thr, lim, mo, big)
        nc, ns = cidx.numel(), sidx.numel()
        assert torch.equal(cidx, torch.nonzero(flags & densify.CLONE).flatten())
        # the C-ABI's optional counters (one atomic per workgroup)
        from gsr_amd import _lib
        counts = torch.full((2,), 7, dtype=torch.int32, device="cuda")
        flags2 = torch.empty_like(flags)
        assert _lib.load().gsr_densify_classify(
            P, m.xyz_gradient_accum.data_ptr(), m.denom.data_ptr(), m._scaling.data_ptr(),
            m._opacity.data_ptr(), thr, lim, mo, 1, big, flags2.data_ptr(), counts.data_ptr(),
            torch.cuda.current_stream().cuda_stream) == 0
        assert torch.equal(flags, flags2) and counts.tolist() == [nc, ns]
        t32 = lambda x: torch.tensor(x, dtype=torch.float32, device="cuda")  # noqa: E731
        clone = (torch.norm(g[:, None], dim=-1) >= t32(thr)) & (smax <= t32(lim))
        split = (g >= t32(thr)) & (smax > t32(lim))
        low = op < t32(mo)
        bigw = smax > t32(big)
        exp = (clone.to(torch.uint8) * densify.CLONE | split.to(torch.uint8) * densify.SPLIT
               | low.to(torch.uint8) * densify.LOW_OPACITY | bigw.to(torch.uint8) * densify.BIG_WS)
        bad = torch.nonzero(flags != exp).flatten()
        assert bad.numel() == 0, (k, bad[:8].tolist(), flags[bad[:8]].tolist(),
                                  exp[bad[:8]].tolist())
        assert nc == int(clone.sum()) and ns == int(split.sum())


def _pair(P, **kw):
    m = _model(P, **kw)
    return m, RefDensify(m)


@pytest.mark.gpu
@pytest.mark.parametrize("iteration", [300, 3000])
def test_prune_points_matches_reference(iteration):
    m, ref = _pair(50_001)
    mask = torch.rand(50_001, device="cuda") > 0.6
    m.prune_points(mask, iteration, True)
    ref.prune_points(mask, iteration)
    _assert_same(m, ref)


@pytest.mark.gpu
def test_postfix_clone_split_match_reference():
    m, ref = _pair(40_000)
    grads = (m.xyz_gradient_accum / m.denom)
    grads[grads.isnan()] = 0.0
    m.densify_and_clone(grads, THR, EXTENT, True)
    ref.clone(grads.clone(), THR, EXTENT)
    _assert_same(m, ref)
    torch.manual_seed(11)
    m.densify_and_split(grads, THR, EXTENT, 3000, True)
    torch.manual_seed(11)
    ref.split(grads.clone(), THR, EXTENT, 3000)
    _assert_same(m, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("include_feature", [True, False])
@pytest.mark.parametrize("iteration,max_screen", [(3000, None), (3000, 20), (2500, None)])
def test_densify_and_prune_matches_reference(include_feature, iteration, max_screen):
    P = 120_007
    m, ref = _pair(P, seed=2, include_feature=include_feature, big_rows=64)
    if iteration == 2500:
        m.args.prune_from_iter = ref.args.prune_from_iter = 2600  # prune inactive
    torch.manual_seed(5)
    m.densify_and_prune(THR, MIN_OP, EXTENT, max_screen, iteration, include_feature)
    torch.manual_seed(5)
    ref.densify_and_prune(THR, MIN_OP, EXTENT, max_screen, iteration)
    _assert_same(m, ref)
    assert m._xyz.shape[0] != P  # something was cloned / split / pruned


@pytest.mark.gpu
@pytest.mark.parametrize("include_feature", [True, False])
def test_densify_and_prune_with_proximity_matches_reference(include_feature):
    """iteration < 2000: clone + split, then proximity densification (3-NN: gsr_dist_knn3 here,
    the CPU oracle's distCUDA2 in the restatement), then the prune."""
    P = 20_000
    m, ref = _pair(P, seed=6, include_feature=include_feature)
    extent = 1e-4  # proximity picks points whose mean squared 3-NN distance exceeds 5e-4
    torch.manual_seed(8)
    m.densify_and_prune(THR, MIN_OP, extent, None, 1500, include_feature)
    torch.manual_seed(8)
    ref.densify_and_prune(THR, MIN_OP, extent, None, 1500)
    _assert_same(m, ref)


@pytest.mark.gpu
def test_densify_edge_cases():
    # nothing selected, nothing pruned
    m, ref = _pair(4096, state=False)
    m.densify_and_prune(1e9, 0.0, EXTENT, None, 3000)
    ref.densify_and_prune(1e9, 0.0, EXTENT, None, 3000)
    _assert_same(m, ref)
    # everything pruned
    m, ref = _pair(5000)
    torch.manual_seed(1)
    m.densify_and_prune(THR, 2.0, EXTENT, None, 3000)
    torch.manual_seed(1)
    ref.densify_and_prune(THR, 2.0, EXTENT, None, 3000)
    _assert_same(m, ref)
    assert m._xyz.shape[0] == 0


@pytest.mark.gpu
def test_optimizer_steps_after_densify():
    """FusedAdam keeps stepping the rebuilt parameters (state keyed by the new nn.Parameters)."""
    m = _model(30_000)
    torch.manual_seed(0)
    m.densify_and_prune(THR, MIN_OP, EXTENT, None, 3000)
    for p in m.parameters():
        p.grad = torch.ones_like(p)
    before = m._xyz.detach().clone()
    m.optimizer.step()
    assert not torch.equal(before, m._xyz.detach())
    for g in m.optimizer.param_groups:
        assert float(m.optimizer.state[g["params"][0]]["step"]) == 8.0


def _dp_worker(rank, world, init, q):
    import torch.distributed as dist
    from gsr_amd.parallel import allreduce_densification_stats
    dist.init_process_group("gloo", init_method=init, rank=rank, world_size=world)
    m = _model(30_000, seed=12)                 # same replica on every rank
    gen = torch.Generator(device="cuda").manual_seed(100 + rank)
    vs = torch.zeros((30_000, 3), device="cuda", requires_grad=True)
    for _ in range(3):                           # each rank sees its own views
        radii = torch.randint(0, 20, (30_000,), generator=gen, device="cuda", dtype=torch.int32)
        vs.grad = torch.randn((30_000, 3), generator=gen, device="cuda") * 2e-3
        m.update_densification_stats(vs, radii)
    allreduce_densification_stats(m.xyz_gradient_accum, m.denom, m.max_radii2D)
    # numpy: pickled by value (torch CPU tensors would go through fds of an exiting process)
    stats = [t.cpu().numpy() for t in (m.xyz_gradient_accum, m.denom, m.max_radii2D)]
    g = torch.Generator(device="cuda").manual_seed(7)
    m.densify_and_prune(THR, MIN_OP, EXTENT, None, 3000, True, generator=g)
    q.put((rank, stats, {k: v.cpu().numpy() for k, v in model_arrays(m).items()}))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
def test_densify_data_parallel_replicas_stay_identical():
    """Two ranks (gloo, both on cuda:0): statistics all-reduced (SUM / SUM / MAX), then
    densify_and_prune with an identically seeded generator -> bit-identical replicas, equal to the
    reference restatement run once on the reduced statistics."""
    import torch.multiprocessing as mp
    from test_parallel import _init_method
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    init = _init_method()
    procs = [ctx.Process(target=_dp_worker, args=(r, 2, init, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in procs], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, s0, a0), (_, s1, a1) = res
    assert list(a0) == list(a1)
    for k in a0:
        assert np.array_equal(a0[k], a1[k]), k
    m = _model(30_000, seed=12)
    m.xyz_gradient_accum, m.denom, m.max_radii2D = [torch.from_numpy(t).cuda() for t in s0]
    ref = RefDensify(m)
    # the restatement draws torch.normal from the default generator: seed it like the ranks'
    torch.cuda.manual_seed(7)
    ref.densify_and_prune(THR, MIN_OP, EXTENT, None, 3000)
    b = ref.arrays()
    for k in a0:
        assert np.array_equal(a0[k], b[k].cpu().numpy()), k


@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_densify_and_prune_5m_config5():
    """BASELINE config 5: densify_and_prune on a 5M-row model at iteration
    2500 (clone + split + prune, past the proximity window; gaussian_model.py:591-608), the
    gradient threshold at the statistics' 90th percentile as bench.py's training leg sets it, so
    ~10 % of the rows clone or split: parameters, statistics and Adam state bit-exact against the
    restatement of the reference."""
    P = 5_000_000
    m, ref = _pair(P, seed=21, big_rows=64)
    g = (m.xyz_gradient_accum / m.denom).nan_to_num(0.0).reshape(-1)
    thr = float(torch.quantile(g[g > 0][: 1 << 24], 0.9))
    torch.manual_seed(5)
    m.densify_and_prune(thr, MIN_OP, EXTENT, None, 2500, True)
    torch.manual_seed(5)
    ref.densify_and_prune(thr, MIN_OP, EXTENT, None, 2500)
    _assert_same(m, ref)
    n = m._xyz.shape[0]
    assert n != P and n > 0.5 * P, n
