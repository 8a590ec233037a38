"""The forward preprocess's float32 outputs entry by entry against float64.

The decision-locked gradient check (tests/test_f64_parity.py) hands the float64 blend the float32
run's projected splats, so the preprocess's own rounding is compared here, unlocked: the GPU's
splat records of the benchmarked path (render_views through ViewPipeline.run_views, the multi-view
preprocess with the colour pre-pass; read back by gsr_test_splat_records) against the float64
oracle's preprocess (preprocess_one, forward.cu:155-256) of the same views.  Per output entry --
screen position, conic, opacity, depth, RGB, language feature -- of every Gaussian visible in both:

    |gpu - f64| <= C u B        u = 2^-24, C = 1 (no relative floor)

with B the first-order float32 rounding bound of that entry's own chain of float operations
(tests/pre_bound.py: the oracle's expressions, in its order, with |error| propagated through each
operation -- a worst case, every rounding aligned).  The float32 oracle is held to the same bound
(calibration; its worst ratio is ~1, reached by depth = a dot product whose last rounding is the
whole error), and a 1e-5 relative error injected into the float64 conic and colour is caught on
most entries.  The GPU's records are also bitwise the float32 oracle's (asserted: the multi-view
preprocess evaluates the reference's float32 expressions in the reference's order).  The tracker's float64 values equal the float64 oracle's exactly on every column the
oracle evaluates in double (checked: it follows the same expressions).  Radii are exact
(test_fused_parity).  Statistics: gpurun_out/pre_f64_stats.jsonl.
"""
import json
import os

import numpy as np
import pytest

from f64_ref import _raster, oracle_inputs
from fused_ref import kernel_activations, run_bench_path, splat_records
from gsr_amd.model import SplatModel
from gsr_amd.synthetic import make_cameras, make_gaussians, upstream_grads
from oracle.oracle import set_threads
from pre_bound import COLUMNS, bound_stats, camera_args, preprocess_bound

pytestmark = pytest.mark.gpu

C_PRE = 1.0
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STATS = os.path.join(ROOT, "gpurun_out", "pre_f64_stats.jsonl")

CASES = {
    "small_3views": dict(P=20_000, W=200, H=150, views=3, seed=8),
    "cfg2_100k_800x800": dict(P=100_000, W=800, H=800, views=2, seed=0),
    "cfg3_1m_1008x756": dict(P=1_000_000, W=1008, H=756, views=2, seed=0),
    "cfg5_5m_1920x1080": dict(P=5_000_000, W=1920, H=1080, views=1, seed=0),
}
F64_COLS = list(range(10))   # x .. b: evaluated in double by the float64 oracle
FEAT_COLS = [10, 11, 12]     # its language feature starts from float products (SH_C0 * l)


@pytest.mark.timeout(900)
@pytest.mark.parametrize("case", list(CASES))
def test_preprocess_within_float32_rounding_of_f64(case):
    c = CASES[case]
    n = int(os.environ.get("OMP_NUM_THREADS") or 0) or (os.cpu_count() or 1)
    set_threads(min(n, 32))
    m = SplatModel(make_gaussians(c["P"], sh_degree=3, seed=c["seed"]), device="cuda")
    cams = [x.to("cuda") for x in make_cameras(c["views"], c["W"], c["H"], seed=c["seed"])]
    grads = upstream_grads(c["H"], c["W"], seed=1, device="cuda")
    act = kernel_activations(m)
    recs = []
    vg, _ = run_bench_path(m, cams, grads, streams=2, multi=True,
                           capture=lambda pkgs: recs.extend(splat_records(pkgs)))
    inp = oracle_inputs(m, act)
    del m
    rec = {"case": case, "C": C_PRE, "views": []}
    fails = []
    for v, cam in enumerate(cams):
        o32, o64 = _raster(inp, cam, "f32"), _raster(inp, cam, "f64")
        a32, a64 = o32.preprocess_f64(), o64.preprocess_f64()
        val, B = preprocess_bound(inp["xyz"], inp["sc"], inp["rot"], inp["op"], inp["shs"],
                                  inp["deg"], inp["lang"], **camera_args(cam))
        assert np.array_equal(vg[v]["radii"], o32.radii), (case, v)
        rows = (o32.radii > 0) & (o64.radii > 0)
        # the tracker follows the float64 oracle's expressions exactly
        assert np.array_equal(val[rows][:, F64_COLS], a64[rows][:, F64_COLS]), (case, v)
        ref = a64.copy()
        ref[:, FEAT_COLS] = val[:, FEAT_COLS]
        gpu = recs[v][:, :13]
        st_gpu = bound_stats(gpu, ref, B, rows, C_PRE, rel=0.0)
        st_f32 = bound_stats(a32, ref, B, rows, C_PRE, rel=0.0)
        vis = rows.sum()
        eq = {k: float(np.mean(gpu[rows, i] == a32[rows, i].astype(np.float32)))
              for i, k in enumerate(COLUMNS)}
        # negative controls: 1e-5 relative in the float64 conic / colour
        ctl = ref.copy()
        ctl[:, 2:5] *= 1.0 + 1e-5
        ctl[:, 7:10] *= 1.0 + 1e-5
        st_ctl = bound_stats(gpu, ctl, B, rows, C_PRE, rel=0.0)
        rec["views"].append({"visible": int(vis),
                             "visible_f32_vs_f64_differ": int(((o32.radii > 0) != (o64.radii > 0)).sum()),
                             "gpu": st_gpu, "f32": st_f32, "gpu_bitwise_eq_f32": eq,
                             "control_fail_frac": {k: st_ctl[k]["fail"] / max(1, vis)
                                                   for k in ("conic_a", "conic_c", "r", "g", "b")}})
        # the multi-view preprocess follows the reference's float32 expressions in its order:
        # bit for bit the float32 restatement's outputs (measured: every visible entry, every
        # config), which the rounding bound above then covers entry by entry
        for k, f in eq.items():
            if f != 1.0:
                fails.append(("gpu != f32 oracle", v, k, f))
        for k in COLUMNS:
            if st_f32[k].get("fail"):
                fails.append(("f32", v, k, st_f32[k]))
            if st_gpu[k].get("fail"):
                fails.append(("gpu", v, k, st_gpu[k]))
        for k in ("conic_a", "conic_c", "r", "g", "b"):
            assert st_ctl[k]["fail"] >= 0.5 * vis, (case, v, k, st_ctl[k])
        del o32, o64
    os.makedirs(os.path.dirname(STATS), exist_ok=True)
    with open(STATS, "a") as fh:
        fh.write(json.dumps(rec) + "\n")
    assert not fails, fails
