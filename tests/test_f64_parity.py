"""Per-entry gradient parity against a float64 evaluation.

The benchmarked path (tests/fused_ref.py run_bench_path: render() with the reference's default
flags through the fused multi-view call) is compared entry by entry with the float64 build of the
oracle (tests/f64_ref.py): every raw-leaf gradient entry at >= 1 % of its tensor's maximum must
satisfy

    |gpu - f64| <= C u B        u = 2^-24, C = 1 (no relative floor, since round 6)

where B is the entry's float32 rounding scale: the sum over its per-pixel terms of |term| times
the length of the float32 chain that term went through (T's recovery over the pixel's list),
propagated through the per-Gaussian backward with |J| (f64_ref.py explains it).

Decision-locked: the float64 evaluation blends the float32 oracle's instance
lists AND its per-pixel decisions (n_contrib and which list positions passed alpha >= 1/255 /
power <= 0, OracleRaster.accept_bits), the per-Gaussian SH colour clamp decisions that mask
dL/dRGB (OracleRaster.clamped) and the projected splats the blend evaluates (screen means, conic +
opacity: their float32 rounding, up to 6e-5 px at x ~ 1500, moves G by ~1e-4 relative at a
splat's edge at 1920x1080 -- a preprocess effect the blend's rounding scale B does not model), so
it sums exactly the terms float32 summed and no pixel is excluded for a float32-vs-float64
threshold flip.  What is still left out of the entry-wise
statistics, counted separately and capped at max(50, 1e-4 P) together: Gaussians behind a
GPU-vs-float32 image flip (the Gaussians that can reach the flipped pixels,
fused_ref.pixel_contributors) and Gaussians whose visibility (radius > 0)
differs between float32 and float64 (the per-Gaussian backward's gate).  The float32
oracle -- the reference's own arithmetic, restated -- is held to the same bound (it is the
calibration: its worst ratio |f32 - f64| / (u B) is <= 0.14 at these sizes, the GPU's <= 0.34 in
round 5, profiles/r05_f64_stats.jsonl; since round 6 C = 1 and the 1e-5
relative floor is gone -- every entry is held to its rounding scale alone), so passing says
the GPU is as accurate as the reference's float32 arithmetic, entry by entry.  Negative controls
show the bound catches a 1e-5 systematic error in the colour terms and a 1e-5 error in the conic
the blend evaluates (f64_ref.controls_1e5).  The preprocess's own float32 outputs are checked
entry by entry, unlocked, in tests/test_pre_f64_parity.py.  The scale-relative 1e-5 check stays in
tests/test_fused_parity.py.  Statistics: gpurun_out/f64_stats.jsonl.

VERDICT r3 also proposed |gpu - f64| <= max(2 |f32 - f64|, 1e-5 |f64|); it is reported
(`gpu_within_2x_f32`) but not asserted: two float32 evaluations with different (equally valid)
arithmetic have independent rounding, and the 2x test fails a sizeable fraction of entries for
independent errors of equal size.
"""
import json
import os

import numpy as np
import pytest
import torch

from f64_ref import controls_1e5, oracle_inputs, rounding_stats, run_f64_path
from fused_ref import LEAVES, flipped_pixels, pixel_contributors, kernel_activations, \
    run_bench_path, run_oracle_path
from gsr_amd.model import SplatModel
from gsr_amd.synthetic import make_cameras, make_gaussians, upstream_grads
from oracle.oracle import set_threads

pytestmark = pytest.mark.gpu

C_BOUND = 1.0
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STATS = os.path.join(ROOT, "gpurun_out", "f64_stats.jsonl")

CASES = {
    "small_6views_multi": dict(P=20_000, W=200, H=150, views=6, streams=3, seed=8, deg=3),
    "cfg2_100k_800x800_multi": dict(P=100_000, W=800, H=800, views=3, streams=3, seed=0, deg=3),
    "cfg3_1m_1008x756_multi": dict(P=1_000_000, W=1008, H=756, views=3, streams=3, seed=0, deg=3),
    "cfg5_5m_1920x1080_multi": dict(P=5_000_000, W=1920, H=1080, views=2, streams=2, seed=0,
                                    deg=3),
}


def _threads():
    n = int(os.environ.get("OMP_NUM_THREADS") or 0) or (os.cpu_count() or 1)
    return set_threads(min(n, 32))


@pytest.mark.timeout(1500)
@pytest.mark.parametrize("case", list(CASES))
def test_gradients_within_float32_rounding_of_f64(case):
    c = CASES[case]
    _threads()
    m = SplatModel(make_gaussians(c["P"], sh_degree=3, seed=c["seed"]), device="cuda",
                   active_sh_degree=c["deg"])
    cams = [x.to("cuda") for x in make_cameras(c["views"], c["W"], c["H"], seed=c["seed"])]
    grads = upstream_grads(c["H"], c["W"], seed=1, device="cuda")
    act = kernel_activations(m)
    vg, gg = run_bench_path(m, cams, grads, streams=c["streams"], multi=True)
    print(f"[{case}] GPU path done", flush=True)
    vo, go = run_oracle_path(m, cams, grads, act)
    print(f"[{case}] f32 oracle done", flush=True)
    inp = oracle_inputs(m, act)
    del m
    # f64 blends the f32 binning's lists with the f32 blend's per-pixel decisions
    lists = [(v["point_list"], v["ranges"]) for v in vo]
    decisions = [v.pop("decisions") for v in vo]
    clamps = [v.pop("clamped") for v in vo]  # the SH colour clamp decisions, locked too
    geometry = [(v["xy"], v["conic_opacity"]) for v in vo]  # and the projected splats
    v64, g64, B = run_f64_path(inp, cams, grads, lists=lists, decisions=decisions, clamps=clamps,
                               geometry=geometry,
                               progress=lambda s: print(f"[{case}] {s}", flush=True))
    P = vo[0]["radii"].shape[0]
    hit_gpu = np.zeros(P, bool)
    hit_vis = np.zeros(P, bool)
    nflip64 = pix_gpu = 0
    for a, b, d in zip(vg, vo, v64):
        off, _ = flipped_pixels(a, b)  # GPU vs f32: images off by > 1e-5 (test_fused_parity)
        pix_gpu += int(off.sum())
        hit_gpu |= pixel_contributors(b, off, P)  # (rare) the Gaussians reaching them
        # f32 vs f64 under the lock: the same decisions by construction (checked here)
        nflip64 += int((d["n_contrib"] != b["n_contrib"]).sum())
        hit_vis |= (d["radii"] > 0) != (b["radii"] > 0)  # visibility decided the other way
        assert np.array_equal(a["radii"], b["radii"]), case
    hit = hit_gpu | hit_vis
    rec = {"case": case, "gaussians_excluded": int(hit.sum()),
           "excluded_gpu_vs_f32": int(hit_gpu.sum()), "gpu_vs_f32_pixels": pix_gpu,
           "excluded_visibility_f32_vs_f64": int(hit_vis.sum()),
           "f64_decision_flips": nflip64, "decision_locked": True, "C": C_BOUND, "grads": {}}
    for n in LEAVES:
        st = rounding_stats(gg[n], go[n], g64[n], B[n], exclude=hit, C=C_BOUND, rel=0.0)
        rec["grads"][n] = st
    os.makedirs(os.path.dirname(STATS), exist_ok=True)
    with open(STATS, "a") as fh:
        fh.write(json.dumps(rec) + "\n")
    # the lock leaves no float32-vs-float64 decision flip; the entry-wise statistics cover every
    # Gaussian but the few behind a GPU-vs-float32 flip or a visibility flip
    assert nflip64 == 0, nflip64
    assert rec["gaussians_excluded"] <= max(50, 1e-4 * P), rec
    for n in LEAVES:
        st = rec["grads"][n]
        # calibration: the reference's float32 arithmetic meets the bound ...
        assert st["f32_fail"] == 0, (case, n, st)
        # ... and so does every GPU entry
        assert st["gpu_fail"] == 0, (case, n, st)

    # negative controls: a 1e-5 error in the colour terms, and a 1e-5 error
    # in the conic the float64 blend evaluates, each caught on >= 1 % of some leaf's entries at
    # the small scene.  Recorded, not asserted, at config 2: there every entry sums hundreds of
    # per-pixel terms, so its worst-case float32 rounding scale u B exceeds 1e-5 of its value
    # for >= 99.9 % of the SH-coefficient entries (measured: a 1e-5 colour error then stands out
    # of that bound on 0.1 % of them) -- no rigorous rounding bound can tell a 1e-5 systematic
    # error from float32 rounding at that depth; the GPU's actual errors stay <= 0.07 u B.
    # (The two extra float64 evaluations run at the small and config-2 sizes only.)
    if c["P"] > 100_000:
        return
    ctl = controls_1e5(inp, cams, grads, geometry, dict(lists=lists, decisions=decisions,
                                                         clamps=clamps))
    rec["controls"] = {}
    for name, g64c in ctl.items():
        fr = {}
        for n in LEAVES:
            st = rounding_stats(gg[n], go[n], g64c[n], B[n], exclude=hit, C=C_BOUND, rel=0.0)
            fr[n] = st["gpu_fail"] / max(1, st["n_big"])
        rec["controls"][name] = fr
        if case == "small_6views_multi":
            assert max(fr.values()) >= 0.01, (case, name, fr)
    with open(STATS.replace(".jsonl", "_controls.jsonl"), "a") as fh:
        fh.write(json.dumps({"case": case, "controls": rec["controls"]}) + "\n")
