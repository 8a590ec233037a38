"""Micro-benchmark of the densification row at P Gaussians, SH degree 3,
language features on, Adam state present -- gsr_amd.densify vs the restatement of the reference
(tests/densify_ref.py: boolean-mask indexing + torch.cat, scene/gaussian_model.py:400-612).

  stats:  train.py:219-220 per training step (max_radii2D + add_densification_stats)
  dnp:    densify_and_prune at iteration 3000 (clone + split + prune; no proximity), whole call
  compact: the gsr_compact_rows launch inside dnp alone, with its algorithmic bytes
           (surviving old rows read once from every source array, appendix rows read, every
           output row written) -> GB/s against the 8 TB/s HBM peak

Prints one JSON line.  usage: python scripts/densify_bench.py [--P 1000000] [--reps 20]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sdp-gs_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

from densify_ref import RefDensify  # noqa: E402
from gsr_amd import densify  # noqa: E402
from test_densify import EXTENT, MIN_OP, THR, _model  # noqa: E402

HBM_PEAK = 8.0e12


def _time(fn, reps, setup=None):
    ts = []
    for _ in range(reps):
        if setup:
            setup()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return 1e3 * ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--P", type=int, default=1_000_000)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    P = a.P
    base = _model(P, seed=3)
    gen = torch.Generator(device="cuda").manual_seed(1)
    radii = torch.randint(0, 30, (P,), generator=gen, device="cuda", dtype=torch.int32)
    vs = torch.zeros((P, 3), device="cuda", requires_grad=True)
    vs.grad = torch.randn((P, 3), generator=gen, device="cuda") * 1e-3
    vis = radii > 0

    # ---- per-step statistics
    ref = RefDensify(base)
    t_stats_ref = _time(lambda: ref.update_stats(vs.grad, radii, vis), 5 * a.reps)
    t_stats = _time(lambda: base.update_densification_stats(vs, radii, vis), 5 * a.reps)

    # ---- densify_and_prune on fresh copies
    holder = {}

    def mk_ours():
        holder["m"] = _model(P, seed=3)
        torch.manual_seed(0)

    def mk_ref():
        holder["r"] = RefDensify(_model(P, seed=3))
        torch.manual_seed(0)

    reps = max(3, a.reps // 4)
    t_dnp = _time(lambda: holder["m"].densify_and_prune(THR, MIN_OP, EXTENT, None, 3000), reps,
                  mk_ours)
    t_dnp_ref = _time(lambda: holder["r"].densify_and_prune(THR, MIN_OP, EXTENT, None, 3000),
                      reps, mk_ref)
    n_after = holder["m"]._xyz.shape[0]

    # ---- the compaction launch alone (same arrays / index as dnp's final rebuild)
    m = _model(P, seed=3)
    torch.manual_seed(0)
    captured = {}
    orig = densify.compact_rows

    def spy(arrays, n_old, index, n_out):
        captured.update(arrays=arrays, n_old=n_old, index=index, n_out=n_out)
        return orig(arrays, n_old, index, n_out)

    densify.compact_rows = spy
    try:
        m.densify_and_prune(THR, MIN_OP, EXTENT, None, 3000)
    finally:
        densify.compact_rows = orig
    c = captured
    idx = c["index"][:c["n_out"]].long()
    n_old_kept = int((idx < c["n_old"]).sum())
    n_new_kept = c["n_out"] - n_old_kept
    alg = 0
    for src, ext, _, dst in c["arrays"]:
        rb = dst.element_size() * (dst.numel() // c["n_out"])
        alg += rb * c["n_out"]                                     # write
        alg += rb * (n_old_kept if src is not None else 0)         # old rows read
        alg += rb * (n_new_kept if ext is not None else 0)         # appendix rows read
    alg += 4 * c["n_out"]                                          # index
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        orig(c["arrays"], c["n_old"], c["index"], c["n_out"])
    ev0.record()
    for _ in range(a.reps):
        orig(c["arrays"], c["n_old"], c["index"], c["n_out"])
    ev1.record()
    torch.cuda.synchronize()
    t_compact = ev0.elapsed_time(ev1) / a.reps
    gbs = alg / (t_compact * 1e-3) / 1e9
    print(json.dumps({
        "bench": "densify", "P": P, "P_after": n_after, "arrays": len(c["arrays"]),
        "stats_ms": round(t_stats, 4), "stats_ref_ms": round(t_stats_ref, 4),
        "stats_speedup": round(t_stats_ref / t_stats, 2),
        "densify_and_prune_ms": round(t_dnp, 3), "densify_and_prune_ref_ms": round(t_dnp_ref, 3),
        "densify_and_prune_speedup": round(t_dnp_ref / t_dnp, 2),
        "compact_ms": round(t_compact, 4), "compact_bytes": alg,
        "compact_GBps": round(gbs, 1), "compact_frac_hbm": round(gbs * 1e9 / HBM_PEAK, 3)}))


if __name__ == "__main__":
    main()
