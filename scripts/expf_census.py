"""Threshold census: how far do the blend's decisions drift when G = exp(power)
is evaluated by libm's expf (what a CUDA build's expf stands for) instead of splat_exp, the
deterministic exp the HIP kernels and the checker share?

For each view of BASELINE configs 3 (1M Gaussians, 1008x756) and 5 (5M, 1920x1080) the CPU oracle
runs the forward twice (oracle/Makefile: libgsr_oracle.so and libgsr_oracle_expf.so, same source)
and counts the pixels whose alpha >= 1/255 or T < 1e-4 decision differs: their n_contrib differs or
their final T differs by more than rounding (a flipped 1/255 splat moves T by ~0.4 %).  Also the
max image difference over all pixels and over the pixels without a flip, and the float64 build's
flips against splat_exp for comparison.  Output: one JSON document (profiles/r04_expf_census.json).

usage: python scripts/expf_census.py [out.json] [--threads N] [--quick]
"""
from __future__ import annotations

import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "sdp-gs_amd"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402

import oracle.oracle as O  # noqa: E402
from gsr_amd.synthetic import make_cameras, make_gaussians  # noqa: E402

CASES = {"cfg3_1m_1008x756": (1_000_000, 1008, 756, 3), "cfg5_5m_1920x1080": (5_000_000, 1920, 1080, 2)}


def run_case(P, W, H, V):
    g = make_gaussians(P, sh_degree=3, seed=0)
    with torch.no_grad():
        op = torch.sigmoid(g.opacity).view(-1).numpy()
        sc = torch.exp(g.scaling).numpy()
        rot = torch.nn.functional.normalize(g.rotation).numpy()
    shs = torch.cat((g.features_dc, g.features_rest), 1).numpy()
    out = []
    for cam in make_cameras(V, W, H, seed=0):
        kw = dict(means3D=g.xyz.numpy(), opacities=op, viewmatrix=cam.world_view_transform.numpy(),
                  projmatrix=cam.full_proj_transform.numpy(), campos=cam.camera_center.numpy(),
                  tanfovx=math.tan(cam.FoVx * 0.5), tanfovy=math.tan(cam.FoVy * 0.5),
                  image_height=H, image_width=W, bg=np.zeros(3, np.float32), sh_degree=3, shs=shs,
                  scales=sc, rotations=rot, shs_language=g.language_feature.numpy(),
                  include_feature=True)
        t0 = time.time()
        res = {}
        for v in ("f32", "expf", "f64"):
            o = O.OracleRaster(variant=v, **kw)
            res[v] = dict(img=np.concatenate([o.color, o.depth, o.alpha, o.feature]).astype(np.float64),
                          T=o.final_T().astype(np.float64), n=o.n_contrib(), radii=o.radii.copy())
            if v == "f32":
                margin = o.margin()
            del o
        a = res["f32"]
        rec = {"pixels": W * H, "seconds": round(time.time() - t0, 1)}
        for v in ("expf", "f64"):
            b = res[v]
            flip = (a["n"] != b["n"]) | (np.abs(a["T"] - b["T"]) > 1e-4 * np.maximum(a["T"], 1e-4))
            d = np.abs(a["img"] - b["img"]).max(0)
            rec[v] = {"decision_flips": int(flip.sum()),
                      "flips_near_threshold": int((flip & (margin < 1e-4)).sum()),
                      "radii_differ": int((a["radii"] != b["radii"]).sum()),
                      "max_image_delta": float(d.max()),
                      "max_image_delta_unflipped": float(d[~flip].max()) if (~flip).any() else 0.0,
                      "pixels_off_1e-5": int((d > 1e-5).sum())}
        out.append(rec)
        print(json.dumps(rec), flush=True)
    return out


def main():
    args = sys.argv[1:]
    threads = int(args[args.index("--threads") + 1]) if "--threads" in args else (os.cpu_count() or 1)
    path = next((a for a in args if a.endswith(".json")), os.path.join(ROOT, "profiles", "r04_expf_census.json"))
    O.set_threads(threads)
    doc = {"what": "blend decisions: splat_exp (HIP kernels and checker) vs libm expf vs float64 exp, "
                   "CPU oracle forward (scripts/expf_census.py)", "threads": threads, "cases": {}}
    cases = {"small_20k_200x150": (20_000, 200, 150, 2)} if "--quick" in args else CASES
    for name, (P, W, H, V) in cases.items():
        print(name, flush=True)
        doc["cases"][name] = run_case(P, W, H, V)
    with open(path, "w") as fh:
        json.dump(doc, fh, indent=1)
    print("wrote", path)


if __name__ == "__main__":
    main()
