"""Backward-blend list statistics of the bench scene (CPU, C oracle): per wave half (8x4 pixels),
how many list entries round 5's conservative test kept (ellipse of alpha >= 1/255 against the
half's rectangle of pixel centres, without its safety margin; round 6 replaced it by the band form,
gsr_device.h band_extent)
against a pixel-exact test (some pixel centre of the half inside the ellipse) and against the
entries that actually contribute (the forward's accepted pairs).  Lockstep steps per wave = the
max over its two halves.  Test-side tool (uses oracle/), not part of the product.

  python scripts/list_stats.py [--gaussians 1000000] [--width 1008 --height 756]
"""
import argparse
import math
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "sdp-gs_amd"), os.path.join(ROOT, "scripts")]

from oracle.oracle import OracleRaster, build, set_threads  # noqa: E402
from gsr_amd.model import SplatModel  # noqa: E402
from gsr_amd.synthetic import make_cameras, make_gaussians  # noqa: E402
from blend_stats import positions_per_pixel  # noqa: E402


def qform(a, b, c, dx, dy):
    return a * dx * dx + c * dy * dy + 2.0 * b * dx * dy


def box_min(a, b, c, dx0, dx1, dy0, dy1):
    """min of the positive-definite form over [dx0, dx1] x [dy0, dy1]."""
    inside = (dx0 <= 0) & (dx1 >= 0) & (dy0 <= 0) & (dy1 >= 0)
    kx, ky = -b / c, -b / a
    best = np.full(a.shape, np.inf)
    for dx in (dx0, dx1):
        dy = np.clip(kx * dx, dy0, dy1)
        best = np.minimum(best, qform(a, b, c, dx, dy))
    for dy in (dy0, dy1):
        dx = np.clip(ky * dy, dx0, dx1)
        best = np.minimum(best, qform(a, b, c, dx, dy))
    return np.where(inside, 0.0, best)


def pixel_min(a, b, c, mx, my, x0, y0):
    """min of the form over the 8x4 integer pixel centres x0..x0+7, y0..y0+3."""
    best = np.full(a.shape, np.inf)
    for r in range(4):
        dy = (y0 + r) - my
        xs = mx - b * dy / a  # continuous minimiser along the row
        for xi in (np.floor(xs), np.ceil(xs)):
            xi = np.clip(xi, x0, x0 + 7)
            best = np.minimum(best, qform(a, b, c, xi - mx, dy))
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gaussians", type=int, default=1_000_000)
    ap.add_argument("--width", type=int, default=1008)
    ap.add_argument("--height", type=int, default=756)
    ap.add_argument("--threads", type=int, default=8)
    args = ap.parse_args()
    build()
    set_threads(args.threads)
    H, W = args.height, args.width
    model = SplatModel(make_gaussians(args.gaussians, sh_degree=3, seed=0), device="cpu")
    cam = make_cameras(12, W, H, seed=0)[0]
    with torch.no_grad():
        r = OracleRaster(means3D=model.get_xyz.numpy(), opacities=model.get_opacity.numpy(),
                         shs=model.get_features.numpy(), sh_degree=3,
                         scales=model.get_scaling.numpy(), rotations=model.get_rotation.numpy(),
                         shs_language=model.get_language_feature.numpy(), include_feature=True,
                         bg=np.zeros(3, np.float32), viewmatrix=cam.world_view_transform.numpy(),
                         projmatrix=cam.full_proj_transform.numpy(),
                         campos=cam.camera_center.numpy(), tanfovx=math.tan(cam.FoVx * 0.5),
                         tanfovy=math.tan(cam.FoVy * 0.5), image_height=H, image_width=W)
    gx, gy = (W + 15) // 16, (H + 15) // 16
    pl, rg = r.point_list().astype(np.int64), r.ranges().astype(np.int64)
    xy = r.means2D().astype(np.float64)
    co = r.conic_opacity().astype(np.float64)
    nc = r.n_contrib().reshape(H, W).astype(np.int64)
    ncp = np.zeros((gy * 16, gx * 16), np.int64)
    ncp[:H, :W] = nc
    # per tile: instance -> tile, list position
    lens = rg[:, 1] - rg[:, 0]
    tile_of = np.repeat(np.arange(gx * gy), lens)
    pos = np.arange(pl.size) - np.repeat(rg[:, 0], lens)
    g = pl
    a, b, c, op = co[g, 0], co[g, 1], co[g, 2], co[g, 3]
    qc = 2.0 * np.log(np.maximum(255.0 * op, 1e-30))
    mx, my = xy[g, 0], xy[g, 1]
    tx, ty = tile_of % gx, tile_of // gx
    # the forward's accepted pairs -> contributing (half, entry)
    nca, offs, words = r.accept_bits()
    pix, ppos = positions_per_pixel(nca, offs, words, H, W)
    py, px = pix // W, pix % W
    tile = (py // 16) * gx + px // 16
    half = ((py % 16) // 8) * 4 + ((px % 16) // 8) * 2 + (py % 8) // 4  # quadrant * 2 + half
    key = np.unique((tile.astype(np.int64) * 8 + half) * (1 << 20) + ppos)
    contrib = np.bincount(key >> 20, minlength=gx * gy * 8).reshape(gx * gy, 8)
    # the forward's per-block bounding box of the cut ellipse (gsr_render.hip block_mask):
    # half-extents sqrt(qc c / det), sqrt(qc a / det), without its small margins
    det = a * c - b * b
    hx = np.sqrt(np.maximum(qc, 0) * c / det)
    hy = np.sqrt(np.maximum(qc, 0) * a / det)
    res = {}
    for name in ("rect", "pixel", "quad&bbox"):
        cnt = np.zeros((gx * gy, 8), np.int64)
        for h in range(8):
            q, hh = h // 2, h % 2
            x0 = tx * 16 + (q % 2) * 8
            y0 = ty * 16 + (q // 2) * 8 + hh * 4
            # the half's largest n_contrib: entries behind it are left out of its list
            hm = ncp.reshape(gy, 16, gx, 16)[:, (q // 2) * 8 + hh * 4:(q // 2) * 8 + hh * 4 + 4, :,
                                              (q % 2) * 8:(q % 2) * 8 + 8].max(axis=(1, 3)).reshape(-1)
            within = pos < hm[tile_of]
            if name == "rect":
                keep = box_min(a, b, c, x0 - mx, x0 + 7 - mx, y0 - my, y0 + 3 - my) <= qc
            elif name == "pixel":
                keep = pixel_min(a, b, c, mx, my, x0, y0) <= qc
            else:
                qy0 = ty * 16 + (q // 2) * 8
                quad = box_min(a, b, c, x0 - mx, x0 + 7 - mx, qy0 - my, qy0 + 7 - my) <= qc
                bbox = (x0 <= mx + hx) & (x0 + 7 >= mx - hx) & (y0 <= my + hy) & (y0 + 3 >= my - hy)
                keep = quad & bbox
            keep = within & keep
            cnt[:, h] = np.bincount(tile_of[keep], minlength=gx * gy)
        res[name] = cnt
    waves = gx * gy * 4
    for name, cnt in list(res.items()) + [("contributing", contrib)]:
        steps = np.maximum(cnt[:, 0::2], cnt[:, 1::2]).sum()
        print(f"{name:13s}: entries per half {cnt.mean():7.2f}, lockstep steps per wave "
              f"{steps / waves:7.2f}")


if __name__ == "__main__":
    main()
