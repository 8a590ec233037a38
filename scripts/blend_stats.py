"""Blend statistics of the bench scene (CPU, C oracle): how many (pixel group, splat) entries
have a contributing pixel, for pixel groups of several shapes -- the quadrant a backward wave owns
(8x8), its halves (8x4), its 4x4 blocks.  Test-side tool (uses oracle/), not part of the product.

  python scripts/blend_stats.py [--views 2] [--gaussians 1000000] [--width 1008 --height 756]
"""
import argparse
import math
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "sdp-gs_amd"))

from oracle.oracle import OracleRaster, build, set_threads  # noqa: E402
from gsr_amd.model import SplatModel  # noqa: E402
from gsr_amd.synthetic import make_cameras, make_gaussians  # noqa: E402


def positions_per_pixel(nc, offs, words, H, W):
    """-> (pixel index, list position) of every accepted (pixel, entry) pair."""
    nwords = np.diff(offs).astype(np.int64)
    bits = np.unpackbits(words.view(np.uint8), bitorder="little")
    pix_of_word = np.repeat(np.arange(H * W), nwords)
    base = np.repeat(offs[:-1].astype(np.int64), nwords)
    widx = np.arange(words.size)[: pix_of_word.size]
    word_in_pixel = widx - base
    set_idx = np.nonzero(bits[: 32 * pix_of_word.size])[0]
    w = set_idx >> 5
    return pix_of_word[w], word_in_pixel[w] * 32 + (set_idx & 31)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--views", type=int, default=2)
    ap.add_argument("--gaussians", type=int, default=1_000_000)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--width", type=int, default=1008)
    ap.add_argument("--height", type=int, default=756)
    args = ap.parse_args()
    build()
    set_threads(args.threads)
    H, W = args.height, args.width
    model = SplatModel(make_gaussians(args.gaussians, sh_degree=3, seed=0), device="cpu")
    cams = make_cameras(12, W, H, seed=0)
    with torch.no_grad():
        kw = dict(means3D=model.get_xyz.numpy(), opacities=model.get_opacity.numpy(),
                  shs=model.get_features.numpy(), sh_degree=3, scales=model.get_scaling.numpy(),
                  rotations=model.get_rotation.numpy(),
                  shs_language=model.get_language_feature.numpy(), include_feature=True,
                  bg=np.zeros(3, np.float32))
    gx, gy = (W + 15) // 16, (H + 15) // 16
    shapes = {"quadrant 8x8": (8, 8), "half 8x4": (8, 4), "block 4x4": (4, 4)}
    tot = {k: [0, 0] for k in shapes}  # (entries summed over groups, wave steps)
    waves = 0
    for v in range(args.views):
        cam = cams[v]
        r = OracleRaster(**kw, viewmatrix=cam.world_view_transform.numpy(),
                         projmatrix=cam.full_proj_transform.numpy(),
                         campos=cam.camera_center.numpy(),
                         tanfovx=math.tan(cam.FoVx * 0.5), tanfovy=math.tan(cam.FoVy * 0.5),
                         image_height=H, image_width=W)
        nc, offs, words = r.accept_bits()
        pix, pos = positions_per_pixel(nc, offs, words, H, W)
        py, px = pix // W, pix % W
        tile = (py // 16) * gx + px // 16
        waves += gx * gy * 4
        for name, (bw, bh) in shapes.items():
            # group id inside the tile, and the wave (quadrant) it belongs to
            lx, ly = px % 16, py % 16
            g = (ly // bh) * (16 // bw) + lx // bw
            quad = (ly // 8) * 2 + lx // 8
            key = (tile.astype(np.int64) * 64 + g) * (1 << 20) + pos
            uk = np.unique(key)
            grp = uk >> 20
            t_of, g_of = grp // 64, grp % 64
            cnt = np.bincount(grp.astype(np.int64), minlength=gx * gy * 64)
            tot[name][0] += int(cnt.sum())
            # wave steps: groups of one quadrant proceed in lockstep -> max over them
            gxx = np.arange(64) % (16 // bw)
            gyy = np.arange(64) // (16 // bw)
            q_of_g = ((gyy * bh) // 8) * 2 + (gxx * bw) // 8
            c2 = cnt.reshape(gx * gy, 64)
            steps = 0
            for q in range(4):
                sel = np.nonzero((q_of_g == q) & (gyy < 16 // bh))[0]
                steps += int(c2[:, sel].max(axis=1).sum())
            tot[name][1] += steps
            del quad, t_of, g_of
    print(f"views={args.views} P={args.gaussians} waves={waves}")
    for name in shapes:
        e, s = tot[name]
        print(f"{name}: contributing (group, entry) pairs per wave {e / waves:.1f}, "
              f"lockstep steps per wave {s / waves:.1f}")


if __name__ == "__main__":
    main()
