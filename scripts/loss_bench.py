"""Micro-benchmark of the loss row: photometric (L1 + SSIM) forward+backward and the depth Pearson
loss at 3x756x1008 (the LLFF bench camera) -- gsr_amd.losses vs the PyTorch restatement of the
reference (tests/loss_ref.py: F.conv2d SSIM + autograd, torchmetrics-style Pearson).  One JSON line."""
from __future__ import annotations

import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "sdp-gs_amd"), os.path.join(ROOT, "tests")]

import loss_ref  # noqa: E402
from gsr_amd import losses  # noqa: E402


def _ms(fn, reps=50):
    for _ in range(5):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    H, W = 756, 1008
    g = torch.Generator(device="cuda").manual_seed(0)
    gt = torch.rand((3, H, W), generator=g, device="cuda")
    img = (gt + 0.1 * torch.randn((3, H, W), generator=g, device="cuda")).clamp(0, 1)
    x = img.clone().requires_grad_(True)
    mono = torch.rand((1, H, W), generator=g, device="cuda") * 50 + 1
    depth = (mono * 3 + torch.randn((1, H, W), generator=g, device="cuda")).requires_grad_(True)

    def ours_photo():
        loss, _ = losses.photometric_loss(x, gt, 0.2)
        loss.backward()

    def ref_photo():
        loss = 0.8 * loss_ref.l1_loss(x, gt) + 0.2 * (1 - loss_ref.ssim(x[None], gt[None]))
        loss.backward()

    def ours_depth():
        losses.depth_pearson_loss(mono, depth).backward()

    def ref_depth():
        m, d = mono.reshape(-1, 1), depth.reshape(-1, 1)
        min((1 - loss_ref.pearson_corrcoef(m, d)),
            (1 - loss_ref.pearson_corrcoef(1 / (-m + 200), d))).backward()

    xd = depth.detach().clone().requires_grad_(True)

    def ours_view():
        tot, _ = losses.train_view_loss(x, xd, gt, mono, 0.2, 0.05)
        tot.backward()

    out = {"bench": "losses", "shape": [3, H, W],
           "train_view_loss_fwd_bwd_ms": round(_ms(ours_view), 4),
           "photometric_fwd_bwd_ms": round(_ms(ours_photo), 4),
           "photometric_ref_ms": round(_ms(ref_photo), 4),
           "depth_pearson_fwd_bwd_ms": round(_ms(ours_depth), 4),
           "depth_pearson_ref_ms": round(_ms(ref_depth), 4)}
    out["photometric_speedup"] = round(out["photometric_ref_ms"] / out["photometric_fwd_bwd_ms"], 2)
    out["depth_pearson_speedup"] = round(out["depth_pearson_ref_ms"] / out["depth_pearson_fwd_bwd_ms"], 2)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
