"""Test oracle for the loss row: PyTorch restatements of the reference's
losses, differentiable, in any dtype (float64 is the accuracy yardstick, float32 shows what the
reference itself computes).

  l1_loss, gaussian, create_window, ssim / _ssim   <- utils/loss_utils.py:106-162
  pearson_corrcoef                                 <- torchmetrics.functional.pearson_corrcoef
      (the reference imports it at train.py:22 and utils/loss_utils.py:16; torchmetrics is not
      installed here and environment.yml does not pin it: restated from its published
      single-update algorithm -- means, var via Tensor.var * (n - 1), corr_xy against the prior
      mean 0, each / (n - 1), r = corr / sqrt(var_x var_y), clamp to [-1, 1].  Parity unpinned
      beyond that restatement.)
Test infrastructure only.
"""
from __future__ import annotations

from math import exp

import torch
import torch.nn.functional as F


def l1_loss(x, y):
    return torch.abs(x - y).mean()


def gaussian(window_size, sigma, dtype):
    g = torch.tensor([exp(-(x - window_size // 2) ** 2 / float(2 * sigma ** 2))
                      for x in range(window_size)], dtype=torch.float32)
    return (g / g.sum()).to(dtype)


def create_window(window_size, channel, dtype):
    w1 = gaussian(window_size, 1.5, dtype).unsqueeze(1)
    w2 = w1.mm(w1.t()).unsqueeze(0).unsqueeze(0)
    return w2.expand(channel, 1, window_size, window_size).contiguous()


def ssim(img1, img2, window_size=11, size_average=True):
    channel = img1.size(-3)
    window = create_window(window_size, channel, img1.dtype).to(img1.device)
    pad = window_size // 2
    mu1 = F.conv2d(img1, window, padding=pad, groups=channel)
    mu2 = F.conv2d(img2, window, padding=pad, groups=channel)
    mu1_sq, mu2_sq, mu1_mu2 = mu1.pow(2), mu2.pow(2), mu1 * mu2
    s1 = F.conv2d(img1 * img1, window, padding=pad, groups=channel) - mu1_sq
    s2 = F.conv2d(img2 * img2, window, padding=pad, groups=channel) - mu2_sq
    s12 = F.conv2d(img1 * img2, window, padding=pad, groups=channel) - mu1_mu2
    C1, C2 = 0.01 ** 2, 0.03 ** 2
    m = ((2 * mu1_mu2 + C1) * (2 * s12 + C2)) / ((mu1_sq + mu2_sq + C1) * (s1 + s2 + C2))
    return m.mean() if size_average else m.mean(1).mean(1).mean(1)


def pearson_corrcoef(preds, target):
    n = preds.shape[0]
    mx, my = preds.mean(0), target.mean(0)
    var_x = preds.var(0) * (n - 1)
    var_y = target.var(0) * (n - 1)
    corr_xy = ((preds - mx) * (target - 0.0)).sum(0)
    var_x, var_y, corr_xy = var_x / (n - 1), var_y / (n - 1), corr_xy / (n - 1)
    r = (corr_xy / (var_x * var_y).sqrt()).squeeze()
    return torch.clamp(r, -1.0, 1.0)
