#!/usr/bin/env python3
"""Optimizer-step micro-benchmark: one Adam step over GaussianModel's
seven parameter groups at P Gaussians (62 floats per Gaussian), PyTorch's Adam (foreach, and
fused=True when the build offers it) vs gsr FusedAdam (one HIP launch).  Prints one JSON line
with ms/step and HBM GB/s of the 28 algorithmic bytes per element (read p, g, m, v; write p, m, v).
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "sdp-gs_amd"))
import torch  # noqa: E402

from gsr_amd.optim import FusedAdam  # noqa: E402


def groups(P, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    shapes = [(P, 3), (P, 1, 3), (P, 15, 3), (P, 1), (P, 3), (P, 4), (P, 3)]
    lrs = [1.6e-4, 2.5e-3, 1.25e-4, 5e-2, 5e-3, 1e-3, 2.5e-3]
    out = []
    for s, lr in zip(shapes, lrs):
        p = torch.nn.Parameter(torch.randn(s, device="cuda", generator=g))
        p.grad = torch.randn(s, device="cuda", generator=g)
        out.append({"params": [p], "lr": lr})
    return out


def time_opt(make, P, iters=20):
    opt = make(groups(P))
    for _ in range(3):
        opt.step()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        opt.step()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    P = int(os.environ.get("ADAM_P", "1000000"))
    elems = 62 * P
    res = {"P": P, "elements": elems, "bytes_per_step": 28 * elems}
    res["torch_foreach_ms"] = time_opt(lambda g: torch.optim.Adam(g, lr=0.0, eps=1e-15), P)
    try:
        res["torch_fused_ms"] = time_opt(lambda g: torch.optim.Adam(g, lr=0.0, eps=1e-15, fused=True), P)
    except Exception as e:  # not every build has the fused kernel for this device
        res["torch_fused_ms"] = None
        res["torch_fused_error"] = str(e)[:120]
    res["gsr_fused_ms"] = time_opt(lambda g: FusedAdam(g, lr=0.0, eps=1e-15), P)
    for k in ("torch_foreach_ms", "torch_fused_ms", "gsr_fused_ms"):
        if res.get(k):
            res[k.replace("_ms", "_GBs")] = round(28 * elems / (res[k] * 1e-3) / 1e9, 1)
    res["hbm_peak_GBs"] = 8000.0
    res["gsr_fused_frac"] = round(res["gsr_fused_GBs"] / 8000.0, 4)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
