#!/usr/bin/env python3
"""GPU probe: do the fused path's in-kernel activations (gsr_test_activations: sigmoid / exp /
normalize as gsr_device.h evaluates them) equal torch's getters (scene/gaussian_model.py:33-41)
bit for bit?  Also reports which float32 evaluation order reproduces torch's row norm of
F.normalize (candidates emulated exactly with float64 intermediates)."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sdp-gs_amd"))
from gsr_amd import _lib  # noqa: E402


def f32(x):
    return x.to(torch.float32)


def main():
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(0)
    P = 4_000_000
    op = (torch.randn(P, generator=g) * 4).to(dev)
    sc = (torch.randn(P, 3, generator=g) * 3 - 2).to(dev)
    rot = torch.randn(P, 4, generator=g).to(dev)
    L = _lib.load()
    o_op, o_sc, o_rot = torch.empty_like(op), torch.empty_like(sc), torch.empty_like(rot)
    _lib.check(L.gsr_test_activations(op.data_ptr(), sc.data_ptr(), rot.data_ptr(), P,
                                      o_op.data_ptr(), o_sc.data_ptr(), o_rot.data_ptr(),
                                      torch.cuda.current_stream().cuda_stream))
    t_op, t_sc = torch.sigmoid(op), torch.exp(sc)
    t_rot = torch.nn.functional.normalize(rot)
    res = {"sigmoid_mismatch": int((o_op != t_op).sum()), "exp_mismatch": int((o_sc != t_sc).sum()),
           "normalize_mismatch": int((o_rot != t_rot).sum())}
    # torch's norm vs candidate float32 evaluation orders
    n_t = rot.norm(dim=1)
    x, y, z, w = (rot[:, k].double() for k in range(4))
    sq = lambda a: f32(a * a).double()  # noqa: E731  exact square rounded once
    fma = lambda a, b, c: f32(a * b + c).double()  # noqa: E731  single rounding (a*b exact)
    add = lambda a, b: f32(a + b).double()  # noqa: E731
    cands = {
        "seq": add(add(add(sq(x), sq(y)), sq(z)), sq(w)),
        "fma_chain": fma(w, w, fma(z, z, fma(y, y, sq(x)))),
        "pairs_01_23": add(add(sq(x), sq(y)), add(sq(z), sq(w))),
        "pairs_02_13": add(add(sq(x), sq(z)), add(sq(y), sq(w))),
        "fma_pairs_01_23": add(fma(y, y, sq(x)), fma(w, w, sq(z))),
        "fma_pairs_02_13": add(fma(z, z, sq(x)), fma(w, w, sq(y))),
    }
    res["norm_candidates_mismatch"] = {
        k: int((torch.sqrt(f32(v)) != n_t).sum()) for k, v in cands.items()}
    res["sigmoid_as_ops_mismatch"] = int((1.0 / (1.0 + torch.exp(-op)) != t_op).sum())
    print(json.dumps(res))


if __name__ == "__main__":
    main()
