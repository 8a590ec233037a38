"""Micro-benchmark of distCUDA2 on libgsr (gsr_dist_knn3): uniform and clustered clouds at 1M and
5M points.  Prints one JSON line (median ms over reps, points/s)."""
from __future__ import annotations

import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "sdp-gs_amd"), os.path.join(ROOT, "tests")]

from gsr_amd.knn import distCUDA2  # noqa: E402
from test_knn import _cloud  # noqa: E402


def main():
    out = {"bench": "knn3"}
    for kind in ("uniform", "blobs"):
        for P in (1_000_000, 5_000_000):
            p = torch.from_numpy(_cloud(kind, P, seed=1)).cuda()
            for _ in range(2):
                distCUDA2(p)
            ts = []
            for _ in range(7):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                distCUDA2(p)
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            ts.sort()
            out[f"{kind}_{P // 1_000_000}M_ms"] = round(ts[len(ts) // 2], 3)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
