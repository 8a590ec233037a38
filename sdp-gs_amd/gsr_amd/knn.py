"""distCUDA2 on libgsr (include/gsr_knn.h).

`distCUDA2(points)` stands in for `simple_knn._C.distCUDA2`, the un-vendored native KNN the
reference imports at scene/gaussian_model.py:20 and unpacks as `dist, nearest_indices =
distCUDA2(xyz)` (create_from_pcd :198, proximity :514): per point the mean squared distance to its
3 nearest other points (float32 [P]) and their indices (int32 [P,3], nearest first).  Exact search
(gsr_knn.hip); no CPU path.
"""
from __future__ import annotations

import torch

from . import _lib


def distCUDA2(points: torch.Tensor):
    if not points.is_cuda:
        raise RuntimeError("distCUDA2 runs on HIP tensors only (no CPU path)")
    if points.dtype != torch.float32 or points.dim() != 2 or points.shape[1] != 3:
        raise ValueError("distCUDA2 expects float32 points of shape [P, 3]")
    pts = points.detach().contiguous()
    P = pts.shape[0]
    dev = pts.device
    mean = torch.empty(P, dtype=torch.float32, device=dev)
    idx = torch.empty((P, 3), dtype=torch.int32, device=dev)
    L = _lib.load()
    scratch = torch.empty(max(int(L.gsr_knn_scratch_bytes(P)), 1), dtype=torch.uint8, device=dev)
    with torch.cuda.device(dev):
        rc = L.gsr_dist_knn3(P, pts.data_ptr(), mean.data_ptr(), idx.data_ptr(),
                             scratch.data_ptr(), torch.cuda.current_stream(dev).cuda_stream)
    if rc != 0:
        raise RuntimeError(f"gsr_dist_knn3 failed with status {rc}")
    return mean, idx
