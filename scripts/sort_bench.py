"""Micro-benchmark of the device radix sort (test hook) on depth-like and tile-like keys.
Run under `rocprofv3 --kernel-trace --stats` for per-kernel times."""
import sys, os, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "sdp-gs_amd"))
import numpy as np
import torch
from gsr_amd import _lib

L = _lib.load()
rng = np.random.default_rng(0)
cases = [("depth1M", rng.lognormal(1.0, 0.5, 1_000_000).astype(np.float32).view(np.uint32), 32),
         ("tiles3M", np.minimum(rng.exponential(300.0, 2_960_000), 3023).astype(np.uint32), 12)]
if os.environ.get("SORT_LARGE", "0") == "1":  # config 5: 5M Gaussians, 16.3M instances, 8160 tiles
    cases += [("depth5M", rng.lognormal(1.0, 0.5, 5_000_000).astype(np.float32).view(np.uint32), 32),
              ("tiles16M", np.minimum(rng.exponential(800.0, 16_250_000), 8159).astype(np.uint32), 13)]
for name, keys, bits in cases:
    n = keys.size
    k0 = torch.tensor(keys.view(np.int32), device="cuda")
    v0 = torch.arange(n, dtype=torch.int32, device="cuda")
    scratch = torch.empty(int(L.gsr_test_sort_scratch_bytes(n)), dtype=torch.uint8, device="cuda")
    k, v = k0.clone(), v0.clone()
    s = torch.cuda.current_stream().cuda_stream
    for it in range(25):
        k.copy_(k0); v.copy_(v0)
        _lib.check(L.gsr_test_radix_sort_pairs(k.data_ptr(), v.data_ptr(), n, bits, scratch.data_ptr(), s))
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for it in range(20):
        _lib.check(L.gsr_test_radix_sort_pairs(k.data_ptr(), v.data_ptr(), n, bits, scratch.data_ptr(), s))
    e1.record(); torch.cuda.synchronize()
    print(name, "ms/sort (incl. host sync per call)", e0.elapsed_time(e1) / 20)
