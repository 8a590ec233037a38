"""Phase timing of the one-sweep radix pass (build with EXTRA=-DGSR_SORT_TRACE=1; run with
GSR_LIB_PATH pointing at that build).  Per partition (workgroup) of the LAST pass of a sort:
start, ranked, scanned, looked back, reordered, stored (100 MHz wall clock).  Prints quantiles
of each phase and of the start / end spread across partitions."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "sdp-gs_amd"))
from gsr_amd import _lib  # noqa: E402

L = _lib.load()
L.gsr_test_sort_trace.restype = ctypes.c_int
L.gsr_test_sort_trace.argtypes = [ctypes.c_void_p, ctypes.c_int]
rng = np.random.default_rng(0)
cases = [("depth1M", rng.lognormal(1.0, 0.5, 1_000_000).astype(np.float32).view(np.uint32), 32),
         ("tiles3M", np.minimum(rng.exponential(300.0, 2_960_000), 3023).astype(np.uint32), 12)]
if os.environ.get("SORT_LARGE", "0") == "1":  # config 5 sizes
    cases += [("depth5M", rng.lognormal(1.0, 0.5, 5_000_000).astype(np.float32).view(np.uint32), 32),
              ("tiles16M", np.minimum(rng.exponential(800.0, 16_250_000), 8159).astype(np.uint32), 13)]
out = {}
for name, keys, bits in cases:
    n = keys.size
    k0 = torch.tensor(keys.view(np.int32), device="cuda")
    v0 = torch.arange(n, dtype=torch.int32, device="cuda")
    scratch = torch.empty(int(L.gsr_test_sort_scratch_bytes(n)), dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(5):
        k, v = k0.clone(), v0.clone()
        _lib.check(L.gsr_test_radix_sort_pairs(k.data_ptr(), v.data_ptr(), n, bits,
                                               scratch.data_ptr(), s))
    torch.cuda.synchronize()
    parts = min((n + 4095) // 4096, 16384)
    tr = np.zeros((parts, 8), np.uint64)
    assert L.gsr_test_sort_trace(tr.ctypes.data, parts) == 0
    t = tr[:, :6].astype(np.int64)
    t0 = t[:, 0].min()
    rel = (t - t0) * 10 / 1000.0  # us
    ph = np.diff(t, axis=1) * 10 / 1000.0
    q = lambda a: [round(float(np.quantile(a, x)), 2) for x in (0.1, 0.5, 0.9, 1.0)]  # noqa
    out[name] = {"parts": parts,
                 "start_us_q": q(rel[:, 0]), "end_us_q": q(rel[:, 5]),
                 "rank_us_q": q(ph[:, 0]), "scan_us_q": q(ph[:, 1]), "lookback_us_q": q(ph[:, 2]),
                 "reorder_us_q": q(ph[:, 3]), "store_us_q": q(ph[:, 4]),
                 "xcc_hist": np.bincount(tr[:, 6].astype(np.int64) & 0xF, minlength=8).tolist()}
print(json.dumps(out, indent=1))
