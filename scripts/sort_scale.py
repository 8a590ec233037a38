"""How the one-sweep sort's time scales with the key count: the question behind batching the
binning chains of several views into one launch per stage (1M depth keys vs 6M, 3M tile keys vs
18M).  Run under `rocprofv3 --kernel-trace`; `--analyse <trace dir>` then prints, per
configuration, the span from the totals kernel's start to the last pass's end (what a stream
waits) and the summed kernel time.

usage: rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ss -o run -- \
           python3 scripts/sort_scale.py
       python3 scripts/sort_scale.py --analyse gpurun_out/ss"""
import sys

CONFIGS = [(1_000_000, 32, "depth"), (6_000_000, 32, "depth"), (3_000_000, 12, "tiles"),
           (18_000_000, 12, "tiles")]
REPS = 6


def run():
    import numpy as np
    import torch
    sys.path.insert(0, __file__.rsplit("/", 2)[0] + "/sdp-gs_amd")
    from gsr_amd import _lib
    L = _lib.load()
    s = torch.cuda.current_stream().cuda_stream
    for n, bits, kind in CONFIGS:
        rng = np.random.default_rng(n)
        if kind == "depth":
            keys = rng.lognormal(1.5, 0.7, size=n).astype(np.float32).view(np.uint32) + 0
        else:
            keys = np.minimum(rng.exponential(600.0, size=n), 3023).astype(np.uint32)
        k0 = torch.tensor(keys.view(np.int32), device="cuda")
        v0 = torch.arange(n, dtype=torch.int32, device="cuda")
        scratch = torch.empty(int(L.gsr_test_sort_scratch_bytes(n)), dtype=torch.uint8,
                              device="cuda")
        for _ in range(REPS):
            k, v = k0.clone(), v0.clone()
            torch.cuda.synchronize()
            _lib.check(L.gsr_test_radix_sort_pairs(k.data_ptr(), v.data_ptr(), n, bits,
                                                   scratch.data_ptr(), s))
            torch.cuda.synchronize()
        print(n, bits, "ok", flush=True)


def analyse(d):
    import csv
    import glob
    f = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    calls, cur = [], None
    for r in rows:
        name = r["Kernel_Name"]
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if "radix_totals" in name:
            cur = [s, e, e - s, 0]
            calls.append(cur)
        elif "radix_onesweep" in name and cur is not None:
            cur[1] = e
            cur[2] += e - s
            cur[3] += 1
    i = 0
    for n, bits, kind in CONFIGS:
        mine = calls[i:i + REPS][1:]  # first rep warms up
        i += REPS
        span = sorted(c[1] - c[0] for c in mine)[len(mine) // 2] / 1e3
        busy = sorted(c[2] for c in mine)[len(mine) // 2] / 1e3
        print(f"n={n:>10} bits={bits:2d} passes={mine[0][3]}  span {span:7.1f} us  "
              f"kernels {busy:7.1f} us  ({span / n * 1e6:.2f} us per M keys)")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--analyse":
        analyse(sys.argv[2])
    else:
        run()
