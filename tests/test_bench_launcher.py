"""bench.py --gpus N: the launcher path, on CPU.

With --gpus N > 1 and no torch.distributed environment, bench.py starts
`python -m torch.distributed.run --nproc-per-node N` as a child process (never an exec of a
process that touched the GPU), relays rank 0's JSON line and exits non-zero when a rank fails.
The ranks here are a stand-in script over gloo (the real ranks need the GPU)."""
import json
import os
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

RANK_SCRIPT = textwrap.dedent("""
    import json, os, sys
    import torch, torch.distributed as dist
    dist.init_process_group("gloo")
    r, w = dist.get_rank(), dist.get_world_size()
    t = torch.tensor([float(r + 1)])
    dist.all_reduce(t)
    if r == 0:
        print("progress line that is not the result", flush=True)
        print(json.dumps({"metric": "m", "value": float(t), "n_gpus": w,
                          "argv": sys.argv[1:]}), flush=True)
    dist.destroy_process_group()
    sys.exit(int(os.environ.get("FAIL_RANK", "-1") == str(r)))
""")


def test_launch_ranks_relays_rank0_line(tmp_path):
    import bench
    script = tmp_path / "rank.py"
    script.write_text(RANK_SCRIPT)
    rc, line = bench.launch_ranks(["--steps", "2"], 2, script=str(script))
    assert rc == 0
    rec = json.loads(line)
    assert rec["n_gpus"] == 2 and rec["value"] == 3.0 and rec["argv"] == ["--steps", "2"]


def test_launch_ranks_reports_a_failed_rank(tmp_path):
    import bench
    script = tmp_path / "rank.py"
    script.write_text(RANK_SCRIPT)
    env = dict(os.environ, FAIL_RANK="1")
    rc, line = bench.launch_ranks([], 2, script=str(script), env=env)
    assert rc != 0


def test_bench_gpus2_without_gpu_exits_nonzero():
    """The real entry point takes the launcher branch (WORLD_SIZE unset) and propagates the ranks'
    failure (no GPU here) as a non-zero exit without printing a result line."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["GSR_DIST_BACKEND"] = "gloo"
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps",
                        "1", "--warmup", "0", "--no-cpu-baseline", "--no-extra-legs"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode != 0
    assert '"metric"' not in p.stdout


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_dist2_roofline_bracket_is_collective_free():
    """at N > 1 the dominant kernel's bracket is timed in a reducer-free
    region, so its average launch time stays that of N = 1 (round 5's 2-rank rehearsal read
    render_bwd at 25.6 ms, 33x its N = 1 time, because the bracket spanned the all-reduce).  Two
    gloo ranks share this box's one GPU (so some slowdown from sharing the card is expected, not
    a collective); the line also reports the step time the all-reduce adds
    (collective_exposed_ms).  The ranks are child processes of bench.py's launcher."""
    def run(n):
        env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
        env["GSR_DIST_BACKEND"] = "gloo"
        p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n),
                            "--steps", "5", "--warmup", "2", "--workload", "tiny_20k_320x240",
                            "--no-cpu-baseline", "--no-extra-legs"],
                           env=env, capture_output=True, text=True, timeout=500)
        assert p.returncode == 0, p.stderr[-2000:]
        return json.loads([ln for ln in p.stdout.splitlines() if '"metric"' in ln][-1])
    one, two = run(1), run(2)
    assert one["collective_exposed_ms"] is None
    assert two["collective_exposed_ms"] is not None
    # the dominant kernel can differ between the two runs on a scene this small: compare the N = 2
    # bracket with the same kernel's N = 1 launch time.  The two ranks' timed regions run at the
    # same time on the one GPU, so the bracket also holds the other rank's kernels: a fair share
    # is ~2x, and on this tiny scene a short kernel beside the other rank's wider launches has
    # measured up to ~3.6x; a bracket that spans the all-reduce read 33x (round 5).
    r2 = two["roofline"]
    base = one["kernels"][r2["kernel"]]["avg_ms"]
    assert r2["avg_ms"] <= 5.0 * base, (r2["kernel"], r2["avg_ms"], base)
