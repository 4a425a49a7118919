"""bench.py's multi-rank path end to end on the GPU box.

The driver's scaling runs launch bench.py under torch.distributed.run with one
rank per GPU over RCCL.  The one-GPU test box cannot host RCCL ranks on
distinct devices, so this test runs the same script with two ranks sharing
the GPU and gloo carrying the reduce (RTGPU_BENCH_BACKEND=gloo): bucket
sharding, the per-rank renders, the combine to rank 0, the barrier/max-over-
ranks timing and the JSON line are the production code.  The combined
frame's checksum must equal the single-rank run's exactly (every pixel has
one contributor; the RNG is keyed by global pixel id).  The line must also
split the multi-rank step into each rank's render time and tile count and
the combine's own time (`ranks`), and state its timed region."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--steps", "1", "--warmup", "1", "--no-cpu-baseline", "--no-count", "--no-configs", "--no-balance",
        "--width", "320", "--spp", "8"]


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _line(out):
    return json.loads(out.strip().splitlines()[-1])


@pytest.mark.gpu
@pytest.mark.parametrize("dealing", ["static", "dynamic"])
def test_two_ranks_combine_to_the_single_rank_frame(dealing):
    env = dict(os.environ)
    one = subprocess.run([sys.executable, "bench.py"] + ARGS, cwd=ROOT, env=env, capture_output=True, text=True,
                         timeout=240)
    assert one.returncode == 0, one.stderr[-3000:]
    env["RTGPU_BENCH_BACKEND"] = "gloo"
    two = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                          "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "2",
                          "--dealing", dealing] + ARGS, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert two.returncode == 0, two.stderr[-3000:]
    a, b = _line(one.stdout), _line(two.stdout)
    assert a["n_gpus"] == 1 and b["n_gpus"] == 2
    assert b["config"]["parallelism"] == ("tiles-rr2" if dealing == "static" else "tiles-dyn2")
    assert a["config"]["image_finite"] and b["config"]["image_finite"]
    assert a["config"]["frame_sum"] == b["config"]["frame_sum"] > 0
    # a scaling line splits into per-rank render time, tiles and the combine
    r = b["ranks"]
    assert len(r["render_ms"]) == len(r["reduce_ms"]) == len(r["tiles"]) == 2
    assert sum(r["tiles"]) == r["tiles_total"] and min(r["tiles"]) > 0
    assert all(x > 0 for x in r["render_ms"]) and all(x >= 0 for x in r["reduce_ms"])
    assert "ranks" not in a
    for line in (a, b):
        assert line["timed_region"]["d2h_ms"] > 0 and line["timed_region"]["value_with_d2h"] < line["value"]
