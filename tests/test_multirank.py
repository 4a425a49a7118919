"""Multi-GPU path of bench.py / SURVEY.md §8(e), rehearsed on CPU.

One process per rank (torch.distributed, gloo, world size 2, 127.0.0.1): each
rank takes its round-robin share of the 32x32 buckets (shard_buckets, bucket k
-> rank k mod world), renders only those into a zeroed full frame and the
frames are combined with one reduce(sum) to rank 0 — exactly what bench.py
does over RCCL.  The renders here are the CPU oracle's fp32 mode (no GPU in
this suite); the GPU path shares the bucket and combine logic and is checked
bucket-by-bucket in tests/test_gpu_parity.py.

Checks: the shards partition the frame (every pixel exactly one owner), and
the combined frame equals the single-process full-frame render bit for bit
(the RNG is keyed by global pixel id; each pixel has one contributor).
"""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WIDTH, SPP, SEED = 96, 2, 5


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _scene():
    import sys
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    import __graft_entry__ as ge
    g = ge.load_package()
    from oracle import oracle_py as O
    return g, O, g.Scene("cornell-lucy", width=WIDTH, lucy_rings=30, lucy_cols=40)


def _rank(rank, world, port, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g, O, s = _scene()
        cam = s.camera
        W, H = cam.image_width, cam.image_height
        buckets = g.generate_buckets(W, H, 32)
        mine = g.shard_buckets(buckets, rank, world)
        frame = O.render(s.desc, cam, g.make_params(SPP, cam.max_depth, seed=SEED, buckets=mine), fp32=True,
                         threads=2)
        owner = np.zeros((H, W), np.int64)
        for (x, y, w, h) in mine:
            owner[y:y + h, x:x + w] += 1
        t = torch.from_numpy(frame.copy())
        o = torch.from_numpy(owner)
        dist.reduce(t, dst=0, op=dist.ReduceOp.SUM)
        dist.reduce(o, dst=0, op=dist.ReduceOp.SUM)
        if rank == 0:
            np.save(out_path + ".frame.npy", t.numpy())
            np.save(out_path + ".owner.npy", o.numpy())
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_sharded_render_combines_to_full_frame(tmp_path, g, O):
    world = 2
    out = str(tmp_path / "combined")
    mp.start_processes(_rank, args=(world, _free_port(), out), nprocs=world, join=True, start_method="spawn")
    combined = np.load(out + ".frame.npy")
    owner = np.load(out + ".owner.npy")
    assert (owner == 1).all(), "buckets must partition the frame"
    _, _, s = _scene()
    cam = s.camera
    full = O.render(s.desc, cam, g.make_params(SPP, cam.max_depth, seed=SEED), fp32=True, threads=4)
    assert np.array_equal(combined, full)
    assert combined.sum() > 0


def test_shards_balance_work(g):
    """Round-robin over the centre-out bucket order gives every rank the
    same number of buckets (±1) for the bench frame at 1, 2, 4 and 8 ranks."""
    b = g.generate_buckets(1200, 675, 32)
    assert len(b) == 38 * 22
    for world in (1, 2, 4, 8):
        sizes = [len(g.shard_buckets(b, r, world)) for r in range(world)]
        assert max(sizes) - min(sizes) <= 1
        assert sum(sizes) == len(b)


def _rank_dynamic(rank, world, port, out_path, slow_rank):
    """bench.py's dynamic dealing across ranks: runs of the whole tile list
    claimed through the process group's store (dynamic_runs), each rendered
    before the next claim; slow_rank sleeps after each run, as a device with a
    lower clock would take longer."""
    import sys
    import time
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g, O, s = _scene()
        if ROOT not in sys.path:
            sys.path.insert(0, ROOT)
        import bench
        from torch.distributed import distributed_c10d
        store = distributed_c10d._get_default_store()
        cam = s.camera
        W, H = cam.image_width, cam.image_height
        tiles = g.split_buckets(g.generate_buckets(W, H, 32), 16)
        frame = None
        owner = np.zeros((H, W), np.int64)
        runs = 0
        for a, b in bench.dynamic_runs(lambda k: store.add("deal_test", k), len(tiles), world):
            mine = tiles[a:b]
            part = O.render(s.desc, cam, g.make_params(SPP, cam.max_depth, seed=SEED, buckets=mine), fp32=True,
                            threads=2)
            for (x, y, w, h) in mine:
                owner[y:y + h, x:x + w] += 1
            frame = part.copy() if frame is None else frame + part   # zero outside the run's tiles
            runs += 1
            if rank == slow_rank:
                time.sleep(0.4)
        t = torch.from_numpy(frame)
        o = torch.from_numpy(owner)
        n = torch.tensor([int(owner.sum()), runs], dtype=torch.int64)
        counts = [torch.zeros(2, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(counts, n)
        dist.reduce(t, dst=0, op=dist.ReduceOp.SUM)
        dist.reduce(o, dst=0, op=dist.ReduceOp.SUM)
        if rank == 0:
            np.save(out_path + ".frame.npy", t.numpy())
            np.save(out_path + ".owner.npy", o.numpy())
            np.save(out_path + ".counts.npy", torch.stack(counts).numpy())
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_dynamic_dealing_across_ranks(tmp_path, g, O):
    """Every tile is claimed by exactly one rank, the combined frame equals the
    one-process render bit for bit, and the rank that takes longer per run
    renders fewer pixels (bucket_renderer.go:193-213: a slow worker just
    takes fewer buckets)."""
    world = 2
    out = str(tmp_path / "dyn")
    mp.start_processes(_rank_dynamic, args=(world, _free_port(), out, 1), nprocs=world, join=True,
                       start_method="spawn")
    combined = np.load(out + ".frame.npy")
    owner = np.load(out + ".owner.npy")
    counts = np.load(out + ".counts.npy")
    assert (owner == 1).all(), "claimed runs must partition the frame"
    _, _, s = _scene()
    cam = s.camera
    full = O.render(s.desc, cam, g.make_params(SPP, cam.max_depth, seed=SEED), fp32=True, threads=4)
    assert np.array_equal(combined, full)
    px = counts[:, 0]
    assert px.sum() == cam.image_width * cam.image_height
    assert px[0] > px[1], f"the slow rank should render fewer pixels: {px.tolist()}"


def test_dynamic_runs_rule():
    """dynamic_runs (bench.py) on one rank: the runs tile the list in order,
    the first is half a fair share and later ones shrink to the minimum."""
    import sys
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    import bench
    box = [0]

    def add(k):
        box[0] += k
        return box[0]
    runs = list(bench.dynamic_runs(add, 1000, 4))
    assert runs[0] == (0, 125)
    assert all(a == b0 for (_, a), (b0, _) in zip(runs, runs[1:])) and runs[-1][1] == 1000
    sizes = [b - a for a, b in runs]
    assert sizes[1] == -(-(1000 - 125) // 8) and min(sizes[:-1]) >= 250 // 16
