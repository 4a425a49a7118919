#!/usr/bin/env python3
"""Benchmark: Msamples/s (pixels x spp / s) of the path-tracing hot path.

Workload (N=1 and every N): CornellBoxLucy (scenes.go:714-817) overridden to
1200x675, 500 spp, depth 5 — the configuration BASELINE.json's roofline
target is quoted on — with the deterministic synthetic 280K-triangle Lucy
stand-in (the real mesh is a Git-LFS pointer).  One step =
one full-quality render of the frame (every pixel x every sample), scene
already resident in HBM, output a device float3 accumulation buffer.

Multi-GPU (torchrun, one rank per GPU): the 32x32 buckets of the frame are
dealt round-robin to ranks; each rank renders its buckets into a zeroed
full-frame buffer, then one RCCL reduce(sum) to rank 0 combines them (each
pixel has exactly one contributor).  Total work is fixed: strong scaling.

Output: one JSON line on rank 0 (contract in the task statement), with
`roofline` for the render kernel (algorithmic bytes per launch from the
instrumented kernel's traversal counts x the per-unit sizes of SURVEY.md
§8(d) / DESIGN.md, over the render kernel's HIP-event time measured on its
stream) and `cpu_baseline` (the CPU oracle's fp64 restatement of the Go path,
multithreaded, on a bounded sample of the same workload; rank 0, N=1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# Algorithmic bytes per unit of work.
BYTES = {
    "node_visits": 128,      # one BVH4 node = four 24-B child boxes + four child items
    "tri_tests": 36,         # v0, e1, e2 fp32
    "sphere_tests": 32,
    "quad_tests": 64,
    "plane_tests": 32,
    "instance_visits": 96,   # 3x4 affine + inverse (SURVEY: 96 B)
    "instance_box_tests": 32,  # world-space instance culling box
    "volume_tests": 64,
    "material_fetches": 32,
    "env_lookups": 48,       # 4 texels x 12 B
}
ACCUM_BYTES_PER_SAMPLE = 12
# Per-ray state each wavefront kernel streams:
# extend: queue entry 4 + ray o,d 32 + hit record 16 = 52 B per ray;
# shadow: direction 16 + pending contribution 16 + a share of the per-path
# origin / throughput / L read-modify-write 16 = 48 B per shadow ray.
RAY_IO_BYTES = {"extend": 52, "shadow": 48}
HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md: 8.0 TB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--scene", default="cornell-lucy")
    ap.add_argument("--width", type=int, default=1200)
    ap.add_argument("--aspect", type=float, default=16.0 / 9.0)
    ap.add_argument("--spp", type=int, default=500)
    ap.add_argument("--depth", type=int, default=0, help="0: scene default")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--blas", choices=["sah", "reference", "device"], default="sah",
                    help="mesh BLAS builder: host SAH (default), the caller's topology, or the GPU LBVH "
                         "(build.hip); the world BVH is SAH except for 'reference'")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-count", action="store_true", help="skip the instrumented count run")
    ap.add_argument("--cpu-spp", type=int, default=48, help="spp of the CPU baseline sample")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0: min(16, cpu_count)")
    return ap.parse_args()


def main():
    args = parse()
    import numpy as np
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # one rank per GPU; RTGPU_BENCH_BACKEND=gloo (with ranks sharing the
    # visible GPUs) rehearses the multi-rank path on a one-GPU box
    backend = os.environ.get("RTGPU_BENCH_BACKEND", "nccl")
    ndev = max(torch.cuda.device_count(), 1)
    dev_index = local % ndev if world > 1 else 0
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(dev_index)
        dist.init_process_group(backend)
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", dev_index)

    import __graft_entry__ as ge
    g = ge.load_package()

    scene_kw = {}
    if args.width:
        scene_kw["width"] = args.width
    if args.aspect:
        scene_kw["aspect"] = args.aspect
    if args.spp:
        scene_kw["spp"] = args.spp
    if args.depth:
        scene_kw["max_depth"] = args.depth
    t_build = time.time()
    scene = g.Scene(args.scene, **scene_kw)
    cam = scene.camera
    W, H, spp, depth = cam.image_width, cam.image_height, cam.samples_per_pixel, cam.max_depth
    ctx = g.Context(dev_index)
    ctx.set_blas_builder(args.blas)
    ctx.set_tlas_builder("reference" if args.blas == "reference" else "sah")
    ctx.upload(scene.desc)
    info = ctx.info()
    t_build = time.time() - t_build

    buckets = g.generate_buckets(W, H, 32)
    mine = g.shard_buckets(buckets, rank, world)
    params = g.make_params(spp, depth, seed=args.seed, buckets=mine)
    accum = torch.zeros(H * W * 3, dtype=torch.float32, device=dev)
    stream = torch.cuda.current_stream(dev)

    kernel_ms = []
    kernel_times = []

    def step(timed: bool):
        accum.zero_()
        ctx.render_device(cam, params, accum.data_ptr(), stream.cuda_stream)
        if timed:
            kernel_ms.append(ctx.last_render_kernel_ms())
            kernel_times.append(ctx.last_kernel_times())
        if dist is not None:
            if backend == "nccl":
                dist.reduce(accum, dst=0, op=dist.ReduceOp.SUM)   # RCCL over xGMI
            else:
                host = accum.cpu()
                dist.reduce(host, dst=0, op=dist.ReduceOp.SUM)
                if rank == 0:
                    accum.copy_(host)

    # one HIP event before each extend/shade/shadow launch (and after each
    # shadow launch) on the render stream: per-kernel launch durations
    ctx.set_kernel_timing(True)
    for _ in range(args.warmup):
        step(False)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    samples_per_step = W * H * spp
    value = samples_per_step * args.steps / elapsed / 1e6
    ms_per_step = elapsed / args.steps * 1e3
    img_ok = bool(torch.isfinite(accum).all().item()) if rank == 0 else True
    # checksum of the combined frame: identical for any rank count (each pixel
    # has one contributor and the RNG is keyed by global pixel id)
    frame_sum = float(accum.double().sum().item()) if rank == 0 else None

    roofline = None
    work = None
    kernels = None
    if rank == 0 and not args.no_count:
        work_k = ctx.count_work_by_kernel(cam, params)
        work = {k: sum(w[k] for w in work_k.values()) for k in work_k["extend"]}
        kernels = {}
        for kname in ("extend", "shade", "shadow"):
            wk = work_k[kname]
            alg = sum(BYTES[k] * wk[k] for k in BYTES)
            if kname == "extend":
                alg += RAY_IO_BYTES["extend"] * wk["rays"]
            elif kname == "shadow":
                alg += RAY_IO_BYTES["shadow"] * wk["shadow_rays"]
            launches = int(np.mean([t[f"{kname}_launches"] for t in kernel_times]))
            ms_tot = float(np.mean([t[f"{kname}_ms"] for t in kernel_times]))
            kernels[kname] = {"launches": launches, "ms_total": round(ms_tot, 3),
                              "ms_avg": round(ms_tot / max(launches, 1), 4),
                              "alg_bytes_per_launch": int(alg / max(launches, 1)),
                              "achieved_GBs": round(alg / (ms_tot / 1e3) / 1e9, 2) if ms_tot > 0 else None}
        dom = max(kernels, key=lambda k: kernels[k]["ms_total"])
        kd = kernels[dom]
        traffic = None
        pmc = os.path.join(ROOT, "profiles", f"pmc_{args.scene}_{W}x{H}.json")
        if os.path.exists(pmc):
            try:
                traffic = json.load(open(pmc))["kernels"][dom]["hbm_bytes_per_launch"]
            except Exception:
                traffic = None
        roofline = {"bound": "hbm", "achieved": kd["achieved_GBs"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(kd["achieved_GBs"] / HBM_PEAK_GBS, 4), "traffic": traffic,
                    "kernel": f"k_{dom}", "kernel_ms_avg": kd["ms_avg"], "launches_per_step": kd["launches"],
                    "alg_bytes_per_launch": kd["alg_bytes_per_launch"],
                    "pipeline_ms_avg": round(float(np.mean(kernel_ms)), 3)}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import oracle_py as O
        threads = args.cpu_threads or min(16, os.cpu_count() or 1)
        cpu_spp = args.cpu_spp
        # bounded sample: every pixel of the same frame at cpu_spp samples,
        # same scene/BVH/depth, fp64 (the reference's arithmetic)
        cp = g.make_params(cpu_spp, depth, seed=args.seed)
        tc = time.perf_counter()
        O.render(scene.desc, cam, cp, fp32=False, threads=threads)
        tcpu = time.perf_counter() - tc
        cpu = {"value": round(W * H * cpu_spp / tcpu / 1e6, 4), "unit": "Msamples/s", "cores": threads,
               "kind": "port",
               "sample": f"{args.scene} {W}x{H} x {cpu_spp} spp depth {depth} (fp64 C restatement of the Go path, "
                         f"{threads} threads), {tcpu:.1f} s"}

    if rank == 0:
        line = {
            "metric": "Msamples/sec (pixels x SPP / s)",
            "value": round(value, 3),
            "unit": "Msamples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (deterministic 280K-tri Lucy stand-in; scene geometry per scenes.go)",
            "config": {"workload": f"{args.scene} {W}x{H} {spp}spp depth {depth}", "scene": args.scene,
                       "width": W, "height": H, "spp": spp, "max_depth": depth,
                       "parallelism": f"tiles-rr{world}", "buckets": len(buckets), "blas": args.blas,
                       "triangles": info.triangles, "bvh_nodes": info.nodes,
                       "scene_build_s": round(t_build, 2), "device_bvh_build_ms": round(ctx.last_build_ms(), 2),
                       "image_finite": img_ok, "frame_sum": frame_sum},
            "roofline": roofline,
            "cpu_baseline": cpu,
        }
        if kernels is not None:
            line["kernels"] = kernels
        if work is not None:
            line["work_per_sample"] = {k: round(v / max(work["samples"], 1), 3) for k, v in work.items()
                                       if k != "samples"}
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    ctx.close()


if __name__ == "__main__":
    main()
