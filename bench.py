#!/usr/bin/env python3
"""Headline benchmark: Msamples/s on the book-1 random-spheres scene at
1920x1080, "512 spp" (= 22^2 = 484 traced strata, camera.rs:212), max_depth 50 (C3: 10, C5: 40),
f64 -- BASELINE.json configs[1] (C2) on 1..8 MI355X.

A step renders one whole frame: every rank renders its interleaved rows
(row_offset = rank, row_stride = N) with the gfx950 kernel through the C ABI
(rt_render_device on torch's current stream), then the linear framebuffer is
gathered to rank 0 over RCCL (N > 1).  Scaling is strong: the frame is fixed,
ranks split it.  value = traced samples of all steps / max-over-ranks time.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--no-cpu-baseline]
  python bench.py --workload c4        # BASELINE configs[3]: 1M-triangle OBJ, 1920x1080, 256 spp
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
      --master-port P bench.py --gpus N --steps K --warmup W
"""
import argparse
import ctypes
import importlib
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
PKG = "raytracer-2025_amd"

FP64_VECTOR_PEAK_TFLOPS = 78.6  # MI355X spec (half the 157.3 TF f32 vector rate)
HBM_PEAK_GBS = 8000.0


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


WORKLOADS = {  # BASELINE.json configs[1..4]: default width, spp
    "c2": (1920, 512),
    "c3": (800, 1024),
    "c4": (1920, 256),
    "c5": (3840, 4096),
}


def build_workload(scenes, scene, workload, width, spp):
    """(world, lights, cam, description) of a bench workload."""
    if workload == "c2":
        world, lights, cam = scenes.random_spheres(scene, width, spp)
        return world, lights, cam, "C2: book-1 random spheres"
    if workload == "c3":
        world, lights, cam = scenes.cornell_smoke(scene, width, spp)
        return world, lights, cam, "C3: book-2 Cornell box + smoke boxes (quads, media, light sampling)"
    if workload == "c5":
        world, lights, cam = scenes.final_scene(scene, width, spp, 40, aspect_ratio=16 / 9)
        return world, lights, cam, "C5: book-2 final scene, aspect 16/9"
    import tempfile
    obj = os.path.join(tempfile.gettempdir(), "rt_terrain_707", "terrain.obj")
    if not os.path.exists(obj):
        scenes.write_terrain_obj(os.path.dirname(obj), 707)
    world, lights, cam = scenes.obj_terrain(scene, obj, width, spp)
    return world, lights, cam, "C4: synthetic 1M-triangle OBJ terrain (999 698 triangles, 2 models) + 2 spheres"


def cpu_baseline(threads, row_stride, spp, workload="c2"):
    """The TEST-ONLY oracle (reference algorithm, f64, recursive ray_color,
    reference BVH topology) on the host cores: a bounded sample of the same
    C2 workload -- every `row_stride`-th row of the 1920x1080 frame at `spp`
    (sqrt_spp^2 strata).  Per-sample cost does not depend on spp."""
    so = os.path.join(ROOT, "oracle", "_build", "liboracle.so")
    if not os.path.exists(so):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, stdout=subprocess.DEVNULL)
    capi = importlib.import_module(PKG + ".capi")
    rt = importlib.import_module(PKG + ".raytracer")
    scenes = importlib.import_module(PKG + ".scenes")
    api = capi.Api(ctypes.CDLL(so), "orc_", capi.ORACLE_EXTRAS)
    scene = rt.Scene(api)
    world, lights, cam, desc = build_workload(scenes, scene, workload, WORKLOADS[workload][0], spp)
    c = cam.to_c()
    opts = capi.RtRenderOpts()
    api.render_opts_default(ctypes.byref(opts))
    opts.seed = 1
    opts.row_offset = 0
    opts.row_stride = row_stride
    opts.threads = threads
    st = capi.RtStats()
    t0 = time.perf_counter()
    api.check(api.render_f64(scene.s, world.h, -1 if lights is None else lights.h, ctypes.byref(c), ctypes.byref(opts),
                             None, None, ctypes.byref(st), None))
    dt = time.perf_counter() - t0
    return {
        "value": st.samples / dt / 1e6,
        "unit": "Msamples/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{desc.split(':')[0]} scene, every {row_stride}th row of {cam.image_width}x{cam.image_height} at {spp} spp ({cam.sqrt_spp**2} traced), "
                  f"{st.samples} samples in {dt:.1f} s on {threads} threads of '{cpu_model()}' "
                  "(oracle/: reference-semantics C++ restatement, not the Rust binary)",
    }


def load_pmc_traffic(path):
    """HBM bytes per launch of the path kernel from a committed rocprofv3 PMC
    summary (profiles/), or None."""
    try:
        with open(path) as f:
            d = json.load(f)
        return d.get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--width", type=int, default=None, help="default: the config's width")
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="c2",
                    help="c2 = BASELINE configs[1] (the headline metric); c3 / c4 / c5 = configs[2] / [3] / [4]")
    ap.add_argument("--spp", type=int, default=None, help="default: the config's spp")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--reference-bvh", action="store_true",
                    help="A/B only: keep the reference BVH topology instead of the SAH rebuild")
    ap.add_argument("--backend", default="nccl", help="nccl (= RCCL) on GPU nodes; gloo only to rehearse ranks on one GPU")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--cpu-row-stride", type=int, default=2)
    ap.add_argument("--cpu-spp", type=int, default=None, help="default: 64 (c2), 36 (c4) -> ~10 s of oracle work")
    args = ap.parse_args()
    if args.spp is None:
        args.spp = WORKLOADS[args.workload][1]
    if args.width is None:
        args.width = WORKLOADS[args.workload][0]

    import torch
    import torch.distributed as dist

    world_size = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world_size != args.gpus:
        if world_size == 1 and args.gpus > 1:
            print("bench.py: --gpus N > 1 must be launched with torch.distributed.run (one process per GPU)",
                  file=sys.stderr)
            sys.exit(2)
    distributed = world_size > 1
    local_dev = local_rank % torch.cuda.device_count()
    torch.cuda.set_device(local_dev)
    device = torch.device("cuda", local_dev)
    if distributed:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group(args.backend)

    pkg = importlib.import_module(PKG)
    rt = importlib.import_module(PKG + ".raytracer")
    scenes = importlib.import_module(PKG + ".scenes")
    capi = importlib.import_module(PKG + ".capi")
    pdist = importlib.import_module(PKG + ".dist")
    api = pkg.load()

    scene = rt.Scene(api)
    world, lights, cam, desc = build_workload(scenes, scene, args.workload, args.width, args.spp)
    H, W = cam.image_height, cam.image_width
    c = cam.to_c()
    opts = capi.RtRenderOpts()
    api.render_opts_default(ctypes.byref(opts))
    opts.seed = args.seed
    opts.row_offset = rank
    opts.row_stride = world_size
    opts.flags = 1 if args.reference_bvh else 0  # RT_FLAG_REFERENCE_BVH
    rows = api.shard_rows(ctypes.byref(c), ctypes.byref(opts))
    out = torch.empty((max(rows, 1), W, 3), dtype=torch.float32, device=device)
    stream = torch.cuda.current_stream(device)
    opts.stream = ctypes.c_void_p(stream.cuda_stream)
    lights_h = -1 if lights is None else lights.h
    kernel_ms = []

    def step(record):
        api.check(api.render_device(scene.s, world.h, lights_h, ctypes.byref(c), ctypes.byref(opts),
                                    ctypes.c_void_p(out.data_ptr())))
        st = capi.RtStats()
        api.check(api.render_device_wait(scene.s, ctypes.byref(st)))  # HIP events around the path kernel
        if record:
            kernel_ms.append(st.kernel_ms)
        if rank == 0 and st.kernel_ms > 5000.0:  # long frames (C5 on few GPUs): show progress
            print("bench.py: frame %.1f s" % (st.kernel_ms / 1e3), file=sys.stderr, flush=True)
        if distributed:
            shard = out[:rows] if args.backend == "nccl" else out[:rows].cpu()
            frame = pdist.gather_frame(shard, H, W)
        else:
            frame = out
        return frame, st

    for _ in range(args.warmup):
        step(False)
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        frame, st = step(True)
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if distributed:
        rdev = device if args.backend == "nccl" else torch.device("cpu")
        t = torch.tensor([elapsed], dtype=torch.float64, device=rdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
        km = torch.tensor([sum(kernel_ms) / len(kernel_ms)], dtype=torch.float64, device=rdev)
        dist.all_reduce(km, op=dist.ReduceOp.MAX)
        kernel_avg_ms = km.item()
    else:
        kernel_avg_ms = sum(kernel_ms) / len(kernel_ms)

    sqrt_spp = cam.sqrt_spp
    frame_samples = W * H * sqrt_spp * sqrt_spp
    value = frame_samples * args.steps / elapsed / 1e6
    if rank == 0:
        assert torch.isfinite(frame).all().item()
        wc_path = os.path.join(ROOT, "bench_data", f"work_counts_{args.workload}.json")
        wc = json.load(open(wc_path))
        # one launch of the path kernel processes this rank's rows
        launch_samples = W * rows * sqrt_spp * sqrt_spp
        flops = wc["flops_per_sample"] * launch_samples
        achieved = flops / (kernel_avg_ms * 1e-3) / 1e12
        traffic = (load_pmc_traffic(os.path.join(ROOT, "profiles", "r01", f"pmc_{args.workload}.json"))
                   if world_size == 1 else None)
        line = {
            "metric": {"c2": "Msamples/s (pixels x traced spp / s), book-1 random spheres 1920x1080, 512 spp (484 traced)",
                       "c3": "Msamples/s (pixels x traced spp / s), book-2 Cornell box + smoke 800x800, 1024 spp",
                       "c4": "Msamples/s (pixels x traced spp / s), synthetic 1M-triangle OBJ 1920x1080, 256 spp",
                       "c5": "Msamples/s (pixels x traced spp / s), book-2 final scene 3840x2160, 4096 spp"}[args.workload],
            "value": round(value, 3),
            "unit": "Msamples/s",
            "n_gpus": world_size,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": {"c2": "synthetic: book-1 random spheres from SplitMix64(2025) (raytracer-2025_amd/data)",
                     "c3": "the reference's cornell_box (main.rs:541-639) + two smoke boxes",
                     "c4": "synthetic: displaced-grid terrain OBJ/MTL written by scenes.write_terrain_obj(707)",
                     "c5": "the reference's final_scene (main.rs:384-539), randomness from SplitMix64(2025)"}[args.workload]
                    + ", render RNG seed " + str(args.seed),
            "config": {
                "workload": f"{desc} {W}x{H}, spp {args.spp} ({sqrt_spp**2} traced), max_depth {cam.max_depth}, "
                            "one frame per step, rows interleaved across ranks, RCCL gather to rank 0",
                "frame_samples": frame_samples,
                "parallelism": f"row-shard x{world_size}",
                "bvh": "reference topology" if args.reference_bvh else "binned SAH collapsed to 4-wide f32 nodes",
            },
            "roofline": {
                "bound": "valu-fp64",
                "achieved": round(achieved, 4),
                "peak": FP64_VECTOR_PEAK_TFLOPS,
                "unit": "TFLOP/s",
                "frac": round(achieved / FP64_VECTOR_PEAK_TFLOPS, 5),
                "traffic": traffic,
                "kernel": "rt_path_kernel",
                "kernel_ms_avg": round(kernel_avg_ms, 3),
                "flops_per_sample": round(wc["flops_per_sample"], 1),
                "note": "algorithmic f64 FLOPs (reference algorithm on the reference BVH topology, "
                        "bench_data/work_counts_<workload>.json) per launch / path-kernel time (HIP events on the render stream)",
            },
        }
        if world_size == 1 and not args.no_cpu_baseline:
            cpu_spp = args.cpu_spp or {"c2": 64, "c3": 400, "c4": 36, "c5": 16}[args.workload]
            line["cpu_baseline"] = cpu_baseline(args.cpu_threads, args.cpu_row_stride, cpu_spp, args.workload)
        print(json.dumps(line), flush=True)
    if distributed:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
