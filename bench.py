#!/usr/bin/env python3
"""Headline benchmark: Msamples/s on the book-1 random-spheres scene at
1920x1080, "512 spp" (= 22^2 = 484 traced strata, camera.rs:212), max_depth 50 (C3: 10, C5: 40),
f64 -- BASELINE.json configs[1] (C2) on 1..8 MI355X.

A step renders one whole frame through the C ABI (rt_render_device on
torch's current stream).  With N > 1 ranks (torch.distributed.run, one
process per GPU) every rank passes the library an RCCL communicator
(rt_comm_init; the unique id travels over the torch process group): rank r
renders the rows r, r + N, ... and the library gathers the linear framebuffer
to rank 0 in one ncclSend/ncclRecv group.  --in-process drives N devices from
one process (rt_render_opts.devices).  Scaling is strong: the frame is fixed,
ranks split it.  value = traced samples of all steps / max-over-ranks time.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--no-cpu-baseline]
  python bench.py --workload c4        # BASELINE configs[3]: 1M-triangle OBJ, 1920x1080, 256 spp
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
      --master-port P bench.py --gpus N --steps K --warmup W
  python bench.py --gpus N              # N > 1 without a launcher: in-process over devices 0..N-1

Mode (select_mode): under torch.distributed.run (WORLD_SIZE > 1) one process
per GPU, the library's RCCL communicator gathering to rank 0; with --gpus N >
1 and no launcher (or --in-process), one process drives devices 0..N-1
through rt_render_opts.devices -- ncclCommInitAll communicators and one
ncclSend / ncclRecv group onto device 0.  The line names the gather the
library used (rt_render_gather_mode) and its device time.
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


def usable_cpus():
    """The host CPUs this job may run on: the affinity mask, capped by a cgroup
    CPU quota when one is set (a GPU box gives a job a share of a large host;
    os.cpu_count() reports the whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            q, per = open(path).read().split()[:2]
            if q != "max":
                quota = max(1, int(-(-int(q) // int(per))))
        except (OSError, ValueError):
            pass
    if quota is None:
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = max(1, -(-q // per))
        except (OSError, ValueError):
            pass
    return (min(n, quota) if quota else n), {"affinity": n, "cgroup_quota": quota, "os_cpu_count": os.cpu_count()}


def host_topology():
    """Sockets / cores / threads of the whole host (lscpu), which a GPU box's
    job only gets a share of."""
    out = {}
    try:
        r = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10)
        for line in r.stdout.splitlines():
            k, _, v = line.partition(":")
            k, v = k.strip(), v.strip()
            if k in ("CPU(s)", "Socket(s)", "Core(s) per socket", "Thread(s) per core", "Model name"):
                out[k] = int(v) if v.isdigit() else v
    except (OSError, subprocess.SubprocessError):
        pass
    return out


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def select_mode(world_size, gpus, in_process):
    """How bench.py runs --gpus N: "single" (one GPU, or this rank's rows of a
    gloo rehearsal), "ranks" (torch.distributed.run, one process per GPU) or
    "in-process" (one process, rt_render_opts.devices).  A plain
    `python bench.py --gpus N` (N > 1, no launcher) is in-process, so the
    multi-GPU line never depends on how the driver starts the script.
    Raises ValueError for a launcher whose world size is not --gpus."""
    if world_size > 1:
        if in_process:
            raise ValueError("--in-process runs as one process, not under torch.distributed.run")
        if world_size != gpus:
            raise ValueError(f"WORLD_SIZE {world_size} but --gpus {gpus}")
        return "ranks"
    if gpus > 1 or in_process:
        return "in-process"
    return "single"


def parse_devices(text, gpus, device_count):
    """The in-process device list: --devices "0,0,..." (a test may repeat a
    device; the check build sends such a list through its RCCL stand-in),
    else 0..gpus-1.  Raises ValueError when it does not fit the host."""
    if text:
        devs = [int(x) for x in text.split(",") if x.strip() != ""]
        if len(devs) != gpus:
            raise ValueError(f"--devices names {len(devs)} devices, --gpus is {gpus}")
    else:
        devs = list(range(gpus))
    bad = [d for d in devs if d < 0 or d >= device_count]
    if bad:
        raise ValueError(f"--gpus {gpus} needs devices {devs}, this host has {device_count}")
    return devs


GATHER_MODES = {0: "none", 1: "rccl-communicator", 2: "rccl-device-list", 3: "peer-copy"}


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


def _oracle_render(api, capi, scene, world, lights, cam, row_stride, threads):
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
    # a progress line per CPU run (each well under the GPU box's 3-minute
    # silence limit; C5's baseline is several of them)
    print(f"bench.py: cpu baseline run: {threads} threads, every {row_stride}th row, {dt:.1f} s",
          file=sys.stderr, flush=True)
    return st.samples, dt


def physical_cores():
    """{logical cpu: its core's sibling list} of the CPUs this process may run
    on, from sysfs (None when the topology is not readable)."""
    try:
        allowed = sorted(os.sched_getaffinity(0))
        sib = {}
        for c in allowed:
            txt = open(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list").read().strip()
            cpus = []
            for part in txt.split(","):
                a, _, b = part.partition("-")
                cpus.extend(range(int(a), int(b or a) + 1))
            sib[c] = tuple(sorted(cpus))
        return sib
    except (OSError, ValueError):
        return None


def cpu_busy(interval=1.0):
    """{cpu: busy fraction over `interval` s} from /proc/stat (None if unreadable)."""
    def snap():
        out = {}
        for line in open("/proc/stat"):
            if line.startswith("cpu") and line[3:4].isdigit():
                f = line.split()
                v = list(map(int, f[1:]))
                idle = v[3] + (v[4] if len(v) > 4 else 0)
                out[int(f[0][3:])] = (sum(v), idle)
        return out
    try:
        a = snap()
        time.sleep(interval)
        b = snap()
    except (OSError, ValueError):
        return None
    res = {}
    for c in b:
        if c in a:
            dt = b[c][0] - a[c][0]
            res[c] = 1.0 - (b[c][1] - a[c][1]) / dt if dt > 0 else 1.0
    return res


def smt_yield(api, capi, scene, world, lights, cam, row_stride, budget):
    """Measured SMT yield of the oracle: k threads pinned one per physical
    core against 2k threads on the same k cores' two hardware threads each
    (k = budget / 2, inside the job's CPU quota), on the same sample.  The
    whole-host estimate scales the 2-thread-per-core rate by the host's
    physical cores -- no assumption that a second hardware thread doubles a
    core's rate."""
    sib = physical_cores()
    if not sib:
        return None
    # the least busy physical cores (a GPU box's job shares its host: the
    # low-numbered cores carry the system's and other jobs' threads)
    busy = cpu_busy()
    cores, seen = [], set()
    for c, s in sorted(sib.items()):
        if s[0] not in seen and all(x in sib for x in s):
            seen.add(s[0])
            cores.append(s)
    if busy:
        cores.sort(key=lambda s: (max(busy.get(x, 1.0) for x in s), s[0]))
    smt = sum(len(s) == 2 for s in cores) >= len(cores) // 2 and any(len(s) == 2 for s in cores)
    if smt:
        cores = [s for s in cores if len(s) == 2]
    k = min(len(cores), max(1, budget // 2 if smt else budget))
    pick = cores[:k]
    saved = os.sched_getaffinity(0)
    try:
        os.sched_setaffinity(0, {s[0] for s in pick})
        n1, dt1 = _oracle_render(api, capi, scene, world, lights, cam, row_stride, k)
        n2, dt2 = n1, dt1
        if smt:
            os.sched_setaffinity(0, {x for s in pick for x in s})
            n2, dt2 = _oracle_render(api, capi, scene, world, lights, cam, row_stride, 2 * k)
    finally:
        os.sched_setaffinity(0, saved)
    r1, r2 = n1 / dt1 / 1e6, n2 / dt2 / 1e6
    out = {"cores": k, "one_thread_per_core": round(r1, 4), "unit": "Msamples/s", "cpus": [list(s) for s in pick],
           "busy_before": [round(max(busy.get(x, 0.0) for x in s), 3) for s in pick] if busy else None}
    if smt:
        out.update({"two_threads_per_core": round(r2, 4), "yield": round(r2 / r1, 4),
                    "sample": f"every {row_stride}th row; {k} threads pinned one per core ({dt1:.1f} s), then "
                              f"{2 * k} threads on those cores' {2 * k} hardware threads ({dt2:.1f} s)"})
    else:
        out.update({"two_threads_per_core": None, "yield": None,
                    "sample": f"every {row_stride}th row; {k} threads pinned one per core ({dt1:.1f} s); no SMT"})
    out["per_core_busy"] = round(r2 / k, 5)
    return out


def cpu_baseline(threads, row_stride, spp, workload="c2", cpu_info=None):
    """The TEST-ONLY oracle (reference algorithm, f64, recursive ray_color,
    reference BVH topology, pixels over `threads` host threads as rayon does)
    on the host: a bounded sample of the same workload -- every
    `row_stride`-th row of the frame at `spp` (sqrt_spp^2 strata); per-sample
    cost does not depend on spp.  For C2 also BASELINE configs[0] in full
    (book-1 random spheres 400x225, 100 spp), as BASELINE.md plans."""
    # the timed build: -O3 (cargo --release's opt-level), no work counters
    # (oracle/Makefile liboracle_fast.so); the counting build the tests and
    # scripts/work_counts.py use is timed once beside it on the same sample
    so = os.path.join(ROOT, "oracle", "_build", "liboracle_fast.so")
    so_counting = os.path.join(ROOT, "oracle", "_build", "liboracle.so")
    if not (os.path.exists(so) and os.path.exists(so_counting)):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, stdout=subprocess.DEVNULL)
    capi = importlib.import_module(PKG + ".capi")
    rt = importlib.import_module(PKG + ".raytracer")
    scenes = importlib.import_module(PKG + ".scenes")
    api = capi.Api(ctypes.CDLL(so), "orc_", capi.ORACLE_EXTRAS)
    scene = rt.Scene(api)
    world, lights, cam, desc = build_workload(scenes, scene, workload, WORKLOADS[workload][0], spp)
    samples, dt = _oracle_render(api, capi, scene, world, lights, cam, row_stride, threads)
    api_c = capi.Api(ctypes.CDLL(so_counting), "orc_", capi.ORACLE_EXTRAS)
    scene_c = rt.Scene(api_c)
    world_c, lights_c, cam_c, _ = build_workload(scenes, scene_c, workload, WORKLOADS[workload][0], spp)
    samples_c, dt_c = _oracle_render(api_c, capi, scene_c, world_c, lights_c, cam_c, row_stride, threads)
    # one thread on a proportionally sparser sample: the per-core rate
    samples1, dt1 = _oracle_render(api, capi, scene, world, lights, cam, row_stride * max(1, threads), 1)
    info = cpu_info or {}
    topo = host_topology()
    res = {
        "value": samples / dt / 1e6,
        "unit": "Msamples/s",
        "cores": threads,
        "kind": "port",
        "build": "oracle/_build/liboracle_fast.so (g++ -O3 -ffp-contract=off, work counters compiled out)",
        "sample": f"{desc.split(':')[0]} scene, every {row_stride}th row of {cam.image_width}x{cam.image_height} at {spp} spp ({cam.sqrt_spp**2} traced), "
                  f"{samples} samples in {dt:.1f} s on {threads} threads of '{cpu_model()}' "
                  f"(all CPUs this job may use: affinity {info.get('affinity')}, cgroup quota {info.get('cgroup_quota')}, "
                  f"os.cpu_count {info.get('os_cpu_count')}; oracle/: reference-semantics C++ restatement, not the Rust binary)",
    }
    per_core = samples1 / dt1 / 1e6
    res["per_core"] = {"value": per_core, "unit": "Msamples/s", "seconds": round(dt1, 2), "samples": samples1,
                       "sample": f"1 thread, every {row_stride * max(1, threads)}th row at {spp} spp"}
    res["host"] = topo
    rc = samples_c / dt_c / 1e6
    res["counting_build"] = {"value": round(rc, 4), "unit": "Msamples/s", "seconds": round(dt_c, 2),
                             "timed_over_counting": round(res["value"] / rc, 4),
                             "build": "oracle/_build/liboracle.so (-O2, thread-local work counters: the tests' and "
                                      "scripts/work_counts.py's build; not the baseline)"}
    # the whole host (every physical core, both hardware threads), ESTIMATED
    # from the measured SMT rate per core: k cores, two threads each, on the
    # same rows as the measured baseline (per-row cost varies: sky rows are
    # cheap), times the host's physical cores
    smt = smt_yield(api, capi, scene, world, lights, cam, row_stride, threads)
    res["smt"] = smt
    phys = None
    if isinstance(topo.get("Socket(s)"), int) and isinstance(topo.get("Core(s) per socket"), int):
        phys = topo["Socket(s)"] * topo["Core(s) per socket"]
    if smt and phys:
        per_core_smt = smt["per_core_busy"]
        # the other side of the bound: every core of a fully loaded node held
        # at its guaranteed base clock instead of the boost the 8 measured
        # cores may run at (AMD spec of the box's part: base / max boost)
        clocks = {"EPYC 9575F": (3.3, 5.0)}
        spec = next((v for k, v in clocks.items() if k in str(topo.get("Model name", ""))), None)
        res["whole_host_estimated"] = {
            "value": round(per_core_smt * phys, 3), "unit": "Msamples/s", "physical_cores": phys,
            "hw_threads": topo.get("CPU(s)"),
            "basis": f"ESTIMATED, not measured: {per_core_smt:.4f} Msamples/s per physical core with both hardware "
                     f"threads busy (measured on {smt['cores']} cores, SMT yield {smt['yield']}) x {phys} "
                     f"physical cores ({topo.get('Socket(s)')} sockets x {topo.get('Core(s) per socket')}); "
                     "assumes every core of the node runs at the measured per-core rate (no memory-bandwidth or "
                     "clock loss when all are busy): an upper bound on the node's rate"}
        if spec:
            lo = per_core_smt * phys * spec[0] / spec[1]
            res["whole_host_estimated"]["lower_bound"] = round(lo, 3)
            res["whole_host_estimated"]["lower_bound_basis"] = (
                f"the same per-core rate scaled by base / max boost clock ({spec[0]} / {spec[1]} GHz, the part's "
                "spec): every core of the loaded node at its guaranteed base clock, the measured cores at full boost "
                "-- the most the all-core load can cost in clock" +
                (" (memory bandwidth is not this oracle's bound: C2's world is 123 KB)" if workload == "c2" else
                 "; a memory-bound share of the work is not bounded"))
    if workload == "c2":
        s1 = rt.Scene(api)
        w1, l1, cam1 = scenes.random_spheres(s1, 400, 100)
        n1, dt1 = _oracle_render(api, capi, s1, w1, l1, cam1, 1, threads)
        res["c1_full"] = {"value": n1 / dt1 / 1e6, "unit": "Msamples/s", "seconds": round(dt1, 3), "samples": n1,
                          "config": "BASELINE configs[0]: book-1 random spheres 400x225, 100 spp (10^2 traced), depth 50, "
                                    f"whole frame, {threads} threads"}
    return res


def latest_profile(name):
    """profiles/rNN/<name> of the newest round that has it, or None."""
    base = os.path.join(ROOT, "profiles")
    try:
        rounds = sorted((d for d in os.listdir(base) if d.startswith("r")), reverse=True)
    except OSError:
        return None
    for r in rounds:
        p = os.path.join(base, r, name)
        if os.path.exists(p):
            return p
    return None


def load_profile_field(name, field):
    """One field of a committed rocprofv3 summary (profiles/), or None."""
    p = latest_profile(name)
    if not p:
        return None, None
    try:
        with open(p) as f:
            return json.load(f).get(field), os.path.relpath(p, ROOT)
    except (OSError, ValueError):
        return None, None


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
    ap.add_argument("--no-host-rate", action="store_true", help="skip the host-buffer (PCIe-inclusive) frame")
    ap.add_argument("--reference-bvh", action="store_true",
                    help="A/B only: keep the reference BVH topology instead of the SAH rebuild")
    ap.add_argument("--backend", default="nccl",
                    help="nccl: ranks gather through the library's RCCL communicator (rt_comm_init); "
                         "gloo: rehearse ranks on one GPU with a torch gather (harness only)")
    ap.add_argument("--in-process", action="store_true",
                    help="one process drives --gpus N devices through rt_render_opts.devices (no torchrun)")
    # test hooks (tests/test_bench_gpu.py): a repeated device list, the
    # bounds-checked build (with RT_RCCL_LIB / RT_CHECK_RCCL_DUPS: the RCCL
    # stand-in), the frame's hash in the line
    ap.add_argument("--devices", default=None, help=argparse.SUPPRESS)
    ap.add_argument("--lib", choices=("product", "check"), default="product", help=argparse.SUPPRESS)
    ap.add_argument("--frame-hash", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = every CPU this job may use")
    ap.add_argument("--cpu-row-stride", type=int, default=2)
    ap.add_argument("--cpu-spp", type=int, default=None, help="default: 64 (c2), 36 (c4) -> ~10 s of oracle work")
    args = ap.parse_args()
    if args.spp is None:
        args.spp = WORKLOADS[args.workload][1]
    if args.width is None:
        args.width = WORKLOADS[args.workload][0]

    if args.lib == "check":  # before the package is imported: it reads RT_MI355X_LIB once
        os.environ["RT_MI355X_LIB"] = os.path.join(ROOT, PKG, "librt_mi355x_check.so")
    import torch
    import torch.distributed as dist

    world_size = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    try:
        mode = select_mode(world_size, args.gpus, args.in_process)
        devices = parse_devices(args.devices, args.gpus, torch.cuda.device_count()) if mode == "in-process" else None
    except ValueError as e:
        print(f"bench.py: {e}", file=sys.stderr)
        sys.exit(2)
    in_process = mode == "in-process"
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
    lib_gather = distributed and args.backend == "nccl"
    comm = None
    gather_note = None
    if lib_gather:
        # the frame gather is the library's RCCL group; the id travels over the torch process group
        uid = (ctypes.c_uint8 * 128)()
        ok = 1
        if rank == 0 and api.comm_unique_id(uid) != 0:
            ok = 0
        box = [bytes(uid), ok]
        dist.broadcast_object_list(box, src=0)
        uid = (ctypes.c_uint8 * 128).from_buffer_copy(box[0])
        comm = api.comm_init(uid, world_size, rank) if box[1] else None
        # every rank must agree on the path: fall back to the torch gather
        # (harness) only if some rank could not build the communicator
        flag = torch.tensor([1 if comm else 0], dtype=torch.int32, device=device)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        if flag.item() == 0:
            gather_note = "rt_comm_init failed (" + (api.last_error() or b"").decode() + "): torch gather instead"
            if comm:
                api.comm_destroy(comm)
            comm = None
            lib_gather = False
            print("bench.py: " + gather_note, file=sys.stderr, flush=True)
    if lib_gather:
        opts, keep = rt.Camera._opts(api, args.seed, 0, 1, 0, 1 if args.reference_bvh else 0, comm=comm)
        rows = H if rank == 0 else 0
    elif in_process:
        opts, keep = rt.Camera._opts(api, args.seed, 0, 1, 0, 1 if args.reference_bvh else 0, devices=devices)
        rows = H
    else:
        # N = 1, or the gloo rehearsal: this rank renders its interleaved rows itself
        opts, keep = rt.Camera._opts(api, args.seed, rank, world_size, 0, 1 if args.reference_bvh else 0)
        rows = api.shard_rows(ctypes.byref(c), ctypes.byref(opts))
    out = torch.empty((max(rows, 1), W, 3), dtype=torch.float32, device=device)
    stream = torch.cuda.current_stream(device)
    opts.stream = ctypes.c_void_p(stream.cuda_stream)
    lights_h = -1 if lights is None else lights.h
    kernel_ms, gather_ms = [], []

    def step(record):
        ptr = ctypes.c_void_p(out.data_ptr()) if rows > 0 else None
        api.check(api.render_device(scene.s, world.h, lights_h, ctypes.byref(c), ctypes.byref(opts), ptr))
        st = capi.RtStats()
        api.check(api.render_device_wait(scene.s, ctypes.byref(st)))  # HIP events around the path kernel
        if record:
            kernel_ms.append(st.kernel_ms)
            gather_ms.append(st.gather_ms)
        if rank == 0 and st.kernel_ms > 5000.0:  # long frames (C5 on few GPUs): show progress
            print("bench.py: frame %.1f s" % (st.kernel_ms / 1e3), file=sys.stderr, flush=True)
        if distributed and not lib_gather:
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
    kernel_avg_ms = sum(kernel_ms) / len(kernel_ms)
    if distributed:
        rdev = device if args.backend == "nccl" else torch.device("cpu")
        t = torch.tensor([elapsed, kernel_avg_ms], dtype=torch.float64, device=rdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kernel_avg_ms = t[0].item(), t[1].item()

    sqrt_spp = cam.sqrt_spp
    frame_samples = W * H * sqrt_spp * sqrt_spp
    value = frame_samples * args.steps / elapsed / 1e6
    if rank == 0:
        assert torch.isfinite(frame).all().item()
        wc_path = os.path.join(ROOT, "bench_data", f"work_counts_{args.workload}.json")
        wc = json.load(open(wc_path))
        # one launch of the path kernel processes this rank's (or device's) rows
        parts = max(world_size, args.gpus if in_process else 1)
        launch_rows = -(-H // parts)
        launch_samples = W * launch_rows * sqrt_spp * sqrt_spp
        flops = wc["flops_per_sample"] * launch_samples
        achieved = flops / (kernel_avg_ms * 1e-3) / 1e12
        tps, traffic_src = load_profile_field(f"pmc_{args.workload}.json", "hbm_bytes_per_sample")
        traffic = round(tps * launch_samples) if tps else None
        exec_fps, exec_src = load_profile_field(f"valu_{args.workload}.json", "executed_f64_flops_per_sample")
        n = world_size if distributed else (args.gpus if in_process else 1)
        gmode = GATHER_MODES.get(api.render_gather_mode(scene.s), "?") if (lib_gather or in_process) else None
        how = ("one frame per step on one GPU" if n == 1 else
               f"one frame per step, rows interleaved over {n} GPUs, " +
               ("RCCL gather to rank 0 inside librt_mi355x.so (rt_comm_init)" if lib_gather else
                f"gather onto device {devices[0]} inside librt_mi355x.so (rt_render_opts.devices {devices}: {gmode})"
                if in_process else "torch gather to rank 0 (" + (gather_note or "gloo rehearsal harness") + ")"))
        line = {
            "metric": {"c2": "Msamples/s (pixels x traced spp / s), book-1 random spheres 1920x1080, 512 spp (484 traced)",
                       "c3": "Msamples/s (pixels x traced spp / s), book-2 Cornell box + smoke 800x800, 1024 spp",
                       "c4": "Msamples/s (pixels x traced spp / s), synthetic 1M-triangle OBJ 1920x1080, 256 spp",
                       "c5": "Msamples/s (pixels x traced spp / s), book-2 final scene 3840x2160, 4096 spp"}[args.workload],
            "value": round(value, 3),
            "unit": "Msamples/s",
            "n_gpus": n,
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
                "workload": f"{desc} {W}x{H}, spp {args.spp} ({sqrt_spp**2} traced), max_depth {cam.max_depth}, {how}",
                "frame_samples": frame_samples,
                "parallelism": f"row-shard x{n}",
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
                "frac_basis": "reference-algorithm work: algorithmic f64 FLOPs of the reference algorithm on the "
                              "reference BVH topology (bench_data/work_counts_<workload>.json) per launch / path-kernel "
                              "time (HIP events on the render stream) -- a throughput normalisation, not hardware "
                              "utilisation; frac_executed is the executed-instruction view",
                "traffic_source": (traffic_src + " (HBM bytes per traced sample from the rocprofv3 request "
                                   "counters x this launch's samples)") if traffic_src else None,
            },
        }
        if traffic:
            gbs = traffic / (kernel_avg_ms * 1e-3) / 1e9
            line["roofline"]["hbm_gbs"] = round(gbs, 3)
            line["roofline"]["hbm_peak_gbs"] = HBM_PEAK_GBS
            line["roofline"]["hbm_frac"] = round(gbs / HBM_PEAK_GBS, 6)
            line["roofline"]["hbm_note"] = ("traffic / path-kernel time; the read bytes are L2 miss requests "
                                            "(TCC_EA0_RDREQ_*), which also count Infinity Cache (MALL) hits: an upper "
                                            "bound on DRAM bytes")
        if exec_fps:
            ach_e = exec_fps * launch_samples / (kernel_avg_ms * 1e-3) / 1e12
            line["roofline"]["achieved_executed"] = round(ach_e, 4)
            line["roofline"]["frac_executed"] = round(ach_e / FP64_VECTOR_PEAK_TFLOPS, 5)
            line["roofline"]["executed_source"] = exec_src + " (rocprofv3 SQ_INSTS_VALU_*_F64 x 64 lanes x exec " \
                                                             "density, per traced sample) x this launch's samples"
        if n > 1:
            line["gather"] = gmode or ("torch-" + args.backend)
            line["gather_ms_avg"] = round(sum(gather_ms) / len(gather_ms), 3)
            line["launch"] = mode
        if args.lib != "product":
            line["lib"] = os.path.basename(os.environ["RT_MI355X_LIB"])
        if args.frame_hash:
            import hashlib
            line["frame_sha256"] = hashlib.sha256(frame[:H].contiguous().cpu().numpy().tobytes()).hexdigest()
        if world_size == 1 and not in_process and not args.no_host_rate:
            # the PCIe-inclusive rate: rt_render into caller-owned host buffers
            # (linear f32 + sRGB bytes), SURVEY §8(d)'s t_render
            hopts, _hk = rt.Camera._opts(api, args.seed, 0, 1, 0, 1 if args.reference_bvh else 0)
            import numpy as np
            hl = np.empty((H, W, 3), dtype=np.float32)
            hs = np.empty((H, W, 3), dtype=np.uint8)
            hst = capi.RtStats()
            th = time.perf_counter()
            api.check(api.render(scene.s, world.h, lights_h, ctypes.byref(c), ctypes.byref(hopts),
                                 hl.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
                                 hs.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), ctypes.byref(hst)))
            dh = time.perf_counter() - th
            line["host_inclusive"] = {"value": round(frame_samples / dh / 1e6, 3), "unit": "Msamples/s",
                                      "ms": round(dh * 1e3, 3), "kernel_ms": round(hst.kernel_ms, 3),
                                      "note": "one rt_render into host buffers (linear f32 + sRGB u8, PCIe copy "
                                              "included), after the timed steps; not `value`"}
        if world_size == 1 and not in_process and not args.no_cpu_baseline:
            cpu_spp = args.cpu_spp or {"c2": 64, "c3": 400, "c4": 36, "c5": 16}[args.workload]
            threads, info = usable_cpus()
            if args.cpu_threads:
                threads = args.cpu_threads
            cb = cpu_baseline(threads, args.cpu_row_stride, cpu_spp, args.workload, info)
            # the north-star ratios, GPU value over each CPU rate (vs_baseline
            # stays the driver's: BASELINE.md holds no published number)
            cb["speedup"] = round(value / cb["value"], 2)
            if cb.get("whole_host_estimated"):
                wh = cb["whole_host_estimated"]
                cb["speedup_whole_host"] = round(value / wh["value"], 2)
                if wh.get("lower_bound"):
                    cb["speedup_whole_host_range"] = [round(value / wh["value"], 2), round(value / wh["lower_bound"], 2)]
            line["cpu_baseline"] = cb
        print(json.dumps(line), flush=True)
    if comm:
        api.comm_destroy(comm)
    if distributed:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
