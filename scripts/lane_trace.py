#!/usr/bin/env python3
"""Lane trace (GPU box): renders a workload's row shard with
librt_mi355x_trace.so (-DRT_WAVE_TRACE: per lane of the grid, s_memrealtime at
start and exit, queue entries taken, rays) and prints how the launch ends --
when lanes start and finish relative to the kernel's span, and how many lanes
are still working in each tenth of it.
  python scripts/lane_trace.py [workload] [spp] [row_stride ...]"""
import ctypes
import importlib
import json
import os
import sys

import numpy as np
import torch  # noqa: F401  (one HIP runtime: load torch first)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
capi = importlib.import_module("raytracer-2025_amd.capi")
rt = importlib.import_module("raytracer-2025_amd.raytracer")
scenes = importlib.import_module("raytracer-2025_amd.scenes")
import bench  # noqa: E402


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "c2"
    spp = int(sys.argv[2]) if len(sys.argv) > 2 else bench.WORKLOADS[wl][1]
    strides = [int(x) for x in sys.argv[3:]] or [1, 8]
    torch.cuda.init()
    lib = ctypes.CDLL(os.path.join(ROOT, "raytracer-2025_amd", os.environ.get("TRACE_LIB", "librt_mi355x_trace.so")))
    lib.rt_lane_trace.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_uint64]
    lib.rt_ray_hist.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_uint64]
    api = capi.Api(lib, "rt_")
    s = rt.Scene(api)
    world, lights, cam, desc = bench.build_workload(scenes, s, wl, bench.WORKLOADS[wl][0], spp)
    cam.render(world, lights, seed=1, want_srgb=False)
    n = 1 << 19
    buf = (ctypes.c_ulonglong * (n * 12))()
    for stride in strides:
        ctypes.memset(buf, 0, ctypes.sizeof(buf))
        torch.cuda.synchronize()
        assert lib.rt_ray_hist(None, 0) == 0
        _, _, st = cam.render(world, lights, seed=1, row_stride=stride, want_srgb=False)
        assert lib.rt_lane_trace(buf, n) == 0
        hist = (ctypes.c_ulonglong * 1024)()
        assert lib.rt_ray_hist(hist, 1024) == 0
        a = np.frombuffer(buf, dtype=np.uint64).reshape(n, 12).astype(np.int64)
        a = a[a[:, 1] > 0]
        t0, t1 = a[:, 0].min(), a[:, 1].max()
        span = (t1 - t0) / 100.0  # 100 MHz -> us
        end = (a[:, 1] - t0) / 100.0
        start = (a[:, 0] - t0) / 100.0
        tenth = [float(np.mean(end > span * k / 10.0)) for k in range(10)]
        rec = {
            "workload": desc, "spp": spp, "row_stride": stride, "lanes": int(len(a)),
            "kernel_ms": round(st.kernel_ms, 3), "trace_span_ms": round(span / 1e3, 3),
            "start_us_max": round(float(start.max()), 1),
            "end_ms_pct": {p: round(float(np.percentile(end, p)) / 1e3, 3) for p in (1, 10, 50, 90, 99, 100)},
            "lanes_working_at_tenths": [round(x, 4) for x in tenth],
            "busy_fraction": round(float(np.sum(end - start) / (len(a) * span)), 4),
            "entries_per_lane": {"min": int(a[:, 2].min()), "mean": round(float(a[:, 2].mean()), 2),
                                 "max": int(a[:, 2].max())},
            "rays_per_lane": {"min": int(a[:, 3].min()), "mean": round(float(a[:, 3].mean()), 1),
                              "max": int(a[:, 3].max())},
        }
        # the waves' queue atomics: per wave (lane 0 of each wave), the wait
        # from issue to return summed over the launch, the count, and when
        # the first one returned
        w0 = a[::64]
        wait_ms = (w0[:, 10] & ((1 << 40) - 1)) / 1e5
        cnt = w0[:, 10] >> 40
        first = w0[:, 11] / 1e5
        rec["queue_atomics_per_wave"] = {
            "count_mean": round(float(cnt.mean()), 2), "count_max": int(cnt.max()),
            "wait_ms_mean": round(float(wait_ms.mean()), 4), "wait_ms_max": round(float(wait_ms.max()), 4),
            "wait_share_of_span": round(float(wait_ms.mean()) / (span / 1e3), 4),
            "first_return_ms_pct": {p: round(float(np.percentile(first[cnt > 0], p)), 3) for p in (1, 50, 99, 100)}
            if (cnt > 0).any() else None}
        # rays begun per 0.25 ms of the launch, as a fraction of the launch's
        # median rate: the ramp (first ms), steady state and drain
        h = np.frombuffer(hist, dtype=np.uint64).astype(np.float64)
        nb = int(np.nonzero(h)[0].max()) + 1 if h.any() else 0
        med = float(np.median(h[:nb][h[:nb] > 0])) if nb else 0.0
        med = med if med > 0 else 1.0
        rec["rays_per_quarter_ms_vs_median"] = {"first_8": [round(x / med, 3) for x in h[:8]],
                                                "last_8": [round(x / med, 3) for x in h[max(0, nb - 8):nb]],
                                                "buckets": nb, "nonzero": int(np.count_nonzero(h)),
                                                "rays": float(h.sum()), "median_rays": med,
                                                "lost_vs_median_ms": round(float(np.sum(np.maximum(0.0, med - h[:nb]))) / med * 0.25, 3)}
        # the last lanes to finish: when they took their last queue entry, which
        # one (pixel row of the shard, stratum row / part), rays since then
        S = cam.sqrt_spp
        last = np.argsort(a[:, 1])[-8:][::-1]
        rec["last_lanes"] = [{"end_ms": round((a[i, 1] - t0) / 1e5, 3), "last_entry_ms": round((a[i, 4] - t0) / 1e5, 3),
                              "q": int(a[i, 5]), "pixel": int(a[i, 5] // S), "rays_after": int(a[i, 3] - a[i, 6]),
                              "entries": int(a[i, 2])} for i in last]
        # the slowest waves: rounds (rays) their busiest lane traced after the
        # wave's queue ran dry, and the rate
        idx = np.arange(len(a))
        wend = {}
        for w in np.unique(idx // 64):
            sl = slice(w * 64, w * 64 + 64)
            wend[int(w)] = int(a[sl, 1].max())
        slow = sorted(wend, key=wend.get)[-5:][::-1]
        rec["slow_waves"] = []
        for w in slow:
            sl = slice(w * 64, w * 64 + 64)
            t_dry = a[sl, 4].max()
            ra = a[sl, 3] - a[sl, 6]
            rec["slow_waves"].append({"end_ms": round((wend[w] - t0) / 1e5, 3),
                                      "last_refill_ms": round((t_dry - t0) / 1e5, 3),
                                      "max_rays_after_last_entry": int(ra.max()),
                                      "lanes_rays_after_gt10": int((ra > 10).sum()),
                                      "us_per_round": round((wend[w] - t_dry) / 100.0 / max(1, int(ra.max())), 2),
                                      "steps_after_busiest": int((a[sl, 8] - a[sl, 9])[np.argmax(ra)]),
                                      "steps_per_ray_busiest": round(float((a[sl, 8] - a[sl, 9])[np.argmax(ra)]) / max(1, int(ra.max())), 1),
                                      "memtime_mhz": round(float(a[sl, 7].max()) / ((wend[w] - a[sl, 0].min()) / 100.0), 1)})
        life = (a[:, 1] - a[:, 0]) / 100.0
        rec["steps_per_ray_mean"] = round(float(a[:, 8].sum()) / float(a[:, 3].sum()), 2)
        rec["memtime_mhz_median"] = round(float(np.median(a[:, 7] / np.maximum(life, 1e-9))), 1)
        rec["last_entry_ms_pct"] = {p: round(float(np.percentile((a[:, 4] - t0) / 1e5, p)), 3) for p in (50, 99, 100)}
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
