"""bench.py's output contract on the GPU: one JSON line with the driver's
keys, the roofline and cpu_baseline objects, consistent arithmetic (value =
frame samples x steps / wall time), at a small size so it runs in seconds."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_bench(*args):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                       timeout=110, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_bench_line_contract():
    d = run_bench("--steps", "2", "--warmup", "1", "--width", "256", "--spp", "16", "--cpu-spp", "1",
                  "--cpu-row-stride", "16")
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["unit"] == "Msamples/s" and d["n_gpus"] == 1 and d["steps"] == 2 and d["warmup"] == 1
    assert d["higher_is_better"] is True and d["scaling"] in ("strong", "weak") and d["dtype"] == "f64"
    assert d["vs_baseline"] is None
    W, H = 256, 144
    samples = W * H * 16
    assert d["config"]["frame_samples"] == samples
    assert abs(d["value"] - samples * 2 / (d["ms_per_step"] * 2 * 1e-3) / 1e6) <= 1e-3 * d["value"] + 1e-3
    rf = d["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in rf, k
    assert rf["peak"] == 78.6 and rf["unit"] == "TFLOP/s"
    assert abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-3
    assert 0 < rf["kernel_ms_avg"] <= d["ms_per_step"] * 1.05
    if rf["traffic"] is not None:  # HBM bytes from the committed PMC summary: the GB/s view of them
        assert rf["hbm_peak_gbs"] == 8000.0
        assert abs(rf["hbm_gbs"] - rf["traffic"] / (rf["kernel_ms_avg"] * 1e-3) / 1e9) <= 1e-3 * rf["hbm_gbs"] + 1e-3
        assert abs(rf["hbm_frac"] - rf["hbm_gbs"] / 8000.0) < 1e-5
    cb = d["cpu_baseline"]
    for k in ("value", "unit", "cores", "kind", "sample", "speedup", "smt"):
        assert k in cb, k
    assert cb["kind"] == "port" and cb["value"] > 0 and cb["cores"] >= 1
    assert abs(cb["speedup"] - d["value"] / cb["value"]) <= 0.01 * cb["speedup"] + 0.01
    if cb["smt"]:  # SMT yield measured on the box's own cores, not assumed
        assert cb["smt"]["one_thread_per_core"] > 0 and cb["smt"]["per_core_busy"] > 0
        whole = cb["whole_host_estimated"]
        assert whole["value"] > 0 and "ESTIMATED" in whole["basis"]
        assert abs(cb["speedup_whole_host"] - d["value"] / whole["value"]) <= 0.01 * cb["speedup_whole_host"] + 0.01


def test_bench_two_ranks_gloo():
    """The N > 1 path (torch.distributed.run, rows interleaved, frame gathered
    to rank 0) with 2 ranks sharing the one GPU over gloo: one JSON line from
    rank 0, n_gpus 2, the whole frame's samples."""
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
                        "--gpus", "2", "--steps", "2", "--warmup", "1", "--width", "256", "--spp", "16",
                        "--backend", "gloo", "--no-cpu-baseline"],
                       capture_output=True, text=True, timeout=110, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["frame_samples"] == 256 * 144 * 16 and d["value"] > 0


def _bench_env(**extra):
    env = dict(os.environ)
    env.update(extra)
    return env


def test_bench_multi_gpu_without_launcher_standin(rccl_standin):
    """`python bench.py --gpus 8`, the shape of the driver's bench command
    with no torch.distributed.run, renders in-process over a device list
    (rt_render_opts.devices -> ncclCommInitAll -> one send / receive group).
    On the one-GPU box the list is device 0 eight times, through the check
    build and the RCCL stand-in (RT_CHECK_RCCL_DUPS=1 sends a repeated list
    through the RCCL group): one JSON line, n_gpus 8, the RCCL device-list
    gather, and a frame hash equal to the one-GPU frame's."""
    so, _ = rccl_standin
    common = ["--steps", "2", "--warmup", "1", "--width", "256", "--spp", "16", "--no-cpu-baseline",
              "--no-host-rate", "--lib", "check", "--frame-hash"]
    env = _bench_env(RT_RCCL_LIB=so, RT_CHECK_RCCL_DUPS="1")
    r1 = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", *common],
                        capture_output=True, text=True, timeout=110, cwd=ROOT, env=env)
    assert r1.returncode == 0, r1.stderr[-3000:]
    one = json.loads([l for l in r1.stdout.splitlines() if l.startswith("{")][0])
    r8 = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8",
                         "--devices", ",".join(["0"] * 8), *common],
                        capture_output=True, text=True, timeout=110, cwd=ROOT, env=env)
    assert r8.returncode == 0, r8.stderr[-3000:]
    lines = [l for l in r8.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r8.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 8 and d["launch"] == "in-process" and d["gather"] == "rccl-device-list"
    assert d["lib"] == "librt_mi355x_check.so" and one["lib"] == "librt_mi355x_check.so"
    assert d["gather_ms_avg"] > 0 and d["config"]["frame_samples"] == 256 * 144 * 16
    assert d["frame_sha256"] == one["frame_sha256"]


def test_bench_repeated_devices_peer_copy():
    """The product library with a repeated device list (real RCCL refuses two
    ranks on one device): the parts reach device 0 by peer copies, named in the
    line, and the frame is the one-GPU frame."""
    common = ["--steps", "1", "--warmup", "1", "--width", "128", "--spp", "4", "--no-cpu-baseline",
              "--no-host-rate", "--frame-hash"]
    r1 = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", *common],
                        capture_output=True, text=True, timeout=110, cwd=ROOT)
    assert r1.returncode == 0, r1.stderr[-3000:]
    one = json.loads([l for l in r1.stdout.splitlines() if l.startswith("{")][0])
    r3 = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "3", "--devices", "0,0,0",
                         *common], capture_output=True, text=True, timeout=110, cwd=ROOT)
    assert r3.returncode == 0, r3.stderr[-3000:]
    d = json.loads([l for l in r3.stdout.splitlines() if l.startswith("{")][0])
    assert d["n_gpus"] == 3 and d["gather"] == "peer-copy" and d["frame_sha256"] == one["frame_sha256"]
