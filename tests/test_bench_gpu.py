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
