"""bench.py's launch-mode selection (CPU only): a plain `python bench.py
--gpus N` with N > 1 and no launcher runs in-process over devices 0..N-1
(the driver's bench command must not exit without a line);
under torch.distributed.run each rank renders its rows."""
import importlib.util
import os

import pytest

from conftest import ROOT


@pytest.fixture(scope="module")
def bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_mode_selection(bench):
    assert bench.select_mode(1, 1, False) == "single"
    for n in (2, 4, 8):
        assert bench.select_mode(1, n, False) == "in-process"  # no launcher: never an exit
        assert bench.select_mode(n, n, False) == "ranks"
    assert bench.select_mode(1, 1, True) == "in-process"
    with pytest.raises(ValueError):
        bench.select_mode(4, 8, False)  # launcher and --gpus disagree
    with pytest.raises(ValueError):
        bench.select_mode(2, 2, True)


def test_device_list(bench):
    assert bench.parse_devices(None, 8, 8) == list(range(8))
    assert bench.parse_devices("0,0,0,0,0,0,0,0", 8, 1) == [0] * 8
    with pytest.raises(ValueError):
        bench.parse_devices(None, 8, 1)  # eight GPUs asked, one present: an error, not a silent 1-GPU line
    with pytest.raises(ValueError):
        bench.parse_devices("0,1", 3, 4)
    with pytest.raises(ValueError):
        bench.parse_devices("0,5", 2, 4)


def test_gather_mode_names_match_header(bench):
    text = open(os.path.join(ROOT, "include", "rt_mi355x.h")).read()
    for code, name in ((0, "NONE"), (1, "RCCL_COMM"), (2, "RCCL_DEVICES"), (3, "PEER_COPY")):
        assert f"#define RT_GATHER_{name} {code}" in text
    assert set(bench.GATHER_MODES) == {0, 1, 2, 3}
