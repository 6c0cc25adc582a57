"""The work queue's row parts on CPU (rtk_row_parts in librt_mi355x.so, no
device needed): every stratum row of sqrt_spp = S samples goes out as `parts`
queue entries of ceil(S / parts) consecutive samples, summed in part order by
the reduce (and by rt_render_partials_get).  The split is a function of the
whole frame -- never of a row shard -- so 1..8 GPUs sum every row alike and
produce the same bits; no part may be empty (a lane would trace sample S);
the part sums of the whole frame stay within the memory budget."""
import ctypes

import pytest

GiB = 1 << 30


@pytest.fixture(scope="module")
def row_parts(product):
    import importlib
    lib = ctypes.CDLL(importlib.import_module("raytracer-2025_amd").LIB_PATH)
    f = lib.rtk_row_parts
    f.restype = ctypes.c_uint32
    f.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64]
    return f


@pytest.mark.parametrize("S", list(range(1, 70)) + [100, 128, 256, 1000])
@pytest.mark.parametrize("part_samples", [0, 1, 2, 5, 6, 7, 11, 16])
def test_parts_cover_the_row_without_empty_parts(row_parts, S, part_samples):
    p = row_parts(16, 16, S, part_samples, 1 << 62)  # no budget or queue-size cap here
    assert p >= 1
    if part_samples == 0 or S <= part_samples:
        assert p == 1
        return
    length = -(-S // p)
    assert (p - 1) * length < S <= p * length  # the last part holds >= 1 sample
    assert length <= part_samples or p == S  # parts no longer than asked
    assert p <= S


def test_budget_bounds_the_part_sums(row_parts):
    # C5: 3840 x 2160 at 64^2: whole rows are 12.7 GB of part sums already
    assert row_parts(3840, 2160, 64, 6, 8 * GiB) == 1
    # C2 (the headline): 22 samples per row -> 4 parts of 6, 4.4 GB
    assert row_parts(1920, 1080, 22, 6, 8 * GiB) == 4
    for W, H, S in ((1920, 1080, 22), (800, 800, 32), (3840, 2160, 16), (1920, 1080, 45)):
        p = row_parts(W, H, S, 6, 8 * GiB)
        assert p == 1 or W * H * S * p * 24 <= 8 * GiB


def test_queue_of_the_whole_frame_fits_32_bits(row_parts):
    # 3840 x 2160 at 1000^2 samples: 8.3e12 whole rows already -- no parts
    assert row_parts(3840, 2160, 1000, 6, 1 << 62) == 1
    p = row_parts(1920, 1080, 100, 6, 1 << 62)
    assert p > 1 and 1920 * 1080 * 100 * p < 0xFFF00000
