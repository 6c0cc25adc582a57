"""The work queue's split on CPU (rtk_row_parts / rtk_tail_rows in
librt_mi355x.so, no device needed).  The stratum rows of a frame's last
image rows -- its tail -- go out as `parts` queue entries of ceil(S / parts)
consecutive samples each, summed in part order by the reduce (and by
rt_render_partials_get); every other stratum row is one entry.  The split is a
function of the whole frame -- never of a row shard -- so 1..8 GPUs sum every
row alike and produce the same bits; no part may be empty (a lane would trace
sample S); the tail's extra part sums stay within the memory budget and the
frame's queue within 2^32 entries."""
import ctypes

import pytest

GiB = 1 << 30


@pytest.fixture(scope="module")
def lib(product):
    import importlib
    lib = ctypes.CDLL(importlib.import_module("raytracer-2025_amd").LIB_PATH)
    lib.rtk_row_parts.restype = ctypes.c_uint32
    lib.rtk_row_parts.argtypes = [ctypes.c_uint32, ctypes.c_uint32]
    lib.rtk_tail_rows.restype = ctypes.c_uint32
    lib.rtk_tail_rows.argtypes = [ctypes.c_uint32] * 4 + [ctypes.c_uint64, ctypes.c_uint32]
    return lib


@pytest.mark.parametrize("S", list(range(1, 70)) + [100, 128, 256, 1000])
@pytest.mark.parametrize("part_samples", [0, 1, 2, 4, 5, 6, 7, 11, 16])
def test_parts_cover_the_row_without_empty_parts(lib, S, part_samples):
    p = lib.rtk_row_parts(S, part_samples)
    assert p >= 1
    if part_samples == 0 or S <= part_samples:
        assert p == 1
        return
    length = -(-S // p)
    assert (p - 1) * length < S <= p * length  # the last part holds >= 1 sample
    assert length <= part_samples or p == S  # parts no longer than asked
    assert p <= S


def test_tail_is_the_asked_share_of_the_frame(lib):
    # C2 (the headline): 22 samples per stratum row -> 6 parts; the last 1/4
    # of 1080 rows, 1.4 GB of extra part sums
    assert lib.rtk_row_parts(22, 4) == 6
    assert lib.rtk_tail_rows(1920, 1080, 22, 6, 2 * GiB, 250) == 270
    assert lib.rtk_tail_rows(1920, 1080, 22, 6, 2 * GiB, 125) == 135
    # the whole frame asked: as many rows as 2 GiB of extra part sums hold
    assert lib.rtk_tail_rows(1920, 1080, 22, 6, 2 * GiB, 1000) == 2 * GiB // (1920 * 22 * 5 * 24)
    assert lib.rtk_tail_rows(1920, 1080, 22, 6, 1 << 62, 1000) == 1080
    # rounds up: a tiny frame still ends on parts
    assert lib.rtk_tail_rows(16, 9, 4, 2, 1 << 62, 250) == 3
    # nothing to split
    assert lib.rtk_tail_rows(1920, 1080, 22, 1, 2 * GiB, 250) == 0
    assert lib.rtk_tail_rows(1920, 1080, 22, 6, 2 * GiB, 0) == 0


@pytest.mark.parametrize("W,H,S,ps", [(1920, 1080, 22, 4), (800, 800, 32, 4), (1920, 1080, 16, 4),
                                      (3840, 2160, 64, 4), (3840, 2160, 16, 4), (1920, 1080, 45, 6)])
def test_budget_bounds_the_tail_part_sums(lib, W, H, S, ps):
    p = lib.rtk_row_parts(S, ps)
    for budget in (GiB // 4, 2 * GiB, 8 * GiB):
        t = lib.rtk_tail_rows(W, H, S, p, budget, 250)
        assert t <= -(-H * 250 // 1000)
        assert t * W * S * (p - 1) * 24 <= budget
        # as many rows as the budget holds
        assert t == -(-H * 250 // 1000) or (t + 1) * W * S * (p - 1) * 24 > budget
    # C5 (3840 x 2160 at 64^2): whole rows are 12.7 GB; the default 2-GiB budget
    # still gives its launch a tail of parts
    if (W, H, S) == (3840, 2160, 64):
        assert lib.rtk_tail_rows(W, H, S, p, 2 * GiB, 250) >= 20


def test_queue_of_the_whole_frame_fits_32_bits(lib):
    # 3840 x 2160 at 1000^2 samples: 8.3e12 whole rows already -- no tail
    assert lib.rtk_tail_rows(3840, 2160, 1000, 250, 1 << 62, 1000) == 0
    W, H, S = 1920, 1080, 100
    p = lib.rtk_row_parts(S, 4)
    t = lib.rtk_tail_rows(W, H, S, p, 1 << 62, 1000)
    assert 0 < t < H
    assert W * H * S + t * W * S * (p - 1) < 0xFFF00000


@pytest.mark.parametrize("H,tail", [(1080, 540), (1080, 0), (1080, 1080), (54, 14), (7, 3), (2160, 48)])
def test_shard_tails_are_each_shards_last_rows(lib, H, tail):
    """rtk_shard_whole_rows: for every partition of the frame into N row
    interleaved shards (rows k, k + N, ...), a shard's whole rows are exactly
    its rows above the frame's tail and come first, so the shards' whole rows
    together are the frame's H - tail rows and each shard ends on tail rows."""
    f = lib.rtk_shard_whole_rows
    f.restype = ctypes.c_uint32
    f.argtypes = [ctypes.c_uint32] * 5
    for n in (1, 2, 3, 4, 7, 8):
        total = 0
        for k in range(n):
            rows = len(range(k, H, n))
            w = f(H, tail, k, n, rows)
            img = [k + r * n for r in range(rows)]
            assert all(y < H - tail for y in img[:w]) and all(y >= H - tail for y in img[w:])
            total += w
        assert total == H - tail


def _split(lib, W, H, S, parts, parts2, budget, permille, fine_permille):
    f = lib.rtk_tail_split
    f.restype = None
    f.argtypes = [ctypes.c_uint32] * 5 + [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                          ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32)]
    t, fi = ctypes.c_uint32(), ctypes.c_uint32()
    f(W, H, S, parts, parts2, budget, permille, fine_permille, ctypes.byref(t), ctypes.byref(fi))
    return t.value, fi.value


@pytest.mark.parametrize("W,H,S", [(1920, 1080, 22), (800, 800, 32), (1920, 1080, 16), (3840, 2160, 64),
                                   (16, 9, 4), (1920, 1080, 100)])
@pytest.mark.parametrize("budget", [GiB // 4, 4 * GiB, 1 << 62])
def test_fine_rows_are_the_last_rows_of_the_tail(lib, W, H, S, budget):
    """rtk_tail_split: the fine rows (parts of ~1 sample) are the frame's last
    rows, inside the tail (fine <= tail <= H), about the asked shares, their
    extra part sums within half the budget and the whole split's within the
    budget and the 2^32 queue; with no finer parts asked it is rtk_tail_rows."""
    p, p2 = lib.rtk_row_parts(S, 4), lib.rtk_row_parts(S, 1)
    t, fi = _split(lib, W, H, S, p, p2, budget, 500, 30)
    assert fi <= t <= H
    assert fi <= -(-H * 30 // 1000)
    if p2 > p:
        assert fi * W * S * (p2 - 1) * 24 <= budget // 2
    extra = fi * W * S * (p2 - 1) + (t - fi) * W * S * (p - 1)
    assert extra * 24 <= budget
    assert W * H * S + extra < 0xFFF00000
    if budget == 1 << 62 and p > 1 and W * H * S * p2 < 0xFFF00000 // 2:
        assert fi == -(-H * 30 // 1000) and t == max(fi, -(-H * 500 // 1000))
    # no finer parts: the old tail, no fine rows
    t0, f0 = _split(lib, W, H, S, p, p, budget, 500, 30)
    assert f0 == 0 and t0 == lib.rtk_tail_rows(W, H, S, p, budget, 500)
    # C4 (1920 x 1080 at 16^2, 4 GiB): 33 fine rows of 16 one-sample parts
    if (W, H, S, budget) == (1920, 1080, 16, 4 * GiB):
        assert (t, fi) == (540, 33)
