"""ImageTexture's PNG decoding (raytracer-2025_amd/csrc/rt_png.hpp, shared by
the library's loaders and the oracle) against PIL: the `image` crate's
into_rgba32f (8-bit v / 255, 16-bit v / 65535, gray -> (g, g, g), palette +
tRNS -> RGBA) on the reference's own PNG assets read in place (4-bit palette,
8-bit gray, RGB, RGBA) and on synthetic files of every color type / bit depth
PIL writes; then palette's sRGB EOTF in f32 (utils/image.rs:63-82) against
the formula in numpy.  Interlaced (Adam7) files are written by the test
itself (PIL reads them but does not write them) with every filter type.  A
missing file is Image::EMPTY; a JPEG goes to the library's JPEG decoder
(tests/test_jpeg_cpu.py), the oracle refuses it."""
import struct
import zlib
import os
import subprocess

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
BUILD = os.path.join(HERE, "_build")
REF_ASSETS = "/root/reference/assets/Final"

PIL = pytest.importorskip("PIL.Image")


@pytest.fixture(scope="module", params=["product", "oracle"])
def dump(request):
    """The library's decoder (rt_png.hpp) and, independently written, the
    oracle's (oracle/orc_png.hpp): both against PIL."""
    os.makedirs(BUILD, exist_ok=True)
    exe = os.path.join(BUILD, "png_dump_%s.%d" % (request.param, os.getpid()))  # one per pytest worker
    flags = ["-DORACLE_PNG"] if request.param == "oracle" else []
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", *flags, os.path.join(HERE, "cpp", "png_dump.cpp"),
                    "-o", exe, "-lz"], check=True)

    def run(path, raw, tmp):
        out = os.path.join(str(tmp), "dump.bin")
        r = subprocess.run([exe, path, out, "1" if raw else "0"], capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr
        with open(out, "rb") as f:
            st, w, h = map(int, f.readline().split())
            px = np.frombuffer(f.read(), dtype=np.float32)
        return st, px.reshape(h, w, 4) if st == 0 else None
    run.kind = request.param
    return run


def pil_rgba01(path):
    im = PIL.open(path)
    if im.mode in ("I;16", "I;16B", "I"):
        a = np.asarray(im, dtype=np.float32) / 65535.0
        return np.stack([a, a, a, np.ones_like(a)], axis=-1)
    return np.asarray(im.convert("RGBA"), dtype=np.float32) / 255.0


def srgb_to_linear(x):
    x = x.astype(np.float32)
    return np.where(x <= np.float32(0.04045), x / np.float32(12.92),
                    np.power((x + np.float32(0.055)) / np.float32(1.055), np.float32(2.4))).astype(np.float32)


@pytest.mark.parametrize("name", ["diamond_ore.png", "diamond_pickaxe.png", "stone.png", "torch.png", "flame.png",
                                  "门_框_Metallic.png"])
def test_reference_assets_match_pil(dump, tmp_path, name):
    path = os.path.join(REF_ASSETS, name)
    if not os.path.exists(path):
        pytest.skip("reference assets not mounted")
    st, px = dump(path, True, tmp_path)
    assert st == 0
    ref = pil_rgba01(path)
    assert px.shape == ref.shape
    np.testing.assert_array_equal(px, ref)
    st, lin = dump(path, False, tmp_path)
    np.testing.assert_allclose(lin[..., :3], srgb_to_linear(ref[..., :3]), rtol=2e-6, atol=1e-7)
    np.testing.assert_array_equal(lin[..., 3], ref[..., 3])


@pytest.mark.parametrize("mode", ["L", "LA", "RGB", "RGBA", "P", "P_trns", "1", "I;16"])
def test_synthetic_modes_match_pil(dump, tmp_path, mode):
    rng = np.random.default_rng(len(mode))
    h, w = 23, 37  # odd sizes: sub-byte rows, every filter type PIL picks
    if mode in ("L", "LA", "RGB", "RGBA"):
        ch = {"L": 1, "LA": 2, "RGB": 3, "RGBA": 4}[mode]
        a = rng.integers(0, 256, size=(h, w, ch), dtype=np.uint8)
        a[: h // 2] = (np.arange(w)[None, :, None] * 7 % 256).astype(np.uint8)  # smooth half: Sub/Up/Paeth rows
        im = PIL.fromarray(a[..., 0] if ch == 1 else a, mode)
    elif mode.startswith("P"):
        im = PIL.fromarray(rng.integers(0, 200, size=(h, w, 3), dtype=np.uint8), "RGB").quantize(colors=13)
        if mode == "P_trns":
            im.info["transparency"] = 3
    elif mode == "1":
        im = PIL.fromarray((rng.random((h, w)) > 0.5).astype(np.uint8) * 255, "L").convert("1")
    else:
        im = PIL.fromarray(rng.integers(0, 65536, size=(h, w), dtype=np.uint16))  # mode I;16
    path = str(tmp_path / f"m_{mode.replace(';', '')}.png")
    kw = {"transparency": 3} if mode == "P_trns" else {}
    im.save(path, **kw)
    st, px = dump(path, True, tmp_path)
    assert st == 0
    ref = pil_rgba01(path)
    np.testing.assert_array_equal(px, ref)


def test_missing_and_unsupported(dump, tmp_path):
    st, _ = dump(str(tmp_path / "absent.png"), False, tmp_path)
    assert st == 1  # Image::EMPTY -> cyan
    (tmp_path / "broken.png").write_bytes(b"\x89PNG\r\n\x1a\n" + b"\x00" * 40)
    assert dump(str(tmp_path / "broken.png"), False, tmp_path)[0] == 1  # decode error -> EMPTY, as the reference
    PIL.new("RGB", (8, 8)).save(str(tmp_path / "x.jpg"))
    # the library decodes JPEG (rt_jpeg.hpp); the oracle's reader refuses it
    assert dump(str(tmp_path / "x.jpg"), False, tmp_path)[0] == (0 if dump.kind == "product" else 3)


ADAM7 = [(0, 0, 8, 8), (4, 0, 8, 8), (0, 4, 4, 8), (2, 0, 4, 4), (0, 2, 2, 4), (1, 0, 2, 2), (0, 1, 1, 2)]


def _pack_row(samples, depth):
    """One scanline's samples (uint array) packed at `depth` bits, big-endian."""
    if depth == 16:
        return samples.astype(">u2").tobytes()
    if depth == 8:
        return samples.astype(np.uint8).tobytes()
    bits = np.zeros(len(samples) * depth, dtype=np.uint8)
    for b in range(depth):
        bits[b::depth] = (samples >> (depth - 1 - b)) & 1
    return np.packbits(bits).tobytes()


def _filter(row, prev, bpp, ft):
    out = bytearray(len(row))
    for i in range(len(row)):
        a = row[i - bpp] if i >= bpp else 0
        b = prev[i] if prev is not None else 0
        c = prev[i - bpp] if (prev is not None and i >= bpp) else 0
        if ft == 0:
            pred = 0
        elif ft == 1:
            pred = a
        elif ft == 2:
            pred = b
        elif ft == 3:
            pred = (a + b) >> 1
        else:
            p = a + b - c
            pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
            pred = a if (pa <= pb and pa <= pc) else (b if pb <= pc else c)
        out[i] = (row[i] - pred) & 255
    return bytes(out)


def write_adam7_png(path, img, ctype, depth, rng, plte=None):
    """img: (h, w, channels) uint array; every pass row gets a random filter type."""
    h, w, ch = img.shape
    bpp = max(1, ch * depth // 8)
    data = bytearray()
    for x0, y0, dx, dy in ADAM7:
        sub = img[y0::dy, x0::dx]
        if sub.shape[0] == 0 or sub.shape[1] == 0:
            continue
        prev = None
        for r in sub:
            row = _pack_row(r.reshape(-1), depth)
            ft = int(rng.integers(0, 5))
            data += bytes([ft]) + _filter(row, prev, bpp, ft)
            prev = row

    def chunk(t, d):
        return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xffffffff)
    png = b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, depth, ctype, 0, 0, 1))
    if plte is not None:
        png += chunk(b"PLTE", plte)
    png += chunk(b"IDAT", zlib.compress(bytes(data))) + chunk(b"IEND", b"")
    with open(path, "wb") as f:
        f.write(png)


@pytest.mark.parametrize("kind", ["rgb8", "rgba16", "gray1", "gray4", "gray16", "palette2", "la8"])
@pytest.mark.parametrize("size", [(1, 1), (5, 3), (9, 9), (37, 23)])
def test_interlaced_adam7_matches_pil(dump, tmp_path, kind, size):
    """Adam7 (PNG 1.2 section 8): seven sub-images, each its own filtered
    scanlines, scattered back onto the grid -- against PIL's decoding."""
    rng = np.random.default_rng(sum(map(ord, kind)) + size[0])
    w, h = size
    ctype, depth, ch = {"rgb8": (2, 8, 3), "rgba16": (6, 16, 4), "gray1": (0, 1, 1), "gray4": (0, 4, 1),
                        "gray16": (0, 16, 1), "palette2": (3, 2, 1), "la8": (4, 8, 2)}[kind]
    img = rng.integers(0, 1 << depth, size=(h, w, ch), dtype=np.uint32)
    plte = bytes(rng.integers(0, 256, size=12, dtype=np.uint8)) if ctype == 3 else None
    path = str(tmp_path / f"a7_{kind}.png")
    write_adam7_png(path, img, ctype, depth, rng, plte)
    st, px = dump(path, True, tmp_path)
    assert st == 0
    if depth == 16 and ctype in (2, 4, 6):
        # PIL keeps 8 bits of 16-bit color; into_rgba32f is v / 65535: check
        # the grid against PIL's high bytes and the values against the samples
        np.testing.assert_array_equal(np.round(px * 65535).astype(np.uint32) >> 8,
                                      np.round(pil_rgba01(path) * 255).astype(np.uint32))
        exp = img.astype(np.float32) / np.float32(65535)
        if ch == 4:
            np.testing.assert_array_equal(px, exp)
    else:
        np.testing.assert_array_equal(px, pil_rgba01(path))
