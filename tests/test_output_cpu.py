"""Output stage on CPU: rt_write_png (main.rs:39-47
img.save + create_dir_all) decoded back with Python's zlib, and
rt_camera_from_json (camera.rs:119-159) against Python's json on a synthetic
file and, when present, the reference's own assets/Final/camera.json."""
import ctypes
import json
import os
import struct
import zlib

import numpy as np
import pytest


def read_png(path):
    data = open(path, "rb").read()
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    pos, idat, ihdr = 8, b"", None
    while pos < len(data):
        n, typ = struct.unpack(">I4s", data[pos:pos + 8])
        body = data[pos + 8:pos + 8 + n]
        crc, = struct.unpack(">I", data[pos + 8 + n:pos + 12 + n])
        assert zlib.crc32(typ + body) & 0xFFFFFFFF == crc
        if typ == b"IHDR":
            ihdr = struct.unpack(">IIBBBBB", body)
        elif typ == b"IDAT":
            idat += body
        pos += 12 + n
    w, h, depth, ctype, _, _, _ = ihdr
    assert (depth, ctype) == (8, 2)
    raw = zlib.decompress(idat)
    rows = [raw[y * (1 + 3 * w) + 1:(y + 1) * (1 + 3 * w)] for y in range(h)]
    assert all(raw[y * (1 + 3 * w)] == 0 for y in range(h))
    return np.frombuffer(b"".join(rows), dtype=np.uint8).reshape(h, w, 3)


@pytest.mark.parametrize("w,h", [(1, 1), (7, 3), (300, 250)])  # 300x250x3 > one 64 KiB stored block
def test_png_roundtrip(product, rt, tmp_path, w, h):
    img = np.random.default_rng(w * h).integers(0, 256, (h, w, 3), dtype=np.uint8)
    path = tmp_path / "output" / "final" / "final.png"  # parents created (main.rs:42-43)
    rt.save_png(product, str(path), img)
    np.testing.assert_array_equal(read_png(str(path)), img)


def test_png_errors(product, capi, tmp_path):
    assert product.write_png(str(tmp_path / "x.png").encode(), 0, 1, None) == -1
    (tmp_path / "file").write_text("")
    rc = product.write_png(str(tmp_path / "file" / "x.png").encode(), 1, 1, (ctypes.c_uint8 * 3)())
    assert rc == -1  # "Cannot create all the parents"


CAM = {"aspect_ratio": 1.7777777777777777, "image_width": 1920, "vertical_fov_in_degrees": 23,
       "look_from": [1.842332124710083, 1.9965558052062988, 9.644098281860352],
       "look_at": [1.6544842720031738, 1.9639147520065308, 8.662442207336426],
       "vec_up": [-0.014803536236286163, 0.9994282126426697, -0.030399203300476074],
       "defocus_angle_in_degrees": 0.0, "focus_distance": 1.0000004646134415}


def check_camera(cam, d):
    assert cam.aspect_ratio == d["aspect_ratio"] and cam.image_width == d["image_width"]
    assert cam.vertical_fov_in_degrees == d["vertical_fov_in_degrees"]
    for k in ("look_from", "look_at", "vec_up"):
        assert list(getattr(cam, k)) == d[k]
    assert cam.defocus_angle_in_degrees == d["defocus_angle_in_degrees"]
    assert cam.focus_distance == d["focus_distance"]
    # everything else is Camera::default (camera.rs:76-104)
    assert cam.samples_per_pixel == 10 and cam.max_depth == 10 and cam.background is None and cam.toon_map == 0


def test_camera_from_json(product, rt, tmp_path):
    p = tmp_path / "camera.json"
    p.write_text(json.dumps(dict(CAM, extra={"ignored": [1, 2, {"x": None}]}), indent=2))
    check_camera(rt.Camera.from_json(product, str(p)), CAM)


@pytest.mark.parametrize("edit", [
    lambda d: d.pop("focus_distance"),
    lambda d: d.__setitem__("image_width", 19.5),
    lambda d: d.__setitem__("image_width", -1),
    lambda d: d.__setitem__("look_at", [1, 2]),
])
def test_camera_from_json_errors(product, rt, capi, tmp_path, edit):
    d = json.loads(json.dumps(CAM))
    edit(d)
    p = tmp_path / "bad.json"
    p.write_text(json.dumps(d))
    with pytest.raises(capi.RtError) as e:
        rt.Camera.from_json(product, str(p))
    assert e.value.code == -1


REF_CAMERA = "/root/reference/assets/Final/camera.json"


@pytest.mark.skipif(not os.path.exists(REF_CAMERA), reason="reference assets not present (GPU box)")
def test_reference_camera_json(product, rt):
    """The reference's own camera file (read in place), against Python's json."""
    check_camera(rt.Camera.from_json(product, REF_CAMERA), json.load(open(REF_CAMERA)))
