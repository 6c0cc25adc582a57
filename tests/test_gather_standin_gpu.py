"""The nranks > 1 framebuffer gathers on the one-GPU box (SURVEY §8e,
DESIGN §7), through a test-only RCCL stand-in.

librt_mi355x.so gathers the row parts of an N-GPU render onto the root with
one ncclSend / ncclRecv group (rt_render.cpp launch): with a communicator per
process (rt_comm_init -> ncclCommInitRank), or with ncclCommInitAll
communicators over an in-process device list.  Real RCCL refuses two ranks on
one device, so with one GPU neither branch could run with more than one rank.
tests/cpp/fake_rccl.cpp implements librccl's point-to-point subset with
hipMemcpyPeerAsync (any number of ranks per device, RCCL's matching and stream
order, byte counts checked per pair).  Only the CHECK build
(librt_mi355x_check.so: the same host code and kernels, plus bounds checks)
loads it, when RT_RCCL_LIB names it -- the product library opens librccl and
nothing else:

* the communicator branch: N host threads, one rank and one scene each, all
  on device 0 (camera.rs:178-197's rayon pool, replaced by row shards + the
  gather);
* the device-list branch: RT_CHECK_RCCL_DUPS=1 sends a repeated device list
  through the RCCL group instead of the peer-copy fallback.

Every gathered frame -- the linear f32 rows and the to_rgb bytes -- must equal
the single-device frame bit for bit, for N = 2, 3 and 8 on a C2-style sphere
world (basic tier) and a C5-style final scene (full tier)."""
import ctypes
import os
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHECK_SO = os.path.join(ROOT, "raytracer-2025_amd", "librt_mi355x_check.so")


@pytest.fixture(scope="module")
def chk(capi, gpu):
    assert os.path.exists(CHECK_SO), "check build absent (__graft_entry__.build() makes it)"
    return capi.Api(ctypes.CDLL(CHECK_SO), "rt_")


@pytest.fixture(scope="module")
def standin(rccl_standin):
    return rccl_standin


def _world(rt, scenes, api, kind):
    s = rt.Scene(api)
    if kind == "spheres":  # C2's world and camera, basic tier
        world, lights, cam = scenes.random_spheres(s, 72, 9)
    else:  # C5's world, full tier
        world, lights, cam = scenes.final_scene(s, 64, 4, 8, aspect_ratio=16 / 9)
    return s, world, lights, cam


@pytest.mark.parametrize("kind", ["spheres", "final"])
@pytest.mark.parametrize("nranks", [2, 3, 8])
def test_communicator_ranks_gather_bit_equal(gpu, chk, rt, scenes, standin, monkeypatch, kind, nranks):
    """nranks threads, one rt_comm each (ncclCommInitRank through the
    stand-in), each rendering its rows r, r + n, ...; rank 0 receives the
    frame (f32 rows and sRGB bytes: a host-buffer render gathers both)."""
    so, counts = standin
    ref_s, ref_w, ref_l, ref_cam = _world(rt, scenes, gpu, kind)
    ref, ref_srgb, ref_st = ref_cam.render(ref_w, ref_l, seed=11)
    H, W = ref.shape[:2]
    monkeypatch.setenv("RT_RCCL_LIB", so)
    uid = (ctypes.c_uint8 * 128)()
    chk.check(chk.comm_unique_id(uid))
    jobs = [_world(rt, scenes, chk, kind) for _ in range(nranks)]
    comms, results, errors = [None] * nranks, [None] * nranks, []
    c0 = counts()

    def rank(r):
        try:
            comms[r] = chk.comm_init(uid, nranks, r)
            assert comms[r], chk.last_error()
            s, world, lights, cam = jobs[r]
            results[r] = cam.render(world, lights, seed=11, comm=comms[r])
            # the communicator (and the scene's slot buffers) serve a second frame
            lin2, _, _ = cam.render(world, lights, seed=11, want_srgb=False, comm=comms[r])
            if r == 0:
                np.testing.assert_array_equal(lin2, ref)
        except Exception as e:  # reported on the test's thread
            errors.append((r, e))
    ts = [threading.Thread(target=rank, args=(r,)) for r in range(nranks)]
    try:
        for t in ts:
            t.start()
        for t in ts:
            t.join(timeout=150)
        assert not any(t.is_alive() for t in ts), "a rank hung"
        assert not errors, errors
    finally:
        for c in comms:
            if c:
                chk.comm_destroy(c)
    lin, srgb, st = results[0]
    np.testing.assert_array_equal(lin, ref)
    np.testing.assert_array_equal(srgb, ref_srgb)
    assert st.n_devices == 1 and st.gather_ms > 0  # one device per rank (rt_stats)
    for r in range(1, nranks):  # only the root's buffers receive the frame
        assert not results[r][0].any() and not results[r][1].any()
    # each rank renders its own rows' samples
    assert sum(results[r][2].samples for r in range(nranks)) == ref_st.samples
    # every rank of a host-buffer render sends its f32 rows and its to_rgb
    # bytes (rt_render.cpp launch), in both frames: 4 copies per rank, the
    # frame twice in f32 and twice in u8
    copies, nbytes = counts()
    assert copies - c0[0] == 4 * nranks
    assert nbytes - c0[1] == H * W * 3 * (4 + 1) * 2


@pytest.mark.parametrize("kind", ["spheres", "final"])
@pytest.mark.parametrize("nranks", [2, 3, 8])
def test_device_list_rccl_branch_bit_equal(gpu, chk, capi, rt, scenes, standin, monkeypatch, kind, nranks):
    """The check build with RT_CHECK_RCCL_DUPS=1: devices = [0] * n goes
    through ncclCommInitAll and one send / receive group (the branch an
    8-GPU in-process render takes), not the peer-copy fallback."""
    so, counts = standin
    ref_s, ref_w, ref_l, ref_cam = _world(rt, scenes, gpu, kind)
    ref, ref_srgb, _ = ref_cam.render(ref_w, ref_l, seed=12)
    monkeypatch.setenv("RT_RCCL_LIB", so)
    monkeypatch.setenv("RT_CHECK_RCCL_DUPS", "1")
    s, world, lights, cam = _world(rt, scenes, chk, kind)
    c0 = counts()
    lin, srgb, st = cam.render(world, lights, seed=12, devices=[0] * nranks)
    np.testing.assert_array_equal(lin, ref)
    np.testing.assert_array_equal(srgb, ref_srgb)
    assert st.n_devices == nranks and st.gather_ms > 0
    copies, nbytes = counts()
    assert copies - c0[0] == 2 * nranks  # f32 rows and sRGB bytes of every part, through the stand-in
    assert nbytes - c0[1] == ref.size * 5
    # and a second frame on the cached communicator set, device-side output
    import torch
    c = cam.to_c()
    opts, keep = rt.Camera._opts(chk, 12, 0, 1, 0, 0, devices=[0] * nranks)
    out = torch.zeros(ref.shape, dtype=torch.float32, device="cuda")
    opts.stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    chk.check(chk.render_device(s.s, world.h, -1 if lights is None else lights.h, ctypes.byref(c), ctypes.byref(opts),
                                ctypes.c_void_p(out.data_ptr())))
    stt = capi.RtStats()
    chk.check(chk.render_device_wait(s.s, ctypes.byref(stt)))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out.cpu().numpy(), ref)
    assert counts()[0] - copies == nranks
