"""Multi-GPU through the C ABI on the one-GPU box.

The library splits a render into parts -- part k of n renders the shard rows
k, k + n, ... (camera.rs:178-197's rayon pool, replaced) -- and gathers them
onto the root: RCCL send/recv in one group between distinct devices (and with
a communicator from rt_comm_init, one process per GPU), peer copies when a
device is listed twice.  On one GPU the device list {0, 0} exercises the
host-thread split, the per-slot device worlds and the re-interleave; a
one-rank communicator exercises the RCCL group (send to self, receive on the
root) and the gather events.  Every multi-part frame must equal the
single-device frame bit for bit (the same (pixel, sample) work, another
device)."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _scene(rt, scenes, api, width=64, spp=4):
    s = rt.Scene(api)
    world, lights, cam = scenes.random_spheres(s, width, spp)
    return s, world, lights, cam


@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 0, 0]])
def test_device_list_equals_single_device(gpu, rt, scenes, devices):
    s, world, lights, cam = _scene(rt, scenes, gpu, 70, 9)  # 39 rows: parts of 13 / 13 / 13 and 20 / 19
    ref, ref_srgb, st0 = cam.render(world, lights, seed=4)
    lin, srgb, st = cam.render(world, lights, seed=4, devices=devices)
    np.testing.assert_array_equal(lin, ref)
    # each part's to_rgb bytes come from its f64 pixel sums (color.rs:27-36),
    # gathered beside the f32 rows: the 8-bit image does not depend on the
    # device count either
    np.testing.assert_array_equal(srgb, ref_srgb)
    assert st.samples == st0.samples and st.panics == 0
    assert st.n_devices == max(1, len(devices))
    if len(devices) > 1:
        assert st.gather_ms > 0
    else:
        assert st.gather_ms == 0


def test_device_list_with_shard(gpu, rt, scenes):
    """A shard (row_offset 1, row_stride 3) split again over two parts."""
    s, world, lights, cam = _scene(rt, scenes, gpu, 64, 4)
    ref, _, _ = cam.render(world, lights, seed=2, row_offset=1, row_stride=3, want_srgb=False)
    lin, _, st = cam.render(world, lights, seed=2, row_offset=1, row_stride=3, want_srgb=False, devices=[0, 0])
    np.testing.assert_array_equal(lin, ref)
    assert st.n_devices == 2


def test_more_parts_than_rows(gpu, rt, scenes):
    s, world, lights, cam = _scene(rt, scenes, gpu, 8, 1)  # 4 rows, 5 parts: part 4 renders nothing
    ref, _, _ = cam.render(world, lights, seed=3, want_srgb=False)
    lin, _, _ = cam.render(world, lights, seed=3, want_srgb=False, devices=[0, 0, 0, 0, 0])
    np.testing.assert_array_equal(lin, ref)


def test_one_rank_communicator(gpu, rt, scenes, capi):
    """rt_comm_unique_id / rt_comm_init / an RCCL gather of one rank onto itself."""
    s, world, lights, cam = _scene(rt, scenes, gpu, 64, 4)
    ref, _, _ = cam.render(world, lights, seed=5, want_srgb=False)
    uid = (ctypes.c_uint8 * 128)()
    gpu.check(gpu.comm_unique_id(uid))
    comm = gpu.comm_init(uid, 1, 0)
    assert comm, gpu.last_error()
    try:
        lin, _, st = cam.render(world, lights, seed=5, want_srgb=False, comm=comm)
        np.testing.assert_array_equal(lin, ref)
        assert st.n_devices == 1 and st.gather_ms > 0
        ref2, ref_srgb, _ = cam.render(world, lights, seed=5)
        lin3, srgb3, _ = cam.render(world, lights, seed=5, comm=comm)  # the to_rgb bytes gathered too
        np.testing.assert_array_equal(lin3, ref2)
        np.testing.assert_array_equal(srgb3, ref_srgb)
        lin2, _, _ = cam.render(world, lights, seed=5, want_srgb=False, comm=comm)  # the communicator is reusable
        np.testing.assert_array_equal(lin2, ref)
    finally:
        gpu.comm_destroy(comm)


def test_comm_and_devices_are_exclusive(gpu, rt, scenes, capi):
    s, world, lights, cam = _scene(rt, scenes, gpu, 16, 1)
    uid = (ctypes.c_uint8 * 128)()
    gpu.check(gpu.comm_unique_id(uid))
    comm = gpu.comm_init(uid, 1, 0)
    try:
        with pytest.raises(capi.RtError) as e:
            cam.render(world, lights, comm=comm, devices=[0, 0])
        assert e.value.code == -1
    finally:
        gpu.comm_destroy(comm)


def test_render_device_calls_are_ordered(gpu, rt, scenes, capi):
    """Two rt_render_device calls on one scene, on two streams, without a wait
    between them: the second's kernels wait for the first's (they share the
    scene's work buffers), so both frames are right."""
    import torch

    s, world, lights, cam = _scene(rt, scenes, gpu, 96, 16)
    ref_a, _, _ = cam.render(world, lights, seed=21, want_srgb=False)
    ref_b, _, _ = cam.render(world, lights, seed=22, want_srgb=False)
    c = cam.to_c()
    outs, streams = [], [torch.cuda.Stream(), torch.cuda.Stream()]
    for seed, st in zip((21, 22), streams):
        opts = capi.RtRenderOpts()
        gpu.render_opts_default(ctypes.byref(opts))
        opts.seed = seed
        opts.stream = ctypes.c_void_p(st.cuda_stream)
        out = torch.empty((cam.image_height, cam.image_width, 3), dtype=torch.float32, device="cuda")
        gpu.check(gpu.render_device(s.s, world.h, -1, ctypes.byref(c), ctypes.byref(opts),
                                    ctypes.c_void_p(out.data_ptr())))
        outs.append(out)
    stt = capi.RtStats()
    gpu.check(gpu.render_device_wait(s.s, ctypes.byref(stt)))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(outs[0].cpu().numpy(), ref_a)
    np.testing.assert_array_equal(outs[1].cpu().numpy(), ref_b)


def test_render_device_on_device_list(gpu, rt, scenes, capi):
    """rt_render_device with a device list: the frame lands in the caller's buffer on devices[0]."""
    import torch

    s, world, lights, cam = _scene(rt, scenes, gpu, 64, 4)
    ref, _, _ = cam.render(world, lights, seed=8, want_srgb=False)
    c = cam.to_c()
    opts, keep = rt.Camera._opts(gpu, 8, 0, 1, 0, 0, devices=[0, 0])
    out = torch.zeros((cam.image_height, cam.image_width, 3), dtype=torch.float32, device="cuda")
    opts.stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    gpu.check(gpu.render_device(s.s, world.h, -1, ctypes.byref(c), ctypes.byref(opts), ctypes.c_void_p(out.data_ptr())))
    st = capi.RtStats()
    gpu.check(gpu.render_device_wait(s.s, ctypes.byref(st)))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out.cpu().numpy(), ref)
    assert st.n_devices == 2


def test_two_threads_share_a_communicator(gpu, rt, scenes):
    """Two scenes rendered at once from two host threads, both gathering
    through one rt_comm: each gather's RCCL group is enqueued whole under the
    communicator's lock, so every frame is its own scene's, bit-equal to a
    render on one thread (ctypes releases the GIL inside the library)."""
    import threading

    jobs = [_scene(rt, scenes, gpu, 80, 9), _scene(rt, scenes, gpu, 72, 4)]
    refs = [cam.render(world, lights, seed=30 + k, want_srgb=False)[0] for k, (s, world, lights, cam) in enumerate(jobs)]
    uid = (ctypes.c_uint8 * 128)()
    gpu.check(gpu.comm_unique_id(uid))
    comm = gpu.comm_init(uid, 1, 0)
    assert comm, gpu.last_error()
    errors, frames = [], [[], []]

    def worker(k):
        try:
            s, world, lights, cam = jobs[k]
            for _ in range(6):
                frames[k].append(cam.render(world, lights, seed=30 + k, want_srgb=False, comm=comm)[0])
        except Exception as e:  # reported below, on the test's thread
            errors.append(e)
    try:
        ts = [threading.Thread(target=worker, args=(k,)) for k in range(2)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(timeout=100)
        assert not any(t.is_alive() for t in ts), "a render thread hung"
        assert not errors, errors
        for k in range(2):
            assert len(frames[k]) == 6
            for f in frames[k]:
                np.testing.assert_array_equal(f, refs[k])
    finally:
        gpu.comm_destroy(comm)

