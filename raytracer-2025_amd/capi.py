"""ctypes declarations of the C ABI in include/rt_mi355x.h.

`bind(lib, prefix)` attaches argtypes/restype for every entry point of a loaded
library whose symbols are `<prefix><name>` (prefix "rt_" for librt_mi355x.so).
The same declarations serve the test-only oracle (prefix "orc_"), which the
tests load themselves; this package never loads it.
"""
import ctypes as C

c_double3 = C.c_double * 3
c_double4 = C.c_double * 4


class RtCamera(C.Structure):
    """rt_camera -- Camera pub fields (src/camera.rs:45-61)."""

    _fields_ = [
        ("aspect_ratio", C.c_double),
        ("image_width", C.c_uint32),
        ("samples_per_pixel", C.c_uint32),
        ("max_depth", C.c_uint32),
        ("background_tex", C.c_int32),
        ("vertical_fov_in_degrees", C.c_double),
        ("look_from", c_double3),
        ("look_at", c_double3),
        ("vec_up", c_double3),
        ("defocus_angle_in_degrees", C.c_double),
        ("focus_distance", C.c_double),
        ("toon_map", C.c_int32),
        ("reserved", C.c_int32),
    ]


class RtWorldInfo(C.Structure):
    _fields_ = [
        ("device_bytes", C.c_uint64),
        ("bvh_nodes", C.c_uint32),
        ("primitives", C.c_uint32),
        ("bvh_leaves", C.c_uint32),
        ("stack_need", C.c_uint32),
        ("kernel_tier", C.c_uint32),
        ("features", C.c_uint32),
    ]


class RtRenderOpts(C.Structure):
    _fields_ = [
        ("struct_size", C.c_uint32),
        ("reserved0", C.c_uint32),
        ("seed", C.c_uint64),
        ("row_offset", C.c_uint32),
        ("row_stride", C.c_uint32),
        ("threads", C.c_uint32),
        ("flags", C.c_uint32),
        ("stream", C.c_void_p),
        ("n_devices", C.c_uint32),
        ("reserved", C.c_uint32),
        ("devices", C.POINTER(C.c_int32)),
        ("comm", C.c_void_p),
    ]


class RtStats(C.Structure):
    _fields_ = [
        ("samples", C.c_uint64),
        ("rays", C.c_uint64),
        ("panics", C.c_uint64),
        ("n_devices", C.c_uint64),
        ("render_ms", C.c_double),
        ("kernel_ms", C.c_double),
        ("flatten_ms", C.c_double),
        ("gather_ms", C.c_double),
    ]


_P = C.c_void_p
_I = C.c_int32
_U = C.c_uint32
_D = C.c_double
_DP = C.POINTER(C.c_double)

# name -> (restype, argtypes); the exact list include/rt_mi355x.h declares.
SIGNATURES = {
    "abi_version": (_I, []),
    "last_error": (C.c_char_p, []),
    "scene_create": (_P, []),
    "scene_destroy": (None, [_P]),
    "tex_solid": (_I, [_P, _DP]),
    "tex_checker": (_I, [_P, _D, _I, _I]),
    "tex_image": (_I, [_P, _U, _U, C.POINTER(C.c_float), _I]),
    "tex_image_file": (_I, [_P, C.c_char_p, _I, _I]),
    "tex_noise": (_I, [_P, _D, C.c_uint64]),
    "tex_sky_gradient": (_I, [_P, _DP, _DP]),
    "mat_empty": (_I, [_P]),
    "mat_lambertian": (_I, [_P, _I]),
    "mat_metal": (_I, [_P, _DP, _D]),
    "mat_dielectric": (_I, [_P, _I, _D]),
    "mat_diffuse_light": (_I, [_P, _I, _I]),
    "mat_isotropic": (_I, [_P, _I]),
    "mat_transparent": (_I, [_P]),
    "mat_mix": (_I, [_P, _I, _I, _D]),
    "mat_mix_image": (_I, [_P, _I, _I, _I]),
    "sphere": (_I, [_P, _DP, _D, _I]),
    "sphere_moving": (_I, [_P, _DP, _DP, _D, _I]),
    "quad": (_I, [_P, _DP, _DP, _DP, _I]),
    "triangle": (_I, [_P, _DP, _DP, _DP, _I]),
    "hittables_new": (_I, [_P]),
    "hittables_add": (_I, [_P, _I, _I]),
    "bvh_new": (_I, [_P, _I]),
    "build_box": (_I, [_P, _DP, _DP, _I]),
    "transform_new": (_I, [_P, _I, _DP, _DP, _DP]),
    "constant_medium_new": (_I, [_P, _I, _D, _I]),
    "wavefront_load": (_I, [_P, C.c_char_p, _I]),
    "quat_from_axis_angle": (_I, [_DP, _D, _DP]),
    "quat_from_euler": (None, [_D, _D, _D, _DP]),
    "camera_default": (None, [C.POINTER(RtCamera)]),
    "camera_image_height": (_U, [C.POINTER(RtCamera)]),
    "render_opts_default": (None, [C.POINTER(RtRenderOpts)]),
    "render": (_I, [_P, _I, _I, C.POINTER(RtCamera), C.POINTER(RtRenderOpts), C.POINTER(C.c_float),
                    C.POINTER(C.c_uint8), C.POINTER(RtStats)]),
    "shard_rows": (_U, [C.POINTER(RtCamera), C.POINTER(RtRenderOpts)]),
    "render_device": (_I, [_P, _I, _I, C.POINTER(RtCamera), C.POINTER(RtRenderOpts), _P]),
    "render_device_wait": (_I, [_P, C.POINTER(RtStats)]),
    "render_gather_mode": (_I, [_P]),
    "to_rgb_device": (_I, [_P, _P, C.c_uint64, _I, _P]),
    "write_png": (_I, [C.c_char_p, C.c_uint32, C.c_uint32, _P]),
    "camera_from_json": (_I, [C.c_char_p, C.POINTER(RtCamera)]),
    "world_info_get": (_I, [_P, _I, _I, _I, _U, C.POINTER(RtWorldInfo)]),
    "render_partials_get": (_I, [_P, _DP, C.c_uint64]),
    "math_selftest": (_I, [_I, _I, _DP, _DP, _DP, C.c_uint64]),
    "bvh_selftest": (_I, [_P, _I]),
    "world_selftest": (_I, [_P, _I, _I, _I]),
    "comm_unique_id": (_I, [C.POINTER(C.c_uint8)]),
    "comm_init": (_P, [C.POINTER(C.c_uint8), _I, _I]),
    "comm_destroy": (None, [_P]),
}

# Entry points of the product library only (the oracle renders on host cores
# and has no communicator, device-side partial sums or parallel builders).
GPU_ONLY = ("render_gather_mode", "render_partials_get", "math_selftest", "bvh_selftest", "world_selftest", "comm_unique_id", "comm_init", "comm_destroy")

# Entry points only a CPU implementation has (the oracle).
ORACLE_EXTRAS = {
    # the f64 per-(pixel, stratum row) sums, [rows x W][sqrt_spp][3] (as rt_render_partials_get)
    "render_partials": (_I, [_P, _I, _I, C.POINTER(RtCamera), C.POINTER(RtRenderOpts), _DP, C.POINTER(RtStats)]),
    "render_f64": (_I, [_P, _I, _I, C.POINTER(RtCamera), C.POINTER(RtRenderOpts), _DP, C.POINTER(C.c_uint8),
                        C.POINTER(RtStats), C.POINTER(C.c_uint64)]),
    "work_count_fields": (_U, []),
}

STATUS = {
    0: "RT_OK", -1: "RT_EINVAL", -2: "RT_EHANDLE", -3: "RT_EMOVED", -4: "RT_EDEGENERATE",
    -5: "RT_EPANIC", -6: "RT_EUNSUPPORTED", -7: "RT_EDEVICE", -8: "RT_ENOMEM", -9: "RT_ESTACK",
}


class RtError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"{STATUS.get(code, code)}: {msg}")
        self.code = code


class Api:
    """Typed view of one loaded implementation of the ABI."""

    def __init__(self, lib, prefix, extras=None):
        self.lib = lib
        self.prefix = prefix
        sigs = dict(SIGNATURES)
        sigs.update(extras or {})
        self.missing = []
        for name, (res, args) in sigs.items():
            try:
                fn = getattr(lib, prefix + name)
            except AttributeError:
                self.missing.append(prefix + name)
                continue
            fn.restype = res
            fn.argtypes = args
            setattr(self, name, fn)

    def check(self, rc):
        if rc is not None and rc < 0:
            err = self.last_error()
            raise RtError(rc, err.decode() if err else "")
        return rc


def d3(v):
    return c_double3(*[float(x) for x in v])


def d4(v):
    return c_double4(*[float(x) for x in v])
