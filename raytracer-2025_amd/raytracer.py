"""Host-side mirror of the reference's scene API over the C ABI.

Names and argument meanings follow the Rust crate `raytracer`
(/root/reference/src): textures (texture.rs), materials (material.rs), shapes
(shapes/*.rs, bvh.rs, hits.rs, volume.rs), Quaternion (utils/quaternion.rs)
and Camera (camera.rs).  A `Scene` is one `rt_scene` on one implementation of
the ABI; the gfx950 library is the product, and tests may hand the same scene
script the test-only oracle to compare against.

    scene = Scene(api)
    ground = scene.Lambertian(scene.SolidColor((0.5, 0.5, 0.5)))
    world = scene.Hittables()
    world.add(scene.Sphere((0, -1000, 0), 1000, ground))
    cam = Camera(); cam.image_width = 400; ...
    img = cam.render(world, None)          # Camera::render, camera.rs:161
"""
import ctypes as C
import math
import os

import numpy as np

from .capi import Api, RtCamera, RtError, RtRenderOpts, RtStats, d3, d4


class Texture:
    def __init__(self, scene, h):
        self.scene, self.h = scene, h


class Material:
    def __init__(self, scene, h):
        self.scene, self.h = scene, h


class Hittable:
    """An owned object handle (Box<dyn Hittable>)."""

    def __init__(self, scene, h, kind):
        self.scene, self.h, self.kind = scene, h, kind


class Hittables(Hittable):
    """hits.rs:9-76 -- `add` moves the object in (hits.rs:27-30)."""

    def add(self, obj):
        self.scene.api.check(self.scene.api.hittables_add(self.scene.s, self.h, obj.h))


class Quaternion:
    """utils/quaternion.rs -- (w, x, y, z); constructors evaluated by the library."""

    def __init__(self, w=1.0, x=0.0, y=0.0, z=0.0):
        self.wxyz = (float(w), float(x), float(y), float(z))

    @staticmethod
    def identity():
        return Quaternion()

    @staticmethod
    def from_axis_angle(api, axis, angle_in_degrees):
        out = (C.c_double * 4)()
        api.check(api.quat_from_axis_angle(d3(axis), float(angle_in_degrees), out))
        return Quaternion(*out)

    @staticmethod
    def from_euler(api, yaw, pitch, roll):
        out = (C.c_double * 4)()
        api.quat_from_euler(float(yaw), float(pitch), float(roll), out)
        return Quaternion(*out)


class Scene:
    def __init__(self, api: Api):
        self.api = api
        self.s = api.scene_create()
        if not self.s:
            raise RtError(-8, "scene_create failed")

    def close(self):
        if self.s:
            self.api.scene_destroy(self.s)
            self.s = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _c(self, rc):
        return self.api.check(rc)

    # ---- textures (texture.rs)
    def SolidColor(self, rgb):
        return Texture(self, self._c(self.api.tex_solid(self.s, d3(rgb))))

    def CheckerTexture(self, scale, even, odd):
        return Texture(self, self._c(self.api.tex_checker(self.s, float(scale), even.h, odd.h)))

    def ImageTexture(self, rgba=None, linear_interp=False):
        """rgba: HxWx4 float32 linear, or None for a missing file (cyan)."""
        if rgba is None:
            return Texture(self, self._c(self.api.tex_image(self.s, 0, 0, None, int(linear_interp))))
        a = np.ascontiguousarray(rgba, dtype=np.float32)
        h, w = a.shape[:2]
        ptr = a.ctypes.data_as(C.POINTER(C.c_float))
        return Texture(self, self._c(self.api.tex_image(self.s, w, h, ptr, int(linear_interp))))

    def ImageTexture_file(self, path, raw=False, linear_interp=None):
        """ImageTexture::new(file) / new_raw_image(file) (texture.rs:82-97) with
        the path given directly; PNG, JPEG and Radiance HDR decoded by the
        library, the format taken from the extension (missing -> cyan)."""
        interp = raw if linear_interp is None else linear_interp
        return Texture(self, self._c(self.api.tex_image_file(self.s, os.fsencode(path), int(raw), int(interp))))

    def NoiseTexture(self, scale, seed=0):
        return Texture(self, self._c(self.api.tex_noise(self.s, float(scale), int(seed))))

    def SkyGradient(self, horizon=(1.0, 1.0, 1.0), zenith=(0.5, 0.7, 1.0)):
        return Texture(self, self._c(self.api.tex_sky_gradient(self.s, d3(horizon), d3(zenith))))

    # ---- materials (material.rs)
    def EmptyMaterial(self):
        return Material(self, self._c(self.api.mat_empty(self.s)))

    def Lambertian(self, tex):
        return Material(self, self._c(self.api.mat_lambertian(self.s, tex.h)))

    def Metal(self, albedo, fuzz):
        return Material(self, self._c(self.api.mat_metal(self.s, d3(albedo), float(fuzz))))

    def Dielectric(self, tex, refraction_index):
        return Material(self, self._c(self.api.mat_dielectric(self.s, tex.h, float(refraction_index))))

    def DiffuseLight(self, tex, material=None):
        return Material(self, self._c(self.api.mat_diffuse_light(self.s, tex.h, -1 if material is None else material.h)))

    def Isotropic(self, tex):
        return Material(self, self._c(self.api.mat_isotropic(self.s, tex.h)))

    def Transparent(self):
        return Material(self, self._c(self.api.mat_transparent(self.s)))

    def Mix(self, mat1, mat2, ratio):
        return Material(self, self._c(self.api.mat_mix(self.s, mat1.h, mat2.h, float(ratio))))

    def Mix_from_image(self, mat1, mat2, image_tex):
        """Mix::from_image (material.rs:235-247): ratio = the texture's alpha."""
        return Material(self, self._c(self.api.mat_mix_image(self.s, mat1.h, mat2.h, image_tex.h)))

    # ---- hittables
    def Sphere(self, center, radius, mat):
        return Hittable(self, self._c(self.api.sphere(self.s, d3(center), float(radius), mat.h)), "sphere")

    def Sphere_new_with_motion(self, center1, center2, radius, mat):
        return Hittable(self, self._c(self.api.sphere_moving(self.s, d3(center1), d3(center2), float(radius), mat.h)), "sphere")

    def Quad(self, anchor, u, v, mat):
        return Hittable(self, self._c(self.api.quad(self.s, d3(anchor), d3(u), d3(v), mat.h)), "quad")

    def Triangle(self, anchor, u, v, mat):
        """Triangle::new -> Option: None when degenerate (triangle.rs:29-31)."""
        rc = self.api.triangle(self.s, d3(anchor), d3(u), d3(v), mat.h)
        if rc == -4:
            return None
        return Hittable(self, self._c(rc), "triangle")

    def Hittables(self):
        return Hittables(self, self._c(self.api.hittables_new(self.s)), "list")

    def BVH(self, hittables):
        return Hittable(self, self._c(self.api.bvh_new(self.s, hittables.h)), "bvh")

    def build_box(self, a, b, mat):
        return Hittables(self, self._c(self.api.build_box(self.s, d3(a), d3(b), mat.h)), "list")

    def Transform(self, obj, offset=None, quaternion=None, scale=None):
        off = d3(offset) if offset is not None else None
        q = d4(quaternion.wxyz) if quaternion is not None else None
        sc = d3(scale) if scale is not None else None
        return Hittable(self, self._c(self.api.transform_new(self.s, obj.h, off, q, sc)), "transform")

    def ConstantMedium(self, boundary, density, tex):
        return Hittable(self, self._c(self.api.constant_medium_new(self.s, boundary.h, float(density), tex.h)), "medium")

    def Wavefont(self, obj_path, vanilla_material=True):
        """Wavefont::new (shapes/obj.rs:117-134); returns the Hittables of its
        per-model BVHs.  The reference's Option<Wavefont> is None when the OBJ
        cannot be opened: here that raises RtError(RT_EINVAL)."""
        rc = self.api.wavefront_load(self.s, os.fsencode(obj_path), 1 if vanilla_material else 0)
        return Hittables(self, self._c(rc), "list")


class Camera:
    """camera.rs:45-104 -- pub fields with Camera::default values."""

    def __init__(self):
        self.aspect_ratio = 1.0
        self.image_width = 100
        self.samples_per_pixel = 10
        self.max_depth = 10
        self.background = None  # Texture; None = SolidColor(BLACK)
        self.vertical_fov_in_degrees = 90.0
        self.look_from = (0.0, 0.0, 0.0)
        self.look_at = (0.0, 0.0, -1.0)
        self.vec_up = (0.0, 1.0, 0.0)
        self.defocus_angle_in_degrees = 0.0
        self.focus_distance = 10.0
        self.toon_map = 0  # ToonMap::None

    @staticmethod
    def from_json(api, path):
        """Camera::from_json (camera.rs:119-159): the CameraParams fields from a
        JSON file over Camera::default (path given directly)."""
        c = RtCamera()
        api.check(api.camera_from_json(os.fsencode(path), C.byref(c)))
        cam = Camera()
        cam.aspect_ratio = c.aspect_ratio
        cam.image_width = c.image_width
        cam.vertical_fov_in_degrees = c.vertical_fov_in_degrees
        cam.look_from = tuple(c.look_from)
        cam.look_at = tuple(c.look_at)
        cam.vec_up = tuple(c.vec_up)
        cam.defocus_angle_in_degrees = c.defocus_angle_in_degrees
        cam.focus_distance = c.focus_distance
        return cam

    def to_c(self):
        c = RtCamera()
        c.aspect_ratio = float(self.aspect_ratio)
        c.image_width = int(self.image_width)
        c.samples_per_pixel = int(self.samples_per_pixel)
        c.max_depth = int(self.max_depth)
        c.background_tex = -1 if self.background is None else self.background.h
        c.vertical_fov_in_degrees = float(self.vertical_fov_in_degrees)
        c.look_from = d3(self.look_from)
        c.look_at = d3(self.look_at)
        c.vec_up = d3(self.vec_up)
        c.defocus_angle_in_degrees = float(self.defocus_angle_in_degrees)
        c.focus_distance = float(self.focus_distance)
        c.toon_map = int(self.toon_map)
        return c

    @property
    def image_height(self):
        h = int(self.image_width / self.aspect_ratio)
        return max(h, 1)

    @property
    def sqrt_spp(self):
        return int(math.sqrt(self.samples_per_pixel))

    def traced_samples(self):
        """pixels x floor(sqrt(spp))^2 -- what camera.rs:183-192 traces."""
        return self.image_width * self.image_height * self.sqrt_spp ** 2

    @staticmethod
    def _opts(api, seed, row_offset, row_stride, threads, flags, devices=None, comm=None):
        opts = RtRenderOpts()
        api.render_opts_default(C.byref(opts))
        opts.seed = int(seed)
        opts.row_offset = int(row_offset)
        opts.row_stride = int(row_stride)
        opts.threads = int(threads)
        opts.flags = int(flags)
        keep = None
        if devices is not None and len(devices) > 1:
            keep = (C.c_int32 * len(devices))(*[int(d) for d in devices])
            opts.n_devices = len(devices)
            opts.devices = C.cast(keep, C.POINTER(C.c_int32))
        if comm is not None:
            opts.comm = comm
        return opts, keep

    def render(self, world, lights=None, seed=1, row_offset=0, row_stride=1, threads=0, want_srgb=True, flags=0,
               devices=None, comm=None):
        """Camera::render (camera.rs:161).  Returns (linear HxWx3 f32, srgb HxWx3 u8 or None, RtStats).
        devices: HIP device ordinals to split the rows over (in-process
        multi-GPU, one gather onto devices[0]); comm: an rt_comm* of
        rt_comm_init (one process per GPU; the frame arrives on rank 0)."""
        scene = world.scene
        api = scene.api
        cam = self.to_c()
        opts, _keep = self._opts(api, seed, row_offset, row_stride, threads, flags, devices, comm)
        rows = api.shard_rows(C.byref(cam), C.byref(opts))
        W = self.image_width
        lin = np.zeros((rows, W, 3), dtype=np.float32)
        srgb = np.zeros((rows, W, 3), dtype=np.uint8) if want_srgb else None
        stats = RtStats()
        rc = api.render(scene.s, world.h, -1 if lights is None else lights.h, C.byref(cam), C.byref(opts),
                        lin.ctypes.data_as(C.POINTER(C.c_float)),
                        srgb.ctypes.data_as(C.POINTER(C.c_uint8)) if srgb is not None else None, C.byref(stats))
        api.check(rc)
        return lin, srgb, stats

    def render_partials(self, world, lights=None, seed=1, row_offset=0, row_stride=1, threads=0, flags=0):
        """Parity tooling: the f64 sum over s_j of ray_color for every (pixel,
        stratum row s_i) of the shard, (rows, W, sqrt_spp, 3) -- the GPU's
        per-item sums (rt_render_partials_get) or the oracle's
        (orc_render_partials).  Returns (partials, RtStats)."""
        scene = world.scene
        api = scene.api
        cam = self.to_c()
        opts, _keep = self._opts(api, seed, row_offset, row_stride, threads, flags)
        rows = api.shard_rows(C.byref(cam), C.byref(opts))
        S = self.sqrt_spp
        part = np.zeros((rows, self.image_width, S, 3), dtype=np.float64)
        stats = RtStats()
        lh = -1 if lights is None else lights.h
        ptr = part.ctypes.data_as(C.POINTER(C.c_double))
        if hasattr(api, "render_partials"):  # the oracle
            api.check(api.render_partials(scene.s, world.h, lh, C.byref(cam), C.byref(opts), ptr, C.byref(stats)))
        else:
            api.check(api.render(scene.s, world.h, lh, C.byref(cam), C.byref(opts), None, None, C.byref(stats)))
            if part.size:
                api.check(api.render_partials_get(scene.s, ptr, part.size))
        return part, stats


def save_png(api, path, srgb):
    """img.save(path) after create_dir_all (main.rs:39-47): srgb is HxWx3 u8."""
    a = np.ascontiguousarray(srgb, dtype=np.uint8)
    h, w = a.shape[:2]
    api.check(api.write_png(os.fsencode(path), w, h, a.ctypes.data_as(C.c_void_p)))
