"""raytracer-2025_amd -- MI355X (gfx950) render path for caidj0/Raytracer-2025.

The product is librt_mi355x.so (HIP kernels + C ABI, include/rt_mi355x.h),
built in-tree next to this file.  `load()` loads it and fails loudly if it is
missing or was not built; there is no CPU fallback.
"""
import ctypes
import os

from .capi import Api, RtError  # noqa: F401

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "librt_mi355x.so")
# RT_MI355X_LIB names another build of the same ABI for a whole test run (the
# check build: `make -C raytracer-2025_amd check`, librt_mi355x_check.so)
if os.environ.get("RT_MI355X_LIB"):
    LIB_PATH = os.path.abspath(os.environ["RT_MI355X_LIB"])

_api = None


def load():
    """The gfx950 implementation of the ABI (prefix rt_)."""
    global _api
    if _api is None:
        # One HIP runtime per process: torch ships its own libamdhip64 (SONAME
        # libamdhip64.so.7).  Loading torch first makes librt_mi355x.so bind to
        # that copy instead of pulling /opt/rocm's in beside it.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} is missing: run `make -C raytracer-2025_amd` or __graft_entry__.build()")
        lib = ctypes.CDLL(LIB_PATH)
        api = Api(lib, "rt_")
        if api.missing:
            raise RuntimeError(f"{LIB_PATH} lacks symbols: {api.missing}")
        _api = api
    return _api
