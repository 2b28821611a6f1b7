"""ctypes binding of librmr_group.so (include/rmr_group.h): every GPU of the node from one process.

`DeviceGroup` is the single-process counterpart of multi_gpu.FrameRenderer's one-process-per-GPU
path: the same round-robin tile partition, the same two frames in flight, one RCCL reduce per frame,
here through ncclCommInitAll inside librmr_group.so. The C++ host uses the same library
(host/Graphics.cpp Graphics::setDevices / RenderFrame, rmr_cli --gpus N).
"""
import ctypes as C
import json
import os

import numpy as np

from . import abi
from ._lib import HERE, RMRError
from ._lib import lib as _rmr_lib

GROUP_LIB_PATH = os.path.join(HERE, "librmr_group.so")
GROUP_EXPORTS = [
    "rmr_group_create", "rmr_group_destroy", "rmr_group_last_error", "rmr_group_size", "rmr_group_context",
    "rmr_group_set_image_size", "rmr_group_set_params", "rmr_group_set_view", "rmr_group_load_scene_json",
    "rmr_group_load_builtin_scene", "rmr_group_set_env_map", "rmr_group_set_tile_size", "rmr_group_reload",
    "rmr_group_render_frame", "rmr_group_sync", "rmr_group_read_frame", "rmr_group_save_bmp",
    "rmr_group_get_stats", "rmr_group_reset_stats", "rmr_group_partition",
]
_glib = []


def group_lib():
    """The ctypes handle of librmr_group.so (librmr.so is loaded first, after torch: one HIP runtime)."""
    if _glib:
        return _glib[0]
    if not os.path.exists(GROUP_LIB_PATH):
        raise RuntimeError("librmr_group.so not built: run `python -c 'import __graft_entry__ as g; g.build()'`")
    _rmr_lib()
    L = C.CDLL(GROUP_LIB_PATH)
    vp, fp, ip = C.c_void_p, C.POINTER(C.c_float), C.POINTER(C.c_int)
    sig = {
        "rmr_group_create": (C.c_int, [C.POINTER(vp), ip, C.c_int]),
        "rmr_group_destroy": (None, [vp]),
        "rmr_group_last_error": (C.c_char_p, [vp]),
        "rmr_group_size": (C.c_int, [vp]),
        "rmr_group_context": (vp, [vp, C.c_int, C.c_int]),
        "rmr_group_set_image_size": (C.c_int, [vp, C.c_int, C.c_int]),
        "rmr_group_set_params": (C.c_int, [vp, C.POINTER(abi.Params)]),
        "rmr_group_set_view": (C.c_int, [vp, fp, fp, fp, fp, fp]),
        "rmr_group_load_scene_json": (C.c_int, [vp, C.c_int, C.c_char_p, C.c_size_t]),
        "rmr_group_load_builtin_scene": (C.c_int, [vp, C.c_int]),
        "rmr_group_set_env_map": (C.c_int, [vp, C.c_void_p, C.c_int, C.c_int]),
        "rmr_group_set_tile_size": (C.c_int, [vp, C.c_int]),
        "rmr_group_reload": (C.c_int, [vp]),
        "rmr_group_render_frame": (C.c_int, [vp, fp, C.c_uint32]),
        "rmr_group_sync": (C.c_int, [vp]),
        "rmr_group_read_frame": (C.c_int, [vp, fp, C.c_size_t]),
        "rmr_group_save_bmp": (C.c_int, [vp, C.c_char_p]),
        "rmr_group_get_stats": (C.c_int, [vp, C.c_int, C.POINTER(abi.Stats)]),
        "rmr_group_reset_stats": (C.c_int, [vp]),
        "rmr_group_partition": (C.c_int, [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_int32), C.c_int]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _glib.append(L)
    return L


def group_partition(W, H, tile, member, n):
    """rmr_group_partition: member m's tiles (tx, ty) of n, as an (k, 2) int32 array (no GPU)."""
    L = group_lib()
    cnt = L.rmr_group_partition(W, H, tile, member, n, None, 0)
    if cnt < 0:
        raise RMRError(cnt, "rmr_group_partition: bad arguments")
    out = np.zeros((max(cnt, 1), 2), np.int32)
    L.rmr_group_partition(W, H, tile, member, n, out.ctypes.data_as(C.POINTER(C.c_int32)), cnt)
    return out[:cnt]


class DeviceGroup:
    """rmr_group over `devices` (HIP device indices): frames tile-partitioned over them, one reduce each."""

    def __init__(self, devices, width=1024, height=1024, tile=32):
        self._L = group_lib()
        self._g = C.c_void_p()
        devs = (C.c_int * len(devices))(*devices)
        rc = self._L.rmr_group_create(C.byref(self._g), devs, len(devices))
        if rc != abi.RMR_OK:
            raise RMRError(rc, "rmr_group_create failed for devices %s" % (list(devices),))
        self.W, self.H = width, height
        self._chk(self._L.rmr_group_set_image_size(self._g, width, height))
        self._chk(self._L.rmr_group_set_tile_size(self._g, tile))

    def _chk(self, rc):
        if rc != abi.RMR_OK:
            raise RMRError(rc, (self._L.rmr_group_last_error(self._g) or b"").decode(errors="replace"))

    def close(self):
        if self._g:
            self._L.rmr_group_destroy(self._g)
            self._g = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def size(self):
        return self._L.rmr_group_size(self._g)

    def load_scene(self, scene, variant):
        if isinstance(variant, str):
            variant = abi.VARIANTS[variant]
        if isinstance(scene, dict):
            text = json.dumps(scene)
        elif os.path.exists(scene):
            with open(scene) as f:
                text = f.read()
        else:
            text = scene
        b = text.encode()
        self._chk(self._L.rmr_group_load_scene_json(self._g, variant, b, len(b)))

    def load_builtin(self, variant):
        if isinstance(variant, str):
            variant = abi.VARIANTS[variant]
        self._chk(self._L.rmr_group_load_builtin_scene(self._g, variant))

    def set_params(self, params):
        self._chk(self._L.rmr_group_set_params(self._g, C.byref(params)))

    def set_view(self, view15):
        v = np.ascontiguousarray(view15, np.float32).reshape(15)
        parts = [np.ascontiguousarray(v[3 * i:3 * i + 3]) for i in range(5)]
        self._view = parts
        self._chk(self._L.rmr_group_set_view(self._g, *[p.ctypes.data_as(C.POINTER(C.c_float)) for p in parts]))

    def reload(self):
        self._chk(self._L.rmr_group_reload(self._g))

    def render_frame(self, times):
        t = np.ascontiguousarray(times, np.float32)
        self._times = t
        self._chk(self._L.rmr_group_render_frame(self._g, t.ctypes.data_as(C.POINTER(C.c_float)), len(t)))

    def sync(self):
        self._chk(self._L.rmr_group_sync(self._g))

    def read_frame(self):
        out = np.zeros((self.H, self.W, 4), np.float32)
        self._chk(self._L.rmr_group_read_frame(self._g, out.ctypes.data_as(C.POINTER(C.c_float)), out.nbytes))
        return out

    def stats(self, member=0):
        s = abi.Stats()
        self._chk(self._L.rmr_group_get_stats(self._g, member, C.byref(s)))
        return s

    def reset_stats(self):
        self._chk(self._L.rmr_group_reset_stats(self._g))
